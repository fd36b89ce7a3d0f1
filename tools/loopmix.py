"""Instruction mix of the loops of one kernel in a hipcc -S listing.
    python tools/loopmix.py file.s mangled_name_substring"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", s, re.M) if sys.argv[2] in m.group(1)]
for name in names[:4]:
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    body = s[i:j].splitlines()
    labels = {}
    for n, l in enumerate(body):
        t = l.strip()
        if re.match(r'^\.LBB\S+:', t):
            labels[t[:-1]] = n
    print(name[:110])
    for n, l in enumerate(body):
        t = l.strip()
        m = re.match(r's_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)', t)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < n and n - labels[tgt] > 40:
            c = collections.Counter()
            for x in body[labels[tgt]:n + 1]:
                x = x.strip()
                if not x or x[0] in ';.':
                    continue
                op = x.split()[0]
                k = ('mfma' if 'mfma' in op else 'ds_read' if op.startswith('ds_read') else
                     'ds_write' if op.startswith('ds_write') else 'buf_ld' if op.startswith('buffer_load') else
                     'buf_st' if op.startswith('buffer_store') else 'global' if op.startswith('global') else
                     'valu' if op.startswith('v_') else 'salu' if op.startswith('s_') else op)
                c[k] += 1
            print('  ', tgt, n - labels[tgt], dict(c))
