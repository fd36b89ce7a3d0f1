"""LDS-DMA drain check: in every loop of every kernel of a hipcc -S listing, find s_waitcnt vmcnt(N)
instructions the COMPILER inserted (outside inline asm) that force an LDS-DMA (buffer_load ... lds)
issued earlier in the SAME loop iteration to complete -- the wait that turns a prefetch ring into a
synchronous load.  The compiler inserts one before an LDS read it cannot prove disjoint from an
in-flight DMA, and behind any VGPR-destination load whose result it needs (round 6: the records
GEMM's level-shape select became an indexed kernel-argument load, and its mask / reference-point
LDS reads sat behind the next tile's DMA; profiles/r06i_records_ring_ab.txt).

The control-flow graph is rebuilt from the listing (labels, fall-through, s_branch / s_cbranch_*);
each compiler wait is followed backwards along every predecessor path, counting vector-memory
instructions, until the header of its innermost loop (the block the compiler marks "Loop Header")
is passed: a DMA met on such a path before the wait's N younger ops are used up is one the wait
forces to land in the iteration that issued it.

    python tools/dma_drain_check.py FILE.s [...]          # kernels with a drain, and where
"""
import re
import sys

VMEM = re.compile(r'^(buffer_|global_|flat_|scratch_)')
BR = re.compile(r'^s_(branch|cbranch_\w+)\s+(\.LBB\S+)')


def kernels(path):
    L = open(path).read().split('\n')
    i = 0
    while i < len(L):
        m = re.match(r'^(_Z\S+):', L[i])
        if not m:
            i += 1
            continue
        j = i + 1
        while j < len(L) and not L[j].startswith('.Lfunc_end'):
            j += 1
        yield m.group(1), L[i + 1:j]
        i = j


def blocks(body):
    """[(label, is_header, [(line, text, in_asm)], succ labels)]"""
    out, cur, inasm = [], None, False
    for n, l in enumerate(body):
        t = l.strip()
        mm = re.match(r'^(\.LBB\S+):', t)
        if mm:
            if cur is not None and cur[3] is None:
                cur[3] = [mm.group(1)]   # fall-through
            cur = [mm.group(1), 'Loop Header' in t, [], None]
            out.append(cur)
            continue
        if cur is None:
            cur = ['<entry>', False, [], None]
            out.append(cur)
        if t.startswith(';;#ASMSTART'):
            inasm = True
            continue
        if t.startswith(';;#ASMEND'):
            inasm = False
            continue
        if not t or t[0] in ';.':
            continue
        if cur[3] is not None:   # code after a terminator without a label: a new anonymous block
            cur = ['<anon%d>' % n, False, [], None]
            out.append(cur)
        cur[2].append((n, t, inasm))
        op = t.split()[0]
        b = BR.match(t)
        if b:
            if b.group(1) == 'branch':
                cur[3] = [b.group(2)]
            else:
                cur[3] = [b.group(2), None]   # None: fall-through, resolved below
        elif op in ('s_endpgm', 's_setpc_b64'):
            cur[3] = []
    for k, blk in enumerate(out):
        nxt = out[k + 1][0] if k + 1 < len(out) else None
        if blk[3] is None:
            blk[3] = [nxt] if nxt else []
        else:
            blk[3] = [nxt if s is None else s for s in blk[3] if (s is not None or nxt)]
    return out


def drains(body):
    bl = blocks(body)
    idx = {b[0]: k for k, b in enumerate(bl)}
    preds = {k: [] for k in range(len(bl))}
    for k, b in enumerate(bl):
        for s in b[3]:
            if s in idx:
                preds[idx[s]].append(k)
    # natural loops of the compiler's marked headers: the blocks that reach a back edge's source
    # without passing the header; a block's loop is the smallest one containing it
    loops = []
    for h, b in enumerate(bl):
        if not b[1]:
            continue
        # back edges: predecessors of the header that the header reaches (the entry edge does not)
        reach, fw = set(), [h]
        while fw:
            j = fw.pop()
            for s2 in bl[j][3]:
                q = idx.get(s2)
                if q is not None and q not in reach:
                    reach.add(q)
                    fw.append(q)
        body_set = {h}
        work = [j for j in preds[h] if j in reach]
        while work:
            j = work.pop()
            if j in body_set:
                continue
            body_set.add(j)
            work.extend(preds[j])
        loops.append((len(body_set), h, body_set))
    loops.sort()
    out = []
    for k, b in enumerate(bl):
        for pos, (n, t, inasm) in enumerate(b[2]):
            mm = re.match(r's_waitcnt (?:.*\s)?vmcnt\((\d+)\)', t)
            if not mm or inasm:
                continue
            N = int(mm.group(1))
            inner = [h for _, h, bs in loops if k in bs]
            if not inner:
                continue   # not in a loop: a drain there costs one latency per kernel
            hdr = inner[0]
            # backwards walk: (block, index of the last instruction to look at, younger vmem ops)
            stack = [(k, pos - 1, 0)]
            seen = set()
            forced = False
            while stack and not forced:
                bk, i, cnt = stack.pop()
                if (bk, i, cnt) in seen:
                    continue
                seen.add((bk, i, cnt))
                ins = bl[bk][2]
                while i >= 0:
                    t2 = ins[i][1]
                    if VMEM.match(t2.split()[0]):
                        if t2.endswith(' lds') and cnt >= N:
                            forced = True   # older than the N youngest: must land here
                            break
                        cnt = min(cnt + 1, N)
                    i -= 1
                if forced:
                    continue
                if hdr is not None and bk == hdr:
                    continue   # the iteration starts here
                for p in preds[bk]:
                    stack.append((p, len(bl[p][2]) - 1, cnt))
            if forced:
                nxt = b[2][pos + 1][1].split()[0] if pos + 1 < len(b[2]) else ''
                out.append((n, N, nxt))
    return out


def main():
    bad = 0
    for path in sys.argv[1:]:
        for name, body in kernels(path):
            d = drains(body)
            if d:
                bad += 1
                print('%s  %s' % (path.split('/')[-1], name[:150]))
                for n, N, nxt in d[:4]:
                    print('    line %d: s_waitcnt vmcnt(%d) lands an LDS-DMA of this iteration; next: %s' % (n, N, nxt))
    print('%d kernel(s) with a compiler-inserted wait that drains an in-flight LDS-DMA' % bad)


if __name__ == '__main__':
    main()
