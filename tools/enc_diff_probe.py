"""Where do the encoder-kernel and gather-kernel outputs differ? (debug probe)"""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, 'tests'))
from kinet_amd import kernels as K  # noqa: E402
from oracle import msda_oracle as O  # noqa: E402
from test_msda_gpu import _encoder_inputs  # noqa: E402

shapes = ((40, 67), (20, 34), (10, 17), (5, 9))
B, M, P = 2, 8, 4
value, ss, offlog, ref, qmask = _encoder_inputs(B, shapes, M, P, 2, 0.0, 31, None)
plan = K.encoder_plan(shapes, value.device)
od = torch.bfloat16
o0, loc, aw = K.msda_fused(value, ss, offlog, ref, M, 4, P, qmask, head_major=True, out_dtype=od, want_loc_attw=True)
o1 = K.msda_encoder(value, plan, offlog, ref, M, qmask, out_dtype=od)
torch.cuda.synchronize()
v = value.float().permute(1, 2, 0, 3).contiguous().cpu().numpy()
ro = torch.from_numpy(O.fwd(v, ss.cpu().numpy(), loc.cpu().numpy(), aw.cpu().numpy())).reshape(o0.shape)
e0 = (o0.float().cpu() - ro).abs()
e1 = (o1.float().cpu() - ro).abs()
print('max err vs oracle: gather', e0.max().item(), 'encoder', e1.max().item())
d = (o0.float() - o1.float()).abs().cpu()
idx = torch.argsort(d.reshape(-1), descending=True)[:8]
starts = np.cumsum([0] + [h * w for h, w in shapes])
for i in idx.tolist():
    b_, q, c = np.unravel_index(i, d.shape)
    lvl = int(np.searchsorted(starts, q, side='right') - 1)
    qq = q - starts[lvl]
    print(f'b={b_} q={q} lvl={lvl} row={qq // shapes[lvl][1]} col={qq % shapes[lvl][1]} ch={c} head={c // 32}: '
          f'gather {o0[b_, q, c].item():.5f} enc {o1[b_, q, c].item():.5f} oracle {ro[b_, q, c].item():.5f}')
m = c // 32
print('loc', loc[b_, q, m].cpu().numpy().reshape(-1, 2)[:16])
print('aw', aw[b_, q, m].cpu().numpy().reshape(-1))
o1b, l1, a1 = K.msda_encoder(value, plan, offlog, ref, M, qmask, out_dtype=od, want_loc_attw=True)
torch.cuda.synchronize()
print('enc with loc_out equal to without:', torch.equal(o1b, o1), torch.equal(l1, loc), torch.equal(a1, aw))
d = (o0.float() - o1b.float()).abs()
tol = torch.maximum(o0.float().abs(), o1b.float().abs()) * 2 * 2.0 ** -7 + 1e-5
bad = (d > tol).nonzero()
print('n bad', bad.shape[0])
for b_, q, c in bad[:10].tolist():
    print(b_, q, c, o0[b_, q, c].item(), o1b[b_, q, c].item(), ro[b_, q, c].item())
