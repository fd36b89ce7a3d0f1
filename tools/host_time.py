import sys, time, torch
sys.path.insert(0, '/root/repo')
from kinet_amd.models import build_model, nested_tensor_from_tensor_list
from kinet_amd.models.config import load_args
torch.manual_seed(0)
m, _, _ = build_model(load_args('train_deformable', device='cuda'))
m = m.cuda().eval(); m.set_compute_dtype(torch.bfloat16)
x = nested_tensor_from_tensor_list([torch.randn(3, 800, 1333, device='cuda') for _ in range(8)])
with torch.no_grad():
    for _ in range(3): m(x)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter(); m(x); t1 = time.perf_counter()
        torch.cuda.synchronize(); t2 = time.perf_counter()
        ts.append((t1 - t0, t2 - t0))
print('host enqueue ms / total ms per forward:', [(round(a * 1e3, 2), round(b * 1e3, 2)) for a, b in ts])
