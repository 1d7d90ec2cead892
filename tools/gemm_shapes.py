"""Time the transformer's fp32 GEMM shapes on hipBLASLt (torch) at the bench config."""
import torch, time
dev = torch.device('cuda:0')
T, d, ff = 204800, 128, 512
def bench(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1) / n
shapes = {'qkv': (d, 3 * d), 'out': (d, d), 'w1': (d, ff), 'w2': (ff, d)}
tot = 0
for name, (k, n) in shapes.items():
    x = torch.randn(T, k, device=dev); w = torch.randn(n, k, device=dev); b = torch.randn(n, device=dev)
    dy = torch.randn(T, n, device=dev)
    fl = 2 * T * k * n
    t_f = bench(lambda: torch.nn.functional.linear(x, w, b))
    t_dx = bench(lambda: dy @ w)
    t_dw = bench(lambda: dy.t() @ x)
    t_db = bench(lambda: dy.sum(0))
    tot += t_f + t_dx + t_dw + t_db
    print(f"{name:4s} K={k:4d} N={n:4d}  fwd {t_f:.3f}ms {fl/t_f/1e9:6.1f}TF  dX {t_dx:.3f}ms {fl/t_dx/1e9:6.1f}TF  dW {t_dw:.3f}ms {fl/t_dw/1e9:6.1f}TF  db {t_db:.3f}ms")
print('per layer total ms', tot, 'x2 layers', 2 * tot)

import sys
sys.path.insert(0, '.')
import __graft_entry__
asme = __graft_entry__.load_package()
tot2 = 0
for name, (k, n) in shapes.items():
    x = torch.randn(T, k, device=dev); dy = torch.randn(T, n, device=dev)
    nb = int(asme._lib.load().asme_linear_weight_grad_workspace(T, n, k))
    ws = torch.empty(nb // 4, device=dev); dw = torch.empty(n, k, device=dev); db = torch.empty(n, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    f = lambda: asme._lib.call("asme_linear_weight_grad", dy.data_ptr(), n, x.data_ptr(), k, T, n, k, ws.data_ptr(), nb,
                               dw.data_ptr(), db.data_ptr(), 0, s)
    t = bench(f)
    tot2 += t
    print(f"{name:4s} asme dW+db {t:.3f}ms {2*T*k*n/t/1e9:6.1f}TF  err {float((dw - dy.t() @ x).abs().max()):.2e}")
print('asme dW+db per layer', tot2)
