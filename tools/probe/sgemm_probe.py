"""Driver for sgemm.hip (weight-stationary streaming GEMM probe): correctness + TF/s vs torch."""
import ctypes, os, torch
import torch.nn.functional as F
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsgemm.so"))
lib.run_sgemm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                          ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
s = torch.cuda.current_stream().cuda_stream
T = 204800


def timeit(f, iters=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


cases = [(128, 128, False, [46, 47, 48, 49]), (128, 512, False, [46, 47, 48, 49]), (128, 384, False, [46, 47, 49]),
         (512, 128, False, [43, 50, 52])]
only = os.environ.get("SG_CASES")
if only:
    cases = [cases[int(i)] for i in only.split(",")]
for K, N, trans, variants in cases:
    x = torch.randn(T, K, device="cuda")
    if trans:
        w = torch.randn(K, N, device="cuda") * 0.05
        b = None
        ref = x @ w
        tf = lambda: x @ w  # noqa
    else:
        w = torch.randn(N, K, device="cuda") * 0.05
        b = torch.randn(N, device="cuda")
        ref = F.linear(x, w, b)
        tf = lambda: F.linear(x, w, b)  # noqa
    y = torch.empty(T, N, device="cuda")
    fl = 2.0 * T * K * N
    tt = timeit(tf)
    out = [f"torch {tt:6.1f}us {fl / tt / 1e6:5.1f}TF"]
    for v in variants:
        y.zero_()
        f = lambda: lib.run_sgemm(v, x.data_ptr(), T, K, w.data_ptr(), b.data_ptr() if b is not None else None, N,  # noqa
                                  y.data_ptr(), 256, s)
        rc = f()
        torch.cuda.synchronize()
        err = ((y - ref).abs().max() / ref.abs().max()).item() if v < 11 or v in (19, 22, 23, 24, 25, 26, 27, 28, 32, 34, 35, 36) or v >= 40 else 0.0
        t = timeit(f)
        out.append(f"v{v}: {t:6.1f}us {fl / t / 1e6:5.1f}TF err {err:.1e} rc {rc}")
    print(f"K={K} N={N} trans={trans}: " + " | ".join(out), flush=True)
