"""A/B timing of asme_ws_linear from two builds in one process (tools/probe/ab/lib_<X>.so), interleaved reps so
box-to-box clock differences cancel.  Usage: python tools/probe/ab_ws.py A B"""
import ctypes
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
libs = {}
for name in sys.argv[1:] or ["A", "B"]:
    lib = ctypes.CDLL(os.path.join(here, "ab", f"lib_{name}.so"))
    lib.asme_ws_linear.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                   ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    libs[name] = lib
dev = torch.device("cuda", 0)
M = 204800
cfgs = [(128, 512, 0, 0, 0.0, 1), (128, 512, 0, 1, 0.2, 1), (128, 512, 1, 2, 0.2, 0), (512, 128, 0, 0, 0.0, 1),
        (512, 128, 1, 0, 0.0, 0), (128, 384, 0, 0, 0.0, 1), (128, 128, 0, 0, 0.0, 1), (384, 128, 1, 0, 0.0, 0)]
for K, N, trans, epi, p, hb in cfgs:
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) if not trans else torch.randn(K, N, device=dev)
    b = torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev)
    aux = torch.randn(M, N, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    res = {n: [] for n in libs}
    for rep in range(5):
        for n, lib in libs.items():
            f = lambda: lib.asme_ws_linear(x.data_ptr(), M, K, w.data_ptr(), N, trans, b.data_ptr() if hb else None, epi,
                                           aux.data_ptr() if epi == 1 else None, aux.data_ptr() if epi == 2 else None,
                                           p, 12345, y.data_ptr(), s)
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[n].append(e0.elapsed_time(e1) / 10 * 1e3)
    print(f"K={K:3d} N={N:3d} trans={trans} epi={epi}: " + "  ".join(f"{n} {min(v):6.1f}" for n, v in res.items()),
          flush=True)
