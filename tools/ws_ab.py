"""Same-process A/B of asme_ws_linear at the bench step's shapes (M = 204,800 tokens): every library named on the
command line (default: the in-tree libasme_mi.so) is loaded side by side and the reps interleave, so box clock
differences cancel.  Usage: python tools/ws_ab.py [lib.so ...] [--only K:N:trans:epi,...] [--reps R]"""
import argparse
import ctypes
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INTREE = os.path.join(ROOT, "recsys-22-user-attributes-recommender_amd", "libasme_mi.so")
# (K, N, trans, epi, p, bias): the eight products of a SASRec block at d = 128, d_ff = 512
CFGS = [(128, 384, 0, 0, 0.0, 1), (128, 128, 0, 0, 0.0, 1), (128, 512, 0, 1, 0.2, 1), (512, 128, 0, 0, 0.0, 1),
        (128, 512, 1, 2, 0.2, 0), (512, 128, 1, 0, 0.0, 0), (128, 128, 1, 0, 0.0, 0), (384, 128, 1, 0, 0.0, 0),
        (128, 512, 0, 0, 0.0, 1)]

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="*")
ap.add_argument("--only", default="")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--p", type=float, default=None, help="override the dropout probability")
a = ap.parse_args()
libs = {}
for path in a.libs or [INTREE]:
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.asme_ws_linear.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                   ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    libs[os.path.basename(path)] = lib
only = {tuple(int(v) for v in s.split(":")) for s in a.only.split(",") if s}
dev = torch.device("cuda", 0)
M = 204800
total = {n: 0.0 for n in libs}
for K, N, trans, epi, p, hb in CFGS:
    p = p if a.p is None or epi == 0 else a.p
    if only and (K, N, trans, epi) not in only:
        continue
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) if not trans else torch.randn(K, N, device=dev)
    b = torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev)
    aux = torch.randn(M, N, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    res = {n: [] for n in libs}
    outs = {}
    for rep in range(a.reps):
        for n, lib in libs.items():
            def f():
                rc = lib.asme_ws_linear(x.data_ptr(), M, K, w.data_ptr(), N, trans, b.data_ptr() if hb else None,
                                        epi, aux.data_ptr() if epi == 1 else None,
                                        aux.data_ptr() if epi == 2 else None, p, 12345, y.data_ptr(), s)
                assert rc == 0, rc
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[n].append(e0.elapsed_time(e1) / a.iters * 1e3)
            if rep == 0 and epi != 2:
                outs[n] = y.clone()
    ref = next(iter(outs.values())) if outs else None
    diffs = " ".join(f"d={float((o - ref).abs().max()):.1e}" for o in list(outs.values())[1:]) if ref is not None else ""
    for n in libs:
        total[n] += min(res[n])
    print(f"K={K:3d} N={N:3d} trans={trans} epi={epi}: " + "  ".join(f"{n} {min(v):6.1f}" for n, v in res.items())
          + f"  {diffs}", flush=True)
print("sum: " + "  ".join(f"{n} {v:7.1f}" for n, v in total.items()))
