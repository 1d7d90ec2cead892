"""Experiment: asme_ws_linear reading X pre-split into its three bf16 planes (asme_ws_linear_planes:
no split VALU in the GEMM, 6 instead of 4 bytes per X element) vs reading fp32 X, at the K = 128 products a
LayerNorm produces the input of (QKV forward 128 -> 384, FFN-in forward + GELU / dropout 128 -> 512), M = 204,800.
Also times the split itself (the extra bytes a producer epilogue would write).  Same process, interleaved reps."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

asme = __graft_entry__.load_package()
lib = asme._lib.load()
P = ctypes.c_void_p
lib.asme_ws_split_planes.argtypes = [P, ctypes.c_int64, ctypes.c_int64, P, P]
lib.asme_ws_linear_planes.argtypes = [P, ctypes.c_int64, ctypes.c_int64, P, ctypes.c_int64, P, ctypes.c_int, P,
                                      ctypes.c_float, ctypes.c_uint64, P, P]
dev = torch.device("cuda", 0)
M, K = 204800, 128
torch.manual_seed(0)
x = torch.randn(M, K, device=dev)
planes = torch.empty(3 * M * K, device=dev, dtype=torch.bfloat16)
s = torch.cuda.current_stream().cuda_stream
L_ = asme._lib


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


split = lambda: lib.asme_ws_split_planes(x.data_ptr(), M, K, planes.data_ptr(), s)  # noqa: E731
split()
for N, epi, p in ((384, 0, 0.0), (512, 1, 0.2), (512, 0, 0.0), (128, 0, 0.0)):
    w = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    y0, y1 = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
    f0, f1 = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)

    def fp32():
        L_.call("asme_ws_linear", x.data_ptr(), M, K, w.data_ptr(), N, 0, b.data_ptr(), epi,
                f0.data_ptr() if epi == 1 else None, None, p, 7, y0.data_ptr(), s)

    def pl():
        rc = lib.asme_ws_linear_planes(planes.data_ptr(), M, K, w.data_ptr(), N, b.data_ptr(), epi,
                                       f1.data_ptr() if epi == 1 else None, p, 7, y1.data_ptr(), s)
        assert rc == 0, lib.asme_mi_last_error()
    res = {"fp32": [], "planes": []}
    for _ in range(3):
        res["fp32"].append(timed(fp32))
        res["planes"].append(timed(pl))
    same = torch.equal(y0, y1) and (epi != 1 or torch.equal(f0, f1))
    print(f"K=128 N={N} epi={epi}: fp32 X {min(res['fp32']):.1f} us   planes {min(res['planes']):.1f} us   "
          f"bit-identical {same}", flush=True)
print(f"split of X (M x 128: 105 MB in, 157 MB out): {timed(split):.1f} us")
