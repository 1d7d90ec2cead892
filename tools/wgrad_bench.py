"""asme_linear_weight_grad at the SASRec bench shapes (T = 204,800 tokens, d = 128, d_ff = 512): per-shape time,
fp32-equivalent TFLOP/s, GB/s of the algorithmic bytes (dY + X read once) and max error vs torch fp32.
Usage: python tools/wgrad_bench.py [--iters N]   (ASME_MI_LIB=... for an A/B build)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402


def bench(fn, n):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="qkv,out,w1,w2")
    a = ap.parse_args()
    asme = __graft_entry__.load_package()
    dev = torch.device("cuda:0")
    T, d, ff = 204800, 128, 512
    shapes = {"qkv": (d, 3 * d), "out": (d, d), "w1": (d, ff), "w2": (ff, d)}
    tot = 0.0
    torch.manual_seed(0)
    for name, (k, n) in shapes.items():
        if name not in a.shapes.split(","):
            continue
        x = torch.randn(T, k, device=dev)
        dy = torch.randn(T, n, device=dev)
        nb = int(asme._lib.load().asme_linear_weight_grad_workspace(T, n, k))
        ws = torch.empty(nb // 4 + 1, device=dev)
        dw = torch.empty(n, k, device=dev)
        db = torch.empty(n, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        f = lambda: asme._lib.call("asme_linear_weight_grad", dy.data_ptr(), n, x.data_ptr(), k, T, n, k,  # noqa
                                   ws.data_ptr(), nb, dw.data_ptr(), db.data_ptr(), 0, s)
        t = bench(f, a.iters)
        tot += t
        ref = dy.t() @ x
        err = float((dw - ref).abs().max() / ref.abs().max())
        print(f"{name:4s} K={k:4d} N={n:4d}  {t * 1e3:7.1f} us  {2 * T * k * n / t / 1e9:6.1f} TF/s  "
              f"{T * (k + n) * 4 / t / 1e6:6.0f} GB/s  rel err {err:.1e}")
    print(f"sum of the 4 shapes {tot * 1e3:.1f} us (x2 layers per step: {2 * tot * 1e3:.1f} us)")


if __name__ == "__main__":
    main()
