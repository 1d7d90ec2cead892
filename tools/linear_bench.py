"""Fused-linear kernels vs torch (hipBLASLt) at the bench shapes: correctness + timing.
Usage: python tools/linear_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import __graft_entry__  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    asme = __graft_entry__.load_package()
    call, ptr, st = asme._lib.call, asme._lib.ptr, asme._lib.stream
    dev = torch.device("cuda", 0)
    T = 204800
    for K, N in [(128, 384), (128, 128), (128, 512), (512, 128)]:
        x = torch.randn(T, K, device=dev)
        w = torch.randn(N, K, device=dev) * 0.05
        b = torch.randn(N, device=dev)
        y = torch.empty(T, N, device=dev)
        ref = F.linear(x, w, b)
        call("asme_linear_fwd", ptr(x), K, T, K, ptr(w), ptr(b), N, ptr(y), N, st())
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        t_me = timeit(lambda: call("asme_linear_fwd", ptr(x), K, T, K, ptr(w), ptr(b), N, ptr(y), N, st()))
        t_th = timeit(lambda: F.linear(x, w, b))
        fl = 2.0 * T * K * N
        print(f"fwd K={K} N={N}: err {err:.2e}  mine {t_me:.1f} us ({fl / t_me / 1e6:.1f} TF/s)  "
              f"torch {t_th:.1f} us ({fl / t_th / 1e6:.1f} TF/s)")
        # backward dx = dy . w  (dy: T x N, w: N x K)
        dy = torch.randn(T, N, device=dev)
        dx = torch.empty(T, K, device=dev)
        ref = dy @ w
        call("asme_linear_dx", ptr(dy), N, T, N, ptr(w), K, ptr(dx), K, 0, st())
        err = ((dx - ref).abs().max() / ref.abs().max()).item()
        t_me = timeit(lambda: call("asme_linear_dx", ptr(dy), N, T, N, ptr(w), K, ptr(dx), K, 0, st()))
        t_th = timeit(lambda: dy @ w)
        print(f"dx  K={K} N={N}: err {err:.2e}  mine {t_me:.1f} us ({fl / t_me / 1e6:.1f} TF/s)  "
              f"torch {t_th:.1f} us ({fl / t_th / 1e6:.1f} TF/s)")


if __name__ == "__main__":
    main()
