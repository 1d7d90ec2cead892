"""Weight-stationary GEMM (asme_ws_linear) at the bench shapes, every epilogue: device time per launch.
Usage: python tools/ws_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

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
    L = asme._lib
    dev = torch.device("cuda", 0)
    M = 204800
    torch.manual_seed(0)
    import sys as _s
    cfgs = [(128, 512, 0, 0, 0.0, 1), (128, 512, 1, 0, 0.0, 0)] * 3 if "--variance" in _s.argv else None
    for K, N, trans, epi, p, hb in cfgs or [(128, 512, 0, 0, 0.0, 1), (128, 512, 0, 0, 0.0, 0), (128, 512, 0, 1, 0.0, 1),
                                    (128, 512, 0, 1, 0.2, 1), (128, 512, 1, 0, 0.0, 0), (128, 512, 1, 2, 0.2, 0),
                                    (512, 128, 0, 0, 0.0, 1), (128, 384, 0, 0, 0.0, 1), (128, 384, 0, 0, 0.0, 0),
                                    (128, 128, 0, 0, 0.0, 1), (384, 128, 1, 0, 0.0, 0), (512, 128, 1, 0, 0.0, 0)]:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) if not trans else torch.randn(K, N, device=dev)
        b = torch.randn(N, device=dev)
        y = torch.empty(M, N, device=dev)
        aux = torch.randn(M, N, device=dev)

        def run():
            L.call("asme_ws_linear", L.ptr(x), M, K, L.ptr(w), N, trans, L.ptr(b if hb else None), epi,
                   L.ptr(aux if epi == 1 else None), L.ptr(aux if epi == 2 else None), p, 12345, L.ptr(y), L.stream())
        us = timeit(run)
        fl = 2.0 * M * N * K
        print(f"K={K:4d} N={N:4d} trans={trans} epi={epi} p={p} bias={hb}: {us:7.1f} us  {fl / us / 1e6:6.1f} TF/s")


if __name__ == "__main__":
    main()
