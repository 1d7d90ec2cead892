"""Cost of each fused epilogue at the bench shapes (T=204800): plain GEMM vs GEMM+epilogue, p=0 / 0.2."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402
from tools.linear_bench import timeit  # noqa: E402


def main():
    asme = __graft_entry__.load_package()
    call, ptr, st = asme._lib.call, asme._lib.ptr, asme._lib.stream
    dev = torch.device("cuda", 0)
    T, D, Fd = 204800, 128, 512
    x = torch.randn(T, D, device=dev)
    xf = torch.randn(T, Fd, device=dev)
    w1 = torch.randn(Fd, D, device=dev) * 0.05
    w2 = torch.randn(D, Fd, device=dev) * 0.05
    b1, b2 = torch.randn(Fd, device=dev), torch.randn(D, device=dev)
    y1 = torch.empty(T, Fd, device=dev)
    pre = torch.empty(T, Fd, device=dev)
    y2 = torch.empty(T, D, device=dev)
    s2 = torch.empty(T, D, device=dev)
    stt = torch.empty(T, 2, device=dev)
    lw, lb = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    res = torch.randn(T, D, device=dev)
    rows = int(asme._lib.load().asme_linear_partials_rows(T))
    part = torch.empty(rows, 2 * D, device=dev)
    r = {}
    r["fwd K128 N512 plain"] = timeit(lambda: call("asme_linear_fwd", ptr(x), D, T, D, ptr(w1), ptr(b1), Fd, ptr(y1), Fd, st()))
    for p in (0.0, 0.2):
        r[f"fwd K128 N512 gelu p={p}"] = timeit(lambda: call("asme_linear_gelu_dropout_fwd", ptr(x), D, T, D, ptr(w1), ptr(b1), Fd, p, 5, ptr(pre), ptr(y1), Fd, st()))
    r["gelu standalone p=0.2"] = timeit(lambda: call("asme_gelu_dropout_fwd", ptr(pre), T * Fd, 0.2, 5, ptr(y1), st()))
    r["fwd K512 N128 plain"] = timeit(lambda: call("asme_linear_fwd", ptr(xf), Fd, T, Fd, ptr(w2), ptr(b2), D, ptr(y2), D, st()))
    r["fwd K128 N128 plain"] = timeit(lambda: call("asme_linear_fwd", ptr(x), D, T, D, ptr(w2[:, :D].contiguous()), ptr(b2), D, ptr(y2), D, st()))
    wo = torch.randn(D, D, device=dev) * 0.05
    for p in (0.0, 0.2):
        r[f"fwd K512 N128 resln p={p}"] = timeit(lambda: call("asme_linear_residual_ln_fwd", ptr(xf), Fd, T, Fd, ptr(w2), ptr(b2), D, ptr(res), p, 3, p, 4, ptr(lw), ptr(lb), 1e-5, ptr(s2), ptr(y2), ptr(stt), st()))
        r[f"fwd K128 N128 resln p={p}"] = timeit(lambda: call("asme_linear_residual_ln_fwd", ptr(x), D, T, D, ptr(wo), ptr(b2), D, ptr(res), p, 3, 0.0, 0, ptr(lw), ptr(lb), 1e-5, ptr(s2), ptr(y2), ptr(stt), st()))
    r["resln standalone p=0.2/0.2"] = timeit(lambda: call("asme_residual_ln_fwd", ptr(res), ptr(x), T, D, 0.2, 3, 0.2, 4, ptr(lw), ptr(lb), 1e-5, ptr(s2), ptr(y2), ptr(stt), st()))
    dy = torch.randn(T, D, device=dev)
    r["dx K512(out) from N128 plain"] = timeit(lambda: call("asme_linear_dx", ptr(dy), D, T, D, ptr(w2), Fd, ptr(y1), Fd, 0, st()))
    for p in (0.0, 0.2):
        r[f"dx gelu_bwd p={p}"] = timeit(lambda: call("asme_linear_dx_gelu_bwd", ptr(dy), D, T, D, ptr(w2), Fd, ptr(pre), p, 5, ptr(y1), Fd, st()))
    dyf = torch.randn(T, Fd, device=dev)
    r["dx 128(out) from 512 plain"] = timeit(lambda: call("asme_linear_dx", ptr(dyf), Fd, T, Fd, ptr(w1), D, ptr(y2), D, 0, st()))
    for p in (0.0, 0.2):
        r[f"dx resln_bwd p={p}"] = timeit(lambda: call("asme_linear_dx_residual_ln_bwd", ptr(dyf), Fd, T, Fd, ptr(w1), D, ptr(s2), ptr(stt), ptr(lw), ptr(res), p, 3, p, 4, ptr(y2), ptr(x), ptr(part), st()))
    for k, v in r.items():
        print(f"{k:32s} {v:8.1f} us")


if __name__ == "__main__":
    main()
