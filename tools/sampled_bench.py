"""SASRec sampled head (asme_sampled_logits_fwd / _bwd) at the bench shape: T = 204,800 tokens, d = 128, pos / neg
ids uniform over a 614k-row table (the step's staged rows).  Usage: python tools/sampled_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402


def main():
    asme = __graft_entry__.load_package()
    dev = torch.device("cuda:0")
    T, D, V = 204800, 128, 614400
    torch.manual_seed(0)
    H = torch.randn(T, D, device=dev)
    E = torch.randn(V, D, device=dev)
    pos = torch.randint(0, V, (T,), device=dev)
    neg = torch.randint(0, V, (T,), device=dev)
    po, no = torch.empty(T, device=dev), torch.empty(T, device=dev)
    gp, gn = torch.randn(T, device=dev), torch.randn(T, device=dev)
    dh = torch.empty(T, D, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    call, ptr = asme._lib.call, asme._lib.ptr
    fwd = lambda: call("asme_sampled_logits_fwd", ptr(H), ptr(E), ptr(pos), ptr(neg), T, D, V, ptr(po), ptr(no), s)  # noqa
    bwd = lambda: call("asme_sampled_logits_bwd", ptr(H), ptr(E), ptr(pos), ptr(neg), T, D, V, ptr(gp), ptr(gn),  # noqa
                       ptr(dh), None, s)
    for name, fn, nbytes in (("fwd", fwd, T * D * 4 * 3 + T * 24), ("bwd", bwd, T * D * 4 * 3 + T * 24 + T * D * 4)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name}: {us:.1f} us  {nbytes / us / 1e3:.0f} GB/s")
    ref = (E[pos] * H).sum(1)
    print("max err", float((po - ref).abs().max()))


if __name__ == "__main__":
    main()
