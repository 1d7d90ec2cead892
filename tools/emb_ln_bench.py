"""asme_embedding_ln_fwd / _bwd timing at the headline's in-step shape (SASRec: LN1 + dropout + LN2 + dropout +
block 0's LN3; T = 1024 x 200 tokens, d = 128) reading rows in slot order from a staged-rows buffer (3T rows), as
the training step does.  Prints us per call and the fraction of the 8 TB/s roofline on the algorithmic bytes
bench.py uses, for p = 0.2 (the headline) and p = 0 (no Philox / keep bytes), plus the copy ceiling of the same
read / write pattern.  Usage: python tools/emb_ln_bench.py [--iters N]   (ASME_MI_LIB=... for a variant build)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402


def timed(fn, iters):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seq", type=int, default=200)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--order", choices=["slot", "random"], default="slot")
    ap.add_argument("--basic", action="store_true", help="only the p = 0.2 / 0 timings (no in-step probes)")
    a = ap.parse_args()
    asme = __graft_entry__.load_package()
    L_ = asme._lib
    dev = torch.device("cuda", 0)
    B, L, D = a.batch, a.seq, a.dim
    T = B * L
    torch.manual_seed(0)
    src = torch.randn(3 * T, D, device=dev)
    ids = (torch.arange(T, device=dev) if a.order == "slot" else torch.randint(0, 3 * T, (T,), device=dev))
    pos = torch.randn(L, D, device=dev)
    ln = [(torch.rand(D, device=dev) + 0.5, torch.randn(D, device=dev) * 0.1) for _ in range(3)]
    out, lno = torch.empty(T, D, device=dev), torch.empty(T, D, device=dev)
    stats, stats3 = torch.empty(T, 4, device=dev), torch.empty(T, 2, device=dev)
    keep = torch.empty(T, D // 4, device=dev, dtype=torch.uint8)
    dout, dln = torch.randn(T, D, device=dev), torch.randn(T, D, device=dev)
    d_rows = torch.empty(T, D, device=dev)
    npart = 2048
    part = torch.empty(npart, 6 * D, device=dev)
    fwd_bytes = T * 8 + 3 * T * D * 4 + T * 16 + T * 8
    bwd_bytes = T * 8 + 4 * T * D * 4 + T * 16 + T * 8
    P = L_.ptr
    for p in (0.2, 0.0):
        def fwd():
            L_.call("asme_embedding_ln_fwd", P(ids), T, L, P(src), src.shape[0], D, P(pos), P(ln[0][0]), P(ln[0][1]),
                    1e-5, p, 11, None, P(ln[1][0]), P(ln[1][1]), 1e-5, p, 12, P(ln[2][0]), P(ln[2][1]), 1e-5, P(out),
                    P(stats), P(lno), P(stats3), P(keep) if p > 0 else None, None, L_.stream())

        def bwd():
            L_.call("asme_embedding_ln_bwd", P(ids), T, L, P(src), src.shape[0], D, P(pos), P(ln[0][0]), P(ln[0][1]),
                    p, 11, None, P(ln[1][0]), P(ln[1][1]), p, 12, P(ln[2][0]), P(stats3), P(keep) if p > 0 else None,
                    P(dout), P(dln), P(stats), P(d_rows), None, P(part), npart, L_.stream())
        f = timed(fwd, a.iters)
        b = timed(bwd, a.iters)
        print(f"p={p}: fwd {f:.1f} us ({fwd_bytes / f / 8e6:.3f} of 8 TB/s)  bwd {b:.1f} us "
              f"({bwd_bytes / b / 8e6:.3f})", flush=True)
    if a.basic:
        return
    # in-step conditions: the lazy-Adam stage writes ~0.9 GB of staged rows right before the forward (dirty lines
    # still draining from the L2 / MALL); each call bracketed by its own event pair, as bench.py's KernelTimer does
    big = torch.empty(3 * 3 * T * D, device=dev)
    import ctypes
    # (build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probe/stream_probe.hip -o tools/probe/libstream.so)
    probe = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe", "libstream.so"))
    probe.run_stream.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 6 + [ctypes.c_int64, ctypes.c_void_p]
    nb4 = big.numel() // 4

    def pre_op(kind, i):
        if kind == "fill 0.9 GB":
            big.fill_(float(i))
        elif kind == "NT write 0.9 GB":
            probe.run_stream(3, 1, 8192, None, None, None, None, big.data_ptr(), None, nb4, L_.stream())
        elif kind == "read 0.9 GB":
            probe.run_stream(2, 0, 8192, big.data_ptr(), None, None, None, big.data_ptr(), None, nb4, L_.stream())
    for pre in ("none", "fill 0.9 GB", "NT write 0.9 GB", "read 0.9 GB"):
        evs = []
        for i in range(a.iters):
            pre_op(pre, i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fwd_p = 0.2
            L_.call("asme_embedding_ln_fwd", P(ids), T, L, P(src), src.shape[0], D, P(pos), P(ln[0][0]), P(ln[0][1]),
                    1e-5, fwd_p, 11, None, P(ln[1][0]), P(ln[1][1]), 1e-5, fwd_p, 12, P(ln[2][0]), P(ln[2][1]), 1e-5,
                    P(out), P(stats), P(lno), P(stats3), P(keep), None, L_.stream())
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize()
        t = sorted(x.elapsed_time(y) * 1e3 for x, y in evs[3:])
        print(f"fwd p=0.2 after {pre}, per-call events: median {t[len(t) // 2]:.1f} us (min {t[0]:.1f})")
    del big
    # copy ceilings of the same pattern: fwd reads 1 row and writes 2 per token, bwd reads 4 and writes 1
    dst2 = torch.empty(2, T, D, device=dev)
    c = timed(lambda: dst2.copy_(src[:T].unsqueeze(0).expand(2, T, D)), a.iters)
    print(f"copy 1 read -> 2 writes of T rows: {c:.1f} us ({3 * T * D * 4 / c / 8e6:.3f})")
    four = torch.randn(4, T, D, device=dev)
    s = timed(lambda: torch.sum(four, 0, out=d_rows), a.iters)
    print(f"sum of 4 row streams -> 1: {s:.1f} us ({5 * T * D * 4 / s / 8e6:.3f})")


if __name__ == "__main__":
    main()
