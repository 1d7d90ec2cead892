"""Embedding-kernel timing at the bench shape (T = 1024 x 200 tokens, |V| = 10M, d = 128).

Usage: python tools/emb_bench.py [--iters N]
Times asme_embedding_fwd / _bwd (SASRec form: position add, LN1, dropout, LN2, dropout) at p = 0 and p = 0.2,
and two gather ceilings: torch.index_select of the same rows and a sequential copy of T rows, so the
kernel's distance from the random-row-gather limit is visible.
"""
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seq", type=int, default=200)
    ap.add_argument("--items", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--partials", type=int, default=0, help="backward partial rows (ops._EMB_PARTIALS; 0: default)")
    a = ap.parse_args()
    asme = __graft_entry__.load_package()
    if a.partials:
        asme.ops._EMB_PARTIALS = a.partials
    dev = torch.device("cuda", 0)
    B, L, V, D = a.batch, a.seq, a.items + 3, a.dim
    T = B * L
    torch.manual_seed(0)
    table = torch.randn(V, D, device=dev)
    pos = torch.randn(L, D, device=dev, requires_grad=True)
    ids = torch.randint(3, V, (B, L), device=dev)
    ln1 = (torch.ones(D, device=dev), torch.zeros(D, device=dev))
    ln2 = (torch.ones(D, device=dev), torch.zeros(D, device=dev))
    gb = 1e-9
    emb_bytes = T * 8 + 2 * T * D * 4 + T * 16
    bwd_bytes = T * 8 + 3 * T * D * 4 + T * 16
    for p in (0.0, 0.2):
        spec = asme.ops.EmbeddingSpec(seq_len=L, p1=p, p2=p)
        with torch.no_grad():
            f = timed(lambda: asme.ops.embedding(ids, table, pos, ln1, None, ln2, spec), a.iters)
        out = asme.ops.embedding(ids, table, pos, ln1, None, ln2, spec)
        g = torch.randn_like(out)
        with asme._lib.KernelTimer(["asme_embedding_fwd", "asme_embedding_bwd"]) as kt:
            for _ in range(a.iters):
                asme.ops.embedding(ids, table, pos, ln1, None, ln2, spec)
                torch.autograd.grad(out, [pos], g, retain_graph=True)
        st = kt.summary()
        kf, kb = st["asme_embedding_fwd"]["avg_ms"] * 1e3, st["asme_embedding_bwd"]["avg_ms"] * 1e3
        print(f"p={p}: fwd loop {f:.1f} us; kernels: fwd {kf:.1f} us ({emb_bytes * gb / (kf * 1e-6):.0f} GB/s)  "
              f"bwd {kb:.1f} us ({bwd_bytes * gb / (kb * 1e-6):.0f} GB/s)")
    flat = ids.reshape(-1)
    s = timed(lambda: table.index_select(0, flat), a.iters)
    print(f"torch index_select of the T rows: {s:.1f} us ({(T * 8 + 2 * T * D * 4) * gb / (s * 1e-6):.0f} GB/s)")
    src = table[:T]
    c = timed(lambda: src.clone(), a.iters)
    print(f"sequential copy of T rows: {c:.1f} us ({2 * T * D * 4 * gb / (c * 1e-6):.0f} GB/s)")


if __name__ == "__main__":
    main()
