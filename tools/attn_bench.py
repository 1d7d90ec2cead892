"""Attention-only timing at the bench shape (B=1024, L=200, H=2, dk=64, causal).

Usage: python tools/attn_bench.py [--dropout P] [--iters N] [--bidir]
Prints per-call fwd / bwd times from HIP events (the bwd call launches the dQ and dK/dV kernels).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dropout", type=float, default=0.2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seq", type=int, default=200)
    ap.add_argument("--heads", type=int, default=2)
    ap.add_argument("--dk", type=int, default=64)
    ap.add_argument("--bidir", action="store_true")
    a = ap.parse_args()
    asme = __graft_entry__.load_package()
    dev = torch.device("cuda", 0)
    B, L, H, dk = a.batch, a.seq, a.heads, a.dk
    D = H * dk
    torch.manual_seed(0)
    qkv = torch.randn(B, L, 3 * D, device=dev, requires_grad=True)
    lengths = torch.randint(L // 2, L + 1, (B,), device=dev)
    valid = (torch.arange(L, device=dev).unsqueeze(0) < lengths.unsqueeze(1)).to(torch.uint8)
    g = torch.randn(B, L, D, device=dev)
    causal = not a.bidir
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf, tb = [], []
    for it in range(a.iters + 3):
        ev[0].record()
        out = asme.ops.attention(qkv, valid, H, causal, a.dropout)
        ev[1].record()
        out.backward(g)
        ev[2].record()
        torch.cuda.synchronize()
        if it >= 3:
            tf.append(ev[0].elapsed_time(ev[1]))
            tb.append(ev[1].elapsed_time(ev[2]))
        qkv.grad = None
    unit = 2.0 * B * H * dk * (L * (L + 1) / 2 if causal else L * L)  # one causal-aware matmul pass
    f = sum(tf) / len(tf)
    b = sum(tb) / len(tb)
    print(f"fwd {f * 1e3:.1f} us  ({2 * unit / f / 1e9:.1f} TF/s)   bwd {b * 1e3:.1f} us  "
          f"({5 * unit / b / 1e9:.1f} TF/s at 5 passes, {7 * unit / b / 1e9:.1f} at 7)")


if __name__ == "__main__":
    main()
