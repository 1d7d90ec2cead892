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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3, help="alternations of the modes (same process: A/B without box drift)")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seq", type=int, default=200)
    ap.add_argument("--heads", type=int, default=2)
    ap.add_argument("--dk", type=int, default=64)
    ap.add_argument("--bidir", action="store_true")
    ap.add_argument("--modes", default="0,1", help="attention kernel families to alternate (ops.attention kernels=): 0 auto (resident "
                                                   "kernels where the head fits LDS), 1 streaming")
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
    modes = [int(m) for m in a.modes.split(",")]
    res = {m: ([], []) for m in modes}
    for rep in range(a.reps):
        for mode in modes:
            for it in range(a.iters + 2):
                ev[0].record()
                out = asme.ops.attention(qkv, valid, H, causal, a.dropout, kernels=mode)
                ev[1].record()
                out.backward(g)
                ev[2].record()
                torch.cuda.synchronize()
                if it >= 2:
                    res[mode][0].append(ev[0].elapsed_time(ev[1]))
                    res[mode][1].append(ev[1].elapsed_time(ev[2]))
                qkv.grad = None
    unit = 2.0 * B * H * dk * (L * (L + 1) / 2 if causal else L * L)  # one causal-aware matmul pass
    for mode in modes:
        tf, tb = sorted(res[mode][0]), sorted(res[mode][1])
        f, b = tf[len(tf) // 2], tb[len(tb) // 2]
        print(f"mode {mode} {'bidir' if a.bidir else 'causal'}: fwd {f * 1e3:.1f} us ({2 * unit / f / 1e9:.1f} TF/s)"
              f"   bwd {b * 1e3:.1f} us ({5 * unit / b / 1e9:.1f} TF/s at 5 passes)  (medians)")


if __name__ == "__main__":
    main()
