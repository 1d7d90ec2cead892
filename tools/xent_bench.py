"""Fused logits head + cross-entropy at the BERT4Rec C3 shape: the training form (dH folded into the forward:
asme_linear_xent_fwd_dh + asme_linear_xent_bwd_dw) against the two-pass form (asme_linear_xent_fwd +
asme_linear_xent_bwd), alternated in one process, and the materialised path.

Usage: python tools/xent_bench.py [--rows M] [--items V] [--dim d]
M defaults to the expected non-ignored rows of a B=1024, L=200 cloze batch (0.9*0.2*T + 0.1*B = 36,966).
Executed FLOP per step: two-pass 2 (fwd) + 8 (bwd: dH and dW each recompute the logits) MVd; training form
4 (fwd: logits + dH) + 4 (bwd: logits recompute + dW) MVd; algorithmic 6 MVd (the logits GEMM and its two
gradient GEMMs).
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import __graft_entry__  # noqa: E402

PEAK = 2516.6 / 6  # bf16x6: dense bf16 MFMA peak / 6 (csrc/logits.hip)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=36966)
    ap.add_argument("--items", type=int, default=27003)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    asme = __graft_entry__.load_package()
    dev = torch.device("cuda", 0)
    M, V, d = a.rows, a.items, a.dim
    torch.manual_seed(0)
    h = (torch.randn(M, d, device=dev) * 0.3).requires_grad_(True)
    W = (torch.randn(V, d, device=dev) * 0.3).requires_grad_(True)
    b = (torch.randn(V, device=dev) * 0.1).requires_grad_(True)
    t = torch.randint(3, V, (M,), device=dev)
    mvd = float(M) * V * d
    names = {True: ("asme_linear_xent_fwd_dh", "asme_linear_xent_bwd_dw"),
             False: ("asme_linear_xent_fwd", "asme_linear_xent_bwd")}
    res = {True: ([], []), False: ([], [])}
    for _ in range(a.reps):
        for form in (True, False):
            asme.ops.XENT_TRAINING_FORM = form
            with asme._lib.KernelTimer(list(names[form])) as kt:
                for _ in range(a.iters + 1):
                    loss = asme.ops.linear_cross_entropy(h, W, b, t, 0)
                    loss.backward()
            st = kt.summary()
            res[form][0].append(st[names[form][0]]["avg_ms"])
            res[form][1].append(st[names[form][1]]["avg_ms"])
    asme.ops.XENT_TRAINING_FORM = True
    for form, (fx, bx) in ((True, (4, 4)), (False, (2, 8))):
        f, bw = statistics.median(res[form][0]), statistics.median(res[form][1])
        label = "training form" if form else "two-pass form"
        print(f"{label}: fwd {f:.3f} ms ({fx * mvd / f / 1e9:.1f} TF/s executed, {fx * mvd / f / 1e9 / PEAK:.2f}), "
              f"bwd {bw:.3f} ms ({bx * mvd / bw / 1e9:.1f} TF/s executed, {bx * mvd / bw / 1e9 / PEAK:.2f}); "
              f"step {f + bw:.3f} ms, algorithmic {6 * mvd / (f + bw) / 1e9:.1f} TF/s "
              f"({6 * mvd / (f + bw) / 1e9 / PEAK:.2f} of the bf16x6 ceiling)")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for i in range(a.iters + 1):
        if i == 1:
            ev[0].record()
        logits = F.linear(h, W, b)
        loss = asme.ops.cross_entropy(logits, t, 0)
        loss.backward()
        del logits, loss
    ev[1].record()
    torch.cuda.synchronize()
    m = ev[0].elapsed_time(ev[1]) / a.iters
    print(f"materialised (library GEMM {M * V * 4 / 1e9:.1f} GB logits + CE kernels + 2 GEMMs): {m:.3f} ms/step "
          f"({6 * mvd / m / 1e9:.1f} TF/s algorithmic)")


if __name__ == "__main__":
    main()
