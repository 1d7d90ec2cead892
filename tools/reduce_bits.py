"""Bit-identity probe for the fixed-order reductions: dW / db of asme_linear_weight_grad at the bench's shapes (split-T
slabs summed by sum_slabs_kernel / sum_slabs_cols_kernel) and asme_reduce_rows at the LayerNorm-partials and wider
shapes, with fixed seeds; saves the results for comparison with another library build (ASME_MI_LIB=...).
Usage: python tools/reduce_bits.py OUT.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402


def main():
    asme = __graft_entry__.load_package()
    L = asme._lib
    dev = torch.device("cuda", 0)
    out = {}
    for (T, N, K) in [(204800, 128, 128), (204800, 384, 128), (204800, 512, 128), (204800, 128, 512), (5000, 128, 128),
                      (70000, 256, 64)]:
        torch.manual_seed(T + N + K)
        dy, x = torch.randn(T, N, device=dev), torch.randn(T, K, device=dev)
        nb = int(L.load().asme_linear_weight_grad_workspace(T, N, K))
        ws = torch.empty(nb // 4 + 1, device=dev)
        dw, db = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
        L.call("asme_linear_weight_grad", L.ptr(dy), N, L.ptr(x), K, T, N, K, L.ptr(ws), nb, L.ptr(dw), L.ptr(db), 0,
               L.stream())
        out[f"wgrad_{T}_{N}_{K}"] = (dw.cpu(), db.cpu())
    for (R, W) in [(1024, 256), (1024, 768), (2048, 512), (300, 4000), (1000, 33)]:
        torch.manual_seed(R * 7 + W)
        part = torch.randn(R, W, device=dev)
        o = torch.empty(W, device=dev)
        L.call("asme_reduce_rows", L.ptr(part), R, W, L.ptr(o), 0, L.stream())
        out[f"rows_{R}_{W}"] = (o.cpu(),)
    torch.cuda.synchronize()
    torch.save(out, sys.argv[1])
    print("saved", len(out), "results to", sys.argv[1])


if __name__ == "__main__":
    main()
