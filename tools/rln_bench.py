"""A/B of the fused attention output projection + residual + pre-LN (asme_ws_linear_residual_ln) against the separate
Linear (asme_ws_linear) + asme_residual_ln_fwd at the bench shape (T = B*L = 204,800 tokens, d = 128), forward only,
same process, alternating; per-call times from HIP events on the torch stream."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib  # noqa: E402

asme = importlib.import_module("recsys-22-user-attributes-recommender_amd")


def main():
    ops = asme.ops
    dev = torch.device("cuda")
    T, d = 1024 * 200, 128
    torch.manual_seed(0)
    x = torch.randn(T, d, device=dev)
    w = torch.randn(d, d, device=dev) / d ** 0.5
    b = torch.randn(d, device=dev)
    res = torch.randn(T, d, device=dev)
    norm = torch.nn.LayerNorm(d).to(dev)

    def fused():
        return ops.linear_residual_ln(x, w, b, res, norm, 0.2, 0.0)

    def separate():
        return ops.residual_ln(res, ops.linear(x, w, b), norm, 0.2, 0.0)

    with torch.no_grad():
        for f in (fused, separate):
            for _ in range(5):
                f()
        for rnd in range(3):
            for name, f in (("fused", fused), ("separate", separate)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(50):
                    f()
                e1.record()
                torch.cuda.synchronize()
                print(f"round {rnd} {name:9s} {1000 * e0.elapsed_time(e1) / 50:7.1f} us per call", flush=True)


if __name__ == "__main__":
    main()
