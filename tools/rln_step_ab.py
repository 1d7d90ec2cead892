"""Same-process A/B of the SASRec headline step with the attention output projection fused with its residual + pre-LN
(TransformerLayer.fuse_output_projection = True, asme_ws_linear_residual_ln) against the separate kernels (False):
bench.bench_sasrec alternated ROUNDS times, printing sequences/s, ms/step and the two affected kernels' per-call
times.  Usage: python tools/rln_step_ab.py [ROUNDS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402
import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sys.argv = [sys.argv[0], "--legs", "none", "--cpu-baseline", "0", "--eval-steps", "0", "--steps", "20"]
    args = bench.parse()
    asme = __graft_entry__.load_package()
    dev = torch.device("cuda", 0)
    layer = asme.layers.TransformerLayer
    for rnd in range(rounds):
        for fused in (True, False):
            layer.fuse_output_projection = fused
            torch.manual_seed(0)
            r = bench.bench_sasrec(args, asme, dev, 1, 0, "uniform", with_eval=False)
            ks = {x["kernel"]: x["avg_ms"] for x in r.get("rooflines", [])}
            print(f"round {rnd} fused={fused!s:5s} {r['value']:10.1f} seq/s {r['ms_per_step']:.3f} ms/step "
                  f"ws_linear_residual_ln={ks.get('asme_ws_linear_residual_ln')} residual_ln_fwd="
                  f"{ks.get('asme_residual_ln_fwd')} ws_linear={ks.get('asme_ws_linear')}", flush=True)
            torch.cuda.empty_cache()
    layer.fuse_output_projection = True


if __name__ == "__main__":
    main()
