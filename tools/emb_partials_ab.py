"""A/B of the embedding backward's partial-row count (= its grid: one LN-partial row per workgroup) in the headline
bench: python tools/emb_partials_ab.py N [bench args...] runs bench.py with ops._EMB_PARTIALS = N and prints the
step rate and the embedding kernels' times."""
import json
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402


def main():
    n = int(sys.argv[1])
    asme = __graft_entry__.load_package()
    asme.ops._EMB_PARTIALS = n
    out = os.path.join("gpurun_out", f"embp_{n}.json")
    sys.argv = ["bench.py"] + sys.argv[2:]
    real_stdout = sys.stdout
    with open(out, "w") as f:
        sys.stdout = f
        try:
            runpy.run_path("bench.py", run_name="__main__")
        finally:
            sys.stdout = real_stdout
    r = json.loads(open(out).read().strip().splitlines()[-1])
    st = {x["kernel"]: x["avg_ms"] for x in r["rooflines"]}
    print(f"partials {n}: {r['value']} seq/s {r['ms_per_step']} ms  emb_ln_bwd {st.get('asme_embedding_ln_bwd')} "
          f"reduce_rows {st.get('asme_reduce_rows')}", flush=True)


if __name__ == "__main__":
    main()
