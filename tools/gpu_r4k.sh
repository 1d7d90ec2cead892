#!/bin/bash
# same-box A/B of the headline step: this tree's library vs the round-4a library (tools/variants/libasme_mi_r4a.so)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so
for i in 1 2 3; do for lib in $NEW tools/variants/libasme_mi_r4a.so; do
  ASME_MI_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --legs none > gpurun_out/kab.json 2> gpurun_out/kab.err || exit 1
  python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/kab.json").read().strip().splitlines()[-1])
r = {x["kernel"]: x["avg_ms"] * x["launches"] for x in d["rooflines"]}
top = sorted(r.items(), key=lambda kv: -kv[1])[:8]
print(sys.argv[1][-22:], d["value"], d["ms_per_step"], " ".join(f"{k[5:]}={v:.3f}" for k, v in top))
PY
done; done
