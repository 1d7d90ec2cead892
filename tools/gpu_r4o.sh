#!/bin/bash
# lazy-Adam replay with the per-step constants split (replay_const): parity tests, standalone flush A/B and the headline
# bench A/B against the previous adam.hip (tools/variants/libasme_mi_old.so), same box
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so
OLD=tools/variants/libasme_mi_old.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_optim.py tests/test_gpu_kernels.py -k "lazy or stage or flush or resume or sharded" > gpurun_out/r4o_tests.log 2>&1 || { tail -30 gpurun_out/r4o_tests.log; exit 1; }
tail -3 gpurun_out/r4o_tests.log
for lib in $NEW $OLD tools/variants/libasme_mi_a2.so $NEW $OLD tools/variants/libasme_mi_a2.so; do
  for a in "--k 25 --wd 1e-3 --spread" "--k 35 --wd 1e-3 --spread" "--k 25 --wd 0 --spread"; do
    echo -n "${lib: -14} $a: "; ASME_MI_LIB=$lib timeout -k 10 120 python tools/flush_bench.py $a 2>&1 | grep flush || exit 1
  done
done
for i in 1 2; do for lib in $NEW $OLD; do
  ASME_MI_LIB=$lib timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --legs none > gpurun_out/oab.json 2> gpurun_out/oab.err || exit 1
  python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/oab.json").read().strip().splitlines()[-1])
r = {x["kernel"]: x["avg_ms"] * x["launches"] for x in d["rooflines"]}
print(sys.argv[1][-14:], d["value"], d["ms_per_step"], "flush", d.get("flush_ms"), "stage", round(r.get("asme_lazy_adam_stage", 0), 3))
PY
done; done
