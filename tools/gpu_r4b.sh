#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_wsgemm.py > gpurun_out/r4b_t.log 2>&1
rc=$?; tail -3 gpurun_out/r4b_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ws_ab.py tools/variants/libasme_mi_ct4.so recsys-22-user-attributes-recommender_amd/libasme_mi.so --reps 5 > gpurun_out/r4b_ab.log 2>&1 || exit 1
cat gpurun_out/r4b_ab.log
bash tools/gpu_logits_diag.sh > gpurun_out/logits_diag.log 2>&1; cat gpurun_out/logits_diag.log
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "csr or dedup or table_grad" > gpurun_out/r4b_csr.log 2>&1
rc=$?; tail -3 gpurun_out/r4b_csr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --legs sasrec_zipf --cpu-baseline 0 > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r4b_bench.json").read().strip().splitlines()[-1])
print("headline", d["value"], d["ms_per_step"])
for r in d["rooflines"][:8]: print("  ", r["kernel"], r["avg_ms"], r["frac"], r["launches"])
z = d["workloads"]["sasrec_zipf"]
print("zipf", z["value"], z["ms_per_step"])
for r in z["rooflines"][:10]: print("  ", r["kernel"], r["avg_ms"], r["frac"], r["launches"])
PY
