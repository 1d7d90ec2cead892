#!/bin/bash
# 16x16x32 CE gradient passes: xent tests, then C3-shape A/B vs the 32x32x16 kernel and vs no-SLP; ws GEMM no-SLP A/B
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_xent.py > gpurun_out/r4h_t.log 2>&1
rc=$?; tail -2 gpurun_out/r4h_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "csr or dedup or table_grad" > gpurun_out/r4h_csr.log 2>&1
rc=$?; tail -2 gpurun_out/r4h_csr.log; [ $rc -eq 0 ] || exit $rc
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so
for lib in $NEW tools/variants/libasme_mi_m32.so tools/variants/libasme_mi_lgnoslp.so $NEW tools/variants/libasme_mi_m32.so tools/variants/libasme_mi_lgnoslp.so; do
  echo "== xent $lib"; ASME_MI_LIB=$lib timeout -k 10 120 python tools/xent_bench.py --reps 2 --iters 3 2>&1 | grep -E "training form" || exit 1
done
timeout -k 10 300 python tools/ws_ab.py $NEW tools/variants/libasme_mi_wsnoslp.so --reps 5 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attention or attn" > gpurun_out/r4h_ta.log 2>&1
rc=$?; tail -2 gpurun_out/r4h_ta.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for lib in $NEW tools/variants/libasme_mi_attnc1.so; do
  echo "== attn $lib"; ASME_MI_LIB=$lib timeout -k 10 200 python tools/attn_bench.py --modes 0 --reps 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  ASME_MI_LIB=$lib timeout -k 10 200 python tools/attn_bench.py --modes 0 --reps 2 --bidir 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/zipf_kt -o run --output-format csv -- \
    python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --legs none --ids zipf > gpurun_out/zipf_kt.log 2>&1 || exit $?
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/zipf_kt/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e3:10.1f} us {int(r["Calls"]):5d}x {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:80]}')
PY
for i in 1 2; do for lib in $NEW tools/variants/libasme_mi_shold.so; do
  ASME_MI_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --legs none --ids zipf > gpurun_out/zab.json 2> gpurun_out/zab.err || exit 1
  python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/zab.json").read().strip().splitlines()[-1])
r = {x["kernel"]: x["avg_ms"] for x in d["rooflines"]}
print(sys.argv[1][-22:], "zipf", d["value"], d["ms_per_step"], "dedup", r.get("asme_dedup_ids_segments"), "csr", r.get("asme_occurrence_csr"), "reduce", r.get("asme_table_grad_reduce_apply"))
PY
done; done
