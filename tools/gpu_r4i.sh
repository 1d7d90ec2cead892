#!/bin/bash
# dedup / CSR hash aggregation over 4 occurrences per thread: kernel tests, then the Zipf and uniform legs A/B
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "csr or dedup or table_grad or shard or bucket" > gpurun_out/r4i_t.log 2>&1
rc=$?; tail -2 gpurun_out/r4i_t.log; [ $rc -eq 0 ] || exit $rc
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so
for ids in zipf uniform; do for i in 1 2; do for lib in $NEW tools/variants/libasme_mi_hash1.so tools/variants/libasme_mi_hash2.so; do
  ASME_MI_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --legs none --ids $ids > gpurun_out/zab.json 2> gpurun_out/zab.err || exit 1
  python - "$lib" "$ids" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/zab.json").read().strip().splitlines()[-1])
r = {x["kernel"]: x["avg_ms"] for x in d["rooflines"]}
print(sys.argv[1][-22:], sys.argv[2], d["value"], d["ms_per_step"], "dedup", r.get("asme_dedup_ids_segments"), "csr", r.get("asme_occurrence_csr"), "reduce", r.get("asme_table_grad_reduce_apply"))
PY
done; done; done
