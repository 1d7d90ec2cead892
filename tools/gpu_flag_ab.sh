#!/bin/bash
# Tests, then bench.py alternated between bench flag sets (same library, same process order each round).
# TESTS="..." [PYTEST_K="..."] FLAGSETS="--ids-ahead on|--ids-ahead off" [ROUNDS=2] [BENCH_ARGS=...]
# Each GPU step runs under its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
KARGS=(); [ -n "${PYTEST_K:-}" ] && KARGS=(-k "$PYTEST_K")
timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider $TESTS "${KARGS[@]}" > gpurun_out/fab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
IFS='|' read -ra SETS <<< "${FLAGSETS:-}"
for i in $(seq ${ROUNDS:-2}); do
 for k in "${!SETS[@]}"; do
  f="${SETS[$k]}"
  timeout -k 10 240 python bench.py --steps ${STEPS:-20} --warmup 5 --cpu-baseline 0 --legs none --eval-steps 0 \
      --full-json gpurun_out/fab_full_$k.json ${BENCH_ARGS:-} $f > gpurun_out/fab_$k.log 2>&1 || { tail -5 gpurun_out/fab_$k.log; exit 1; }
  python - "$f" $k ${KERNELS:-} <<'P'
import json, sys
j = json.load(open(f"gpurun_out/fab_full_{sys.argv[2]}.json"))
ks = {r["kernel"]: r["avg_ms"] for r in j.get("rooflines", [])}
keys = sys.argv[3:]
print(f"[{sys.argv[1]}]", j["value"], j["ms_per_step"], "flush", j.get("flush_ms"), "hits", j.get("ids_ahead_hits"),
      " ".join(f"{k.replace('asme_', '')}={ks.get(k)}" for k in keys))
P
 done
done
