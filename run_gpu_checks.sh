#!/bin/bash
# GPU-box check script: every GPU step has its own time limit; a crash/fault/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 0 = pass, 1 = test failures (no fault)
timeout -k 10 ${PYTEST_TIMEOUT:-420} python -m pytest tests -m gpu -q -p no:cacheprovider -k "${PYTEST_K:-}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok $rc || exit $rc
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-420} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
fi
exit 0
