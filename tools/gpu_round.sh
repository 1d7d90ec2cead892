#!/bin/bash
# One GPU-box checkpoint: the GPU test suite (every step time-limited; a fault/timeout ends the script),
# smoke, then the default bench line (headline + C3/C5 legs + CPU baselines).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 \
    --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${BENCH:-1}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-500} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench.json
fi
exit 0
