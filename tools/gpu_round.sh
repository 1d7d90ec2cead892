#!/bin/bash
# One GPU-box checkpoint, as the driver runs it at round end: the whole GPU suite, smoke(), then the default bench
# line.  OUT=gpurun_out/<tag> (default gpurun_out/round); BENCH_ARGS extra bench flags; BENCH=0 skips the bench.
# Every GPU step runs under its own time limit; a fault / timeout / abort ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/round}; mkdir -p $OUT
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
if [ "${BENCH:-1}" != "0" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --full-json $OUT/bench_full.json ${BENCH_ARGS:-} \
      > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
  python tools/bench_summary.py $OUT/bench.json
fi
exit 0
