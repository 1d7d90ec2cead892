# Round-end measurement A: the whole GPU suite and smoke (as the driver runs them), then the PMC traffic passes and
# kernel traces of the three workloads (tools/pmc_all.sh, no bench line: part B runs it with the new traffic file)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
TAG=${TAG:-r3s}; OUT=gpurun_out/final_${TAG}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
TAG=$TAG BENCH= bash tools/pmc_all.sh || exit $?
