# Round-end measurement B: the whole GPU suite and smoke on the final code, then the default bench line (all legs,
# CPU baselines) and the MFMA-busy passes (tools/final_pass.sh), then a kernel trace of the headline bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
TAG=${TAG:-r3s}; OUT=gpurun_out/final_${TAG}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
TAG=$TAG bash tools/final_pass.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- \
    python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --legs none > $OUT/kt.log 2>&1 || exit $?
echo final-b done
