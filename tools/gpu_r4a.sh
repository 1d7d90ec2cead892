#!/bin/bash
# round 4, first checkpoint: the new / changed GPU tests first, then the whole suite, smoke and the bench line
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 280 --timeout-method thread \
  tests/test_gpu_sharded_multirank.py tests/test_gpu_dataparallel.py tests/test_gpu_optim.py \
  tests/test_gpu_embedding_ln.py "tests/test_gpu_models.py::test_bert4rec_anchor_ndcg" \
  "tests/test_gpu_kernels.py::test_sharded_module_single_rank_matches_unsharded" \
  -k "not multirank_matches_unsharded" > gpurun_out/r4a_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -15 gpurun_out/r4a_new.log
[ $rc -eq 0 ] || exit $rc
BENCH=1 BENCH_ARGS="--steps 20 --warmup 5" PYTEST_TIMEOUT=900 bash tools/gpu_round.sh
