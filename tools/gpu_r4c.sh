#!/bin/bash
# logits gradient kernel (two-stage pipeline) vs the single-stage engine: xent tests, then the C3-shape timing
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_xent.py > gpurun_out/r4c_t.log 2>&1
rc=$?; tail -3 gpurun_out/r4c_t.log; [ $rc -eq 0 ] || exit $rc
for lib in recsys-22-user-attributes-recommender_amd/libasme_mi.so tools/variants/libasme_mi_old.so recsys-22-user-attributes-recommender_amd/libasme_mi.so tools/variants/libasme_mi_old.so; do
  echo "== $lib"
  ASME_MI_LIB=$lib timeout -k 10 120 python tools/xent_bench.py --reps 2 --iters 3 2>&1 | grep -E "form" || exit 1
done
