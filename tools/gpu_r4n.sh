#!/bin/bash
# CE gradient passes: non-temporal partial-slab stores vs default policy (xent tests, C3-shape A/B)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_xent.py > gpurun_out/r4n_t.log 2>&1
rc=$?; tail -2 gpurun_out/r4n_t.log; [ $rc -eq 0 ] || exit $rc
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so
for lib in $NEW tools/variants/libasme_mi_nt0.so $NEW tools/variants/libasme_mi_nt0.so $NEW tools/variants/libasme_mi_nt0.so; do
  echo "== xent $lib"; ASME_MI_LIB=$lib timeout -k 10 120 python tools/xent_bench.py --reps 2 --iters 3 2>&1 | grep -E "training form" || exit 1
done
