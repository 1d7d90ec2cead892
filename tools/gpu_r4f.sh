#!/bin/bash
# round-4 f: xent + attention kernel tests; C3-shape CE A/B; attention A/B (pipelined dK/dV vs HEAD); clock pass
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_xent.py tests/test_gpu_kernels.py -k "xent or logits or attention or attn" > gpurun_out/r4f_t.log 2>&1
rc=$?; tail -2 gpurun_out/r4f_t.log; [ $rc -eq 0 ] || exit $rc
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so
for i in 1 2; do
  for lib in $NEW tools/variants/libasme_mi_attnold.so; do
    echo "== attn $lib"; ASME_MI_LIB=$lib timeout -k 10 200 python tools/attn_bench.py --modes 0 --reps 2 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
  done
done
echo "== attn bidir"; for lib in $NEW tools/variants/libasme_mi_attnold.so; do
  ASME_MI_LIB=$lib timeout -k 10 200 python tools/attn_bench.py --modes 0 --reps 2 --bidir 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
done
for lib in $NEW tools/variants/libasme_mi_old.so $NEW tools/variants/libasme_mi_old.so; do
  echo "== xent $lib"; ASME_MI_LIB=$lib timeout -k 10 120 python tools/xent_bench.py --reps 2 --iters 3 2>&1 | grep -E "training form" || exit 1
done
