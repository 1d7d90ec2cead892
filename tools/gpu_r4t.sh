#!/bin/bash
# embedding backward: LN2's w / b in LDS as well (this tree), + a third wave per SIMD (tools/variants/libasme_mi_w3.so,
# amdgpu_waves_per_eu 3), against the previous commit (tools/variants/libasme_mi_embold.so), same box
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for lib in recsys-22-user-attributes-recommender_amd/libasme_mi.so tools/variants/libasme_mi_w3.so; do
  ASME_MI_LIB=$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
      tests/test_gpu_embedding_ln.py tests/test_gpu_models.py > gpurun_out/r4t_t.log 2>&1
  rc=$?; tail -1 gpurun_out/r4t_t.log; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for lib in recsys-22-user-attributes-recommender_amd/libasme_mi.so tools/variants/libasme_mi_w3.so tools/variants/libasme_mi_embold.so; do echo -n "${lib: -12} "
    ASME_MI_LIB=$lib timeout -k 10 200 python tools/emb_partials_ab.py 2048 --legs none --cpu-baseline 0 2> gpurun_out/embp.err || { tail -5 gpurun_out/embp.err; exit 1; }
  done
done
