#!/bin/bash
# embedding backward: LN parameters in LDS + keep bits with the row loads (this tree) vs the previous kernel
# (tools/variants/libasme_mi_embold.so), and its grid (partial-row count) in the headline bench, same box
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_embedding_ln.py tests/test_gpu_models.py > gpurun_out/r4r_t.log 2>&1
rc=$?; tail -2 gpurun_out/r4r_t.log; [ $rc -eq 0 ] || exit $rc
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so
OLD=tools/variants/libasme_mi_embold.so
for i in 1 2; do
  for lib in $NEW $OLD; do echo -n "${lib: -12} "
    ASME_MI_LIB=$lib timeout -k 10 200 python tools/emb_partials_ab.py 2048 --legs none --cpu-baseline 0 2> gpurun_out/embp.err || { tail -5 gpurun_out/embp.err; exit 1; }
  done
  for n in 768 1536 2304 3072; do echo -n "new "
    timeout -k 10 200 python tools/emb_partials_ab.py $n --legs none --cpu-baseline 0 2> gpurun_out/embp.err || { tail -5 gpurun_out/embp.err; exit 1; }
  done
done
