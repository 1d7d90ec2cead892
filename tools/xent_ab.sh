#!/bin/bash
# Same-box A/B of the CE head passes (tools/xent_bench.py at the C3 shape) between the in-tree library and variants,
# alternated ROUNDS times.  VARIANTS="name ..." (tools/variants/libasme_mi_<name>.so); OUT=<dir>.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/xent_ab}; mkdir -p $OUT
for i in $(seq ${ROUNDS:-2}); do
  for v in intree ${VARIANTS:-}; do
    [ $v = intree ] && lib=recsys-22-user-attributes-recommender_amd/libasme_mi.so || lib=tools/variants/libasme_mi_$v.so
    echo "== $v" >> $OUT/xent_ab.txt
    ASME_MI_LIB=$lib timeout -k 10 180 python tools/xent_bench.py ${XENT_ARGS:-} >> $OUT/xent_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $OUT/xent_ab.txt
