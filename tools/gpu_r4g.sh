#!/bin/bash
# -fno-slp-vectorize A/B: ws GEMM shapes (tools/ws_ab.py) and the C3-shape CE head
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so
timeout -k 10 300 python tools/ws_ab.py $NEW tools/variants/libasme_mi_wsnoslp.so --reps 5 2>&1 | grep -v amdgpu.ids || exit 1
for lib in $NEW tools/variants/libasme_mi_lgnoslp.so $NEW tools/variants/libasme_mi_lgnoslp.so; do
  echo "== xent $lib"; ASME_MI_LIB=$lib timeout -k 10 120 python tools/xent_bench.py --reps 2 --iters 3 2>&1 | grep -E "training form" || exit 1
done
