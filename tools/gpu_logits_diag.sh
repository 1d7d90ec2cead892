#!/bin/bash
# fdh-pass ablations (ASME_LOGITS_DIAG builds) at the C3 shape, one process per library
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for lib in recsys-22-user-attributes-recommender_amd/libasme_mi.so tools/variants/libasme_mi_l*.so; do
  echo "== $lib"
  ASME_MI_LIB=$lib timeout -k 10 120 python tools/xent_bench.py --reps 2 --iters 3 2>&1 | grep -E "training form" || exit 1
done
