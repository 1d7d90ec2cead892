#!/bin/bash
# SQ counter passes over the C3-shape CE head (tools/xent_bench.py): gradient-pass kernel vs the single-stage engine
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
for V in new old; do
  if [ $V = new ]; then LIB=recsys-22-user-attributes-recommender_amd/libasme_mi.so; else LIB=tools/variants/libasme_mi_old.so; fi
  ASME_MI_LIB=$LIB PMC_CMD="python tools/xent_bench.py --reps 1 --iters 2" PMC_REGEX="logits_(grad|engine)_kernel" TAG=$V \
      bash tools/pmc_generic.sh || exit $?
  python tools/pmc_summary.py gpurun_out/pmc_$V logits > gpurun_out/pmc_$V.txt; cat gpurun_out/pmc_$V.txt
done
