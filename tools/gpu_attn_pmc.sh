#!/bin/bash
# SQ counters of the attention kernels (bf16x6 mode 0 vs fp32 resident mode 2) at the bench shape
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
for M in 0 2; do
  PMC_CMD="python tools/attn_bench.py --iters 3 --mode $M" PMC_REGEX="attn" TAG=attn$M tools/pmc_generic.sh || exit $?
  python tools/pmc_summary.py gpurun_out/pmc_attn$M attn
done
