#!/bin/bash
# Two rocprofv3 PMC passes (separate runs, --kernel-trace free) over a command; CSVs under gpurun_out/pmc/<tag>.
# Usage (on the GPU box): tools/pmc_kernel.sh TAG python tools/xent_bench.py --iters 1
set -u
TAG="$1"; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
OUT="gpurun_out/pmc/$TAG"
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d "$OUT" -o p1 -- "$@" > "$OUT/p1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d "$OUT" -o p2 -- "$@" > "$OUT/p2.log" 2>&1 || exit $?
echo "pmc $TAG done"
