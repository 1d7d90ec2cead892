#!/bin/bash
# Generic SQ counter passes for one python command: PMC_CMD="python tools/x.py" PMC_REGEX=... TAG=...
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-x}; mkdir -p $OUT
P=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  P=$((P+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "${PMC_REGEX}" -d $OUT/p$P -o run \
      --output-format csv -- ${PMC_CMD} > $OUT/p$P.log 2>&1 || exit $?
done
