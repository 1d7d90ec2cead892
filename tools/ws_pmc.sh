#!/bin/bash
# SQ / GRBM counters of asme_ws_linear builds (tools/build_variant.sh) on one shape (effective clock = GRBM_GUI_ACTIVE / 8 / wall)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/wspmc
export TMPDIR=/tmp
SHAPE=${SHAPE:-128:512:0:0}
for lib in "$@"; do
  n=$(basename $lib .so)
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
     -d gpurun_out/wspmc/$n -o pmc --output-format csv -- python3 tools/ws_ab.py $lib --reps 1 --iters 3 --only $SHAPE > gpurun_out/wspmc/$n.log 2>&1 || exit 1
done
