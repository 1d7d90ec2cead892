#!/bin/bash
# Attention-kernel counters at the bench shape (separate passes; no --pmc with traces).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/attn; export TMPDIR=/tmp
timeout -k 10 120 python tools/attn_bench.py > gpurun_out/attn/time.txt 2>&1 || exit $?
timeout -k 10 120 python tools/attn_bench.py --dropout 0 >> gpurun_out/attn/time.txt 2>&1 || exit $?
cat gpurun_out/attn/time.txt
rocprofv3 -L > gpurun_out/attn/counters.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/attn/kt -o run --output-format csv -- \
    python tools/attn_bench.py --iters 5 > /dev/null 2>&1 || exit $?
P=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  P=$((P+1))
  timeout -k 10 200 rocprofv3 --pmc $SET --kernel-include-regex attn -d gpurun_out/attn/pmc$P -o run \
      --output-format csv -- python tools/attn_bench.py --iters 3 > gpurun_out/attn/pmc$P.log 2>&1 || exit $?
done
