#!/bin/bash
# Round-end counter passes: PMC HBM traffic + kernel-trace stats for the three bench workloads (tools/pmc_all.sh) and
# the MFMA-busy passes (SASRec step GEMM / attention kernels; the BERT4Rec C3 logits head), all without the bench line.
# TAG=r6 -> gpurun_out/pmc_${TAG}/ and gpurun_out/final_${TAG}/.  Every GPU step has its own limit; failures end it.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
TAG=${TAG:-r6}
TAG=$TAG bash tools/pmc_all.sh || exit $?
OUT=gpurun_out/final_${TAG}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "ws_gemm|weight_grad|attn|sum_slabs" \
    -d $OUT/mfma -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --legs none --eval-steps 0 \
    --kernel-events off > $OUT/mfma.log 2>&1 || exit $?
echo "mfma done"
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "logits_engine|logits_grad|fdh_finish|scale_rows|lce_" \
    -d $OUT/mfma_b4r -o run --output-format csv -- python bench.py --workload bert4rec --items 27000 --steps 2 --warmup 1 \
    --cpu-baseline 0 --legs none --kernel-events off > $OUT/mfma_b4r.log 2>&1 || exit $?
echo "mfma_b4r done"
exit 0
