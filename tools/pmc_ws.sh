# SQ counters of the weight-stationary GEMM at the bench step's shapes (three passes, <= 8 SQ counters each)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/pmc_ws; mkdir -p $OUT
timeout -k 10 120 python tools/ws_ab.py > $OUT/time.txt 2>&1 || exit $?
cat $OUT/time.txt
P=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  P=$((P+1))
  timeout -k 10 120 rocprofv3 --pmc $SET --kernel-include-regex "ws_gemm" -d $OUT/p$P -o run --output-format csv -- \
      python tools/ws_ab.py --reps 1 --iters 2 > $OUT/p$P.log 2>&1 || exit $?
done
python tools/pmc_summary.py $OUT ws_gemm > $OUT/summary.txt
