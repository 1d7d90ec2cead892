#!/bin/bash
# GPU-box pass for the BERT4Rec (C3) / KeBERT4Rec (C5) bench lines: the bench with its CPU baseline, a kernel
# trace, and PMC HBM counters (FETCH_SIZE / WRITE_SIZE in separate passes).  Usage: TAG=r2e WL=bert4rec tools/profile_masked.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r2}; WL=${WL:-bert4rec}
if [ "$WL" = bert4rec ]; then ITEMS=27000; else ITEMS=13000; fi
OUT=gpurun_out/prof_${TAG}_${WL}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --workload $WL --items $ITEMS > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
echo "bench: $(tail -c 400 $OUT/bench.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
    python bench.py --workload $WL --items $ITEMS --steps 5 --warmup 2 --cpu-baseline 0 > "$OUT/kt.log" 2>&1 || exit $?
echo "kernel trace done"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "attn|weight_grad|sum_slabs|ws_gemm|residual|logits_engine|split_planes|lce_rows|lce_finish|sum_parts" \
      -d "$OUT/pmc_$C" -o run --output-format csv -- \
      python bench.py --workload $WL --items $ITEMS --steps 2 --warmup 1 --cpu-baseline 0 > "$OUT/pmc_$C.log" 2>&1 || exit $?
  echo "pmc $C done"
done
exit 0
