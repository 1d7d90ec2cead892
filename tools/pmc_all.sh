# PMC HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) + kernel-trace stats for the three bench workloads.
# Usage: TAG=r3 bash tools/pmc_all.sh   (writes gpurun_out/pmc_${TAG}/<workload>/...)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r3}
export TMPDIR=/tmp
RX='asme|attn|emb_|lazy|adam|residual|gelu|ln_|weight_grad|sum_slabs|ws_gemm|sampled|posneg|claim|dedup|csr_|chained|grad_chunk|grad_span|logits_engine|logits_grad|lce_|fdh|scale_rows|split_planes|sum_parts|bce|cloze|reduce_rows|pos_partial'
for W in ${WORKLOADS:-sasrec-neg bert4rec kebert4rec}; do
  case $W in
    sasrec-neg) ARGS="--workload sasrec-neg";;
    bert4rec) ARGS="--workload bert4rec --items 27000";;
    kebert4rec) ARGS="--workload kebert4rec --items 13000";;
  esac
  OUT=gpurun_out/pmc_${TAG}/$W
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- \
      python bench.py $ARGS --steps 5 --warmup 2 --cpu-baseline 0 --legs none --eval-steps 0 > $OUT/kt.log 2>&1 || exit $?
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$RX" -d $OUT/pmc_$C -o run --output-format csv -- \
        python bench.py $ARGS --steps 2 --warmup 1 --cpu-baseline 0 --legs none --eval-steps 0 --kernel-events off > $OUT/pmc_$C.log 2>&1 || exit $?
  done
  echo "$W done"
done
