#!/bin/bash
# GPU-box profiling pass for one round: bench (with CPU baseline), kernel-trace stats, and PMC HBM
# counters (FETCH_SIZE / WRITE_SIZE in separate passes, as MI355X_MICROARCH.md prescribes).
# Usage: TAG=r1 tools/profile_round.sh      (each GPU step has its own limit; failures end the script)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r1}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
echo "bench: $(tail -c 300 $OUT/bench.json)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
    python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --legs none > "$OUT/kt.log" 2>&1 || exit $?
echo "kernel trace done"
if [ -n "${PMC:-1}" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex "${PMC_REGEX:-asme|attn|emb|lazy|adam|residual|gelu|ln_|weight_grad|sum_slabs|ws_gemm|sampled|posneg|claim|flag|compact|inverse|dedup|csr_|grad_chunk|grad_span}" \
        -d "$OUT/pmc_$C" -o run --output-format csv -- \
        python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --legs none > "$OUT/pmc_$C.log" 2>&1 || exit $?
    echo "pmc $C done"
  done
fi
exit 0
