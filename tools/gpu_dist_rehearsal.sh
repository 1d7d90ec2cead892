#!/bin/bash
# Multi-rank rehearsal of the bench's N > 1 path on ONE GPU over gloo (the driver runs the real N = 2..8 over RCCL on
# an 8-GPU node): the driver's own form `python bench.py --gpus N` (bench.py launches the N ranks itself), then the
# torchrun form, then the one-rank sharded path over RCCL.  OUT=gpurun_out/<tag>.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/dist}; mkdir -p $OUT
for N in ${NS:-2}; do
  timeout -k 10 400 python bench.py --gpus $N --backend gloo --legs none --cpu-baseline 0 --steps 3 --warmup 1 \
      --full-json $OUT/launch_$N.full.json > $OUT/launch_$N.json 2> $OUT/launch_$N.err || { tail -5 $OUT/launch_$N.err; exit 1; }
  python tools/bench_summary.py $OUT/launch_$N.json
done
if [ -n "${TORCHRUN:-}" ]; then
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29602 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-baseline 0 --legs none --backend gloo \
      --full-json $OUT/torchrun_2.full.json > $OUT/torchrun_2.json 2> $OUT/torchrun_2.err || { tail -5 $OUT/torchrun_2.err; exit 1; }
  python tools/bench_summary.py $OUT/torchrun_2.json
fi
