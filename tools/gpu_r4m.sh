#!/bin/bash
# same-box, same-process-launcher overhead of the row-sharded path at one rank (1-rank RCCL group) against the
# unsharded step: alternated three times (torchrun with one process for both, so the launcher is the same)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do for mode in plain sharded; do
  extra=""; [ $mode = sharded ] && extra="--sharded"
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 \
      bench.py --steps 20 --warmup 5 --cpu-baseline 0 --legs none $extra > gpurun_out/sh_$mode.json 2> gpurun_out/sh_$mode.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/sh_$mode.json').read().strip().splitlines()[-1]); print('$mode', d['value'], d['ms_per_step'], d['config']['parallelism'])"
done; done
