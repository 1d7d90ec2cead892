#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for P in 0.2 0.0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$P -o run --output-format csv -- \
     python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --dropout $P > gpurun_out/ab_$P.log 2>&1 || exit $?
done
