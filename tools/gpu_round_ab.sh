#!/bin/bash
# Same-box A/B of the headline step between this tree and an earlier round's tree snapshotted (with its own built
# library) under tools/variants/<SNAP>/: bench.py --legs none --eval-steps 0 [BENCH_ARGS], alternated ROUNDS times.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/round_ab}; mkdir -p $OUT
ROOT=$(pwd)
for i in $(seq ${ROUNDS:-3}); do
  for t in now ${SNAP:-r5snap}; do
    if [ $t = now ]; then d=$ROOT; else d=$ROOT/tools/variants/$t; fi
    (cd $d && timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --legs none --eval-steps 0 \
        ${BENCH_ARGS:-} --full-json $ROOT/$OUT/full_$t.json > $ROOT/$OUT/b_$t.log 2>&1) || { tail -5 $OUT/b_$t.log; exit 1; }
    python -c "import json,sys; j=json.load(open('$OUT/full_$t.json')); print('$t', j['value'], j['ms_per_step'], 'flush', j.get('flush_ms'))"
  done
done
