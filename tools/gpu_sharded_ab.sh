#!/bin/bash
# Same-box A/B: the unsharded step against the 1-rank row-sharded step (an RCCL group of one: every exchange kernel
# and collective runs, the fabric does not) and its overlapped-negatives leg, alternated ROUNDS times.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/sharded_ab}; mkdir -p $OUT
for i in $(seq ${ROUNDS:-2}); do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --legs none --eval-steps 0 \
      --full-json $OUT/full_u.json > $OUT/b_u.log 2>&1 || { tail -5 $OUT/b_u.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --legs sasrec_overlap --eval-steps 0 \
      --sharded --full-json $OUT/full_s.json > $OUT/b_s.log 2>&1 || { tail -5 $OUT/b_s.log; exit 1; }
  python - $OUT <<'P'
import json, sys
u = json.load(open(f"{sys.argv[1]}/full_u.json")); s = json.load(open(f"{sys.argv[1]}/full_s.json"))
o = s["workloads"]["sasrec_overlap"]
print("unsharded", u["value"], u["ms_per_step"], "| sharded", s["value"], s["ms_per_step"], s["config"]["parallelism"],
      "| sharded+overlap", o["value"], o["ms_per_step"])
P
done
