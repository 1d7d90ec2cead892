#!/bin/bash
# Round-end pass on one box: the whole GPU suite + smoke() + the default bench line (tools/gpu_round.sh), a kernel
# trace of the headline for the step breakdown, then the counter passes (tools/round_pmc.sh).  TAG names the outputs.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
TAG=${TAG:-r6final}
OUT=gpurun_out/$TAG bash tools/gpu_round.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/kt -o run --output-format csv -- \
    python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --legs none --eval-steps 0 > gpurun_out/$TAG/kt.log 2>&1 || exit $?
echo "kernel trace done"
TAG=$TAG bash tools/round_pmc.sh || exit $?
exit 0
