# kernel trace of the 1-rank sharded (RCCL) bench step
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/shtr; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/shtr -o run --output-format csv -- \
    python bench.py --sharded --steps 5 --warmup 2 --cpu-baseline 0 --kernel-events off > gpurun_out/shtr/log.txt 2>&1 || exit $?
tail -c 300 gpurun_out/shtr/log.txt
