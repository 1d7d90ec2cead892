# HIP API + kernel trace of a short bench run (no counters), to find host syncs between kernels
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/api; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d gpurun_out/api -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 2 --cpu-baseline 0 --kernel-events off > gpurun_out/api/log.txt 2>&1 || exit $?
ls gpurun_out/api
