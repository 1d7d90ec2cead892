#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/flush
timeout -k 10 120 python tools/flush_bench.py > gpurun_out/flush/t.txt 2>&1 || exit $?
timeout -k 10 120 python tools/flush_bench.py --k 1 >> gpurun_out/flush/t.txt 2>&1 || exit $?
cat gpurun_out/flush/t.txt
for C in FETCH_SIZE WRITE_SIZE; do
timeout -k 10 200 rocprofv3 --pmc $C --kernel-include-regex lazy -d gpurun_out/flush/$C -o run --output-format csv -- python tools/flush_bench.py > /dev/null 2>&1 || exit $?
done
PMC_CMD="python tools/flush_bench.py" PMC_REGEX=lazy TAG=flush bash tools/pmc_generic.sh
