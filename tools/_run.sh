set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; echo "tests rc=$?" >> gpurun_out/t.log
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/b1.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/kt3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-baseline 0 > $GRAFT_REPO_ROOT/gpurun_out/kt3.log 2>&1
