set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "table_grad or sparse or lazy or sasrec" > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/b1.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $R/gpurun_out/b.log 2>&1
