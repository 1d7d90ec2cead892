set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lazy or adam or sparse or sharded" > gpurun_out/t.log 2>&1 || exit 1
for wd in 0 0.001; do for k in 13 200; do timeout -k 10 120 python tools/flush_bench.py --k $k --wd $wd >> gpurun_out/f.log 2>&1 || exit 1; done; done
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/b1.log 2>&1 || exit 1
