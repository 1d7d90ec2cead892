set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/b1.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 30 > gpurun_out/b2.log 2>&1
