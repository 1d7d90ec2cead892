set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "weight_grad" > gpurun_out/t.log 2>&1; echo "tests rc=$?" >> gpurun_out/t.log
