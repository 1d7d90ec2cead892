set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lazy or adam or sparse or sharded or flush" > gpurun_out/t.log 2>&1; echo "tests rc=$?" >> gpurun_out/t.log
for i in 1 2; do
ASME_MI_LIB=$PWD/tools/probe/ab/libasme_head.so timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bA$i.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bB$i.log 2>&1 || exit 1
done
