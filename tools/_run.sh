set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
ASME_MI_LIB=$PWD/tools/probe/ab/libasme_head.so timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bA$i.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bB$i.log 2>&1 || exit 1
done
