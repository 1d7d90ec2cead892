set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 120 python tools/attn_bench.py >> gpurun_out/ab.log 2>&1 || exit 1
ASME_MI_LIB=$PWD/tools/probe/ab/libasme_ns.so timeout -k 10 120 python tools/attn_bench.py >> gpurun_out/ab.log 2>&1 || exit 1
done
