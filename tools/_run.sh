set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bon$i.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 --kernel-events off > gpurun_out/boff$i.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --workload bert4rec --items 27000 --cpu-baseline 0 > gpurun_out/c3.json 2> gpurun_out/c3.err || exit 1
