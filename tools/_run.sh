set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload bert4rec --items 27000 --cpu-baseline 0 > gpurun_out/c3.json 2> gpurun_out/c3.err || exit 1
timeout -k 10 300 python bench.py --workload kebert4rec --items 13000 --cpu-baseline 0 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
timeout -k 10 300 python bench.py --sharded --cpu-baseline 0 > gpurun_out/sh.json 2> gpurun_out/sh.err || exit 1
timeout -k 10 300 python bench.py --producer gpu --cpu-baseline 0 > gpurun_out/pg.json 2> gpurun_out/pg.err || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/b1.log 2>&1 || exit 1
