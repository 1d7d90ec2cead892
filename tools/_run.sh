set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for wi in bert4rec:27000 kebert4rec:13000; do w=${wi%%:*}; it=${wi##*:}
timeout -k 10 300 python bench.py --workload $w --items $it --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit $?
python -c "import json;d=json.loads(open('gpurun_out/b_$w.json').read().strip().splitlines()[-1]);print('$w',d['value'],d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_b4r -o run --output-format csv -- python bench.py --workload bert4rec --items 27000 --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/kt_b4r.log 2>&1 || exit $?
echo kt done
