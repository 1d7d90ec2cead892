set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_optim.py tests/test_gpu_models.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
for wi in bert4rec:27000 kebert4rec:13000 sasrec-neg:10000000; do w=${wi%%:*}; it=${wi##*:}
timeout -k 10 300 python bench.py --workload $w --items $it --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit $?
python -c "import json;d=json.loads(open('gpurun_out/b_$w.json').read().strip().splitlines()[-1]);print('$w',d['value'],d['ms_per_step'])"
done
