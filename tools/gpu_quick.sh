# GPU tests (full suite) then a short headline bench + kernel trace of it: one box per call
set -u
mkdir -p gpurun_out
TAG=${TAG:-q}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_${TAG}.log 2>&1; rc=$?; tail -4 gpurun_out/t_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || exit $?
python -c "import json; r=json.loads(open('gpurun_out/b_${TAG}.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'], [(w, x['value'], x['ms_per_step']) for w, x in r.get('workloads', {}).items()])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${TAG} -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --legs none > gpurun_out/kt_${TAG}.log 2>&1 || exit $?
echo done
