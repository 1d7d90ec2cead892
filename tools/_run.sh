set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/b_s.json 2> gpurun_out/b_s.err || exit $?
python -c "import json;d=json.loads(open('gpurun_out/b_s.json').read().strip().splitlines()[-1]);print('sasrec',d['value'],d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_s -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/kt_s.log 2>&1 || exit $?
echo kt done
