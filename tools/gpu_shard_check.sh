# full GPU suite, then the headline step unsharded vs one-rank row-sharded (the sharded path's fixed overhead)
set -u
mkdir -p gpurun_out
TAG=${TAG:-s}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_${TAG}.log 2>&1; rc=$?; tail -3 gpurun_out/t_${TAG}.log; [ $rc -eq 0 ] || exit $rc
for mode in "" "--sharded"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --legs none $mode > gpurun_out/b_${TAG}${mode}.json 2> gpurun_out/b_${TAG}${mode}.err || exit $?
  python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2] or 'unsharded', r['value'], r['ms_per_step'], r['flush_ms'])" gpurun_out/b_${TAG}${mode}.json "$mode"
done
