set -u
mkdir -p gpurun_out
TAG=${TAG:-s}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sharded_multirank.py -m gpu -x -q -p no:cacheprovider --timeout 300 -k "shard or sharded or bucket or dedup or table or csr" > gpurun_out/t_${TAG}.log 2>&1; rc=$?; tail -3 gpurun_out/t_${TAG}.log; [ $rc -eq 0 ] || exit $rc
for mode in "" "--sharded"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --legs none $mode > gpurun_out/b_${TAG}${mode}.json 2> gpurun_out/b_${TAG}${mode}.err || exit $?
  python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2] or 'unsharded', r['value'], r['ms_per_step'], r['flush_ms'], r['host_issue_ms'])" gpurun_out/b_${TAG}${mode}.json "$mode"
done
