# masked-workload changes: the affected GPU tests, then the C3 / C5 bench lines
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_elementwise.py tests/test_gpu_prefetch.py \
    tests/test_gpu_xent.py > gpurun_out/rows_t.log 2>&1; rc=$?; tail -3 gpurun_out/rows_t.log; [ $rc -eq 0 ] || exit $rc
for W in bert4rec:27000 kebert4rec:13000; do
  timeout -k 10 300 python bench.py --workload ${W%%:*} --items ${W##*:} --steps 20 --warmup 5 --cpu-baseline 0 --legs none \
      > gpurun_out/rows_${W%%:*}.json 2>/dev/null || exit $?
  tail -1 gpurun_out/rows_${W%%:*}.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('${W%%:*}', r['value'], r['ms_per_step'])"
done
