# rows-at-rest lazy Adam: the lazy tests, then the headline bench alternating ASME_REST_ROWS=1 / 0 in one box
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_kernels.py -k "lazy or staged" tests/test_gpu_optim.py > gpurun_out/rest_t.log 2>&1
rc=$?; tail -3 gpurun_out/rest_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for r in 1 0; do
    ASME_REST_ROWS=$r timeout -k 10 200 python bench.py --legs none --cpu-baseline 0 > gpurun_out/rest_b$r$i.json 2>gpurun_out/rest_b$r$i.err || exit $?
    python -c "import json; r=json.loads(open('gpurun_out/rest_b$r$i.json').read().strip().splitlines()[-1]); st=[x for x in r['rooflines'] if x['kernel']=='asme_lazy_adam_stage']; print('rest=$r', r['value'], r['ms_per_step'], 'flush', r['flush_ms'], 'stage', st[0]['avg_ms'] if st else None)"
  done
done
