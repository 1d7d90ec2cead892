# weight-gradient slab sums, one thread per column: weight-gradient / model tests, then the bench alternating the
# in-tree library and the previous build
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_wsgemm.py tests/test_gpu_kernels.py -k "weight or grad or linear or wgrad" tests/test_gpu_models.py \
    > gpurun_out/slabs_t.log 2>&1
rc=$?; tail -3 gpurun_out/slabs_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in intree prev; do
    if [ $v = intree ]; then unset ASME_MI_LIB; else export ASME_MI_LIB=tools/variants/libasme_mi_$v.so; fi
    timeout -k 10 200 python bench.py --legs none --cpu-baseline 0 > gpurun_out/slabs_$v$i.json 2>gpurun_out/slabs_$v$i.err || exit $?
    python -c "import json; r=json.loads(open('gpurun_out/slabs_$v$i.json').read().strip().splitlines()[-1]); st={x['kernel']: x['avg_ms'] for x in r['rooflines']}; print('$v', r['value'], r['ms_per_step'], 'wgrad', st.get('asme_linear_weight_grad'))"
  done
done
unset ASME_MI_LIB
