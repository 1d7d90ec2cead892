#!/bin/bash
# residual + LayerNorm kernels: LN parameters loaded with the rows (forward) / staged in LDS (backward), this tree vs
# the previous commit (tools/variants/libasme_mi_normold.so): kernel + model tests, then the bench, same box
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_elementwise.py tests/test_gpu_embedding_ln.py > gpurun_out/r4z_t.log 2>&1
rc=$?; tail -1 gpurun_out/r4z_t.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/r4z_t.log; exit $rc; }
for i in 1 2 3; do
  for lib in recsys-22-user-attributes-recommender_amd/libasme_mi.so tools/variants/libasme_mi_normold.so; do echo -n "${lib: -12} "
    ASME_MI_LIB=$lib timeout -k 10 200 python tools/emb_partials_ab.py 2048 --legs none --cpu-baseline 0 2> gpurun_out/embp.err || { tail -5 gpurun_out/embp.err; exit 1; }
    python -c "import json; r=json.loads(open('gpurun_out/embp_2048.json').read().strip().splitlines()[-1]); st={x['kernel']: x['avg_ms'] for x in r['rooflines']}; print('   ln_fwd', st.get('asme_residual_ln_fwd'), 'ln_bwd', st.get('asme_residual_ln_bwd'))"
  done
done
