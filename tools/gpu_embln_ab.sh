# fused embedding + block-0 LayerNorm: its tests and the model parity tests, then the headline bench alternating
# ASME_FUSE_EMB_LN=1 / 0 in one box, then (if built: tools/build_variant.sh diagN wsgemm.hip -DASME_WS_DIAG=N) the ws
# GEMM diagnostic builds (tools/ws_ab.py)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_embedding_ln.py tests/test_gpu_models.py tests/test_gpu_elementwise.py > gpurun_out/embln_t.log 2>&1
rc=$?; tail -3 gpurun_out/embln_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for r in 1 0; do
    ASME_FUSE_EMB_LN=$r timeout -k 10 200 python bench.py --legs none --cpu-baseline 0 > gpurun_out/embln_b$r$i.json 2>gpurun_out/embln_b$r$i.err || exit $?
    python -c "import json; r=json.loads(open('gpurun_out/embln_b$r$i.json').read().strip().splitlines()[-1]); st={x['kernel']: x['avg_ms'] for x in r['rooflines']}; print('fuse=$r', r['value'], r['ms_per_step'], 'emb', st.get('asme_embedding_fwd'), st.get('asme_embedding_bwd'))"
  done
done
V=""; for v in 1 2 3 4; do [ -f tools/variants/libasme_mi_diag$v.so ] && V="$V tools/variants/libasme_mi_diag$v.so"; done
[ -z "$V" ] || timeout -k 10 300 python tools/ws_ab.py recsys-22-user-attributes-recommender_amd/libasme_mi.so $V --reps 3
