set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
run() { echo "== $1"; shift; timeout -k 10 200 "$@" 2>&1 | grep -v "amdgpu.ids"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "attention or attn" > gpurun_out/t6.log 2>&1
rc=$?; tail -2 gpurun_out/t6.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
run "permlane" python tools/attn_bench.py || exit 1
run "shfl" env ASME_MI_LIB=tools/variants/libasme_mi_shfl.so python tools/attn_bench.py || exit 1
done
