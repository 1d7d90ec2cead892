# Weight-gradient A/B on the GPU box: the weight-grad tests, then tools/wgrad_bench.py alternating between the
# in-tree library and tools/variants/libasme_mi_$VARIANT.so (default: head)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "weight_grad" > gpurun_out/wg_t.log 2>&1
rc=$?; tail -3 gpurun_out/wg_t.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  echo "== in-tree"; timeout -k 10 200 python tools/wgrad_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== ${VARIANT:-head}"; ASME_MI_LIB=tools/variants/libasme_mi_${VARIANT:-head}.so timeout -k 10 200 python tools/wgrad_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
