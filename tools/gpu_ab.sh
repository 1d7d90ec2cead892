# A/B of a tool between the in-tree library and tools/variants/libasme_mi_$VARIANT.so, alternating twice
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider $TESTS > gpurun_out/tab.log 2>&1
rc=$?; tail -2 gpurun_out/tab.log; [ $rc -le 1 ] || exit $rc
fi
for i in 1 2; do
  echo "== in-tree"; timeout -k 10 200 python $TOOL 2>&1 | grep -v amdgpu.ids || exit 1
  for v in $VARIANTS; do echo "== $v"; ASME_MI_LIB=tools/variants/libasme_mi_$v.so timeout -k 10 200 python $TOOL 2>&1 | grep -v amdgpu.ids || exit 1; done
done
