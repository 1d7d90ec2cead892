set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${TESTS:-tests/test_gpu_sharded_multirank.py tests/test_gpu_kernels.py tests/test_gpu_eval.py tests/test_gpu_optim.py} > gpurun_out/t5.log 2>&1
rc=$?; tail -5 gpurun_out/t5.log; [ $rc -le 1 ] || exit $rc
if [ -n "${BENCH_ARGS:-}" ]; then
timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/b5.log 2>&1 || exit $?
python - <<'P'
import json
j=json.loads(open("gpurun_out/b5.log").read().strip().splitlines()[-1])
print(j["value"], j["ms_per_step"], j.get("flush_ms"))
for r in j["rooflines"]: print("  ", r["kernel"], r["avg_ms"], r["frac"], r["launches"])
P
fi
