set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_optim.py tests/test_gpu_kernels.py tests/test_gpu_models.py > gpurun_out/t2.log 2>&1
rc=$?; tail -5 gpurun_out/t2.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/b2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --producer resident > gpurun_out/b2r.log 2>&1 || exit $?
python - <<'P'
import json
for f in ("gpurun_out/b2.log","gpurun_out/b2r.log"):
    j=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, j["value"], j["ms_per_step"], j["flush_ms"])
    for r in j["rooflines"]: print("  ", r["kernel"], r["avg_ms"], r["frac"], r["launches"])
P
