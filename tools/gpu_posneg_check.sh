set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
TESTS="tests/test_gpu_batches.py tests/test_gpu_models.py" ROUNDS=1 bash tools/gpu_bench_ab.sh || exit $?
python - <<'P'
import json
j = json.loads(open("gpurun_out/bab.log").read().strip().splitlines()[-1])
print("posneg ms", {r["kernel"]: r["avg_ms"] for r in j["rooflines"]}.get("asme_posneg_sample"))
P
