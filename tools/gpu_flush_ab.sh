set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_optim.py tests/test_gpu_kernels.py tests/test_gpu_sharded_multirank.py > gpurun_out/tf.log 2>&1
rc=$?; tail -2 gpurun_out/tf.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
 for lib in "" tools/variants/libasme_mi_v4lazy.so; do
  echo "== ${lib:-in-tree}"
  ASME_MI_LIB=${lib:-recsys-22-user-attributes-recommender_amd/libasme_mi.so} timeout -k 10 120 python tools/flush_bench.py --k 25 --wd 1e-3 --spread 2>&1 | grep flush || exit 1
  ASME_MI_LIB=${lib:-recsys-22-user-attributes-recommender_amd/libasme_mi.so} timeout -k 10 120 python tools/flush_bench.py --k 13 --wd 1e-3 2>&1 | grep flush || exit 1
 done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bf.log 2>&1 || exit 1
python - <<'P'
import json
j=json.loads(open("gpurun_out/bf.log").read().strip().splitlines()[-1])
print(j["value"], j["ms_per_step"], j.get("flush_ms"))
for r in j["rooflines"]: print("  ", r["kernel"], r["avg_ms"], r["frac"])
P
