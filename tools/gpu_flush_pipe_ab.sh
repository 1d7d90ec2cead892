# A/B of the pipelined full-table flush (lazy_flush_kernel) tilings against the in-tree library, then the bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for i in 1 2; do
 for lib in recsys-22-user-attributes-recommender_amd/libasme_mi.so ${VARIANTS:-}; do
  echo "== $lib"
  ASME_MI_LIB=$lib timeout -k 10 120 python tools/flush_bench.py --k 25 --wd 1e-3 --spread 2>&1 | grep flush || exit 1
 done
done
if [ -n "${BENCH:-}" ]; then
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bf.log 2>&1 || exit 1
python - <<'P'
import json
j=json.loads(open("gpurun_out/bf.log").read().strip().splitlines()[-1])
print(j["value"], j["ms_per_step"], j.get("flush_ms"))
P
fi
