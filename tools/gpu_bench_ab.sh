# Tests, then bench.py alternated between the in-tree library and tools/variants/libasme_mi_$V.so (each GPU step
# under its own limit; a failure ends the script).  TESTS="..." VARIANTS="a b" [ROUNDS=2]
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider $TESTS > gpurun_out/tab.log 2>&1
rc=$?; tail -3 gpurun_out/tab.log; [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq ${ROUNDS:-2}); do
 for lib in recsys-22-user-attributes-recommender_amd/libasme_mi.so ${VARIANTS:-}; do
  ASME_MI_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --full-json gpurun_out/bab_full.json ${BENCH_ARGS:-} > gpurun_out/bab.log 2>&1 || exit 1
  python - "$lib" ${KERNELS:-} <<'P'
import json, sys
j = json.load(open("gpurun_out/bab_full.json"))
ks = {r["kernel"]: r["avg_ms"] for r in j.get("rooflines", []) + (j.get("eval") or {}).get("rooflines", [])}
keys = ["asme_lazy_adam_stage", "asme_embedding_ln_fwd", "asme_embedding_ln_bwd"] + sys.argv[2:]
print(sys.argv[1].split("/")[-1], j["value"], j["ms_per_step"], "flush", j.get("flush_ms"),
      "eval", (j.get("eval") or {}).get("value"),
      " ".join(f"{k.replace('asme_', '')}={ks.get(k)}" for k in keys))
P
 done
done
