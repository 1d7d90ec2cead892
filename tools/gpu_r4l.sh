#!/bin/bash
# embedding backward without the LN2 registers (template flag): embedding tests, then the headline step A/B against
# the previous kernel (embold) and a 4-waves-per-SIMD build (embwpe4)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_embedding_ln.py tests/test_gpu_kernels.py -k "emb or Emb or gather" > gpurun_out/r4l_t.log 2>&1
rc=$?; tail -2 gpurun_out/r4l_t.log; [ $rc -eq 0 ] || exit $rc
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so
for i in 1 2 3; do for lib in $NEW tools/variants/libasme_mi_embc.so; do
  ASME_MI_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --legs none > gpurun_out/lab.json 2> gpurun_out/lab.err || exit 1
  python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/lab.json").read().strip().splitlines()[-1])
r = {x["kernel"]: (x["avg_ms"], x["frac"]) for x in d["rooflines"]}
print(sys.argv[1][-24:], d["value"], d["ms_per_step"], "emb_bwd", r.get("asme_embedding_ln_bwd"), "emb_fwd", r.get("asme_embedding_ln_fwd"))
PY
done; done
