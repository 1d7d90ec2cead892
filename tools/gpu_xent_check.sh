set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_xent.py tests/test_gpu_models.py -x -q -p no:cacheprovider --timeout 200 > gpurun_out/t_xent.log 2>&1; rc=$?; tail -3 gpurun_out/t_xent.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload bert4rec --items 27000 --steps 10 --warmup 3 --cpu-baseline 0 --legs none > gpurun_out/b_bert.json 2> gpurun_out/b_bert.err || exit $?
python - <<'PY'
import json
r = json.loads(open("gpurun_out/b_bert.json").read().strip().splitlines()[-1])
print(r["value"], r["ms_per_step"])
for x in r.get("rooflines", []):
    print(x["kernel"], x["avg_ms"], x["launches"], x.get("frac"))
PY
