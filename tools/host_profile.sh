# host-side cost of issuing a training step: cProfile over bench.py (steps only dominate the call counts)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/host.prof bench.py --steps 20 --warmup 3 --legs none \
    --cpu-baseline 0 --kernel-events off > gpurun_out/host_bench.json 2> gpurun_out/host_bench.err || exit $?
python - <<'PY'
import pstats, json
r = json.loads(open("gpurun_out/host_bench.json").read().strip().splitlines()[-1])
print("value", r["value"], "ms", r["ms_per_step"], "host_issue_ms", r["host_issue_ms"])
p = pstats.Stats("gpurun_out/host.prof")
p.sort_stats("tottime").print_stats(35)
PY
