"""Print the headline, every workload and the named target kernels of a bench.py stdout line (one line each)."""
import json
import sys

line = open(sys.argv[1]).read().strip().splitlines()[-1]
r = json.loads(line)
print(f"{r['config'].get('workload')}: {r['value']} {r['unit']} {r['ms_per_step']} ms/step n_gpus={r['n_gpus']} "
      f"{r['config'].get('parallelism')} roofline {r['roofline']['kernel'] if r.get('roofline') else None} "
      f"{r['roofline']['frac'] if r.get('roofline') else None}  ({len(line)} chars)")
for name, w in (r.get("workloads") or {}).items():
    print(f"  {name}: {w['value']} {w['ms_per_step']} ms/step {w.get('parallelism')}")
if r.get("eval"):
    e = r["eval"]
    print(f"  eval: {e['value']} {e['ms_per_step']} ms/step, roofline {e.get('roofline')}")
print("  targets:", r.get("target_kernels"))
