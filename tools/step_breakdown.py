"""Per-step kernel breakdown from a rocprofv3 kernel trace: splits the trace at each launch of a marker kernel
(default: the embedding forward, first kernel of a step) and averages the middle steps.
Usage: python tools/step_breakdown.py <run_kernel_trace.csv> [marker-substring]"""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0][:70]


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "emb_fwd4_kernel"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    steps = [(starts[k], starts[k + 1]) for k in range(len(starts) - 1)][1:]  # drop the first (warm) step
    acc = collections.defaultdict(float)
    walls = []
    for a, b in steps:
        seg = rows[a:b]
        walls.append((int(rows[b]["Start_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3)
        for r in seg:
            acc[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = len(steps)
    busy = sum(acc.values()) / n
    print(f"{n} steps, wall {sum(walls) / n:.1f} us/step, kernels {busy:.1f} us/step, gaps {sum(walls) / n - busy:.1f}")
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"{v / n:9.1f}  {k}")


if __name__ == "__main__":
    main()
