"""Per-step kernel breakdown from a rocprofv3 kernel trace of bench.py: the last complete step (between two
launches of the step's first kernel), launches, busy time, gaps, library kernels.
Usage: python tools/step_breakdown.py <run_kernel_trace.csv> [first-kernel regex] [stream id]
With a stream id (the training stream, 0) the step is cut on that stream's kernels only; the other streams' kernels
inside the step's span (the next batch's producer and table-id plan, bench --ids-ahead) are listed separately."""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else r"posneg_kernel"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    side = []
    if len(sys.argv) > 3:
        side = [r for r in rows if r["Stream_Id"] != sys.argv[3]]
        rows = [r for r in rows if r["Stream_Id"] == sys.argv[3]]
    idx = [i for i, r in enumerate(rows) if re.search(first, r["Kernel_Name"])]
    steps = list(zip(idx[:-1], idx[1:]))[1:]  # (the first interval holds the model set-up)

    def gaps(ab):
        x, y = ab
        span = int(rows[y]["Start_Timestamp"]) - int(rows[x]["Start_Timestamp"])
        return span - sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[x:y])

    for x, y in steps:
        print(f"step: launches {y - x}, span {(int(rows[y]['Start_Timestamp']) - int(rows[x]['Start_Timestamp'])) / 1e3:.1f} us,"
              f" gaps {gaps((x, y)) / 1e3:.1f} us")
    # the steady-state step: the one with the fewest gaps (the bench brackets the C-ABI calls of its last two timed
    # steps with HIP events, which add ~10 us per call boundary)
    a, b = min(steps, key=gaps)
    print("steady-state step below")
    span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
    busy = collections.defaultdict(float)
    calls = collections.Counter()
    for r in rows[a:b]:
        n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))[:90]
        busy[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        calls[n] += 1
    tot = sum(busy.values())
    print(f"launches {b - a}  span {span:.1f} us  busy {tot:.1f} us  gaps {span - tot:.1f} us")
    lib = [n for n in busy if "at::native" in n or "rocprim" in n or "rocclr" in n]
    print("library kernels:", ", ".join(f"{n} x{calls[n]}" for n in lib) or "none")
    for n, v in sorted(busy.items(), key=lambda x: -x[1]):
        print(f"{v:8.1f} us {calls[n]:3d}x  {n}")
    t_a, t_b = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    inside = [r for r in side if t_a <= int(r["Start_Timestamp"]) < t_b]
    if side:
        sb = collections.defaultdict(float)
        for r in inside:
            sb[re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))[:90]] += \
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"other streams inside the step: {len(inside)} launches, {sum(sb.values()):.1f} us (overlapped)")
        for n, v in sorted(sb.items(), key=lambda x: -x[1]):
            print(f"{v:8.1f} us  {n}")


if __name__ == "__main__":
    main()
