"""Summarise tools/pmc_kernel.sh CSVs: per kernel (name filter), counters averaged over its dispatches, and
derived fractions (MFMA busy of all SIMD cycles, wave-cycle split)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pat not in k:
            continue
        agg[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    v = {n: sum(x) / len(x) for n, x in c.items()}
    out = {n: f"{x:.4g}" for n, x in sorted(v.items())}
    if "GRBM_GUI_ACTIVE" in v and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
        simd_cycles = v["GRBM_GUI_ACTIVE"] / 8 * 1024
        out["mfma_busy_frac"] = f"{v['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:.3f}"
    if "SQ_WAVE_CYCLES" in v:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS"):
            if n in v:
                out[n + "_frac"] = f"{v[n] / v['SQ_WAVE_CYCLES']:.3f}"
    print(k)
    for n, x in out.items():
        print(f"   {n} = {x}")
