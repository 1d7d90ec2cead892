"""Summarise tools/pmc_generic.sh output: python tools/pmc_summary.py gpurun_out/pmc_TAG"""
import collections
import csv
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for p in ("p1", "p2"):
    for r in csv.DictReader(open(f"{d}/{p}/run_counter_collection.csv")):
        nm = r["Kernel_Name"]
        k = (nm.split("::")[1] if "::" in nm else nm).split("(")[0][:60] + "|" + r.get("Grid_Size", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] in ("GRBM_GUI_ACTIVE", "SQ_INSTS_LDS"):
            n[(k, p)] += 1
for k, v in agg.items():
    c1, c2 = max(n[(k, "p1")], 1), max(n[(k, "p2")], 1)
    wc = v["SQ_WAVE_CYCLES"] or 1
    gui = v["GRBM_GUI_ACTIVE"] / c1 / 8
    print(f"{k}: launches {c1}/{c2}  cycles/launch {gui:.3g}  waves/SIMD {4 * v['SQ_WAVE_CYCLES'] / c1 / 1024 / max(gui, 1):.2f}")
    print(f"   wait_any {v['SQ_WAIT_ANY'] / wc:.2f} wait_inst {v['SQ_WAIT_INST_ANY'] / wc:.2f} active {v['SQ_ACTIVE_INST_ANY'] / wc:.2f}"
          f"  mfma_util {v['SQ_VALU_MFMA_BUSY_CYCLES'] / c2 / 1024 / max(gui, 1):.2f}  valu/launch {v['SQ_INSTS_VALU'] / c2:.3g}"
          f"  lds {v['SQ_INSTS_LDS'] / c2:.3g} salu {v['SQ_INSTS_SALU'] / c2:.3g} ldsconf {v['SQ_LDS_BANK_CONFLICT'] / c2:.3g}"
          f" waitinstlds {v['SQ_WAIT_INST_LDS'] / c2:.3g}")
