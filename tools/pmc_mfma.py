"""MFMA utilisation per C-ABI call from a rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE pass over bench.py:
busy = sum over the call's kernels of SQ_VALU_MFMA_BUSY_CYCLES / sum of (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs),
i.e. the fraction of all SIMD cycles of the call's kernels in which the matrix pipe was busy.
Usage: python tools/pmc_mfma.py <run_counter_collection.csv> <out.json> B L ITEMS DIM LAYERS [WORKLOAD ROWS]"""
import collections
import csv
import json
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import MAP  # noqa: E402


def main():
    path, out = sys.argv[1], sys.argv[2]
    B, L, items, dim, layers = (int(x) for x in sys.argv[3:8])
    per = collections.defaultdict(dict)  # dispatch -> counter -> value, name
    for r in csv.DictReader(open(path)):
        d = per[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["name"] = r["Kernel_Name"]
    busy = collections.defaultdict(float)
    cyc = collections.defaultdict(float)
    last = None  # kernels mapped to None belong to the call launched just before them (dispatch order)
    for _, d in sorted(per.items()):
        for rx, api, _ in MAP:
            if re.search(rx, d["name"]):
                api = api if api is not None else last
                last = api
                if api is not None:
                    busy[api] += d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
                    cyc[api] += d.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 1024
                break
    res = {api: round(busy[api] / cyc[api], 4) for api in busy if cyc[api] > 0 and busy[api] > 0}
    cfg = {"batch": B, "seq_len": L, "items": items, "dim": dim, "layers": layers}
    if len(sys.argv) > 8:  # the logits-head profile bench.py looks up for the masked workloads
        cfg = {"workload": sys.argv[8], "rows": int(sys.argv[9]), "items": items, "dim": dim}
    json.dump({"config": cfg,
               "source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE over bench.py --steps 2",
               "mfma_busy": res}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
