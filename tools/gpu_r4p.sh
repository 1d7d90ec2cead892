#!/bin/bash
# flush tiling variants after the constants left the replay loop, and one PMC pass over the flush kernel
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out/r4p
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so
for i in 1 2; do for lib in $NEW tools/variants/libasme_mi_pf6.so tools/variants/libasme_mi_pf8.so tools/variants/libasme_mi_rpw32.so tools/variants/libasme_mi_rpw8.so; do
  echo -n "${lib: -16}: "; ASME_MI_LIB=$lib timeout -k 10 120 python tools/flush_bench.py --k 25 --wd 1e-3 --spread 2>&1 | grep flush || exit 1
done; done
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex lazy_pipe -d gpurun_out/r4p/pmc -o run --output-format csv -- python tools/flush_bench.py --k 25 --wd 1e-3 --spread > gpurun_out/r4p/pmc.txt 2>&1 || exit 1
F=$(find gpurun_out/r4p/pmc -name "*counter_collection.csv" -print -quit)
python - "$F" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
per = collections.defaultdict(dict)
for (d, c), v in agg.items():
    per[d][c] = sum(v)
for d, cs in sorted(per.items(), key=lambda kv: int(kv[0]))[-2:]:
    print(d, {k: f"{v:.4g}" for k, v in sorted(cs.items())})
PY
