#!/bin/bash
# xent tests, C3-shape A/B (gradient-pass kernel vs single-stage engine), and one clock / MFMA-busy counter pass each
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_xent.py > gpurun_out/r4e_t.log 2>&1
rc=$?; tail -2 gpurun_out/r4e_t.log; [ $rc -eq 0 ] || exit $rc
NEW=recsys-22-user-attributes-recommender_amd/libasme_mi.so; OLD=tools/variants/libasme_mi_old.so
for lib in $NEW $OLD $NEW $OLD; do
  echo "== $lib"; ASME_MI_LIB=$lib timeout -k 10 120 python tools/xent_bench.py --reps 2 --iters 3 2>&1 | grep -E "training form" || exit 1
done
for V in new old; do
  if [ $V = new ]; then LIB=$NEW; else LIB=$OLD; fi
  ASME_MI_LIB=$LIB timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "logits_(grad|engine)_kernel" \
      -d gpurun_out/clk_$V -o run --output-format csv -- python tools/xent_bench.py --reps 1 --iters 2 > gpurun_out/clk_$V.log 2>&1 || exit $?
done
python - <<'PY'
import csv, glob, collections
for tag in ("new", "old"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/clk_{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-40:]
            dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            agg[k][r["Counter_Name"]].append((float(r["Counter_Value"]), dt))
    for k, c in agg.items():
        g = c["GRBM_GUI_ACTIVE"]; m = c["SQ_VALU_MFMA_BUSY_CYCLES"]
        clk = sum(v / 8 / dt for v, dt in g) / len(g) / 1e9
        busy = sum(v for v, _ in m) / len(m) / (sum(v for v, _ in g) / len(g) / 8 * 1024)
        print(f"{tag} {k}: clock {clk:.3f} GHz, mfma busy {busy:.3f}, {sum(dt for _, dt in g) / len(g) * 1e3:.3f} ms")
PY
