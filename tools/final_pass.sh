# Round-end measurement, part 1: the default bench line (all legs + CPU baselines) and the MFMA-busy counter passes
# (SASRec step GEMM/attention kernels; the BERT4Rec C3 logits head).  Part 2 is tools/pmc_all.sh.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
TAG=${TAG:-r3z}; OUT=gpurun_out/final_${TAG}; mkdir -p $OUT
if [ "${BENCH:-1}" != "0" ]; then
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -1 $OUT/bench.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], [(w, x['value']) for w, x in r.get('workloads', {}).items()])"
fi
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "ws_gemm|weight_grad|attn|sum_slabs" \
    -d $OUT/mfma -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --legs none --eval-steps 0 \
    --kernel-events off > $OUT/mfma.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "logits_engine|logits_grad|fdh_finish|scale_rows|lce_" \
    -d $OUT/mfma_b4r -o run --output-format csv -- python bench.py --workload bert4rec --items 27000 --steps 2 --warmup 1 \
    --cpu-baseline 0 --legs none --kernel-events off > $OUT/mfma_b4r.log 2>&1 || exit $?
python tools/pmc_mfma.py $(find $OUT/mfma -name "*counter_collection.csv") $OUT/mfma_busy.json 1024 200 10000000 128 2
python tools/pmc_mfma.py $(find $OUT/mfma_b4r -name "*counter_collection.csv") $OUT/logits_mfma_busy.json 1024 200 27003 128 2 bert4rec 36966
echo final-part1 done
