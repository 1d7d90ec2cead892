# one rocprofv3 counter pass (MFMA busy + GPU active cycles) over a short bench run
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/mfma; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "ws_gemm|weight_grad|attn|sum_slabs" \
    -d gpurun_out/mfma -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/mfma/log.txt 2>&1 || exit $?
find gpurun_out/mfma -name "*counter_collection.csv"
