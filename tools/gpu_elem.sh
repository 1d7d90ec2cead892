# element-wise parity diagnostics (prints every tensor's excess; no -x so every case reports)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_elementwise.py -v -s --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/elem.log 2>&1
rc=$?; grep -E "excess|passed|failed|Error" gpurun_out/elem.log | tail -80; [ $rc -le 1 ]
