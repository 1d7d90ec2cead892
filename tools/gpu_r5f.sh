#!/bin/bash
# Round-5 A/B: the attention forward skipping the keep-nibble image that the family-0 backward never reads, against a
# variant that always stores it (tools/build_variant.sh nib1 attention.hip -DASME_ATTN_SKIP_NIB=0); attention tests
# first, then attn_bench (causal and bidirectional) and the SASRec / BERT4Rec steps.  A failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_kernels.py tests/test_gpu_models.py > gpurun_out/t_f.log 2>&1
rc=$?; tail -2 gpurun_out/t_f.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" gpurun_out/t_f.log | head -8; exit $rc; }
TOOL="tools/attn_bench.py --modes 0" VARIANTS="nib1" bash tools/gpu_ab.sh || exit 1
TOOL="tools/attn_bench.py --modes 0 --bidir" VARIANTS="nib1" bash tools/gpu_ab.sh || exit 1
VARIANTS="tools/variants/libasme_mi_nib1.so" BENCH_ARGS="--legs none --eval-steps 0" bash tools/gpu_bench_ab.sh || exit 1
VARIANTS="tools/variants/libasme_mi_nib1.so" BENCH_ARGS="--workload bert4rec --items 27000" bash tools/gpu_bench_ab.sh || exit 1
