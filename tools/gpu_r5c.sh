#!/bin/bash
# Round-5 A/B box: the kernel tests of the changed sources, then the 8-lane embedding forward (kernel alone, then the
# step) and the chunk-major XCD mapping of the logits engine (SASRec step + eval leg, BERT4Rec C3 head), each against
# a variant library built from the same tree (tools/build_variant.sh lpr16 / xcd0); PMC=1 adds the round's PMC passes.
# Every GPU step is time-limited; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_kernels.py tests/test_gpu_embedding_ln.py tests/test_gpu_xent.py tests/test_gpu_eval.py \
    > gpurun_out/t_ab.log 2>&1
rc=$?; tail -2 gpurun_out/t_ab.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" gpurun_out/t_ab.log | head -8; exit $rc; }
TOOL=tools/emb_ln_bench.py VARIANTS="lpr16" bash tools/gpu_ab.sh 2>&1 | grep -v "copy\|sum of" || exit 1
L=tools/variants/libasme_mi_
VARIANTS="${L}lpr16.so ${L}xcd0.so" BENCH_ARGS="--legs none --eval-steps 2" \
    KERNELS="asme_catalog_rank_x6" bash tools/gpu_bench_ab.sh || exit 1
VARIANTS="${L}xcd0.so" BENCH_ARGS="--workload bert4rec --items 27000" \
    KERNELS="asme_linear_xent_fwd_dh asme_linear_xent_bwd_dw" bash tools/gpu_bench_ab.sh || exit 1
[ "${PMC:-0}" = "1" ] || exit 0
TAG=r5 BENCH=0 bash tools/final_pass.sh > gpurun_out/fp.log 2>&1 || { tail -3 gpurun_out/fp.log; exit 1; }
tail -1 gpurun_out/fp.log
TAG=r5 bash tools/pmc_all.sh > gpurun_out/pa.log 2>&1 || { tail -3 gpurun_out/pa.log; exit 1; }
tail -1 gpurun_out/pa.log
