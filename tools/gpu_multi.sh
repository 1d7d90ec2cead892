#!/bin/bash
# One GPU call, several steps (each under its own limit; a failure ends the script), outputs under $OUT:
#   TESTS / PYTEST_K        pytest selection                      -> $OUT/pytest.log
#   EMB_VARIANTS            tools/emb_ab.sh over these variants   -> $OUT/emb_ab.txt
#   WS_VARIANTS             tools/ws_ab.py over these variants    -> $OUT/ws_ab.txt  (WS_ONLY: --only shapes)
#   ATTN_VARIANTS           tools/attn_bench.py per library       -> $OUT/attn_ab.txt
#   BENCH_VARIANTS          tools/gpu_bench_ab.sh over libraries   -> stdout
#   BENCH_FLAGSETS          tools/gpu_flag_ab.sh flag sets         -> stdout
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/multi}; mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  KARGS=(); [ -n "${PYTEST_K:-}" ] && KARGS=(-k "$PYTEST_K")
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      $TESTS "${KARGS[@]}" > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${EMB_VARIANTS:-}" ]; then
  VARIANTS="$EMB_VARIANTS" EMB_ARGS="${EMB_ARGS:---basic --iters 30}" bash tools/emb_ab.sh > $OUT/emb_ab.txt 2>&1 || exit 1
  grep -v amdgpu.ids $OUT/emb_ab.txt
fi
if [ -n "${WS_VARIANTS:-}" ]; then
  libs="recsys-22-user-attributes-recommender_amd/libasme_mi.so"
  for v in $WS_VARIANTS; do libs="$libs tools/variants/libasme_mi_$v.so"; done
  ONLY=(); [ -n "${WS_ONLY:-}" ] && ONLY=(--only "$WS_ONLY")
  timeout -k 10 300 python tools/ws_ab.py $libs --reps ${WS_REPS:-3} "${ONLY[@]}" > $OUT/ws_ab.txt 2>&1 || exit 1
  grep -v amdgpu.ids $OUT/ws_ab.txt
fi
if [ -n "${ATTN_VARIANTS:-}" ]; then
  for i in 1 2; do
    for v in intree $ATTN_VARIANTS; do
      [ $v = intree ] && lib=recsys-22-user-attributes-recommender_amd/libasme_mi.so || lib=tools/variants/libasme_mi_$v.so
      echo "== $v" >> $OUT/attn_ab.txt
      ASME_MI_LIB=$lib timeout -k 10 120 python tools/attn_bench.py --modes 0 --reps 2 ${ATTN_ARGS:-} >> $OUT/attn_ab.txt 2>&1 || exit 1
    done
  done
  grep -v amdgpu.ids $OUT/attn_ab.txt
fi
if [ -n "${BENCH_VARIANTS:-}" ]; then
  VARIANTS="$(for v in $BENCH_VARIANTS; do echo -n "tools/variants/libasme_mi_$v.so "; done)" KERNELS="${KERNELS:-}" \
      bash tools/gpu_bench_ab.sh || exit 1
fi
if [ -n "${BENCH_FLAGSETS:-}" ]; then
  FLAGSETS="$BENCH_FLAGSETS" bash tools/gpu_flag_ab.sh || exit 1
fi
exit 0
