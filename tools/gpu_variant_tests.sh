#!/bin/bash
# GPU tests against the in-tree library and then against each variant library (ASME_MI_LIB), each under its own
# limit; a failure ends the script.  OUT=<dir> TESTS="..." VARIANTS="name ..." (tools/variants/libasme_mi_<name>.so)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/vtests}; mkdir -p $OUT
for v in intree ${VARIANTS:-}; do
  [ $v = intree ] && lib=recsys-22-user-attributes-recommender_amd/libasme_mi.so || lib=tools/variants/libasme_mi_$v.so
  ASME_MI_LIB=$lib timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider $TESTS > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
exit 0
