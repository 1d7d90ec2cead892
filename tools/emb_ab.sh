#!/bin/bash
# Embedding LN kernels standalone (tools/emb_ln_bench.py) for the in-tree library and tools/variants/libasme_mi_$V.so,
# alternated ROUNDS times.  VARIANTS="a b" [ROUNDS=2]; each run under its own time limit, a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for i in $(seq ${ROUNDS:-2}); do
 for lib in recsys-22-user-attributes-recommender_amd/libasme_mi.so ${VARIANTS:-}; do
  case $lib in *.so) p=$lib;; *) p=tools/variants/libasme_mi_$lib.so;; esac
  echo "== $lib"
  ASME_MI_LIB=$p timeout -k 10 120 python tools/emb_ln_bench.py ${EMB_ARGS:-} || exit 1
 done
done
