set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
run() { echo "== $1"; shift; timeout -k 10 200 "$@" 2>&1 | grep -v "amdgpu.ids\|index_select\|sequential"; }
run "default (2048)" python tools/emb_bench.py || exit 1
run "wpe4 2048" env ASME_MI_LIB=tools/variants/libasme_mi_wpe4.so python tools/emb_bench.py || exit 1
run "wpe4 4096" env ASME_MI_LIB=tools/variants/libasme_mi_wpe4.so python tools/emb_bench.py --partials 4096 || exit 1
run "wpe5 2560" env ASME_MI_LIB=tools/variants/libasme_mi_wpe5.so python tools/emb_bench.py --partials 2560 || exit 1
run "wpe5 5120" env ASME_MI_LIB=tools/variants/libasme_mi_wpe5.so python tools/emb_bench.py --partials 5120 || exit 1
