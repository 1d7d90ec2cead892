#!/bin/bash
# Build an A/B variant of libasme_mi.so: recompile ONE source with extra defines, link with the other objects.
# Usage: tools/build_variant.sh NAME SOURCE.hip "-DFOO=1 ..."   -> tools/variants/libasme_mi_NAME.so
# Run a tool against it with ASME_MI_LIB=tools/variants/libasme_mi_NAME.so (same process layout as the product).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
CSRC="$ROOT/recsys-22-user-attributes-recommender_amd/csrc"
NAME="$1"; SRC="$2"; DEFS="${3:-}"
make -C "$CSRC" -s -j8 >/dev/null
OBJ="/tmp/asme_variant_${NAME}.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics $DEFS -c "$CSRC/$SRC" -o "$OBJ"
SRCS=$(sed -n "s/^SRCS := //p" "$CSRC/Makefile")
OBJS=""
for s in $SRCS; do [ "$s" = "$SRC" ] || OBJS="$OBJS $CSRC/build/$s.o"; done
mkdir -p "$ROOT/tools/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS "$OBJ" -o "$ROOT/tools/variants/libasme_mi_${NAME}.so"
echo "$ROOT/tools/variants/libasme_mi_${NAME}.so"
