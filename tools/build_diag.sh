#!/bin/bash
# Build libgrl variants with extra -D flags for A/B probes:
#   tools/build_diag.sh NAME "-DFLAG=1 ..." [SOURCE]  -> graph-representation-learning_amd/grl/diag/libgrl_NAME.so
# SOURCE (default linear) is the csrc/*.hip file rebuilt with the flags.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/graph-representation-learning_amd/csrc
OUT=$ROOT/graph-representation-learning_amd/grl/diag
OBJ=$ROOT/build/diag_$1
mkdir -p "$OUT" "$OBJ"
make -s -C "$CS" >/dev/null
SRC=${3:-linear}
SRCFILE=$CS/$SRC.hip
if [ -f "$SRC" ]; then SRCFILE=$SRC; SRC=$(basename "$SRC" .hip); fi  # a file elsewhere (e.g. an older revision)
cp "$ROOT"/build/obj/*.o "$OBJ/"
EXTRA=""
[ "$SRC" = attention ] && EXTRA="-mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize"  # as the Makefile builds it
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" -I"$CS" -Wno-unused-result -DGRL_DIAG $EXTRA $2 -c "$SRCFILE" -o "$OBJ/$SRC.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libgrl_$1.so" "$OBJ"/*.o -L/opt/rocm/lib -lrocprofiler-sdk-roctx
echo "$OUT/libgrl_$1.so"
