#!/bin/bash
# Build libgrl variants with extra -D flags for A/B probes:
#   tools/build_diag.sh NAME "-DFLAG=1 ..."  -> graph-representation-learning_amd/grl/diag/libgrl_NAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/graph-representation-learning_amd/csrc
OUT=$ROOT/graph-representation-learning_amd/grl/diag
OBJ=$ROOT/build/diag_$1
mkdir -p "$OUT" "$OBJ"
make -s -C "$CS" >/dev/null
for f in common spmm graph attention embed; do cp "$ROOT/build/obj/$f.o" "$OBJ/"; done
cp "$ROOT/build/obj/layout_graph.o" "$OBJ/"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" -Wno-unused-result $2 -c "$CS/linear.hip" -o "$OBJ/linear.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libgrl_$1.so" "$OBJ"/*.o
echo "$OUT/libgrl_$1.so"
