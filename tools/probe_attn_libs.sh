#!/bin/bash
# A/B of libgrl variants on the attention probe: tools/probe_attn_libs.sh LIB.so... (N list in $ATTN_N)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for lib in "$@"; do
  echo "== $lib"
  GRL_LIB_PATH=$(realpath "$lib") timeout -k 10 200 python tools/probe_attn.py ${ATTN_N:-4096 16384 131072} || exit 1
done
