#!/bin/bash
# A/B of attention path options in one library, interleaved, two rounds:
#   tools/ab_attn_opt.sh "attn_dh16=0" "attn_dh16=1"   (ATTN_N: the N values)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for rep in 1 2; do
  for o in "$@"; do
    timeout -k 10 200 python tools/probe_attn.py ${ATTN_N:-100000 131072} $o >> gpurun_out/ab_attn_opt.log 2>&1 || exit 1
  done
done
