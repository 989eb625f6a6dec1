#!/bin/bash
# A/B of an env switch on the attention probe, interleaved, 3 rounds:
#   tools/ab_env.sh VAR    (runs VAR=1 then VAR=0; N from ATTN_N)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for rep in 1 2 3; do
  for v in 1 0; do
    echo "== $1=$v" >> gpurun_out/ab_env.log
    env "$1=$v" timeout -k 10 200 python tools/probe_attn.py ${ATTN_N:-100000 16384} >> gpurun_out/ab_env.log 2>&1 || exit 1
  done
done
