#!/bin/bash
# A/B of the dQ-in-dK attention backward (GRL_ATTN_FUSED_DQ=1, default) against
# the separate dQ kernel (=0), interleaved on one box, 3 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for rep in 1 2 3; do
  for f in 1 0; do
    echo "GRL_ATTN_FUSED_DQ=$f" >> gpurun_out/ab_fused_dq.log
    GRL_ATTN_FUSED_DQ=$f timeout -k 10 200 python tools/probe_attn.py ${ATTN_N:-100000 131072 16384} \
      >> gpurun_out/ab_fused_dq.log 2>&1 || exit 1
  done
done
