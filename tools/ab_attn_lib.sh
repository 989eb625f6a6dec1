#!/bin/bash
# A/B of the fused attention between the default libgrl and diag builds,
# interleaved (tools/probe_attn.py: fwd and fwd+bwd at large N):
#   tools/ab_attn_lib.sh NAME...   (diag/libgrl_NAME.so built by tools/build_diag.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L=graph-representation-learning_amd/grl
rm -f /tmp/ab_attn_ref.pt.*
export AB_SAVE=/tmp/ab_attn_ref.pt  # out and grads compared bitwise with the first (default) library's
for rep in 1 2; do
  for lib in $L/libgrl.so $(for n in "$@"; do echo $L/diag/libgrl_$n.so; done); do
    echo "$lib" >> gpurun_out/ab_attn_lib.log
    GRL_LIB_PATH=$lib timeout -k 10 200 python tools/probe_attn.py ${ATTN_N:-16384 65536 131072} \
      >> gpurun_out/ab_attn_lib.log 2>&1 || exit 1
  done
done
