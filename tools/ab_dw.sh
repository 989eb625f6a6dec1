#!/bin/bash
# A/B of the x6 dW GEMM between the in-tree libgrl and diag builds, interleaved, 3 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L=graph-representation-learning_amd/grl
rm -f /tmp/ab_dw_ref.pt
for rep in 1 2 3; do
  for lib in $L/libgrl.so $(for n in "$@"; do echo $L/diag/libgrl_$n.so; done); do
    AB_SAVE=/tmp/ab_dw_ref.pt GRL_LIB_PATH=$lib timeout -k 10 200 python tools/probe_dw.py >> gpurun_out/ab_dw.log 2>&1 || exit 1
  done
done
