#!/bin/bash
# A/B of the persistent GraphConv kernel: the in-tree libgrl (status word,
# sync check), the same with GRL_WS_STATUS=poison (no sync), and diag builds
# named on the command line (tools/build_diag.sh), interleaved, three rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L=graph-representation-learning_amd/grl
export AB_SAVE=/tmp/ab_ws_ref.pt
rm -f $AB_SAVE
for rep in 1 2 3; do
  timeout -k 10 200 python tools/probe_ws_status.py >> gpurun_out/ab_ws_status.log 2>&1 || exit 1
  GRL_WS_STATUS=poison timeout -k 10 200 python tools/probe_ws_status.py >> gpurun_out/ab_ws_status.log 2>&1 || exit 1
  for n in "$@"; do
    GRL_LIB_PATH=$L/diag/libgrl_$n.so timeout -k 10 200 python tools/probe_ws_status.py >> gpurun_out/ab_ws_status.log 2>&1 || exit 1
  done
done
