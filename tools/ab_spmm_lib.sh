#!/bin/bash
# A/B of the typed SpMM between the default libgrl and diag builds, interleaved:
#   tools/ab_spmm_lib.sh NAME...   (diag/libgrl_NAME.so built by tools/build_diag.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L=graph-representation-learning_amd/grl
for rep in $(seq 1 ${REPS:-2}); do
  for lib in $L/libgrl.so $(for n in "$@"; do echo $L/diag/libgrl_$n.so; done); do
    for f in ${DIMS:-256}; do
      GRL_LIB_PATH=$lib PROBE_F=$f timeout -k 10 200 python tools/probe_spmm_ab.py >> gpurun_out/ab_spmm_lib.log 2>&1 || exit 1
    done
  done
done
