#!/bin/bash
# A/B of graphconv.hip builds (tools/build_diag.sh NAME "-D..." graphconv) on the
# one-kernel GraphConv, interleaved, two rounds, quick probe:
#   AB_SHAPES=256x256,512x512 tools/ab_wide.sh NAME...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L=graph-representation-learning_amd/grl
for rep in 1 2; do
  for lib in $L/libgrl.so $(for n in "$@"; do echo $L/diag/libgrl_$n.so; done); do
    GRL_LIB_PATH=$lib PROBE_QUICK=1 PROBE_SHAPES=${AB_SHAPES:-256x256,512x512} timeout -k 10 300 \
      python -u tools/probe_wide.py >> gpurun_out/ab_wide.log 2>&1 || exit 1
  done
done
