#!/bin/bash
# A/B of the fused GraphConv kernel between the default libgrl and diag builds
# (tools/build_diag.sh NAME "-D..." graphconv), interleaved, two rounds:
#   tools/ab_fused_lib.sh NAME...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L=graph-representation-learning_amd/grl
for n in $([ -z "$AB_SKIP_TESTS" ] && echo "$@"); do  # parity first: the fused tests on each build
  GRL_LIB_PATH=$L/diag/libgrl_$n.so timeout -k 10 300 python -m pytest -q -x tests/test_gpu_graphconv.py -m gpu \
    -k fused > gpurun_out/ab_fused_tests_$n.log 2>&1 || { echo "tests failed on $n"; exit 1; }
done
for rep in 1 2; do
  for lib in $L/libgrl.so $(for n in "$@"; do echo $L/diag/libgrl_$n.so; done); do
    GRL_LIB_PATH=$lib timeout -k 10 200 python tools/probe_fused.py >> gpurun_out/ab_fused_lib.log 2>&1 || exit 1
  done
done
