#!/bin/bash
# A/B of the x6 GEMMs between the default libgrl and diag builds, interleaved,
# after the GEMM parity tests on each diag build:
#   tools/ab_gemm_lib.sh NAME...   (diag/libgrl_NAME.so built by tools/build_diag.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L=graph-representation-learning_amd/grl
for n in "$@"; do
  GRL_LIB_PATH=$L/diag/libgrl_$n.so timeout -k 10 300 python -m pytest -q -x tests/test_gpu_kernels.py \
    -k "gemm or x6 or linear" > gpurun_out/ab_gemm_tests_$n.log 2>&1 || exit 1
done
for rep in 1 2; do
  for lib in $L/libgrl.so $(for n in "$@"; do echo $L/diag/libgrl_$n.so; done); do
    echo "$lib" >> gpurun_out/ab_gemm_lib.log
    GRL_LIB_PATH=$lib timeout -k 10 200 python tools/probe_x6.py child >> gpurun_out/ab_gemm_lib.log 2>&1 || exit 1
  done
done
