#!/bin/bash
# A/B of attention builds AND path options, interleaved, two rounds:
#   tools/ab_attn_mix.sh "-" "-:attn_dh16=1" "dh_hpf" ...
# each entry is LIB[:NAME=VALUE...]; LIB "-" is the default libgrl, else
# diag/libgrl_LIB.so (tools/build_diag.sh); ATTN_N: the N values
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
L=graph-representation-learning_amd/grl
for rep in 1 2; do
  for e in "$@"; do
    lib=${e%%:*}; opts=""; [ "$lib" != "$e" ] && opts=$(echo "${e#*:}" | tr ':' ' ')
    path=$L/libgrl.so; [ "$lib" != "-" ] && path=$L/diag/libgrl_$lib.so
    echo "== $e" >> gpurun_out/ab_attn_mix.log
    GRL_LIB_PATH=$path timeout -k 10 200 python tools/probe_attn.py ${ATTN_N:-100000} $opts \
      >> gpurun_out/ab_attn_mix.log 2>&1 || exit 1
  done
done
