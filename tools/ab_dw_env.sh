#!/bin/bash
# A/B of an env switch on the x6 dW probe, interleaved, 3 rounds, bits checked
# against the first run:  tools/ab_dw_env.sh VAR   (runs VAR=1 then VAR=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
rm -f /tmp/ab_dw_env_ref.pt
for rep in 1 2 3; do
  for v in 1 0; do
    echo "== $1=$v" >> gpurun_out/ab_dw_env.log
    env "$1=$v" AB_SAVE=/tmp/ab_dw_env_ref.pt timeout -k 10 200 python tools/probe_dw.py >> gpurun_out/ab_dw_env.log 2>&1 || exit 1
  done
done
