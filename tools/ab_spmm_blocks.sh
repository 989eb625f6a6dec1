# A/B of the persistent SpMM grid size (GRL_SPMM_BLOCKS_PER_CU, four-wave
# blocks per CU; read per process): C3 forward p=0 (the headline kernel),
# forward p=0.3 and the CSC backward p=0.3, from bench.py's own line.
# Usage: bash tools/ab_spmm_blocks.sh "16 24" [rounds]
set -e
vals=${1:-"16 8 12 24 32"}
rounds=${2:-2}
for r in $(seq 1 $rounds); do
for b in $vals; do
  v=$(timeout -k 10 120 python bench.py --option spmm_blocks_per_cu=$b --cpu-seconds 0 --steps 30 --warmup 10 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['dropedge_train_p0.3']; print(round(d['roofline']['kernel_ms'],3), round(t['fwd_ms'],3), round(t['bwd_ms'],3))")
  echo "round $r blocks/CU $b: fwd p0 / fwd p0.3 / bwd p0.3 ms = $v"
done
done
