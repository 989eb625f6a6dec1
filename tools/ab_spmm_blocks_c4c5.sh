set -e
for r in 1 2; do
for b in 16 24 28; do
  v=$(timeout -k 10 150 python bench.py --option spmm_blocks_per_cu=$b --cpu-seconds 0 --steps 20 --warmup 5 --c4-reference 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms'],3), round(d['C4_one_gpu']['ms'],3))")
  echo "round $r blocks/CU $b: C3 fwd / C4 fwd ms = $v"
done
done
for b in 16 24; do
  v=$(timeout -k 10 300 python bench.py --option spmm_blocks_per_cu=$b --workload C5 --cpu-seconds 0 --steps 5 --warmup 2 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3))")
  echo "blocks/CU $b: C5 fwd ms / frac = $v"
done
