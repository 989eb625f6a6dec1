#!/bin/bash
# One GPU-box session: each GPU step runs under its own time limit; the
# session stops at the first step that exits nonzero -- a fault, abort,
# segfault or time limit, and also an ordinary failure (the steps are
# chained as with &&).  Usage: tools/gpu_session.sh STEP...
#   steps: tests smoke bench bench_extras bench_drop bench_c5 bench_c5s prof_bench prof_fwd prof_bwd
#          prof_linear prof_layer prof_attn prof_c1 pmc_fwd_fetch pmc_fwd_write pmc_list pmc_linear_mfma
#          pmc_fwd_tlb pmc_c4_tlb; round 4: ab_attn_hu tests_r4 pmc_infer_l2 pmc_wide_mfma prof_wide;
#          round 5: pmc_wide_l2 pmc_wide_mfma5; round 6: rank2 rank4 rank8 tests_r6a
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"

fatal() { case "$1" in 124|134|137|139|13[0-9]|14[0-9]) return 0;; esac; [ "$1" -gt 128 ]; }

run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name (rc=$rc): stopping session"; exit $rc; fi
  if [ "$rc" -ne 0 ]; then echo "$name failed (rc=$rc): stopping session"; exit $rc; fi
  return 0
}

for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench_extras) run bench_extras 600 python bench.py --extras --cpu-seconds 0 ;;
    bench_drop) run bench_drop 600 python bench.py --p 0.3 --cpu-seconds 0 ;;
    bench_c5) run bench_c5 900 python bench.py --workload C5 --steps 5 --warmup 2 ;;
    bench_c5s) run bench_c5s 600 python bench.py --graph rmat --nodes-per-gpu 1048576 --avg-deg 64 --dim 512 \
                  --p 0.2 --steps 10 --warmup 3 ;;
    prof_bench) run prof_bench 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv \
                  -- python bench.py ;;
    prof_fwd) run prof_fwd 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_fwd" -o run --output-format csv \
                  -- python bench.py --only fwd --steps 20 --warmup 3 ;;
    prof_bwd) run prof_bwd 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bwd" -o run --output-format csv \
                  -- python bench.py --only bwd --steps 10 --warmup 2 ;;
    prof_linear) run prof_linear 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_linear" -o run --output-format csv \
                  -- python bench.py --only linear --steps 10 --warmup 2 ;;
    prof_layer) run prof_layer 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_layer" -o run --output-format csv \
                  -- python bench.py --only layer --steps 5 --warmup 2 ;;
    prof_attn) run prof_attn 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_attn" -o run --output-format csv \
                  -- python tools/probe_attn.py ;;
    probe_x6) run probe_x6 300 python tools/probe_x6.py ;;
    prof_c1) run prof_c1 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c1" -o run --output-format csv \
                  -- python bench.py --only c1 --steps 20 ;;
    pmc_fwd_fetch) run pmc_fwd_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fwd_fetch" -o run \
                  --output-format csv -- python bench.py --only fwd --steps 5 --warmup 1 ;;
    pmc_fwd_write) run pmc_fwd_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_fwd_write" -o run \
                  --output-format csv -- python bench.py --only fwd --steps 5 --warmup 1 ;;
    pmc_list) run pmc_list 120 rocprofv3 -L ;;
    pmc_linear_mfma) run pmc_linear_mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES \
                  --kernel-trace -d "$OUT/pmc_linear_mfma" -o run --output-format csv \
                  -- python bench.py --only linear --steps 5 --warmup 1 ;;
    pmc_linear_mfma_f32) run pmc_linear_mfma_f32 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES \
                  GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES --kernel-trace -d "$OUT/pmc_linear_mfma_f32" -o run \
                  --output-format csv -- python bench.py --only linear --steps 5 --warmup 1 --option gemm_x6=0 ;;
    pmc_fwd_tlb) run pmc_fwd_tlb 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
                  --kernel-trace -d "$OUT/pmc_fwd_tlb" -o run --output-format csv \
                  -- python bench.py --only fwd --steps 5 --warmup 1 ;;
    pmc_c4_tlb) run pmc_c4_tlb 400 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
                  --kernel-trace -d "$OUT/pmc_c4_tlb" -o run --output-format csv \
                  -- python bench.py --only fwd --nodes-per-gpu 4000000 --steps 5 --warmup 1 ;;
    pmc_x6_a) run pmc_x6_a 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
                  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
                  --kernel-trace -d "$OUT/pmc_x6_a" -o run --output-format csv \
                  -- python bench.py --only linear --steps 5 --warmup 1 ;;
    pmc_x6_b) run pmc_x6_b 300 rocprofv3 --pmc SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL \
                  SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 \
                  --kernel-trace -d "$OUT/pmc_x6_b" -o run --output-format csv \
                  -- python bench.py --only linear --steps 5 --warmup 1 ;;
    tests_dist) run pytest_gpu_dist 600 python -u -m pytest tests/test_gpu_dist.py -m gpu -v -rf --timeout 300 \
                  --timeout-method thread ;;
    tests_configs) run pytest_gpu_configs 1000 python -u -m pytest tests/test_gpu_configs.py -m gpu -v -s -rf \
                  --timeout 600 --timeout-method thread ;;
    tests_dp) run pytest_gpu_dp 300 python -u -m pytest tests/test_gpu_dp.py -m gpu -v -s -rf --timeout 240 \
                  --timeout-method thread ;;
    tests_capture) run pytest_gpu_capture 300 python -u -m pytest tests/test_gpu_graph_capture.py -m gpu -v -s -rf \
                  --timeout 240 --timeout-method thread ;;
    c1) run c1 300 python bench.py --only c1 --steps 20 ;;
    tests_new) run pytest_gpu_new 900 python -u -m pytest tests/test_gpu_blocked.py tests/test_gpu_graphconv.py \
                  -m gpu -v -s -rf --timeout 600 --timeout-method thread ;;
    pmc_calib_fetch) run pmc_calib_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_calib_fetch" \
                  -o run --output-format csv -- python tools/pmc_calib.py ;;
    pmc_calib_write) run pmc_calib_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_calib_write" \
                  -o run --output-format csv -- python tools/pmc_calib.py ;;
    prof_c5) run prof_c5 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv \
                  -- python bench.py --workload C5 --only fwd --steps 5 --warmup 1 ;;
    pmc_c5_tlb) run pmc_c5_tlb 600 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
                  TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum --kernel-trace -d "$OUT/pmc_c5_tlb" -o run \
                  --output-format csv -- python bench.py --workload C5 --only fwd --steps 3 --warmup 1 ;;
    pmc_c5_fetch) run pmc_c5_fetch 600 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace -d "$OUT/pmc_c5_fetch" \
                  -o run --output-format csv -- python bench.py --workload C5 --only fwd --steps 3 --warmup 1 ;;
    probe_cumask) run probe_cumask 400 python tools/probe_cumask.py ;;
    tests_relabel) run pytest_gpu_relabel 300 python -u -m pytest tests/test_gpu_relabel.py -m gpu -v -rf \
                  --timeout 240 --timeout-method thread ;;
    bench_c5full) run bench_c5full 900 python bench.py --workload C5 --steps 5 --warmup 2 ;;
    pmc_c5_fetch2) run pmc_c5_fetch2 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_c5_fetch2" -o run \
                  --output-format csv -- python bench.py --workload C5 --only fwd --steps 3 --warmup 1 ;;
    pmc_c5_write) run pmc_c5_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_c5_write" -o run \
                  --output-format csv -- python bench.py --workload C5 --only fwd --steps 3 --warmup 1 ;;
    prof_c5b) run prof_c5b 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5b" -o run --output-format csv \
                  -- python bench.py --workload C5 --only fwd --steps 5 --warmup 1 ;;
    probe_contig) run probe_contig 300 python tools/probe_contig.py ;;
    tests_warper) run pytest_gpu_warper 600 python -u -m pytest tests/test_gpu_warper.py tests/test_gpu_graph_capture.py \
                  -m gpu -v -rf --timeout 300 --timeout-method thread ;;
    tests_attn) run pytest_gpu_attn 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_model.py -m gpu -q -rf \
                  --timeout 300 --timeout-method thread ;;
    ab_attn) export ATTN_N="100000 131072"; run ab_attn 900 tools/ab_attn_lib.sh ${AB_LIBS:-attn_prev} ;;
    prof_attn100k) run prof_attn100k 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_attn100k" -o run \
                  --output-format csv -- python tools/probe_attn.py 100000 ;;
    pmc_attn100k) run pmc_attn100k 300 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA \
                  SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
                  --kernel-trace -d "$OUT/pmc_attn100k" -o run --output-format csv -- python tools/probe_attn.py 100000 ;;
    tests_rows) run pytest_gpu_rows 600 python -u -m pytest tests/test_gpu_dist.py -k rows_pipelined -m gpu -v -rf \
                  --timeout 300 --timeout-method thread ;;
    probe_c1p) run probe_c1p 300 python tools/probe_c1_procedure.py ;;
    ab_dw) rm -f gpurun_out/ab_dw.log; run ab_dw 900 tools/ab_dw.sh ${AB_LIBS:-x6t_il} ;;
    tests_r3) run pytest_gpu_r3 600 python -u -m pytest tests/test_gpu_halo_async.py tests/test_gpu_graphconv.py \
                  tests/test_gpu_embed.py tests/test_gpu_dist.py::test_bench_spawns_its_ranks_without_a_launcher \
                  -m gpu -v -rf --timeout 240 --timeout-method thread ;;
    pmc_infer_mfma) run pmc_infer_mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES \
                  SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d "$OUT/pmc_infer_mfma" -o run --output-format csv \
                  -- python bench.py --only infer --steps 5 --warmup 1 ;;
    pmc_layer_mfma) run pmc_layer_mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES \
                  SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d "$OUT/pmc_layer_mfma" -o run --output-format csv \
                  -- python bench.py --only layer --steps 3 --warmup 1 ;;
    prof_attn_fused) run prof_attn_fused 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_attn_fused" -o run \
                  --output-format csv -- python tools/probe_attn.py 100000 ;;
    ab_attn_hu) export ATTN_N="100000"; rm -f gpurun_out/ab_attn_lib.log; run ab_attn_hu 500 tools/ab_attn_lib.sh attn_b20 attn_pin0 attn_hu0 attn_r3 ;;
    tests_r4) run pytest_gpu_r4 900 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_procedure_golden.py \
                  tests/test_gpu_warper.py tests/test_gpu_dp.py tests/test_gpu_sharded_model.py tests/test_gpu_rccl.py \
                  tests/test_gpu_graph_capture.py -m gpu -q -rf --timeout 300 --timeout-method thread ;;
    pmc_infer_l2) run pmc_infer_l2 300 timeout -s KILL 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum \
                  GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/pmc_infer_l2" -o run --output-format csv \
                  -- python bench.py --only infer --steps 5 --warmup 1 ;;
    pmc_wide_mfma) export PROBE_QUICK=1 PROBE_SHAPES=512x256,512x512; run pmc_wide_mfma 300 timeout -s KILL 240 \
                  rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA \
                  --kernel-trace -d "$OUT/pmc_wide_mfma" -o run --output-format csv -- python tools/probe_wide.py; \
                  unset PROBE_QUICK PROBE_SHAPES ;;
    prof_wide) export PROBE_SHAPES=512x256,512x512,1024x512; run prof_wide 400 rocprofv3 --kernel-trace --stats \
                  -d "$OUT/prof_wide" -o run --output-format csv -- python tools/probe_wide.py; unset PROBE_SHAPES ;;
    pmc_wide_l2) export PROBE_QUICK=1 PROBE_SHAPES=${PROBE_SHAPES:-256x256,512x512}; run pmc_wide_l2 300 \
                  timeout -s KILL 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
                  GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/pmc_wide_l2" -o run --output-format csv \
                  -- python tools/probe_wide.py; unset PROBE_QUICK PROBE_SHAPES ;;
    pmc_wide_mfma5) export PROBE_QUICK=1 PROBE_SHAPES=${PROBE_SHAPES:-256x256,512x512}; run pmc_wide_mfma5 300 \
                  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES \
                  SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d "$OUT/pmc_wide_mfma5" -o run --output-format csv \
                  -- python tools/probe_wide.py; unset PROBE_QUICK PROBE_SHAPES ;;
    rank2|rank4|rank8) P=${step#rank}
                  run probe_rank$P 300 python tools/probe_rank_shard.py --world $P --json "$OUT/rank$P.json"
                  run prof_rank$P 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rank$P" -o run \
                    --output-format csv -- python tools/probe_rank_shard.py --world $P --no-parity
                  run pmcf_rank$P 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace \
                    -d "$OUT/pmcf_rank$P" -o run --output-format csv -- python tools/probe_rank_shard.py --world $P --no-parity
                  run pmcw_rank$P 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace \
                    -d "$OUT/pmcw_rank$P" -o run --output-format csv -- python tools/probe_rank_shard.py --world $P --no-parity ;;
    tests_r6a) run pytest_gpu_r6a 600 python -u -m pytest tests/test_gpu_graph_parallel.py tests/test_gpu_dist.py \
                  -m gpu -v -rf --timeout 300 --timeout-method thread ;;
    ab_wide) rm -f gpurun_out/ab_wide.log; run ab_wide 900 tools/ab_wide.sh ${AB_LIBS} ;;
    pmc_wide_roles) for lib in libgrl.so diag/libgrl_wi4.so diag/libgrl_wi8.so; do n=$(basename $lib .so)
                  GRL_LIB_PATH=graph-representation-learning_amd/grl/$lib PROBE_QUICK=1 PROBE_SHAPES=512x512,256x256 \
                  run pmc_roles_$n 300 timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
                  SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d "$OUT/pmc_roles_$n" -o run \
                  --output-format csv -- python tools/probe_wide.py; done ;;
    rehearse_p2) run rehearse_p2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                  --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --dist-backend gloo --steps 3 \
                  --warmup 1 --cpu-seconds 5 ;;
    ab_fused) rm -f gpurun_out/ab_fused_lib.log; run ab_fused 900 tools/ab_fused_lib.sh ${AB_LIBS} ;;
    ab_attn_opt) rm -f gpurun_out/ab_attn_opt.log; run ab_attn_opt 900 tools/ab_attn_opt.sh ${AB_OPTS} ;;
    tests_dh16) run pytest_gpu_dh16 600 python -u -m pytest tests/test_gpu_attention.py -m gpu -v -rf --timeout 300 \
                  --timeout-method thread -k "dh_on_16 or eight_wave or backward_matches" ;;
    tests_kq16) run pytest_gpu_kq16 600 python -u -m pytest tests/test_gpu_attention.py -m gpu -v -s -rf --timeout 300 \
                  --timeout-method thread -k "kq_on_16 or dh_on_16 or key_chunks or fused_dq_backward or backward_matches" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== session done"
