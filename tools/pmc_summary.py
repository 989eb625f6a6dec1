#!/usr/bin/env python
"""Summarise rocprofv3 PMC passes (tools/gpu_session.sh pmc_linear_mfma,
pmc_fwd_tlb, pmc_c4_tlb) per kernel into profiles/r01_pmc_mfma_tlb.json.

MFMA utilisation of the dense step (BASELINE north_star): per-SIMD busy
cycles SQ_VALU_MFMA_BUSY_CYCLES (64 per v_mfma_f32_32x32x2_f32) over the
available SIMD cycles = GRBM_GUI_ACTIVE / 8 XCDs (rocprofv3 sums the XCDs)
x 1024 SIMDs (256 CUs x 4).  The quotient GRBM_GUI_ACTIVE / 8 / duration is
the clock the chip held (MI355X_MICROARCH.md, DVFS give-back).

  python tools/pmc_summary.py gpurun_out
"""
import collections
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SIMDS = 256 * 4


def per_kernel(path, substr):
    acc = collections.defaultdict(list)
    dur = []
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if substr in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    if not acc:
        raise SystemExit(f"no rows for {substr!r} in {path}")
    n = len(next(iter(acc.values())))
    return {k: sum(v) / len(v) for k, v in acc.items()}, sum(dur) / len(dur), n


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    out = {}
    c, t, n = per_kernel(os.path.join(root, "pmc_linear_mfma"), "gemm256p_kernel<true, false, 0, 3>")
    clk = c["GRBM_GUI_ACTIVE"] / 8 / t
    out["linear_fwd_C3"] = {
        "kernel": "gemm256p_kernel<true,false,0,3> (grl_linear_fwd, M=1e6, K=1792, C=256)", "dispatches": n,
        "duration_ms": t * 1e3, "counters_avg": c, "clock_GHz": clk / 1e9,
        "mfma_busy_frac": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * SIMDS),
        "tflops": 2 * 1e6 * 1792 * 256 / t / 1e12,
        "note": "SQ_VALU_MFMA_BUSY_CYCLES = 64 x number of 32x32x2 f32 MFMAs (224M per launch); "
                "busy fraction is against the clock the chip held, TFLOP/s against wall time"}
    for key, d, desc in (("spmm_fwd_C3_tlb", "pmc_fwd_tlb", "C3: N=1M, X 1.02 GB"),
                         ("spmm_fwd_C4shape_tlb", "pmc_c4_tlb", "C4 shape on one GPU: N=4M, X 4.1 GB")):
        c, t, n = per_kernel(os.path.join(root, d), "spmm_kernel<4, 1, 8, false, false>")
        hit, miss = c["TCP_UTCL1_TRANSLATION_HIT_sum"], c["TCP_UTCL1_TRANSLATION_MISS_sum"]
        out[key] = {"kernel": "spmm_kernel<4,1,8,false,false> (grl_typed_spmm_fwd)", "workload": desc,
                    "dispatches": n, "duration_ms": t * 1e3, "counters_avg": c,
                    "utcl1_miss_rate": miss / (hit + miss)}
    path = os.path.join(HERE, "..", "profiles", "r01_pmc_mfma_tlb.json")
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
