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
    for key, d, kern, desc, note in (
            ("linear_fwd_C3_x6", "pmc_linear_mfma", "gemm_x6_kernel<0>",
             "gemm_x6_kernel<STORE> (grl_linear_fwd, M=1e6, K=1792, C=256; default large-M path)",
             "SQ_VALU_MFMA_BUSY_CYCLES = 32 x number of 32x32x16 bf16 MFMAs (6 per fp32 32x32x16 block: 168M "
             "per launch); TFLOP/s = fp32-equivalent flops (2MKC) over wall time"),
            ("linear_fwd_C3_f32mfma", "pmc_linear_mfma_f32", "gemm256p_kernel<true, false, 0, 3>",
             "gemm256p_kernel<KC,RC,STORE,3> (grl_linear_fwd with gemm_x6 = 0)",
             "SQ_VALU_MFMA_BUSY_CYCLES = 64 x number of 32x32x2 f32 MFMAs (224M per launch)")):
        if not os.path.isdir(os.path.join(root, d)):
            continue
        c, t, n = per_kernel(os.path.join(root, d), kern)
        clk = c["GRBM_GUI_ACTIVE"] / 8 / t
        out[key] = {"kernel": desc, "dispatches": n, "duration_ms": t * 1e3, "counters_avg": c,
                    "clock_GHz": clk / 1e9,
                    "mfma_busy_frac": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * SIMDS),
                    "tflops": 2 * 1e6 * 1792 * 256 / t / 1e12,
                    "note": note + "; busy fraction is against the clock the chip held"}
    for key, d, desc in (("spmm_fwd_C3_tlb", "pmc_fwd_tlb", "C3: N=1M, X 1.02 GB"),
                         ("spmm_fwd_C4shape_tlb", "pmc_c4_tlb", "C4 shape on one GPU: N=4M, X 4.1 GB")):
        if not os.path.isdir(os.path.join(root, d)):
            continue
        c, t, n = per_kernel(os.path.join(root, d), "spmm_kernel<4, 1, 8, false, false>")
        hit, miss = c["TCP_UTCL1_TRANSLATION_HIT_sum"], c["TCP_UTCL1_TRANSLATION_MISS_sum"]
        out[key] = {"kernel": "spmm_kernel<4,1,8,false,false> (grl_typed_spmm_fwd)", "workload": desc,
                    "dispatches": n, "duration_ms": t * 1e3, "counters_avg": c,
                    "utcl1_miss_rate": miss / (hit + miss)}
    path = os.path.join(HERE, "..", "profiles", "r01_pmc_mfma_tlb.json")
    if os.path.exists(path):  # keep entries this run did not re-measure
        old = json.load(open(path))
        old.update(out)
        out = old
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
