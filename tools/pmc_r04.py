#!/usr/bin/env python
"""Summarise the round-4 GraphConv PMC passes (tools/gpu_session.sh
pmc_infer_mfma, pmc_layer_mfma, pmc_wide_mfma, pmc_infer_l2) per kernel into
profiles/r04_pmc_graphconv.json.

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024
SIMDs); clock = GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md);
VALU per MFMA = SQ_INSTS_VALU / SQ_INSTS_MFMA (SQ_INSTS_VALU counts the MFMAs
too).  L2: TCP_TCC_READ_REQ_sum requests from the CUs' L1s to the L2 (x 64
B: the request granularity, an upper bound on the bytes), TCC hit rate.

  python tools/pmc_r04.py gpurun_out [profiles/NAME.json]
"""
import collections
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SIMDS = 256 * 4
PASSES = {"pmc_infer_mfma": "C3 one-kernel inference (bench --only infer)",
          "pmc_layer_mfma": "C3 layer fwd+bwd, p = 0.3 (bench --only layer)",
          "pmc_wide_mfma": "wide one-kernel shapes (tools/probe_wide.py, PROBE_QUICK, 512x256 and 512x512)",
          "pmc_infer_l2": "C3 one-kernel inference, L2 traffic (bench --only infer)",
          "pmc_wide_l2": "one-kernel shapes 256x256 and 512x512, L2 and fabric traffic (tools/probe_wide.py, PROBE_QUICK)",
          "pmc_wide_mfma5": "one-kernel shapes 256x256 and 512x512 (tools/probe_wide.py, PROBE_QUICK)"}


def per_kernel(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        k = r["Kernel_Name"]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k][r.get("Dispatch_Id", len(dur[k]))] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k, cs in acc.items():
        d = list(dur[k].values())
        t = sum(d) / len(d)
        c = {n: sum(v) / len(v) for n, v in cs.items()}
        e = {"dispatches": len(d), "duration_ms": t * 1e3, "counters_avg": c}
        if "GRBM_GUI_ACTIVE" in c:
            e["clock_GHz"] = c["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                e["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * SIMDS)
        if c.get("SQ_INSTS_MFMA"):
            e["valu_per_mfma"] = c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"]
        if "TCP_TCC_READ_REQ_sum" in c:
            e["l2_read_GB_at_64B"] = c["TCP_TCC_READ_REQ_sum"] * 64 / 1e9
        if "TCC_EA0_RDREQ_sum" in c:  # fabric reads (HBM + Infinity Cache), 64 B per request as FETCH_SIZE counts them
            e["fabric_read_GB_at_64B"] = c["TCC_EA0_RDREQ_sum"] * 64 / 1e9
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            e["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        out[k] = e
    return out


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    res = {}
    for d, desc in PASSES.items():
        p = os.path.join(root, d)
        if not os.path.exists(os.path.join(p, "run_counter_collection.csv")):
            continue
        ks = per_kernel(p)
        keep = {k: v for k, v in ks.items() if "grl::" in k and v["duration_ms"] > 0.2}
        res[d] = {"workload": desc, "kernels": keep}
    name = sys.argv[2] if len(sys.argv) > 2 else "r04_pmc_graphconv.json"
    path = os.path.join(HERE, "..", "profiles", name)
    json.dump(res, open(path, "w"), indent=1, sort_keys=True)
    for d, v in res.items():
        print(d, v["workload"])
        for k, e in v["kernels"].items():
            print(f"  {k[:100]}: {e['duration_ms']:.3f} ms, " + ", ".join(
                f"{n} {e[n]:.3f}" for n in ("clock_GHz", "mfma_busy_frac", "valu_per_mfma", "l2_read_GB_at_64B",
                                            "l2_hit_rate", "fabric_read_GB_at_64B") if n in e))


if __name__ == "__main__":
    main()
