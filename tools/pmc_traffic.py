#!/usr/bin/env python
"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs of
`bench.py --only fwd`) into HBM bytes per launch of the forward SpMM kernel,
with the gfx950 corrections of MI355X_MICROARCH.md §HBM:
  * both counters are in KiB;
  * FETCH_SIZE reports about half the bytes of a wide (16 B/lane) coalesced
    read: the factor is the one measured on the SpMM itself
    (profiles/r02_pmc_calibration.json, tools/pmc_calib.py: x1.896);
  * WRITE_SIZE is exact for 16 B/lane streaming stores.
Writes/updates profiles/pmc_traffic.json under the bench workload key
(bench.traffic_key: workload, world size and shard shape, e.g.
C3_w1_er_n1000000_deg32_L6_d256_p0); bench.load_traffic returns a record
only for that workload at that world size and the kernel family named in it.

  python tools/pmc_traffic.py KEY FETCH_DIR WRITE_DIR [KERNEL_SUBSTR]
"""
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def per_dispatch(path, counter, substr):
    vals = []
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if substr in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {substr!r} in {path}")
    return vals


def main():
    key, fdir, wdir = sys.argv[1:4]
    substr = sys.argv[4] if len(sys.argv) > 4 else "spmm_kernel<4, 1, 8, false, false, false>"
    f = per_dispatch(fdir, "FETCH_SIZE", substr)
    w = per_dispatch(wdir, "WRITE_SIZE", substr)
    # FETCH_SIZE correction measured on this kernel's own access pattern (tools/pmc_calib.py:
    # a permutation graph reading every 1 KiB row once from a 4 GB table), not assumed
    calib = os.path.join(HERE, "..", "profiles", "r02_pmc_calibration.json")
    factor = json.load(open(calib))["fetch_correction"] if os.path.exists(calib) else 2.0
    fetch_b = sum(f) / len(f) * 1024 * factor
    write_b = sum(w) / len(w) * 1024
    out_path = os.path.join(HERE, "..", "profiles", "pmc_traffic.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    d[key] = {"kernel": substr, "dispatches": [len(f), len(w)],
              "FETCH_SIZE_KiB_avg": sum(f) / len(f), "WRITE_SIZE_KiB_avg": sum(w) / len(w),
              "fetch_bytes_raw": sum(f) / len(f) * 1024, "fetch_bytes_x2": sum(f) / len(f) * 1024 * 2,
              "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
              "hbm_bytes_per_launch": fetch_b + write_b,
              "correction": f"FETCH_SIZE KiB x1024 x{factor:.4f} (calibrated: profiles/r02_pmc_calibration.json; "
                            "the guide's gfx950 half-count would be x2); WRITE_SIZE KiB x1024 (calibrated exact)"}
    json.dump(d, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(d[key], indent=1))


if __name__ == "__main__":
    main()
