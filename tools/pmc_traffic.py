#!/usr/bin/env python
"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs of
`bench.py --only fwd`) into HBM bytes per launch of the forward SpMM kernel,
with the gfx950 corrections of MI355X_MICROARCH.md §HBM:
  * both counters are in KiB;
  * FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced read
    -> x2 (the SpMM gathers whole 1 KiB rows with 16 B/lane loads);
  * WRITE_SIZE is exact for 16 B/lane streaming stores.
Writes/updates profiles/pmc_traffic.json under the bench workload key.

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
    substr = sys.argv[4] if len(sys.argv) > 4 else "spmm_kernel<4, 1, 8, false, false>"
    f = per_dispatch(fdir, "FETCH_SIZE", substr)
    w = per_dispatch(wdir, "WRITE_SIZE", substr)
    fetch_b = sum(f) / len(f) * 1024 * 2
    write_b = sum(w) / len(w) * 1024
    out_path = os.path.join(HERE, "..", "profiles", "pmc_traffic.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    d[key] = {"kernel": substr, "dispatches": [len(f), len(w)],
              "FETCH_SIZE_KiB_avg": sum(f) / len(f), "WRITE_SIZE_KiB_avg": sum(w) / len(w),
              "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
              "hbm_bytes_per_launch": fetch_b + write_b,
              "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count on 16B/lane reads); WRITE_SIZE KiB x1024"}
    json.dump(d, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(d[key], indent=1))


if __name__ == "__main__":
    main()
