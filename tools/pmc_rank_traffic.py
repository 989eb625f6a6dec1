#!/usr/bin/env python
"""Fold the rocprofv3 passes of tools/probe_rank_shard.py (run with
--no-parity, so the only SpMM launches are the rank's column-slice
aggregations) into profiles/pmc_traffic.json under bench.traffic_key for the
C4 workload at that world size, as bench.load_traffic reads it: HBM bytes of
one rank's aggregation STEP (its K slice launches; bench's N > 1 `achieved`
and kernel time are per step too), with the same gfx950 corrections as
tools/pmc_traffic.py (FETCH_SIZE KiB x1024 x the calibrated factor of
profiles/r02_pmc_calibration.json, WRITE_SIZE KiB x1024).  The kernel time
of the same launches comes from the --kernel-trace --stats pass.

  python tools/pmc_rank_traffic.py PROBE_JSON FETCH_DIR WRITE_DIR STATS_CSV
"""
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SLICE = ("spmm_kernel<", "spmm_pair_kernel<")


def per_dispatch(path, counter):
    vals, names = [], set()
    for r in csv.DictReader(open(_find(path))):
        if r["Counter_Name"] == counter and any(s in r["Kernel_Name"] for s in SLICE):
            vals.append(float(r["Counter_Value"]))
            names.add(r["Kernel_Name"].replace("void ", "").replace("grl::(anonymous namespace)::", "").split("(")[0])
    if not vals:
        raise SystemExit(f"no {counter} rows for the slice kernels in {path}")
    return vals, sorted(names)


def _find(path):
    for root, _, files in os.walk(path):
        for f in files:
            if f.endswith("counter_collection.csv"):
                return os.path.join(root, f)
    raise SystemExit(f"no counter_collection.csv under {path}")


def stats_ms(path):
    calls, total = 0, 0.0
    for r in csv.DictReader(open(path)):
        if any(s in r["Name"] for s in SLICE):
            calls += int(r["Calls"])
            total += float(r["TotalDurationNs"])
    return calls, total / 1e6


def main():
    probe_json, fdir, wdir, stats = sys.argv[1:5]
    sys.path[:0] = [os.path.join(ROOT, "graph-representation-learning_amd"), ROOT]
    probe = json.load(open(probe_json))
    K = probe["chunks"]
    f, names = per_dispatch(fdir, "FETCH_SIZE")
    w, _ = per_dispatch(wdir, "WRITE_SIZE")
    calib = os.path.join(ROOT, "profiles", "r02_pmc_calibration.json")
    factor = json.load(open(calib))["fetch_correction"]
    fetch_b = sum(f) / len(f) * 1024 * factor * K  # per step = K slice launches
    write_b = sum(w) / len(w) * 1024 * K
    calls, tot_ms = stats_ms(stats)
    step_ms = tot_ms / calls * K if calls else None

    class A:  # bench.traffic_key's argument object for the C4 workload
        graph, avg_deg, types, dim, p = "er", 32.0, 6, 256, 0.0

    from bench import traffic_key

    key = traffic_key("C4", probe["world"], A, probe["n_loc"])
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    d[key] = {"kernel": "spmm_kernel / spmm_pair_kernel (grl_typed_spmm_fwd_slice)", "kernels_seen": names,
              "rank": probe["rank"], "per": f"one rank's aggregation step: {K} slice launches",
              "dispatches": [len(f), len(w)],
              "FETCH_SIZE_KiB_avg_per_launch": sum(f) / len(f), "WRITE_SIZE_KiB_avg_per_launch": sum(w) / len(w),
              "fetch_bytes_corrected": fetch_b, "write_bytes": write_b, "hbm_bytes_per_launch": fetch_b + write_b,
              "alg_bytes_step": probe["alg_bytes_step"],
              "alg_bytes_step_incl_slice_rewalks": probe["alg_bytes_step_incl_slice_rewalks"],
              "rocprof_step_ms": step_ms, "event_step_ms": probe["aggregate_ms_mean"],
              "halo_mode": probe["halo_mode"], "table_rows": probe["table_rows"],
              "correction": f"FETCH_SIZE KiB x1024 x{factor:.4f} (calibrated: profiles/r02_pmc_calibration.json); "
                            "WRITE_SIZE KiB x1024; x K slices per step",
              "source": "tools/probe_rank_shard.py on one GPU (rank's shard built in-process, tables filled as "
                        "the exchange leaves them)"}
    json.dump(d, open(out_path, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(d[key], indent=1))


if __name__ == "__main__":
    main()
