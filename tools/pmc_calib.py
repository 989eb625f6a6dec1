"""Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on the SpMM's own
access pattern (the x2 "gfx950 half-count" correction applied to
FETCH_SIZE must be measured, not assumed; MI355X_MICROARCH.md §HBM:
"calibrate on a known byte count in your own access pattern").

Workload: a permutation graph -- one edge type, no self term, row n gathers
source row perm[n] -- so every X row is read exactly once, through the very
kernel and load width of the benchmark (spmm_kernel<4,1,8,...>, 1 KiB rows,
16 B per lane), from a 4 GB table (16x the 256 MiB Infinity Cache: nothing
is re-read on-die).  Known bytes per launch:
  reads  = N*F*4 (X) + N*4 (colidx) + (N+1)*4 (rowptr)
  writes = N*F*4 (Z)
Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` in separate
passes (tools/gpu_session.sh pmc_calib_fetch / pmc_calib_write), then
`python tools/pmc_calib.py --summarize gpurun_out` writes
profiles/r02_pmc_calibration.json with the raw counters and their ratio to
the known bytes."""
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
N, F, STEPS = 4_000_000, 256, 6


def run():
    sys.path.insert(0, os.path.join(HERE, "..", "graph-representation-learning_amd"))
    import torch

    from grl import TypedGraph
    from grl.ops import spmm_forward

    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(0)
    rowptr = torch.arange(N + 1, dtype=torch.int32, device=dev)
    colidx = torch.randperm(N, generator=gen, device=dev).to(torch.int32)
    g = TypedGraph(rowptr, colidx, 1, has_self=False)
    X = torch.randn(N, F, generator=gen, device=dev)
    Z = torch.empty(N, F, device=dev)
    for _ in range(STEPS):
        spmm_forward(X, g, out=Z)
    torch.cuda.synchronize()
    assert torch.equal(Z, X[colidx.long()])
    print("calibration run done", flush=True)


def _avg(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv")))
            if "spmm_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows in {path}")
    return sum(vals) / len(vals), len(vals)


def summarize(root):
    fetch_kib, nf = _avg(os.path.join(root, "pmc_calib_fetch"), "FETCH_SIZE")
    write_kib, nw = _avg(os.path.join(root, "pmc_calib_write"), "WRITE_SIZE")
    reads = N * F * 4 + N * 4 + (N + 1) * 4
    writes = N * F * 4
    out = {"workload": f"permutation graph N={N}, F={F}: each 1 KiB X row gathered exactly once "
                       "(spmm_kernel<4,1,8,false,false>, 16 B/lane loads, 4 GB table)",
           "known_read_bytes": reads, "known_write_bytes": writes,
           "FETCH_SIZE_KiB_avg": fetch_kib, "WRITE_SIZE_KiB_avg": write_kib, "dispatches": [nf, nw],
           "fetch_ratio_raw": fetch_kib * 1024 / reads, "write_ratio_raw": write_kib * 1024 / writes,
           "fetch_correction": reads / (fetch_kib * 1024), "write_correction": writes / (write_kib * 1024)}
    path = os.path.join(HERE, "..", "profiles", "r02_pmc_calibration.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
