"""Per-kernel summary of a rocprofv3 PMC pass over the attention kernels
(tools/gpu_session.sh pmc_attn100k): VALU and LDS instructions per MFMA,
MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024
SIMDs)), and the clock the chip held (GRBM_GUI_ACTIVE / 8 / duration).
  python tools/pmc_attn.py DIR [OUT.json]"""
import collections
import csv
import json
import os
import re
import sys


def main():
    d = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        m = re.search(r"(attn_\w+(<[^>]*>)?)", r["Kernel_Name"])
        if not m:
            continue
        name = m.group(1)
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[(name, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for name, c in acc.items():
        ds = [v for (k, _), v in dur.items() if k == name]
        mf = c["SQ_INSTS_MFMA"]
        if not mf:
            continue
        active = c["GRBM_GUI_ACTIVE"] / 8
        out[name] = {"dispatches": len(ds), "ms_avg": 1e3 * sum(ds) / len(ds),
                     "valu_per_mfma": (c["SQ_INSTS_VALU"] - mf) / mf, "lds_per_mfma": c["SQ_INSTS_LDS"] / mf,
                     "mfma_busy": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (active * 1024),
                     "clock_GHz": active / sum(ds) / 1e9}
        print(name, {k: round(v, 3) for k, v in out[name].items()})
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
