"""Per-launch HBM traffic of each kernel from rocprofv3 --pmc CSV passes.

usage: python scripts/pmc_traffic.py <dir with FETCH pass> <dir with WRITE pass> [out.json [dir with MFMA pass]]

Reads every *counter_collection.csv under the two directories, sums each counter per
dispatch, and averages per kernel name.  gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE (KiB) reports half the bytes of a wide coalesced streaming read, so
read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KiB) is exact for 16-B stores.
The optional MFMA pass (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE) gives each kernel's MFMA-busy fraction:
busy SIMD-cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), averaged over its dispatches.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name") or row.get("Kernel-Name") or row.get("KernelName")
                disp = row.get("Dispatch_Id") or row.get("Dispatch-Id") or row.get("Correlation_Id")
                cn = row.get("Counter_Name")
                cv = float(row.get("Counter_Value", 0) or 0)
                per[(k, disp)][cn] += cv
    return per


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    agg = defaultdict(lambda: {"n_fetch": 0, "fetch_kib": 0.0, "n_write": 0, "write_kib": 0.0})
    for (k, _), c in fetch.items():
        if "FETCH_SIZE" in c:
            agg[k]["n_fetch"] += 1
            agg[k]["fetch_kib"] += c["FETCH_SIZE"]
    for (k, _), c in write.items():
        if "WRITE_SIZE" in c:
            agg[k]["n_write"] += 1
            agg[k]["write_kib"] += c["WRITE_SIZE"]
    out = {}
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["fetch_kib"]):
        rd = 2 * a["fetch_kib"] * 1024 / max(a["n_fetch"], 1)
        wr = a["write_kib"] * 1024 / max(a["n_write"], 1)
        out[k] = {"launches": a["n_fetch"], "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                  "hbm_bytes_per_launch": rd + wr}
    if len(sys.argv) > 4:
        mf = load(sys.argv[4])
        acc = defaultdict(list)
        for (k, _), c in mf.items():
            if c.get("GRBM_GUI_ACTIVE", 0) > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                acc[k].append(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024))
        for k, v in acc.items():
            out.setdefault(k, {})["mfma_busy"] = round(sum(v) / len(v), 4)
    for k, v in [kv for kv in out.items() if "launches" in kv[1]][:25]:
        print(f"{v['launches']:5d}  rd {v['read_bytes_per_launch'] / 1e6:9.2f} MB  wr {v['write_bytes_per_launch'] / 1e6:9.2f} MB  {k[:110]}")
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
