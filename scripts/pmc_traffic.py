#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc passes.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR CELLS_PER_LAUNCH OUT_JSON

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts
TCC_EA0_RDREQ x 64 B and reads exactly half the bytes of a wide coalesced
16-B-per-lane stream, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane
streaming stores.  Both are reported in KiB per dispatch.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, substr):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter and substr in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fdir, wdir, substr, cells, out = sys.argv[1:6]
    cells = int(cells)
    fetch = per_dispatch(fdir, "FETCH_SIZE", substr)
    write = per_dispatch(wdir, "WRITE_SIZE", substr)
    if not fetch or not write:
        raise SystemExit(f"no {substr} dispatches with counters in {fdir} / {wdir}")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    read_bytes = 2.0 * f_kib * 1024  # gfx950: FETCH_SIZE reads half of a 16-B/lane stream
    write_bytes = w_kib * 1024
    res = {
        "kernel": substr,
        "dispatches": {"fetch": len(fetch), "write": len(write)},
        "fetch_size_kib_raw": f_kib,
        "write_size_kib_raw": w_kib,
        "hbm_read_bytes_per_launch": read_bytes,
        "hbm_write_bytes_per_launch": write_bytes,
        "hbm_bytes_per_launch": read_bytes + write_bytes,
        "workload_cells_per_launch": cells,
        "algorithmic_bytes_per_launch": 24 * cells,
        "traffic_over_algorithmic": (read_bytes + write_bytes) / (24 * cells),
        "correction": "FETCH_SIZE x2 (gfx950 wide-stream undercount), WRITE_SIZE as is; KiB -> bytes x1024",
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
