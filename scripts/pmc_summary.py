#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 --pmc output directories.

usage: pmc_summary.py OUT_JSON DIR [DIR ...]
Rows: kernel -> counter -> {"mean": per-dispatch mean, "dispatches": n}.
No correction is applied here (see DESIGN.md for the gfx950 factors)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "").replace("(anonymous namespace)::", "")
                    name = name.split("(")[0][:80]
                    acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {k: {c: {"mean": sum(v) / len(v), "dispatches": len(v)} for c, v in cs.items()} for k, cs in acc.items()}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k, cs in sorted(res.items()):
        print(k, {c: round(x["mean"]) for c, x in cs.items()})


if __name__ == "__main__":
    main()
