#!/usr/bin/env python3
"""HBM traffic per converge of one type from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE) of `bench.py --type <mode>`.

usage: pmc_converge.py OUT_JSON FETCH_DIR WRITE_DIR FIRST SKIP COUNT [KEEP_PREFIXES]

Dispatches are cut into converges at every launch of kernel FIRST (the one
that opens a converge: k_tlog_prep, k_uj_items, ...); every dispatch up to the
next FIRST whose name starts with one of KEEP_PREFIXES (comma-separated,
default "k_tlog_,jydscan::") belongs to it.  Converges SKIP .. SKIP+COUNT-1
(0 = the bench's setup converge, so SKIP = warmup + 1 picks the timed ones)
are averaged.  gfx950 corrections (MI355X_MICROARCH.md, calibrated in
profiles/r02_pmc_modes.json): FETCH_SIZE x 2, WRITE_SIZE as is; both in KiB."""
import csv
import glob
import json
import os
import sys


def dispatches(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                name = name.split("<")[0]
                rows.append((int(r["Dispatch_Id"]), name, float(r["Counter_Value"])))
    rows.sort()
    return rows


def converges(rows, first, keep):
    out, cur = [], None
    for _, name, v in rows:
        if name == first:
            cur = {}
            out.append(cur)
        if cur is not None and any(name.startswith(k) for k in keep):
            cur[name] = cur.get(name, 0.0) + v
    return out


def main():
    out, fdir, wdir, first = sys.argv[1:5]
    skip, count = int(sys.argv[5]), int(sys.argv[6])
    keep = (sys.argv[7] if len(sys.argv) > 7 else "k_tlog_,jydscan::").split(",")
    fc = converges(dispatches(fdir, "FETCH_SIZE"), first, keep)[skip:skip + count]
    wc = converges(dispatches(wdir, "WRITE_SIZE"), first, keep)[skip:skip + count]
    if not fc or not wc:
        sys.exit(f"no converges found (fetch {len(fc)}, write {len(wc)})")
    kern = sorted(set().union(*fc, *wc))
    per = {k: {"read_MB": sum(c.get(k, 0) for c in fc) / len(fc) * 2 * 1024 / 1e6,
               "written_MB": sum(c.get(k, 0) for c in wc) / len(wc) * 1024 / 1e6} for k in kern}
    tot_r = sum(v["read_MB"] for v in per.values())
    tot_w = sum(v["written_MB"] for v in per.values())
    res = {"converges_averaged": len(fc), "first_converge": skip, "per_kernel": per, "read_MB": tot_r,
           "written_MB": tot_w, "moved_MB": tot_r + tot_w,
           "note": "FETCH_SIZE x 2 (gfx950), WRITE_SIZE as is; KiB -> MB; per converge"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps({k: round(v, 1) for k, v in res.items() if k.endswith("_MB")}))


if __name__ == "__main__":
    main()
