#!/usr/bin/env python3
"""HBM traffic per UJSON converge from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE) of `bench.py --type ujson`.

usage: pmc_ujson.py OUT_JSON FETCH_DIR WRITE_DIR [LAST_N]

The dispatches of the UJSON converge kernels (k_uj_*) are cut into converges
at every k_uj_items / k_uj_docs launch that starts one (k_uj_items since
round 6, k_uj_docs before); the LAST_N converges (the timed ones, default 4)
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
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                rows.append((int(r["Dispatch_Id"]), name, float(r["Counter_Value"])))
    rows.sort()
    return rows


def converges(rows):
    first = "k_uj_items" if any(n == "k_uj_items" for _, n, _ in rows) else "k_uj_docs"
    out, cur = [], None
    for _, name, v in rows:
        if not name.startswith("k_uj_") or name.startswith("k_uj_cmp") or name.startswith("k_uj_gather") \
                or name.startswith("k_uj_sizes_read"):
            continue
        if name == first:
            cur = {}
            out.append(cur)
        if cur is not None:
            cur[name] = cur.get(name, 0.0) + v
    return out


def main():
    out, fdir, wdir = sys.argv[1:4]
    last = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    fc, wc = converges(dispatches(fdir, "FETCH_SIZE")), converges(dispatches(wdir, "WRITE_SIZE"))
    fc, wc = fc[-last:], wc[-last:]
    kern = sorted(set().union(*fc, *wc))
    per = {k: {"read_MB": sum(c.get(k, 0) for c in fc) / len(fc) * 2 * 1024 / 1e6,
               "written_MB": sum(c.get(k, 0) for c in wc) / len(wc) * 1024 / 1e6} for k in kern}
    tot_r = sum(v["read_MB"] for v in per.values())
    tot_w = sum(v["written_MB"] for v in per.values())
    res = {"converges_averaged": len(fc), "per_kernel": per, "read_MB": tot_r, "written_MB": tot_w,
           "moved_MB": tot_r + tot_w, "note": "FETCH_SIZE x 2 (gfx950), WRITE_SIZE as is; KiB -> MB"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k, v in per.items():
        print(f"{k:16s} read {v['read_MB']:8.1f} MB  written {v['written_MB']:8.1f} MB")
    print(f"converge: read {tot_r:.1f} MB, written {tot_w:.1f} MB, moved {tot_r + tot_w:.1f} MB")


if __name__ == "__main__":
    main()
