"""Repeat the config-5 UJSON converge sequence (bench.py --type ujson: 1M
docs, Zipf(1.1), R = 16) on fresh engines in ONE process and report, per
repetition, the engine's cumulative counters and a hash of the whole store
(every document's elements, vv and cloud).  The merge is a deterministic
function of its inputs, so every repetition must print the same line;
JY_LIB selects the library under test.

usage: python tools/uj_repro.py [--reps N] [--steps S] [--docs D]"""
import argparse
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--steps", type=int, default=18)
    ap.add_argument("--docs", type=int, default=1 << 20)
    args = ap.parse_args()
    import torch
    from bench_modes import _to_dev
    from jylis_amd import synth as S
    from jylis_amd._lib import UJSON
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoUJSON
    D = args.docs
    st, dl = S.ujson_tables(D, seed=S.BASE_SEED + 5, rounds=args.steps, R=16)
    dev = torch.device("cuda", 0)
    seen = {}
    for rep in range(args.reps):
        eng = Engine(device=0)
        try:
            repo = RepoUJSON(eng)
            repo.converge_deltas(st)
            batches = []
            for b in dl:
                slots = eng.lookup(UJSON, (b["key_bytes"], b["key_offs"]))
                eo, vo, co = (np.asarray(b[k], np.uint64) for k in ("el_offs", "vv_offs", "cloud_offs"))
                dots, elems = repo._sort_segments(eo, repo._pack(b["dot_ids"], b["dot_seqs"]), np.asarray(b["elems"]))
                (vv,) = repo._sort_segments(vo, repo._pack(b["vv_ids"], b["vv_seqs"]))
                (cloud,) = repo._sort_segments(co, repo._pack(b["cloud_ids"], b["cloud_seqs"]))
                batches.append(tuple(_to_dev(a, dev) for a in (slots, eo, dots, elems, vo, vv, co, cloud)))
            eng.sync()
            s0 = eng.ujson_stats()
            for b in batches:
                eng.ujson_converge(*b)
            eng.sync()
            s1 = eng.ujson_stats()
            h = hashlib.sha1()
            for a in eng.ujson_read(np.arange(eng.nkeys(UJSON), dtype=np.uint32)):
                h.update(np.ascontiguousarray(a).tobytes())
            key = (s1["touched_el"] - s0["touched_el"], s1["touched_cloud"] - s0["touched_cloud"],
                   s1["out_cloud"] - s0["out_cloud"], h.hexdigest()[:16])
            seen[key] = seen.get(key, 0) + 1
            print("rep", rep, "touched_el %d touched_cloud %d out_cloud %d state %s" % key, flush=True)
        finally:
            eng.close()
    print("distinct outcomes:", len(seen), flush=True)


if __name__ == "__main__":
    main()
