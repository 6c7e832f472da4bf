"""Localise a nondeterministic UJSON converge: run the config-5 sequence on
fresh engines (one process), fingerprint every delta document after every
converge, and report the first converge and the documents where a
repetition departs from repetition 0 (with their segment sizes).

usage: python tools/uj_diag.py [--reps N] [--steps S] [--docs D]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

M = np.uint64(0x9E3779B97F4A7C15)


def _mix(x):
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _seg_hash(offs, vals, n):
    """per segment: wrapping sum of mixed (value, position) -- order sensitive"""
    offs = np.asarray(offs, np.int64)
    out = np.zeros(n, np.uint64)
    if offs[-1] == 0:
        return out
    pos = np.arange(int(offs[-1]), dtype=np.uint64) - np.repeat(offs[:-1], np.diff(offs)).astype(np.uint64)
    h = _mix(np.asarray(vals[:int(offs[-1])], np.uint64) ^ (pos * M))
    nz = np.nonzero(np.diff(offs))[0]
    out[nz] = np.add.reduceat(h, offs[:-1][nz])
    return out


def fingerprint(eng, slots):
    eo, dots, elems, vv, co, cloud = eng.ujson_read(slots)
    n = len(slots)
    with np.errstate(over="ignore"):
        h = _seg_hash(eo, dots, n) * np.uint64(3) + _seg_hash(eo, elems, n) * np.uint64(5) + \
            _seg_hash(co, cloud, n) * np.uint64(7)
        h += (_mix(np.asarray(vv, np.uint64)) * (np.arange(vv.shape[1], dtype=np.uint64) + np.uint64(1))).sum(
            axis=1, dtype=np.uint64)
    return h, np.diff(np.asarray(eo, np.int64)), np.diff(np.asarray(co, np.int64))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--steps", type=int, default=18)
    ap.add_argument("--docs", type=int, default=1 << 20)
    ap.add_argument("--serial", action="store_true",
                    help="fingerprint the delta docs around every converge (synchronises between converges)")
    args = ap.parse_args()
    import torch
    from bench_modes import _to_dev
    from jylis_amd import synth as S
    from jylis_amd._lib import UJSON
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoUJSON
    st, dl = S.ujson_tables(args.docs, seed=S.BASE_SEED + 5, rounds=args.steps, R=16)
    dev = torch.device("cuda", 0)
    ref = None
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
                dsz = (np.diff(eo.astype(np.int64)), np.diff(co.astype(np.int64)), np.diff(vo.astype(np.int64)))
                batches.append((slots, tuple(_to_dev(a, dev) for a in (slots, eo, dots, elems, vo, vv, co, cloud)),
                                dsz))
            eng.sync()
            if not args.serial:
                # converges pipelined as in the bench; the whole store fingerprinted at the end
                for slots, b, dsz in batches:
                    eng.ujson_converge(*b)
                eng.sync()
                allslots = np.arange(eng.nkeys(UJSON), dtype=np.uint32)
                fp = fingerprint(eng, allslots)
                if ref is None:
                    ref = fp
                    print("rep 0: reference", flush=True)
                    continue
                docs = np.nonzero(ref[0] != fp[0])[0]
                print("rep", rep, "identical" if len(docs) == 0 else "differs in %d docs" % len(docs), flush=True)
                hits = {}
                for j, (slots, b, dsz) in enumerate(batches):
                    pos = {int(x): i for i, x in enumerate(slots)}
                    for d in docs[:12]:
                        if int(d) in pos:
                            i = pos[int(d)]
                            hits.setdefault(int(d), []).append((j, int(dsz[0][i]), int(dsz[1][i]), int(dsz[2][i])))
                for d in docs[:12]:
                    print("  doc %d: final el %d/%d cloud %d/%d; in converges (j, delta el, cloud, vv): %s"
                          % (d, ref[1][d], fp[1][d], ref[2][d], fp[2][d], hits.get(int(d), [])[:8]), flush=True)
                continue
            fps = []
            for j, (slots, b, dsz) in enumerate(batches):
                before = fingerprint(eng, slots)
                eng.ujson_converge(*b)
                eng.sync()
                fps.append((before, fingerprint(eng, slots)))
            if ref is None:
                ref = fps
                print("rep 0: reference", flush=True)
                continue
            bad = None
            for j, ((b0, a0), (b1, a1)) in enumerate(zip(ref, fps)):
                if not np.array_equal(b0[0], b1[0]):
                    bad = (j, "before", np.nonzero(b0[0] != b1[0])[0])
                    break
                if not np.array_equal(a0[0], a1[0]):
                    bad = (j, "after", np.nonzero(a0[0] != a1[0])[0])
                    break
            if bad is None:
                print("rep", rep, "identical", flush=True)
                continue
            j, when, docs = bad
            slots, _, dsz = batches[j]
            print("rep", rep, "differs at converge", j, when, "in", len(docs), "of", len(slots), "delta docs",
                  flush=True)
            (b0, a0), (b1, a1) = ref[j], fps[j]
            for d in docs[:12]:
                print("  doc slot %d: state el %d cloud %d | delta el %d cloud %d vv %d | after el %d/%d cloud %d/%d"
                      % (slots[d], b0[1][d], b0[2][d], dsz[0][d], dsz[1][d], dsz[2][d], a0[1][d], a1[1][d],
                         a0[2][d], a1[2][d]), flush=True)
        finally:
            eng.close()


if __name__ == "__main__":
    main()
