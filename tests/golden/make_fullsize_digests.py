#!/usr/bin/env python3
"""Full-size golden digests for SURVEY 8d configs 3, 4 and 5 (run in the build
container; the GPU box only reads the JSON this writes).

The exact seeded sequences the bench converges (bench_modes.bench_tlog /
bench_ujson at rank 0: the state, then one delta round per warmup + timed
step) are fed through the CPU oracle (oracle/jy_oracle.cpp, the restatement
of RepoManagerCore.converge_deltas + pony-crdt's joins, pinned by the
reference's own vectors: tests/test_oracle_kat.py), and the canonical state
digest (oracle.digest_repo) is recorded after every converge, with a digest
of every input batch so the GPU test can tell a changed generator from a
wrong merge.  tests/test_fullsize_gpu.py runs the same sequences through the
HIP path and compares.

  python tests/golden/make_fullsize_digests.py [--only treg|tlog|ujson|gcount|pncount]

(TREG, config 3: synth.treg_tables -- one delta per register per round over
8.39M registers, dense timestamp ties with shared 8-byte value prefixes.)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
from jylis_amd import synth as S  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "fullsize_digests.json")

# the bench's sequences (gpu_round.sh: --warmup 2 / 6, --steps 8)
CONFIGS = {
    "treg": {"ctype": O.TREG, "keys": 8 << 20, "seed": S.BASE_SEED + 3, "rounds": 6},
    "tlog": {"ctype": O.TLOG, "keys": 4 << 20, "seed": S.BASE_SEED + 4, "rounds": 10},
    "ujson": {"ctype": O.UJSON, "keys": 1 << 20, "seed": S.BASE_SEED + 5, "rounds": 14, "R": 16},
}


# configs 1 and 2 (round 5): the bench's counter sequences -- the state, then
# the `rounds` distinct delta batches of its chain (bench.py / bench_gcount
# cycle them; the batches after the first cycle change nothing).  The oracle
# cannot hold 16M keys x 64 replicas x 2 signs of hash maps at once, and the
# digest is a wrapping sum over keys, so key ranges are converged and
# digested separately (CHUNK keys each, on every CPU) and their digests summed.
COUNTERS = {
    "gcount": {"ctype": O.GCOUNT, "keys": 1 << 20, "R": 16, "nsigns": 1, "seed": S.BASE_SEED + 1, "rounds": 4,
               "prefix": "s0:g", "width": 7, "wrap_frac": False},
    "pncount": {"ctype": O.PNCOUNT, "keys": 16 << 20, "R": 64, "nsigns": 2, "seed": S.BASE_SEED + 2, "rounds": 4,
                "prefix": "s0:p", "width": 8, "wrap_frac": True},
}
CHUNK = 1 << 16


def counter_chunk(job):
    """the oracle's digests after every converge, keys [a, b) of a counter config"""
    name, a, b = job
    c = COUNTERS[name]
    O.load()
    K, R, G = c["keys"], c["R"], c["nsigns"]
    n = b - a
    kb, ko = S.counter_keys(n, prefix=c["prefix"].encode(), width=c["width"], start=a)
    rids = S.replica_ids(R, c["seed"])
    cells = ((np.arange(G, dtype=np.uint64)[:, None, None] * np.uint64(R * K)) +
             (np.arange(R, dtype=np.uint64)[None, :, None] * np.uint64(K)) +
             np.arange(a, b, dtype=np.uint64)[None, None, :])
    cur = S.counter_state_np(K, R, G, c["seed"], wrap_frac=c["wrap_frac"], cells=cells)
    repo = O.Repo(c["ctype"])
    out = []
    for j in range(-1, c["rounds"]):
        if j >= 0:
            cur = S.counter_delta_np(cur, j, c["seed"], cells=cells)
        repo.converge(_all_columns(cur, rids, kb, ko))
        out.append(O.digest_repo(repo))
    return out


def _all_columns(arr, rids, kb, ko):
    """one table carrying every replica column of [nsigns][R][n]: each key's
    delta holds all R replica entries.  The join is per (key, replica), so
    this converges to exactly what the R peer batches one column each
    (S.counter_batch_tables, the bench's shape) converge to, with R times
    fewer per-key delta objects for the oracle to build"""
    G, R, n = arr.shape
    t = {"key_bytes": kb, "key_offs": ko}
    for g, pre in zip(range(G), ("p_", "n_") if G == 2 else ("",)):
        t[pre + "offs"] = np.arange(n + 1, dtype=np.uint64) * np.uint64(R)
        t[pre + "ids"] = np.tile(np.asarray(rids, np.uint64), n)
        t[pre + "vals"] = np.ascontiguousarray(arr[g].T).reshape(-1).astype(np.uint64)
    return t


def run_counter(name, workers):
    import multiprocessing as mp
    c = COUNTERS[name]
    jobs = [(name, a, min(a + CHUNK, c["keys"])) for a in range(0, c["keys"], CHUNK)]
    t0 = time.time()
    tot = [[0, 0, 0, 0] for _ in range(c["rounds"] + 1)]
    with mp.get_context("fork").Pool(workers) as pool:
        for k, res in enumerate(pool.imap_unordered(counter_chunk, jobs)):
            for i, d in enumerate(res):
                tot[i] = [(x + y) % (1 << 64) for x, y in zip(tot[i], d)]
            if k % 16 == 0:
                print(f"{name}: {k + 1}/{len(jobs)} key ranges in {time.time() - t0:.0f} s", flush=True)
    return {**{k: v for k, v in c.items() if k != "ctype"}, "ctype": int(c["ctype"]), "chunk": CHUNK,
            "states": [[str(x) for x in d] for d in tot],
            "digest": "oracle.digest_repo summed over key ranges: {digest, keys, non-zero entries, "
                      "wrapping sum of the entries}"}


def sequence(name):
    c = CONFIGS[name]
    if name == "treg":
        return S.treg_tables(c["keys"], seed=c["seed"], rounds=c["rounds"])
    if name == "tlog":
        return S.tlog_tables(c["keys"], seed=c["seed"], rounds=c["rounds"])
    return S.ujson_tables(c["keys"], seed=c["seed"], rounds=c["rounds"], R=c["R"])


def run(name):
    c = CONFIGS[name]
    t0 = time.time()
    st, dl = sequence(name)
    print(f"{name}: generated in {time.time() - t0:.1f} s", flush=True)
    repo = O.Repo(c["ctype"])
    inputs, states = [], []
    for i, b in enumerate([st] + dl):
        inputs.append(list(O.digest_table(c["ctype"], b)))
        t1 = time.time()
        repo.converge(b)
        states.append(list(O.digest_repo(repo)))
        print(f"{name}: converge {i} in {time.time() - t1:.1f} s -> {states[-1]}", flush=True)
    return {**{k: v for k, v in c.items() if k != "ctype"}, "ctype": int(c["ctype"]),
            "inputs": [[str(x) for x in d] for d in inputs],
            "states": [[str(x) for x in d] for d in states],
            "digest": "oracle.digest_repo / digest_table: {digest, keys, entries or elements, bytes or cloud dots}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=sorted(CONFIGS) + sorted(COUNTERS))
    ap.add_argument("--workers", type=int, default=os.cpu_count() or 1)
    a = ap.parse_args()
    O.build()
    O.load()
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in sorted(CONFIGS) + sorted(COUNTERS):
        if a.only and name != a.only:
            continue
        out[name] = run_counter(name, a.workers) if name in COUNTERS else run(name)
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
