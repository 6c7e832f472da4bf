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

  python tests/golden/make_fullsize_digests.py [--only treg|tlog|ujson]

(TREG, config 3: synth.treg_tables -- one delta per register per round over
8.39M registers, dense timestamp ties with shared 8-byte value prefixes.)
"""
import argparse
import json
import os
import sys
import time

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
    ap.add_argument("--only", choices=sorted(CONFIGS))
    a = ap.parse_args()
    O.build()
    O.load()
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in sorted(CONFIGS):
        if a.only and name != a.only:
            continue
        out[name] = run(name)
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
