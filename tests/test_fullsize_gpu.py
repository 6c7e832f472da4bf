"""Configs 3, 4 and 5 at FULL size against the oracle (config 3: TREG over
8.39M registers, below); configs 4 and 5: the exact seeded
sequences the bench converges (4M TLOG logs x 10 delta rounds; 1M UJSON
documents, Zipf(1.1), x 14 delta rounds) through the HIP path, the canonical
state digest after every converge compared with the oracle's
(tests/golden/fullsize_digests.json, made by
tests/golden/make_fullsize_digests.py in the build container), then the
whole sequence again with every converge enqueued back to back (the way the
bench pipelines them) and the final digest compared.

Reference: RepoTLOG.converge / RepoUJSON.converge (jylis/repo_tlog.pony:66-67,
repo_ujson.pony:65-66) over RepoManagerCore.converge_deltas
(repo_manager.pony:92-93); the digests are defined in oracle/jy_oracle.cpp
(or_digest_*) and cross-checked on CPU by tests/test_digest.py."""
import json
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize_digests.json")


def _progress(msg):
    """long test: a line per converge into $JY_PROGRESS (the GPU runner's
    liveness file), if set"""
    p = os.environ.get("JY_PROGRESS")
    if p:
        with open(p, "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


def _golden(name):
    if not os.path.exists(GOLDEN):
        pytest.fail("tests/golden/fullsize_digests.json is missing: run tests/golden/make_fullsize_digests.py")
    g = json.load(open(GOLDEN))[name]
    return g, [tuple(int(x) for x in d) for d in g["inputs"]], [tuple(int(x) for x in d) for d in g["states"]]


def _dev(a, dev):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).to(dev)


def _tlog_digest(O, eng, kb, ko, arena):
    from jylis_amd._lib import TLOG
    K = len(ko) - 1
    cut, offs, ts, pre, lr = eng.tlog_read(np.arange(K, dtype=np.uint32))
    return O.digest_tlog_handles(kb, ko, cut, offs, ts, pre, lr, arena)


@pytest.mark.timeout(1200)
def test_tlog_config4_fullsize(oracle_mod):
    import torch
    from jylis_amd import synth as S
    from jylis_amd._lib import TLOG
    from jylis_amd.engine import Engine
    O = oracle_mod
    g, inputs, states = _golden("tlog")
    K = g["keys"]
    st, dl = S.tlog_tables(K, seed=g["seed"], rounds=g["rounds"])
    batches = [st] + dl
    _progress(f"tlog: generated {len(batches)} batches")
    for i, b in enumerate(batches):  # the same inputs as the oracle's
        assert O.digest_table(TLOG, b) == inputs[i], f"generator drift at batch {i}"
    dev = torch.device("cuda", 0)
    for pipelined in (False, True):
        eng = Engine(device=0, key_capacity=[1024, 1024, 1024, K, 1024])
        try:
            slots = eng.intern(TLOG, (st["key_bytes"], st["key_offs"]))
            assert (slots == np.arange(K)).all()
            dslots = _dev(slots, dev)
            devb = []
            for b in batches:
                pre, lr = eng.pack_values(TLOG, (b["val_bytes"], b["val_offs"]))
                devb.append((dslots,) + tuple(_dev(a, dev) for a in (b["cutoff"], b["ent_offs"], b["ts"], pre, lr)))
            n, _ = eng.arena_usage(TLOG)
            arena = np.frombuffer(eng.arena_read(TLOG, 0, n), np.uint8)  # merges append nothing to it
            for i, b in enumerate(devb):
                eng.tlog_converge(*b)
                if not pipelined:
                    got = _tlog_digest(O, eng, st["key_bytes"], st["key_offs"], arena)
                    _progress(f"tlog converge {i}: {got}")
                    assert got == states[i], f"TLOG state after converge {i} differs from the oracle's"
            if pipelined:
                eng.sync()
                got = _tlog_digest(O, eng, st["key_bytes"], st["key_offs"], arena)
                _progress(f"tlog pipelined: {got} {eng.tlog_stats()}")
                assert got == states[-1], "TLOG state after the pipelined sequence differs from the oracle's"
        finally:
            eng.close()


def _ujson_digest(O, eng, kb, ko):
    D = len(ko) - 1
    eo, dots, elems, vv, co, cloud = eng.ujson_read(np.arange(D, dtype=np.uint32))
    col_ids = np.array([eng.replica_id(c) for c in range(eng.replica_count())], np.uint64)
    return O.digest_ujson_packed(kb, ko, eo, dots, elems, vv, co, cloud, col_ids)


@pytest.mark.timeout(1200)
def test_ujson_config5_fullsize(oracle_mod):
    import torch
    from jylis_amd import synth as S
    from jylis_amd._lib import UJSON
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    g, inputs, states = _golden("ujson")
    D = g["keys"]
    st, dl = S.ujson_tables(D, seed=g["seed"], rounds=g["rounds"], R=g["R"])
    _progress(f"ujson: generated {1 + len(dl)} batches")
    for i, b in enumerate([st] + dl):
        assert O.digest_table(UJSON, b) == inputs[i], f"generator drift at batch {i}"
    dev = torch.device("cuda", 0)
    for pipelined in (False, True):
        eng = Engine(device=0, counter_columns=16)
        try:
            repo = RepoUJSON(eng)
            repo.converge_deltas(st)  # the bench's setup converge (host marshalling)
            slots = eng.lookup(UJSON, (st["key_bytes"], st["key_offs"]))
            assert (slots == np.arange(D)).all()
            if not pipelined:
                got = _ujson_digest(O, eng, st["key_bytes"], st["key_offs"])
                assert got == states[0], "UJSON state after the setup converge differs from the oracle's"
            devb = []
            for b in dl:  # as bench_modes.bench_ujson: device batches
                s = eng.lookup(UJSON, (b["key_bytes"], b["key_offs"]))
                eo, vo, co = (np.asarray(b[k], np.uint64) for k in ("el_offs", "vv_offs", "cloud_offs"))
                dots, elems = repo._sort_segments(eo, repo._pack(b["dot_ids"], b["dot_seqs"]), np.asarray(b["elems"]))
                (vv,) = repo._sort_segments(vo, repo._pack(b["vv_ids"], b["vv_seqs"]))
                (cloud,) = repo._sort_segments(co, repo._pack(b["cloud_ids"], b["cloud_seqs"]))
                devb.append(tuple(_dev(a, dev) for a in (s, eo, dots, elems, vo, vv, co, cloud)))
            for i, b in enumerate(devb):
                eng.ujson_converge(*b)
                if not pipelined:
                    got = _ujson_digest(O, eng, st["key_bytes"], st["key_offs"])
                    _progress(f"ujson converge {i + 1}: {got}")
                    assert got == states[i + 1], f"UJSON state after converge {i + 1} differs from the oracle's"
            if pipelined:
                eng.sync()
                got = _ujson_digest(O, eng, st["key_bytes"], st["key_offs"])
                _progress(f"ujson pipelined: {got}")
                assert got == states[-1], "UJSON state after the pipelined sequence differs from the oracle's"
        finally:
            eng.close()


@pytest.mark.timeout(900)
def test_treg_config3_fullsize(oracle_mod):
    """Config 3 at full size: 8.39M registers, one delta per register per
    round (synth.treg_tables: dense timestamp ties, shared 8-byte prefixes),
    the rounds alternating between the block form (jy_treg_converge_block)
    and the keyed form with the slots in HBM; the digest after every
    converge against the oracle's, then the whole sequence pipelined"""
    import torch
    from jylis_amd import synth as S
    from jylis_amd._lib import TREG
    from jylis_amd.engine import Engine
    O = oracle_mod
    g, inputs, states = _golden("treg")
    K = g["keys"]
    st, dl = S.treg_tables(K, seed=g["seed"], rounds=g["rounds"])
    batches = [st] + dl
    _progress(f"treg: generated {len(batches)} batches")
    for i, b in enumerate(batches):
        assert O.digest_table(TREG, b) == inputs[i], f"generator drift at batch {i}"
    dev = torch.device("cuda", 0)
    for pipelined in (False, True):
        eng = Engine(device=0, key_capacity=[1024, 1024, K, 1024, 1024])
        try:
            slots = eng.intern(TREG, (st["key_bytes"], st["key_offs"]))
            assert (slots == np.arange(K)).all()
            dslots = _dev(slots, dev)
            devb = []
            for b in batches:
                pre, lr = eng.pack_values(TREG, (b["val_bytes"], b["val_offs"]))
                devb.append(tuple(_dev(a, dev) for a in (b["ts"], pre, lr)))
            for i, (ts, pre, lr) in enumerate(devb):
                if i % 2 == 0:
                    eng.treg_converge_block(0, ts, pre, lr)
                else:
                    eng.treg_converge(dslots, ts, pre, lr)
                if not pipelined:
                    got = _treg_digest(O, eng, st["key_bytes"], st["key_offs"])
                    _progress(f"treg converge {i}: {got}")
                    assert got == states[i], f"TREG state after converge {i} differs from the oracle's"
            if pipelined:
                eng.sync()
                got = _treg_digest(O, eng, st["key_bytes"], st["key_offs"])
                _progress(f"treg pipelined: {got}")
                assert got == states[-1], "TREG state after the pipelined sequence differs from the oracle's"
        finally:
            eng.close()


def _treg_digest(O, eng, kb, ko):
    from jylis_amd._lib import TREG
    K = len(ko) - 1
    ts, pre, lr = eng.treg_read(np.arange(K, dtype=np.uint32))
    n, _ = eng.arena_usage(TREG)
    arena = np.frombuffer(eng.arena_read(TREG, 0, n), np.uint8) if n else np.zeros(0, np.uint8)
    return O.digest_treg_handles(kb, ko, ts, pre, lr, arena)


def _counter_digest(O, eng, ctype, kb, ko, ids, R, chunk=1 << 20):
    """the engine's dense counter state of every key, digested in key chunks
    (the digest is a wrapping sum over keys)"""
    K = len(ko) - 1
    tot = [0, 0, 0, 0]
    for s0 in range(0, K, chunk):
        n = min(chunk, K - s0)
        vals = eng.counter_export(ctype, R, s0, n)
        a, b = int(ko[s0]), int(ko[s0 + n])
        d = O.digest_counter_dense(kb[a:b], ko[s0:s0 + n + 1] - np.uint64(a), ids, vals)
        tot = [(x + y) % (1 << 64) for x, y in zip(tot, d)]
    return tuple(tot)


@pytest.mark.timeout(1500)
@pytest.mark.parametrize("name", ["gcount", "pncount"])
def test_counter_config_fullsize(oracle_mod, name):
    """Configs 1 and 2 at full size: the bench's exact sequences (bench_gcount:
    1M keys x 16 replicas; bench.py's headline: 16M keys x 64 replicas x
    {P, N}) -- the state, then the chain of distinct delta batches, each one
    block converge of every peer column -- with the canonical digest of the
    WHOLE state after every converge against the oracle's (made key range by
    key range by tests/golden/make_fullsize_digests.py), then every batch
    re-applied (idempotence: the digest must not move).
    Reference: RepoGCOUNT.converge / RepoPNCOUNT.converge
    (jylis/repo_gcount.pony:50-51, repo_pncount.pony:52-53)."""
    import torch
    from jylis_amd import synth as S
    from jylis_amd.engine import Engine
    O = oracle_mod
    gj = json.load(open(GOLDEN))
    if name not in gj:
        pytest.fail(f"tests/golden/fullsize_digests.json has no {name}: run make_fullsize_digests.py --only {name}")
    g = gj[name]
    states = [tuple(int(x) for x in d) for d in g["states"]]
    ctype, K, R, G, seed = g["ctype"], g["keys"], g["R"], g["nsigns"], g["seed"]
    kb, ko = S.counter_keys(K, prefix=g["prefix"].encode(), width=g["width"])
    ids = S.replica_ids(R, seed)
    dev = torch.device("cuda", 0)
    caps = [1024] * 5
    caps[ctype] = K
    eng = Engine(device=0, counter_columns=R, key_capacity=caps)
    try:
        slots = eng.intern(ctype, (kb, ko))
        assert slots[0] == 0 and slots[-1] == K - 1
        cols = eng.replica_cols(ids.tolist())
        assert (cols == np.arange(R)).all()

        def apply(x):
            if G == 2:
                eng.pncount_converge_block(cols, 0, x[0], x[1])
            else:
                eng.gcount_converge_block(cols, 0, x[0])
        cur = torch.empty((G, R, K), dtype=torch.int64, device=dev)
        S.counter_rows_torch(cur, seed, wrap_frac=g["wrap_frac"])
        apply(cur)
        got = _counter_digest(O, eng, ctype, kb, ko, ids, R)
        _progress(f"{name} state: {got}")
        assert got == states[0], f"{name}: the loaded state differs from the oracle's"
        first = None
        for j in range(g["rounds"]):
            nxt = torch.empty_like(cur)
            S.counter_rows_torch(nxt, seed, rnd=j, prev=cur)
            if j == 0:
                first = nxt
            apply(nxt)
            got = _counter_digest(O, eng, ctype, kb, ko, ids, R)
            _progress(f"{name} converge {j + 1}: {got}")
            assert got == states[j + 1], f"{name}: state after delta batch {j} differs from the oracle's"
            if j > 0:
                del cur
            cur = nxt
        apply(first)  # the bench cycles its batches: nothing moves
        apply(cur)
        assert _counter_digest(O, eng, ctype, kb, ko, ids, R) == states[-1], f"{name}: a re-applied batch moved"
    finally:
        eng.close()
