"""UJSON: the HIP dot-kernel join against the CPU oracle (bit-exact on the
canonical state: element dots, version vector, compacted cloud).

Edge cases: concurrent INS/RM of one value (add wins, ujson.md:61,103),
CLR racing INS, re-delivered deltas (idempotence), clouds that compact into
the version vector, equal dots in state and delta, repeated docs in one
batch, malformed deltas (unsorted dots, column beyond the vv width)."""
import numpy as np
import pytest

from helpers import assert_state_equal, random_history

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_history_parity(oracle_mod, engine, seed):
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    want = O.Repo(O.UJSON, 5)
    got = RepoUJSON(engine)
    for b in random_history(O, O.UJSON, seed, nops=400):
        want.converge(b)
        got.converge_deltas(b)
    assert_state_equal(O.UJSON, want.state(), got.state())


def test_add_wins_and_redelivery(oracle_mod, engine):
    """replica a removes value 7 while replica b concurrently re-inserts it:
    after exchange both see 7 (add wins); re-delivering every delta is a no-op"""
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    a, b = O.Repo(O.UJSON, 11), O.Repo(O.UJSON, 22)
    a.ujson_ins("doc", 7)
    a.ujson_ins("doc", 8)
    d0 = a.flush().table()
    b.converge(d0)
    a.ujson_rm("doc", 7)
    b.ujson_ins("doc", 7)
    b.ujson_clr("other")  # no key creation on CLR of a missing doc
    da, db = a.flush().table(), b.flush().table()
    want = O.Repo(O.UJSON, 33)
    got = RepoUJSON(engine)
    for t in (d0, da, db, da, d0, db):
        want.converge(t)
        got.converge_deltas(t)
    assert_state_equal(O.UJSON, want.state(), got.state())
    assert got.elements("doc") == {7, 8}


def test_repeated_docs_in_one_batch(oracle_mod, engine):
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    r = O.Repo(O.UJSON, 3)
    parts = []
    for e in (1, 2, 3):
        r.ujson_ins("k", e)
        parts.append(r.flush().table())
    r.ujson_rm("k", 2)
    parts.append(r.flush().table())
    # concatenate the four 1-doc batches into one batch naming "k" four times
    cat = {}
    for k in parts[0]:
        if k.endswith("offs"):
            acc = [np.zeros(1, np.uint64)]
            base = 0
            for p in parts:
                acc.append(p[k][1:] + np.uint64(base))
                base = int(acc[-1][-1]) if len(acc[-1]) else base
            cat[k] = np.concatenate(acc)
        else:
            cat[k] = np.concatenate([p[k] for p in parts])
    want = O.Repo(O.UJSON, 9)
    got = RepoUJSON(engine)
    want.converge(cat)
    got.converge_deltas(cat)
    assert_state_equal(O.UJSON, want.state(), got.state())
    assert got.elements("k") == {1, 3}


def test_malformed_delta_is_skipped(engine):
    from jylis_amd.engine import pack_dot
    engine.intern(4, ["good", "bad"])
    slots = np.array([0, 1], np.uint32)
    eo = np.array([0, 1, 3], np.uint64)
    dots = np.concatenate([pack_dot([0], [1]), pack_dot([0, 0], [5, 2])])  # second doc unsorted
    elems = np.array([10, 11, 12], np.uint64)
    vo = np.zeros(3, np.uint64)
    co = np.array([0, 1, 2], np.uint64)
    cloud = np.concatenate([pack_dot([0], [1]), pack_dot([0], [9])])
    engine.ujson_converge(slots, eo, dots, elems, vo, np.zeros(0, np.uint64), co, cloud)
    assert engine.skipped() == 1
    eoffs, d, e, vv, coffs, cl = engine.ujson_read(slots)
    assert list(e) == [10] and vv[0][0] == 1 and len(cl) == 0  # dot (0,1) compacted into vv
    assert vv[1].sum() == 0


@pytest.mark.parametrize("R", [16, 4, 40])  # R = 40: vv rows wider than a doc tile row batch
def test_synthetic_zipf(oracle_mod, R):
    """config-5 shaped stream at 3000 docs: Zipf(1.1) popularity, INS/RM/CLR mix"""
    from jylis_amd import synth as S
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    eng = Engine(device=0, ujson_columns=R)
    try:
        st, dl = S.ujson_tables(3000, seed=S.BASE_SEED + 5, rounds=3, R=R)
        want = O.Repo(O.UJSON, 1)
        got = RepoUJSON(eng)
        for b in [st] + dl:
            want.converge(b)
            got.converge_deltas(b)
        assert_state_equal(O.UJSON, want.state(), got.state())
    finally:
        eng.close()


def test_many_rounds_pool_reuse(oracle_mod):
    """six Zipf rounds on small pools: only touched documents are rewritten,
    the pools are compacted several times, state compared after every round"""
    from jylis_amd import synth as S
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    eng = Engine(device=0, ujson_columns=8, entry_capacity=1024)
    try:
        st, dl = S.ujson_tables(2000, seed=S.BASE_SEED + 50, rounds=6, R=8)
        want = O.Repo(O.UJSON, 1)
        got = RepoUJSON(eng)
        for b in [st] + dl:
            want.converge(b)
            got.converge_deltas(b)
            assert_state_equal(O.UJSON, want.state(), got.state())
        full = want.state()  # a full-state delta changes nothing
        want.converge(full)
        got.converge_deltas(full)
        assert_state_equal(O.UJSON, want.state(), got.state())
    finally:
        eng.close()


def test_hot_document_long_segments(oracle_mod):
    """one document of 24,000 elements next to small ones: long segments go
    through U1's tile maps, and the read gathers a document over many tiles
    (jy_ujson_read is flattened over the output); deltas insert and remove
    thousands of its dots"""
    from jylis_amd import synth as S
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    R = 8
    ids = S.replica_ids(R, 77)
    rng = np.random.default_rng(12)
    keys = [b"hot"] + [b"cold%d" % i for i in range(40)]

    def table(docs):
        """docs: list of (key, {(col, seq): elem}, {col: n}, {(col, seq)})"""
        from jylis_amd.engine import encode_keys
        t = {k: [] for k in ("dot_ids", "dot_seqs", "elems", "vv_ids", "vv_seqs", "cloud_ids", "cloud_seqs")}
        eo, vo, co = [0], [0], [0]
        for _, els, vv, cl in docs:
            for (c, q), e in sorted(els.items()):
                t["dot_ids"].append(ids[c]), t["dot_seqs"].append(q), t["elems"].append(e)
            for c, n in sorted(vv.items()):
                t["vv_ids"].append(ids[c]), t["vv_seqs"].append(n)
            for c, q in sorted(cl):
                t["cloud_ids"].append(ids[c]), t["cloud_seqs"].append(q)
            eo.append(len(t["elems"])), vo.append(len(t["vv_ids"])), co.append(len(t["cloud_ids"]))
        out = {k: np.array(v, np.uint64) for k, v in t.items()}
        out["key_bytes"], out["key_offs"] = encode_keys([d[0] for d in docs])
        out["el_offs"], out["vv_offs"], out["cloud_offs"] = (np.array(x, np.uint64) for x in (eo, vo, co))
        return out

    hot = {(c, q): int(rng.integers(1, 1 << 40)) for c in range(R) for q in range(1, 3001)}
    state = [(b"hot", hot, {c: 3000 for c in range(R)}, set())]
    for k in keys[1:]:
        els = {(int(c), q): int(rng.integers(1, 99)) for c in rng.integers(0, R, 3) for q in (1, 2)}
        state.append((k, els, {c: 2 for c in range(R)}, set()))
    batches = [table(state)]
    for rnd in range(3):
        # the hot doc: 2000 fresh dots, 2500 of its dots removed (context only)
        new = {(int(c), 3000 + 1000 * rnd + int(q)): int(rng.integers(1, 1 << 40))
               for c, q in zip(rng.integers(0, R, 2000), rng.integers(1, 900, 2000))}
        rm = {(int(c), int(q)) for c, q in zip(rng.integers(0, R, 2500), rng.integers(1, 3001, 2500))}
        docs = [(b"hot", new, {}, set(new) | rm)]
        docs.append((keys[1 + rnd], {(0, 10 + rnd): 5}, {}, {(0, 10 + rnd), (1, 1)}))
        batches.append(table(docs))
    eng = Engine(device=0, ujson_columns=R)
    try:
        want = O.Repo(O.UJSON, 1)
        got = RepoUJSON(eng)
        for b in batches:
            want.converge(b)
            got.converge_deltas(b)
            assert_state_equal(O.UJSON, want.state(), got.state())
    finally:
        eng.close()


def test_hot_document_long_cloud(oracle_mod):
    """a document whose causal context holds thousands of gapped cloud dots
    over every column, then deltas that fill some gaps (the runs fold into the
    vv) and leave others: long cloud segments take the wave-cooperative
    searches of U2 / U3 on both the state and the delta side, and the waves
    straddle column boundaries"""
    from jylis_amd import synth as S
    from jylis_amd.engine import Engine, encode_keys
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    R = 6
    ids = S.replica_ids(R, 91)
    rng = np.random.default_rng(21)

    def table(docs):
        t = {k: [] for k in ("dot_ids", "dot_seqs", "elems", "vv_ids", "vv_seqs", "cloud_ids", "cloud_seqs")}
        eo, vo, co = [0], [0], [0]
        for _, els, vv, cl in docs:
            for (c, q), e in sorted(els.items()):
                t["dot_ids"].append(ids[c]), t["dot_seqs"].append(q), t["elems"].append(e)
            for c, n in sorted(vv.items()):
                t["vv_ids"].append(ids[c]), t["vv_seqs"].append(n)
            for c, q in sorted(cl):
                t["cloud_ids"].append(ids[c]), t["cloud_seqs"].append(q)
            eo.append(len(t["elems"])), vo.append(len(t["vv_ids"])), co.append(len(t["cloud_ids"]))
        out = {k: np.array(v, np.uint64) for k, v in t.items()}
        out["key_bytes"], out["key_offs"] = encode_keys([d[0] for d in docs])
        out["el_offs"], out["vv_offs"], out["cloud_offs"] = (np.array(x, np.uint64) for x in (eo, vo, co))
        return out

    # state: vv = 1 per column, the odd seqs 3, 5, ... up to ~2 * 700 in the
    # cloud, an element under every fourth cloud dot
    cl = {(c, q) for c in range(R) for q in range(3, 3 + 2 * int(rng.integers(500, 900)), 2)}
    els = {d: int(rng.integers(1, 1 << 30)) for d in sorted(cl)[::4]}
    batches = [table([(b"hot", els, {c: 1 for c in range(R)}, cl), (b"cold", {(0, 1): 3}, {0: 1}, set())])]
    for rnd in range(3):
        # fill the gaps 2, 4, ... of some columns up to a random point (a
        # contiguous run folds), plus scattered even dots further up
        dcl = set()
        for c in range(R):
            top = int(rng.integers(0, 1200))
            dcl |= {(c, q) for q in range(2, top, 2)}
            dcl |= {(c, int(q)) for q in rng.integers(top, 2000, 40) if q % 2 == 0}
        dels = {d: int(rng.integers(1, 1 << 30)) for d in sorted(dcl)[::7]}
        batches.append(table([(b"hot", dels, {}, dcl)]))
    eng = Engine(device=0, ujson_columns=R)
    try:
        want = O.Repo(O.UJSON, 1)
        got = RepoUJSON(eng)
        for b in batches:
            want.converge(b)
            got.converge_deltas(b)
            assert_state_equal(O.UJSON, want.state(), got.state())
    finally:
        eng.close()
