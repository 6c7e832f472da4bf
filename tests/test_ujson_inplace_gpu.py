"""UJSON in-place layout of long documents (k_ujson.hip, round 6) against the
CPU oracle, bit-exact, after every batch.

A document of at least `long_min` elements keeps one element run and one
cloud run per replica column with room; an append-shaped delta (every dot
above what the state's column holds, or already covered and removing
nothing) is appended in place, anything else demotes the document to the
regular merge path, and a column run that overflows moves to a larger run.
The tests force the layout onto small documents (long_min 1..8) so every
path runs: promotion, in-place appends, cloud folds into the vv (empty cloud
runs), regrowth, demotion (a removed live element, a vv entry above the
state's, a dot below the column's top that the state has not seen), repeated
and malformed deltas of a long document, compaction with long documents,
reads, the write path and flush, and pipelined converges (determinism).
The semantics are the reference's join (ujson.md:172-182,
repo_ujson.pony:65-66) as the oracle restates it."""
import hashlib

import numpy as np
import pytest

from helpers import assert_state_equal, random_history

pytestmark = pytest.mark.gpu


def _engine(R=8, long_min=1, **kw):
    from jylis_amd.engine import Engine
    e = Engine(device=0, ujson_columns=R, **kw)
    e.ujson_set_inplace(long_min)
    return e


def _table(ids, docs):
    """docs: [(key, {(col, seq): elem}, {col: n}, {(col, seq)})] -> batch table"""
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


def _run(O, eng, batches, check_every=True):
    from jylis_amd.repo import RepoUJSON
    want = O.Repo(O.UJSON, 1)
    got = RepoUJSON(eng)
    for b in batches:
        want.converge(b)
        got.converge_deltas(b)
        if check_every:
            assert_state_equal(O.UJSON, want.state(), got.state())
    assert_state_equal(O.UJSON, want.state(), got.state())
    return eng.ujson_stats()


@pytest.mark.parametrize("long_min", [1, 3])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_inplace_history_parity(oracle_mod, seed, long_min):
    """oracle write-path histories (INS / RM / CLR on four replicas, partial
    gossip, full-state deltas) with every document in the long layout"""
    O = oracle_mod
    eng = _engine(R=16, long_min=long_min)
    try:
        st = _run(O, eng, random_history(O, O.UJSON, seed, nops=400))
        assert st["promoted"] > 0 and st["inplace_docs"] > 0
    finally:
        eng.close()


@pytest.mark.parametrize("R", [16, 5])
def test_inplace_synthetic_zipf(oracle_mod, R):
    """config-5 shaped stream (Zipf(1.1), INS / RM / CLR mix) over 8 rounds:
    hot documents promoted, appended in place round after round, regrown"""
    from jylis_amd import synth as S
    O = oracle_mod
    eng = _engine(R=R, long_min=8)
    try:
        st0, dl = S.ujson_tables(2000, seed=S.BASE_SEED + 61, rounds=8, R=R)
        st = _run(O, eng, [st0] + dl)
        assert st["promoted"] > 0 and st["inplace_docs"] > 0 and st["inplace_added_el"] > 0
    finally:
        eng.close()


def test_inplace_appends_folds_and_regrowth(oracle_mod):
    """one document appended to over many rounds: fresh dots contiguous with
    the vv (folded while its column's cloud is empty), past gaps (the cloud
    run fills), enough of them to outgrow every column run several times; a
    neighbour document stays regular"""
    from jylis_amd import synth as S
    O = oracle_mod
    R = 6
    ids = S.replica_ids(R, 17)
    rng = np.random.default_rng(5)
    top = [0] * R
    batches = []
    for rnd in range(12):
        els, cl = {}, set()
        for c in range(R):
            for _ in range(int(rng.integers(0, 60 * (rnd + 1)))):
                top[c] += 1 if rng.random() < 0.9 or c < 2 else 3  # columns 0, 1 never gap: they fold
                els[(c, top[c])] = int(rng.integers(1, 1 << 40))
                cl.add((c, top[c]))
        batches.append(_table(ids, [(b"hot", els, {}, cl), (b"cold", {(0, rnd + 1): 9}, {}, {(0, rnd + 1)})]))
    eng = _engine(R=R, long_min=4)
    try:
        st = _run(O, eng, batches)
        assert st["inplace_docs"] >= 10 and st["inplace_folded"] > 0 and st["demoted"] == 0
    finally:
        eng.close()


def test_inplace_demotions(oracle_mod):
    """deltas that are not append-shaped for a long document: a context dot
    removing a live element near the run's start (trimmed in place) or deep
    in it (demoted), a vv entry covering the run's first elements (trimmed,
    except those the delta re-sends), a vv entry above the state's, an unseen
    dot below the column's top (demoted), a re-sent element (covered: stays in
    place)"""
    from jylis_amd import synth as S
    O = oracle_mod
    R = 4
    ids = S.replica_ids(R, 23)
    base = {(c, q): 1000 * c + q for c in range(R) for q in range(1, 41)}
    vv = {c: 40 for c in range(R)}
    b0 = _table(ids, [(b"d", base, vv, set())])
    # covered re-send (in place) + fresh appends
    b1 = _table(ids, [(b"d", {(1, 5): 1005, (2, 41): 7}, {}, {(1, 5), (2, 41)})])
    # observed remove of live (0, 7): demote
    b2 = _table(ids, [(b"d", {}, {}, {(0, 7)})])
    # vv entry above the state's column 3: demote (removes (3, 41..44) absent ones, raises vv)
    b3 = _table(ids, [(b"d", {(1, 60): 3}, {3: 44}, {(1, 60)})])
    # a dot below the column's top the state never saw (a gap filled late): demote
    b4 = _table(ids, [(b"d", {(1, 50): 4}, {}, {(1, 50)})])
    # RM of an element the delta keeps (context dot + the element itself): in place
    b5 = _table(ids, [(b"d", {(2, 10): 2010, (2, 99): 5}, {}, {(2, 10), (2, 99)})])
    # a deep document: a removal past the trim span demotes it, one near the
    # start and a vv entry covering a prefix (one of its elements re-sent) trim
    deep = {(0, q): 7 * q for q in range(1, 401)}
    b6 = _table(ids, [(b"deep", deep, {0: 400}, set())])
    b7 = _table(ids, [(b"deep", {(0, 401): 1}, {}, {(0, 350), (0, 401)})])
    b8 = _table(ids, [(b"deep", {(0, 5): 35, (0, 402): 2}, {0: 12}, {(0, 3), (0, 402)})])
    eng = _engine(R=R, long_min=8)
    try:
        st = _run(O, eng, [b0, b1, b2, b3, b4, b5, b1, b5, b6, b7, b8])
        assert st["demoted"] >= 3 and st["inplace_docs"] >= 4
    finally:
        eng.close()


def test_inplace_repeated_and_malformed(oracle_mod):
    """a long document named twice in one DEVICE batch (both copies skipped:
    one would append, the other demote), the same batch from host memory
    (applied as ordered rounds, as the reference's per-pair loop would), and
    a malformed delta of a long document (skipped); the document still
    converges in place afterwards"""
    from jylis_amd import synth as S
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    R = 4
    ids = S.replica_ids(R, 29)
    base = {(c, q): 10 * q + c for c in range(R) for q in range(1, 21)}
    b0 = _table(ids, [(b"L", base, {c: 20 for c in range(R)}, set())])
    dup = _table(ids, [(b"L", {(0, 21): 1}, {}, {(0, 21)}), (b"L", {}, {}, {(1, 3)})])
    eng = _engine(R=R, long_min=4)
    try:
        want = O.Repo(O.UJSON, 1)
        got = RepoUJSON(eng)
        want.converge(b0)
        got.converge_deltas(b0)
        before = got.state()
        import torch
        dev = torch.device("cuda", 0)
        eng.ujson_converge(*[_dev(a, dev) for a in _dev_args(eng, dup)])
        assert eng.skipped() >= 1
        assert_state_equal(O.UJSON, before, got.state())
        dup2 = _table(ids, [(b"L", {(0, 21): 1}, {}, {(0, 21)}), (b"L", {}, {3: 20}, {(0, 7)})])
        eng.ujson_converge(*_dev_args(eng, dup2))  # host: rounds in order
        for part in ([(b"L", {(0, 21): 1}, {}, {(0, 21)})], [(b"L", {}, {3: 20}, {(0, 7)})]):
            want.converge(_table(ids, part))
        assert_state_equal(O.UJSON, want.state(), got.state())
        before = got.state()
        # malformed: dots not ascending
        from jylis_amd.engine import pack_dot
        slots = eng.lookup(4, [b"L"])
        bad = (slots, np.array([0, 2], np.uint64), np.concatenate([pack_dot([0], [30]), pack_dot([0], [25])]),
               np.array([1, 2], np.uint64), np.zeros(2, np.uint64), np.zeros(0, np.uint64),
               np.array([0, 1], np.uint64), pack_dot([0], [30]))
        eng.ujson_converge(*bad)
        assert_state_equal(O.UJSON, before, got.state())
        b1 = _table(ids, [(b"L", {(2, 21): 5, (3, 22): 6}, {}, {(2, 21), (3, 22)})])
        want.converge(b1)
        got.converge_deltas(b1)
        assert_state_equal(O.UJSON, want.state(), got.state())
        assert eng.ujson_stats()["inplace_docs"] >= 1
    finally:
        eng.close()


def _dev(a, dev):
    import torch
    a = np.ascontiguousarray(a)
    a = a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32) if a.dtype == np.uint32 else a
    return torch.from_numpy(a).to(dev)


def _dev_args(eng, t):
    from jylis_amd.repo import RepoUJSON
    r = RepoUJSON(eng)
    slots = eng.intern(4, (t["key_bytes"], t["key_offs"]))
    eo, vo, co = (np.asarray(t[k], np.uint64) for k in ("el_offs", "vv_offs", "cloud_offs"))
    dots, elems = r._sort_segments(eo, r._pack(t["dot_ids"], t["dot_seqs"]), np.asarray(t["elems"]))
    (vv,) = r._sort_segments(vo, r._pack(t["vv_ids"], t["vv_seqs"]))
    (cloud,) = r._sort_segments(co, r._pack(t["cloud_ids"], t["cloud_seqs"]))
    return slots, eo, dots, elems, vo, vv, co, cloud


def test_inplace_compaction(oracle_mod):
    """small pools: compactions lay every long document out regular again
    (the long pools empty) and the documents are promoted anew"""
    from jylis_amd import synth as S
    O = oracle_mod
    eng = _engine(R=8, long_min=2, entry_capacity=1024)
    try:
        st0, dl = S.ujson_tables(1500, seed=S.BASE_SEED + 62, rounds=7, R=8)
        st = _run(O, eng, [st0] + dl)
        assert st["promoted"] > 0
    finally:
        eng.close()


@pytest.mark.parametrize("seed", [1, 2])
def test_inplace_write_path(oracle_mod, seed):
    """local INS / RM / CLR on long documents (the write kernels walk the
    column runs) interleaved with peer batches; every flush and the state"""
    from test_ujson_write_gpu import IDENT, _apply_oracle, _canon_ujson
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    rng = np.random.default_rng(900 + seed)
    eng = _engine(R=16, long_min=2)
    try:
        want = O.Repo(O.UJSON, IDENT)
        got = RepoUJSON(eng)
        peers = random_history(O, O.UJSON, seed + 10, nops=150)
        keys = [f"doc{i}" for i in range(6)]
        for step in range(14):
            cmds = []
            for _ in range(int(rng.integers(1, 40))):
                k = keys[int(rng.integers(0, len(keys)))]
                x = rng.random()
                cmds.append(("INS", k, int(rng.integers(1, 9))) if x < 0.7 else
                            ("RM", k, int(rng.integers(1, 9))) if x < 0.95 else ("CLR", k))
            for c in cmds:
                _apply_oracle(want, c)
            got.write(cmds, IDENT)
            for b in peers[step * 3:step * 3 + 3]:
                want.converge(b)
                got.converge_deltas(b)
            assert_state_equal(O.UJSON, want.state(), got.state())
            if rng.random() < 0.5:
                assert _canon_ujson(got.flush_deltas()) == _canon_ujson(want.flush().table())
        assert _canon_ujson(got.flush_deltas()) == _canon_ujson(want.flush().table())
        assert eng.ujson_stats()["promoted"] > 0
    finally:
        eng.close()


def test_inplace_pipelined_deterministic():
    """a Zipf sequence with hot long documents converged back to back (no
    read in between) twice on fresh engines: identical stores"""
    from jylis_amd import synth as S
    from jylis_amd.repo import RepoUJSON

    def run():
        eng = _engine(R=16, long_min=16)
        try:
            st0, dl = S.ujson_tables(20000, seed=S.BASE_SEED + 63, rounds=6, R=16)
            repo = RepoUJSON(eng)
            for b in [st0] + dl:
                repo.converge_deltas(b)
            s = repo.state()
            h = hashlib.sha256()
            for k in sorted(s):
                h.update(k.encode())
                h.update(np.ascontiguousarray(s[k]).tobytes())
            return h.hexdigest(), eng.ujson_stats()
        finally:
            eng.close()
    a, sa = run()
    b, sb = run()
    assert a == b
    assert sa["inplace_docs"] > 0
