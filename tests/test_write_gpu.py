"""Counter write path on the GPU (jy_counter_write / _deltas_size / _flush)
against the CPU oracle, bit-exact.

The reference's local writes: RepoGCOUNT.inc (repo_gcount.pony:57-60) and
RepoPNCOUNT.inc/dec (repo_pncount.pony:59-67) add to this replica's entry
(wrapping) and record the post-write total in the key's pending delta;
flush_deltas (repo_gcount.pony:18-23) emits and clears those deltas.  The
streams interleave write batches (keys repeating inside a batch, values near
2^64 so the own entry wraps, negative i64 bit-cast for PNCOUNT) with peer
batches and echoes of this replica's own older state (max-merge over a
wrapped own entry), and flush at random points."""
import numpy as np
import pytest

from helpers import assert_state_equal, random_history

pytestmark = pytest.mark.gpu

IDENT = 0x5EED_0000_ABCD_1234


def _canon(ctype, t):
    """batch table -> {key: per-sign sorted (id, value) pairs}"""
    pres = ("",) if ctype == 0 else ("p_", "n_")
    ko = np.asarray(t["key_offs"], np.uint64)
    kb = np.asarray(t["key_bytes"], np.uint8)
    out = {}
    for i in range(len(ko) - 1):
        k = bytes(kb[int(ko[i]):int(ko[i + 1])])
        row = []
        for p in pres:
            o = np.asarray(t[p + "offs"], np.uint64)
            a, b = int(o[i]), int(o[i + 1])
            row.append(sorted(zip(np.asarray(t[p + "ids"], np.uint64)[a:b].tolist(),
                                  np.asarray(t[p + "vals"], np.uint64)[a:b].tolist())))
        out[k] = row
    return out


def _vals(rng, n):
    v = rng.integers(0, 1 << 62, n, dtype=np.uint64)
    big = rng.random(n) < 0.3  # near 2^64: the own entry wraps
    v[big] = np.uint64(2**64 - 1) - rng.integers(0, 1 << 20, int(big.sum()), dtype=np.uint64)
    return v


@pytest.mark.parametrize("ctype", [0, 1])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_writes_flush_parity(oracle_mod, engine, ctype, seed):
    from jylis_amd.repo import REPOS
    O = oracle_mod
    rng = np.random.default_rng(100 + seed)
    want = O.Repo(ctype, IDENT)
    got = REPOS[ctype](engine)
    peers = random_history(O, ctype, seed, nops=150)
    keys = [f"k{i}" for i in range(18)]
    echoes = []
    flushed = 0
    for step in range(16):
        n = int(rng.integers(1, 48))
        ks = [keys[i] for i in rng.integers(0, len(keys), n)]
        v = _vals(rng, n)
        if ctype == 0:
            for k, x in zip(ks, v):
                want.gcount_inc(k, int(x))
            got.inc(ks, v, IDENT)
        else:
            dec = rng.random(n) < 0.5
            for k, x, d in zip(ks, v, dec):
                (want.pncount_dec if d else want.pncount_inc)(k, int(np.int64(x.view(np.int64))))
            ik = [k for k, d in zip(ks, dec) if not d]
            dk = [k for k, d in zip(ks, dec) if d]
            if ik:
                got.inc(ik, v[~dec].view(np.int64), IDENT)
            if dk:
                got.dec(dk, v[dec].view(np.int64), IDENT)
        if rng.random() < 0.4:
            echoes.append(want.state())
        for b in peers[step * 3:step * 3 + 3]:
            want.converge(b)
            got.converge_deltas(b)
        if echoes and rng.random() < 0.3:
            e = echoes.pop(0)  # this replica's own older totals coming back
            want.converge(e)
            got.converge_deltas(e)
        assert got.deltas_size() == want.deltas_size()
        if rng.random() < 0.5:
            w = _canon(ctype, want.flush().table())
            g = _canon(ctype, got.flush_deltas(IDENT))
            assert g == w
            flushed += 1
            assert got.deltas_size() == 0
    w = _canon(ctype, want.flush().table())
    g = _canon(ctype, got.flush_deltas(IDENT))
    assert g == w
    assert flushed > 0
    assert_state_equal(ctype, want.state(), got.state())
    exp = [(want.gcount_get if ctype == 0 else want.pncount_get)(k) for k in keys]
    dt = np.int64 if ctype else np.uint64
    np.testing.assert_array_equal(got.get(keys).astype(dt), np.array(exp, dtype=dt))


def test_flushed_delta_converges_on_a_peer(oracle_mod, engine):
    """a GPU replica's flushed delta folds into an oracle peer: test_cluster
    shape (2 + 3 + 4 -> 9) with the GPU node as one of the writers"""
    from jylis_amd.repo import RepoGCOUNT
    O = oracle_mod
    gpu = RepoGCOUNT(engine)
    gpu.inc(["foo"], [2], IDENT)
    others = [O.Repo(O.GCOUNT, i + 7) for i in range(2)]
    for r, v in zip(others, (3, 4)):
        r.gcount_inc("foo", v)
    peer = O.Repo(O.GCOUNT, 99)
    peer.converge(gpu.flush_deltas(IDENT))
    for r in others:
        b = r.flush().table()
        peer.converge(b)
        gpu.converge_deltas(b)
    assert peer.gcount_get("foo") == 9
    assert int(gpu.get(["foo"])[0]) == 9
    assert gpu.deltas_size() == 0


def test_write_errors(engine):
    from jylis_amd.engine import EngineError
    from jylis_amd.repo import RepoGCOUNT, RepoPNCOUNT
    g = RepoGCOUNT(engine)
    g.inc(["a"], [1], IDENT)
    with pytest.raises(EngineError):  # another column while deltas are pending
        g.inc(["a"], [1], IDENT + 1)
    slot = engine.lookup(0, ["a"])
    with pytest.raises(EngineError):  # DEC on a GCOUNT
        engine.counter_write(0, 1, engine.replica_col(IDENT), slot, [1])
    with pytest.raises(EngineError):  # a slot that was never interned
        engine.counter_write(1, 0, engine.replica_col(IDENT), np.array([5], np.uint32), [1])
    p = RepoPNCOUNT(engine)
    p.dec(["a"], [-3], IDENT)
    assert int(p.get(["a"])[0]) == 3
    assert g.flush_deltas(IDENT)["vals"].tolist() == [1]


def _canon_treg(t):
    ko = np.asarray(t["key_offs"], np.uint64)
    kb = np.asarray(t["key_bytes"], np.uint8)
    vo = np.asarray(t["val_offs"], np.uint64)
    vb = np.asarray(t["val_bytes"], np.uint8)
    return {bytes(kb[int(ko[i]):int(ko[i + 1])]): (int(t["ts"][i]), bytes(vb[int(vo[i]):int(vo[i + 1])]))
            for i in range(len(ko) - 1)}


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_treg_set_flush_parity(oracle_mod, engine, seed):
    """RepoTREG.set batches (repeated keys, dense timestamp ties, shared
    8-byte prefixes, losing SETs that still create the delta key) interleaved
    with peer batches; flushes compared with the oracle's flush_deltas"""
    from jylis_amd.repo import RepoTREG
    O = oracle_mod
    rng = np.random.default_rng(200 + seed)
    want = O.Repo(O.TREG, IDENT)
    got = RepoTREG(engine)
    peers = random_history(O, O.TREG, seed, nops=150)
    keys = [f"r{i}" for i in range(14)]
    alphabet = np.frombuffer(b"aab\x00\xff", np.uint8)
    for step in range(16):
        n = int(rng.integers(1, 40))
        ks = [keys[i] for i in rng.integers(0, len(keys), n)]
        vals = [b"prefix__" * int(rng.integers(0, 2)) + bytes(rng.choice(alphabet, int(rng.integers(0, 6))))
                for _ in range(n)]
        ts = rng.integers(0, 8, n).astype(np.uint64)
        for k, v, t in zip(ks, vals, ts):
            want.treg_set(k, v, int(t))
        got.set(ks, vals, ts)
        for b in peers[step * 3:step * 3 + 3]:
            want.converge(b)
            got.converge_deltas(b)
        assert got.deltas_size() == want.deltas_size()
        if rng.random() < 0.5:
            assert _canon_treg(got.flush_deltas()) == _canon_treg(want.flush().table())
            assert got.deltas_size() == 0
    assert _canon_treg(got.flush_deltas()) == _canon_treg(want.flush().table())
    assert_state_equal(O.TREG, want.state(), got.state())
