"""Value-arena reclamation (jy_arena_collect) for TREG and TLOG: registers and
logs whose long values are replaced many times, pending deltas holding long
values across a collection, then parity with the oracle (state and flushed
deltas) and a smaller arena afterwards."""
import numpy as np
import pytest

from helpers import assert_state_equal

pytestmark = pytest.mark.gpu

IDENT = 0x5EED_0000_0000_A7E0


def _long(rng, tag):
    return (b"long-value-%d-" % tag) + bytes(rng.integers(97, 123, int(rng.integers(0, 30))).astype(np.uint8))


def test_treg_collect(oracle_mod, engine):
    from jylis_amd import _lib
    from jylis_amd.repo import RepoTREG
    from test_write_gpu import _canon_treg
    O = oracle_mod
    rng = np.random.default_rng(7)
    want = O.Repo(O.TREG, IDENT)
    got = RepoTREG(engine)
    got._arena_live = 1 << 40  # no automatic collection: this test calls it
    keys = [f"r{i}" for i in range(300)]
    for step in range(12):
        n = 400
        ks = [keys[i] for i in rng.integers(0, len(keys), n)]
        vals = [_long(rng, step) for _ in range(n)]
        ts = rng.integers(0, 50, n).astype(np.uint64) + np.uint64(step * 10)
        kb = [k.encode() for k in ks]
        # a peer batch (converge) and local SETs (pending deltas)
        from jylis_amd.engine import encode_keys
        kbb, ko = encode_keys(kb[: n // 2])
        vb, vo = encode_keys(vals[: n // 2])
        batch = {"key_bytes": kbb, "key_offs": ko, "ts": ts[: n // 2], "val_bytes": vb, "val_offs": vo}
        want.converge(batch)
        got.converge_deltas(batch)
        for k, v, t in zip(ks[n // 2:], vals[n // 2:], ts[n // 2:]):
            want.treg_set(k, v, int(t))
        got.set(ks[n // 2:], vals[n // 2:], ts[n // 2:])
        if step in (4, 9):
            before, _ = engine.arena_usage(_lib.TREG)
            live = engine.arena_collect(_lib.TREG)
            after, _ = engine.arena_usage(_lib.TREG)
            assert after == live < before
        if step == 6:
            assert _canon_treg(got.flush_deltas()) == _canon_treg(want.flush().table())
    assert _canon_treg(got.flush_deltas()) == _canon_treg(want.flush().table())
    assert_state_equal(O.TREG, want.state(), got.state())


def test_tlog_collect(oracle_mod, engine):
    from jylis_amd import _lib
    from jylis_amd.repo import RepoTLOG
    from test_tlog_write_gpu import _canon_tlog
    O = oracle_mod
    rng = np.random.default_rng(8)
    want = O.Repo(O.TLOG, IDENT)
    got = RepoTLOG(engine)
    got._arena_live = 1 << 40
    keys = [f"l{i}" for i in range(40)]
    for step in range(10):
        cmds = []
        for _ in range(200):
            k = keys[int(rng.integers(0, len(keys)))]
            if rng.random() < 0.85:
                cmds.append(("INS", k, _long(rng, step), int(rng.integers(0, 20)) + step * 15))
            else:
                cmds.append(("TRIMAT", k, step * 15 + int(rng.integers(0, 10))))
        for c in cmds:
            if c[0] == "INS":
                want.tlog_ins(c[1], c[2], c[3])
            else:
                want.tlog_trimat(c[1], c[2])
        got.write(cmds)
        if step in (3, 7):
            before, _ = engine.arena_usage(_lib.TLOG)
            live = engine.arena_collect(_lib.TLOG)
            assert live < before
        if step == 5:
            assert _canon_tlog(got.flush_deltas()) == _canon_tlog(want.flush().table())
    assert _canon_tlog(got.flush_deltas()) == _canon_tlog(want.flush().table())
    assert_state_equal(O.TLOG, want.state(), got.state())
