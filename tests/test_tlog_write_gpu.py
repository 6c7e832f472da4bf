"""TLOG write path on the GPU (jy_tlog_write / _deltas_size / _flush) against
the CPU oracle, bit-exact.

The reference's local writes (repo_tlog.pony:85-111): INS writes the entry
(ignored below the cutoff or as a duplicate), TRIMAT raises the cutoff, TRIM
n raises it to the n-th newest entry's timestamp (n == 0 clears; past the end
does nothing), CLR raises it past the newest entry (U64 wraps).  Where the
state changed, the same change lands in the key's pending delta; every
command creates the delta key.  flush_deltas (repo_tlog.pony:21-25) emits and
clears them.  The streams repeat keys inside a batch (applied in order), tie
timestamps, share 8-byte value prefixes, put long values in the arena, and
interleave peer batches."""
import numpy as np
import pytest

from helpers import assert_state_equal, random_history

pytestmark = pytest.mark.gpu

IDENT = 0x5EED_0000_0000_7106


def _canon_tlog(t):
    """batch table -> {key: (cutoff, [(value, ts) newest first])}"""
    ko = np.asarray(t["key_offs"], np.uint64)
    kb = np.asarray(t["key_bytes"], np.uint8)
    eo = np.asarray(t["ent_offs"], np.uint64)
    vo = np.asarray(t["val_offs"], np.uint64)
    vb = np.asarray(t["val_bytes"], np.uint8)
    ts = np.asarray(t["ts"], np.uint64)
    cut = np.asarray(t["cutoff"], np.uint64)
    out = {}
    for i in range(len(ko) - 1):
        k = bytes(kb[int(ko[i]):int(ko[i + 1])])
        ents = [(bytes(vb[int(vo[j]):int(vo[j + 1])]), int(ts[j])) for j in range(int(eo[i]), int(eo[i + 1]))]
        out[k] = (int(cut[i]), ents)
    return out


def _apply_oracle(want, cmd):
    op = cmd[0]
    if op == "INS":
        want.tlog_ins(cmd[1], cmd[2], cmd[3])
    elif op == "TRIMAT":
        want.tlog_trimat(cmd[1], cmd[2])
    elif op == "TRIM":
        want.tlog_trim(cmd[1], cmd[2])
    else:
        want.tlog_clr(cmd[1])


def _random_cmds(rng, keys, n):
    alphabet = np.frombuffer(b"ab\x00\xff", np.uint8)
    cmds = []
    for _ in range(n):
        k = keys[int(rng.integers(0, len(keys)))]
        r = rng.random()
        if r < 0.6:
            v = b"sharedp_" * int(rng.integers(0, 3)) + bytes(rng.choice(alphabet, int(rng.integers(0, 5))))
            ts = int(rng.integers(0, 12)) if rng.random() < 0.95 else (1 << 64) - 1
            cmds.append(("INS", k, v, ts))
        elif r < 0.75:
            cmds.append(("TRIMAT", k, int(rng.integers(0, 14))))
        elif r < 0.9:
            cmds.append(("TRIM", k, int(rng.integers(0, 7))))
        else:
            cmds.append(("CLR", k))
    return cmds


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_tlog_write_flush_parity(oracle_mod, engine, seed):
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    rng = np.random.default_rng(300 + seed)
    want = O.Repo(O.TLOG, IDENT)
    got = RepoTLOG(engine)
    peers = random_history(O, O.TLOG, seed, nops=120)
    keys = [f"log{i}" for i in range(12)]
    for step in range(16):
        cmds = _random_cmds(rng, keys, int(rng.integers(1, 40)))
        for c in cmds:
            _apply_oracle(want, c)
        got.write(cmds)
        for b in peers[step * 3:step * 3 + 3]:
            want.converge(b)
            got.converge_deltas(b)
        assert got.deltas_size() == want.deltas_size()
        if rng.random() < 0.5:
            assert _canon_tlog(got.flush_deltas()) == _canon_tlog(want.flush().table())
            assert got.deltas_size() == 0
    assert _canon_tlog(got.flush_deltas()) == _canon_tlog(want.flush().table())
    assert_state_equal(O.TLOG, want.state(), got.state())


def test_tlog_write_edges(oracle_mod, engine):
    """CLR of an empty log (no change, key still pending), CLR at the largest
    timestamp (cutoff wraps to 0: no raise), TRIM past the end, TRIM 0, an
    INS below the cutoff, a duplicate INS, TRIMAT that does not raise"""
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    want = O.Repo(O.TLOG, IDENT)
    got = RepoTLOG(engine)
    cmds = [("CLR", "e"), ("INS", "w", b"x", (1 << 64) - 1), ("CLR", "w"), ("INS", "t", b"a", 5),
            ("INS", "t", b"b", 7), ("TRIM", "t", 9), ("INS", "t", b"a", 5), ("TRIMAT", "t", 6),
            ("INS", "t", b"c", 5), ("TRIMAT", "t", 3), ("TRIM", "t", 0), ("INS", "z", b"long value " * 3, 4),
            ("TRIM", "z", 1)]
    for c in cmds:
        _apply_oracle(want, c)
    got.write(cmds)
    assert got.deltas_size() == want.deltas_size() == 4
    assert _canon_tlog(got.flush_deltas()) == _canon_tlog(want.flush().table())
    assert_state_equal(O.TLOG, want.state(), got.state())
