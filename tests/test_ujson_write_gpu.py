"""UJSON write path on the GPU (jy_ujson_write / _deltas_size / _flush) on
opaque element handles, against the CPU oracle, bit-exact.

The reference's local writes (repo_ujson.pony:74-110): INS adds an element
under a fresh dot of this replica (creating the key), RM removes every
element equal to the value (observed remove), CLR removes every element; RM
and CLR of a missing key do nothing.  The pending delta records the fresh
dot's element and the removed dots (context only: an element the pending
delta already holds stays, oracle UJSON::remove / clear).  flush_deltas
(repo_ujson.pony:22-26) emits and clears them.  Streams repeat docs inside a
batch (applied in order), hit RM on elements inserted earlier in the same
batch, and interleave peer batches (other replicas' concurrent inserts
survive an RM: add wins)."""
import numpy as np
import pytest

from helpers import assert_state_equal, random_history

pytestmark = pytest.mark.gpu

IDENT = 0x5EED_0000_0000_0533


def _canon_ujson(t):
    """batch table -> {key: (sorted (id, seq, elem), sorted vv (id, n), sorted cloud (id, seq))}"""
    ko = np.asarray(t["key_offs"], np.uint64)
    kb = np.asarray(t["key_bytes"], np.uint8)
    out = {}
    for i in range(len(ko) - 1):
        k = bytes(kb[int(ko[i]):int(ko[i + 1])])

        def seg(name, cols):
            o = np.asarray(t[name], np.uint64)
            a, b = int(o[i]), int(o[i + 1])
            return sorted(zip(*[np.asarray(t[c], np.uint64)[a:b].tolist() for c in cols]))
        out[k] = (seg("el_offs", ("dot_ids", "dot_seqs", "elems")), seg("vv_offs", ("vv_ids", "vv_seqs")),
                  seg("cloud_offs", ("cloud_ids", "cloud_seqs")))
    return out


def _apply_oracle(want, c):
    if c[0] == "INS":
        want.ujson_ins(c[1], c[2])
    elif c[0] == "RM":
        want.ujson_rm(c[1], c[2])
    else:
        want.ujson_clr(c[1])


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_ujson_write_flush_parity(oracle_mod, engine, seed):
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    rng = np.random.default_rng(400 + seed)
    want = O.Repo(O.UJSON, IDENT)
    got = RepoUJSON(engine)
    peers = random_history(O, O.UJSON, seed, nops=150)
    keys = [f"doc{i}" for i in range(10)]
    for step in range(16):
        cmds = []
        for _ in range(int(rng.integers(1, 30))):
            k = keys[int(rng.integers(0, len(keys)))]
            x = rng.random()
            if x < 0.6:
                cmds.append(("INS", k, int(rng.integers(1, 8))))
            elif x < 0.9:
                cmds.append(("RM", k, int(rng.integers(1, 8))))
            else:
                cmds.append(("CLR", k))
        for c in cmds:
            _apply_oracle(want, c)
        got.write(cmds, IDENT)
        for b in peers[step * 3:step * 3 + 3]:
            want.converge(b)
            got.converge_deltas(b)
        assert got.deltas_size() == want.deltas_size()
        if rng.random() < 0.5:
            assert _canon_ujson(got.flush_deltas()) == _canon_ujson(want.flush().table())
            assert got.deltas_size() == 0
    assert _canon_ujson(got.flush_deltas()) == _canon_ujson(want.flush().table())
    assert_state_equal(O.UJSON, want.state(), got.state())


def test_ujson_write_edges(oracle_mod, engine):
    """RM / CLR of a missing key (no key, no delta), RM of an absent value
    (delta key only), INS then RM then INS of one value in one batch, CLR
    then INS, the same value inserted twice (two dots)"""
    from jylis_amd.repo import RepoUJSON
    O = oracle_mod
    want = O.Repo(O.UJSON, IDENT)
    got = RepoUJSON(engine)
    cmds = [("RM", "missing", 3), ("CLR", "missing2"), ("INS", "a", 5), ("RM", "a", 9), ("INS", "b", 1),
            ("RM", "b", 1), ("INS", "b", 1), ("INS", "c", 2), ("CLR", "c"), ("INS", "c", 4), ("INS", "d", 7),
            ("INS", "d", 7)]
    for c in cmds:
        _apply_oracle(want, c)
    got.write(cmds, IDENT)
    assert got.deltas_size() == want.deltas_size() == 4
    from jylis_amd import engine as E
    assert got.slots_of(["missing"])[0] == E._lib.JY_NO_SLOT
    assert _canon_ujson(got.flush_deltas()) == _canon_ujson(want.flush().table())
    assert_state_equal(O.UJSON, want.state(), got.state())
