"""TREG: the HIP LWW select against the CPU oracle (bit-exact).

Edge cases: timestamp ties broken by Pony String order (bytewise unsigned,
then shorter-is-less), values sharing 8-byte prefixes, embedded NULs and
0xFF bytes, empty values, keys created by converge but never set (GET shows
("", 0), not nil: repo_treg.pony:52,55-61)."""
import numpy as np
import pytest

from helpers import assert_state_equal, random_history

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_history_parity(oracle_mod, engine, seed):
    from jylis_amd.repo import RepoTREG
    O = oracle_mod
    want = O.Repo(O.TREG)
    got = RepoTREG(engine)
    for b in random_history(O, O.TREG, seed, val_len=20):
        want.converge(b)
        got.converge_deltas(b)
    assert_state_equal(O.TREG, want.state(), got.state())


def _batch(keys, vals, ts):
    from jylis_amd.engine import encode_keys
    kb, ko = encode_keys(keys)
    vb, vo = encode_keys(vals)
    return {"key_bytes": kb, "key_offs": ko, "ts": np.array(ts, np.uint64), "val_bytes": vb, "val_offs": vo}


TIES = [  # (state, delta) at equal timestamps
    (b"", b"a"), (b"a", b""), (b"abc", b"abd"), (b"abcdefgh", b"abcdefgh\x00"),
    (b"abcdefghij", b"abcdefghik"), (b"abcdefghijk", b"abcdefghij"), (b"\xff", b"\x00\x00"),
    (b"same-long-value!", b"same-long-value!"), (b"a\x00", b"a"), (b"zzzzzzzzzzzzzzzzzzzz1", b"zzzzzzzzzzzzzzzzzzzz2"),
]


def test_tie_break_order(oracle_mod, engine):
    from jylis_amd.repo import RepoTREG
    O = oracle_mod
    want = O.Repo(O.TREG)
    got = RepoTREG(engine)
    keys = [f"t{i}" for i in range(len(TIES))]
    s = _batch(keys, [a for a, _ in TIES], [7] * len(TIES))
    d = _batch(keys, [b for _, b in TIES], [7] * len(TIES))
    for b in (s, d):
        want.converge(b)
        got.converge_deltas(b)
    assert_state_equal(O.TREG, want.state(), got.state())
    for k, (a, b) in zip(keys, TIES):
        assert got.get(k) == (max(a, b), 7)  # python bytes order == Pony String order


def test_existence_and_nil(oracle_mod, engine):
    from jylis_amd.repo import RepoTREG
    got = RepoTREG(engine)
    got.converge_deltas(_batch(["e"], [b""], [0]))  # ("", 0) delta still creates the key
    assert got.get("e") == (b"", 0)
    assert got.get("never") is None


def test_repeated_key_in_one_batch(oracle_mod, engine):
    """several deltas for one key in one call are split into rounds (exact LWW join)"""
    from jylis_amd.repo import RepoTREG
    O = oracle_mod
    want = O.Repo(O.TREG)
    got = RepoTREG(engine)
    b = _batch(["k", "k", "j", "k"], [b"x", b"zz", b"q", b"y"], [3, 3, 1, 2])
    want.converge(b)
    got.converge_deltas(b)
    assert_state_equal(O.TREG, want.state(), got.state())
    assert got.get("k") == (b"zz", 3)


def test_large_random(oracle_mod, engine):
    """50k keys, dense timestamp ties, ~20% shared 8-byte prefixes"""
    from jylis_amd.repo import RepoTREG
    O = oracle_mod
    rng = np.random.default_rng(5)
    n = 50000
    keys = [f"r{i}" for i in range(n)]
    prefixes = [bytes(rng.integers(0, 256, 8).astype(np.uint8)) for _ in range(16)]

    def vals():
        out = []
        for _ in range(n):
            L = int(rng.integers(1, 17))
            if rng.random() < 0.2:
                out.append((prefixes[rng.integers(16)] + bytes(rng.integers(0, 256, 8).astype(np.uint8)))[:max(L, 9)])
            else:
                out.append(bytes(rng.integers(0, 256, L).astype(np.uint8)))
        return out

    want = O.Repo(O.TREG)
    got = RepoTREG(engine)
    for _ in range(3):
        b = _batch(keys, vals(), rng.integers(0, 4, n))
        want.converge(b)
        got.converge_deltas(b)
    assert_state_equal(O.TREG, want.state(), got.state())


@pytest.mark.parametrize("dup_rounds", [(), (5,), (2, 9)])
def test_many_merges_between_reads(engine, dup_rounds):
    """Device batches merged back to back with no read in between: the
    duplicate list's bound passes its capacity every few launches.  With no
    duplicate pushed since the last fold the engine waits for launches in
    flight instead of folding an empty list; batches listed in `dup_rounds`
    repeat slots (in-launch duplicates), which must still be folded exactly.
    Checked against a numpy LWW over every applied batch (8-byte values:
    the (ts, value) order is (ts, prefix))."""
    import torch
    from jylis_amd._lib import TREG
    rng = np.random.default_rng(17 + len(dup_rounds))
    n = 200_000
    slots = engine.intern(TREG, [b"m%07d" % i for i in range(n)])
    assert (slots == np.arange(n)).all()
    best_ts = np.zeros(n, np.uint64)
    best_pre = np.zeros(n, np.uint64)
    dev = torch.device("cuda", 0)
    for r in range(14):
        s = np.arange(n, dtype=np.uint32)
        if r in dup_rounds:
            s = rng.integers(0, n, n).astype(np.uint32)  # repeats inside the launch
        ts = rng.integers(1, 1 << 12, n).astype(np.uint64) + np.uint64(r << 10)
        pre = rng.integers(1 << 56, 1 << 63, n, dtype=np.uint64)  # 8 nonzero-leading bytes
        lr = np.full(n, 8, np.uint64)
        engine.treg_converge(*(torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to(dev)
                               for a in (s, ts, pre, lr)))
        order = np.lexsort((pre, ts))
        cand_ts, cand_pre = best_ts[s[order]], best_pre[s[order]]
        win = (ts[order] > cand_ts) | ((ts[order] == cand_ts) & (pre[order] > cand_pre))
        # apply in ascending order so the last assignment per slot is the maximum
        so, to, po = s[order][win], ts[order][win], pre[order][win]
        best_ts[so] = to
        best_pre[so] = po
    gts, gpre, glr = engine.treg_read(np.arange(n, dtype=np.uint32))
    np.testing.assert_array_equal(gts, best_ts)
    np.testing.assert_array_equal(gpre, best_pre)


def test_duplicate_list_overflow_fails_loudly():
    """A device batch that repeats slots more often than the duplicate list
    holds (a test-only 64-record list the host never folds ahead of time,
    JY_CFG_TREG_DUP_TEST): the records past the capacity are dropped, the
    next call fails with JY_ERANGE, and no memory outside the list is
    touched -- every slot the batch does not name reads as before."""
    import torch
    from jylis_amd._lib import CFG_TREG_DUP_TEST, JY_ERANGE, TREG
    from jylis_amd.engine import Engine, EngineError
    eng = Engine(device=0, flags=CFG_TREG_DUP_TEST)
    try:
        n = 4096
        slots = eng.intern(TREG, [b"o%05d" % i for i in range(n)])
        assert (slots == np.arange(n)).all()
        rng = np.random.default_rng(3)
        ts0 = rng.integers(1, 1 << 20, n).astype(np.uint64)
        pre0 = rng.integers(1, 1 << 63, n, dtype=np.uint64)
        lr0 = np.full(n, 8, np.uint64)
        eng.treg_converge(np.arange(n, dtype=np.uint32), ts0, pre0, lr0)
        before = eng.treg_read(np.arange(n, dtype=np.uint32))
        # 1,000 entries on 8 slots: 992 duplicates, past the 64-record list
        m = 1000
        s = (np.arange(m) % 8).astype(np.uint32)
        ts = np.full(m, 1 << 40, np.uint64) + np.arange(m, dtype=np.uint64)
        pre = rng.integers(1, 1 << 63, m, dtype=np.uint64)
        lr = np.full(m, 8, np.uint64)
        dev = torch.device("cuda", 0)
        args = [torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to(dev)
                for a in (s, ts, pre, lr)]
        eng.treg_converge(*args)
        torch.cuda.synchronize()
        # the read fails loudly; its outputs are still written: every slot
        # outside the batch is bit-identical to before
        out = [np.zeros(n, np.uint64) for _ in range(3)]
        idx = np.arange(n, dtype=np.uint32)
        rc = eng.lib.jy_treg_read(eng.h, n, idx.ctypes.data, *(o.ctypes.data for o in out))
        assert rc == JY_ERANGE, rc
        for o, b in zip(out, before):
            np.testing.assert_array_equal(o[8:], b[8:])
        with pytest.raises(EngineError) as ei:  # sticky: later merges refuse too
            eng.treg_converge(np.arange(8, dtype=np.uint32), ts0[:8], pre0[:8], lr0[:8])
        assert ei.value.code == JY_ERANGE
    finally:
        eng.close()


def test_block_converge_parity(oracle_mod, engine):
    """jy_treg_converge_block (entry i -> slot slot0 + i): whole-range and
    sub-range blocks from host memory and HBM, interleaved with keyed batches
    that repeat slots inside a launch (the claim bitmaps' parity must
    survive the block launches in between); ties, shared 8-byte prefixes and
    long values, against the oracle repo"""
    import torch
    from jylis_amd._lib import TREG
    from jylis_amd.engine import encode_keys
    from jylis_amd.repo import RepoTREG
    O = oracle_mod
    rng = np.random.default_rng(23)
    n = 30000
    keys = [f"b{i}" for i in range(n)]
    want = O.Repo(O.TREG)
    got = RepoTREG(engine)
    got.converge_deltas(_batch(keys, [b""] * n, np.zeros(n, np.int64)))  # interns in order
    slots = engine.lookup(TREG, [k.encode() for k in keys])
    assert (slots == np.arange(n)).all()
    want.converge(_batch(keys, [b""] * n, np.zeros(n, np.int64)))
    prefixes = [bytes(rng.integers(0, 256, 8).astype(np.uint8)) for _ in range(8)]

    def vals(m):
        out = []
        for _ in range(m):
            L = int(rng.integers(0, 20))
            if rng.random() < 0.3:
                out.append((prefixes[rng.integers(8)] + bytes(rng.integers(97, 100, 12).astype(np.uint8)))[:max(L, 9)])
            else:
                out.append(bytes(rng.integers(0, 256, L).astype(np.uint8)))
        return out

    dev = torch.device("cuda", 0)
    for step in range(6):
        if step % 3 == 2:  # keyed, with repeats inside the launch
            idx = rng.integers(0, n, n)
            v = vals(n)
            ts = rng.integers(0, 6, n)
            b = _batch([keys[i] for i in idx], v, ts)
            want.converge(b)
            got.converge_deltas(b)
            continue
        lo = 0 if step % 2 == 0 else int(rng.integers(1, n // 2))
        hi = n if step % 2 == 0 else int(rng.integers(lo + 1, n))
        m = hi - lo
        v = vals(m)
        ts = rng.integers(0, 6, m).astype(np.uint64)
        vb, vo = encode_keys(v)
        pre, lr = engine.pack_values(TREG, (vb, vo))
        if step in (1, 3):
            engine.treg_converge_block(lo, *(torch.from_numpy(a.view(np.int64)).to(dev) for a in (ts, pre, lr)))
        else:
            engine.treg_converge_block(lo, ts, pre, lr)
        want.converge(_batch(keys[lo:hi], v, ts))
    assert_state_equal(O.TREG, want.state(), got.state())
    with pytest.raises(Exception):
        engine.treg_converge_block(n - 1, np.zeros(2, np.uint64), np.zeros(2, np.uint64), np.zeros(2, np.uint64))
