"""jy_counter_converge_keys: one peer counter batch WITH its key strings in
one call -- the keys interned on the device (_data_for, create on miss,
repo_gcount.pony:36-41) feed the COO max-merge directly.  Checked against a
numpy recomputation of the same cells (max per (key, replica, sign)) and
against the two-call path (jy_keys_intern + jy_*count_converge) on a second
engine: same slots, same state."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _batch(rng, nkeys, ncells, pool):
    ks = [pool[i] for i in rng.integers(0, len(pool), nkeys)]
    ks = list(dict.fromkeys(ks))  # one delta per key (the sender's Map)
    ck = rng.integers(0, len(ks), ncells).astype(np.uint32)
    return ks, ck


@pytest.mark.parametrize("ctype_name", ["GCOUNT", "PNCOUNT"])
@pytest.mark.parametrize("mem", ["host", "device"])
def test_converge_keys_matches_two_calls(ctype_name, mem):
    import torch
    from jylis_amd import _lib
    from jylis_amd.engine import Engine, encode_keys
    ctype = _lib.TYPE_NAMES[ctype_name]
    rng = np.random.default_rng(5 + ctype)
    pool = [b"k%d" % i for i in range(5000)] + [b"", b"\x00\xff", b"long" * 300]
    a, b = Engine(device=0), Engine(device=0)
    try:
        ids = [101, 202, 303, 404]
        cols_a, cols_b = a.replica_cols(ids), b.replica_cols(ids)
        assert list(cols_a) == list(cols_b)
        for rnd in range(5):
            ks, ck = _batch(rng, int(rng.integers(1, 3000)), int(rng.integers(1, 9000)), pool)
            col = cols_a[rng.integers(0, len(ids), len(ck))]
            val = rng.integers(0, 1 << 63, len(ck), dtype=np.uint64)
            val[rng.random(len(ck)) < 0.05] = np.uint64(2**64 - 1)
            sign = rng.integers(0, 2, len(ck)).astype(np.uint8) if ctype == _lib.PNCOUNT else None
            kb, ko = encode_keys(ks)
            if mem == "host":
                a.counter_converge_keys(ctype, (kb, ko), col, val, cell_key=ck, sign=sign)
            else:
                dev = torch.device("cuda", 0)
                t = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x).view(dt)).to(dev)
                a.counter_converge_keys(ctype, (t(kb, np.uint8), t(ko, np.int64)), t(col, np.int16),
                                        t(val, np.int64), cell_key=t(ck, np.int32),
                                        sign=None if sign is None else t(sign, np.uint8))
                torch.cuda.synchronize()
            # the two-call path on engine b
            slots = b.intern(ctype, (kb, ko))
            cs = slots[ck]
            if ctype == _lib.GCOUNT:
                b.gcount_converge(cs, col, val)
            else:
                p, n = sign == 0, sign == 1
                b.pncount_converge((cs[p], col[p], val[p]) if p.any() else None,
                                   (cs[n], col[n], val[n]) if n.any() else None)
            assert a.nkeys(ctype) == b.nkeys(ctype)
            np.testing.assert_array_equal(a.lookup(ctype, (kb, ko)), slots)
        nk = a.nkeys(ctype)
        got = a.counter_export(ctype, len(ids), 0, nk)
        want = b.counter_export(ctype, len(ids), 0, nk)
        np.testing.assert_array_equal(got, want)
        assert np.count_nonzero(got) > 0
    finally:
        a.close()
        b.close()


def test_converge_keys_rejects_bad_cells(engine):
    from jylis_amd import _lib
    from jylis_amd.engine import encode_keys
    kb, ko = encode_keys([b"a", b"b"])
    cols = engine.replica_cols([7])
    with pytest.raises(RuntimeError):
        engine.counter_converge_keys(_lib.GCOUNT, (kb, ko), cols[[0, 0]], np.array([1, 2], np.uint64),
                                     cell_key=np.array([0, 2], np.uint32))  # key 2 does not exist
    with pytest.raises(RuntimeError):
        engine.counter_converge_keys(_lib.PNCOUNT, (kb, ko), cols[[0, 0]], np.array([1, 2], np.uint64),
                                     sign=np.array([0, 3], np.uint8))
    assert engine.nkeys(_lib.GCOUNT) == 0  # nothing interned by a refused call
