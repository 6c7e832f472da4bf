"""Device key directory (k_keys.hip) against the reference's key semantics:
`_data_for(key)` creates on miss, `_data(key)?` only looks up
(repo_gcount.pony:36-41,53-55).  The oracle here is a Python dict handing out
dense slots in order of first occurrence, per type."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def first_occurrence(keys, table):
    out = []
    for k in keys:
        if k not in table:
            table[k] = len(table)
        out.append(table[k])
    return np.array(out, dtype=np.uint32)


def random_keys(rng, n, pool):
    """keys drawn from a pool with repeats, empty keys, shared prefixes, long keys"""
    idx = rng.integers(0, len(pool), n)
    return [pool[i] for i in idx]


def make_pool(rng, m):
    pool = [b""]
    for i in range(m):
        kind = i % 4
        if kind == 0:
            pool.append(b"key:%d" % i)
        elif kind == 1:
            pool.append(b"shared-prefix-" + bytes(rng.integers(0, 256, int(rng.integers(0, 6)), dtype=np.uint8)))
        elif kind == 2:
            pool.append(bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8)))
        else:
            pool.append(b"L" * int(rng.integers(100, 3000)) + b"%d" % i)
    return list(dict.fromkeys(pool))


def test_host_intern_matches_first_occurrence(engine):
    from jylis_amd._lib import GCOUNT, TLOG
    rng = np.random.default_rng(1)
    pool = make_pool(rng, 3000)
    tables = {GCOUNT: {}, TLOG: {}}
    for rnd in range(6):
        for t in tables:
            ks = random_keys(rng, int(rng.integers(1, 4000)), pool)
            got = engine.intern(t, ks)
            np.testing.assert_array_equal(got, first_occurrence(ks, tables[t]), err_msg=f"round {rnd} type {t}")
            assert engine.nkeys(t) == len(tables[t])


def test_device_intern_and_cross_lookup(engine):
    import torch
    from jylis_amd._lib import JY_NO_SLOT, TREG
    from jylis_amd.engine import encode_keys
    rng = np.random.default_rng(2)
    pool = make_pool(rng, 20000)
    table = {}
    for rnd in range(4):
        ks = random_keys(rng, 50000, pool)
        kb, ko = encode_keys(ks)
        got = engine.intern_device(TREG, torch.from_numpy(kb.copy()).cuda(),
                                   torch.from_numpy(ko.astype(np.int64)).cuda())
        np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), first_occurrence(ks, table))
        assert engine.nkeys(TREG) == len(table)
    # host lookups (cache misses -> device directory) agree; absent keys have no slot
    probe = pool[:500] + [b"never-interned-%d" % i for i in range(50)]
    want = np.array([table.get(k, JY_NO_SLOT) for k in probe], dtype=np.uint32)
    np.testing.assert_array_equal(engine.lookup(TREG, probe), want)
    np.testing.assert_array_equal(engine.lookup(TREG, probe), want)  # now from the cache
    # device lookup never creates
    kb, ko = encode_keys(probe)
    got = engine.intern_device(TREG, torch.from_numpy(kb.copy()).cuda(), torch.from_numpy(ko.astype(np.int64)).cuda(),
                               create=False)
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want)
    assert engine.nkeys(TREG) == len(table)


@pytest.mark.parametrize("mem", ["host", "device"])
def test_long_keys_found_again(engine, mem):
    """keys of every length class around the 16 bytes a table record holds,
    interned through the device directory (> 1024 keys: no host cache), are
    found again by a later probe -- lookup and a second intern give the same
    slots and create nothing; then again after the table has grown (rehash).
    (A miscompiled probe once lost every key over 16 bytes.)"""
    import torch
    from jylis_amd._lib import TLOG
    from jylis_amd.engine import encode_keys
    lens = [0, 1, 7, 8, 9, 15, 16, 17, 23, 24, 25, 31, 32, 33, 100, 1200, 4097]
    special = [(b"%d:" % n + b"x" * n)[:n] for n in lens] + [b"long" * 300, b"abcdefghijklmnopq"]
    filler = [b"f%d" % i for i in range(1100)]

    def intern(ks, create=True):
        if mem == "host":
            return engine.intern(TLOG, ks) if create else engine.lookup(TLOG, ks)
        kb, ko = encode_keys(ks)
        return engine.intern_device(TLOG, torch.from_numpy(kb.copy()).cuda(),
                                    torch.from_numpy(ko.astype(np.int64)).cuda(),
                                    create=create).cpu().numpy().view(np.uint32)
    table = {}
    for rnd in range(3):
        ks = special + filler + [b"grow%d-%d" % (rnd, i) for i in range(rnd * 3000)]
        s1 = intern(ks)
        np.testing.assert_array_equal(s1, first_occurrence(ks, table), err_msg=f"round {rnd}")
        assert engine.nkeys(TLOG) == len(table)
        np.testing.assert_array_equal(intern(ks, create=False), s1)
        np.testing.assert_array_equal(intern(ks), s1)
        assert engine.nkeys(TLOG) == len(table)


def test_heavy_duplicates_and_growth(engine):
    """many lanes racing on the same few keys, then enough keys to rehash
    the table several times"""
    import torch
    from jylis_amd._lib import UJSON
    from jylis_amd.engine import encode_keys
    table = {}
    ks = [b"hot%d" % (i % 5) for i in range(100000)]
    kb, ko = encode_keys(ks)
    got = engine.intern_device(UJSON, torch.from_numpy(kb.copy()).cuda(), torch.from_numpy(ko.astype(np.int64)).cuda())
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), first_occurrence(ks, table))
    for rnd in range(3):
        ks = [b"doc:%d" % i for i in range(rnd * 150000, (rnd + 2) * 150000)]
        kb, ko = encode_keys(ks)
        got = engine.intern_device(UJSON, torch.from_numpy(kb.copy()).cuda(),
                                   torch.from_numpy(ko.astype(np.int64)).cuda())
        np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), first_occurrence(ks, table))
    assert engine.nkeys(UJSON) == len(table)


def test_device_interned_keys_converge(engine, oracle_mod):
    """slots from the device directory address the same state the host path
    does: a GCOUNT converge through them reads back per key"""
    import torch
    from jylis_amd._lib import GCOUNT
    from jylis_amd.engine import encode_keys
    keys = [b"g%d" % i for i in range(1000)]
    kb, ko = encode_keys(keys)
    slots = engine.intern_device(GCOUNT, torch.from_numpy(kb.copy()).cuda(),
                                 torch.from_numpy(ko.astype(np.int64)).cuda()).cpu().numpy().view(np.uint32)
    col = np.full(len(keys), engine.replica_col(0xABCDEF), np.uint16)
    vals = np.arange(len(keys), dtype=np.uint64) * np.uint64(3)
    engine.gcount_converge(slots, col, vals)
    np.testing.assert_array_equal(engine.gcount_get(engine.lookup(GCOUNT, keys)), vals)


def test_large_host_batches_through_copy_pool(engine):
    """Host batches of several MiB go through the chunked parallel staging
    (host_copy.hip: worker threads copy 1-MiB chunks into pinned memory, each
    chunk's DMA issued as it lands) and the pinned slot readback.  Odd sizes
    leave a partial last chunk; the result must equal the first-occurrence
    slots and the COO converge must equal a numpy max over the same cells."""
    from jylis_amd._lib import GCOUNT
    rng = np.random.default_rng(7)
    n = 700_001  # key bytes ~8.4 MB, offsets 5.6 MB, slots 2.8 MB: every stage is chunked
    ids = rng.integers(0, 400_000, n)
    ks = [b"big-key-%07d" % i for i in ids.tolist()]
    table = {}
    want = first_occurrence(ks, table)
    got = engine.intern(GCOUNT, ks)
    np.testing.assert_array_equal(got, want)
    assert engine.nkeys(GCOUNT) == len(table)
    # cells from host memory: slots 2.8 MB, columns 1.4 MB, values 5.6 MB
    cols = engine.replica_cols([11, 22, 33]).astype(np.uint16)
    first_col = cols[rng.integers(0, 3, n)]
    val = rng.integers(1, 1 << 62, n, dtype=np.uint64)
    engine.gcount_converge(got, first_col, val)
    which = rng.integers(0, 3, n)
    col = cols[which]
    engine.gcount_converge(got, col, val)  # again, with other columns: max-merge per cell
    sums = engine.gcount_get(np.arange(len(table), dtype=np.uint32))
    cell = np.zeros((len(table), 3), np.uint64)
    ci = {int(c): i for i, c in enumerate(cols)}
    first_cols = np.array([ci[int(c)] for c in first_col], np.int64)
    np.maximum.at(cell, (got.astype(np.int64), first_cols), val)
    np.maximum.at(cell, (got.astype(np.int64), which), val)
    np.testing.assert_array_equal(np.asarray(sums, np.uint64), cell.sum(axis=1, dtype=np.uint64))
