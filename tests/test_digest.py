"""The canonical state digests behind the full-size pins (tests/golden/
fullsize_digests.json): the oracle's own maps, an oracle-format table and the
engine's read-back layout (value handles + arena; packed dots + dense vv)
must give the same digest, and the digest must see every field."""
import numpy as np
import pytest

from helpers import random_history


def _handles(t):
    """an oracle TLOG table -> the engine's read-back layout (pre, lr, arena)"""
    vb, vo = np.asarray(t["val_bytes"], np.uint8), np.asarray(t["val_offs"], np.int64)
    n = len(vo) - 1
    pre = np.zeros(n, np.uint64)
    lr = np.zeros(n, np.uint64)
    arena = bytearray(b"\xAA" * 24)  # junk before: offsets are real offsets
    for j in range(n):
        v = bytes(vb[vo[j]:vo[j + 1]])
        pre[j] = int.from_bytes((v[:8] + b"\0" * 8)[:8], "big")
        if len(v) > 8:
            while len(arena) % 8:
                arena.append(0)
            lr[j] = (len(arena) << 24) | len(v)
            arena += v
        else:
            lr[j] = len(v)
    return pre, lr, np.frombuffer(bytes(arena), np.uint8)


def _packed(t, R=16):
    """an oracle UJSON table -> packed dots over a column dictionary, dense vv"""
    ids = np.unique(np.concatenate([np.asarray(t[k], np.uint64) for k in ("dot_ids", "vv_ids", "cloud_ids")]))
    rng = np.random.default_rng(1)
    col_ids = ids[rng.permutation(len(ids))]  # any column order
    col = {int(x): c for c, x in enumerate(col_ids)}
    assert len(col_ids) <= R

    def pack(i, q):
        return np.array([(col[int(a)] << 48) | int(b) for a, b in zip(i, q)], np.uint64)
    n = len(t["key_offs"]) - 1
    vv = np.zeros((n, R), np.uint64)
    vo = np.asarray(t["vv_offs"], np.int64)
    for i in range(n):
        for j in range(vo[i], vo[i + 1]):
            vv[i, col[int(t["vv_ids"][j])]] = t["vv_seqs"][j]
    return (pack(t["dot_ids"], t["dot_seqs"]), np.asarray(t["elems"], np.uint64), vv,
            pack(t["cloud_ids"], t["cloud_seqs"]), col_ids)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tlog_digests_agree(oracle_mod, seed):
    O = oracle_mod
    r = O.Repo(O.TLOG)
    for b in random_history(O, O.TLOG, seed, nops=200, val_len=20):
        r.converge(b)
    t = r.state()
    d = O.digest_repo(r)
    assert d == O.digest_table(O.TLOG, t)
    pre, lr, arena = _handles(t)
    assert d == O.digest_tlog_handles(t["key_bytes"], t["key_offs"], t["cutoff"], t["ent_offs"], t["ts"], pre, lr,
                                      arena)
    assert d[1] == len(t["key_offs"]) - 1 and d[2] == len(t["ts"])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_ujson_digests_agree(oracle_mod, seed):
    O = oracle_mod
    r = O.Repo(O.UJSON)
    for b in random_history(O, O.UJSON, seed, nops=200):
        r.converge(b)
    t = r.state()
    d = O.digest_repo(r)
    assert d == O.digest_table(O.UJSON, t)
    dots, elems, vv, cloud, col_ids = _packed(t)
    assert d == O.digest_ujson_packed(t["key_bytes"], t["key_offs"], t["el_offs"], dots, elems, vv, t["cloud_offs"],
                                      cloud, col_ids)


def test_digest_sees_every_field(oracle_mod):
    """one changed cutoff, timestamp, value byte, entry order, element, vv
    entry or cloud dot changes the digest"""
    O = oracle_mod
    r = O.Repo(O.TLOG)
    for b in random_history(O, O.TLOG, 9, nops=200, val_len=20):
        r.converge(b)
    t = r.state()
    base = O.digest_table(O.TLOG, t)[0]
    j = int(np.argmax(np.diff(np.asarray(t["val_offs"], np.int64))))  # an entry with a non-empty value
    for mut in ("cutoff", "ts", "val_bytes"):
        u = {k: np.array(v, copy=True) for k, v in t.items()}
        idx = {"cutoff": 0, "ts": j, "val_bytes": int(t["val_offs"][j])}[mut]
        u[mut][idx] ^= 1
        assert O.digest_table(O.TLOG, u)[0] != base, mut
    u = {k: np.array(v, copy=True) for k, v in t.items()}
    eo = np.asarray(t["ent_offs"], np.int64)
    i = int(np.argmax(np.diff(eo)))  # a key with >= 2 entries: swap its first two
    a = eo[i]
    u["ts"][[a, a + 1]] = u["ts"][[a + 1, a]]
    assert O.digest_table(O.TLOG, u)[0] != base
    r = O.Repo(O.UJSON)
    for b in random_history(O, O.UJSON, 9, nops=200):
        r.converge(b)
    t = r.state()
    base = O.digest_table(O.UJSON, t)[0]
    for mut in ("elems", "dot_seqs", "vv_seqs", "cloud_seqs"):
        if len(t[mut]) == 0:
            continue
        u = {k: np.array(v, copy=True) for k, v in t.items()}
        u[mut][0] ^= 2
        assert O.digest_table(O.UJSON, u)[0] != base, mut


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_treg_digests_agree(oracle_mod, seed):
    """TREG (the config-3 pin): repo, table and read-back forms agree, and a
    changed timestamp or value byte changes the digest"""
    O = oracle_mod
    r = O.Repo(O.TREG)
    for b in random_history(O, O.TREG, seed, nops=200, val_len=20):
        r.converge(b)
    t = r.state()
    d = O.digest_repo(r)
    assert d == O.digest_table(O.TREG, t)
    pre, lr, arena = _handles(t)
    assert d == O.digest_treg_handles(t["key_bytes"], t["key_offs"], t["ts"], pre, lr, arena)
    assert d[1] == len(t["key_offs"]) - 1
    j = int(np.argmax(np.diff(np.asarray(t["val_offs"], np.int64))))
    for mut, idx in (("ts", j), ("val_bytes", int(t["val_offs"][j]))):
        u = {k: np.array(v, copy=True) for k, v in t.items()}
        u[mut][idx] ^= 1
        assert O.digest_table(O.TREG, u)[0] != d[0], mut


@pytest.mark.parametrize("ctype", [0, 1])
@pytest.mark.parametrize("seed", [4, 5])
def test_counter_dense_digest_agrees(oracle_mod, ctype, seed):
    """the engine's dense read-back ([sign][col][key], any column order, zero
    cells = absent) digests like the oracle's maps (configs 1 and 2 pins)"""
    O = oracle_mod
    r = O.Repo(ctype)
    for b in random_history(O, ctype, seed, nops=200, nkeys=30):
        r.converge(b)
    t = r.state()
    d = O.digest_repo(r)
    kb, ko = np.asarray(t["key_bytes"], np.uint8), np.asarray(t["key_offs"], np.uint64)
    n = len(ko) - 1
    pres = ("",) if ctype == O.GCOUNT else ("p_", "n_")
    ids = np.unique(np.concatenate([np.asarray(t[p + "ids"], np.uint64) for p in pres]))
    ids = ids[np.random.default_rng(seed).permutation(len(ids))]
    col = {int(x): c for c, x in enumerate(ids)}
    vals = np.zeros((len(pres), len(ids) + 2, n), np.uint64)  # two unused columns
    for s_, p in enumerate(pres):
        offs = np.asarray(t[p + "offs"], np.int64)
        for i in range(n):
            for j in range(offs[i], offs[i + 1]):
                vals[s_, col[int(t[p + "ids"][j])], i] = t[p + "vals"][j]
    allids = np.concatenate([ids, np.array([7, 9], np.uint64)])
    assert O.digest_counter_dense(kb, ko, allids, vals, threads=3) == d
    assert d[1] == n
    # every field is seen: a value, a key, a column's replica
    v2 = vals.copy()
    v2[0, 0, n // 2] ^= np.uint64(1 << 40)
    assert O.digest_counter_dense(kb, ko, allids, v2)[0] != d[0]
    ids2 = allids.copy()
    ids2[0] ^= np.uint64(1)
    assert O.digest_counter_dense(kb, ko, ids2, vals)[0] != d[0]
