"""ctypes wrapper of the CPU oracle (oracle/jy_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product path.

Batches and states travel as dicts of numpy arrays ("tables"):
  common   key_bytes u8, key_offs u64[n+1]
  GCOUNT   offs, ids, vals                 (per key CSR of replica id -> value)
  PNCOUNT  p_offs, p_ids, p_vals, n_offs, n_ids, n_vals
  TREG     ts, val_bytes, val_offs
  TLOG     cutoff, ent_offs, ts, val_bytes, val_offs
  UJSON    el_offs, dot_ids, dot_seqs, elems, vv_offs, vv_ids, vv_seqs,
           cloud_offs, cloud_ids, cloud_seqs
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libjy_oracle.so")
GCOUNT, PNCOUNT, TREG, TLOG, UJSON = 0, 1, 2, 3, 4

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    P, U64, I64, I32, U32 = C.c_void_p, C.c_uint64, C.c_int64, C.c_int32, C.c_uint32
    sig = {
        "or_table_new": (P, []), "or_table_free": (None, [P]),
        "or_table_set": (None, [P, C.c_char_p, P, U64, U64]),
        "or_table_nfields": (U64, [P]), "or_table_field_name": (C.c_char_p, [P, U64]),
        "or_table_field_data": (P, [P, U64]), "or_table_field_nbytes": (U64, [P, U64]),
        "or_table_field_elem": (U64, [P, U64]),
        "or_repo_new": (P, [I32, U64]), "or_repo_free": (None, [P]), "or_repo_nkeys": (U64, [P]),
        "or_batch_import": (P, [I32, P]), "or_batch_free": (None, [P]), "or_batch_size": (U64, [P]),
        "or_batch_export": (P, [P]), "or_converge": (None, [P, P]), "or_state_export": (P, [P]),
        "or_flush": (P, [P]), "or_deltas_size": (U64, [P]),
        "or_gcount_get": (U64, [P, C.c_char_p, U64]), "or_pncount_get": (I64, [P, C.c_char_p, U64]),
        "or_treg_get": (I32, [P, C.c_char_p, U64, P, P, U64, P]),
        "or_tlog_size": (U64, [P, C.c_char_p, U64]), "or_tlog_cutoff": (U64, [P, C.c_char_p, U64]),
        "or_gcount_inc": (None, [P, C.c_char_p, U64, U64]),
        "or_pncount_inc": (None, [P, C.c_char_p, U64, I64]),
        "or_pncount_dec": (None, [P, C.c_char_p, U64, I64]),
        "or_treg_set": (None, [P, C.c_char_p, U64, C.c_char_p, U64, U64]),
        "or_tlog_ins": (None, [P, C.c_char_p, U64, C.c_char_p, U64, U64]),
        "or_tlog_trimat": (None, [P, C.c_char_p, U64, U64]),
        "or_tlog_trim": (None, [P, C.c_char_p, U64, U64]),
        "or_tlog_clr": (None, [P, C.c_char_p, U64]),
        "or_ujson_ins": (None, [P, C.c_char_p, U64, U64]),
        "or_ujson_rm": (None, [P, C.c_char_p, U64, U64]),
        "or_ujson_clr": (None, [P, C.c_char_p, U64]),
        "or_ujson_touch": (None, [P, C.c_char_p, U64]),
        "or_digest_repo": (I32, [P, P]),
        "or_digest_counter_dense": (I32, [U64, P, P, U32, U32, P, P, U64, U32, P]),
        "or_digest_table": (I32, [I32, P, P]),
        "or_digest_tlog_handles": (I32, [U64, P, P, P, P, P, P, P, P, U64, P]),
        "or_digest_treg_handles": (I32, [U64, P, P, P, P, P, P, U64, P]),
        "or_digest_ujson_packed": (I32, [U64, P, P, P, P, P, P, U64, P, P, P, U64, P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


_DT = {1: np.uint8, 8: np.uint64}


def _table_out(t):
    lib = load()
    out = {}
    for i in range(lib.or_table_nfields(t)):
        name = lib.or_table_field_name(t, i).decode()
        nb = lib.or_table_field_nbytes(t, i)
        elem = lib.or_table_field_elem(t, i)
        arr = np.empty(nb // elem, dtype=_DT[elem])
        if nb:
            C.memmove(arr.ctypes.data, lib.or_table_field_data(t, i), nb)
        out[name] = arr
    lib.or_table_free(t)
    return out


def _table_in(d):
    lib = load()
    t = lib.or_table_new()
    for name, arr in d.items():
        a = np.ascontiguousarray(arr)
        if a.dtype.itemsize not in (1, 8):
            a = a.astype(np.uint64)
        lib.or_table_set(t, name.encode(), a.ctypes.data, a.nbytes, a.dtype.itemsize)
    return t


def _b(k):
    return k.encode() if isinstance(k, str) else bytes(k)


class Batch:
    """A decoded delta batch (Array[(String, Any box)]) held by the oracle."""

    def __init__(self, ctype, table=None, handle=None):
        lib = load()
        self.ctype = ctype
        if handle is None:
            t = _table_in(table)
            handle = lib.or_batch_import(ctype, t)
            lib.or_table_free(t)
        self.h = handle

    def __len__(self):
        return int(load().or_batch_size(self.h))

    def table(self):
        return _table_out(load().or_batch_export(self.h))

    def __del__(self):
        if getattr(self, "h", None):
            load().or_batch_free(self.h)
            self.h = None


class Repo:
    """RepoXXX restated on CPU (one per type, like one RepoManager)."""

    def __init__(self, ctype, identity=0):
        self.lib = load()
        self.ctype = ctype
        self.h = self.lib.or_repo_new(ctype, identity)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.or_repo_free(self.h)
            self.h = None

    def nkeys(self):
        return int(self.lib.or_repo_nkeys(self.h))

    def converge(self, batch):
        if not isinstance(batch, Batch):
            batch = Batch(self.ctype, batch)
        self.lib.or_converge(self.h, batch.h)

    def state(self):
        return _table_out(self.lib.or_state_export(self.h))

    def flush(self):
        return Batch(self.ctype, handle=self.lib.or_flush(self.h))

    def deltas_size(self):
        return int(self.lib.or_deltas_size(self.h))

    # reads
    def gcount_get(self, k):
        k = _b(k)
        return int(self.lib.or_gcount_get(self.h, k, len(k)))

    def pncount_get(self, k):
        k = _b(k)
        return int(self.lib.or_pncount_get(self.h, k, len(k)))

    def treg_get(self, k):
        k = _b(k)
        ts, vlen = C.c_uint64(), C.c_uint64()
        buf = C.create_string_buffer(1 << 16)
        ok = self.lib.or_treg_get(self.h, k, len(k), C.byref(ts), buf, 1 << 16, C.byref(vlen))
        return (buf.raw[: vlen.value], ts.value) if ok else None

    def tlog_size(self, k):
        k = _b(k)
        return int(self.lib.or_tlog_size(self.h, k, len(k)))

    def tlog_cutoff(self, k):
        k = _b(k)
        return int(self.lib.or_tlog_cutoff(self.h, k, len(k)))

    # writes
    def gcount_inc(self, k, v):
        k = _b(k)
        self.lib.or_gcount_inc(self.h, k, len(k), v)

    def pncount_inc(self, k, v):
        k = _b(k)
        self.lib.or_pncount_inc(self.h, k, len(k), v)

    def pncount_dec(self, k, v):
        k = _b(k)
        self.lib.or_pncount_dec(self.h, k, len(k), v)

    def treg_set(self, k, v, ts):
        k, v = _b(k), _b(v)
        self.lib.or_treg_set(self.h, k, len(k), v, len(v), ts)

    def tlog_ins(self, k, v, ts):
        k, v = _b(k), _b(v)
        self.lib.or_tlog_ins(self.h, k, len(k), v, len(v), ts)

    def tlog_trimat(self, k, ts):
        k = _b(k)
        self.lib.or_tlog_trimat(self.h, k, len(k), ts)

    def tlog_trim(self, k, n):
        k = _b(k)
        self.lib.or_tlog_trim(self.h, k, len(k), n)

    def tlog_clr(self, k):
        k = _b(k)
        self.lib.or_tlog_clr(self.h, k, len(k))

    def ujson_ins(self, k, elem):
        k = _b(k)
        self.lib.or_ujson_ins(self.h, k, len(k), elem)

    def ujson_rm(self, k, elem):
        k = _b(k)
        self.lib.or_ujson_rm(self.h, k, len(k), elem)

    def ujson_clr(self, k):
        k = _b(k)
        self.lib.or_ujson_clr(self.h, k, len(k))

    def ujson_touch(self, k):
        k = _b(k)
        self.lib.or_ujson_touch(self.h, k, len(k))


def split_keys(table):
    kb, ko = table["key_bytes"], table["key_offs"]
    return [bytes(kb[ko[i]:ko[i + 1]]) for i in range(len(ko) - 1)]


# ---- canonical state digests (tests/golden full-size pins; see or_digest_* in
# jy_oracle.cpp): {digest, keys, entries / elements, value bytes / cloud dots}

def _digest_out(rc, out):
    if rc != 0:
        raise ValueError(f"digest failed ({rc})")
    return tuple(int(x) for x in out)


def digest_repo(repo):
    out = np.zeros(4, np.uint64)
    return _digest_out(load().or_digest_repo(repo.h, out.ctypes.data), out)


def digest_counter_dense(kb, ko, ids, vals, threads=None):
    """the engine's dense counter read-back: vals [nsigns][ncols][n] (nsigns 1:
    GCOUNT, 2: PNCOUNT), column c holding replica ids[c]"""
    import os
    vals = np.ascontiguousarray(vals, np.uint64)
    if vals.ndim == 2:
        vals = vals[None]
    nsigns, ncols, n = vals.shape
    keep = [_c(kb, np.uint8), _c(ko, np.uint64), _c(ids, np.uint64)]
    assert len(keep[1][0]) == n + 1 and len(keep[2][0]) >= ncols
    out = np.zeros(4, np.uint64)
    T = threads or min(32, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 1)
    rc = load().or_digest_counter_dense(n, keep[0][1], keep[1][1], nsigns, ncols, keep[2][1], vals.ctypes.data, n, T,
                                        out.ctypes.data)
    return _digest_out(rc, out)


def digest_table(ctype, table):
    out = np.zeros(4, np.uint64)
    t = _table_in(table)
    try:
        return _digest_out(load().or_digest_table(ctype, t, out.ctypes.data), out)
    finally:
        load().or_table_free(t)


def _c(a, dt):
    a = np.ascontiguousarray(a, dt)
    return a, a.ctypes.data


def digest_tlog_handles(kb, ko, cut, eo, ts, pre, lr, arena):
    """the engine's TLOG read-back (value handles + the arena bytes)"""
    keep = [_c(kb, np.uint8), _c(ko, np.uint64), _c(cut, np.uint64), _c(eo, np.uint64), _c(ts, np.uint64),
            _c(pre, np.uint64), _c(lr, np.uint64), _c(arena, np.uint8)]
    out = np.zeros(4, np.uint64)
    n = len(keep[1][0]) - 1
    rc = load().or_digest_tlog_handles(n, *(p for _, p in keep[:7]), keep[7][1], len(keep[7][0]), out.ctypes.data)
    return _digest_out(rc, out)


def digest_treg_handles(kb, ko, ts, pre, lr, arena):
    """the engine's TREG read-back (per key ts + value handle, the arena bytes)"""
    keep = [_c(kb, np.uint8), _c(ko, np.uint64), _c(ts, np.uint64), _c(pre, np.uint64), _c(lr, np.uint64),
            _c(arena, np.uint8)]
    out = np.zeros(4, np.uint64)
    n = len(keep[1][0]) - 1
    rc = load().or_digest_treg_handles(n, *(p for _, p in keep[:5]), keep[5][1], len(keep[5][0]), out.ctypes.data)
    return _digest_out(rc, out)


def digest_ujson_packed(kb, ko, eo, dots, elems, vv, co, cloud, col_ids):
    """the engine's UJSON read-back (packed dots, dense vv [n][R])"""
    vv = np.ascontiguousarray(vv, np.uint64)
    R = vv.shape[1] if vv.ndim == 2 else 0
    keep = [_c(kb, np.uint8), _c(ko, np.uint64), _c(eo, np.uint64), _c(dots, np.uint64), _c(elems, np.uint64),
            (vv, vv.ctypes.data), _c(co, np.uint64), _c(cloud, np.uint64), _c(col_ids, np.uint64)]
    out = np.zeros(4, np.uint64)
    n = len(keep[1][0]) - 1
    rc = load().or_digest_ujson_packed(n, keep[0][1], keep[1][1], keep[2][1], keep[3][1], keep[4][1], keep[5][1], R,
                                       keep[6][1], keep[7][1], keep[8][1], len(keep[8][0]), out.ctypes.data)
    return _digest_out(rc, out)
