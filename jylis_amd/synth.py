"""Seeded synthetic delta streams, numpy and torch.

Everything derives from splitmix64 over a cell index, so the host (numpy) and
device (torch) generators produce identical bits: small cases are checked
against the oracle on the host, full-size bench inputs are generated in HBM.

Base seed 0x4A594C4953 ("JYLIS"); config c uses base + c.
"""
import numpy as np

BASE_SEED = 0x4A594C4953
GOLDEN = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB
MASK64 = (1 << 64) - 1


def splitmix64_np(x):
    z = (np.asarray(x, dtype=np.uint64) + np.uint64(GOLDEN))
    z = (z ^ (z >> np.uint64(30))) * np.uint64(M1)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(M2)
    return z ^ (z >> np.uint64(31))


def _s64(v):
    """u64 constant -> the int64 with the same bits"""
    v &= MASK64
    return v - (1 << 64) if v >= (1 << 63) else v


def _srl(t, n):
    """logical shift right of an int64 tensor (bits as u64)"""
    import torch
    return (t >> n) & torch.tensor((1 << (64 - n)) - 1, dtype=torch.int64, device=t.device)


def splitmix64_torch(x):
    """x: int64 tensor holding u64 bits; wrapping int64 arithmetic == u64 arithmetic"""
    z = x + _s64(GOLDEN)
    z = (z ^ _srl(z, 30)) * _s64(M1)
    z = (z ^ _srl(z, 27)) * _s64(M2)
    return z ^ _srl(z, 31)


def replica_ids(n, seed=BASE_SEED):
    return splitmix64_np(np.arange(n, dtype=np.uint64) + np.uint64(seed))


def counter_keys(n, prefix=b"p", width=8, start=0):
    """fixed-width decimal keys b'p00000000'.. as (bytes, offs), vectorised"""
    idx = np.arange(start, start + n, dtype=np.uint64)
    digits = np.empty((n, width), np.uint8)
    v = idx.copy()
    for j in range(width - 1, -1, -1):
        digits[:, j] = (v % np.uint64(10)).astype(np.uint8) + ord("0")
        v //= np.uint64(10)
    pre = np.frombuffer(prefix, np.uint8)
    rows = np.concatenate([np.broadcast_to(pre, (n, len(pre))), digits], axis=1)
    L = rows.shape[1]
    return np.ascontiguousarray(rows).reshape(-1), np.arange(n + 1, dtype=np.uint64) * np.uint64(L)


# ---- counters (configs 1 and 2) --------------------------------------------

def counter_state_np(K, R, nsigns, seed, wrap_frac=True, cells=None):
    """initial state [nsigns][R][K] u64: uniform [0, 2^40); 10% near 2^64 (wrap).
    `cells` (flat indices sign*R*K + col*K + slot) evaluates only those cells."""
    if cells is None:
        cell = np.arange(nsigns * R * K, dtype=np.uint64).reshape(nsigns, R, K)
    else:
        cell = np.asarray(cells, np.uint64)
    h = splitmix64_np(cell * np.uint64(GOLDEN) + np.uint64(seed))
    s = h >> np.uint64(24)
    if wrap_frac:
        near = (splitmix64_np(h) % np.uint64(10)) == 0
        s = np.where(near, np.uint64(MASK64) - (h >> np.uint64(44)), s)
    return s


def counter_delta_np(prev, rnd, seed, cells=None):
    """next peer batch from `prev`: 75% prev + U[1,1000], 25% stale prev - U[0,1000]"""
    if cells is None:
        cell = np.arange(prev.size, dtype=np.uint64).reshape(prev.shape)
    else:
        cell = np.asarray(cells, np.uint64)
    h = splitmix64_np(cell * np.uint64(GOLDEN) + np.uint64(seed) + np.uint64((rnd + 1) * M2 & MASK64))
    inc = (h % np.uint64(1000)) + np.uint64(1)
    dec = (h >> np.uint64(16)) % np.uint64(1001)
    stale = ((h >> np.uint64(32)) & np.uint64(3)) == 0
    return np.where(stale, prev - dec, prev + inc)


def counter_state_torch(K, R, nsigns, seed, device, wrap_frac=True, out=None):
    import torch
    n = nsigns * R * K
    cell = torch.arange(n, dtype=torch.int64, device=device)
    h = splitmix64_torch(cell * _s64(GOLDEN) + _s64(seed))
    s = _srl(h, 24)
    if wrap_frac:
        hh = splitmix64_torch(h)
        # (u64 hh) % 10 == 0 via unsigned remainder on the two 32-bit halves
        near = _umod(hh, 10) == 0
        s = torch.where(near, -1 - _srl(h, 44), s)
    s = s.view(nsigns, R, K)
    if out is not None:
        out.copy_(s)
        return out
    return s


def _umod(t, m):
    """u64 remainder of int64 bits by a small m"""
    import torch
    hi = _srl(t, 32)
    lo = t & 0xFFFFFFFF
    return ((hi % m) * ((1 << 32) % m) + lo % m) % m


def counter_delta_torch(prev, rnd, seed, out=None):
    import torch
    cell = torch.arange(prev.numel(), dtype=torch.int64, device=prev.device).view(prev.shape)
    h = splitmix64_torch(cell * _s64(GOLDEN) + _s64(seed) + _s64((rnd + 1) * M2))
    inc = _umod(h, 1000) + 1
    dec = _umod(_srl(h, 16), 1001)
    stale = (_srl(h, 32) & 3) == 0
    r = torch.where(stale, prev - dec, prev + inc)
    if out is not None:
        out.copy_(r)
        return out
    return r


def counter_rows_torch(out, seed, rnd=None, prev=None, wrap_frac=True):
    """Fill out[nsigns][R][K] (int64 bits of u64) row by row, bounding temporaries:
    rnd None -> initial state; else the round-`rnd` delta from `prev`."""
    import torch
    nsigns, R, K = out.shape
    ar = torch.arange(K, dtype=torch.int64, device=out.device)
    for s in range(nsigns):
        for c in range(R):
            cell = ar + (s * R + c) * K
            if rnd is None:
                h = splitmix64_torch(cell * _s64(GOLDEN) + _s64(seed))
                v = _srl(h, 24)
                if wrap_frac:
                    near = _umod(splitmix64_torch(h), 10) == 0
                    v = torch.where(near, -1 - _srl(h, 44), v)
            else:
                h = splitmix64_torch(cell * _s64(GOLDEN) + _s64(seed) + _s64((rnd + 1) * M2))
                inc = _umod(h, 1000) + 1
                dec = _umod(_srl(h, 16), 1001)
                stale = (_srl(h, 32) & 3) == 0
                p = prev[s, c]
                v = torch.where(stale, p - dec, p + inc)
            out[s, c].copy_(v)
    return out


def counter_batch_tables(state_or_delta, replica_id_list, key_tab, prefix=""):
    """[R][K] (GCOUNT) or [2][R][K] (PNCOUNT) array -> per-replica oracle batch tables
    (one flushed peer batch per replica column, every key carrying that column)"""
    kb, ko = key_tab
    arr = np.asarray(state_or_delta)
    if arr.ndim == 2:
        arr = arr[None]
    nsigns, R, K = arr.shape
    out = []
    for c in range(R):
        t = {"key_bytes": kb, "key_offs": ko}
        for s, pre in zip(range(nsigns), ("p_", "n_") if nsigns == 2 else ("",)):
            t[pre + "offs"] = np.arange(K + 1, dtype=np.uint64)
            t[pre + "ids"] = np.full(K, replica_id_list[c], np.uint64)
            t[pre + "vals"] = arr[s, c].astype(np.uint64)
        out.append(t)
    return out
