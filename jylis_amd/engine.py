"""Python handle over the C ABI of the engine (include/jylis_gpu.h).

Arrays may be numpy (host memory, staged by the engine) or torch CUDA
tensors (HBM-resident, read in stream order).  Each call mirrors one entry
point; higher-level repo semantics live in jylis_amd.repo.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import DEVICE, GCOUNT, HOST, PNCOUNT, TLOG, TREG, UJSON

LR_LEN_BITS = 24
LR_LEN_MASK = (1 << LR_LEN_BITS) - 1
DOT_SEQ_BITS = 48
DOT_SEQ_MASK = (1 << DOT_SEQ_BITS) - 1


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"jylis engine error {code}: {msg}")
        self.code = code


def _is_torch(x):
    return type(x).__module__.startswith("torch") and hasattr(x, "data_ptr")


def _arg(x, dtype):
    """-> (keepalive, pointer, mem) for a numpy array or a CUDA tensor."""
    if x is None:
        return None, None, HOST
    if _is_torch(x):
        if not x.is_cuda:
            x = x.numpy()
        else:
            assert x.is_contiguous(), "device arrays must be contiguous"
            assert x.element_size() == np.dtype(dtype).itemsize, (x.dtype, dtype)
            return x, C.c_void_p(x.data_ptr()), DEVICE
    a = np.ascontiguousarray(x, dtype=dtype)
    return a, C.c_void_p(a.ctypes.data), HOST


def _same_mem(*mems):
    ms = {m for m in mems}
    if len(ms) > 1:
        raise ValueError("all arrays of one call must live in the same memory (host or device)")
    return ms.pop() if ms else HOST


def encode_keys(keys):
    """list of str/bytes -> (uint8 bytes, uint64 offsets[n+1])"""
    bs = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
    offs = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        offs[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bs), dtype=np.uint8) if bs else np.zeros(0, np.uint8)
    return buf, offs


def pack_dot(col, seq):
    return (np.asarray(col, dtype=np.uint64) << np.uint64(DOT_SEQ_BITS)) | np.asarray(seq, dtype=np.uint64)


def unpack_dot(d):
    d = np.asarray(d, dtype=np.uint64)
    return (d >> np.uint64(DOT_SEQ_BITS)).astype(np.uint32), d & np.uint64(DOT_SEQ_MASK)


class Engine:
    """One engine = one GPU = one key shard."""

    def __init__(self, device=0, counter_columns=16, ujson_columns=16, key_capacity=1024,
                 entry_capacity=8192, arena_capacity=1 << 16, flags=0):
        self.lib = _lib.load()
        cfg = _lib.JyConfig()
        self.lib.jy_config_default(C.byref(cfg))
        cfg.device = device
        cfg.counter_columns = counter_columns
        cfg.ujson_columns = ujson_columns
        cfg.flags = flags
        for t in range(5):
            cfg.key_capacity[t] = key_capacity if np.isscalar(key_capacity) else key_capacity[t]
            cfg.entry_capacity[t] = entry_capacity
            cfg.arena_capacity[t] = arena_capacity
        h = C.c_void_p()
        rc = self.lib.jy_engine_create(C.byref(cfg), C.byref(h))
        if rc != 0 or not h.value:
            raise EngineError(rc, "jy_engine_create failed (no GPU / HIP runtime?)")
        self.h = h
        self.device = device
        self.ujson_columns = ujson_columns

    @classmethod
    def attach(cls, handle, device, ujson_columns=16):
        """a view of an engine someone else owns (a node's shard, jy_node_engine):
        close() leaves it alone"""
        self = cls.__new__(cls)
        self.lib = _lib.load()
        self.h = C.c_void_p(handle)
        self.device = device
        self.ujson_columns = ujson_columns
        self._borrowed = True
        return self

    # -- lifecycle ---------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            if not getattr(self, "_borrowed", False):
                self.lib.jy_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise EngineError(rc, self.lib.jy_last_error(self.h).decode(errors="replace"))

    def sync(self):
        self._check(self.lib.jy_sync(self.h))

    def set_stream(self, stream_ptr):
        self._check(self.lib.jy_set_stream(self.h, C.c_void_p(stream_ptr)))

    def stream(self):
        return self.lib.jy_get_stream(self.h)

    def timing(self, on=True):
        """bracket every merge call's device work with HIP events (jy_timing_enable)"""
        self._check(self.lib.jy_timing_enable(self.h, 1 if on else 0))

    def timing_read(self, cap=4096):
        """-> per-call device durations (ms) since the last read"""
        out = np.zeros(cap, np.float64)
        n = C.c_uint64()
        self._check(self.lib.jy_timing_read(self.h, cap, out.ctypes.data, C.byref(n)))
        return out[:min(n.value, cap)].copy()

    def skipped(self):
        return int(self.lib.jy_skipped(self.h))

    # -- replicas / keys ---------------------------------------------------
    def replica_col(self, rid):
        c = C.c_uint32()
        self._check(self.lib.jy_replica_col(self.h, C.c_uint64(int(rid) & (2**64 - 1)), C.byref(c)))
        return c.value

    def replica_cols(self, rids):
        return np.array([self.replica_col(r) for r in rids], dtype=np.uint16)

    def replica_id(self, col):
        v = C.c_uint64()
        self._check(self.lib.jy_replica_id(self.h, col, C.byref(v)))
        return v.value

    def replica_count(self):
        return int(self.lib.jy_replica_count(self.h))

    def _keys(self, keys):
        if isinstance(keys, tuple):
            kb, ko = keys
            return np.ascontiguousarray(kb, np.uint8), np.ascontiguousarray(ko, np.uint64)
        return encode_keys(keys)

    def intern(self, ctype, keys):
        kb, ko = self._keys(keys)
        n = len(ko) - 1
        out = np.empty(n, dtype=np.uint32)
        self._check(self.lib.jy_keys_intern(self.h, ctype, n, kb.ctypes.data, ko.ctypes.data, out.ctypes.data))
        return out

    def lookup(self, ctype, keys):
        kb, ko = self._keys(keys)
        n = len(ko) - 1
        out = np.empty(n, dtype=np.uint32)
        self._check(self.lib.jy_keys_lookup(self.h, ctype, n, kb.ctypes.data, ko.ctypes.data, out.ctypes.data))
        return out

    def intern_device(self, ctype, key_bytes, key_offs, create=True):
        """bulk interning with keys already in HBM: key_bytes (uint8) and
        key_offs (int64/uint64, n+1) CUDA tensors -> int32 CUDA tensor of slots"""
        import torch
        n = int(key_offs.numel()) - 1
        out = torch.empty(max(n, 1), dtype=torch.int32, device=key_offs.device)
        fn = self.lib.jy_keys_intern_mem if create else self.lib.jy_keys_lookup_mem
        self._check(fn(self.h, ctype, n, key_bytes.data_ptr(), key_offs.data_ptr(), out.data_ptr(), DEVICE))
        return out[:n]

    def key_names(self, ctype, slot0, n):
        """key strings of slots [slot0, slot0 + n) from the device directory (jy_keys_export)"""
        offs = np.zeros(n + 1, np.uint64)
        if n == 0:
            return []
        self._check(self.lib.jy_keys_export(self.h, ctype, slot0, n, offs.ctypes.data, None, 0))
        buf = np.empty(max(int(offs[-1]), 1), np.uint8)
        self._check(self.lib.jy_keys_export(self.h, ctype, slot0, n, offs.ctypes.data, buf.ctypes.data, len(buf)))
        raw = buf.tobytes()
        return [raw[int(offs[i]):int(offs[i + 1])] for i in range(n)]

    def keys_route_part(self, key_bytes, key_offs, nshards):
        """cross-shard key resolution, sender side (jy_keys_route_part): CUDA
        uint8 key bytes + int64 offsets -> (owner i32[n], pos i32[n], lens
        i64[n], bytes u8, counts i64[2 * nshards]) with the keys in owner order"""
        import torch
        n = int(key_offs.numel()) - 1
        dev = key_offs.device
        own = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        pos = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        lens = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        byts = torch.empty(max(int(key_bytes.numel()), 1), dtype=torch.uint8, device=dev)
        cnt = torch.empty(2 * nshards, dtype=torch.int64, device=dev)
        self._check(self.lib.jy_keys_route_part(self.h, n, key_bytes.data_ptr(), key_offs.data_ptr(), nshards,
                                                own.data_ptr(), pos.data_ptr(), lens.data_ptr(), byts.data_ptr(),
                                                cnt.data_ptr()))
        return own[:n], pos[:n], lens[:n], byts, cnt

    def keys_intern_lens(self, ctype, key_bytes, lens):
        """intern received keys given as (bytes, lengths) CUDA tensors -> int32 slots (jy_keys_intern_lens)"""
        import torch
        n = int(lens.numel())
        out = torch.empty(max(n, 1), dtype=torch.int32, device=lens.device)
        if n:
            self._check(self.lib.jy_keys_intern_lens(self.h, ctype, n, key_bytes.data_ptr(), lens.data_ptr(),
                                                     out.data_ptr()))
        return out[:n]

    def keys_route_back(self, pos, answers):
        """slots in input order: out[i] = answers[pos[i]] (jy_keys_route_back)"""
        import torch
        n = int(pos.numel())
        out = torch.empty(max(n, 1), dtype=torch.int32, device=pos.device)
        if n:
            self._check(self.lib.jy_keys_route_back(self.h, n, pos.data_ptr(), answers.data_ptr(), out.data_ptr()))
        return out[:n]

    def nkeys(self, ctype):
        return int(self.lib.jy_keys_count(self.h, ctype))

    def reserve(self, ctype, cap):
        self._check(self.lib.jy_keys_reserve(self.h, ctype, cap))

    def pack_values(self, ctype, values):
        """bytes values -> (pre, lr) uint64 arrays; long values go to the arena"""
        vb, vo = encode_keys(values) if not isinstance(values, tuple) else values
        vb = np.ascontiguousarray(vb, np.uint8)
        vo = np.ascontiguousarray(vo, np.uint64)
        n = len(vo) - 1
        pre = np.empty(n, np.uint64)
        lr = np.empty(n, np.uint64)
        self._check(self.lib.jy_values_pack(self.h, ctype, n, vb.ctypes.data, vo.ctypes.data,
                                            pre.ctypes.data, lr.ctypes.data))
        return pre, lr

    def arena_usage(self, ctype):
        n, c = C.c_uint64(), C.c_uint64()
        self._check(self.lib.jy_arena_usage(self.h, ctype, C.byref(n), C.byref(c)))
        return n.value, c.value

    def arena_reserve(self, ctype, nbytes):
        """room for `nbytes` at the tail of a type's value arena (jy_arena_reserve):
        (device pointer, arena offset); valid until the arena next grows"""
        p, r = C.c_void_p(), C.c_uint64()
        self._check(self.lib.jy_arena_reserve(self.h, ctype, nbytes, C.byref(p), C.byref(r)))
        return p.value or 0, r.value

    def arena_collect(self, ctype):
        """reclaim dead value bytes (jy_arena_collect); unmerged packed handles become invalid.
        Refused while a router holds rounds of this engine's batches in flight: their
        handles would be read again by a drain round (route.py _RunRouter)."""
        holds = getattr(self, "_route_holds", None)
        if holds:
            raise RuntimeError("arena_collect while a router has rounds in flight on this engine: "
                               "call router.drain() first")
        live = C.c_uint64()
        self._check(self.lib.jy_arena_collect(self.h, ctype, C.byref(live)))
        return live.value

    def arena_read(self, ctype, off, n):
        buf = np.empty(max(n, 1), np.uint8)
        self._check(self.lib.jy_arena_read(self.h, ctype, off, n, buf.ctypes.data))
        return bytes(buf[:n])

    def value_bytes(self, ctype, pre, lr):
        """(pre, lr) handle -> bytes"""
        pre, lr = int(pre), int(lr)
        n = lr & LR_LEN_MASK
        if n <= 8:
            return pre.to_bytes(8, "big")[:n]
        return self.arena_read(ctype, lr >> LR_LEN_BITS, n)

    # -- GCOUNT / PNCOUNT --------------------------------------------------
    def gcount_converge(self, slot, col, val):
        a, pa, ma = _arg(slot, np.uint32)
        b, pb, mb = _arg(col, np.uint16)
        c, pc, mc = _arg(val, np.uint64)
        mem = _same_mem(ma, mb, mc)
        self._check(self.lib.jy_gcount_converge(self.h, len(a), pa, pb, pc, mem))

    def counter_converge_keys(self, ctype, keys, col, val, cell_key=None, sign=None):
        """one peer batch with its key strings (jy_counter_converge_keys):
        keys interned on the device, cells merged with the device slots.
        Host keys (list or (bytes, offs)) with host cells, or CUDA tensors
        throughout (keys as (uint8 bytes, int64 offs))."""
        if isinstance(keys, tuple) and hasattr(keys[0], "data_ptr"):
            kb, ko = keys
            nk = int(ko.numel()) - 1
            pkb, pko = C.c_void_p(kb.data_ptr()), C.c_void_p(ko.data_ptr())
            km = DEVICE
        else:
            kb, ko = self._keys(keys)
            nk = len(ko) - 1
            pkb, pko = kb.ctypes.data, ko.ctypes.data
            km = HOST
        c, pc, mc = _arg(col, np.uint16)
        v, pv, mv = _arg(val, np.uint64)
        args = [(c, mc), (v, mv)]
        pk = ps = None
        if cell_key is not None:
            k_, pk, mk = _arg(cell_key, np.uint32)
            args.append((k_, mk))
        if sign is not None:
            s_, ps, ms = _arg(sign, np.uint8)
            args.append((s_, ms))
        mem = _same_mem(km, *[m for _, m in args])
        self._check(self.lib.jy_counter_converge_keys(self.h, ctype, nk, pkb, pko, len(c), pk, ps, pc, pv, mem))

    def gcount_converge_block(self, cols, slot0, vals):
        cols = np.ascontiguousarray(cols, np.uint16)
        v, pv, mv = _arg(vals, np.uint64)
        ncols = len(cols)
        nslots = (v.shape[-1] if v.ndim > 1 else (len(v) // max(ncols, 1)))
        self._check(self.lib.jy_gcount_converge_block(self.h, ncols, cols.ctypes.data, slot0, nslots, pv, mv))

    def gcount_get(self, slots):
        s, ps, ms = _arg(slots, np.uint32)
        if ms == DEVICE:
            import torch
            out = torch.empty(len(s), dtype=torch.int64, device=s.device)
            self._check(self.lib.jy_gcount_get(self.h, len(s), ps, C.c_void_p(out.data_ptr()), DEVICE))
            return out
        out = np.empty(len(s), np.uint64)
        self._check(self.lib.jy_gcount_get(self.h, len(s), ps, out.ctypes.data, HOST))
        return out

    def pncount_converge(self, p=None, n=None):
        """p / n: (slot, col, val) triples (either may be None)"""
        ps = [_arg(x, t) for x, t in zip(p or (None, None, None), (np.uint32, np.uint16, np.uint64))]
        ns = [_arg(x, t) for x, t in zip(n or (None, None, None), (np.uint32, np.uint16, np.uint64))]
        mems = [m for (k, _, m) in ps + ns if k is not None]
        mem = _same_mem(*mems)
        np_ = len(ps[0][0]) if ps[0][0] is not None else 0
        nn = len(ns[0][0]) if ns[0][0] is not None else 0
        self._check(self.lib.jy_pncount_converge(self.h, np_, ps[0][1], ps[1][1], ps[2][1],
                                                 nn, ns[0][1], ns[1][1], ns[2][1], mem))

    def pncount_converge_block(self, cols, slot0, vals_p, vals_n):
        cols = np.ascontiguousarray(cols, np.uint16)
        a, pa, ma = _arg(vals_p, np.uint64)
        b, pb, mb = _arg(vals_n, np.uint64)
        mem = _same_mem(ma, mb)
        ncols = len(cols)
        nslots = a.shape[-1] if a.ndim > 1 else len(a) // max(ncols, 1)
        self._check(self.lib.jy_pncount_converge_block(self.h, ncols, cols.ctypes.data, slot0, nslots, pa, pb, mem))

    def pncount_get(self, slots):
        s, ps, ms = _arg(slots, np.uint32)
        if ms == DEVICE:
            import torch
            out = torch.empty(len(s), dtype=torch.int64, device=s.device)
            self._check(self.lib.jy_pncount_get(self.h, len(s), ps, C.c_void_p(out.data_ptr()), DEVICE))
            return out
        out = np.empty(len(s), np.int64)
        self._check(self.lib.jy_pncount_get(self.h, len(s), ps, out.ctypes.data, HOST))
        return out

    def counter_export(self, ctype, ncols, slot0, nslots):
        nsigns = 1 if ctype == GCOUNT else 2
        out = np.zeros((nsigns, ncols, nslots), np.uint64)
        self._check(self.lib.jy_counter_export(self.h, ctype, ncols, slot0, nslots, out.ctypes.data))
        return out

    # -- counter write path (RepoGCOUNT.inc / RepoPNCOUNT.inc,dec) + flush --
    def counter_write(self, ctype, sign, col, slot, val):
        """n local writes under replica column `col`: s[slot][col] += val
        (wrapping); sign 0 = INC, 1 = DEC (PNCOUNT).  val: uint64 (an i64
        argument bit-cast, repo_pncount.pony:60,65)"""
        a, pa, ma = _arg(slot, np.uint32)
        b, pb, mb = _arg(val if _is_torch(val) else np.asarray(val).astype(np.uint64), np.uint64)
        mem = _same_mem(ma, mb)
        self._check(self.lib.jy_counter_write(self.h, ctype, sign, col, len(a), pa, pb, mem))

    def counter_deltas_size(self, ctype):
        n = C.c_uint64()
        self._check(self.lib.jy_counter_deltas_size(self.h, ctype, C.byref(n)))
        return n.value

    def counter_flush(self, ctype):
        """flush_deltas -> (slots u32[n], vals u64[nsigns][n], mask u32[n])"""
        nsigns = 1 if ctype == GCOUNT else 2
        cap = self.counter_deltas_size(ctype)
        slots = np.zeros(max(cap, 1), np.uint32)
        vals = np.zeros((nsigns, max(cap, 1)), np.uint64)
        mask = np.zeros(max(cap, 1), np.uint32)
        n = C.c_uint64()
        self._check(self.lib.jy_counter_flush(self.h, ctype, max(cap, 1), slots.ctypes.data, vals.ctypes.data,
                                              mask.ctypes.data, C.byref(n), HOST))
        k = n.value
        return slots[:k].copy(), vals[:, :k].copy(), mask[:k].copy()

    # -- TREG --------------------------------------------------------------
    def treg_converge(self, slot, ts, pre, lr):
        a, pa, ma = _arg(slot, np.uint32)
        b, pb, mb = _arg(ts, np.uint64)
        c, pc, mc = _arg(pre, np.uint64)
        d, pd, md = _arg(lr, np.uint64)
        mem = _same_mem(ma, mb, mc, md)
        self._check(self.lib.jy_treg_converge(self.h, len(a), pa, pb, pc, pd, mem))

    def treg_converge_block(self, slot0, ts, pre, lr):
        """a block batch (jy_treg_converge_block): entry i is slot slot0 + i"""
        b, pb, mb = _arg(ts, np.uint64)
        c, pc, mc = _arg(pre, np.uint64)
        d, pd, md = _arg(lr, np.uint64)
        mem = _same_mem(mb, mc, md)
        self._check(self.lib.jy_treg_converge_block(self.h, int(slot0), len(b), pb, pc, pd, mem))

    def treg_set(self, slot, ts, pre, lr):
        """local SETs (RepoTREG.set): state LWW + pending delta"""
        a, pa, ma = _arg(slot, np.uint32)
        b, pb, mb = _arg(ts, np.uint64)
        c, pc, mc = _arg(pre, np.uint64)
        d, pd, md = _arg(lr, np.uint64)
        mem = _same_mem(ma, mb, mc, md)
        self._check(self.lib.jy_treg_set(self.h, len(a), pa, pb, pc, pd, mem))

    def treg_deltas_size(self):
        n = C.c_uint64()
        self._check(self.lib.jy_treg_deltas_size(self.h, C.byref(n)))
        return n.value

    def treg_flush(self):
        """flush_deltas -> (slots, ts, pre, lr) of every pending key"""
        cap = max(self.treg_deltas_size(), 1)
        slots = np.zeros(cap, np.uint32)
        ts, pre, lr = (np.zeros(cap, np.uint64) for _ in range(3))
        n = C.c_uint64()
        self._check(self.lib.jy_treg_flush(self.h, cap, slots.ctypes.data, ts.ctypes.data, pre.ctypes.data,
                                           lr.ctypes.data, C.byref(n), HOST))
        k = n.value
        return slots[:k].copy(), ts[:k].copy(), pre[:k].copy(), lr[:k].copy()

    def treg_read(self, slots):
        s = np.ascontiguousarray(slots, np.uint32)
        n = len(s)
        ts, pre, lr = (np.empty(n, np.uint64) for _ in range(3))
        self._check(self.lib.jy_treg_read(self.h, n, s.ctypes.data, ts.ctypes.data, pre.ctypes.data, lr.ctypes.data))
        return ts, pre, lr

    # -- TLOG --------------------------------------------------------------
    def tlog_converge(self, slot, cutoff, ent_offs, ts, pre, lr):
        a, pa, ma = _arg(slot, np.uint32)
        b, pb, mb = _arg(cutoff, np.uint64)
        c, pc, mc = _arg(ent_offs, np.uint64)
        d, pd, md = _arg(ts, np.uint64)
        e, pe, me = _arg(pre, np.uint64)
        f, pf, mf = _arg(lr, np.uint64)
        mem = _same_mem(ma, mb, mc, md, me, mf)
        self._check(self.lib.jy_tlog_converge(self.h, len(a), pa, pb, pc, len(d), pd, pe, pf, mem))

    def tlog_write(self, ops, slot, ts=None, arg=None, pre=None, lr=None):
        """RepoTLOG.ins / trimat / trim / clr commands (jy_tlog_write), in order"""
        n = len(slot)
        cols = []
        for x, t in ((ops, np.uint8), (slot, np.uint32), (ts, np.uint64), (arg, np.uint64), (pre, np.uint64),
                     (lr, np.uint64)):
            cols.append(_arg(np.zeros(n, t) if x is None else x, t))
        mem = _same_mem(*[m for (_, _, m) in cols])
        (o, po, _), (s, ps, _), (a, pa, _), (b, pb, _), (c, pc, _), (d, pd, _) = cols
        self._check(self.lib.jy_tlog_write(self.h, n, po, ps, pa, pb, pc, pd, mem))

    def tlog_deltas_size(self):
        n = C.c_uint64()
        self._check(self.lib.jy_tlog_deltas_size(self.h, C.byref(n)))
        return n.value

    def tlog_flush(self):
        """flush_deltas -> (slots, cutoffs, offs, ts, pre, lr) of every pending key"""
        k, m = C.c_uint64(), C.c_uint64()
        z = np.zeros(1, np.uint64)
        self._check(self.lib.jy_tlog_flush(self.h, 0, 0, None, None, None, None, None, None, C.byref(k), C.byref(m),
                                           HOST))
        nk, ne = k.value, m.value
        slots = np.zeros(max(nk, 1), np.uint32)
        cut = np.zeros(max(nk, 1), np.uint64)
        offs = np.zeros(nk + 1, np.uint64)
        ts, pre, lr = (np.zeros(max(ne, 1), np.uint64) for _ in range(3))
        if nk:
            self._check(self.lib.jy_tlog_flush(self.h, nk, ne, slots.ctypes.data, cut.ctypes.data, offs.ctypes.data,
                                               ts.ctypes.data, pre.ctypes.data, lr.ctypes.data, C.byref(k),
                                               C.byref(m), HOST))
        del z
        return slots[:nk].copy(), cut[:nk].copy(), offs, ts[:ne].copy(), pre[:ne].copy(), lr[:ne].copy()

    def tlog_stats(self):
        """jy_tlog_stats: merges issued, spilled (re-merged after a compaction), compactions, pool capacity"""
        out = np.zeros(4, np.uint64)
        self._check(self.lib.jy_tlog_stats(self.h, out.ctypes.data))
        return dict(zip(("merges", "spills", "compactions", "pool_entries"), (int(x) for x in out)))

    def tlog_read(self, slots):
        """-> (cutoff[n], offs[n+1], ts, pre, lr) for host slots"""
        s = np.ascontiguousarray(slots, np.uint32)
        n = len(s)
        lens = np.empty(n, np.uint64)
        cut = np.empty(n, np.uint64)
        self._check(self.lib.jy_tlog_read_sizes(self.h, n, s.ctypes.data, lens.ctypes.data, cut.ctypes.data))
        offs = np.zeros(n + 1, np.uint64)
        offs[1:] = np.cumsum(lens, dtype=np.uint64)
        m = int(offs[-1])
        ts, pre, lr = (np.empty(max(m, 1), np.uint64) for _ in range(3))
        self._check(self.lib.jy_tlog_read(self.h, n, s.ctypes.data, offs.ctypes.data, ts.ctypes.data,
                                          pre.ctypes.data, lr.ctypes.data))
        return cut, offs, ts[:m], pre[:m], lr[:m]

    # -- UJSON -------------------------------------------------------------
    def ujson_converge(self, slot, el_offs, dots, elems, vv_offs, vv, cloud_offs, cloud):
        args = [_arg(x, t) for x, t in ((slot, np.uint32), (el_offs, np.uint64), (dots, np.uint64),
                                        (elems, np.uint64), (vv_offs, np.uint64), (vv, np.uint64),
                                        (cloud_offs, np.uint64), (cloud, np.uint64))]
        mem = _same_mem(*[m for (_, _, m) in args])
        (s, ps, _), (eo, peo, _), (d, pd, _), (e, pe, _), (vo, pvo, _), (v, pv, _), (co, pco, _), (c, pc, _) = args
        self._check(self.lib.jy_ujson_converge(self.h, len(s), ps, peo, len(d), pd, pe, pvo, len(v), pv,
                                               pco, len(c), pc, mem))

    def ujson_write(self, ops, slot, elem, col):
        """RepoUJSON.ins / rm / clr on opaque element handles (jy_ujson_write), in order"""
        n = len(slot)
        o, po, mo = _arg(ops, np.uint8)
        s, ps, ms = _arg(slot, np.uint32)
        e, pe, me = _arg(np.zeros(n, np.uint64) if elem is None else elem, np.uint64)
        self._check(self.lib.jy_ujson_write(self.h, n, po, ps, pe, int(col), _same_mem(mo, ms, me)))

    def ujson_deltas_size(self):
        n = C.c_uint64()
        self._check(self.lib.jy_ujson_deltas_size(self.h, C.byref(n)))
        return n.value

    def ujson_flush(self):
        """flush_deltas -> (slots, el_offs, dots, elems, vv[n][R], cloud_offs, cloud) of every pending doc"""
        k, me, mc = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._check(self.lib.jy_ujson_flush(self.h, 0, 0, 0, None, None, None, None, None, None, None,
                                            C.byref(k), C.byref(me), C.byref(mc), HOST))
        nk, ne, nc = k.value, me.value, mc.value
        R = self.ujson_columns
        slots = np.zeros(max(nk, 1), np.uint32)
        eo = np.zeros(nk + 1, np.uint64)
        co = np.zeros(nk + 1, np.uint64)
        dots, elems = np.zeros(max(ne, 1), np.uint64), np.zeros(max(ne, 1), np.uint64)
        cloud = np.zeros(max(nc, 1), np.uint64)
        vv = np.zeros((max(nk, 1), R), np.uint64)
        if nk:
            self._check(self.lib.jy_ujson_flush(self.h, nk, ne, nc, slots.ctypes.data, eo.ctypes.data,
                                                dots.ctypes.data, elems.ctypes.data, vv.ctypes.data, co.ctypes.data,
                                                cloud.ctypes.data, C.byref(k), C.byref(me), C.byref(mc), HOST))
        return slots[:nk].copy(), eo, dots[:ne].copy(), elems[:ne].copy(), vv[:nk].copy(), co, cloud[:nc].copy()

    UJSON_STATS = ("touched_el", "touched_cloud", "out_el", "out_cloud", "delta_el", "delta_cloud", "delta_docs",
                   "calls", "inplace_docs", "inplace_state_el", "inplace_state_cloud", "inplace_added_el",
                   "inplace_added_cloud", "inplace_folded", "promoted", "demoted")

    def ujson_stats(self):
        """cumulative converge counters (jy_ujson_stats_ext): dict of touched /
        written / delta sizes of the regular merge path, then the in-place
        layout's documents, their untouched state sizes, what they appended
        and folded, promotions and demotions"""
        out = np.zeros(16, np.uint64)
        self._check(self.lib.jy_ujson_stats_ext(self.h, out.ctypes.data))
        return {k: int(v) for k, v in zip(self.UJSON_STATS, out)}

    def ujson_set_inplace(self, min_elems):
        """promotion threshold of the UJSON in-place layout (0: no promotions)"""
        self._check(self.lib.jy_ujson_set_inplace(self.h, int(min_elems)))

    def ujson_read(self, slots):
        """-> (el_offs, dots, elems, vv[n][R], cloud_offs, cloud)"""
        s = np.ascontiguousarray(slots, np.uint32)
        n = len(s)
        nel = np.empty(n, np.uint64)
        ncl = np.empty(n, np.uint64)
        self._check(self.lib.jy_ujson_read_sizes(self.h, n, s.ctypes.data, nel.ctypes.data, ncl.ctypes.data))
        eo = np.zeros(n + 1, np.uint64)
        eo[1:] = np.cumsum(nel, dtype=np.uint64)
        co = np.zeros(n + 1, np.uint64)
        co[1:] = np.cumsum(ncl, dtype=np.uint64)
        me, mc = int(eo[-1]), int(co[-1])
        dots = np.empty(max(me, 1), np.uint64)
        elems = np.empty(max(me, 1), np.uint64)
        vv = np.empty((max(n, 1), self.ujson_columns), np.uint64)
        cloud = np.empty(max(mc, 1), np.uint64)
        self._check(self.lib.jy_ujson_read(self.h, n, s.ctypes.data, eo.ctypes.data, dots.ctypes.data,
                                           elems.ctypes.data, vv.ctypes.data, co.ctypes.data, cloud.ctypes.data))
        return eo, dots[:me], elems[:me], vv[:n], co, cloud[:mc]


def key_owner(key, nshards):
    lib = _lib.load()
    b = key.encode() if isinstance(key, str) else bytes(key)
    buf = C.create_string_buffer(b, len(b) or 1)
    return int(lib.jy_key_owner(buf, len(b), nshards))
