"""The node: every GPU of one Jylis node behind one C-ABI handle (jy_node_*,
include/jylis_gpu.h, jylis_amd/csrc/jy_node.hip).

One `converge_*` call replaces Database.converge_deltas ->
RepoManagerCore.converge_deltas (jylis/database.pony:50-51,
jylis/repo_manager.pony:92-93) for the whole node: the batch's keys are
hashed on the device, regrouped by owner shard, exchanged (RCCL over xGMI, or
device copies for the single-GPU tests), interned on their owner and merged
there -- all inside the library; the host only reads the per-owner counts
once.  This class is a thin ctypes caller (tests, bench); the Pony host binds
the same entry points.

The converge calls enqueue (round 5): host arrays are copied before a call
returns; device arrays (CUDA tensors) are read later by the node's worker,
so this wrapper keeps them alive until fence() / sync().  The engines
(`engines`, `engine()`) are shared with the worker: use them after sync(),
or inside `with node.locked():`.
"""
import contextlib
import ctypes as C
import threading

import numpy as np

from . import _lib
from ._lib import DEVICE, GCOUNT, HOST, PNCOUNT, TLOG, TREG, UJSON
from .engine import Engine, EngineError, _arg, _same_mem, pack_dot, DOT_SEQ_BITS

FABRICS = {"rccl": _lib.FABRIC_RCCL, "copy": _lib.FABRIC_COPY}


def unique_id():
    """a fresh ncclUniqueId (128 bytes) for a multi-process node: made by one
    process, shared with the others (e.g. torch.distributed broadcast)"""
    buf = (C.c_uint8 * 128)()
    rc = _lib.load().jy_node_unique_id(buf)
    if rc != 0:
        raise EngineError(rc, "ncclGetUniqueId failed")
    return bytes(buf)


def _seg_ids(offs):
    offs = np.asarray(offs, np.int64)
    return np.repeat(np.arange(len(offs) - 1), np.diff(offs))


class Node:
    """S key shards, one engine each.  `fabric` "copy": one process, every
    shard local, shards may share a GPU (tests); "rccl": an RCCL
    communicator, one GPU per shard -- all shards local (one process), or
    nlocal = 1 per process with a shared `uid` (unique_id())."""

    def __init__(self, nshards, fabric="copy", devices=None, nlocal=None, rank0=0, uid=None, counter_columns=16,
                 ujson_columns=16, key_capacity=1024, entry_capacity=8192, arena_capacity=1 << 16, flags=0):
        self.lib = _lib.load()
        nlocal = nshards if nlocal is None else nlocal
        if devices is None:
            devices = [0] * nlocal if fabric == "copy" else list(range(rank0, rank0 + nlocal))
        assert len(devices) == nlocal
        cfg = _lib.JyNodeConfig()
        cfg.nshards, cfg.nlocal, cfg.rank0, cfg.fabric = nshards, nlocal, rank0, FABRICS[fabric]
        for i, d in enumerate(devices):
            cfg.devices[i] = d
        if uid is not None:
            assert len(uid) == 128
            for i, b in enumerate(uid):
                cfg.unique_id[i] = b
        self.lib.jy_config_default(C.byref(cfg.engine))
        cfg.engine.counter_columns = counter_columns
        cfg.engine.ujson_columns = ujson_columns
        cfg.engine.flags = flags
        for t in range(5):
            cfg.engine.key_capacity[t] = key_capacity if np.isscalar(key_capacity) else key_capacity[t]
            cfg.engine.entry_capacity[t] = entry_capacity
            cfg.engine.arena_capacity[t] = arena_capacity
        h = C.c_void_p()
        rc = self.lib.jy_node_create(C.byref(cfg), C.byref(h))
        if rc != 0 or not h.value:
            raise EngineError(rc, "jy_node_create failed (no GPU, or RCCL could not form the communicator)")
        self.h = h
        self.S, self.nlocal, self.rank0 = nshards, nlocal, rank0
        self.devices = list(devices)
        self.ujson_columns = ujson_columns
        self.engines = [Engine.attach(self.lib.jy_node_engine(h, rank0 + i), devices[i], ujson_columns)
                        for i in range(nlocal)]
        self._held = []  # device inputs of queued calls (the worker reads them later)
        self._held_mu = threading.Lock()

    def close(self):
        if getattr(self, "h", None):
            for e in self.engines:
                e.close()
            self.lib.jy_node_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise EngineError(rc, self.lib.jy_node_last_error(self.h).decode(errors="replace"))

    def sync(self):
        """every queued call done, GPU work included"""
        with self._held_mu:
            held, self._held = self._held, []
        rc = self.lib.jy_node_sync(self.h)  # (drains every stream, failure or not)
        del held
        self._check(rc)

    def fence(self):
        """every queued call issued to the GPU streams (their device inputs are
        then ordered on the node's streams; still alive until the GPU ran)"""
        self._check(self.lib.jy_node_fence(self.h))

    @contextlib.contextmanager
    def locked(self, ctype=None):
        """exclusive use of the node's engines (jy_node_lock / jy_node_unlock);
        with a CRDT type, after that type's queued jobs only
        (jy_node_lock_type; NOFENCE: after none)"""
        rc = self.lib.jy_node_lock(self.h) if ctype is None else self.lib.jy_node_lock_type(self.h, int(ctype))
        try:
            self._check(rc)
            yield self
        finally:
            self.lib.jy_node_unlock(self.h)

    NOFENCE = -1

    def pending(self, ctype=-1):
        """jobs queued or running (of one CRDT type, or all)"""
        n = C.c_uint64()
        self._check(self.lib.jy_node_pending(self.h, int(ctype), C.byref(n)))
        return n.value

    def arena_gc(self, enable=True):
        """the worker reclaims TREG / TLOG arenas after their jobs (jy_node_arena_gc)"""
        self._check(self.lib.jy_node_arena_gc(self.h, 1 if enable else 0))

    def stats(self):
        out = np.zeros(5, np.uint64)
        self._check(self.lib.jy_node_stats(self.h, out.ctypes.data))
        return dict(zip(("keys_in", "keys_received", "bytes_sent", "bytes_received", "exchanges"),
                        (int(x) for x in out)))

    def shard_of(self, key):
        b = key.encode() if isinstance(key, str) else bytes(key)
        buf = C.create_string_buffer(b, len(b) or 1)
        return int(self.lib.jy_node_shard_of(self.h, buf, len(b)))

    def engine(self, shard):
        """the engine of a local shard (reads, local writes, flushes go to the key's owner)"""
        return self.engines[shard - self.rank0]

    def replica_col(self, rid):
        c = C.c_uint32()
        self._check(self.lib.jy_node_replica_col(self.h, C.c_uint64(int(rid) & (2**64 - 1)), C.byref(c)))
        return c.value

    def replica_cols(self, rids):
        return np.array([self.replica_col(r) for r in rids], dtype=np.uint16)

    # -- raw calls (numpy arrays: host; CUDA tensors: device) ----------------
    def _args(self, spec):
        out = [_arg(x, t) for x, t in spec]
        mem = _same_mem(*[m for (k, _, m) in out if k is not None])
        if mem == DEVICE:
            with self._held_mu:
                self._held.append([k for (k, _, _) in out])
        return out, mem

    def counter_converge(self, ctype, kb, ko, cell_offs, col, val, sign=None):
        (k, o, co, c, v, s), mem = self._args([(kb, np.uint8), (ko, np.uint64), (cell_offs, np.uint64),
                                               (col, np.uint16), (val, np.uint64), (sign, np.uint8)])
        n = len(o[0]) - 1
        self._check(self.lib.jy_node_counter_converge(self.h, ctype, n, k[1], o[1], co[1], s[1], c[1], v[1], mem))

    def treg_converge(self, kb, ko, ts, vb, vo):
        (k, o, t, b, bo), mem = self._args([(kb, np.uint8), (ko, np.uint64), (ts, np.uint64), (vb, np.uint8),
                                            (vo, np.uint64)])
        n = len(o[0]) - 1
        self._check(self.lib.jy_node_treg_converge(self.h, n, k[1], o[1], t[1], b[1], bo[1], mem))

    def tlog_converge(self, kb, ko, cutoff, ent_offs, ts, vb, vo):
        (k, o, cu, eo, t, b, bo), mem = self._args([(kb, np.uint8), (ko, np.uint64), (cutoff, np.uint64),
                                                    (ent_offs, np.uint64), (ts, np.uint64), (vb, np.uint8),
                                                    (vo, np.uint64)])
        n = len(o[0]) - 1
        self._check(self.lib.jy_node_tlog_converge(self.h, n, k[1], o[1], cu[1], eo[1], t[1], b[1], bo[1], mem))

    def ujson_converge(self, kb, ko, eo, dots, elems, vvo, vv, co, cloud):
        (k, o, a, d, e, b, v, c, cl), mem = self._args([(kb, np.uint8), (ko, np.uint64), (eo, np.uint64),
                                                        (dots, np.uint64), (elems, np.uint64), (vvo, np.uint64),
                                                        (vv, np.uint64), (co, np.uint64), (cloud, np.uint64)])
        n = len(o[0]) - 1
        self._check(self.lib.jy_node_ujson_converge(self.h, n, k[1], o[1], a[1], d[1], e[1], b[1], v[1], c[1], cl[1],
                                                    mem))

    def counter_converge_block(self, ctype, cols_all, slot0, nslots, vals_p, vals_n=None):
        """dense peer columns arriving mixed: vals_* CUDA tensors [nlocal][ncols][S][nslots];
        cols_all[r][c] = the column of shard r's c-th peer"""
        cols = np.ascontiguousarray(cols_all, np.uint16)
        ncols = cols.shape[1]
        with self._held_mu:
            self._held.append([vals_p, vals_n])
        self._check(self.lib.jy_node_counter_converge_block(
            self.h, ctype, ncols, cols.ctypes.data, slot0, nslots, C.c_void_p(vals_p.data_ptr()),
            None if vals_n is None else C.c_void_p(vals_n.data_ptr())))

    # -- oracle-format batch tables (the decoded MsgPushDeltas payload) -------
    def converge_table(self, ctype, t):
        """one decoded peer batch in oracle/oracle.py's table layout, as the
        GPU-backed Repo* would marshal it (jylis_amd/repo.py), in ONE node call"""
        kb = np.ascontiguousarray(t["key_bytes"], np.uint8)
        ko = np.ascontiguousarray(t["key_offs"], np.uint64)
        nk = len(ko) - 1
        if ctype == GCOUNT:
            ids = np.asarray(t["ids"], np.uint64)
            cols = self.replica_cols(ids.tolist()) if len(ids) else np.zeros(0, np.uint16)
            self.counter_converge(GCOUNT, kb, ko, np.asarray(t["offs"], np.uint64), cols,
                                  np.asarray(t["vals"], np.uint64))
        elif ctype == PNCOUNT:
            keys, signs, cols, vals = [], [], [], []
            for g, pre in enumerate(("p_", "n_")):
                ids = np.asarray(t[pre + "ids"], np.uint64)
                keys.append(_seg_ids(t[pre + "offs"]))
                signs.append(np.full(len(ids), g, np.uint8))
                cols.append(self.replica_cols(ids.tolist()) if len(ids) else np.zeros(0, np.uint16))
                vals.append(np.asarray(t[pre + "vals"], np.uint64))
            key = np.concatenate(keys)
            order = np.argsort(key, kind="stable")  # every key's cells together
            offs = np.zeros(nk + 1, np.uint64)
            offs[1:] = np.cumsum(np.bincount(key, minlength=nk), dtype=np.uint64)
            self.counter_converge(PNCOUNT, kb, ko, offs, np.concatenate(cols)[order], np.concatenate(vals)[order],
                                  sign=np.concatenate(signs)[order])
        elif ctype == TREG:
            self.treg_converge(kb, ko, np.asarray(t["ts"], np.uint64), np.asarray(t["val_bytes"], np.uint8),
                               np.asarray(t["val_offs"], np.uint64))
        elif ctype == TLOG:
            self.tlog_converge(kb, ko, np.asarray(t["cutoff"], np.uint64), np.asarray(t["ent_offs"], np.uint64),
                               np.asarray(t["ts"], np.uint64), np.asarray(t["val_bytes"], np.uint8),
                               np.asarray(t["val_offs"], np.uint64))
        elif ctype == UJSON:
            self.ujson_converge(*self.ujson_args(t))
        else:
            raise ValueError(f"unknown CRDT type {ctype}")

    def ujson_args(self, t):
        """a UJSON batch table -> the node call's arrays (key bytes, key offsets,
        element offsets, dots, elements, vv offsets, vv, cloud offsets, cloud):
        replica ids to node columns, every document's dots ascending"""
        def packed(ids, seqs, offs, *payload):
            ids = np.asarray(ids, np.uint64)
            seqs = np.asarray(seqs, np.uint64)
            if len(seqs) and (seqs >> np.uint64(DOT_SEQ_BITS)).any():
                raise ValueError("dot sequence numbers must stay below 2^48")
            cols = self.replica_cols(ids.tolist()).astype(np.uint64) if len(ids) else np.zeros(0, np.uint64)
            p = pack_dot(cols, seqs)
            order = np.lexsort((p, _seg_ids(offs)))  # ascending dots per document
            return (p[order],) + tuple(np.asarray(x, np.uint64)[order] for x in payload)
        kb = np.ascontiguousarray(t["key_bytes"], np.uint8)
        ko = np.ascontiguousarray(t["key_offs"], np.uint64)
        eo, vo, co = (np.asarray(t[k], np.uint64) for k in ("el_offs", "vv_offs", "cloud_offs"))
        dots, elems = packed(t["dot_ids"], t["dot_seqs"], eo, t["elems"])
        (vv,) = packed(t["vv_ids"], t["vv_seqs"], vo)
        (cloud,) = packed(t["cloud_ids"], t["cloud_seqs"], co)
        return kb, ko, eo, dots, elems, vo, vv, co, cloud
