"""GPU-backed Repo* mirrors: the host side of the drop-in boundary.

Each class stands where the reference's RepoGCOUNT / RepoPNCOUNT / RepoTREG /
RepoTLOG / RepoUJSON stand (jylis/repo_*.pony) and exposes the same converge
surface as RepoAny (jylis/repo_manager.pony:5-10):

  converge(key, delta)        one (key, delta) pair   (repo_*.pony `converge`)
  converge_deltas(batch)      a whole decoded batch   (repo_manager.pony:92-93)

converge() queues the pair; the queue is marshalled into structure-of-arrays
and merged in ONE engine call (converge_deltas) by the repo's next entry
point -- deltas_size() on the heartbeat, flush_deltas(), reads, writes -- or
at DRAIN_BOUND pairs.  That is the change INTEGRATION.md describes for the
Pony host (pony/jylis_gpu/*.pony `_drain`).  Batches use the table layout of
oracle/oracle.py (key_bytes/key_offs + per-type CSR columns), the decoded
form of a MsgPushDeltas payload (jylis/msg.pony:20-24).

Error behaviour follows the reference: a batch of the wrong type is ignored
(the `delta' as T box` downcast fails inside `try ... end`,
repo_gcount.pony:50-51).
"""
import numpy as np

from . import engine as E
from ._lib import GCOUNT, PNCOUNT, TLOG, TREG, UJSON


def _keys_of(table):
    return np.ascontiguousarray(table["key_bytes"], np.uint8), np.ascontiguousarray(table["key_offs"], np.uint64)


# Queued (key, delta) pairs that force a drain without waiting for the next
# entry point: bounds the host memory a read-idle replica holds between
# heartbeats and the work one drain call does.
DRAIN_BOUND = 1 << 16


def concat_rows(pairs):
    """[(key bytes, one-key delta table without key columns)] -> one batch
    table: the marshalling of an Array[(String, Any box)] into SoA.  Every
    `*offs` column is an offsets array (CSR, possibly nested: TLOG val_offs
    counts bytes per entry) and is rebased; every other column concatenates."""
    keys = [k for k, _ in pairs]
    out = {"key_bytes": np.frombuffer(b"".join(keys), np.uint8).copy(),
           "key_offs": np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)}
    for name in pairs[0][1]:
        parts = [np.asarray(r[name]) for _, r in pairs]
        if name.endswith("offs"):
            res, base = [np.zeros(1, np.uint64)], 0
            for p in parts:
                p = p.astype(np.uint64)
                res.append(p[1:] - p[0] + np.uint64(base))
                base += int(p[-1] - p[0])
            out[name] = np.concatenate(res)
        else:
            out[name] = np.concatenate(parts)
    return out


class _GpuRepo:
    ctype = None

    def __init__(self, eng, identity=None):
        self.eng = eng
        self.identity = identity  # RepoXXX.create(identity') (repo_manager.pony:6)
        # slot -> key bytes (the engine interns; the host keeps names for reads),
        # one list per engine and type: every repo over the engine shares its slots
        self.names = eng.__dict__.setdefault("_slot_names", {}).setdefault(self.ctype, [])
        self._in = []  # queued (key, delta) pairs of RepoAny.converge

    def _intern(self, table):
        kb, ko = _keys_of(table)
        self._sync_names()
        before = self.eng.nkeys(self.ctype)
        slots = self.eng.intern(self.ctype, (kb, ko))
        after = self.eng.nkeys(self.ctype)
        if after > before:
            fresh = np.nonzero(slots >= before)[0]
            order = np.argsort(slots[fresh], kind="stable")
            seen = set()
            for i in fresh[order]:
                s = int(slots[i])
                if s not in seen:
                    seen.add(s)
                    self.names.append(bytes(kb[ko[i]:ko[i + 1]]))
        return slots

    def _sync_names(self):
        """names of keys interned on the device (route.KeyResolver, Engine.intern_device)
        fetched from the directory (jy_keys_export)"""
        n = self.eng.nkeys(self.ctype)
        if len(self.names) < n:
            self.names.extend(self.eng.key_names(self.ctype, len(self.names), n - len(self.names)))

    def slots_of(self, keys):
        self._drain()
        return self.eng.lookup(self.ctype, keys)

    def converge(self, key, delta_row):
        """RepoAny.converge(key, delta') (repo_manager.pony:10), which
        RepoManagerCore.converge_deltas calls once per pair (:92-93).  The pair
        (delta = a one-key table without key columns) is queued; every queued
        pair is merged in ONE engine call (converge_deltas) by the next entry
        point -- reads, writes, deltas_size (the heartbeat's call,
        repo_manager.pony:86-90), flush_deltas -- or once DRAIN_BOUND pairs
        wait, so a replica that only receives still applies them every tick."""
        kb = key.encode() if isinstance(key, str) else bytes(key)
        self._in.append((kb, delta_row))
        if len(self._in) >= DRAIN_BOUND:
            self._drain()

    def _drain(self):
        if self._in:
            pairs, self._in = self._in, []
            self.converge_deltas(concat_rows(pairs))

    def pending_pairs(self):
        """queued converge pairs not yet handed to the engine"""
        return len(self._in)

    def _sorted_slots(self):
        self._drain()
        self._sync_names()
        order = sorted(range(len(self.names)), key=lambda s: self.names[s])
        return np.array(order, dtype=np.uint32)

    def _keys_table(self, slots):
        self._sync_names()
        names = [self.names[s] for s in slots]
        kb, ko = E.encode_keys(names)
        return {"key_bytes": kb, "key_offs": ko}


class RepoGCOUNT(_GpuRepo):
    """repo_gcount.pony: GCounter per key, per-replica max-merge."""
    ctype = GCOUNT

    def converge_deltas(self, batch, ctype=GCOUNT):
        if ctype != self.ctype:
            return
        kb, ko = _keys_of(batch)
        offs = np.asarray(batch["offs"], np.uint64)
        ids = np.asarray(batch["ids"], np.uint64)
        if len(ids) == 0:
            self._intern(batch)  # converge creates the keys (_data_for) even with no cells
            return
        cols = self.eng.replica_cols(ids.tolist())
        nk = len(ko) - 1
        cell_key = np.repeat(np.arange(nk, dtype=np.uint32), np.diff(offs).astype(np.int64))
        # one call: the keys interned on the device feed the merge (no slot round trip);
        # the host learns new keys' names lazily (_sync_names)
        self.eng.counter_converge_keys(GCOUNT, (kb, ko), cols, np.asarray(batch["vals"], np.uint64), cell_key=cell_key)

    def get(self, keys):
        """GCOUNT GET (repo_gcount.pony:53-55): missing key -> 0"""
        slots = self.slots_of(keys)
        out = np.zeros(len(slots), np.uint64)
        have = slots != E._lib.JY_NO_SLOT
        if have.any():
            out[have] = self.eng.gcount_get(slots[have])
        return out

    def state(self):
        """oracle-format state table (absent replica entries == 0 are dropped)"""
        slots = self._sorted_slots()
        t = self._keys_table(slots)
        t.update(_counter_table(self.eng, GCOUNT, slots, "", 0))
        return t

    # -- local writes + flush_deltas (on the GPU: jy_counter_write / _flush) --
    def inc(self, keys, vals, identity):
        """GCOUNT INC for a batch (repo_gcount.pony:57-60), keys may repeat:
        s[key][identity] += v (wrapping); the pending delta records the total"""
        _counter_write(self, keys, vals, identity, 0)

    def deltas_size(self):
        self._drain()
        return self.eng.counter_deltas_size(self.ctype)

    def flush_deltas(self, identity=None):
        """flush_deltas (repo_gcount.pony:18-23) -> oracle-format batch table"""
        return _counter_flush(self, identity, ("",))


class RepoPNCOUNT(_GpuRepo):
    """repo_pncount.pony: PNCounter per key (two GCounters)."""
    ctype = PNCOUNT

    def converge_deltas(self, batch, ctype=PNCOUNT):
        if ctype != self.ctype:
            return
        kb, ko = _keys_of(batch)
        nk = len(ko) - 1
        keys, signs, cols, vals = [], [], [], []
        for sg, pre in enumerate(("p_", "n_")):
            offs = np.asarray(batch[pre + "offs"], np.uint64)
            ids = np.asarray(batch[pre + "ids"], np.uint64)
            if len(ids) == 0:
                continue
            keys.append(np.repeat(np.arange(nk, dtype=np.uint32), np.diff(offs).astype(np.int64)))
            signs.append(np.full(len(ids), sg, np.uint8))
            cols.append(self.eng.replica_cols(ids.tolist()))
            vals.append(np.asarray(batch[pre + "vals"], np.uint64))
        if not keys:
            self._intern(batch)  # converge creates the keys (_data_for) even with no cells
            return
        self.eng.counter_converge_keys(PNCOUNT, (kb, ko), np.concatenate(cols), np.concatenate(vals),
                                       cell_key=np.concatenate(keys), sign=np.concatenate(signs))

    def get(self, keys):
        """PNCOUNT GET (repo_pncount.pony:55-57): (sum P - sum N) as i64, missing -> 0"""
        slots = self.slots_of(keys)
        out = np.zeros(len(slots), np.int64)
        have = slots != E._lib.JY_NO_SLOT
        if have.any():
            out[have] = self.eng.pncount_get(slots[have])
        return out

    def state(self):
        slots = self._sorted_slots()
        t = self._keys_table(slots)
        t.update(_counter_table(self.eng, PNCOUNT, slots, "p_", 0))
        t.update(_counter_table(self.eng, PNCOUNT, slots, "n_", 1))
        return t

    def inc(self, keys, vals, identity):
        """PNCOUNT INC (repo_pncount.pony:59-62): i64 values bit-cast to u64"""
        _counter_write(self, keys, vals, identity, 0)

    def dec(self, keys, vals, identity):
        """PNCOUNT DEC (repo_pncount.pony:64-67)"""
        _counter_write(self, keys, vals, identity, 1)

    def deltas_size(self):
        self._drain()
        return self.eng.counter_deltas_size(self.ctype)

    def flush_deltas(self, identity=None):
        return _counter_flush(self, identity, ("p_", "n_"))


def _counter_write(repo, keys, vals, identity, sign):
    repo._drain()
    kb, ko = E.encode_keys(keys)
    slots = repo._intern({"key_bytes": kb, "key_offs": ko})
    v = np.asarray(vals)
    v = v.astype(np.int64).view(np.uint64) if v.dtype.kind == "i" else v.astype(np.uint64)
    repo.eng.counter_write(repo.ctype, sign, repo.eng.replica_col(identity), slots, v)


def _counter_flush(repo, identity, prefixes):
    repo._drain()
    identity = repo.identity if identity is None else identity
    slots, vals, mask = repo.eng.counter_flush(repo.ctype)
    t = repo._keys_table(slots)
    rid = np.uint64(int(identity) & (2**64 - 1))
    for g, pre in enumerate(prefixes):
        has = ((mask >> g) & 1).astype(bool)
        offs = np.zeros(len(slots) + 1, np.uint64)
        offs[1:] = np.cumsum(has, dtype=np.uint64)
        t[pre + "offs"] = offs
        t[pre + "ids"] = np.full(int(has.sum()), rid, np.uint64)
        t[pre + "vals"] = vals[g][has]
    return t


def _counter_table(eng, ctype, slots, prefix, sign):
    ncols = eng.replica_count()
    nk = eng.nkeys(ctype)
    if nk == 0 or ncols == 0:
        return {prefix + "offs": np.zeros(len(slots) + 1, np.uint64), prefix + "ids": np.zeros(0, np.uint64),
                prefix + "vals": np.zeros(0, np.uint64)}
    dump = eng.counter_export(ctype, ncols, 0, nk)[sign]  # [col][slot]
    ids_of_col = np.array([eng.replica_id(c) for c in range(ncols)], np.uint64)
    order = np.argsort(ids_of_col, kind="stable")
    offs = [0]
    ids, vals = [], []
    for s in slots:
        col_vals = dump[order, s]
        nz = col_vals != 0
        ids.append(ids_of_col[order][nz])
        vals.append(col_vals[nz])
        offs.append(offs[-1] + int(nz.sum()))
    return {prefix + "offs": np.array(offs, np.uint64),
            prefix + "ids": np.concatenate(ids) if ids else np.zeros(0, np.uint64),
            prefix + "vals": np.concatenate(vals) if vals else np.zeros(0, np.uint64)}


class _ArenaGC:
    """collect the value arena when dead bytes outnumber live ones (after a
    call that consumed every handle it packed)"""
    _arena_live = 0

    def _maybe_collect(self):
        if getattr(self.eng, "_route_holds", None):
            return  # a router's rounds in flight still read handles of this arena (route.py)
        n, _ = self.eng.arena_usage(self.ctype)
        if n > 2 * self._arena_live + (1 << 20):
            self._arena_live = self.eng.arena_collect(self.ctype)


class RepoTREG(_ArenaGC, _GpuRepo):
    """repo_treg.pony: TRegString per key, LWW by (timestamp, value)."""
    ctype = TREG

    def converge_deltas(self, batch, ctype=TREG):
        if ctype != self.ctype:
            return
        slots = self._intern(batch)
        if len(slots) == 0:
            return
        pre, lr = self.eng.pack_values(TREG, (batch["val_bytes"], batch["val_offs"]))
        self.eng.treg_converge(slots, np.asarray(batch["ts"], np.uint64), pre, lr)
        self._maybe_collect()

    def get(self, key):
        """TREG GET (repo_treg.pony:54-63): (value, ts), or None if never touched"""
        s = int(self.slots_of([key])[0])
        if s == E._lib.JY_NO_SLOT:
            return None
        ts, pre, lr = self.eng.treg_read(np.array([s], np.uint32))
        return self.eng.value_bytes(TREG, pre[0], lr[0]), int(ts[0])

    def state(self):
        slots = self._sorted_slots()
        t = self._keys_table(slots)
        ts, pre, lr = self.eng.treg_read(slots) if len(slots) else (np.zeros(0, np.uint64),) * 3
        vals = [self.eng.value_bytes(TREG, p, l) for p, l in zip(pre, lr)]
        vb, vo = E.encode_keys(vals)
        t.update({"ts": ts, "val_bytes": vb, "val_offs": vo})
        return t

    # -- local writes + flush_deltas (jy_treg_set / _flush) --
    def set(self, keys, values, ts):
        """TREG SET for a batch (repo_treg.pony:65-68); keys may repeat (in order)"""
        self._drain()
        kb, ko = E.encode_keys(keys)
        slots = self._intern({"key_bytes": kb, "key_offs": ko})
        pre, lr = self.eng.pack_values(TREG, list(values))
        self.eng.treg_set(slots, np.asarray(ts, np.uint64), pre, lr)
        self._maybe_collect()

    def deltas_size(self):
        self._drain()
        return self.eng.treg_deltas_size()

    def flush_deltas(self):
        """flush_deltas (repo_treg.pony:18-22) -> oracle-format batch table"""
        self._drain()
        slots, ts, pre, lr = self.eng.treg_flush()
        t = self._keys_table(slots)
        vb, vo = E.encode_keys([self.eng.value_bytes(TREG, p, l) for p, l in zip(pre, lr)])
        t.update({"ts": ts, "val_bytes": vb, "val_offs": vo})
        return t


class RepoTLOG(_ArenaGC, _GpuRepo):
    """repo_tlog.pony: TLog[String] per key (sorted log with grow-only cutoff)."""
    ctype = TLOG

    def converge_deltas(self, batch, ctype=TLOG):
        if ctype != self.ctype:
            return
        slots = self._intern(batch)
        if len(slots) == 0:
            return
        pre, lr = self.eng.pack_values(TLOG, (batch["val_bytes"], batch["val_offs"]))
        self.eng.tlog_converge(slots, np.asarray(batch["cutoff"], np.uint64), np.asarray(batch["ent_offs"], np.uint64),
                               np.asarray(batch["ts"], np.uint64), pre, lr)
        self._maybe_collect()

    def get(self, key, count=None):
        """TLOG GET key [count] (repo_tlog.pony:69-83): [(value, ts)], newest first"""
        s = int(self.slots_of([key])[0])
        if s == E._lib.JY_NO_SLOT:
            return []
        cut, offs, ts, pre, lr = self.eng.tlog_read(np.array([s], np.uint32))
        n = len(ts) if count is None else min(count, len(ts))
        return [(self.eng.value_bytes(TLOG, pre[j], lr[j]), int(ts[j])) for j in range(n)]

    def size(self, key):
        s = int(self.slots_of([key])[0])
        return 0 if s == E._lib.JY_NO_SLOT else len(self.eng.tlog_read(np.array([s], np.uint32))[2])

    def cutoff(self, key):
        s = int(self.slots_of([key])[0])
        return 0 if s == E._lib.JY_NO_SLOT else int(self.eng.tlog_read(np.array([s], np.uint32))[0][0])

    def state(self):
        slots = self._sorted_slots()
        t = self._keys_table(slots)
        if len(slots) == 0:
            t.update({"cutoff": np.zeros(0, np.uint64), "ent_offs": np.zeros(1, np.uint64),
                      "ts": np.zeros(0, np.uint64), "val_bytes": np.zeros(0, np.uint8),
                      "val_offs": np.zeros(1, np.uint64)})
            return t
        cut, offs, ts, pre, lr = self.eng.tlog_read(slots)
        vals = [self.eng.value_bytes(TLOG, p, l) for p, l in zip(pre, lr)]
        vb, vo = E.encode_keys(vals)
        t.update({"cutoff": cut, "ent_offs": offs, "ts": ts, "val_bytes": vb, "val_offs": vo})
        return t


    # -- local writes + flush_deltas (jy_tlog_write / _flush) --
    def write(self, cmds):
        """a batch of TLOG write commands, applied in order (keys may repeat):
        ("INS", key, value, ts) | ("TRIMAT", key, ts) | ("TRIM", key, count) |
        ("CLR", key)  -- repo_tlog.pony:85-111"""
        self._drain()
        if not cmds:
            return
        codes = {"INS": E._lib.TLOG_INS, "TRIMAT": E._lib.TLOG_TRIMAT, "TRIM": E._lib.TLOG_TRIM,
                 "CLR": E._lib.TLOG_CLR}
        kb, ko = E.encode_keys([c[1] for c in cmds])
        slots = self._intern({"key_bytes": kb, "key_offs": ko})
        n = len(cmds)
        ops = np.array([codes[c[0]] for c in cmds], np.uint8)
        ts = np.zeros(n, np.uint64)
        arg = np.zeros(n, np.uint64)
        vals = [b""] * n
        for i, c in enumerate(cmds):
            if c[0] == "INS":
                vals[i] = c[2]
                ts[i] = c[3]
            elif c[0] == "TRIMAT":
                ts[i] = c[2]
            elif c[0] == "TRIM":
                arg[i] = c[2]
        pre, lr = self.eng.pack_values(TLOG, vals)
        self.eng.tlog_write(ops, slots, ts, arg, pre, lr)
        self._maybe_collect()

    def ins(self, keys, values, ts):
        self.write([("INS", k, v, int(t)) for k, v, t in zip(keys, values, ts)])

    def trimat(self, keys, ts):
        self.write([("TRIMAT", k, int(t)) for k, t in zip(keys, ts)])

    def trim(self, keys, counts):
        self.write([("TRIM", k, int(c)) for k, c in zip(keys, counts)])

    def clr(self, keys):
        self.write([("CLR", k) for k in keys])

    def deltas_size(self):
        self._drain()
        return self.eng.tlog_deltas_size()

    def flush_deltas(self):
        """flush_deltas (repo_tlog.pony:21-25) -> oracle-format batch table"""
        self._drain()
        slots, cut, offs, ts, pre, lr = self.eng.tlog_flush()
        t = self._keys_table(slots)
        vb, vo = E.encode_keys([self.eng.value_bytes(TLOG, p, l) for p, l in zip(pre, lr)])
        t.update({"cutoff": cut, "ent_offs": offs, "ts": ts, "val_bytes": vb, "val_offs": vo})
        return t


def _seg_ids(offs):
    offs = np.asarray(offs, np.int64)
    return np.repeat(np.arange(len(offs) - 1), np.diff(offs))


class RepoUJSON(_GpuRepo):
    """repo_ujson.pony: UJSON per key (dot kernel over interned (path, value) leaves)."""
    ctype = UJSON

    def _pack(self, ids, seqs):
        ids = np.asarray(ids, np.uint64)
        cols = self.eng.replica_cols(ids.tolist()).astype(np.uint64) if len(ids) else np.zeros(0, np.uint64)
        if len(seqs) and (np.asarray(seqs, np.uint64) >> np.uint64(E.DOT_SEQ_BITS)).any():
            raise ValueError("dot sequence numbers must stay below 2^48")
        return E.pack_dot(cols, seqs)

    @staticmethod
    def _sort_segments(offs, packed, *payload):
        seg = _seg_ids(offs)
        order = np.lexsort((packed, seg))
        return (packed[order],) + tuple(np.asarray(p)[order] for p in payload)

    def converge_deltas(self, batch, ctype=UJSON):
        if ctype != self.ctype:
            return
        slots = self._intern(batch)
        if len(slots) == 0:
            return
        eo, vo, co = (np.asarray(batch[k], np.uint64) for k in ("el_offs", "vv_offs", "cloud_offs"))
        dots, elems = self._sort_segments(eo, self._pack(batch["dot_ids"], batch["dot_seqs"]),
                                          np.asarray(batch["elems"], np.uint64))
        (vv,) = self._sort_segments(vo, self._pack(batch["vv_ids"], batch["vv_seqs"]))
        (cloud,) = self._sort_segments(co, self._pack(batch["cloud_ids"], batch["cloud_seqs"]))
        self.eng.ujson_converge(slots, eo, dots, elems, vo, vv, co, cloud)

    # -- local writes on opaque elements + flush_deltas (jy_ujson_write / _flush) --
    def write(self, cmds, identity):
        """("INS", key, elem) | ("RM", key, elem) | ("CLR", key) | ("TOUCH", key),
        applied in order; RM / CLR of a key that does not exist do nothing
        (repo_ujson.pony:86,108); TOUCH creates the key and its delta and
        changes nothing (SET of an empty node, a path-scoped CLR that matches
        nothing): an RM of handle 0, which no element holds"""
        self._drain()
        codes = {"INS": E._lib.UJSON_INS, "RM": E._lib.UJSON_RM, "CLR": E._lib.UJSON_CLR,
                 "TOUCH": E._lib.UJSON_RM}
        live = []
        for c in cmds:
            if c[0] in ("INS", "TOUCH"):
                live.append(c)
            else:
                s = int(self.slots_of([c[1]])[0])
                if s != E._lib.JY_NO_SLOT:
                    live.append(c)
                elif any(d[0] in ("INS", "TOUCH") and d[1] == c[1] for d in live):
                    live.append(c)  # created earlier in this batch
        if not live:
            return
        kb, ko = E.encode_keys([c[1] for c in live])
        slots = self._intern({"key_bytes": kb, "key_offs": ko})
        ops = np.array([codes[c[0]] for c in live], np.uint8)
        elems = np.array([c[2] if c[0] in ("INS", "RM") else 0 for c in live], np.uint64)
        col = int(self.eng.replica_cols([identity])[0])
        self.eng.ujson_write(ops, slots, elems, col)

    def deltas_size(self):
        self._drain()
        return self.eng.ujson_deltas_size()

    def flush_deltas(self):
        """flush_deltas (repo_ujson.pony:22-26) -> oracle-format batch table"""
        self._drain()
        slots, eo, dots, elems, vv, co, cloud = self.eng.ujson_flush()
        return self._docs_table(slots, eo, dots, elems, vv, co, cloud)

    def elements(self, key):
        """the observable element set of a doc (what GET renders, repo_ujson.pony:68-72)"""
        s = int(self.slots_of([key])[0])
        if s == E._lib.JY_NO_SLOT:
            return set()
        return set(int(x) for x in self.eng.ujson_read(np.array([s], np.uint32))[2])

    def state(self):
        slots = self._sorted_slots()
        if len(slots) == 0:
            return self._docs_table(slots, None, None, None, None, None, None)
        eo, dots, elems, vv, co, cloud = self.eng.ujson_read(slots)
        return self._docs_table(slots, eo, dots, elems, vv, co, cloud)

    def _docs_table(self, slots, eo, dots, elems, vv, co, cloud):
        """device doc rows -> oracle-format table (replica ids, sorted segments)"""
        t = self._keys_table(slots)
        n = len(slots)
        out = {k: [] for k in ("dot_ids", "dot_seqs", "elems", "vv_ids", "vv_seqs", "cloud_ids", "cloud_seqs")}
        eoffs, voffs, coffs = [0], [0], [0]
        if n:
            R = vv.shape[1]
            ids = np.array([self.eng.replica_id(c) for c in range(self.eng.replica_count())] or [0], np.uint64)
            for i in range(n):
                c, q = E.unpack_dot(dots[eo[i]:eo[i + 1]])
                di = ids[c]
                order = np.lexsort((q, di))
                out["dot_ids"].append(di[order])
                out["dot_seqs"].append(q[order])
                out["elems"].append(elems[eo[i]:eo[i + 1]][order])
                eoffs.append(eoffs[-1] + len(order))
                nz = np.nonzero(vv[i])[0]
                vi = ids[nz] if len(nz) else np.zeros(0, np.uint64)
                order = np.argsort(vi, kind="stable")
                out["vv_ids"].append(vi[order])
                out["vv_seqs"].append(vv[i][nz][order])
                voffs.append(voffs[-1] + len(nz))
                c, q = E.unpack_dot(cloud[co[i]:co[i + 1]])
                ci = ids[c]
                order = np.lexsort((q, ci))
                out["cloud_ids"].append(ci[order])
                out["cloud_seqs"].append(q[order])
                coffs.append(coffs[-1] + len(order))
                assert R == self.eng.ujson_columns
        for k, v in out.items():
            t[k] = np.concatenate(v).astype(np.uint64) if v else np.zeros(0, np.uint64)
        t["el_offs"] = np.array(eoffs, np.uint64)
        t["vv_offs"] = np.array(voffs, np.uint64)
        t["cloud_offs"] = np.array(coffs, np.uint64)
        return t


REPOS = {GCOUNT: RepoGCOUNT, PNCOUNT: RepoPNCOUNT, TREG: RepoTREG, TLOG: RepoTLOG, UJSON: RepoUJSON}
