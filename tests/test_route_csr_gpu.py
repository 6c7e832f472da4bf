"""Routing TLOG logs and UJSON documents on the GPU (k_route_csr.hip): the
partition kernels, the fixed-capacity runs with holes, the all-to-all
(route.LocalFabric: S engines on cuda:0) and the per-source routed merge.

After routing, the union of the shards must equal ONE oracle repo that
converged every ingested batch (repo_tlog.pony:66-67, repo_ujson.pony:65-66)
-- bit-exact, including keys that several sources send in one step,
overflowing runs (drain rounds), long TLOG values whose bytes travel in their
own section, and empty batches."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# "async": every async all-to-all runs on a side stream behind a spin delay
# (RCCL's ordering contract: the runs are valid only after wait())
FABRIC = {"sync": {}, "async": {"async_copies": True, "delay_cycles": 400000}}

TLOG_CSRS = [("ent_offs", ["ts"], True)]
UJSON_CSRS = [("el_offs", ["dot_ids", "dot_seqs", "elems"], False), ("vv_offs", ["vv_ids", "vv_seqs"], False),
              ("cloud_offs", ["cloud_ids", "cloud_seqs"], False)]


def _ranges(offs, idx):
    offs = np.asarray(offs, np.int64)
    lo, hi = offs[idx], offs[idx + 1]
    cnt = hi - lo
    noffs = np.zeros(len(idx) + 1, np.int64)
    noffs[1:] = np.cumsum(cnt)
    ent = np.repeat(lo - noffs[:-1], cnt) + np.arange(int(noffs[-1]), dtype=np.int64)
    return noffs.astype(np.uint64), ent


def pick_rows(t, idx, csrs, per_key=()):
    """the table of the keys `idx` (in that order)"""
    from jylis_amd.route import _pick_keys
    from jylis_amd.synth import gather_bytes
    idx = np.asarray(idx, np.int64)
    out = {}
    out["key_bytes"], out["key_offs"] = _pick_keys(np.asarray(t["key_bytes"], np.uint8),
                                                   np.asarray(t["key_offs"], np.uint64), idx)
    for k in per_key:
        out[k] = np.asarray(t[k])[idx]
    for ok, cols, vals in csrs:
        out[ok], ent = _ranges(t[ok], idx)
        for c in cols:
            out[c] = np.asarray(t[c])[ent]
        if vals:
            out["val_bytes"], out["val_offs"] = gather_bytes(t["val_bytes"], t["val_offs"], ent)
    return out


def _dev(a):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype in (np.uint64, np.int64):
        return torch.from_numpy(a.astype(np.uint64).view(np.int64)).to("cuda:0")
    return torch.from_numpy(a.astype(np.uint32).view(np.int32)).to("cuda:0")


def tlog_device_batch(eng, own, slot, t):
    """TlogRouter batch of an oracle-format TLOG table (values packed on `eng`)"""
    from jylis_amd._lib import TLOG
    from jylis_amd.route import long_bytes
    pre, lr = eng.pack_values(TLOG, (t["val_bytes"], t["val_offs"]))
    return (_dev(own), _dev(slot), _dev(np.asarray(t["cutoff"], np.uint64)), _dev(np.asarray(t["ent_offs"], np.uint64)),
            _dev(np.asarray(t["ts"], np.uint64)), _dev(pre), _dev(lr), long_bytes(lr))


def ujson_device_batch(repo, own, slot, t):
    """UjsonRouter batch of an oracle-format UJSON table (dots packed with the
    engine's replica columns, sorted per document)"""
    eo, vo, co = (np.asarray(t[k], np.uint64) for k in ("el_offs", "vv_offs", "cloud_offs"))
    dots, elems = repo._sort_segments(eo, repo._pack(t["dot_ids"], t["dot_seqs"]), np.asarray(t["elems"], np.uint64))
    (vv,) = repo._sort_segments(vo, repo._pack(t["vv_ids"], t["vv_seqs"]))
    (cloud,) = repo._sort_segments(co, repo._pack(t["cloud_ids"], t["cloud_seqs"]))
    return tuple(_dev(x) for x in (own, slot, eo, dots, elems, vo, vv, co, cloud))


class CsrNode:
    """S shards on one GPU; the control plane's role (owner hash, owner-side
    interning) played directly on the shards' repos"""

    def __init__(self, S, ctype, rids=()):
        from jylis_amd.engine import Engine
        from jylis_amd.repo import REPOS
        self.S, self.ctype = S, ctype
        self.engs = [Engine(device=0, ujson_columns=32) for _ in range(S)]
        self.repos = [REPOS[ctype](e) for e in self.engs]
        for e in self.engs:  # one replica registration order on every shard
            e.replica_cols([int(x) for x in rids])

    def close(self):
        for e in self.engs:
            e.close()

    def owner_slots(self, t):
        from jylis_amd.route import _pick_keys, owners
        kb, ko = np.asarray(t["key_bytes"], np.uint8), np.asarray(t["key_offs"], np.uint64)
        own = owners(kb, ko, self.S)
        slot = np.zeros(len(own), np.uint32)
        for d in range(self.S):
            idx = np.nonzero(own == d)[0]
            if len(idx):
                b, o = _pick_keys(kb, ko, idx)
                slot[idx] = self.repos[d]._intern({"key_bytes": b, "key_offs": o})
        return own, slot

    def tlog_ingest(self, rank, t):
        own, slot = self.owner_slots(t)
        return tlog_device_batch(self.engs[rank], own, slot, t)

    def ujson_ingest(self, rank, t):
        own, slot = self.owner_slots(t)
        return ujson_device_batch(self.repos[rank], own, slot, t)

    def union_rows(self):
        from jylis_amd.route import owners
        out = {}
        for d, r in enumerate(self.repos):
            st = r.state()
            rows = table_rows(self.ctype, st)
            kb = np.asarray(st["key_bytes"], np.uint8)
            ko = np.asarray(st["key_offs"], np.uint64)
            if len(ko) > 1:
                assert (owners(kb, ko, self.S) == d).all(), "a shard holds a key it does not own"
            out.update(rows)
        return out


def table_rows(ctype, t):
    """{key: canonical content} of a state table"""
    from jylis_amd._lib import TLOG
    ko = np.asarray(t["key_offs"], np.int64)
    kb = np.asarray(t["key_bytes"], np.uint8)
    rows = {}
    for i in range(len(ko) - 1):
        k = bytes(kb[ko[i]:ko[i + 1]])
        if ctype == TLOG:
            eo, vo = np.asarray(t["ent_offs"], np.int64), np.asarray(t["val_offs"], np.int64)
            ents = [(int(t["ts"][j]), bytes(t["val_bytes"][vo[j]:vo[j + 1]])) for j in range(eo[i], eo[i + 1])]
            rows[k] = (int(t["cutoff"][i]), tuple(ents))
        else:
            def seg(ok, cols):
                o = np.asarray(t[ok], np.int64)
                return tuple(sorted(zip(*(np.asarray(t[c])[o[i]:o[i + 1]].tolist() for c in cols))))
            rows[k] = (seg("el_offs", ["dot_ids", "dot_seqs", "elems"]),
                       tuple(x for x in seg("vv_offs", ["vv_ids", "vv_seqs"]) if x[1] != 0),
                       seg("cloud_offs", ["cloud_ids", "cloud_seqs"]))
    return rows


def _oracle_rows(O, ctype, tables):
    ref = O.Repo(ctype)
    for t in tables:
        ref.converge(t)
    return table_rows(ctype, ref.state())


def _tlog_stream(rng, S, rounds, K=3000):
    """per round, per ingesting rank, a random subset of a shared key space
    (state tables first, then deltas): many keys arrive from several ranks"""
    from jylis_amd.synth import tlog_tables
    out = []
    for rnd in range(rounds):
        per = []
        for r in range(S):
            st, ds = tlog_tables(K, int(rng.integers(1 << 30)), rounds=1)
            t = st if rnd == 0 else ds[0]
            idx = rng.permutation(K)[:int(K * 0.6)]
            per.append(pick_rows(t, idx, TLOG_CSRS, per_key=("cutoff",)))
        out.append(per)
    return out


@pytest.mark.parametrize("fab", sorted(FABRIC))
@pytest.mark.parametrize("S", [1, 2, 3])
def test_tlog_routed_local_fabric(oracle_mod, S, fab):
    from jylis_amd._lib import TLOG
    from jylis_amd.route import LocalFabric, TlogRouter
    rng = np.random.default_rng(60 + S)
    node = CsrNode(S, TLOG)
    try:
        router = TlogRouter(node.engs, LocalFabric(S, **FABRIC[fab]))
        seen = []
        for per in _tlog_stream(rng, S, 3):
            seen += per
            router.step([node.tlog_ingest(r, t) for r, t in enumerate(per)])
        router.drain()
        for e in node.engs:
            e.sync()
        assert node.union_rows() == _oracle_rows(oracle_mod, TLOG, seen)
        assert sum(e.skipped() for e in node.engs) == 0
    finally:
        node.close()


def test_tlog_routed_overflow_and_long_values(oracle_mod):
    """one hot owner overflows its runs (records, entries and value bytes);
    values up to 40 bytes travel in the byte section; an empty batch rides
    along"""
    from jylis_amd._lib import TLOG
    from jylis_amd.route import LocalFabric, TlogRouter, owners
    from jylis_amd.synth import tlog_tables
    S = 2
    rng = np.random.default_rng(9)
    node = CsrNode(S, TLOG)
    try:
        router = TlogRouter(node.engs, LocalFabric(S))
        seen = []
        for rnd in range(3):
            per = []
            for r in range(S):
                st, ds = tlog_tables(4000, 100 * rnd + r, rounds=1)
                t = st if rnd == 0 else ds[0]
                own = owners(np.asarray(t["key_bytes"], np.uint8), np.asarray(t["key_offs"], np.uint64), S)
                hot = np.nonzero(own == 1)[0]
                if r == 1 and rnd == 1:
                    hot = hot[:0]  # an empty batch
                t = pick_rows(t, hot, TLOG_CSRS, per_key=("cutoff",))
                # longer values: 9..40 bytes, some with a shared prefix
                n = len(t["ts"])
                lens = rng.integers(0, 41, n)
                vals = [(b"pfx-shared-" + bytes(rng.integers(97, 123, max(int(L) - 11, 0)).astype(np.uint8)))[:int(L)]
                        for L in lens]
                from jylis_amd.engine import encode_keys
                t["val_bytes"], t["val_offs"] = encode_keys(vals)
                per.append(t)
            seen += per
            router.step([node.tlog_ingest(r, t) for r, t in enumerate(per)])
        router.drain()
        assert router.drains >= 1
        assert node.union_rows() == _oracle_rows(oracle_mod, TLOG, seen)
        # the arena holds routed value bytes: a collection keeps every value
        from jylis_amd._lib import TLOG as T
        for e in node.engs:
            e.arena_collect(T)
        assert node.union_rows() == _oracle_rows(oracle_mod, TLOG, seen)
    finally:
        node.close()


def _ujson_stream(rng, S, rounds, D=1500):
    from jylis_amd.synth import replica_ids, ujson_tables
    out = []
    for rnd in range(rounds):
        per = []
        for r in range(S):
            st, ds = ujson_tables(D, 7, rounds=rnd + 1)  # one history: every rank sees consistent dots
            t = st if rnd == 0 else ds[rnd - 1]
            nk = len(t["key_offs"]) - 1
            idx = rng.permutation(nk)[:int(nk * 0.7)]
            per.append(pick_rows(t, idx, UJSON_CSRS))
        out.append(per)
    return out, replica_ids(16, 7)


@pytest.mark.parametrize("fab", sorted(FABRIC))
@pytest.mark.parametrize("S", [1, 2, 3])
def test_ujson_routed_local_fabric(oracle_mod, S, fab):
    from jylis_amd._lib import UJSON
    from jylis_amd.route import LocalFabric, UjsonRouter
    rng = np.random.default_rng(80 + S)
    stream, rids = _ujson_stream(rng, S, 3)
    node = CsrNode(S, UJSON, rids)
    try:
        router = UjsonRouter(node.engs, LocalFabric(S, **FABRIC[fab]))
        seen = []
        for per in stream:
            seen += per
            router.step([node.ujson_ingest(r, t) for r, t in enumerate(per)])
        router.drain()
        for e in node.engs:
            e.sync()
        assert node.union_rows() == _oracle_rows(oracle_mod, UJSON, seen)
        assert sum(e.skipped() for e in node.engs) == 0
    finally:
        node.close()


def test_ujson_routed_overflow(oracle_mod):
    """every document belongs to one owner: the runs overflow and drain"""
    from jylis_amd._lib import UJSON
    from jylis_amd.route import LocalFabric, UjsonRouter, owners
    from jylis_amd.synth import replica_ids, ujson_tables
    S = 2
    node = CsrNode(S, UJSON, replica_ids(16, 3))
    try:
        router = UjsonRouter(node.engs, LocalFabric(S))
        seen = []
        for rnd in range(3):
            per = []
            for r in range(S):
                st, ds = ujson_tables(2000, 3, rounds=rnd + 1)
                t = st if rnd == 0 else ds[rnd - 1]
                own = owners(np.asarray(t["key_bytes"], np.uint8), np.asarray(t["key_offs"], np.uint64), S)
                per.append(pick_rows(t, np.nonzero(own == 0)[0], UJSON_CSRS))
            seen += per
            router.step([node.ujson_ingest(r, t) for r, t in enumerate(per)])
        router.drain()
        assert router.drains >= 1
        assert node.union_rows() == _oracle_rows(oracle_mod, UJSON, seen)
    finally:
        node.close()


def test_run_layout_holes():
    """a run is a complete converge batch: placed keys first (input order),
    holes after them, CSR offsets closed; the first key that does not fit and
    every later key of its destination overflow; the header counts what was
    placed.  Layout (u64 words): slots (u32, packed), cutoffs, offsets, then
    the ts / pre / lr columns of cap_e entries each."""
    import ctypes as C

    import torch

    from jylis_amd import _lib
    from jylis_amd.engine import Engine
    eng = Engine(device=0)
    try:
        S, cap_k, cap_e = 2, 6, 5
        own = np.array([1, 0, 1, 1, 0, 1], np.uint32)
        slot = np.array([10, 11, 12, 13, 14, 15], np.uint32)
        cut = np.array([5, 6, 7, 8, 9, 3], np.uint64)
        offs = np.array([0, 2, 3, 3, 7, 8, 8], np.uint64)  # key 3: 4 entries overflow owner 1's run
        ts = np.arange(8, dtype=np.uint64)[::-1].copy() + 100
        pre = np.arange(8, dtype=np.uint64) + 1000
        lr = np.minimum(np.arange(8, dtype=np.uint64), 8)  # short values: the handle is the length
        W = int(eng.lib.jy_route_words(_lib.TLOG, cap_k, (C.c_uint64 * 1)(cap_e)))
        assert W == 32
        runs = torch.zeros(S * W, dtype=torch.int64, device="cuda:0")
        byts = torch.zeros(S * 8, dtype=torch.uint8, device="cuda:0")
        hdr = torch.zeros(S * 8, dtype=torch.int64, device="cuda:0")
        ovf = torch.zeros(7, dtype=torch.int32, device="cuda:0")
        d = [_dev(x) for x in (own, slot, cut, offs, ts, pre, lr)]
        eng._check(eng.lib.jy_tlog_route_part(eng.h, 6, *[x.data_ptr() for x in d[:4]], 8,
                                              *[x.data_ptr() for x in d[4:]], S, cap_k, cap_e, 8, 0, _lib.DEVICE,
                                              C.c_void_p(runs.data_ptr()), C.c_void_p(byts.data_ptr()),
                                              C.c_void_p(hdr.data_ptr()), C.c_void_p(ovf.data_ptr())))
        torch.cuda.synchronize()
        r = runs.cpu().numpy().view(np.uint64).reshape(S, W)
        h = hdr.cpu().numpy().reshape(S, 8)
        assert h[0, :3].tolist() == [2, 2, 0] and h[1, :3].tolist() == [2, 2, 0]
        o = ovf.cpu().numpy()
        assert o[0] == 2 and sorted(o[1:3].tolist()) == [3, 5]  # key 5 is after key 3 in owner 1's order
        NO = _lib.JY_NO_SLOT
        for dd, (slots, cuts, eoffs, ents) in enumerate([([11, 14], [6, 9], [0, 1, 2], [2, 7]),
                                                         ([10, 12], [5, 7], [0, 2, 2], [0, 1])]):
            assert r[dd, :3].view(np.uint32).tolist() == slots + [NO] * 4
            assert r[dd, 3:9].tolist() == cuts + [0] * 4
            assert r[dd, 9:16].tolist() == eoffs + [eoffs[-1]] * 4
            assert r[dd, 16:16 + len(ents)].tolist() == ts[ents].tolist()
            assert r[dd, 21:21 + len(ents)].tolist() == pre[ents].tolist()
            assert r[dd, 26:26 + len(ents)].tolist() == lr[ents].tolist()
    finally:
        eng.close()


def test_route_part_host_inputs_match_device():
    """jy_tlog_route_part / jy_ujson_route_part with host inputs (staged through
    pinned memory) build the same runs, headers and overflow as with device
    inputs; a key owned by a shard >= nshards is rejected on the host path"""
    import ctypes as C

    import torch

    from jylis_amd import _lib
    from jylis_amd.engine import Engine
    from jylis_amd.synth import tlog_tables, ujson_tables
    eng = Engine(device=0, ujson_columns=16)
    try:
        S, rng = 3, np.random.default_rng(4)
        st, _ = tlog_tables(700, 9, rounds=1)
        n, nent = len(st["ent_offs"]) - 1, len(st["ts"])
        own = rng.integers(0, S, n).astype(np.uint32)
        slot = np.arange(n, dtype=np.uint32)
        pre, lr = eng.pack_values(_lib.TLOG, (st["val_bytes"], st["val_offs"]))
        cols = [own, slot, np.asarray(st["cutoff"], np.uint64), np.asarray(st["ent_offs"], np.uint64)]
        ents = [np.asarray(st["ts"], np.uint64), pre, lr]
        cap_k, cap_e, cap_b = 200, 1200, 4096
        W = int(eng.lib.jy_route_words(_lib.TLOG, cap_k, (C.c_uint64 * 1)(cap_e)))
        outs = []
        for mem in (_lib.HOST, _lib.DEVICE):
            runs = torch.zeros(S * W, dtype=torch.int64, device="cuda:0")
            byts = torch.zeros(S * cap_b, dtype=torch.uint8, device="cuda:0")
            hdr = torch.zeros(S * 8, dtype=torch.int64, device="cuda:0")
            ovf = torch.zeros(n + 1, dtype=torch.int32, device="cuda:0")
            if mem == _lib.HOST:
                ptr = [a.ctypes.data for a in cols], [a.ctypes.data for a in ents]
            else:
                dv = [_dev(a) for a in cols], [_dev(a) for a in ents]
                ptr = [t.data_ptr() for t in dv[0]], [t.data_ptr() for t in dv[1]]
            eng._check(eng.lib.jy_tlog_route_part(eng.h, n, *ptr[0], nent, *ptr[1], S, cap_k, cap_e, cap_b, 0, mem,
                                                  C.c_void_p(runs.data_ptr()), C.c_void_p(byts.data_ptr()),
                                                  C.c_void_p(hdr.data_ptr()), C.c_void_p(ovf.data_ptr())))
            torch.cuda.synchronize()
            o = ovf.cpu().numpy()
            outs.append((runs.cpu().numpy(), byts.cpu().numpy(), hdr.cpu().numpy(), sorted(o[1:1 + o[0]].tolist())))
        h, d = outs
        for a, b in zip(h, d):
            np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
        assert len(h[3]) > 0  # capacities below a balanced share: some keys overflow
        bad = own.copy()
        bad[5] = S
        rc = eng.lib.jy_tlog_route_part(eng.h, n, bad.ctypes.data, *[a.ctypes.data for a in cols[1:]], nent,
                                        *[a.ctypes.data for a in ents], S, cap_k, cap_e, cap_b, 0, _lib.HOST,
                                        C.c_void_p(runs.data_ptr()), C.c_void_p(byts.data_ptr()),
                                        C.c_void_p(hdr.data_ptr()), C.c_void_p(ovf.data_ptr()))
        assert rc == _lib.JY_ERANGE
        # UJSON: host and device inputs agree as well
        ust, _ = ujson_tables(500, 3, rounds=1, R=16)
        from jylis_amd.repo import RepoUJSON
        repo = RepoUJSON(eng)
        nd = len(ust["el_offs"]) - 1
        uown = rng.integers(0, S, nd).astype(np.uint32)
        b = ujson_device_batch(repo, uown, np.arange(nd, dtype=np.uint32), ust)
        hb = [t.cpu().numpy() for t in b]
        hb = [x.view(np.uint32) if x.dtype == np.int32 else x.view(np.uint64) for x in hb]
        caps = (120, 900, 500, 500)
        Wu = int(eng.lib.jy_route_words(_lib.UJSON, caps[0], (C.c_uint64 * 3)(*caps[1:])))
        res = []
        for mem, src in ((_lib.HOST, [x.ctypes.data for x in hb]), (_lib.DEVICE, [t.data_ptr() for t in b])):
            runs = torch.zeros(S * Wu, dtype=torch.int64, device="cuda:0")
            hdr = torch.zeros(S * 8, dtype=torch.int64, device="cuda:0")
            ovf = torch.zeros(nd + 1, dtype=torch.int32, device="cuda:0")
            own_p, slot_p, eo, dots, elems, vo, vv, co, cloud = src
            eng._check(eng.lib.jy_ujson_route_part(
                eng.h, nd, own_p, slot_p, eo, len(hb[3]), dots, elems, vo, len(hb[6]), vv, co, len(hb[8]), cloud, S,
                *caps, 0, mem, C.c_void_p(runs.data_ptr()), C.c_void_p(hdr.data_ptr()), C.c_void_p(ovf.data_ptr())))
            torch.cuda.synchronize()
            o = ovf.cpu().numpy()
            res.append((runs.cpu().numpy(), hdr.cpu().numpy(), sorted(o[1:1 + o[0]].tolist())))
        for a, b2 in zip(*res):
            np.testing.assert_array_equal(np.asarray(a), np.asarray(b2))
    finally:
        eng.close()
