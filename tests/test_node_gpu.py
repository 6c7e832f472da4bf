"""The node (jy_node_*, jylis_amd/csrc/jy_node.hip): one C-ABI call per
decoded peer batch for every GPU of a node -- keys hashed and regrouped by
owner on the device, exchanged, interned on their owner and merged there.

* S = 1 through a real RCCL communicator (the exchange is RCCL's send/recv
  to itself; the count exchange and the payload go through the same calls
  as at S = 8).
* S = 2, 3 shards on one GPU with the copy fabric (the exchange as device
  copies; everything else is the same code).

After the batches, the union of the shards must equal ONE oracle repo that
converged every batch (RepoManagerCore.converge_deltas,
jylis/repo_manager.pony:92-93), bit-exact, and every key must live on its
owner (jy_key_owner)."""
import numpy as np
import pytest

from helpers import assert_state_equal, join_rows, random_history, split_rows

pytestmark = pytest.mark.gpu

TYPES = [0, 1, 2, 3, 4]
# "rccl1": S = 1 through the regroup + RCCL self exchange that S > 1 runs
# (JY_NODE_REGROUP_ONE); plain S = 1 reads its inputs in place
LAYOUTS = [(1, "rccl"), (1, "rccl1"), (2, "copy"), (3, "copy")]


def _node(S, fabric, **kw):
    import os
    from jylis_amd.node import Node
    if fabric != "rccl1":
        return Node(S, fabric, **kw)
    os.environ["JY_NODE_REGROUP_ONE"] = "1"
    try:
        return Node(S, "rccl", **kw)
    finally:
        del os.environ["JY_NODE_REGROUP_ONE"]


def _union(O, ctype, node):
    from jylis_amd.engine import key_owner
    from jylis_amd.repo import REPOS
    rows = {}
    for sh, eng in enumerate(node.engines):
        st = REPOS[ctype](eng).state()
        part = dict(split_rows(ctype, st))
        for k in part:
            assert key_owner(k, node.S) == node.rank0 + sh, (k, sh)
        rows.update(part)
    return join_rows(ctype, rows)


def _want(O, ctype, batches):
    ref = O.Repo(ctype)
    for b in batches:
        ref.converge(b)
    return join_rows(ctype, split_rows(ctype, ref.state()))


@pytest.mark.parametrize("S,fabric", LAYOUTS)
@pytest.mark.parametrize("ctype", TYPES)
def test_node_history(oracle_mod, ctype, S, fabric):
    """oracle write-path histories (several replicas, partial gossip, full
    state deltas), every flushed batch one node call"""
    from jylis_amd.node import Node
    O = oracle_mod
    node = _node(S, fabric)
    try:
        batches = random_history(O, ctype, seed=100 + 10 * ctype + S, nops=160, nkeys=40)
        for b in batches:
            node.converge_table(ctype, b)
        node.sync()
        assert_state_equal(ctype, _want(O, ctype, batches), _union(O, ctype, node))
        st = node.stats()
        assert st["exchanges"] == len(batches)
    finally:
        node.close()


def _treg_batch(rng, n, keyspace):
    from jylis_amd.engine import encode_keys
    keys = [b"nk%d" % int(x) for x in rng.choice(keyspace, n, replace=False)]
    vals = []
    for _ in keys:
        L = int(rng.integers(0, 30))
        vals.append(bytes(rng.integers(0, 256, L).astype(np.uint8)) if rng.random() < 0.6
                    else (b"common-prefix-" + bytes(rng.integers(97, 100, 12).astype(np.uint8)))[:L])
    kb, ko = encode_keys(keys)
    vb, vo = encode_keys(vals)
    return {"key_bytes": kb, "key_offs": ko, "ts": rng.integers(0, 4, n).astype(np.uint64),
            "val_bytes": vb, "val_offs": vo}


def _dev(a):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    return torch.from_numpy(a).to("cuda:0")


@pytest.mark.parametrize("S,fabric", LAYOUTS)
@pytest.mark.parametrize("mem", ["host", "device"])
def test_node_treg_large(oracle_mod, S, fabric, mem):
    """20K-key batches over a 30K key space: timestamp ties, shared 8-byte
    prefixes and long values (their bytes travel to the owner's arena);
    host-staged and HBM-resident inputs; an empty batch in between"""
    from jylis_amd.engine import encode_keys
    from jylis_amd.node import Node
    O = oracle_mod
    rng = np.random.default_rng(7 + S)
    node = _node(S, fabric)
    try:
        seen = []
        for step in range(4):
            b = _treg_batch(rng, 20000, 30000)
            seen.append(b)
            args = [b["key_bytes"], b["key_offs"], b["ts"], b["val_bytes"], b["val_offs"]]
            node.treg_converge(*(args if mem == "host" else [_dev(a) for a in args]))
            if step == 1:
                kb, ko = encode_keys([])
                node.treg_converge(kb, ko, np.zeros(0, np.uint64), np.zeros(0, np.uint8), np.zeros(1, np.uint64))
        node.sync()
        assert_state_equal(O.TREG, _want(O, O.TREG, seen), _union(O, O.TREG, node))
    finally:
        node.close()


def _tlog_batch(rng, n, keyspace, t0):
    from jylis_amd.engine import encode_keys
    keys = [b"tl%d" % int(x) for x in rng.choice(keyspace, n, replace=False)]
    cut, offs, ts, vals = [], [0], [], []
    for _ in keys:
        m = int(rng.integers(0, 5))
        ents = sorted({(int(t0 + rng.integers(0, 50)),
                        bytes(rng.integers(97, 100, int(rng.integers(0, 20))).astype(np.uint8))) for _ in range(m)},
                      reverse=True)
        c = int(t0 + rng.integers(0, 10)) if rng.random() < 0.1 else 0
        ents = [e for e in ents if e[0] >= c]
        cut.append(c)
        ts += [e[0] for e in ents]
        vals += [e[1] for e in ents]
        offs.append(offs[-1] + len(ents))
    kb, ko = encode_keys(keys)
    vb, vo = encode_keys(vals)
    return {"key_bytes": kb, "key_offs": ko, "cutoff": np.array(cut, np.uint64), "ent_offs": np.array(offs, np.uint64),
            "ts": np.array(ts, np.uint64), "val_bytes": vb, "val_offs": vo}


@pytest.mark.parametrize("S,fabric", LAYOUTS)
@pytest.mark.parametrize("mem", ["host", "device"])
def test_node_tlog_large(oracle_mod, S, fabric, mem):
    """5K-log batches: appends, ties, duplicates, cutoff raises, long values"""
    from jylis_amd.node import Node
    O = oracle_mod
    rng = np.random.default_rng(70 + S)
    node = _node(S, fabric)
    try:
        seen = []
        for step in range(4):
            b = _tlog_batch(rng, 5000, 8000, 1000 + 20 * step)
            seen.append(b)
            args = [b[k] for k in ("key_bytes", "key_offs", "cutoff", "ent_offs", "ts", "val_bytes", "val_offs")]
            node.tlog_converge(*(args if mem == "host" else [_dev(a) for a in args]))
        node.sync()
        assert_state_equal(O.TLOG, _want(O, O.TLOG, seen), _union(O, O.TLOG, node))
    finally:
        node.close()


@pytest.mark.parametrize("S,fabric", LAYOUTS)
def test_node_counter_device(oracle_mod, S, fabric):
    """PNCOUNT batches with HBM-resident keys and cells (the keyed form)"""
    from jylis_amd.engine import encode_keys
    from jylis_amd.node import Node
    O = oracle_mod
    rng = np.random.default_rng(5 + S)
    node = _node(S, fabric)
    try:
        rids = [int(x) for x in rng.integers(1, 2**63, 6)]
        cols = node.replica_cols(rids)
        ref = O.Repo(O.PNCOUNT)
        for step in range(3):
            keys = [b"pc%d" % int(x) for x in rng.choice(9000, 6000, replace=False)]
            kb, ko = encode_keys(keys)
            ncell = rng.integers(0, 5, len(keys))
            offs = np.zeros(len(keys) + 1, np.uint64)
            offs[1:] = np.cumsum(ncell)
            m = int(offs[-1])
            rep = rng.integers(0, 6, m)
            sign = rng.integers(0, 2, m).astype(np.uint8)
            val = rng.integers(0, 2**63, m, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, m).astype(np.uint64)
            node.counter_converge(O.PNCOUNT, _dev(kb), _dev(ko), _dev(offs),
                                  _dev(cols[rep]), _dev(val), sign=_dev(sign))
            # the same batch as an oracle table (one cell per (key, replica, sign): max of repeats)
            key_of = np.repeat(np.arange(len(keys)), ncell)
            t = {"key_bytes": kb, "key_offs": ko}
            for g, pre in enumerate(("p_", "n_")):
                best = {}
                for k_, r_, v_ in zip(key_of[sign == g], rep[sign == g], val[sign == g]):
                    best[(int(k_), rids[int(r_)])] = max(best.get((int(k_), rids[int(r_)]), 0), int(v_))
                items = sorted(best.items())
                o = np.zeros(len(keys) + 1, np.uint64)
                for (k_, _), _v in items:
                    o[k_ + 1] += 1
                t[pre + "offs"] = np.cumsum(o).astype(np.uint64)
                t[pre + "ids"] = np.array([r for (_, r), _ in items], np.uint64)
                t[pre + "vals"] = np.array([v for _, v in items], np.uint64)
            ref.converge(t)
        node.sync()
        want = join_rows(O.PNCOUNT, split_rows(O.PNCOUNT, ref.state()))
        assert_state_equal(O.PNCOUNT, want, _union(O, O.PNCOUNT, node))
    finally:
        node.close()


@pytest.mark.parametrize("S,fabric", LAYOUTS)
def test_node_counter_block(S, fabric):
    """dense peer columns arriving mixed (jy_node_counter_converge_block, the
    bench's routed PNCOUNT step): every shard's cells are the max over the
    columns every local shard ingested for it"""
    import torch
    from jylis_amd._lib import PNCOUNT
    from jylis_amd.node import Node
    K, C = 4096, 3
    node = _node(S, fabric, counter_columns=S * C)
    try:
        cols = node.replica_cols(list(range(1, S * C + 1))).reshape(S, C)  # shard r's peers
        for r, eng in enumerate(node.engines):
            slots = eng.intern(PNCOUNT, [b"s%d:%d" % (r, i) for i in range(K)])
            assert (slots == np.arange(K)).all()
        g = torch.Generator(device="cuda:0").manual_seed(11)
        want = np.zeros((S, 2, S * C, K), np.uint64)
        for _ in range(3):
            vp = torch.randint(0, 2**62, (S, C, S, K), dtype=torch.int64, device="cuda:0", generator=g)
            vn = torch.randint(0, 2**62, (S, C, S, K), dtype=torch.int64, device="cuda:0", generator=g)
            node.counter_converge_block(PNCOUNT, cols, 0, K, vp, vn)
            a, b = vp.cpu().numpy().view(np.uint64), vn.cpu().numpy().view(np.uint64)
            for L in range(S):  # ingest shard L, its c-th peer column, destined to owner d
                for c in range(C):
                    col = int(cols[L, c])
                    for d in range(S):
                        want[d, 0, col] = np.maximum(want[d, 0, col], a[L, c, d])
                        want[d, 1, col] = np.maximum(want[d, 1, col], b[L, c, d])
        node.sync()
        for d, eng in enumerate(node.engines):
            got = eng.counter_export(PNCOUNT, S * C, 0, K)
            np.testing.assert_array_equal(got, want[d])
    finally:
        node.close()


def test_node_rejects_bad_config():
    from jylis_amd.engine import EngineError
    from jylis_amd.node import Node
    with pytest.raises(EngineError):
        Node(2, "rccl", nlocal=1)  # a multi-process node needs the shared unique id
    with pytest.raises(EngineError):
        Node(0, "copy")


@pytest.mark.parametrize("mem", ["host", "device"])
def test_node_one_shard_arena_grows_in_call(oracle_mod, mem):
    """at S = 1 the long values go into the arena on the read-back
    stream beside the key probe -- the arena must be grown (jy_arena_ensure)
    before that stream may run, never under it.  A 4 KiB arena, then TREG and
    TLOG batches whose long values take megabytes: the arena grows inside
    every call, and the states equal the oracle's."""
    O = oracle_mod
    rng = np.random.default_rng(99)
    node = _node(1, "rccl", arena_capacity=1 << 12)
    try:
        eng = node.engines[0]
        seen_r, seen_l = [], []
        caps = []
        for step in range(3):
            b = _treg_batch(rng, 20000, 30000)
            # every value long: 40-200 bytes
            from jylis_amd.engine import encode_keys
            vals = [bytes(rng.integers(0, 256, int(rng.integers(40, 200))).astype(np.uint8)) for _ in range(20000)]
            b["val_bytes"], b["val_offs"] = encode_keys(vals)
            seen_r.append(b)
            args = [b["key_bytes"], b["key_offs"], b["ts"], b["val_bytes"], b["val_offs"]]
            node.treg_converge(*(args if mem == "host" else [_dev(a) for a in args]))
            t = _tlog_batch(rng, 5000, 8000, 1000 + 20 * step)
            # long values, each key's segment kept strictly newest first
            eo = np.asarray(t["ent_offs"], np.int64)
            lv, ts = [], []
            for k in range(len(eo) - 1):
                ents = sorted({(int(t["ts"][j]), bytes(rng.integers(97, 123, int(rng.integers(30, 120))).astype(np.uint8)))
                               for j in range(eo[k], eo[k + 1])}, reverse=True)
                ts += [e[0] for e in ents]
                lv += [e[1] for e in ents]
            t["ts"] = np.array(ts, np.uint64)
            t["val_bytes"], t["val_offs"] = encode_keys(lv)
            seen_l.append(t)
            targs = [t[k] for k in ("key_bytes", "key_offs", "cutoff", "ent_offs", "ts", "val_bytes", "val_offs")]
            node.tlog_converge(*(targs if mem == "host" else [_dev(a) for a in targs]))
            node.sync()
            caps.append(eng.arena_usage(O.TREG)[1])
        assert caps[-1] > (1 << 20) and caps[0] > (1 << 12)
        assert_state_equal(O.TREG, _want(O, O.TREG, seen_r), _union(O, O.TREG, node))
        assert_state_equal(O.TLOG, _want(O, O.TLOG, seen_l), _union(O, O.TLOG, node))
    finally:
        node.close()
