"""Key-hash sharding and the routing exchange, on CPU (gloo, world size 2).

The data plane's HIP partition is restated in numpy (route.partition_counts_np
and the grouping below); the control plane (owner hash, slot directory
exchange) is the product code itself.  Each shard is an oracle repo keyed by
owner-side slots; after routing, the union of the shards equals one oracle
that converged every batch."""
import os
import socket

import numpy as np
import pytest


def test_owner_hash_matches_single_key_form():
    from jylis_amd.engine import encode_keys, key_owner
    from jylis_amd.route import owners
    keys = [f"key-{i}" for i in range(500)] + ["", "\xff"]
    kb, ko = encode_keys(keys)
    own = owners(kb, ko, 8)
    assert [key_owner(k, 8) for k in keys] == own.tolist()
    assert (owners(kb, ko, 1) == 0).all()


def test_partition_counts_np():
    from jylis_amd.route import partition_counts_np
    owner = np.array([0, 1, 1, 3, 0], np.uint32)
    lr = np.array([3, 20 | (5 << 24), 9, 8, 12], np.uint64)
    rec, byt = partition_counts_np(owner, lr, 4)
    assert rec.tolist() == [2, 2, 0, 1] and byt.tolist() == [12, 29, 0, 0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here]
    import torch.distributed as dist

    import oracle as O
    from jylis_amd.engine import encode_keys
    from jylis_amd.route import ShardRouter, _a2a_host, owners
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        # this rank's shard: oracle repo + a slot interner (the engine's role)
        shard = O.Repo(O.TREG)
        names = []
        index = {}

        def intern_local(tab):
            kb, ko = tab
            out = np.empty(len(ko) - 1, np.uint32)
            for i in range(len(ko) - 1):
                k = bytes(kb[ko[i]:ko[i + 1]])
                if k not in index:
                    index[k] = len(names)
                    names.append(k)
                out[i] = index[k]
            return out

        router = ShardRouter(rank, world, intern_local, dist=dist, group=None)
        rng = np.random.default_rng(100 + rank)
        for rnd in range(3):
            # every rank ingests its own peer batch over a shared key space
            keys = [f"k{int(x)}" for x in rng.choice(300, 120, replace=False)]
            vals = [bytes(rng.integers(97, 100, int(rng.integers(0, 14))).astype(np.uint8)) for _ in keys]
            ts = rng.integers(0, 5, len(keys)).astype(np.uint64)
            kb, ko = encode_keys(keys)
            own, slot = router.resolve(kb, ko)
            assert (own == owners(kb, ko, world)).all()
            # data plane, numpy restatement: group records by owner, ship
            # (slot, ts) and values; values as (len, bytes)
            order = np.argsort(own, kind="stable")
            counts = np.bincount(own, minlength=world)
            vb, vo = encode_keys([vals[i] for i in order])
            lens = np.diff(vo.astype(np.int64))
            recs = np.stack([slot[order].astype(np.int64), ts[order].astype(np.int64), lens], 1).reshape(-1)
            byte_counts = [int(lens[int(counts[:d].sum()):int(counts[:d + 1].sum())].sum()) for d in range(world)]
            rrecs, rcnt = _a2a_host(dist, None, recs, [int(c) * 3 for c in counts])
            rbytes, _ = _a2a_host(dist, None, vb, byte_counts)
            rrecs = rrecs.reshape(-1, 3)
            # owner applies every source run (unique keys per run)
            at_b = 0
            batch_keys, batch_vals = [], []
            for r in rrecs:
                s, t, n = int(r[0]), int(r[1]), int(r[2])
                batch_keys.append(names[s])
                batch_vals.append(bytes(rbytes[at_b:at_b + n]))
                at_b += n
            for lo, hi in zip(np.cumsum([0] + [c // 3 for c in rcnt.tolist()])[:-1],
                              np.cumsum([c // 3 for c in rcnt.tolist()])):
                kb2, ko2 = encode_keys(batch_keys[lo:hi])
                vb2, vo2 = encode_keys(batch_vals[lo:hi])
                shard.converge({"key_bytes": kb2, "key_offs": ko2, "ts": rrecs[lo:hi, 1].astype(np.uint64),
                                "val_bytes": vb2, "val_offs": vo2})
            q.put(("batch", rank, rnd, keys, vals, ts.tolist()))
        st = shard.state()
        q.put(("state", rank, O.split_keys(st), st["ts"].tolist(),
               [bytes(st["val_bytes"][st["val_offs"][i]:st["val_offs"][i + 1]]) for i in range(len(st["ts"]))]))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        import traceback
        q.put(("error", rank, traceback.format_exc()))
        raise


def test_two_rank_routing_matches_single_repo(oracle_mod):
    import multiprocessing as mp
    from jylis_amd.engine import encode_keys
    from jylis_amd.route import owners
    O = oracle_mod
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=180) for _ in range(2 * 3 + 2)]
    for p in procs:
        p.join(timeout=60)
    errs = [m for m in msgs if m[0] == "error"]
    assert not errs, errs[0][2]
    # reference: one repo converging every ingested batch
    ref = O.Repo(O.TREG)
    for m in sorted(m for m in msgs if m[0] == "batch"):
        _, rank, rnd, keys, vals, ts = m
        kb, ko = encode_keys(keys)
        vb, vo = encode_keys(vals)
        ref.converge({"key_bytes": kb, "key_offs": ko, "ts": np.array(ts, np.uint64), "val_bytes": vb,
                      "val_offs": vo})
    st = ref.state()
    want = {k: (int(t), bytes(st["val_bytes"][st["val_offs"][i]:st["val_offs"][i + 1]]))
            for i, (k, t) in enumerate(zip(O.split_keys(st), st["ts"]))}
    got = {}
    for m in msgs:
        if m[0] == "state":
            _, rank, keys, ts, vals = m
            kb, ko = encode_keys(keys)
            assert (owners(kb, ko, 2) == rank).all(), "a shard holds a key it does not own"
            for k, t, v in zip(keys, ts, vals):
                got[k] = (t, v)
    assert got == want
