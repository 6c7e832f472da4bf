"""World-size-2 routing with the real data plane: two processes on cuda:0,
each with its own engine (shard), torch.distributed over gloo (the
collectives go through host memory; on an 8-GPU node the same DistFabric
uses RCCL over xGMI).  The key resolution runs on the GPU (route.KeyResolver:
keys regrouped by owner on the device, variable all-to-alls, interned by
the owner's device directory, slots sent back), the
HIP partition kernels build fixed-capacity runs, the runs cross the fabric
and each owner merges what it received; the union of the two shards must
equal one oracle repo that converged every ingested batch."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tlog_table(rank, rnd):
    """rank's TLOG batch of round rnd: a random 60% of a shared key space"""
    from jylis_amd.synth import tlog_tables
    from test_route_csr_gpu import TLOG_CSRS, pick_rows
    st, ds = tlog_tables(1500, 1000 + 10 * rnd + rank, rounds=1)
    t = st if rnd == 0 else ds[0]
    idx = np.random.default_rng(50 + 10 * rnd + rank).permutation(1500)[:900]
    return pick_rows(t, idx, TLOG_CSRS, per_key=("cutoff",))


def _ujson_table(rank, rnd):
    """rank's UJSON batch of round rnd: a random 70% of one document history"""
    from jylis_amd.synth import ujson_tables
    from test_route_csr_gpu import UJSON_CSRS, pick_rows
    st, ds = ujson_tables(1200, 7, rounds=rnd + 1)
    t = st if rnd == 0 else ds[rnd - 1]
    nk = len(t["key_offs"]) - 1
    idx = np.random.default_rng(70 + 10 * rnd + rank).permutation(nk)[:int(nk * 0.7)]
    return pick_rows(t, idx, UJSON_CSRS)


def _worker(rank, world, port, q, seed):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here]
    try:
        import torch
        import torch.distributed as dist

        from jylis_amd._lib import PNCOUNT, TREG
        from jylis_amd.engine import Engine, encode_keys
        from jylis_amd.repo import RepoTREG
        from jylis_amd.route import CounterRouter, DistFabric, KeyResolver, TregRouter, long_bytes
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        eng = Engine(device=0, counter_columns=8, ujson_columns=32)
        repo = RepoTREG(eng)
        fab = DistFabric(dist)

        def resolver(ctype):
            kr = KeyResolver([eng], fab, ctype)

            def resolve(kb, ko):
                kbt = torch.from_numpy(np.ascontiguousarray(kb, np.uint8)).to("cuda:0")
                kot = torch.from_numpy(np.asarray(ko, np.uint64).view(np.int64)).to("cuda:0")
                ((own, slot),) = kr.resolve([(kbt, kot)])
                return own.cpu().numpy().view(np.uint32), slot.cpu().numpy().view(np.uint32)
            return resolve
        resolve_treg = resolver(TREG)
        router = TregRouter([eng], fab)
        rng = np.random.default_rng(seed + rank)

        def dev(a):
            a = np.ascontiguousarray(a)
            return torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda:0")

        for rnd in range(3):
            keys = [f"d{int(x)}" for x in rng.choice(3000, 1800, replace=False)]
            vals = [bytes(rng.integers(97, 100, int(rng.integers(0, 20))).astype(np.uint8)) for _ in keys]
            ts = rng.integers(0, 4, len(keys)).astype(np.uint64)
            kb, ko = encode_keys(keys)
            own, slot = resolve_treg(kb, ko)
            pre, lr = eng.pack_values(TREG, vals)
            router.step([(dev(own), dev(slot), dev(ts), dev(pre), dev(lr), long_bytes(lr))])
            q.put(("batch", rank, rnd, keys, [v.decode() for v in vals], ts.tolist()))
        router.drain()
        st = repo.state()
        from oracle import split_keys
        q.put(("treg", rank, [k.decode() for k in split_keys(st)], st["ts"].tolist(),
               [bytes(st["val_bytes"][st["val_offs"][i]:st["val_offs"][i + 1]]).decode()
                for i in range(len(st["ts"]))]))
        # ---- dense PNCOUNT: each rank ingests 2 peer columns grouped by owner
        K, Cn = 2048, 2
        from jylis_amd import synth as Sy
        eng.intern(PNCOUNT, Sy.counter_keys(K, prefix=f"o{rank}:".encode()))
        cols = eng.replica_cols(Sy.replica_ids(world * Cn, 5).tolist())
        peer = [[int(cols[r * Cn + c]) for c in range(Cn)] for r in range(world)]
        crt = CounterRouter([eng], fab, PNCOUNT)
        for rnd in range(2):
            v = np.random.default_rng(1000 * rnd + rank).integers(0, 1 << 62, (2, Cn, world, K), dtype=np.uint64)
            crt.step([torch.from_numpy(v.view(np.int64)).to("cuda:0")], peer)
        eng.sync()
        q.put(("pn", rank, eng.counter_export(PNCOUNT, world * Cn, 0, K).tolist()))
        # ---- TLOG logs and UJSON documents, routed with their entries
        from jylis_amd.repo import RepoTLOG, RepoUJSON
        from jylis_amd.route import TlogRouter, UjsonRouter
        from jylis_amd.synth import replica_ids
        from test_route_csr_gpu import table_rows, tlog_device_batch, ujson_device_batch
        tl, uj = RepoTLOG(eng), RepoUJSON(eng)
        eng.replica_cols(replica_ids(16, 7).tolist())  # one registration order on every shard
        from jylis_amd._lib import TLOG, UJSON
        resolve_tlog, resolve_ujson = resolver(TLOG), resolver(UJSON)
        trt, urt = TlogRouter([eng], fab), UjsonRouter([eng], fab)
        for rnd in range(3):
            t = _tlog_table(rank, rnd)
            own, slot = resolve_tlog(t["key_bytes"], t["key_offs"])
            trt.step([tlog_device_batch(eng, own, slot, t)])
            u = _ujson_table(rank, rnd)
            own, slot = resolve_ujson(u["key_bytes"], u["key_offs"])
            urt.step([ujson_device_batch(uj, own, slot, u)])
        trt.drain()
        urt.drain()
        q.put(("tlog", rank, table_rows(tl.ctype, tl.state())))
        q.put(("ujson", rank, table_rows(uj.ctype, uj.state())))
        eng.close()
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put(("error", rank, traceback.format_exc()))
        raise


def test_two_process_routing(oracle_mod):
    import multiprocessing as mp
    from jylis_amd.engine import encode_keys
    from jylis_amd.route import owners
    O = oracle_mod
    world, seed = 2, 31
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, seed)) for r in range(world)]
    for p in procs:
        p.start()
    from helpers import collect
    msgs = collect(procs, q, world * 7)
    ref = O.Repo(O.TREG)
    for _, rank, rnd, keys, vals, ts in sorted(m for m in msgs if m[0] == "batch"):
        kb, ko = encode_keys(keys)
        vb, vo = encode_keys(vals)
        ref.converge({"key_bytes": kb, "key_offs": ko, "ts": np.array(ts, np.uint64), "val_bytes": vb,
                      "val_offs": vo})
    st = ref.state()
    want = {k.decode(): (int(t), bytes(st["val_bytes"][st["val_offs"][i]:st["val_offs"][i + 1]]).decode())
            for i, (k, t) in enumerate(zip(O.split_keys(st), st["ts"]))}
    got = {}
    for _, rank, keys, ts, vals in (m for m in msgs if m[0] == "treg"):
        kb, ko = encode_keys(keys)
        assert (owners(kb, ko, world) == rank).all(), "a shard holds a key it does not own"
        got.update({k: (t, v) for k, t, v in zip(keys, ts, vals)})
    assert got == want
    # PNCOUNT: owner d's column (r, c) = max over rounds of rank r's block for d
    K, Cn = 2048, 2
    for _, d, dump in (m for m in msgs if m[0] == "pn"):
        dump = np.array(dump, np.uint64)
        exp = np.zeros((2, world * Cn, K), np.uint64)
        for rnd in range(2):
            for r in range(world):
                v = np.random.default_rng(1000 * rnd + r).integers(0, 1 << 62, (2, Cn, world, K), dtype=np.uint64)
                for c in range(Cn):
                    np.maximum(exp[:, r * Cn + c], v[:, c, d], out=exp[:, r * Cn + c])
        np.testing.assert_array_equal(dump, exp)
    # TLOG / UJSON: the union of the two shards = one oracle repo over every batch
    from test_route_csr_gpu import table_rows
    for ctype, mk in ((O.TLOG, _tlog_table), (O.UJSON, _ujson_table)):
        ref = O.Repo(ctype)
        for rnd in range(3):
            for r in range(world):
                ref.converge(mk(r, rnd))
        want = table_rows(ctype, ref.state())
        name = "tlog" if ctype == O.TLOG else "ujson"
        got = {}
        for m in msgs:
            if m[0] == name:
                assert not set(got) & set(m[2]), "a key on two shards"
                got.update(m[2])
        assert got == want, name
