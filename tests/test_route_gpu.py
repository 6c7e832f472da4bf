"""Routing kernels on the GPU (one process): the HIP partition's counts equal
the numpy restatement, and converging the partitioned runs of a batch equals
converging the batch directly (records and long-value bytes both travel)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _treg_batch(rng, n, keyspace):
    from jylis_amd.engine import encode_keys
    keys = [f"rk{int(x)}" for x in rng.choice(keyspace, n, replace=False)]
    vals = []
    for _ in keys:
        L = int(rng.integers(0, 24))
        vals.append(bytes(rng.integers(0, 256, L).astype(np.uint8)) if rng.random() < 0.7
                    else b"shared-prefix" [:min(L, 13)] + bytes(rng.integers(97, 99, max(L - 13, 0)).astype(np.uint8)))
    ts = rng.integers(0, 4, n).astype(np.uint64)
    kb, ko = encode_keys(keys)
    vb, vo = encode_keys(vals)
    return {"key_bytes": kb, "key_offs": ko, "ts": ts, "val_bytes": vb, "val_offs": vo}


@pytest.mark.parametrize("S", [1, 3, 8])
def test_partition_and_routed_converge(oracle_mod, engine, S):
    import ctypes as C

    import torch

    from helpers import assert_state_equal
    from jylis_amd._lib import TREG
    from jylis_amd.repo import RepoTREG
    from jylis_amd.route import owners, partition_counts_np
    O = oracle_mod
    rng = np.random.default_rng(S)
    want = O.Repo(O.TREG)
    got = RepoTREG(engine)
    lib = engine.lib
    dev = torch.device("cuda", 0)
    for _ in range(4):
        b = _treg_batch(rng, 3000, 5000)
        want.converge(b)
        # every "shard" is this engine: slots are this engine's, owners are hashed over S
        slots = got._intern(b)
        own = owners(b["key_bytes"], b["key_offs"], S)
        pre, lr = engine.pack_values(TREG, (b["val_bytes"], b["val_offs"]))
        n = len(slots)
        rc, bc = np.zeros(S, np.uint64), np.zeros(S, np.uint64)
        engine._check(lib.jy_treg_route_count(engine.h, n, own.ctypes.data, lr.ctypes.data, S, 0,
                                              rc.ctypes.data, bc.ctypes.data))
        erc, ebc = partition_counts_np(own, lr, S)
        assert rc.tolist() == erc.tolist() and bc.tolist() == ebc.tolist()
        recs = torch.empty((n, 4), dtype=torch.int64, device=dev)
        byts = torch.empty(max(int(bc.sum()), 1), dtype=torch.uint8, device=dev)
        ts = np.asarray(b["ts"], np.uint64)
        engine._check(lib.jy_treg_route_scatter(engine.h, n, own.ctypes.data, slots.ctypes.data, ts.ctypes.data,
                                                pre.ctypes.data, lr.ctypes.data, S, rc.ctypes.data, bc.ctypes.data,
                                                0, C.c_void_p(recs.data_ptr()), C.c_void_p(byts.data_ptr())))
        engine.sync()
        # every run holds exactly its owner's records
        r = recs.cpu().numpy().view(np.uint64)
        bounds = np.concatenate([[0], np.cumsum(rc)]).astype(np.int64)
        for d in range(S):
            run = r[bounds[d]:bounds[d + 1]]
            assert sorted(run[:, 0].tolist()) == sorted(slots[own == d].tolist())
        engine._check(lib.jy_treg_converge_routed(engine.h, S, rc.ctypes.data, bc.ctypes.data,
                                                  C.c_void_p(recs.data_ptr()), C.c_void_p(byts.data_ptr())))
    assert_state_equal(O.TREG, want.state(), got.state())


def test_router_world_one(oracle_mod, engine):
    """TregRouter with no process group: partition -> (self) -> converge"""
    from helpers import assert_state_equal
    from jylis_amd._lib import TREG
    from jylis_amd.repo import RepoTREG
    from jylis_amd.route import TregRouter
    O = oracle_mod
    rng = np.random.default_rng(9)
    want = O.Repo(O.TREG)
    got = RepoTREG(engine)
    router = TregRouter(engine, None)
    for _ in range(3):
        b = _treg_batch(rng, 2000, 2500)
        want.converge(b)
        slots = got._intern(b)
        pre, lr = engine.pack_values(TREG, (b["val_bytes"], b["val_offs"]))
        router.exchange_and_converge(np.zeros(len(slots), np.uint32), slots, np.asarray(b["ts"], np.uint64), pre, lr)
    assert_state_equal(O.TREG, want.state(), got.state())
