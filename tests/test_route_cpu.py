"""Key-hash sharding and the exchange medium, on CPU.

The control plane (owner hash, the owner-slot directory exchange of
route.ShardRouter) and the fabrics' collective semantics (equal-split
all-to-all, global max) run here with torch CPU tensors: LocalFabric in one
process, DistFabric over gloo with world size 2.  The data plane (partition
kernels and the routed merge) needs the GPU: tests/test_route_gpu.py and
tests/test_route_dist_gpu.py run it through these same fabrics."""
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
    # balanced enough for the fixed run capacity (CAP_SLACK) at these sizes
    kb, ko = encode_keys([f"t{i:010d}" for i in range(80000)])
    counts = np.bincount(owners(kb, ko, 8), minlength=8)
    from jylis_amd.route import CAP_MARGIN, CAP_SLACK
    assert counts.max() <= 80000 / 8 * CAP_SLACK + CAP_MARGIN


def test_run_caps():
    from jylis_amd.route import run_caps
    assert run_caps(1000, 50, 1) == (1000, 56)  # bytes: 8-byte granules
    cap, capb = run_caps(1 << 20, 1 << 22, 8)
    assert (1 << 17) < cap < (1 << 20) and (1 << 19) < capb < (1 << 22)
    assert run_caps(10, 0, 4) == (10, 8)  # never above the whole batch


def test_local_fabric_semantics():
    import torch
    from jylis_amd.route import LocalFabric
    S = 3
    f = LocalFabric(S)
    ins = [torch.arange(S * 4, dtype=torch.int64) + 100 * r for r in range(S)]
    outs = [torch.empty_like(x) for x in ins]
    f.a2a(outs, ins)
    for r in range(S):
        for s in range(S):
            assert outs[r][s * 4:(s + 1) * 4].tolist() == (ins[s][r * 4:(r + 1) * 4]).tolist()
    ts = [torch.tensor([3]), torch.tensor([9]), torch.tensor([1])]
    f.max_all(ts)
    assert [int(t) for t in ts] == [9, 9, 9]
    assert [m.tolist() for m in f.host_max([np.array([1, 5]), np.array([4, 2]), np.array([0, 0])])] == [[4, 5]] * 3
    # variable all-to-all (key resolution): rank s sends splits[s][r] items to rank r
    splits = np.array([[1, 0, 2], [0, 3, 1], [2, 2, 0]])
    recv = f.host_a2a(splits)
    assert [r.tolist() for r in recv] == [splits[:, r].tolist() for r in range(S)]
    ins = [torch.arange(int(splits[s].sum()), dtype=torch.int64) + 100 * s for s in range(S)]
    outs = [torch.empty(int(recv[r].sum()), dtype=torch.int64) for r in range(S)]
    f.a2a_v(outs, ins, recv, splits)
    for r in range(S):
        want = []
        for s in range(S):
            a = int(splits[s][:r].sum())
            want += (ins[s][a:a + int(splits[s][r])]).tolist()
        assert outs[r].tolist() == want


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
    import torch
    import torch.distributed as dist

    from jylis_amd.engine import encode_keys
    from jylis_amd.route import DistFabric, ShardRouter, owners
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        # ---- fabric collectives (gloo, CPU tensors)
        fab = DistFabric(dist, cpu_group=None)
        x = torch.arange(world * 3, dtype=torch.int64) + 1000 * rank
        out = torch.empty_like(x)
        fab.a2a([out], [x])
        m = torch.tensor([rank * 7 + 1], dtype=torch.int32)
        fab.max_all([m])
        hm = fab.host_max([np.array([rank, 10 - rank], np.int64)])[0]
        # variable all-to-all: rank r sends r + 1 + d items to rank d
        sp = np.array([rank + 1 + d for d in range(world)], np.int64)
        rv = fab.host_a2a([sp])[0]
        vin = torch.arange(int(sp.sum()), dtype=torch.int64) + 1000 * rank
        vout = torch.empty(int(rv.sum()), dtype=torch.int64)
        fab.a2a_v([vout], [vin], [rv], [sp])
        q.put(("fabric", rank, out.tolist(), int(m), hm.tolist(), rv.tolist(), vout.tolist()))
        # ---- control plane: owner-side slots through the directory exchange
        names, index = [], {}

        def intern_local(tab):
            kb, ko = tab
            res = np.empty(len(ko) - 1, np.uint32)
            for i in range(len(ko) - 1):
                k = bytes(kb[ko[i]:ko[i + 1]])
                if k not in index:
                    index[k] = len(names)
                    names.append(k)
                res[i] = index[k]
            return res

        router = ShardRouter(rank, world, intern_local, dist=dist, group=None)
        rng = np.random.default_rng(100 + rank)
        for rnd in range(3):
            keys = [f"k{int(v)}" for v in rng.choice(300, 120, replace=False)]
            kb, ko = encode_keys(keys)
            own, slot = router.resolve(kb, ko)
            assert (own == owners(kb, ko, world)).all()
            q.put(("resolved", rank, keys, own.tolist(), slot.tolist()))
        q.put(("names", rank, [n.decode() for n in names]))
        dist.destroy_process_group()
    except Exception:  # surface worker failures to the parent
        import traceback
        q.put(("error", rank, traceback.format_exc()))
        raise


def test_two_rank_fabric_and_directory():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    from helpers import collect
    msgs = collect(procs, q, world * (1 + 3 + 1))
    for _, rank, out, m, hm, rv, vout in (m for m in msgs if m[0] == "fabric"):
        assert out == [s * 1000 + rank * 3 + j for s in range(world) for j in range(3)]
        assert m == (world - 1) * 7 + 1
        assert hm == [world - 1, 10]
        assert rv == [s + 1 + rank for s in range(world)]
        want = []
        for s in range(world):
            a = sum(s + 1 + d for d in range(rank))
            want += [1000 * s + a + j for j in range(s + 1 + rank)]
        assert vout == want
    names = {m[1]: m[2] for m in msgs if m[0] == "names"}
    for _, rank, keys, own, slot in (m for m in msgs if m[0] == "resolved"):
        for k, o, s in zip(keys, own, slot):
            assert names[o][s] == k, "a slot answered by the owner names another key"
