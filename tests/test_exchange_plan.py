"""The node's exchange schedule on the host (jy_node_exchange_plan: the exact
planner jy_node.hip's RCCL exchange issues), for S = 2..8 shards without a
GPU: the intra-node analogue of Cluster.broadcast_deltas
(/root/reference/jylis/cluster.pony:205-213).

Every shard's per-peer counts come from one consistent S x S count matrix
(what the count exchange delivers); for every wire column every send of
shard s to d meets a receive of d from s of the same size, in the same
order; the sends partition s's owner-order column and the receives d's
source-major column with no gap or overlap; a shard's own part is a copy;
and every rank issues its operations in one peer order (wire, then peer
ascending), so the grouped ncclSend / ncclRecv of all ranks line up."""
import ctypes as C

import numpy as np
import pytest

WIRES = [(0, 4), (1, 1), (0, 8), (2, 8), (3, 16), (2, 1)]  # (count granule, element bytes)
W = 4


def _plan(lib, S, rank, cnt):
    """cnt[s][d][g]: elements shard s sends to d in granule g -> list of ops"""
    send = np.ascontiguousarray(cnt[rank], np.uint64)          # [d][g]
    recv = np.ascontiguousarray(cnt[:, rank, :], np.uint64)    # [s][g]
    gran = np.array([g for g, _ in WIRES], np.int32)
    esz = np.array([e for _, e in WIRES], np.int32)
    cap = 4 * S * len(WIRES)
    ops = np.zeros((cap, 6), np.uint64)
    n = C.c_uint64()
    rc = lib.jy_node_exchange_plan(S, rank, W, len(WIRES), gran.ctypes.data, esz.ctypes.data, send.ctypes.data,
                                   recv.ctypes.data, cap, ops.ctypes.data, C.byref(n))
    assert rc == 0
    assert n.value <= cap
    return [tuple(int(x) for x in o) for o in ops[:n.value]]


@pytest.mark.parametrize("S", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("seed", [1, 2])
def test_exchange_schedule(S, seed):
    from jylis_amd._lib import load
    lib = load()
    rng = np.random.default_rng(100 * S + seed)
    cnt = rng.integers(0, 50, (S, S, W)).astype(np.uint64)
    cnt[rng.random((S, S, W)) < 0.3] = 0  # empty parts: no operation at all
    plans = [_plan(lib, S, r, cnt) for r in range(S)]
    for r, ops in enumerate(plans):
        # one order on every rank: by wire, then by peer
        keys = [(w, p) for (_, w, p, _, _, _) in ops]
        assert keys == sorted(keys)
        for wi, (g, e) in enumerate(WIRES):
            mine = [o for o in ops if o[1] == wi]
            # sends (+ the own copy) partition the owner-order column, in peer order
            so, ro = 0, 0
            for d in range(S):
                sn, rn = int(cnt[r, d, g]) * e, int(cnt[d, r, g]) * e
                if d == r:
                    own = [o for o in mine if o[0] == 0]
                    assert (own == [(0, wi, r, so, ro, sn)]) if sn else not own
                else:
                    snd = [o for o in mine if o[0] == 1 and o[2] == d]
                    rcv = [o for o in mine if o[0] == 2 and o[2] == d]
                    assert (snd == [(1, wi, d, so, 0, sn)]) if sn else not snd
                    assert (rcv == [(2, wi, d, 0, ro, rn)]) if rn else not rcv
                so += sn
                ro += rn
    # every send meets the matching receive, same wire order and size
    for s in range(S):
        for d in range(S):
            if s == d:
                continue
            sends = [(w, b) for (k, w, p, _, _, b) in plans[s] if k == 1 and p == d]
            recvs = [(w, b) for (k, w, p, _, _, b) in plans[d] if k == 2 and p == s]
            assert sends == recvs, (s, d)


def test_exchange_plan_rejects_bad_shapes():
    from jylis_amd._lib import load
    lib = load()
    z = np.zeros(64, np.uint64)
    g = np.zeros(1, np.int32)
    e = np.ones(1, np.int32)
    n = C.c_uint64()
    ops = np.zeros(16, np.uint64)
    assert lib.jy_node_exchange_plan(4, 4, W, 1, g.ctypes.data, e.ctypes.data, z.ctypes.data, z.ctypes.data, 1,
                                     ops.ctypes.data, C.byref(n)) != 0  # rank >= S
    assert lib.jy_node_exchange_plan(0, 0, W, 1, g.ctypes.data, e.ctypes.data, z.ctypes.data, z.ctypes.data, 1,
                                     ops.ctypes.data, C.byref(n)) != 0  # no shard
    g[0] = W
    assert lib.jy_node_exchange_plan(2, 0, W, 1, g.ctypes.data, e.ctypes.data, z.ctypes.data, z.ctypes.data, 1,
                                     ops.ctypes.data, C.byref(n)) != 0  # granule out of range
