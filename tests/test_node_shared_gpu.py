"""The node as the Pony host uses it since round 5: ONE node per process,
shared by the five RepoManager actors (jylis/database.pony:18-23), each
converging its own type's batches from its own thread; the calls enqueue and
one worker per node runs them in call order (include/jylis_gpu.h, "the
node").  Plus the RCCL shapes of a real multi-GPU node:

* every layout on one GPU: S = 1 over RCCL, S = 2 with the copy fabric, and
  the multi-process form (nlocal = 1 with a shared unique id) at world 1;
* with 2+ GPUs visible: one process driving two GPUs over RCCL, and two
  processes with one GPU each and a shared ncclUniqueId -- the cross-rank
  payload send/recv of the exchange (cluster.pony:205-213's counterpart).
  Skipped when fewer than 2 GPUs are visible.

After the batches, the union of the shards must equal ONE oracle repo that
converged every batch (RepoManagerCore.converge_deltas,
jylis/repo_manager.pony:92-93), bit-exact, and every key must live on its
owner."""
import os
import socket
import threading

import numpy as np
import pytest

from helpers import assert_state_equal, join_rows, random_history, split_rows

pytestmark = pytest.mark.gpu

TYPES = [0, 1, 2, 3, 4]


def _ndev():
    import torch
    return torch.cuda.device_count()


def _union_rows(ctype, node):
    from jylis_amd.engine import key_owner
    from jylis_amd.repo import REPOS
    rows = {}
    for sh, eng in enumerate(node.engines):
        part = dict(split_rows(ctype, REPOS[ctype](eng).state()))
        for k in part:
            assert key_owner(k, node.S) == node.rank0 + sh, (k, sh)
        rows.update(part)
    return rows


def _want(O, ctype, batches):
    ref = O.Repo(ctype)
    for b in batches:
        ref.converge(b)
    return join_rows(ctype, split_rows(ctype, ref.state()))


def _histories(O, seed):
    return {t: random_history(O, t, seed=seed + 7 * t, nops=140, nkeys=50) for t in TYPES}


def _replica_ids(batches):
    """every replica identity the batches name, in first-appearance order"""
    seen = {}
    for t in batches:
        for k in ("ids", "p_ids", "n_ids", "dot_ids", "vv_ids", "cloud_ids"):
            if k in t:
                for x in np.asarray(t[k], np.uint64).tolist():
                    seen.setdefault(int(x), None)
    return list(seen)


def _run_threads(node, hist):
    errors = []

    def work(ctype):
        try:
            for b in hist[ctype]:
                node.converge_table(ctype, b)
        except Exception as e:  # reported by the main thread
            errors.append((ctype, repr(e)))
    th = [threading.Thread(target=work, args=(t,)) for t in TYPES]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


@pytest.mark.parametrize("S,fabric", [(1, "rccl"), (2, "copy"), (8, "copy")])
def test_five_types_share_one_node(oracle_mod, S, fabric):
    """five threads (the five RepoManager actors) call one node at once; S = 8
    with the copy fabric is north_star's shard count on one GPU: every
    regroup, count and payload column of the 8-way exchange (everything but
    the RCCL calls, whose schedule tests/test_exchange_plan.py checks)"""
    from jylis_amd.node import Node
    O = oracle_mod
    hist = _histories(O, 500 + S)
    node = Node(S, fabric)
    try:
        _run_threads(node, hist)
        node.sync()
        for t in TYPES:
            assert_state_equal(t, _want(O, t, hist[t]), join_rows(t, _union_rows(t, node)))
        assert node.stats()["exchanges"] == sum(len(h) for h in hist.values())
    finally:
        node.close()


def test_calls_return_before_the_work(oracle_mod):
    """a converge call only enqueues: reads inside node.locked() see every
    call queued before the lock, and a queued job's failure is reported by
    the next call"""
    from jylis_amd.engine import EngineError, encode_keys
    from jylis_amd.node import Node
    from jylis_amd.repo import REPOS
    O = oracle_mod
    node = Node(1, "rccl")
    try:
        hist = random_history(O, O.TREG, seed=91, nops=120, nkeys=30)
        for b in hist:
            node.converge_table(O.TREG, b)
        with node.locked():  # waits for the queued calls, then holds the engines
            got = join_rows(O.TREG, dict(split_rows(O.TREG, REPOS[O.TREG](node.engines[0]).state())))
        assert_state_equal(O.TREG, _want(O, O.TREG, hist), got)
        # a device-side refusal (a value past the 16 MiB handle limit, device
        # inputs) fails the queued job; the next call reports it
        import torch
        kb, ko = encode_keys([b"big"])
        vo = np.array([0, (1 << 24) + 8], np.uint64)

        def dev(a):
            a = np.ascontiguousarray(a)
            return torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to("cuda:0")
        node.treg_converge(dev(kb), dev(ko), dev(np.array([5], np.uint64)),
                           torch.zeros((1 << 24) + 8, dtype=torch.uint8, device="cuda:0"), dev(vo))
        with pytest.raises(EngineError) as ei:
            node.sync()
        assert "16 MiB" in str(ei.value)
        node.sync()  # reported once
        # the device verdict is reset: a later device-input call goes through
        vb2, vo2 = encode_keys([b"fine value, 24 bytes ok"])
        node.treg_converge(dev(kb), dev(ko), dev(np.array([7], np.uint64)), dev(vb2), dev(vo2))
        node.sync()
    finally:
        node.close()


def test_typed_lock_does_not_wait_for_other_types(oracle_mod):
    """jy_node_lock_type (round 6): a TREG read under the lock returns once
    the TREG jobs queued before it are done, while UJSON converges queued
    after them are still waiting; the full lock waits for every job.  Both
    states equal the oracle's."""
    import torch
    from jylis_amd import synth as S
    from jylis_amd.node import Node
    from jylis_amd.repo import REPOS
    O = oracle_mod
    node = Node(1, "rccl")

    def dev(a):
        a = np.ascontiguousarray(a)
        return torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to("cuda:0")
    try:
        tr = random_history(O, O.TREG, seed=93, nops=120, nkeys=40)
        st0, dl = S.ujson_tables(200000, seed=S.BASE_SEED + 77, rounds=1, R=16)
        uj = [st0] + dl * 10  # (re-delivered deltas: idempotent)
        args = [[dev(a) for a in node.ujson_args(b)] for b in (st0, dl[0])]
        for b in tr:
            node.converge_table(O.TREG, b)
        # device inputs: the calls only enqueue (no pinned staging to wait
        # for), so the UJSON jobs queue up behind the TREG ones
        node.ujson_converge(*args[0])
        for _ in range(10):
            node.ujson_converge(*args[1])
        with node.locked(O.TREG):
            waiting = node.pending(O.UJSON)
            got = join_rows(O.TREG, dict(split_rows(O.TREG, REPOS[O.TREG](node.engines[0]).state())))
        assert waiting > 0, "the TREG lock waited for the UJSON jobs"
        assert_state_equal(O.TREG, _want(O, O.TREG, tr), got)
        with node.locked():
            assert node.pending() == 0
        node.sync()
        assert_state_equal(O.UJSON, _want(O, O.UJSON, uj), join_rows(O.UJSON, _union_rows(O.UJSON, node)))
        # deltas_size / flush style access: no fence at all
        node.converge_table(O.UJSON, dl[0])
        with node.locked(Node.NOFENCE):
            pass
        node.sync()
    finally:
        node.close()


def test_multiprocess_form_at_world_one(oracle_mod):
    """the multi-process constructor (nlocal = 1, a shared ncclUniqueId) at
    one rank: the communicator made from a unique id another call produced"""
    from jylis_amd.node import Node, unique_id
    O = oracle_mod
    hist = _histories(O, 900)
    node = Node(1, "rccl", devices=[0], nlocal=1, rank0=0, uid=unique_id())
    try:
        for t in TYPES:
            for b in hist[t]:
                node.converge_table(t, b)
        node.sync()
        for t in TYPES:
            assert_state_equal(t, _want(O, t, hist[t]), join_rows(t, _union_rows(t, node)))
    finally:
        node.close()


@pytest.mark.skipif("not __import__('torch').cuda.device_count() >= 2", reason="needs 2 GPUs")
def test_one_process_two_gpus_rccl(oracle_mod):
    """one process, two GPUs, one RCCL communicator: every payload column of
    the exchange crosses between the GPUs with grouped ncclSend/ncclRecv"""
    from jylis_amd.node import Node
    O = oracle_mod
    hist = _histories(O, 1300)
    node = Node(2, "rccl", devices=[0, 1])
    try:
        _run_threads(node, hist)
        node.sync()
        for t in TYPES:
            assert_state_equal(t, _want(O, t, hist[t]), join_rows(t, _union_rows(t, node)))
        st = node.stats()
        assert st["bytes_sent"] > 0
    finally:
        node.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _empty_table(O, ctype):
    return O.Repo(ctype, 1).flush().table()


def _proc(rank, world, uid, rids, q, seed):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here]
    try:
        import oracle as O
        O.load()
        from jylis_amd.node import Node
        hist = _histories(O, seed)
        node = Node(world, "rccl", devices=[rank], nlocal=1, rank0=rank, uid=uid)
        node.replica_cols(rids)  # one registration order on every process (the header's contract)
        for t in TYPES:
            h = hist[t]
            for j in range((len(h) + world - 1) // world):  # collectives: the same number of calls everywhere
                i = j * world + rank
                node.converge_table(t, h[i] if i < len(h) else _empty_table(O, t))
        node.sync()
        for t in TYPES:
            q.put(("rows", rank, t, _union_rows(t, node)))
        node.close()
    except Exception:
        import traceback
        q.put(("error", rank, traceback.format_exc()))
        raise


@pytest.mark.skipif("not __import__('torch').cuda.device_count() >= 2", reason="needs 2 GPUs")
def test_two_processes_shared_unique_id(oracle_mod):
    """two processes, one GPU each, one communicator from a shared
    ncclUniqueId (jy_node_unique_id): each converges its half of every
    type's history; the union of the two shards equals one oracle repo"""
    import multiprocessing as mp

    from helpers import collect
    from jylis_amd.node import unique_id
    O = oracle_mod
    world, seed = 2, 1700
    hist = _histories(O, seed)
    rids = _replica_ids([b for h in hist.values() for b in h])
    uid = unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_proc, args=(r, world, uid, rids, q, seed)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = collect(procs, q, world * len(TYPES))
    for t in TYPES:
        rows = {}
        for m in msgs:
            if m[2] == t:
                assert not set(rows) & set(m[3]), "a key on two shards"
                rows.update(m[3])
        assert_state_equal(t, _want(O, t, hist[t]), join_rows(t, rows))
