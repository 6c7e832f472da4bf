"""GCOUNT / PNCOUNT: the HIP engine against the CPU oracle (bit-exact).

Streams: oracle write-path histories (INC/DEC on several replicas with
gossip, including wrap-around values), the synthetic config-1/2 shapes at
reduced size, and the dense column-block path at sizes the oracle finishes
in seconds."""
import numpy as np
import pytest

from helpers import assert_state_equal, random_history

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ctype", [0, 1])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_history_parity(oracle_mod, engine, ctype, seed):
    from jylis_amd.repo import REPOS
    O = oracle_mod
    want = O.Repo(ctype, 12345)
    got = REPOS[ctype](engine)
    for b in random_history(O, ctype, seed):
        want.converge(b)
        got.converge_deltas(b)
    assert_state_equal(ctype, want.state(), got.state())
    keys = [f"k{i}" for i in range(14)]  # two never-written keys read as 0
    exp = [(want.gcount_get if ctype == 0 else want.pncount_get)(k) for k in keys]
    np.testing.assert_array_equal(got.get(keys).astype(np.int64 if ctype else np.uint64), np.array(exp, dtype=np.int64 if ctype else np.uint64))


def test_test_cluster_on_gpu(oracle_mod, engine):
    """test_cluster.pony:117-129 through the GPU repo: 2 + 3 + 4 -> 9"""
    from jylis_amd.repo import RepoGCOUNT
    O = oracle_mod
    writers = [O.Repo(O.GCOUNT, i + 1) for i in range(3)]
    for r, v in zip(writers, (2, 3, 4)):
        r.gcount_inc("foo", v)
    gpu = RepoGCOUNT(engine)
    for r in writers:
        gpu.converge_deltas(r.flush().table())
    assert int(gpu.get(["foo"])[0]) == 9


@pytest.mark.parametrize("ctype,K,R", [(0, 6000, 8), (1, 6000, 8), (0, 1500, 64), (1, 1500, 64)])
def test_synthetic_block_and_coo(oracle_mod, engine, ctype, K, R):
    """config-1/2 shaped stream (every peer batch = one replica column over all
    keys): dense block path for half the rounds, COO for the rest.  R=64 is
    config 2's replica count (the headline's k_block_max launch shape)"""
    from jylis_amd import synth as S
    from jylis_amd.repo import REPOS
    O = oracle_mod
    nsigns = 1 if ctype == 0 else 2
    seed = S.BASE_SEED + 1 + ctype
    kb, ko = S.counter_keys(K, prefix=b"g" if ctype == 0 else b"p")
    rids = S.replica_ids(R, seed)
    want = O.Repo(ctype, 1)
    got = REPOS[ctype](engine)
    st = S.counter_state_np(K, R, nsigns, seed, wrap_frac=(ctype == 1))
    batches = [st]
    cur = st
    for rnd in range(4):
        cur = S.counter_delta_np(cur, rnd, seed)
        batches.append(cur)
    slots = got._intern({"key_bytes": kb, "key_offs": ko})
    assert (slots == np.arange(K)).all()
    cols = engine.replica_cols(rids.tolist())
    for i, arr in enumerate(batches):
        for t in S.counter_batch_tables(arr if ctype == 1 else arr[0], rids, (kb, ko)):
            want.converge(t)
        if i % 2 == 0:
            if ctype == 0:
                engine.gcount_converge_block(cols, 0, arr[0])
            else:
                engine.pncount_converge_block(cols, 0, arr[0], arr[1])
        else:
            for t in S.counter_batch_tables(arr if ctype == 1 else arr[0], rids, (kb, ko)):
                got.converge_deltas(t)
    dump = engine.counter_export(ctype, R, 0, K)
    exp = batches[0].copy()
    for b in batches[1:]:
        exp = np.maximum(exp, b)
    assert (cols == np.arange(R)).all()  # fresh engine: columns in registration order
    np.testing.assert_array_equal(dump, exp)
    assert_state_equal(ctype, want.state(), got.state())
    getter = want.gcount_get if ctype == 0 else want.pncount_get
    sample = np.arange(0, K, 97)
    exp_v = np.array([getter(bytes(kb[ko[i]:ko[i + 1]])) for i in sample])
    got_v = (engine.gcount_get if ctype == 0 else engine.pncount_get)(sample.astype(np.uint32))
    np.testing.assert_array_equal(got_v.astype(np.int64), exp_v.astype(np.int64))


def test_block_unaligned_run(engine):
    """odd slot0 / odd nslots use the scalar kernel; results equal numpy max"""
    from jylis_amd import synth as S
    K, R = 1001, 3
    kb, ko = S.counter_keys(K)
    engine.intern(0, (kb, ko))
    cols = engine.replica_cols([11, 22, 33])
    a = S.counter_state_np(K, R, 1, 7)[0]
    engine.gcount_converge_block(cols, 0, a)
    b = S.counter_delta_np(a[:, 1:], 0, 9)  # [R][1000] starting at slot 1
    engine.gcount_converge_block(cols, 1, np.ascontiguousarray(b))
    exp = a.copy()
    exp[:, 1:] = np.maximum(exp[:, 1:], b)
    np.testing.assert_array_equal(engine.counter_export(0, R, 0, K)[0], exp)


def test_empty_and_missing(engine):
    from jylis_amd.repo import RepoGCOUNT, RepoPNCOUNT
    g = RepoGCOUNT(engine)
    g.converge_deltas({"key_bytes": np.zeros(0, np.uint8), "key_offs": np.zeros(1, np.uint64),
                       "offs": np.zeros(1, np.uint64), "ids": np.zeros(0, np.uint64), "vals": np.zeros(0, np.uint64)})
    assert g.get(["nope"])[0] == 0
    p = RepoPNCOUNT(engine)
    assert p.get(["nope"])[0] == 0
    # a batch of the wrong type is swallowed (repo_gcount.pony:51 `try ... end`)
    g.converge_deltas({"key_bytes": np.frombuffer(b"x", np.uint8), "key_offs": np.array([0, 1], np.uint64)},
                      ctype=1)
    assert engine.nkeys(0) == 0
