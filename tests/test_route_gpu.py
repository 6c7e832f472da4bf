"""The routing data plane on the GPU: partition kernels, the fixed-capacity
all-to-all and the routed merge, with S shards hosted in one process
(route.LocalFabric: S engines on cuda:0, the all-to-all as device copies).

After routing, the union of the shards must equal ONE oracle repo that
converged every ingested batch (TREG: repo_treg.pony:51-52; counters:
repo_pncount.pony:52-53) -- bit-exact, including overflowing runs (drain
rounds), keys several sources send in the same step, and long values whose
bytes travel in their own run."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# LocalFabric modes: "async" runs every async all-to-all on a side stream
# behind a spin delay, so a router that read its runs before wait() would see
# stale buffers (the ordering contract of RCCL's async collectives)
FABRIC = {"sync": {}, "async": {"async_copies": True, "delay_cycles": 400000}}


def _treg_batch(rng, n, keyspace, ts_hi=4):
    from jylis_amd.engine import encode_keys
    keys = [f"rk{int(x)}" for x in rng.choice(keyspace, n, replace=False)]
    vals = []
    for _ in keys:
        L = int(rng.integers(0, 24))
        vals.append(bytes(rng.integers(0, 256, L).astype(np.uint8)) if rng.random() < 0.7
                    else b"shared-prefix"[:min(L, 13)] + bytes(rng.integers(97, 99, max(L - 13, 0)).astype(np.uint8)))
    ts = rng.integers(0, ts_hi, n).astype(np.uint64)
    kb, ko = encode_keys(keys)
    vb, vo = encode_keys(vals)
    return {"key_bytes": kb, "key_offs": ko, "ts": ts, "val_bytes": vb, "val_offs": vo}


def _dev(a, dtype):
    import torch
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to("cuda:0")


class _Node:
    """S engines on one GPU + per-shard slot directories (the control plane's
    role: owner hash, owner-side interning)"""

    def __init__(self, S):
        from jylis_amd.engine import Engine
        from jylis_amd.repo import RepoTREG
        self.S = S
        self.engs = [Engine(device=0) for _ in range(S)]
        self.repos = [RepoTREG(e) for e in self.engs]

    def close(self):
        for e in self.engs:
            e.close()

    def ingest(self, rank, b):
        """(owner, owner slot, ts, pre, lr, long bytes) of a batch landing on `rank`"""
        from jylis_amd._lib import TREG
        from jylis_amd.route import owners
        own = owners(b["key_bytes"], b["key_offs"], self.S)
        slot = np.zeros(len(own), np.uint32)
        for d in range(self.S):
            idx = np.nonzero(own == d)[0]
            if len(idx):
                from jylis_amd.route import _pick_keys
                kb, ko = _pick_keys(np.asarray(b["key_bytes"], np.uint8), np.asarray(b["key_offs"], np.uint64), idx)
                slot[idx] = self.repos[d]._intern({"key_bytes": kb, "key_offs": ko})
        from jylis_amd.route import long_bytes
        pre, lr = self.engs[rank].pack_values(TREG, (b["val_bytes"], b["val_offs"]))
        nbytes = long_bytes(lr)
        return (_dev(own, np.uint32), _dev(slot, np.uint32), _dev(b["ts"], np.uint64), _dev(pre, np.uint64),
                _dev(lr, np.uint64), nbytes)

    def union_state(self):
        """merged state tables of the shards (each shard holds only its own keys)"""
        from jylis_amd.route import owners
        out = {}
        for d, r in enumerate(self.repos):
            st = r.state()
            kb, ko = st["key_bytes"], st["key_offs"]
            for i in range(len(ko) - 1):
                k = bytes(kb[ko[i]:ko[i + 1]])
                assert owners(np.frombuffer(k, np.uint8), np.array([0, len(k)], np.uint64), self.S)[0] == d
                out[k] = (int(st["ts"][i]), bytes(st["val_bytes"][st["val_offs"][i]:st["val_offs"][i + 1]]))
        return out


def _oracle_dict(O, batches):
    ref = O.Repo(O.TREG)
    for b in batches:
        ref.converge(b)
    st = ref.state()
    return {k: (int(t), bytes(st["val_bytes"][st["val_offs"][i]:st["val_offs"][i + 1]]))
            for i, (k, t) in enumerate(zip(O.split_keys(st), st["ts"]))}


@pytest.mark.parametrize("direct", [None, True, False])
@pytest.mark.parametrize("fab", sorted(FABRIC))
@pytest.mark.parametrize("S", [1, 2, 3])
def test_treg_routed_local_fabric(oracle_mod, S, fab, direct):
    """every rank ingests its own batch over a shared key space; keys that
    several ranks ingest in the same step meet in one merge launch.  `direct`:
    each shard merges its own entries where they lie (jy_treg_route_part_self)
    or routes them through its own run; None = the router's default (S <= 2)"""
    from jylis_amd.route import LocalFabric, TregRouter
    rng = np.random.default_rng(40 + S)
    node = _Node(S)
    try:
        router = TregRouter(node.engs, LocalFabric(S, **FABRIC[fab]), self_direct=direct)
        seen = []
        for _ in range(4):
            bs = [_treg_batch(rng, 2500, 4000) for _ in range(S)]
            seen += bs
            router.step([node.ingest(r, b) for r, b in enumerate(bs)])
        router.drain()
        for e in node.engs:
            e.sync()
        assert node.union_state() == _oracle_dict(oracle_mod, seen)
    finally:
        node.close()


def test_treg_routed_overflow_drains(oracle_mod):
    """a batch whose keys all belong to one owner overflows its run: the
    overflow is listed on the device and routed by a drain round"""
    from jylis_amd.engine import encode_keys
    from jylis_amd.route import LocalFabric, TregRouter, owners
    S = 2
    rng = np.random.default_rng(7)
    cand = [f"ov{i}" for i in range(20000)]
    kb, ko = encode_keys(cand)
    own = owners(kb, ko, S)
    hot = [k for k, o in zip(cand, own) if o == 1][:6000]
    node = _Node(S)
    try:
        router = TregRouter(node.engs, LocalFabric(S))
        seen = []
        for rnd in range(2):
            bs = []
            for r in range(S):
                keys = [hot[int(i)] for i in rng.choice(len(hot), 5000, replace=False)]
                vals = [bytes(rng.integers(97, 123, int(rng.integers(0, 20))).astype(np.uint8)) for _ in keys]
                kb2, ko2 = encode_keys(keys)
                vb, vo = encode_keys(vals)
                bs.append({"key_bytes": kb2, "key_offs": ko2, "ts": rng.integers(0, 3, 5000).astype(np.uint64),
                           "val_bytes": vb, "val_offs": vo})
            seen += bs
            router.step([node.ingest(r, b) for r, b in enumerate(bs)])
        router.drain()
        assert router.drains >= 1
        assert node.union_state() == _oracle_dict(oracle_mod, seen)
    finally:
        node.close()


@pytest.mark.parametrize("fab", sorted(FABRIC))
def test_treg_routed_full_overlap(oracle_mod, fab):
    """every key arrives from ALL S sources in one routed step
    (every peer flushed the same hot keys): the owners merge the sources'
    runs one launch per source, so the overlapping keys are exact and never
    pile up in the duplicate fold"""
    from jylis_amd.route import LocalFabric, TregRouter
    S = 3
    rng = np.random.default_rng(123)
    node = _Node(S)
    try:
        router = TregRouter(node.engs, LocalFabric(S, **FABRIC[fab]))
        seen = []
        keys = rng.choice(6000, 3000, replace=False)
        for rnd in range(3):
            bs = []
            for r in range(S):
                b = _treg_batch(np.random.default_rng(1000 * rnd + r), 3000, 6000, ts_hi=3)
                # the same key set on every source (values and timestamps differ)
                from jylis_amd.engine import encode_keys
                kb, ko = encode_keys([f"rk{int(x)}" for x in keys])
                b["key_bytes"], b["key_offs"] = kb, ko
                bs.append(b)
            seen += bs
            router.step([node.ingest(r, b) for r, b in enumerate(bs)])
        router.drain()
        assert node.union_state() == _oracle_dict(oracle_mod, seen)
    finally:
        node.close()


def test_treg_device_batch_many_repeats(oracle_mod):
    """a device batch naming each of its keys up to 12 times: the parallel
    fold rounds take the first few occurrences, the one-wave fold the rest"""
    from jylis_amd._lib import TREG
    from jylis_amd.engine import Engine, encode_keys
    from jylis_amd.repo import RepoTREG
    rng = np.random.default_rng(5)
    eng = Engine(device=0)
    try:
        repo = RepoTREG(eng)
        names = [f"m{i}" for i in range(2000)]
        kb, ko = encode_keys(names)
        slots = repo._intern({"key_bytes": kb, "key_offs": ko})
        reps = rng.integers(1, 13, len(names))
        idx = rng.permutation(np.repeat(np.arange(len(names)), reps))
        vals = [bytes(rng.integers(97, 100, int(rng.integers(0, 14))).astype(np.uint8)) for _ in idx]
        ts = rng.integers(0, 4, len(idx)).astype(np.uint64)
        pre, lr = eng.pack_values(TREG, vals)
        eng.treg_converge(_dev(slots[idx], np.uint32), _dev(ts, np.uint64), _dev(pre, np.uint64),
                          _dev(lr, np.uint64))
        want = O_dict = {}
        for i, v, t in zip(idx, vals, ts):
            k = names[i].encode()
            cand = (int(t), v)
            if k not in want or cand > want[k]:
                want[k] = cand
        st = repo.state()
        got = {k: (int(t), bytes(st["val_bytes"][st["val_offs"][i]:st["val_offs"][i + 1]]))
               for i, (k, t) in enumerate(zip(oracle_mod.split_keys(st), st["ts"]))}
        assert got == O_dict
    finally:
        eng.close()


def _keys_dev(keys):
    import torch
    from jylis_amd.engine import encode_keys
    kb, ko = encode_keys(keys)
    return (torch.from_numpy(np.ascontiguousarray(kb, np.uint8)).to("cuda:0"),
            torch.from_numpy(np.asarray(ko, np.uint64).view(np.int64)).to("cuda:0"))


@pytest.mark.parametrize("S", [1, 2, 3])
def test_key_resolver_on_device(oracle_mod, S):
    """cross-shard key resolution on the GPU (k_keyroute.hip,
    route.KeyResolver): owners hashed on the device equal jy_key_owner; every
    key's slot names that key in its owner's directory; a key gets one slot
    whichever rank ingests it, and repeated within a batch; an empty batch,
    the empty key and keys past 8 bytes ride along; the TREG data plane routed
    with those slots equals one oracle repo"""
    from jylis_amd._lib import TREG
    from jylis_amd.engine import encode_keys
    from jylis_amd.route import KeyResolver, LocalFabric, TregRouter, long_bytes, owners
    rng = np.random.default_rng(70 + S)
    node = _Node(S)
    try:
        fab = LocalFabric(S)
        kr = KeyResolver(node.engs, fab, TREG)
        router = TregRouter(node.engs, fab)
        slot_of = {}
        seen = []
        for rnd in range(3):
            keysets, per = [], []
            for r in range(S):
                n = 0 if (rnd == 1 and r == S - 1) else 1500
                keys = [f"rk{int(x)}" + ("-long-key-suffix" if int(x) % 7 == 0 else "")
                        for x in rng.integers(0, 4000, n)]  # repeats inside the batch
                if n and rnd == 2:
                    keys[0] = ""
                per.append(keys)
                keysets.append(_keys_dev(keys))
            res = kr.resolve(keysets)
            batches = []
            for r, (keys, (own, slot)) in enumerate(zip(per, res)):
                own_h = own.cpu().numpy().view(np.uint32)
                slot_h = slot.cpu().numpy().view(np.uint32)
                kb, ko = encode_keys(keys)
                assert (own_h == owners(kb, ko, S)).all()
                for k, o, sl in zip(keys, own_h, slot_h):
                    assert slot_of.setdefault(k, (int(o), int(sl))) == (int(o), int(sl))
                # one delta per key per batch (the contract of a flushed batch)
                first = {}
                for i, k in enumerate(keys):
                    first.setdefault(k, i)
                idx = np.array(sorted(first.values()), np.int64)
                ks = [keys[i] for i in idx]
                vals = [bytes(rng.integers(97, 100, int(rng.integers(0, 20))).astype(np.uint8)) for _ in ks]
                ts = rng.integers(0, 4, len(ks)).astype(np.uint64)
                kb2, ko2 = encode_keys(ks)
                vb, vo = encode_keys(vals)
                seen.append({"key_bytes": kb2, "key_offs": ko2, "ts": ts, "val_bytes": vb, "val_offs": vo})
                pre, lr = node.engs[r].pack_values(TREG, vals)
                batches.append((_dev(own_h[idx], np.uint32), _dev(slot_h[idx], np.uint32), _dev(ts, np.uint64),
                                _dev(pre, np.uint64), _dev(lr, np.uint64), long_bytes(lr)))
            router.step(batches)
        router.drain()
        for d, repo in enumerate(node.repos):
            repo._sync_names()
        for k, (o, sl) in slot_of.items():
            assert node.repos[o].names[sl] == k.encode()
        assert node.union_state() == _oracle_dict(oracle_mod, seen)
    finally:
        node.close()


def test_treg_arena_collect_waits_for_drain(oracle_mod):
    """a drain round re-reads the long-value bytes of a pending
    batch through its handles, so collecting the sending engine's arena
    between step() and drain() would route the wrong bytes.  Collection is
    refused while rounds are in flight; after drain() it runs, and the state
    (long values included) stays exact"""
    from jylis_amd._lib import TREG
    from jylis_amd.engine import encode_keys
    from jylis_amd.route import LocalFabric, TregRouter, owners
    S = 2
    rng = np.random.default_rng(11)
    cand = [f"ac{i}" for i in range(20000)]
    kb, ko = encode_keys(cand)
    hot = [k for k, o in zip(cand, owners(kb, ko, S)) if o == 0][:5000]
    node = _Node(S)
    try:
        router = TregRouter(node.engs, LocalFabric(S))
        seen = []
        for rnd in range(3):
            bs = []
            for r in range(S):
                keys = [hot[int(i)] for i in rng.choice(len(hot), 4000, replace=False)]
                vals = [b"long-value-%d-%d-" % (rnd, r) + bytes(rng.integers(97, 123, 12).astype(np.uint8))
                        for _ in keys]
                kb2, ko2 = encode_keys(keys)
                vb, vo = encode_keys(vals)
                bs.append({"key_bytes": kb2, "key_offs": ko2, "ts": np.full(4000, rnd, np.uint64),
                           "val_bytes": vb, "val_offs": vo})
            seen += bs
            router.step([node.ingest(r, b) for r, b in enumerate(bs)])
            for e in node.engs:
                with pytest.raises(RuntimeError):
                    e.arena_collect(TREG)
        router.drain(collect=True)
        assert router.drains >= 1
        for e in node.engs:
            e.arena_collect(TREG)  # no rounds in flight: allowed
        assert node.union_state() == _oracle_dict(oracle_mod, seen)
    finally:
        node.close()


@pytest.mark.parametrize("flags", [0, 1])
def test_treg_device_batch_repeated_keys(oracle_mod, flags):
    """a device batch naming keys several times (ADVICE: k_treg_lww had no
    in-launch duplicate handling) converges exactly, in both kernel forms
    (flags=1 forces k_treg_lww<true>, the >MALL whole-line form)"""
    import torch

    from helpers import assert_state_equal
    from jylis_amd._lib import TREG
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoTREG
    O = oracle_mod
    rng = np.random.default_rng(11 + flags)
    eng = Engine(device=0, flags=flags)
    try:
        got = RepoTREG(eng)
        want = O.Repo(O.TREG)
        for rnd in range(5):
            b = _treg_batch(rng, 3000, 4000)
            # repeat ~30% of the entries at random positions (some several times)
            rep = rng.integers(0, 3000, 1500)
            order = rng.permutation(3000 + 1500)
            keys = O.split_keys(b) + [O.split_keys(b)[i] for i in rep]
            vb, vo = b["val_bytes"], b["val_offs"]
            vals = [bytes(vb[vo[i]:vo[i + 1]]) for i in range(3000)]
            vals += [bytes(rng.integers(97, 100, int(rng.integers(0, 20))).astype(np.uint8)) for _ in rep]
            ts = np.concatenate([b["ts"], rng.integers(0, 4, len(rep)).astype(np.uint64)])
            keys = [keys[i] for i in order]
            vals = [vals[i] for i in order]
            ts = ts[order]
            from jylis_amd.engine import encode_keys
            kb, ko = encode_keys(keys)
            for k, v, t in zip(keys, vals, ts):
                want.converge({"key_bytes": np.frombuffer(k, np.uint8), "key_offs": np.array([0, len(k)], np.uint64),
                               "ts": np.array([t], np.uint64), "val_bytes": np.frombuffer(v, np.uint8),
                               "val_offs": np.array([0, len(v)], np.uint64)})
            slots = got._intern({"key_bytes": kb, "key_offs": ko})
            pre, lr = eng.pack_values(TREG, vals)
            eng.treg_converge(_dev(slots, np.uint32), _dev(ts, np.uint64), _dev(pre, np.uint64), _dev(lr, np.uint64))
            torch.cuda.synchronize()
        assert_state_equal(O.TREG, want.state(), got.state())
    finally:
        eng.close()


def test_treg_whole_line_kernel_matches_oracle(oracle_mod):
    """k_treg_lww<true> (picked for states over the 256 MiB MALL, ~11.2M+
    slots) on the config-shaped stream: fresh timestamps, dense ties, shared
    prefixes, long values"""
    from helpers import assert_state_equal
    from jylis_amd._lib import CFG_TREG_WHOLE_LINES, TREG
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoTREG
    O = oracle_mod
    rng = np.random.default_rng(3)
    eng = Engine(device=0, flags=CFG_TREG_WHOLE_LINES)
    try:
        got = RepoTREG(eng)
        want = O.Repo(O.TREG)
        for j in range(4):
            b = _treg_batch(rng, 20000, 20000, ts_hi=1 << 3)
            b["ts"] = b["ts"] + np.uint64(j * 2)
            want.converge(b)
            got.converge_deltas(b)
        assert_state_equal(O.TREG, want.state(), got.state())
    finally:
        eng.close()


def test_treg_set_repeated_keys_device(oracle_mod):
    """local SETs on the device with repeated keys: state and flushed delta
    equal the oracle's sequential RepoTREG.set (repo_treg.pony:65-68)"""
    import torch

    from jylis_amd._lib import TREG
    from jylis_amd.engine import Engine, encode_keys
    from jylis_amd.repo import RepoTREG
    from helpers import assert_state_equal
    O = oracle_mod
    rng = np.random.default_rng(5)
    eng = Engine(device=0)
    try:
        got = RepoTREG(eng)
        want = O.Repo(O.TREG, 5)
        keys = [f"s{int(i)}" for i in rng.integers(0, 300, 2000)]
        vals = [bytes(rng.integers(97, 100, int(rng.integers(0, 14))).astype(np.uint8)) for _ in keys]
        ts = rng.integers(0, 5, len(keys)).astype(np.uint64)
        for k, v, t in zip(keys, vals, ts):
            want.treg_set(k, v, int(t))
        kb, ko = encode_keys(keys)
        slots = got._intern({"key_bytes": kb, "key_offs": ko})
        pre, lr = eng.pack_values(TREG, vals)
        eng.treg_set(_dev(slots, np.uint32), _dev(ts, np.uint64), _dev(pre, np.uint64), _dev(lr, np.uint64))
        torch.cuda.synchronize()
        assert_state_equal(O.TREG, want.state(), got.state())

        def by_key(t):
            return {k: (int(x), bytes(t["val_bytes"][t["val_offs"][i]:t["val_offs"][i + 1]]))
                    for i, (k, x) in enumerate(zip(O.split_keys(t), t["ts"]))}
        assert by_key(got.flush_deltas()) == by_key(want.flush().table())
    finally:
        eng.close()


@pytest.mark.parametrize("fab", sorted(FABRIC))
@pytest.mark.parametrize("S", [2, 3])
def test_pncount_routed_local_fabric(S, fab):
    """dense PNCOUNT peer batches grouped by owner, exchanged column by
    column (double-buffered) and block-merged on the owners; checked against
    a numpy max over everything ingested"""
    import torch

    from jylis_amd._lib import PNCOUNT
    from jylis_amd.engine import Engine
    from jylis_amd.route import CounterRouter, LocalFabric
    from jylis_amd import synth as Sy
    K, Cn = 4096, 3
    engs = [Engine(device=0, counter_columns=S * Cn) for _ in range(S)]
    try:
        for r, e in enumerate(engs):
            e.intern(PNCOUNT, Sy.counter_keys(K, prefix=f"o{r}:".encode()))
        rids = Sy.replica_ids(S * Cn, 77)
        cols = []
        for e in engs:
            cols.append(e.replica_cols(rids.tolist()))
        assert all((c == cols[0]).all() for c in cols)  # one registration order on every shard
        peer_cols = [[int(cols[0][r * Cn + c]) for c in range(Cn)] for r in range(S)]
        router = CounterRouter(engs, LocalFabric(S, **FABRIC[fab]), PNCOUNT)
        rng = np.random.default_rng(S)
        want = [np.zeros((2, S * Cn, K), np.uint64) for _ in range(S)]
        for rnd in range(3):
            ing = []
            for r in range(S):
                v = rng.integers(0, 1 << 62, (2, Cn, S, K), dtype=np.uint64)
                v[:, :, :, :7] = np.uint64(2**64 - 3)  # wrap edge
                ing.append(torch.from_numpy(v.view(np.int64)).to("cuda:0"))
                for d in range(S):
                    for c in range(Cn):
                        w = want[d][:, peer_cols[r][c]]
                        np.maximum(w, v[:, c, d], out=w)
            router.step(ing, peer_cols)
        for d, e in enumerate(engs):
            got = e.counter_export(PNCOUNT, S * Cn, 0, K)
            np.testing.assert_array_equal(got, want[d])
            sums = e.pncount_get(np.arange(K, dtype=np.uint32))
            exp = (want[d][0].sum(axis=0, dtype=np.uint64) - want[d][1].sum(axis=0, dtype=np.uint64)).view(np.int64)
            np.testing.assert_array_equal(sums, exp)
    finally:
        for e in engs:
            e.close()
