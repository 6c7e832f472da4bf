"""TLOG: the HIP segmented merge against the CPU oracle (bit-exact).

Edge cases: (ts, value) duplicates across state and delta, timestamp ties
broken by Pony String order (long values sharing 8-byte prefixes), cutoffs
that drop state entries / delta entries / everything, CLR at ts 2^64-1
(cutoff wraps to 0: no-op), TRIM past the end, keys with a cutoff but no
entries, repeated keys in one batch, malformed (unsorted) delta segments."""
import numpy as np
import pytest

from helpers import assert_state_equal, random_history

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_history_parity(oracle_mod, engine, seed):
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    want = O.Repo(O.TLOG)
    got = RepoTLOG(engine)
    for b in random_history(O, O.TLOG, seed, nops=400, val_len=20):
        want.converge(b)
        got.converge_deltas(b)
    assert_state_equal(O.TLOG, want.state(), got.state())


def _log_batch(logs):
    """logs: list of (key, cutoff, [(value, ts), ...]) -> batch table (entries as given)"""
    from jylis_amd.engine import encode_keys
    kb, ko = encode_keys([k for k, _, _ in logs])
    vals, ts, offs = [], [], [0]
    for _, _, ents in logs:
        for v, t in ents:
            vals.append(v)
            ts.append(t)
        offs.append(len(vals))
    vb, vo = encode_keys(vals)
    return {"key_bytes": kb, "key_offs": ko, "cutoff": np.array([c for _, c, _ in logs], np.uint64),
            "ent_offs": np.array(offs, np.uint64), "ts": np.array(ts, np.uint64), "val_bytes": vb, "val_offs": vo}


def _canon(ents):
    """sort + dedupe as a pony TLog would hold them (later ts, then greater value first)"""
    return sorted(set(ents), key=lambda e: (e[1], e[0]), reverse=True)


def test_edge_cases(oracle_mod, engine):
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    big = (1 << 64) - 1
    P = b"prefix!!"  # 8-byte shared prefix
    state = [
        ("dup", 0, _canon([(b"a", 5), (b"b", 5), (b"c", 4)])),
        ("tie", 0, _canon([(P + b"zz", 9), (P + b"a", 9), (P, 9), (b"x", 1)])),
        ("cut", 0, _canon([(b"v%d" % i, i) for i in range(10)])),
        ("cutall", 0, _canon([(b"q", 3), (b"r", 2)])),
        ("wrap", 0, _canon([(b"max", big), (b"low", 1)])),
        ("onlycut", 7, []),
        ("empty", 0, []),
    ]
    delta = [
        ("dup", 0, _canon([(b"b", 5), (b"c", 4), (b"d", 4)])),
        ("tie", 0, _canon([(P + b"zy", 9), (P + b"\x00", 9), (P + b"zz", 9)])),
        ("cut", 6, _canon([(b"v9", 9), (b"new", 7), (b"old", 2)])),
        ("cutall", 100, []),
        ("wrap", 0, []),
        ("onlycut", 3, _canon([(b"late", 8), (b"early", 2)])),
        ("fresh", 0, _canon([(b"", 0), (b"\xff" * 12, 0)])),
    ]
    want = O.Repo(O.TLOG)
    got = RepoTLOG(engine)
    for logs in (state, delta, state):
        b = _log_batch(logs)
        want.converge(b)
        got.converge_deltas(b)
    assert_state_equal(O.TLOG, want.state(), got.state())
    assert got.cutoff("cutall") == 100 and got.size("cutall") == 0
    assert got.get("tie", 2) == [(P + b"zz", 9), (P + b"zy", 9)]
    assert got.get("missing") == [] and got.size("missing") == 0 and got.cutoff("missing") == 0


def test_slow_key_mixes(oracle_mod, engine):
    """slow keys (k_tlog_tile stage 2) whose deltas start with entries newer
    than the log and go on with: a timestamp tie right after them, a duplicate
    or an interleaving entry (in-place insert), a cutoff raise, more than four
    newer entries, a segment that overflows (rebuild, one entry searched),
    each against the oracle over two deltas"""
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    base = [(b"v%d" % i, i) for i in range(1, 11)]  # ts 1..10
    state = [("tie", 0, _canon(base)), ("dup", 0, _canon(base)), ("ins", 0, _canon(base)),
             ("cut", 0, _canon(base)), ("many", 0, _canon(base)), ("grow", 0, [(b"g", 1)]),
             ("grow2", 0, [(b"g", 1)]), ("grow3", 0, [(b"g", 5)])]
    d1 = [("tie", 0, [(b"n2", 20), (b"t", 15), (b"n1", 15)]),          # tie after the prefix (value order)
          ("dup", 0, [(b"x", 30), (b"y", 25), (b"v3", 3)]),            # a duplicate of a state entry
          ("ins", 0, [(b"x", 30), (b"z", 5), (b"a", 4)]),              # interleaves: inserted in place
          ("cut", 6, [(b"x", 40), (b"y", 35), (b"old", 2)]),           # cutoff raise: old dropped
          ("many", 0, [(b"m%d" % i, 60 - i) for i in range(7)]),     # 7 newer entries (prefix of 4)
          ("grow", 0, [(b"n%d" % i, 100 - i) for i in range(12)]),   # past the segment: rebuilt
          ("grow2", 0, [(b"p%d" % i, 50 - i) for i in range(4)] + [(b"o", 1)]),  # prefix + a tie at 1
          ("grow3", 0, [(b"p%d" % i, 50 - i) for i in range(8)] + [(b"h", 3)])]  # rebuilt, one entry searched
    d2 = [("tie", 0, [(b"n3", 21), (b"n2", 20), (b"t", 15)]),          # the prefix, then duplicates
          ("dup", 0, [(b"q", 31), (b"x", 30)]),
          ("ins", 0, [(b"w", 33), (b"v7", 7), (b"v6", 6)]),
          ("many", 0, [(b"m%d" % i, 70 - i) for i in range(9)])]
    want = O.Repo(O.TLOG)
    got = RepoTLOG(engine)
    for logs in (state, d1, d2):
        b = _log_batch(logs)
        want.converge(b)
        got.converge_deltas(b)
        assert_state_equal(O.TLOG, want.state(), got.state())
    assert got.get("cut", 100)[-1] == (b"v6", 6) and got.size("grow") == 13
    assert engine.skipped() == 0


def test_malformed_after_newer_entries_is_skipped(engine):
    """an ordering error after a few valid newer-than-the-log entries (or in
    the value order of equal timestamps) still skips the whole key"""
    from jylis_amd.repo import RepoTLOG
    got = RepoTLOG(engine)
    got.converge_deltas(_log_batch([("k", 0, [(b"s", 1)])]))
    got.converge_deltas(_log_batch([("k", 0, [(b"x", 30), (b"y", 20), (b"z", 25)]),
                                    ("k2", 0, [(b"x", 30), (b"y", 20), (b"z", 20), (b"a", 20)])]))
    assert engine.skipped() == 2
    assert got.get("k") == [(b"s", 1)] and got.get("k2") == []


def test_clr_at_max_timestamp_and_trim_past_end(oracle_mod, engine):
    """CLR with newest ts 2^64-1 sets cutoff ts+1 = 0 (U64 wrap): no effect;
    TRIM n > size raises nothing (repo_tlog.pony:103-111; parity unpinned)"""
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    w = O.Repo(O.TLOG, 1)
    w.tlog_ins("k", b"top", (1 << 64) - 1)
    w.tlog_ins("k", b"x", 10)
    w.tlog_clr("k")
    w.tlog_trim("k", 50)
    w.tlog_ins("j", b"y", 3)
    w.tlog_trim("j", 1)
    got = RepoTLOG(engine)
    want = O.Repo(O.TLOG)
    for b in (w.flush().table(), w.state()):
        want.converge(b)
        got.converge_deltas(b)
    assert_state_equal(O.TLOG, want.state(), got.state())
    assert got.size("k") == 2


def test_repeated_keys_in_one_batch(oracle_mod, engine):
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    logs = [("k", 0, _canon([(b"a", 1)])), ("k", 2, _canon([(b"b", 3)])), ("j", 0, []), ("k", 0, _canon([(b"c", 2)]))]
    want = O.Repo(O.TLOG)
    got = RepoTLOG(engine)
    b = _log_batch(logs)
    want.converge(b)
    got.converge_deltas(b)
    assert_state_equal(O.TLOG, want.state(), got.state())


def test_malformed_segment_is_skipped(engine):
    """an unsorted delta log is not a TLog: the key is left untouched and the
    entry counted as skipped (the reference swallows converge errors)"""
    from jylis_amd.repo import RepoTLOG
    got = RepoTLOG(engine)
    got.converge_deltas(_log_batch([("k", 0, [(b"a", 1), (b"b", 5)]), ("ok", 0, [(b"z", 1)])]))
    assert engine.skipped() == 1
    assert got.get("k") == [] and got.get("ok") == [(b"z", 1)]


def test_large_synthetic(oracle_mod, engine):
    """config-4 shaped stream at 20k keys (geometric lengths, dups, ties, cutoffs)"""
    from jylis_amd import synth as S
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    st, dl = S.tlog_tables(20000, seed=S.BASE_SEED + 4, rounds=2)
    want = O.Repo(O.TLOG)
    got = RepoTLOG(engine)
    for b in [st] + dl:
        want.converge(b)
        got.converge_deltas(b)
    assert_state_equal(O.TLOG, want.state(), got.state())


def test_many_rounds_pool_reuse(oracle_mod):
    """ten config-4 rounds on a small pool: appends, rebuilds (ties, older
    entries, full segments), cutoff drops and several pool compactions, with
    the state compared after every round"""
    from jylis_amd import synth as S
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    eng = Engine(device=0, entry_capacity=1024)
    try:
        st, dl = S.tlog_tables(3000, seed=S.BASE_SEED + 40, rounds=10, mean_state=3, mean_delta=3)
        want = O.Repo(O.TLOG)
        got = RepoTLOG(eng)
        for b in [st] + dl:
            want.converge(b)
            got.converge_deltas(b)
            assert_state_equal(O.TLOG, want.state(), got.state())
        # a full-state delta (everything duplicates) leaves the state as is
        full = want.state()
        want.converge(full)
        got.converge_deltas(full)
        assert_state_equal(O.TLOG, want.state(), got.state())
    finally:
        eng.close()


def test_spilled_merges_in_flight(oracle_mod):
    """merges enqueued back to back, nothing read between them, on a pool too
    small for their rebuilt logs: the device-side check leaves those keys
    alone and spills their deltas, later merges run before the host sees it,
    and the re-merge after a compaction (at the next call that finds the
    merge done, or at the read) still gives the exact join"""
    from jylis_amd import synth as S
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    eng = Engine(device=0, entry_capacity=1024)
    try:
        st, dl = S.tlog_tables(4000, seed=S.BASE_SEED + 41, rounds=6, mean_state=4, mean_delta=3)
        want = O.Repo(O.TLOG)
        got = RepoTLOG(eng)
        for b in [st] + dl:
            want.converge(b)
            got.converge_deltas(b)
        assert_state_equal(O.TLOG, want.state(), got.state())
        stats = eng.tlog_stats()
        assert stats["spills"] >= 1 and stats["compactions"] >= 1, stats
        assert stats["merges"] >= len(dl) + 1
    finally:
        eng.close()


@pytest.mark.parametrize("seed", [11, 12])
def test_inserts_near_the_oldest_end(oracle_mod, engine, seed):
    """Round 6's in-place inserts that move the SHORTER side of a log: long
    logs receive, merge after merge, entries older than almost all of their
    entries (just above the oldest: the prefix moves down into the front
    room), entries near the newest (the suffix moves up), duplicates, ties,
    fresh appends, and cutoff raises that free front room -- until the room
    runs out and logs are rebuilt (update-history capacities) -- against the
    oracle after every merge."""
    from jylis_amd.repo import RepoTLOG
    O = oracle_mod
    rng = np.random.default_rng(seed)
    want = O.Repo(O.TLOG)
    got = RepoTLOG(engine)
    nkeys = 48
    logs = {f"k{i}": sorted({int(t) for t in rng.integers(1000, 100000, 40 + 7 * i)}) for i in range(nkeys)}
    state = [(k, 0, _canon([(b"s%d" % t, t) for t in ts])) for k, ts in logs.items()]
    b = _log_batch(state)
    want.converge(b)
    got.converge_deltas(b)
    cut = {k: 0 for k in logs}
    for merge in range(12):
        delta = []
        for k, ts in logs.items():
            live = [t for t in ts if t >= cut[k]]
            ents = []
            if live:
                lo = live[min(len(live) - 1, int(rng.integers(0, 3)))]  # just above the oldest live entry
                ents.append((b"old%d" % merge, lo + 1 if lo + 1 not in ts else lo))  # an insert near the start (or a tie)
                ents.append((b"s%d" % live[0], live[0]))  # a duplicate of the oldest
                hi = live[-1]
                ents.append((b"near-new%d" % merge, hi - 1))  # an insert near the newest end
            for a in range(int(rng.integers(0, 4))):  # appends
                ents.append((b"new%d.%d" % (merge, a), 200000 + 100 * merge + a))
            c = 0
            if live and rng.random() < 0.25:  # a cutoff raise into the log (frees front room)
                c = live[min(len(live) - 1, int(rng.integers(1, 6)))]
                cut[k] = max(cut[k], c)
            delta.append((k, c, _canon(ents)))
            ts.extend(t for _, t in ents)
            ts.sort()
        b = _log_batch(delta)
        want.converge(b)
        got.converge_deltas(b)
        assert_state_equal(O.TLOG, want.state(), got.state())
