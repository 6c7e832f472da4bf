"""Shared test helpers: oracle-driven delta streams and state comparison."""
import numpy as np


def strip_zero_counters(t, prefixes):
    """GCounter entries holding 0 are unobservable (value() and max-merge treat
    absent == 0); the engine stores replica columns densely, so compare with
    zero entries removed."""
    t = dict(t)
    n = len(t["key_offs"]) - 1
    for p in prefixes:
        offs, ids, vals = t[p + "offs"], t[p + "ids"], t[p + "vals"]
        keep = vals != 0
        new_offs = np.zeros(n + 1, np.uint64)
        if len(offs) > 1:
            # kept entries per segment from a running count (empty segments,
            # trailing ones included, count 0)
            run = np.concatenate([[0], np.cumsum(keep.astype(np.int64))])
            o = np.asarray(offs, np.int64)
            new_offs[1:] = np.cumsum(run[o[1:]] - run[o[:-1]]).astype(np.uint64)
        t[p + "offs"], t[p + "ids"], t[p + "vals"] = new_offs, ids[keep], vals[keep]
    return t


COUNTER_PREFIXES = {0: ("",), 1: ("p_", "n_")}


def assert_state_equal(ctype, want, got):
    if ctype in COUNTER_PREFIXES:
        want = strip_zero_counters(want, COUNTER_PREFIXES[ctype])
        got = strip_zero_counters(got, COUNTER_PREFIXES[ctype])
    assert set(want) == set(got), (sorted(want), sorted(got))
    for k in want:
        np.testing.assert_array_equal(np.asarray(want[k]), np.asarray(got[k]), err_msg=f"field {k}")


def random_history(O, ctype, seed, nrep=4, nops=300, nkeys=12, val_len=14, gossip=0.25):
    """Run random writes on `nrep` oracle replicas with partial gossip and
    return every flushed batch (tables), in emission order."""
    rng = np.random.default_rng(seed)
    reps = [O.Repo(ctype, int(rng.integers(1, 2**63)) * 2 + 1) for _ in range(nrep)]
    keys = [f"k{i}" for i in range(nkeys)]
    batches = []

    for _ in range(nops):
        r = reps[rng.integers(nrep)]
        k = keys[rng.integers(nkeys)]
        random_write(O, ctype, r, k, rng, val_len)
        if rng.random() < gossip:
            b = r.flush().table()
            batches.append(b)
            for o in reps:
                if o is not r and rng.random() < 0.5:
                    o.converge(b)
    for r in reps:
        batches.append(r.flush().table())
        batches.append(r.state())  # full-state deltas too
    return batches


def random_write(O, ctype, r, k, rng, val_len=14):
    """one random local write command of `ctype` on oracle replica r"""
    def rstr():
        n = int(rng.integers(0, val_len))
        # small alphabet -> many shared prefixes / ties
        return bytes(rng.choice(np.frombuffer(b"aab\x00\xff", np.uint8), size=n))

    if ctype == O.GCOUNT:
        r.gcount_inc(k, int(rng.integers(0, 1 << 62)))
    elif ctype == O.PNCOUNT:
        v = int(rng.integers(-(1 << 62), 1 << 62))
        (r.pncount_inc if rng.random() < 0.5 else r.pncount_dec)(k, v)
    elif ctype == O.TREG:
        r.treg_set(k, rstr(), int(rng.integers(0, 6)))
    elif ctype == O.TLOG:
        x = rng.random()
        if x < 0.8:
            r.tlog_ins(k, rstr(), int(rng.integers(0, 40)))
        elif x < 0.9:
            r.tlog_trimat(k, int(rng.integers(0, 30)))
        elif x < 0.97:
            r.tlog_trim(k, int(rng.integers(0, 8)))
        else:
            r.tlog_clr(k)
    elif ctype == O.UJSON:
        x = rng.random()
        if x < 0.65:
            r.ujson_ins(k, int(rng.integers(1, 8)))
        elif x < 0.9:
            r.ujson_rm(k, int(rng.integers(1, 8)))
        else:
            r.ujson_clr(k)


# per-type batch layout: per-key columns, and CSR groups (offsets column,
# data columns, optional nested CSR over the group's items)
ROW_SCHEMA = {
    0: ([], [("offs", ("ids", "vals"), None)]),
    1: ([], [("p_offs", ("p_ids", "p_vals"), None), ("n_offs", ("n_ids", "n_vals"), None)]),
    2: (["ts"], [("val_offs", ("val_bytes",), None)]),
    3: (["cutoff"], [("ent_offs", ("ts",), ("val_offs", ("val_bytes",)))]),
    4: ([], [("el_offs", ("dot_ids", "dot_seqs", "elems"), None), ("vv_offs", ("vv_ids", "vv_seqs"), None),
             ("cloud_offs", ("cloud_ids", "cloud_seqs"), None)]),
}


def split_rows(ctype, table):
    """a batch table -> [(key bytes, one-key delta table)]: the decoded
    Array[(String, Any box)] that RepoManagerCore.converge_deltas walks pair
    by pair (repo_manager.pony:92-93)"""
    per_key, groups = ROW_SCHEMA[ctype]
    kb, ko = np.asarray(table["key_bytes"], np.uint8), np.asarray(table["key_offs"], np.int64)
    rows = []
    for i in range(len(ko) - 1):
        row = {c: np.asarray(table[c])[i:i + 1] for c in per_key}
        for offs, cols, nested in groups:
            o = np.asarray(table[offs], np.int64)
            lo, hi = int(o[i]), int(o[i + 1])
            row[offs] = np.array([0, hi - lo], np.uint64)
            for c in cols:
                row[c] = np.asarray(table[c])[lo:hi]
            if nested:
                noffs, ncols = nested
                no = np.asarray(table[noffs], np.int64)
                row[noffs] = (no[lo:hi + 1] - no[lo]).astype(np.uint64)
                for c in ncols:
                    row[c] = np.asarray(table[c])[no[lo]:no[hi]]
        rows.append((bytes(kb[ko[i]:ko[i + 1]]), row))
    return rows


def collect(procs, q, n, deadline_s=150.0):
    """n messages from worker processes; fail fast on an ("error", rank,
    traceback) message or a dead worker, and kill the rest (a rank stuck in
    a collective its peer never joins would otherwise hang the test)"""
    import queue
    import time
    msgs = []
    t_end = time.time() + deadline_s
    try:
        while len(msgs) < n:
            try:
                m = q.get(timeout=2.0)
            except queue.Empty:
                dead = [p for p in procs if p.exitcode not in (None, 0)]
                if dead:
                    raise AssertionError(f"worker exited with {dead[0].exitcode} before sending its results")
                if time.time() > t_end:
                    raise AssertionError(f"timed out with {len(msgs)} of {n} messages")
                continue
            if m[0] == "error":
                raise AssertionError(f"rank {m[1]} failed:\n{m[2]}")
            msgs.append(m)
    finally:
        if len(msgs) < n:
            for p in procs:
                if p.is_alive():
                    p.kill()
        for p in procs:
            p.join(timeout=30)
    return msgs



def join_rows(ctype, rows):
    """{key: one-key row} (or split_rows' pairs) -> one table sorted by key
    (jylis_amd.repo.concat_rows); empty -> an empty table of the type"""
    from jylis_amd.repo import concat_rows
    rows = dict(rows)
    if rows:
        return concat_rows(sorted(rows.items()))
    per_key, groups = ROW_SCHEMA[ctype]
    t = {"key_bytes": np.zeros(0, np.uint8), "key_offs": np.zeros(1, np.uint64)}
    for c in per_key:
        t[c] = np.zeros(0, np.uint64)
    for offs, cols, nested in groups:
        t[offs] = np.zeros(1, np.uint64)
        for c in cols:
            t[c] = np.zeros(0, np.uint64)
        if nested:
            t[nested[0]] = np.zeros(1, np.uint64)
            for c in nested[1]:
                t[c] = np.zeros(0, np.uint8)
    if ctype == 2:
        t["val_bytes"] = np.zeros(0, np.uint8)
    return t
