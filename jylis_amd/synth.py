"""Seeded synthetic delta streams, numpy and torch.

Everything derives from splitmix64 over a cell index, so the host (numpy) and
device (torch) generators produce identical bits: small cases are checked
against the oracle on the host, full-size bench inputs are generated in HBM.

Base seed 0x4A594C4953 ("JYLIS"); config c uses base + c.
"""
import numpy as np

BASE_SEED = 0x4A594C4953
GOLDEN = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB
MASK64 = (1 << 64) - 1


def splitmix64_np(x):
    z = (np.asarray(x, dtype=np.uint64) + np.uint64(GOLDEN))
    z = (z ^ (z >> np.uint64(30))) * np.uint64(M1)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(M2)
    return z ^ (z >> np.uint64(31))


def _s64(v):
    """u64 constant -> the int64 with the same bits"""
    v &= MASK64
    return v - (1 << 64) if v >= (1 << 63) else v


def _srl(t, n):
    """logical shift right of an int64 tensor (bits as u64)"""
    import torch
    return (t >> n) & torch.tensor((1 << (64 - n)) - 1, dtype=torch.int64, device=t.device)


def splitmix64_torch(x):
    """x: int64 tensor holding u64 bits; wrapping int64 arithmetic == u64 arithmetic"""
    z = x + _s64(GOLDEN)
    z = (z ^ _srl(z, 30)) * _s64(M1)
    z = (z ^ _srl(z, 27)) * _s64(M2)
    return z ^ _srl(z, 31)


def replica_ids(n, seed=BASE_SEED):
    return splitmix64_np(np.arange(n, dtype=np.uint64) + np.uint64(seed))


def counter_keys(n, prefix=b"p", width=8, start=0):
    """fixed-width decimal keys b'p00000000'.. as (bytes, offs), vectorised"""
    idx = np.arange(start, start + n, dtype=np.uint64)
    digits = np.empty((n, width), np.uint8)
    v = idx.copy()
    for j in range(width - 1, -1, -1):
        digits[:, j] = (v % np.uint64(10)).astype(np.uint8) + ord("0")
        v //= np.uint64(10)
    pre = np.frombuffer(prefix, np.uint8)
    rows = np.concatenate([np.broadcast_to(pre, (n, len(pre))), digits], axis=1)
    L = rows.shape[1]
    return np.ascontiguousarray(rows).reshape(-1), np.arange(n + 1, dtype=np.uint64) * np.uint64(L)


# ---- counters (configs 1 and 2) --------------------------------------------

def counter_state_np(K, R, nsigns, seed, wrap_frac=True, cells=None):
    """initial state [nsigns][R][K] u64: uniform [0, 2^40); 10% near 2^64 (wrap).
    `cells` (flat indices sign*R*K + col*K + slot) evaluates only those cells."""
    if cells is None:
        cell = np.arange(nsigns * R * K, dtype=np.uint64).reshape(nsigns, R, K)
    else:
        cell = np.asarray(cells, np.uint64)
    h = splitmix64_np(cell * np.uint64(GOLDEN) + np.uint64(seed))
    s = h >> np.uint64(24)
    if wrap_frac:
        near = (splitmix64_np(h) % np.uint64(10)) == 0
        s = np.where(near, np.uint64(MASK64) - (h >> np.uint64(44)), s)
    return s


def counter_delta_np(prev, rnd, seed, cells=None):
    """next peer batch from `prev`: 75% prev + U[1,1000], 25% stale prev - U[0,1000]"""
    if cells is None:
        cell = np.arange(prev.size, dtype=np.uint64).reshape(prev.shape)
    else:
        cell = np.asarray(cells, np.uint64)
    h = splitmix64_np(cell * np.uint64(GOLDEN) + np.uint64(seed) + np.uint64((rnd + 1) * M2 & MASK64))
    inc = (h % np.uint64(1000)) + np.uint64(1)
    dec = (h >> np.uint64(16)) % np.uint64(1001)
    stale = ((h >> np.uint64(32)) & np.uint64(3)) == 0
    return np.where(stale, prev - dec, prev + inc)


def counter_state_torch(K, R, nsigns, seed, device, wrap_frac=True, out=None):
    import torch
    n = nsigns * R * K
    cell = torch.arange(n, dtype=torch.int64, device=device)
    h = splitmix64_torch(cell * _s64(GOLDEN) + _s64(seed))
    s = _srl(h, 24)
    if wrap_frac:
        hh = splitmix64_torch(h)
        # (u64 hh) % 10 == 0 via unsigned remainder on the two 32-bit halves
        near = _umod(hh, 10) == 0
        s = torch.where(near, -1 - _srl(h, 44), s)
    s = s.view(nsigns, R, K)
    if out is not None:
        out.copy_(s)
        return out
    return s


def _umod(t, m):
    """u64 remainder of int64 bits by a small m"""
    import torch
    hi = _srl(t, 32)
    lo = t & 0xFFFFFFFF
    return ((hi % m) * ((1 << 32) % m) + lo % m) % m


def counter_delta_torch(prev, rnd, seed, out=None):
    import torch
    cell = torch.arange(prev.numel(), dtype=torch.int64, device=prev.device).view(prev.shape)
    h = splitmix64_torch(cell * _s64(GOLDEN) + _s64(seed) + _s64((rnd + 1) * M2))
    inc = _umod(h, 1000) + 1
    dec = _umod(_srl(h, 16), 1001)
    stale = (_srl(h, 32) & 3) == 0
    r = torch.where(stale, prev - dec, prev + inc)
    if out is not None:
        out.copy_(r)
        return out
    return r


def counter_rows_torch(out, seed, rnd=None, prev=None, wrap_frac=True, col_offset=0, col_total=None):
    """Fill out[nsigns][R][K] (int64 bits of u64) row by row, bounding temporaries:
    rnd None -> initial state; else the round-`rnd` delta from `prev`.
    Rows are columns col_offset .. col_offset + R - 1 of a [nsigns][col_total][K]
    stream (default: the whole stream), so any slice of it can be generated alone."""
    import torch
    nsigns, R, K = out.shape
    RT = R if col_total is None else col_total
    ar = torch.arange(K, dtype=torch.int64, device=out.device)
    for s in range(nsigns):
        for c in range(R):
            cell = ar + (s * RT + col_offset + c) * K
            if rnd is None:
                h = splitmix64_torch(cell * _s64(GOLDEN) + _s64(seed))
                v = _srl(h, 24)
                if wrap_frac:
                    near = _umod(splitmix64_torch(h), 10) == 0
                    v = torch.where(near, -1 - _srl(h, 44), v)
            else:
                h = splitmix64_torch(cell * _s64(GOLDEN) + _s64(seed) + _s64((rnd + 1) * M2))
                inc = _umod(h, 1000) + 1
                dec = _umod(_srl(h, 16), 1001)
                stale = (_srl(h, 32) & 3) == 0
                p = prev[s, c]
                v = torch.where(stale, p - dec, p + inc)
            out[s, c].copy_(v)
    return out


def _excl_cumsum(x):
    out = np.zeros(len(x) + 1, np.uint64)
    out[1:] = np.cumsum(x, dtype=np.uint64)
    return out


def gather_bytes(vb, vo, idx):
    """bytes of entries idx of (vb, vo) -> (bytes, offs)"""
    idx = np.asarray(idx, np.int64)
    lens = (vo[idx + 1] - vo[idx]).astype(np.int64)
    offs = _excl_cumsum(lens)
    total = int(offs[-1])
    if total == 0:
        return np.zeros(0, np.uint8), offs
    pos = np.repeat(vo[idx].astype(np.int64) - offs[:-1].astype(np.int64), lens) + np.arange(total)
    return vb[pos], offs


def random_values(rng, n, lo=1, hi=16):
    lens = rng.integers(lo, hi + 1, n)
    offs = _excl_cumsum(lens)
    return rng.integers(0, 256, int(offs[-1]), dtype=np.uint8), offs


def _concat_values(parts):
    """[(bytes, offs)] -> (bytes, offs)"""
    vbs = [p[0] for p in parts]
    lens = np.concatenate([np.diff(p[1].astype(np.int64)) for p in parts])
    return (np.concatenate(vbs) if vbs else np.zeros(0, np.uint8)), _excl_cumsum(lens)


def tlog_tables(K, seed, rounds=1, mean_state=8, cap=64, mean_delta=2, key_prefix=b"l"):
    """Config-4 stream: K logs with state lengths ~ Geom(mean 8,
    cap 64), then `rounds` delta batches with lengths ~ Geom(mean 2): newer
    entries, ~10% duplicates of a state entry, ~5% same-timestamp different-value
    ties, 5% of keys raising the cutoff to a state entry's timestamp.  Every
    segment is canonical (strictly descending).  Returns (state, [deltas])."""
    rng = np.random.default_rng(seed)
    kb, ko = counter_keys(K, prefix=key_prefix)
    Ls = np.minimum(rng.geometric(1.0 / mean_state, K), cap).astype(np.int64)
    soff = _excl_cumsum(Ls)
    N = int(soff[-1])
    seg = np.repeat(np.arange(K), Ls)
    newest = rng.integers(1 << 20, 1 << 40, K).astype(np.uint64)
    gaps = rng.integers(1, 1000, N).astype(np.uint64)
    cg = np.cumsum(gaps, dtype=np.uint64)
    first = soff[:-1].astype(np.int64)
    w = cg - gaps - (cg[first] - gaps[first])[seg]
    sts = newest[seg] - w
    svb, svo = random_values(rng, N)
    state = {"key_bytes": kb, "key_offs": ko, "cutoff": np.zeros(K, np.uint64), "ent_offs": soff, "ts": sts,
             "val_bytes": svb, "val_offs": svo}
    deltas = []
    top = newest.copy()
    for _ in range(rounds):
        Ld = np.minimum(rng.geometric(1.0 / mean_delta, K), cap).astype(np.int64)
        step = rng.integers(1, 100, K).astype(np.uint64)
        # new entries, newest first
        nkey = np.repeat(np.arange(K), Ld)
        rank = np.arange(int(Ld.sum())) - np.repeat(_excl_cumsum(Ld)[:-1].astype(np.int64), Ld)
        nts = top[nkey] + (Ld[nkey] - rank).astype(np.uint64) * step[nkey]
        nval = random_values(rng, len(nkey))
        # a duplicate of one state entry (20% of keys) and a timestamp tie with
        # another (10% of keys with >= 2 entries), appended oldest-last
        i1 = (rng.random(K) * Ls).astype(np.int64)
        i2 = (i1 + 1 + (rng.random(K) * np.maximum(Ls - 1, 1)).astype(np.int64)) % Ls
        has_dup = rng.random(K) < 0.2
        has_tie = (rng.random(K) < 0.1) & (Ls >= 2)
        dkeys = np.nonzero(has_dup)[0]
        tkeys = np.nonzero(has_tie)[0]
        didx = soff[dkeys].astype(np.int64) + i1[dkeys]
        tidx = soff[tkeys].astype(np.int64) + i2[tkeys]
        dval = gather_bytes(svb, svo, didx)
        tval = random_values(rng, len(tkeys))
        keys = np.concatenate([nkey, dkeys, tkeys])
        ts = np.concatenate([nts, sts[didx], sts[tidx]])
        # order inside a segment: new entries first (they are newer), then the
        # older pair by descending timestamp
        grp = np.concatenate([np.zeros(len(nkey)), np.ones(len(dkeys) + len(tkeys))])
        r2 = np.concatenate([rank, np.zeros(len(dkeys) + len(tkeys), np.int64)])
        order = np.lexsort((r2, -ts.astype(np.float64) * grp, grp, keys))
        vb, vo = _concat_values([nval, dval, tval])
        ent_vb, ent_vo = gather_bytes(vb, vo, order)
        offs = _excl_cumsum(np.bincount(keys, minlength=K))
        cut = np.zeros(K, np.uint64)
        ck = np.nonzero(rng.random(K) < 0.05)[0]
        cut[ck] = sts[soff[ck].astype(np.int64) + (rng.random(len(ck)) * Ls[ck]).astype(np.int64)]
        deltas.append({"key_bytes": kb, "key_offs": ko, "cutoff": cut, "ent_offs": offs, "ts": ts[order],
                       "val_bytes": ent_vb, "val_offs": ent_vo})
        top = top + (Ld + 1).astype(np.uint64) * step + np.uint64(1)
    return state, deltas


def treg_tables(K, seed, rounds=1, window=1 << 9, key_prefix=b"g"):
    """Config-3-shaped TREG stream for the full-size pin: K
    registers, then `rounds` delta batches holding one (ts, value) for every
    key in key order.  Round j's timestamps are j * window / 2 + [0, window),
    so about half the keys take each batch and ~K / window keys tie on the
    timestamp; values are 0-16 bytes, 30 % sharing one of 16 8-byte prefixes
    (ties then need the bytes past the prefix).  Returns (state, [deltas])."""
    rng = np.random.default_rng(seed)
    kb, ko = counter_keys(K, prefix=key_prefix)
    prefixes = rng.integers(0, 256, (16, 8), dtype=np.uint8)

    def values():
        vb, vo = random_values(rng, K, 0, 16)
        lens = np.diff(vo.astype(np.int64))
        share = (rng.random(K) < 0.3) & (lens >= 9)
        pick = rng.integers(0, 16, K)
        starts = vo[:-1].astype(np.int64)
        for j in range(8):
            vb[starts[share] + j] = prefixes[pick[share], j]
        return vb, vo

    out = []
    for j in range(rounds + 1):
        vb, vo = values()
        ts = (rng.integers(0, window, K) + j * (window // 2)).astype(np.uint64)
        out.append({"key_bytes": kb, "key_offs": ko, "ts": ts, "val_bytes": vb, "val_offs": vo})
    return out[0], out[1:]


def ujson_tables(D, seed, rounds=1, R=16, leaves=8, zipf=1.1, ops_per_round=None, key_prefix=b"u", id_seed=None):
    """Config-5 stream: D docs with ~`leaves` elements over R
    replicas, then `rounds` delta batches whose ops (70% INS, 20% RM, 10% CLR)
    hit docs with Zipf(zipf) popularity; ops on one doc fold into one delta.
    Tables use replica ids (oracle layout; `id_seed` picks the id set, so
    shards can share one cluster of replicas).  Returns (state, [deltas])."""
    rng = np.random.default_rng(seed)
    ids = replica_ids(R, seed if id_seed is None else id_seed)
    kb, ko = counter_keys(D, prefix=key_prefix)
    # ---- state, vectorised: vv, elements under seen dots, gapped cloud dots
    vv = rng.integers(0, 24, (D, R)).astype(np.int64)
    ne = np.minimum(rng.poisson(leaves, D), 40)
    ed = np.repeat(np.arange(D), ne)
    ec = rng.integers(0, R, len(ed))
    top = vv[ed, ec]
    keep = top > 0
    ed, ec, top = ed[keep], ec[keep], top[keep]
    eq = 1 + (rng.random(len(ed)) * top).astype(np.int64)
    nk = rng.integers(1, 4, D) * (rng.random(D) < 0.25)
    cd = np.repeat(np.arange(D), nk)
    cc = rng.integers(0, R, len(cd))
    cq = vv[cd, cc] + 2 + rng.integers(0, 5, len(cd))
    _, first = np.unique((cd * R + cc) * 64 + cq, return_index=True)
    cd, cc, cq = cd[first], cc[first], cq[first]
    ce = rng.random(len(cd)) < 0.5
    ed, ec, eq = (np.concatenate([x, y[ce]]) for x, y in ((ed, cd), (ec, cc), (eq, cq)))
    _, first = np.unique((ed * R + ec) * 64 + eq, return_index=True)
    ed, ec, eq = ed[first], ec[first], eq[first]
    ee = rng.integers(1, 64, len(ed))
    e_off = _excl_cumsum(np.bincount(ed, minlength=D)).astype(np.int64)
    c_off = _excl_cumsum(np.bincount(cd, minlength=D)).astype(np.int64)
    vd, vc = np.nonzero(vv)
    state = {"key_bytes": kb, "key_offs": ko,
             "el_offs": e_off.astype(np.uint64), "dot_ids": ids[ec], "dot_seqs": eq.astype(np.uint64),
             "elems": ee.astype(np.uint64),
             "vv_offs": _excl_cumsum(np.bincount(vd, minlength=D)), "vv_ids": ids[vc],
             "vv_seqs": vv[vd, vc].astype(np.uint64),
             "cloud_offs": c_off.astype(np.uint64), "cloud_ids": ids[cc], "cloud_seqs": cq.astype(np.uint64)}
    # highest seq any context of a doc has seen per column (fresh dots go above)
    seen = vv.copy()
    np.maximum.at(seen, (cd, cc), cq)

    perm = rng.permutation(D)
    deltas = []
    nops = ops_per_round or max(1, D // 2)
    for _ in range(rounds):
        deltas.append(_ujson_round(D, R, ids, kb, ko, e_off, ec, eq, ee, vv, seen, perm, rng, nops, zipf))
    return state, deltas


def _ujson_round(D, R, ids, kb, ko, e_off, ec, eq, ee, vv, seen, perm, rng, nops, zipf):
    """one round of ops (70% INS, 20% RM, 10% CLR on Zipf-hit docs) folded
    into one delta per doc, vectorised.  Draws the same random numbers in the
    same order as the per-op form (_ujson_round_ref) and returns the same
    table bit for bit (tests/test_synth.py); `seen` advances in place."""
    hit = perm[(rng.zipf(zipf, nops) - 1) % D].astype(np.int64)
    kinds = rng.random(nops)
    reps = rng.integers(0, R, nops).astype(np.int64)
    u = rng.random((nops, 4))
    u0, u1, u2, u3 = u[:, 0], u[:, 1], u[:, 2], u[:, 3]
    n_el = (e_off[1:] - e_off[:-1]).astype(np.int64)
    nd = n_el[hit]
    seen_f = seen.reshape(-1)  # [D * R] view
    # INS: a fresh dot of replica r (sometimes past a gap); per (doc, replica)
    # the seqs continue from `seen` in op order
    ins = np.nonzero(kinds < 0.7)[0]
    key = hit[ins] * R + reps[ins]
    inc = 1 + np.where(u0[ins] < 0.2, 1 + (u1[ins] * 2).astype(np.int64), 0)
    order = np.argsort(key, kind="stable")
    ks, io = key[order], inc[order]
    cs = np.cumsum(io)
    start = np.r_[True, ks[1:] != ks[:-1]] if len(ks) else np.zeros(0, bool)
    base = (cs - io)[np.maximum.accumulate(np.where(start, np.arange(len(ks)), 0))] if len(ks) else cs
    run = cs - base  # inclusive cumsum within each (doc, replica) run
    q = np.empty(len(ins), np.int64)
    q[order] = seen_f[ks] + run
    if len(ks):
        last = np.r_[ks[1:] != ks[:-1], True]
        seen_f[ks[last]] = seen_f[ks[last]] + run[last]
    d_parts, c_parts, q_parts, e_parts = [hit[ins]], [reps[ins]], [q], [1 + (u2[ins] * 63).astype(np.int64)]
    cl_d, cl_c, cl_q = [hit[ins]], [reps[ins]], [q]

    def expand(sel):
        """every element of the docs of ops `sel`: (op index, element index)"""
        cnt = nd[sel]
        rep = np.repeat(np.arange(len(sel)), cnt)
        j = np.repeat(e_off[hit[sel]], cnt) + (np.arange(len(rep)) - np.repeat(np.cumsum(cnt) - cnt, cnt))
        return rep, j.astype(np.int64)
    # RM one element value of the doc: every dot holding it
    rm = np.nonzero((kinds >= 0.7) & (kinds < 0.9) & (nd > 0))[0]
    val = ee[e_off[hit[rm]] + (u1[rm] * nd[rm]).astype(np.int64)]
    rep, j = expand(rm)
    m = ee[j] == val[rep]
    cl_d.append(hit[rm][rep][m])
    cl_c.append(ec[j][m])
    cl_q.append(eq[j][m])
    # CLR: every dot of the doc
    clr = np.nonzero(kinds >= 0.9)[0]
    rep, j = expand(clr)
    cl_d.append(hit[clr][rep])
    cl_c.append(ec[j])
    cl_q.append(eq[j])
    # a version-vector entry carried along (any op kind)
    vo = np.nonzero(u3 < 0.1)[0]
    vc = (u2[vo] * R).astype(np.int64)
    vval = vv[hit[vo], vc]
    keep = vval > 0
    vd, vc, vval = hit[vo][keep], vc[keep], vval[keep]
    # an element the state holds, re-sent
    rs = np.nonzero((u3 > 0.95) & (nd > 0))[0]
    j = e_off[hit[rs]] + (u0[rs] * nd[rs]).astype(np.int64)
    d_parts.append(hit[rs])
    c_parts.append(ec[j])
    q_parts.append(eq[j])
    e_parts.append(ee[j])
    cl_d.append(hit[rs])
    cl_c.append(ec[j])
    cl_q.append(eq[j])
    return _ujson_fold(D, R, ids, kb, ko, np.unique(hit),
                       (np.concatenate(d_parts), np.concatenate(c_parts), np.concatenate(q_parts),
                        np.concatenate(e_parts)),
                       (vd, vc, vval),
                       (np.concatenate(cl_d), np.concatenate(cl_c), np.concatenate(cl_q)))


def _ujson_fold(D, R, ids, kb, ko, docs, els, vvs, cls):
    """one round's ops folded into one delta per doc: element dots (a set; a
    dot always carries one value), vv entries (the state's value), cloud dots
    (a set), each segment sorted by (column, seq); docs ascending"""
    def uniq(d, c, q):
        """first occurrence of every distinct (d, c, q), sorted by (d, c, q)"""
        o = np.lexsort((q, c, d))
        if len(o) == 0:
            return o
        ds, cs, qs = d[o], c[o], q[o]
        new = np.r_[True, (ds[1:] != ds[:-1]) | (cs[1:] != cs[:-1]) | (qs[1:] != qs[:-1])]
        return o[new]
    ed, ec, eq, ee = els
    f = uniq(ed, ec, eq)
    ed, ec, eq, ee = ed[f], ec[f], eq[f], ee[f]
    vd, vc, vq = vvs
    f = uniq(vd, vc, np.zeros_like(vd))
    vd, vc, vq = vd[f], vc[f], vq[f]
    cd, cc, cq = cls
    f = uniq(cd, cc, cq)
    cd, cc, cq = cd[f], cc[f], cq[f]
    pos = np.full(D, -1, np.int64)
    pos[docs] = np.arange(len(docs))

    def offs(d):
        return _excl_cumsum(np.bincount(pos[d], minlength=len(docs)))
    t = {}
    t["key_bytes"], t["key_offs"] = gather_bytes(kb, ko, docs) if len(docs) else (np.zeros(0, np.uint8),
                                                                                  np.zeros(1, np.uint64))
    t["dot_ids"], t["dot_seqs"], t["elems"] = ids[ec], eq.astype(np.uint64), ee.astype(np.uint64)
    t["vv_ids"], t["vv_seqs"] = ids[vc], vq.astype(np.uint64)
    t["cloud_ids"], t["cloud_seqs"] = ids[cc], cq.astype(np.uint64)
    t["el_offs"], t["vv_offs"], t["cloud_offs"] = offs(ed), offs(vd), offs(cd)
    return t


def _ujson_round_ref(D, R, ids, kb, ko, e_off, ec, eq, ee, vv, seen, perm, rng, nops, zipf):
    """the per-op form of one ujson_tables round (rounds 1-3 generated with
    it): the reference _ujson_round is checked against"""
    def doc_elems(d):
        lo, hi = e_off[d], e_off[d + 1]
        return list(zip(ec[lo:hi].tolist(), eq[lo:hi].tolist(), ee[lo:hi].tolist()))

    def table(folded):
        docs = sorted(folded)
        cols = {k: [] for k in ("dot_ids", "dot_seqs", "elems", "vv_ids", "vv_seqs", "cloud_ids", "cloud_seqs")}
        eo, vo, co = [0], [0], [0]
        for d in docs:
            dvv, dels, dcl = folded[d]
            for (c, q), e in sorted(dels.items()):
                cols["dot_ids"].append(ids[c])
                cols["dot_seqs"].append(q)
                cols["elems"].append(e)
            eo.append(eo[-1] + len(dels))
            for c, q in sorted(dvv.items()):
                cols["vv_ids"].append(ids[c])
                cols["vv_seqs"].append(q)
            vo.append(vo[-1] + len(dvv))
            for c, q in sorted(dcl):
                cols["cloud_ids"].append(ids[c])
                cols["cloud_seqs"].append(q)
            co.append(co[-1] + len(dcl))
        sel = np.array(docs, np.int64)
        t = {}
        t["key_bytes"], t["key_offs"] = gather_bytes(kb, ko, sel) if len(sel) else (np.zeros(0, np.uint8),
                                                                                   np.zeros(1, np.uint64))
        for k, v in cols.items():
            t[k] = np.array(v, np.uint64)
        t["el_offs"], t["vv_offs"], t["cloud_offs"] = (np.array(x, np.uint64) for x in (eo, vo, co))
        return t

    hit = perm[(rng.zipf(zipf, nops) - 1) % D].tolist()
    kinds = rng.random(nops).tolist()
    reps = rng.integers(0, R, nops).tolist()
    u = rng.random((nops, 4)).tolist()
    folded = {}
    for d, x, r, (u0, u1, u2, u3) in zip(hit, kinds, reps, u):
        dvv, dels, dcl = folded.setdefault(d, ({}, {}, set()))
        els = doc_elems(d)
        if x < 0.7:  # INS: a fresh dot of replica r (sometimes past a gap)
            q = int(seen[d, r]) + 1 + (1 + int(u1 * 2) if u0 < 0.2 else 0)
            seen[d, r] = q
            dels[(r, q)] = 1 + int(u2 * 63)
            dcl.add((r, q))
        elif x < 0.9:  # RM one element value: every dot holding it
            if els:
                e = els[int(u1 * len(els))][2]
                dcl.update((c, q) for c, q, v in els if v == e)
        else:  # CLR
            dcl.update((c, q) for c, q, _ in els)
        if u3 < 0.1:  # carry a version-vector entry too
            c = int(u2 * R)
            if vv[d, c]:
                dvv[c] = max(dvv.get(c, 0), int(vv[d, c]))
        if u3 > 0.95 and els:  # re-send an element the state holds
            c, q, v = els[int(u0 * len(els))]
            dels[(c, q)] = v
            dcl.add((c, q))
    return table(folded)


def counter_batch_tables(state_or_delta, replica_id_list, key_tab, prefix=""):
    """[R][K] (GCOUNT) or [2][R][K] (PNCOUNT) array -> per-replica oracle batch tables
    (one flushed peer batch per replica column, every key carrying that column)"""
    kb, ko = key_tab
    arr = np.asarray(state_or_delta)
    if arr.ndim == 2:
        arr = arr[None]
    nsigns, R, K = arr.shape
    out = []
    for c in range(R):
        t = {"key_bytes": kb, "key_offs": ko}
        for s, pre in zip(range(nsigns), ("p_", "n_") if nsigns == 2 else ("",)):
            t[pre + "offs"] = np.arange(K + 1, dtype=np.uint64)
            t[pre + "ids"] = np.full(K, replica_id_list[c], np.uint64)
            t[pre + "vals"] = arr[s, c].astype(np.uint64)
        out.append(t)
    return out
