"""Per-type bench modes behind `bench.py --type {gcount,treg,tlog,ujson}`.

The default bench line is PNCOUNT (BASELINE.json configs[1]); these modes
measure the other SURVEY.md 8d configs on the same engine and report their
own roofline (algorithmic bytes per converge / converge time, HIP events on
the engine stream).  Inputs are synthetic (jylis_amd/synth.py); the first
converge of every mode is checked against an independent recomputation.
"""
import os
import sys
import time

import numpy as np

HBM_PEAK_GBS = 8000.0
_HERE = os.path.dirname(os.path.abspath(__file__))


def pmc_traffic(name, workload=None):
    """HBM bytes per converge (or launch) from a committed PMC summary,
    profiles/r06_pmc_bench_<name>.json (scripts/gpu_r06_pmc.sh: separate
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this same bench line,
    scripts/pmc_converge.py: FETCH x2, WRITE as is).  The counters cannot be
    read live beside the timed region, so the line quotes the committed run
    of its own workload -> (bytes or None, source)"""
    path = os.path.join(_HERE, "profiles", f"r06_pmc_bench_{name}.json")
    try:
        import json
        with open(path) as f:
            d = json.load(f)
        if workload is not None and d.get("workload", workload) != workload:
            return None, None
        return float(d["moved_MB"]) * 1e6, os.path.relpath(path, _HERE)
    except Exception:
        return None, None


def with_traffic(roof, name, workload=None):
    t, src = pmc_traffic(name, workload)
    roof["traffic"] = t
    if t is not None:
        roof["traffic_source"] = src
        roof["traffic_note"] = "HBM bytes per converge from the committed PMC passes of this bench line (FETCH x2, WRITE)"
    return roof


def _timed(steps, warmup, step, dist, dev, eng=None, before_timed=None, drain=None):
    """warmup, then exactly `steps` steps bracketed by barrier + synchronize.
    Per-step device time: with `eng`, the engine's own HIP events around each
    merge call's device work (jy_timing_enable; host launch gaps excluded),
    summed per step; otherwise torch events on the current (engine) stream."""
    import torch
    for i in range(warmup):
        step(i)
    if drain is not None:
        drain()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # with `eng`, the engine's own timing events (no system-scope fence) are the
    # per-step device time; otherwise one pair of torch events brackets all the
    # steps (a torch event record writes back and invalidates the caches: one
    # pair per step put ~19 us of idle GPU into every short step)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if before_timed is not None:
        before_timed()
    if eng is not None:
        eng.timing(True)
    host = []
    t0 = time.perf_counter()
    if eng is None:
        ev0.record()
    for i in range(steps):
        h0 = time.perf_counter()
        step(warmup + i)
        host.append(time.perf_counter() - h0)
    if eng is None:
        ev1.record()
    if drain is not None:  # a node's calls only enqueue: its queued work is inside the timed region
        drain()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if os.environ.get("JY_TRACE"):
        print("host s per step:", " ".join(f"{h * 1e3:.3f}ms" for h in host), file=sys.stderr)
    if eng is not None:
        calls = eng.timing_read()
        eng.timing(False)
        per_step = float(np.sum(calls)) / 1e3 / steps
        return elapsed, [per_step] * steps
    return elapsed, [ev0.elapsed_time(ev1) / 1e3 / steps] * steps


def _max_over_ranks(x, dist, dev):
    import torch
    if not dist:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def _ask_owners(dist, cpu_group, rank, world, reqs, answer):
    """answers for sampled keys wherever they live: reqs = [(owner rank,
    owner-side slot)], answer(slots) -> one answer per slot, run by each owner
    on its own engine.  At N > 1 the requests and answers travel over the CPU
    (gloo) group, so every routed line verifies at any world size."""
    if world == 1 or dist is None:
        return list(answer(np.array([s for _, s in reqs], np.uint32))) if reqs else []
    every = [None] * world
    dist.all_gather_object(every, reqs, group=cpu_group)
    mine = [(src, i, s) for src, rq in enumerate(every) for i, (o, s) in enumerate(rq) if o == rank]
    ans = list(answer(np.array([s for _, _, s in mine], np.uint32))) if mine else []
    back = [None] * world
    dist.all_gather_object(back, [(src, i, a) for (src, i, _), a in zip(mine, ans)], group=cpu_group)
    res = [None] * len(reqs)
    for lst in back:
        for src, i, a in lst:
            if src == rank:
                res[i] = a
    return res


def _all_true(ok, dist, dev):
    """every rank verified (min over ranks)"""
    if not dist:
        return bool(ok)
    import torch
    t = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]) == 0.0


def cpu_baseline(mode, rounds=2):
    """The oracle (oracle/jy_oracle.cpp: the reference's Map[String, CRDT] +
    per-key converge loop, repo_manager.pony:92-93) timed single-threaded on a
    bounded sample of the same synthetic stream; only the converge of the
    delta batches is timed (decode excluded).  Units match the GPU mode."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle"))
    import oracle as O
    from jylis_amd import synth as S
    t_conv, units, sample = 0.0, 0, ""
    if mode == "read":
        return None  # no C-level GET loop in the oracle; a Python loop over it would time ctypes
    if mode in ("gcount", "e2e"):  # e2e: the oracle's converge probes its Map by key string, as e2e interns
        K, R = 262144, 16
        seed = S.BASE_SEED + 1
        kb, ko = S.counter_keys(K, prefix=b"g", width=7)
        rids = S.replica_ids(R, seed)
        st = S.counter_state_np(K, R, 1, seed, wrap_frac=False)[0]
        repo = O.Repo(O.GCOUNT, 1)
        for t in S.counter_batch_tables(st, rids, (kb, ko)):
            repo.converge(t)
        cur = st
        for r in range(rounds):
            cur = S.counter_delta_np(cur, r, seed)
            bs = [O.Batch(O.GCOUNT, t) for t in S.counter_batch_tables(cur, rids, (kb, ko))]
            t0 = time.perf_counter()
            for b in bs:
                repo.converge(b)
            t_conv += time.perf_counter() - t0
        units = K * R * rounds
        sample = f"GCOUNT {K} keys x {R} replicas x {rounds} rounds of {R} peer batches"
    elif mode == "treg":
        K = 1 << 20
        rng = np.random.default_rng(S.BASE_SEED + 3)
        from bench_modes import _key_strings, _treg_values
        kb, ko = _key_strings(np.arange(K, dtype=np.uint64), b"t")
        repo = O.Repo(O.TREG)
        bs = []
        for j in range(rounds + 1):
            vb, vo = _treg_values(rng, K)
            bs.append(O.Batch(O.TREG, {"key_bytes": kb, "key_offs": ko, "val_bytes": vb, "val_offs": vo,
                                       "ts": rng.integers(0, 1 << 20, K).astype(np.uint64)}))
        repo.converge(bs[0])
        t0 = time.perf_counter()
        for b in bs[1:]:
            repo.converge(b)
        t_conv = time.perf_counter() - t0
        units = K * rounds
        sample = f"TREG {K} keys x {rounds} delta batches"
    elif mode == "tlog":
        K = 1 << 18
        st, dl = S.tlog_tables(K, seed=S.BASE_SEED + 4, rounds=rounds)
        repo = O.Repo(O.TLOG)
        repo.converge(st)
        n_state = len(st["ts"])
        for d in dl:
            b = O.Batch(O.TLOG, d)
            units += n_state + len(d["ts"])
            t0 = time.perf_counter()
            repo.converge(b)
            t_conv += time.perf_counter() - t0
            n_state = len(repo.state()["ts"])
        sample = f"TLOG {K} logs, {rounds} delta batches"
    elif mode == "ujson":
        D = 1 << 17
        st, dl = S.ujson_tables(D, seed=S.BASE_SEED + 5, rounds=rounds, R=16)
        repo = O.Repo(O.UJSON, 1)
        repo.converge(st)
        for d in dl:
            # units as on the GPU line: dots of the touched documents' state
            # (elements + cloud) plus the delta's dots (untimed bookkeeping)
            cur = repo.state()
            eo, co = cur["el_offs"].astype(np.int64), cur["cloud_offs"].astype(np.int64)
            kb, ko = cur["key_bytes"], cur["key_offs"].astype(np.int64)
            size = {bytes(kb[ko[i]:ko[i + 1]]): (eo[i + 1] - eo[i]) + (co[i + 1] - co[i]) for i in range(len(ko) - 1)}
            dkb, dko = d["key_bytes"], d["key_offs"].astype(np.int64)
            units += sum(int(size.get(bytes(dkb[dko[i]:dko[i + 1]]), 0)) for i in range(len(dko) - 1))
            units += len(d["elems"]) + len(d["cloud_ids"])
            b = O.Batch(O.UJSON, d)
            t0 = time.perf_counter()
            repo.converge(b)
            t_conv += time.perf_counter() - t0
        sample = f"UJSON {D} docs, Zipf(1.1), {rounds} delta batches"
    return {"value": units / t_conv, "unit": "same as value", "cores": 1, "kind": "port",
            "sample": f"{sample} ({units} units, {t_conv:.2f} s converge, oracle/jy_oracle.cpp, 1 thread)"}


def _to_dev(a, dev, dtype=None):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    t = torch.from_numpy(a).to(dev)
    return t if dtype is None else t.to(dtype)


# ---- GCOUNT (config 1: 1M keys x 16 replicas) --------------------------------

def _u64max(a, b):
    """elementwise max of int64 tensors holding u64 bit patterns"""
    import torch
    flip = torch.tensor(-(1 << 63), dtype=torch.int64, device=a.device)
    return torch.maximum(a ^ flip, b ^ flip) ^ flip


def bench_gcount(args, eng, dev, dist, rank, world):
    import torch
    from jylis_amd import synth as S
    K, R = args.keys or (1 << 20), 16
    seed = S.BASE_SEED + 1
    kb, ko = S.counter_keys(K, prefix=f"s{rank}:g".encode(), width=7)
    eng.intern(0, (kb, ko))
    cols = eng.replica_cols(S.replica_ids(R, seed).tolist())
    st = torch.empty((1, R, K), dtype=torch.int64, device=dev)
    S.counter_rows_torch(st, seed, wrap_frac=False)
    eng.gcount_converge_block(cols, 0, st[0])
    nb = max(1, args.batches)
    ds, prev = [], st
    for j in range(nb):
        d = torch.empty_like(st)
        S.counter_rows_torch(d, seed, rnd=j, prev=prev)
        ds.append(d)
        prev = d
    elapsed, kt = _timed(args.steps, args.warmup, lambda i: eng.gcount_converge_block(cols, 0, ds[i % nb][0]),
                         dist, dev, eng=eng)
    t = _max_over_ranks(elapsed, dist, dev)
    # verification: sampled keys recomputed as the max over every batch applied
    sample = torch.from_numpy(np.random.default_rng(5).integers(0, K, 64)).to(dev)
    exp = st[0][:, sample].clone()
    for i in range(args.warmup + args.steps):
        exp = _u64max(exp, ds[i % nb][0][:, sample])
    exp = exp.cpu().numpy().view(np.uint64)
    verified = all(np.array_equal(eng.counter_export(0, R, int(k), 1).reshape(R), exp[:, j])
                   for j, k in enumerate(sample.tolist()))
    cells = R * K
    k = float(np.mean(kt))
    return {"workload": f"GCOUNT converge: {K} keys x {R} replicas per GPU, one full delta batch "
                        f"({R} peer batches) per step (SURVEY 8d config 1)",
            "unit_of_work": "cell merge", "units_per_step_per_gpu": cells, "verified_sampled_keys": bool(verified),
            "value": world * cells * args.steps / t, "ms_per_step": t / args.steps * 1e3,
            "roofline": {"bound": "hbm", "achieved": 24 * cells / k / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": 24 * cells / k / 1e9 / HBM_PEAK_GBS, "kernel": "k_block_max<true>",
                         "kernel_ms_avg": k * 1e3, "bytes_per_unit": 24,
                         "note": "state (128 MiB) + delta fit the 256 MiB Infinity Cache"}}


# ---- TREG (config 3: 64M keys over 8 GPUs = 8M per GPU) -----------------------

def _treg_values(rng, n):
    """random 1-16 byte values, ~20% sharing one of 16 8-byte prefixes"""
    from jylis_amd import synth as S
    vb, vo = S.random_values(rng, n, 1, 16)
    lens = np.diff(vo.astype(np.int64))
    share = (rng.random(n) < 0.2) & (lens >= 8)
    prefixes = rng.integers(0, 256, (16, 8), dtype=np.uint8)
    pick = rng.integers(0, 16, n)
    starts = vo[:-1].astype(np.int64)
    for j in range(8):
        idx = starts[share] + j
        vb[idx] = prefixes[pick[share], j]
    return vb, vo


def bench_treg_overlap(args, eng, dev, dist, rank, world):
    """Routed TREG with keys that several peers flushed in the same step
    (VERDICT r2 #5): S shards (engines) on one GPU exchange through a
    LocalFabric; source r ingests n = G / S records per step, its own share of
    the G keys except that a fraction `overlap` of them are keys of source
    r + 1's share, so those keys reach their owner from two sources in one
    step.  The same run with no overlap is timed first; both per-step times
    are reported (same records per step)."""
    import torch
    from jylis_amd import synth as S_
    from jylis_amd._lib import TREG
    from jylis_amd.engine import Engine
    from jylis_amd.route import LocalFabric, TregRouter, long_bytes, owners
    S = max(2, args.shards)
    G = args.keys or (8 << 20)
    n = G // S
    engs = [eng] + [Engine(device=eng.device, counter_columns=16) for _ in range(S - 1)]
    for e in engs[1:]:
        e.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    gidx = np.arange(G, dtype=np.uint64)
    kb, ko = _key_strings(gidx, b"t")
    own = owners(kb, ko, S)
    slot = np.zeros(G, np.uint32)
    for d in range(S):
        ix = np.nonzero(own == d)[0]
        width = int(ko[1] - ko[0])
        sub = np.ascontiguousarray(kb.reshape(G, width)[ix]).reshape(-1)
        slot[ix] = engs[d].intern(TREG, (sub, np.arange(len(ix) + 1, dtype=np.uint64) * np.uint64(width)))
    rng = np.random.default_rng(S_.BASE_SEED + 31)
    nb = max(1, args.batches, args.warmup + args.steps)

    def keys_of(r, f):
        mine = np.arange(r, G, S, dtype=np.int64)[:n]
        m = int(round(f * n))
        if m:  # the head of source r + 1's share, which source r + 1 ingests too (f <= 1/2)
            other = np.arange((r + 1) % S, G, S, dtype=np.int64)[:n]
            mine = np.concatenate([mine[:n - m], other[:m]])
        return mine

    def batches_for(f, tbase):
        out = []
        for j in range(nb + 1):
            per = []
            for r in range(S):
                k = keys_of(r, f)
                vb, vo = _treg_values(rng, n)
                pre, lr = engs[r].pack_values(TREG, (vb, vo))
                ts = (rng.integers(0, 1 << 20, n) + (j << 18) + tbase).astype(np.uint64)
                per.append((k, tuple(_to_dev(a, dev) for a in (own[k], slot[k], ts, pre, lr)) + (long_bytes(lr),)))
            out.append(per)
        return out

    res = {}
    for run, f in enumerate((0.0, float(args.overlap))):
        # the second run's timestamps lie above every one of the first run's:
        # the state the first run left never wins a key the second run writes
        bs = batches_for(f, run * ((nb + 8) << 18))
        router = TregRouter(engs, LocalFabric(S))
        router.step([b for _, b in bs[0]])
        elapsed, _ = _timed(args.steps, args.warmup, lambda i: router.step([b for _, b in bs[1 + i % nb]]), dist, dev)
        router.drain()
        # verification: sampled keys of source 0's batches, LWW over every
        # source's applied batches that hold them, against the owner's register
        applied = [bs[0]] + [bs[1 + i % nb] for i in range(args.warmup + args.steps)]
        samp = np.random.default_rng(3).choice(keys_of(0, f), 64, replace=False)
        best = {}
        for per in applied:
            for r, (k, b) in enumerate(per):
                pos = {int(x): i for i, x in enumerate(k)}
                hit = [(int(g), pos[int(g)]) for g in samp if int(g) in pos]
                if not hit:
                    continue
                ii = torch.tensor([i for _, i in hit], device=dev)
                ts_h = b[2][ii].cpu().numpy().view(np.uint64)
                pre_h, lr_h = b[3][ii].cpu().numpy().view(np.uint64), b[4][ii].cpu().numpy().view(np.uint64)
                for (g, _), t_, p_, l_ in zip(hit, ts_h, pre_h, lr_h):
                    cand = (int(t_), engs[r].value_bytes(TREG, p_, l_))
                    if g not in best or cand > best[g]:
                        best[g] = cand
        ok = True
        for g in samp:
            e = engs[int(own[g])]
            gts, gpre, glr = e.treg_read(np.array([slot[g]], np.uint32))
            ok = ok and (int(gts[0]), e.value_bytes(TREG, gpre[0], glr[0])) == best[int(g)]
        res[f] = (elapsed / args.steps, ok)
        del bs, router
    for e in engs[1:]:
        e.close()
    (t0, ok0), (t1, ok1) = res[0.0], res[float(args.overlap)]
    return {"workload": f"TREG routed LWW converge: {G} keys over {S} shards on one GPU (LocalFabric), {n} records "
                        f"per source per step; {args.overlap:.0%} of each source's keys shared with another source "
                        f"in the same step (SURVEY 8d config 3, 8e)",
            "unit_of_work": "routed record", "value": S * n / t1, "ms_per_step": t1 * 1e3,
            "no_overlap_ms_per_step": t0 * 1e3, "overlap_vs_no_overlap": t1 / t0, "overlap": args.overlap,
            "verified_sampled_keys": bool(ok0 and ok1)}


def bench_treg(args, eng, dev, dist, rank, world):
    """Routed TREG converge: every rank ingests 1/world of the global key space
    per step and routes records + long value bytes to their owners (RCCL
    all-to-all), which LWW-merge them.  At world 1 the exchange is skipped
    unless --route (then it runs the same kernels against itself)."""
    if args.overlap is not None:
        return bench_treg_overlap(args, eng, dev, dist, rank, world)
    if args.node:
        return bench_treg_node(args, eng, dev, dist, rank, world)
    import torch
    from jylis_amd import synth as S
    from jylis_amd._lib import TREG
    from jylis_amd.route import ShardRouter, TregRouter, long_bytes
    Kper = args.keys or (8 << 20)
    G = Kper * world
    rng = np.random.default_rng(S.BASE_SEED + 3 + 1000 * rank)
    # ingest share of this rank: global keys k = rank, rank + world, ...
    idx = np.arange(rank, G, world, dtype=np.uint64)
    kb, ko = _key_strings(idx, b"t")
    routed = world > 1 or args.route
    t0 = time.perf_counter()
    if args.resolve and not routed:
        raise SystemExit("--resolve needs the routed path (--route or --gpus > 1)")
    if routed:
        import torch.distributed as tdist

        from jylis_amd.route import DistFabric, KeyResolver, LocalFabric
        cpu_group = tdist.new_group(backend="gloo") if world > 1 else None
        fabric = DistFabric(tdist, cpu_group=cpu_group) if world > 1 else LocalFabric(1)
        # owner slots resolved on the GPU (k_keyroute.hip): key strings in HBM
        kr = KeyResolver([eng], fabric, TREG)
        ((own_d, slot_d),) = kr.resolve([(_to_dev(kb, dev), _to_dev(ko, dev))])
        own, slot = own_d.cpu().numpy().view(np.uint32), slot_d.cpu().numpy().view(np.uint32)
        tr = TregRouter([eng], fabric)
    else:
        slot = eng.intern(TREG, (kb, ko))
        own = np.zeros(len(slot), np.uint32)
        cpu_group = None
    setup_s = time.perf_counter() - t0
    n = len(slot)
    m = n // 16 if args.resolve else 0  # --resolve: keys new to the node in every step
    batches, keysets = [], []
    # plain (not routed) and a dense slot range: the block form
    # (jy_treg_converge_block: no slot stream), then the keyed form over a
    # continuation of fresh batches, timed beside it
    block = not routed and not args.resolve and bool((slot == np.arange(len(slot), dtype=slot.dtype)).all())
    nrun = max(1, args.batches, args.warmup + args.steps)
    # batch 0 = initial state; a distinct batch for every step (no replays)
    for j in range((2 if block else 1) * nrun + 1):
        vb, vo = _treg_values(rng, n + m)
        pre, lr = eng.pack_values(TREG, (vb, vo))
        # fresh writes: batch j's timestamps sit 2^18 above batch j-1's in a
        # 2^20 window, so ~70% of keys take the delta and ties are dense
        ts = (rng.integers(0, 1 << 20, n + m) + (j << 18)).astype(np.uint64)
        if args.resolve:
            # the batch as key strings in HBM: this rank's keys + m new ones
            nkb, nko = _key_strings(np.arange(m, dtype=np.uint64) + np.uint64(m * j), b"n%d:" % rank)
            w = int(ko[1] - ko[0])
            keysets.append((_to_dev(np.concatenate([kb, nkb]), dev),
                            _to_dev(np.concatenate([ko, nko[1:] + np.uint64(len(kb))]), dev)))
            batches.append((None, None) + tuple(_to_dev(a, dev) for a in (ts, pre, lr)) + (long_bytes(lr),))
        else:
            batches.append(tuple(_to_dev(a, dev) for a in (own, slot, ts, pre, lr)) + (long_bytes(lr),))
    win = []
    resolve_s = []

    def step_of(b, j=None):
        if args.resolve:
            # the step resolves its key strings on the GPU, then routes the entries
            h0 = time.perf_counter()
            ((o, s_),) = kr.resolve([keysets[j]])
            resolve_s.append(time.perf_counter() - h0)
            b = (o, s_) + b[2:]
        o, s, ts, pre, lr, nbytes = b
        if routed:
            tr.step([b])
        elif use_block[0]:
            eng.treg_converge_block(0, ts, pre, lr)
        else:
            eng.treg_converge(s, ts, pre, lr)

    use_block = [block]
    step_of(batches[0], 0)
    # winners per step from timestamps (ties need the value compare: rare)
    cur = batches[0][2].clone() if not routed else None
    nb = nrun
    elapsed, kt = _timed(args.steps, args.warmup, lambda i: step_of(batches[1 + i % nb], 1 + i % nb), dist, dev,
                         eng=None if routed else eng)
    applied_idx = [0] + [1 + i % nb for i in range(args.warmup + args.steps)]
    keyed = None
    if block:  # the keyed form over the next batches (fresh timestamps: the same winner fractions)
        use_block[0] = False
        el2, kt2 = _timed(args.steps, args.warmup, lambda i: step_of(batches[1 + nb + i % nb], 1 + nb + i % nb),
                          dist, dev, eng=eng)
        applied_idx += [1 + nb + i % nb for i in range(args.warmup + args.steps)]
        keyed = (el2, float(np.mean(kt2)))
    if cur is not None:
        for i in range(args.warmup + args.steps):
            t = batches[1 + i % nb][2]
            w = (t > cur)
            if i >= args.warmup:
                win.append(float(w.float().mean()))
            cur = torch.where(w, t, cur)
    t = _max_over_ranks(elapsed, dist, dev)
    k = float(np.mean(kt))
    wf = float(np.mean(win)) if win else 0.5
    # sampled keys of this rank's ingest: LWW over every applied batch, (ts,
    # value) with the value order of Pony's String (bytewise, shorter first on
    # a prefix), against the OWNER's register (asked over the CPU group at N > 1)
    if routed:
        tr.drain()
    idx = np.random.default_rng(6 + rank).integers(0, n, 128)
    applied = [batches[j] for j in applied_idx]
    best = {}
    for b in applied:
        ts_h = b[2][idx].cpu().numpy().view(np.uint64)
        pre_h, lr_h = b[3][idx].cpu().numpy().view(np.uint64), b[4][idx].cpu().numpy().view(np.uint64)
        for j in range(len(idx)):
            cand = (int(ts_h[j]), eng.value_bytes(TREG, pre_h[j], lr_h[j]))
            if j not in best or cand > best[j]:
                best[j] = cand
    o_h, s_h = own[idx], slot[idx]

    def answer(slots):
        gts, gpre, glr = eng.treg_read(slots)
        return [(int(a), eng.value_bytes(TREG, p, q)) for a, p, q in zip(gts, gpre, glr)]
    got = _ask_owners(dist, cpu_group if routed else None, rank, world,
                      [(int(o), int(x)) for o, x in zip(o_h, s_h)], answer)
    verified = _all_true(all(got[j] == best[j] for j in range(len(idx))), dist, dev)
    # SURVEY 8d prices a key LWW select at 48 B (16 delta + 16 state read +
    # 16 state write, the write counted unconditionally); what the kernel
    # actually moves in this layout is reported beside it
    bytes_per_key = 48
    whole = n * 24 > (256 << 20)  # k_treg_lww<true>: state over the Infinity Cache
    moved = (0 if block else 4) + 24 + 8 + 8 + (16 if whole else 16 * wf) + (16 * (1 - wf) if whole else 0)
    out = {"workload": f"TREG LWW converge: {G} keys over {world} GPU(s) ({Kper} per GPU), one delta per key "
                       f"per step{' routed by owner (all-to-all)' if routed else ''}"
                       + (f"; every step first resolves its {n + m} key strings ({m} new to the node) on the GPU "
                          f"(KeyResolver: regroup by owner, exchange, intern on the owner, slots back)"
                          if args.resolve else "") + " (SURVEY 8d config 3)",
           "unit_of_work": "key LWW select", "units_per_step_per_gpu": n + m,
           "value": world * (n + m) * args.steps / t, "ms_per_step": t / args.steps * 1e3, "setup_s": setup_s,
           "winner_fraction": wf, "verified_sampled_keys": verified}
    if args.resolve:
        out["metric"] = "TREG end-to-end routed ingest (key strings resolved on the GPU + routed LWW)"
        out["resolve_host_ms_avg"] = float(np.mean(resolve_s[-args.steps:])) * 1e3
        out["keys_interned_after"] = int(eng.nkeys(TREG))
    if not routed:
        out["roofline"] = {"bound": "hbm", "achieved": bytes_per_key * n / k / 1e9, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": bytes_per_key * n / k / 1e9 / HBM_PEAK_GBS,
                           "kernel": "k_treg_lww<..., dense>" if block else "k_treg_lww", "kernel_ms_avg": k * 1e3,
                           "bytes_per_unit": bytes_per_key,
                           "bytes_note": "SURVEY 8d: 16 delta + 16 state read + 16 state write per key",
                           "bytes_moved_per_unit": moved,
                           "bytes_moved_note": ("" if block else "4 slot + ") + "24 delta (ts, pre, lr) + 8 state ts "
                                               "read + 8 ts rewritten + 16 handle write x winner fraction (a state "
                                               "over the 256 MiB MALL: every handle written, losers' read)"}
        if Kper == 8 << 20:  # the PMC run's workload (scripts/gpu_r06_pmc.sh MODES=treg)
            with_traffic(out["roofline"], "treg" if block else "treg_keyed")
        if block:
            out["form"] = ("block: the step's batch holds one delta for every slot in slot order "
                           "(jy_treg_converge_block, no slot stream, no claim); the keyed form "
                           "(jy_treg_converge, slot per entry) is timed beside it on fresh batches")
            el2, k2 = keyed
            out["keyed"] = {"ms_per_step": el2 / args.steps * 1e3, "kernel_ms_avg": k2 * 1e3,
                            "value": world * (n + m) * args.steps / el2,
                            "frac": bytes_per_key * n / k2 / 1e9 / HBM_PEAK_GBS,
                            "bytes_moved_per_unit": moved + 4}
            if Kper == 8 << 20:
                t_k, src_k = pmc_traffic("treg_keyed")
                out["keyed"]["traffic"] = t_k
                out["keyed"]["traffic_source"] = src_k
    else:
        out["step_ms_avg_events"] = k * 1e3
        out["self_direct"] = tr.self_direct
        if tr.self_direct:
            out["self_direct_note"] = ("each shard merges its own entries where they lie (jy_treg_route_part_self); "
                                       "only the other shards' entries are placed in runs and exchanged -- at "
                                       "1 GPU the step is owner count + partition pass + the owned merge")
    return out


def node_for(args, dev, dist, rank, world, **engine_kw):
    """the node of a --node run: one process per GPU over RCCL at N > 1 (the
    rank-0 ncclUniqueId shared over the CPU group), or --node-shards shards on
    this GPU at N = 1 (RCCL for one shard, the copy fabric for more)"""
    from jylis_amd.node import Node, unique_id
    if world > 1:
        import torch.distributed as tdist
        cpu = tdist.new_group(backend="gloo")
        box = [unique_id() if rank == 0 else None]
        tdist.broadcast_object_list(box, src=0, group=cpu)
        return Node(world, "rccl", devices=[dev.index], nlocal=1, rank0=rank, uid=box[0], **engine_kw), cpu
    S = max(1, args.node_shards)
    return Node(S, "rccl" if S == 1 else "copy", devices=[dev.index] * S, **engine_kw), None


def bench_treg_node(args, eng, dev, dist, rank, world):
    """TREG through the node (jy_node_treg_converge): every step is ONE call
    per process with a peer batch of KEY STRINGS and values in HBM -- the
    library hashes the keys, regroups them by owner, exchanges (RCCL over
    xGMI at N > 1), interns them on the owner and LWW-merges there.  Nothing
    is pre-resolved: the step pays for the key probe (_data_for) on every
    key, as RepoManagerCore.converge_deltas does (repo_treg.pony:37-42)."""
    import torch
    from jylis_amd import synth as S
    from jylis_amd._lib import TREG
    Kper = args.keys or (8 << 20)
    node, cpu = node_for(args, dev, dist, rank, world, key_capacity=[1024, 1024, 2 * Kper, 1024, 1024])
    shards = node.S
    G = Kper * max(world, shards)
    nproc_keys = G // world  # keys this process ingests per step
    rng = np.random.default_rng(S.BASE_SEED + 3 + 1000 * rank)
    idx = np.arange(rank, G, world, dtype=np.uint64)[:nproc_keys]
    kb, ko = _key_strings(idx, b"t")
    kb_d, ko_d = _to_dev(kb, dev), _to_dev(ko, dev)
    nb = max(1, args.batches, args.warmup + args.steps) + 1
    batches = []
    for j in range(nb):
        vb, vo = _treg_values(rng, nproc_keys)
        ts = (rng.integers(0, 1 << 20, nproc_keys) + (j << 18)).astype(np.uint64)
        batches.append((ts, vb, vo, _to_dev(ts, dev), _to_dev(vb, dev), _to_dev(vo, dev)))

    def step(i):
        b = batches[i]
        node.treg_converge(kb_d, ko_d, b[3], b[4], b[5])

    t0 = time.perf_counter()
    step(0)  # batch 0 creates every key (the setup converge)
    node.sync()
    setup_s = time.perf_counter() - t0
    elapsed, _ = _timed(args.steps, args.warmup, lambda i: step(1 + i % (nb - 1)), dist, dev, drain=node.sync)
    node.sync()
    t = _max_over_ranks(elapsed, dist, dev)
    st = node.stats()
    # sampled keys of this process's ingest: LWW over every applied batch
    # against the owner's register (asked over the CPU group at N > 1)
    samp = np.random.default_rng(6 + rank).integers(0, nproc_keys, 96)
    applied = [0] + [1 + i % (nb - 1) for i in range(args.warmup + args.steps)]
    best = {}
    for j in applied:
        ts, vb, vo = batches[j][:3]
        for q in samp:
            cand = (int(ts[q]), bytes(vb[int(vo[q]):int(vo[q + 1])]))
            if int(q) not in best or cand > best[int(q)]:
                best[int(q)] = cand
    keys = [bytes(kb[int(ko[q]):int(ko[q + 1])]) for q in samp]
    if world == 1:
        ok = True
        for q, k in zip(samp, keys):
            e = node.engine(node.shard_of(k))
            s = e.lookup(TREG, [k])
            gts, gpre, glr = e.treg_read(s)
            ok = ok and (int(gts[0]), e.value_bytes(TREG, gpre[0], glr[0])) == best[int(q)]
    else:
        e = node.engine(rank)

        def answer(slots):
            gts, gpre, glr = e.treg_read(slots)
            return [(int(a), e.value_bytes(TREG, p_, q_)) for a, p_, q_ in zip(gts, gpre, glr)]
        reqs = []
        for k in keys:  # the owner's slot: every owner interned every key it received
            reqs.append((node.shard_of(k), k))
        every = [None] * world
        dist.all_gather_object(every, reqs, group=cpu)
        mine = [(src, i, k) for src, rq in enumerate(every) for i, (o, k) in enumerate(rq) if o == rank]
        ans = answer(e.lookup(TREG, [k for _, _, k in mine])) if mine else []
        back = [None] * world
        dist.all_gather_object(back, [(src, i, a) for (src, i, _), a in zip(mine, ans)], group=cpu)
        got = {}
        for lst in back:
            for src, i, a in lst:
                if src == rank:
                    got[i] = a
        ok = all(got[i] == best[int(q)] for i, q in enumerate(samp))
    verified = _all_true(ok, dist, dev)
    ms = t / args.steps * 1e3
    out = {"workload": f"TREG through the node: {G} keys over {shards} shard(s) ({'RCCL' if world > 1 or shards == 1 else 'copy fabric, one GPU'}), "
                       f"every process converges {nproc_keys} key strings + values per step in ONE jy_node_treg_converge "
                       f"(hash, regroup by owner, exchange, intern on the owner, LWW) (SURVEY 8d config 3, 8e)",
           "unit_of_work": "key LWW select (keyed, routed)", "value": world * nproc_keys * args.steps / t,
           "ms_per_step": ms, "setup_s": setup_s, "node_shards": shards,
           "exchange_bytes_sent_per_step": st["bytes_sent"], "keys_received_per_step": st["keys_received"],
           "verified_sampled_keys": verified}
    if Kper == 8 << 20 and world == 1 and shards == 1:  # the PMC run's workload (scripts/gpu_r06_pmc.sh MODES=node)
        tr, src = pmc_traffic("node")
        out["traffic_per_call"], out["traffic_source"] = tr, src
    node.close()
    return out


def _key_strings(idx, prefix):
    """global key indices -> fixed-width keys (bytes, offs)"""
    n = len(idx)
    width = 10
    digits = np.empty((n, width), np.uint8)
    v = np.asarray(idx, np.uint64).copy()
    for j in range(width - 1, -1, -1):
        digits[:, j] = (v % np.uint64(10)).astype(np.uint8) + ord("0")
        v //= np.uint64(10)
    pre = np.frombuffer(prefix, np.uint8)
    rows = np.concatenate([np.broadcast_to(pre, (n, len(pre))), digits], axis=1)
    return np.ascontiguousarray(rows).reshape(-1), np.arange(n + 1, dtype=np.uint64) * np.uint64(rows.shape[1])


# ---- TLOG (config 4: 4M keys) --------------------------------------------------

def bench_tlog(args, eng, dev, dist, rank, world):
    if world > 1 or args.route:
        return _bench_csr_routed(args, eng, dev, dist, rank, world, "tlog")
    import torch
    from jylis_amd import synth as S
    from jylis_amd._lib import TLOG
    K = args.keys or (4 << 20)
    # a distinct batch for every step: a replayed batch is all duplicates
    nb = max(1, args.batches, args.warmup + args.steps)
    st, dl = S.tlog_tables(K, seed=S.BASE_SEED + 4 + 1000 * rank, rounds=nb)
    slots = eng.intern(TLOG, (st["key_bytes"], st["key_offs"]))
    assert (slots == np.arange(K)).all()
    dev_batches = []
    for b in [st] + dl:
        pre, lr = eng.pack_values(TLOG, (b["val_bytes"], b["val_offs"]))
        dev_batches.append(tuple(_to_dev(a, dev) for a in (slots, b["cutoff"], b["ent_offs"], b["ts"], pre, lr)))
    eng.tlog_converge(*dev_batches[0])
    eng.sync()
    n_state0 = len(st["ts"])

    def step(i):
        eng.tlog_converge(*dev_batches[1 + i % nb])

    st0 = eng.tlog_stats()
    elapsed, kt = _timed(args.steps, args.warmup, step, dist, dev, eng=eng)
    t = _max_over_ranks(elapsed, dist, dev)
    eng.sync()  # settles the last merge: its spill (if any) is counted
    st1 = eng.tlog_stats()
    # replay the same sequence on a fresh engine pass to get exact in/out
    # entry counts per step: state entries are the running total (the engine
    # keeps it), so re-run step by step outside the timed region
    from jylis_amd.engine import Engine
    e2 = Engine(device=eng.device, key_capacity=[1024, 1024, 1024, K, 1024])
    e2.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    e2.intern(TLOG, (st["key_bytes"], st["key_offs"]))
    b2 = []
    for b in [st] + dl:
        pre, lr = e2.pack_values(TLOG, (b["val_bytes"], b["val_offs"]))
        b2.append(tuple(_to_dev(a, dev) for a in (slots, b["cutoff"], b["ent_offs"], b["ts"], pre, lr)))
    e2.tlog_converge(*b2[0])
    byts, ins, moved = [], [], []
    prev = _tlog_total(e2)
    for i in range(args.warmup + args.steps):
        bt = b2[1 + i % nb]
        e2.tlog_converge(*bt)
        now = _tlog_total(e2)
        nd = int(bt[3].numel())
        if i >= args.warmup:
            # 16 B read per input entry + 16 B written per output
            # entry + 24 B per key; moved: what the append layout touches
            byts.append(16 * (prev + nd) + 16 * now + 24 * K)
            moved.append(24 * nd + 32 * max(now - prev, 0) + 64 * int(bt[0].numel()))
            ins.append(prev + nd)
        prev = now
    e2.close()
    verified = _verify_tlog(eng, st, [st] + [dl[i % nb] for i in range(args.warmup + args.steps)], K)
    k = float(np.mean(kt))
    avg_b = float(np.mean(byts))
    units = float(np.mean(ins))
    roof = {"bound": "hbm", "achieved": avg_b / k / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": avg_b / k / 1e9 / HBM_PEAK_GBS,
            "kernel": "TLOG converge (k_tlog_*, all launches of one call)",
            "converge_ms_avg": k * 1e3, "bytes_per_converge": avg_b,
            "bytes_note": "SURVEY 8d: 16 B read per input entry (state + delta) + 16 B written per "
                          "output entry + 24 B per key (a whole-state rewrite)",
            "min_bytes_moved_per_converge": float(np.mean(moved)),
            "frac_moved": float(np.mean(moved)) / k / 1e9 / HBM_PEAK_GBS,
            "min_bytes_moved_note": "append layout lower bound: 24 B per delta entry read + 32 B per "
                                    "net new entry written + 64 B meta per delta key"}
    if K == 4 << 20:  # the PMC run's workload (scripts/gpu_r06_pmc.sh MODES=tlog)
        with_traffic(roof, "tlog")
    return {"workload": f"TLOG converge: {K} logs, state ~Geom(8, cap 64) entries, delta ~Geom(2) per key "
                        f"per step, dups/ties/cutoffs (SURVEY 8d config 4); {n_state0} initial entries",
            "unit_of_work": "log entry (input)", "value": world * units * args.steps / t,
            "ms_per_step": t / args.steps * 1e3, "verified_sampled_keys": bool(verified),
            # merges of warmup + timed steps that spilled (re-merged after a
            # compaction, host never waited) and the compactions they caused
            "spills_compactions": [st1["spills"] - st0["spills"], st1["compactions"] - st0["compactions"]],
            "roofline": roof}


def _verify_tlog(eng, st, applied, K, nsample=128, locate=None, ask=None):
    """sampled logs recomputed from the applied tables (union of entries,
    largest cutoff, newest first, value order bytewise) against the owner's
    log: locate(k) -> (owner, slot), ask(reqs, answer) -> answers (bench runs
    at N > 1); by default slot = key index on this engine"""
    from jylis_amd._lib import TLOG
    samp = np.random.default_rng(7).integers(0, K, nsample)
    want = {int(k): (0, set()) for k in samp}
    for b in applied:
        eo_, vo_ = np.asarray(b["ent_offs"], np.int64), np.asarray(b["val_offs"], np.int64)
        for k in want:
            cut, ents = want[k]
            cut = max(cut, int(b["cutoff"][k]))
            for j in range(eo_[k], eo_[k + 1]):
                ents.add((int(b["ts"][j]), bytes(b["val_bytes"][vo_[j]:vo_[j + 1]])))
            want[k] = (cut, ents)

    def answer(slots):
        cut_g, offs_g, ts_g, pre_g, lr_g = eng.tlog_read(slots)
        return [(int(cut_g[i]), [(int(ts_g[j]), eng.value_bytes(TLOG, pre_g[j], lr_g[j]))
                                 for j in range(offs_g[i], offs_g[i + 1])]) for i in range(len(slots))]
    keys = list(want)
    if locate is None:
        got = answer(np.array(keys, np.uint32))
    else:
        got = ask([locate(k) for k in keys], answer)
    verified = True
    for (k, (cut, ents)), (gcut, gents) in zip(want.items(), got):
        exp = sorted((e for e in ents if e[0] >= cut), reverse=True)
        verified = verified and gcut == cut and gents == exp
    return bool(verified)


def _doc_index(t):
    """the index of every key of a synth table (fixed-width keys ending in 8 digits)"""
    kb, ko = np.asarray(t["key_bytes"], np.uint8), np.asarray(t["key_offs"], np.int64)
    n = len(ko) - 1
    if n == 0:
        return np.zeros(0, np.int64)
    rows = kb.reshape(n, int(ko[1] - ko[0]))[:, -8:].astype(np.int64) - ord("0")
    return rows @ (10 ** np.arange(7, -1, -1, dtype=np.int64))


def _bench_csr_routed(args, eng, dev, dist, rank, world, kind):
    """Routed TLOG / UJSON converge: every rank ingests its own
    peer batches (a key space of its own, keys hash-owned by all ranks) and
    TlogRouter / UjsonRouter partition them into fixed-capacity runs, move
    them with RCCL all-to-alls in key-range chunks (chunk c + 1 in flight
    while chunk c merges) and the owners merge them.  At world 1 (--route)
    the same kernels run against one shard, without an exchange."""
    import torch
    from jylis_amd import synth as S
    from jylis_amd._lib import TLOG, UJSON
    from jylis_amd.repo import RepoUJSON
    from jylis_amd.route import DistFabric, LocalFabric, ShardRouter, TlogRouter, UjsonRouter, long_bytes
    nb = max(1, args.batches, args.warmup + args.steps)
    ctype = TLOG if kind == "tlog" else UJSON
    K = args.keys or ((4 << 20) if kind == "tlog" else (1 << 20))
    t0 = time.perf_counter()
    if kind == "tlog":
        st, dl = S.tlog_tables(K, seed=S.BASE_SEED + 4 + 1000 * rank, rounds=nb, key_prefix=b"l%d:" % rank)
    else:
        # one cluster of 16 replicas: every shard registers the ids in one order
        st, dl = S.ujson_tables(K, seed=S.BASE_SEED + 5 + 1000 * rank, rounds=nb, R=16, key_prefix=b"u%d:" % rank,
                                id_seed=S.BASE_SEED + 5)
        eng.replica_cols(S.replica_ids(16, S.BASE_SEED + 5).tolist())
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    import torch.distributed as tdist
    cpu_group = tdist.new_group(backend="gloo") if world > 1 else None
    ctl = ShardRouter(rank, world, lambda tab: eng.intern(ctype, tab), dist=tdist if world > 1 else None,
                      group=cpu_group)
    own, slot = ctl.resolve(st["key_bytes"], st["key_offs"])
    fabric = DistFabric(tdist, cpu_group=cpu_group) if world > 1 else LocalFabric(1)
    router = (TlogRouter if kind == "tlog" else UjsonRouter)([eng], fabric)
    batches, units = [], []
    repo = RepoUJSON(eng) if kind == "ujson" else None
    for b in [st] + dl:
        di = _doc_index(b)
        o, s_ = own[di], slot[di]
        if kind == "tlog":
            pre, lr = eng.pack_values(TLOG, (b["val_bytes"], b["val_offs"]))
            batches.append(tuple(_to_dev(a, dev) for a in (o, s_, b["cutoff"], b["ent_offs"], b["ts"], pre, lr))
                           + (long_bytes(lr),))
            units.append(len(b["ts"]))
        else:
            eo, vo, co = (np.asarray(b[k], np.uint64) for k in ("el_offs", "vv_offs", "cloud_offs"))
            dots, elems = repo._sort_segments(eo, repo._pack(b["dot_ids"], b["dot_seqs"]), np.asarray(b["elems"]))
            (vv,) = repo._sort_segments(vo, repo._pack(b["vv_ids"], b["vv_seqs"]))
            (cloud,) = repo._sort_segments(co, repo._pack(b["cloud_ids"], b["cloud_seqs"]))
            batches.append(tuple(_to_dev(a, dev) for a in (o, s_, eo, dots, elems, vo, vv, co, cloud)))
            units.append(len(dots) + len(cloud))
    router.step([batches[0]])
    router.drain()
    setup_s = time.perf_counter() - t0
    last = args.warmup + args.steps - 1

    def step(i):
        router.step([batches[1 + i % nb]])
        if i == last:
            router.drain()  # the last step's overflow is part of the timed work

    elapsed, kt = _timed(args.steps, args.warmup, step, dist, dev)
    t = _max_over_ranks(elapsed, dist, dev)
    applied = [st] + [dl[i % nb] for i in range(args.warmup + args.steps)]
    # sampled keys of this rank's ingest against their OWNERS' state (the
    # requests and answers cross the CPU group at N > 1)
    def locate(k):
        return int(own[k]), int(slot[k])

    def ask(reqs, answer):
        return _ask_owners(tdist if world > 1 else None, cpu_group, rank, world, reqs, answer)
    ok = (_verify_tlog(eng, st, applied, K, locate=locate, ask=ask) if kind == "tlog"
          else _verify_ujson(eng, repo, st, applied, K, locate=locate, ask=ask))
    verified = _all_true(ok, dist, dev)
    per_step = float(np.mean([units[1 + i % nb] for i in range(args.warmup, args.warmup + args.steps)]))
    tot = torch.tensor([per_step], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(tot)
    name = ("TLOG converge: {K} logs per rank" if kind == "tlog" else "UJSON converge: {K} docs per rank").format(K=K)
    return {"workload": f"{name}, peer batches routed to their key owners over {world} GPU(s) "
                        f"(fixed-capacity runs, chunked all-to-all overlapped with the merge; SURVEY 8d config "
                        f"{4 if kind == 'tlog' else 5}, 8e)",
            "unit_of_work": "log entry (input)" if kind == "tlog" else "delta dot (input)",
            "value": float(tot[0]) * args.steps / t, "ms_per_step": t / args.steps * 1e3,
            "step_ms_avg_events": float(np.mean(kt)) * 1e3, "generate_s": gen_s, "setup_s": setup_s,
            "routed": True, "chunks": router.chunks if world > 1 else 1, "drain_rounds": router.drains,
            "verified_sampled_keys": verified}


def _tlog_total(eng):
    """live TLOG entries (sum of all slot lengths)"""
    n = eng.nkeys(3)
    if n == 0:
        return 0
    lens = np.empty(n, np.uint64)
    cut = np.empty(n, np.uint64)
    s = np.arange(n, dtype=np.uint32)
    eng._check(eng.lib.jy_tlog_read_sizes(eng.h, n, s.ctypes.data, lens.ctypes.data, cut.ctypes.data))
    return int(lens.sum())


# ---- UJSON (config 5: 1M docs, Zipf) --------------------------------------------

def bench_ujson(args, eng, dev, dist, rank, world):
    if world > 1 or args.route:
        return _bench_csr_routed(args, eng, dev, dist, rank, world, "ujson")
    import torch
    from jylis_amd import synth as S
    from jylis_amd._lib import UJSON
    from jylis_amd.repo import RepoUJSON
    D = args.keys or (1 << 20)
    nb = max(1, args.batches, args.warmup + args.steps)
    t0 = time.perf_counter()
    st, dl = S.ujson_tables(D, seed=S.BASE_SEED + 5 + 1000 * rank, rounds=nb, R=16)
    gen_s = time.perf_counter() - t0
    repo = RepoUJSON(eng)
    repo.converge_deltas(st)
    dev_batches = []
    for b in dl:
        slots = eng.lookup(UJSON, (b["key_bytes"], b["key_offs"]))
        eo, vo, co = (np.asarray(b[k], np.uint64) for k in ("el_offs", "vv_offs", "cloud_offs"))
        dots, elems = repo._sort_segments(eo, repo._pack(b["dot_ids"], b["dot_seqs"]), np.asarray(b["elems"]))
        (vv,) = repo._sort_segments(vo, repo._pack(b["vv_ids"], b["vv_seqs"]))
        (cloud,) = repo._sort_segments(co, repo._pack(b["cloud_ids"], b["cloud_seqs"]))
        dev_batches.append((tuple(_to_dev(a, dev) for a in (slots, eo, dots, elems, vo, vv, co, cloud)),
                            len(slots), len(dots), len(cloud)))
    eng.sync()
    def step(i):
        eng.ujson_converge(*dev_batches[i % nb][0])

    marks = {}
    elapsed, kt = _timed(args.steps, args.warmup, step, dist, dev, eng=eng,
                         before_timed=lambda: marks.update(s0=eng.ujson_stats()))
    s1 = eng.ujson_stats()
    verified = _verify_ujson(eng, repo, st, [dl[i % nb] for i in range(args.warmup + args.steps)], D)
    # what the timed converges really touched and wrote (the engine's own
    # counters: the hot documents grow step by step)
    d = {k: (s1[k] - marks["s0"][k]) / args.steps for k in s1}
    t = _max_over_ranks(elapsed, dist, dev)
    k = float(np.mean(kt))
    R = 16
    # 16 B per element read (touched state + delta) and written,
    # 8 B per cloud dot read and written, 24R B of context per delta doc.
    # The join examines every dot of a touched document; since round 6 the
    # long documents converge in place (their state dots are examined by the
    # join but never read or moved), so the SURVEY bytes count them as the
    # algorithm's (logical) work: state + what the merged document holds.
    st_el = d["touched_el"] + d["inplace_state_el"]
    st_cl = d["touched_cloud"] + d["inplace_state_cloud"]
    out_el = d["out_el"] + d["inplace_state_el"] + d["inplace_added_el"]
    out_cl = d["out_cloud"] + d["inplace_state_cloud"] + d["inplace_added_cloud"]
    bytes_conv = 16 * (st_el + d["delta_el"] + out_el) + 8 * (st_cl + d["delta_cloud"] + out_cl) + 24 * R * d["delta_docs"]
    # what this layout must move: the regular path's rewrite (SURVEY's bytes
    # over the documents it rewrites), and for a document in place its delta
    # dots read once, the appended ones written, and its R column records
    # read and rewritten (32 B each)
    moved = (16 * (d["touched_el"] + d["out_el"]) + 8 * (d["touched_cloud"] + d["out_cloud"]) +
             16 * d["delta_el"] + 8 * d["delta_cloud"] + 16 * d["inplace_added_el"] + 8 * d["inplace_added_cloud"] +
             64 * R * d["inplace_docs"] + 24 * R * (d["delta_docs"] - d["inplace_docs"]))
    dots_examined = st_el + st_cl + d["delta_el"] + d["delta_cloud"]
    roof = {"bound": "hbm", "achieved": bytes_conv / k / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": bytes_conv / k / 1e9 / HBM_PEAK_GBS,
            "frac_moved": moved / k / 1e9 / HBM_PEAK_GBS, "bytes_moved_per_converge": moved,
            "bytes_moved_note": "the regular path's rewrite of the documents it takes, plus for each "
                                "document in place: its delta dots read, the appended ones written, "
                                "R column records read + rewritten",
            "kernel": "UJSON converge (k_uj_*, all launches of one call)",
            "converge_ms_avg": k * 1e3, "bytes_per_converge": bytes_conv,
            "bytes_note": "SURVEY 8d, from jy_ujson_stats_ext over the timed converges: 16 B per "
                          "element read (every state element of a delta's document + delta) and "
                          "written (merged), 8 B per cloud dot read and written, 24R B context per "
                          "delta doc; untouched documents are not counted"}
    if D == 1 << 20:  # the PMC run's workload (scripts/gpu_r06_pmc.sh MODES=ujson: warmup 6, 4 timed converges)
        with_traffic(roof, "ujson")
    return {"workload": f"UJSON converge: {D} docs (~8 leaves, R=16), Zipf(1.1) delta docs per step "
                        f"({int(d['delta_docs'])} docs, {int(d['delta_el'])} dots, {int(d['delta_cloud'])} cloud dots; "
                        f"{int(st_el)} state elements examined, {int(d['inplace_state_el'])} of them in "
                        f"{int(d['inplace_docs'])} documents converged in place), 70/20/10 INS/RM/CLR "
                        f"(SURVEY 8d config 5)",
            "unit_of_work": "dot examined", "value": world * dots_examined * args.steps / t,
            "ms_per_step": t / args.steps * 1e3, "generate_s": gen_s,
            "delta_docs_per_s": world * d["delta_docs"] * args.steps / t, "verified_sampled_docs": verified,
            "per_converge": d,
            "roofline": roof}


# ---- end-to-end ingest: the ABI path the Pony glue calls (host batches) -----------

def bench_e2e(args, eng, dev, dist, rank, world):
    """One step = what RepoGCOUNTGpu._drain does with one decoded peer batch:
    B key strings from host memory interned on the GPU (jy_keys_intern, the
    reference's per-key _data_for probe, repo_gcount.pony:36-41), then the
    (slot, replica column, value) cells merged from host memory through the
    pinned staging ring (jy_gcount_converge COO, JY_HOST).  Wall-clock per
    step, host included; the merge kernel is priced on its own too."""
    import torch
    from jylis_amd import synth as S
    K, R = args.keys or (1 << 24), 16
    B = 1 << 20
    seed = S.BASE_SEED + 11
    kb, ko = S.counter_keys(K, prefix=f"s{rank}:e".encode(), width=8)
    eng.reserve(0, K + K // 8)
    t0 = time.perf_counter()
    eng.intern(0, (kb, ko))
    setup_intern_s = time.perf_counter() - t0
    cols = eng.replica_cols(S.replica_ids(R, seed).tolist())
    rng = np.random.default_rng(seed + rank)
    nb = max(2, args.batches)
    batches = []
    L = int(ko[1] - ko[0])
    for j in range(nb):
        pick = rng.integers(0, K, B)
        # 1 in 16 keys is new to this replica (interned on the fly)
        new = rng.random(B) < 1 / 16
        rows = kb.reshape(K, L)[pick].copy()
        rows[new, 0] = ord("n")
        bkb = np.ascontiguousarray(rows).reshape(-1)
        bko = np.arange(B + 1, dtype=np.uint64) * np.uint64(L)
        col = cols[rng.integers(0, R, B)].astype(np.uint16)
        val = rng.integers(1, 1 << 62, B, dtype=np.uint64)
        batches.append((bkb, bko, col, val))
    times = {"intern": [], "converge": []}

    def step_two_calls(i):
        bkb, bko, col, val = batches[i % nb]
        a = time.perf_counter()
        slots = eng.intern(0, (bkb, bko))
        b = time.perf_counter()
        eng.gcount_converge(slots, col, val)
        c = time.perf_counter()
        times["intern"].append(b - a)
        times["converge"].append(c - b)

    def step(i):
        # one call (jy_counter_converge_keys): keys interned on the device feed the
        # merge, no slot round trip to the host
        bkb, bko, col, val = batches[i % nb]
        eng.counter_converge_keys(0, (bkb, bko), col, val)

    # the two-call path of rounds 1-3 (jy_keys_intern + jy_gcount_converge), timed beside it
    elapsed2, _ = _timed(args.steps, args.warmup, step_two_calls, dist, dev, eng=eng)
    t2 = _max_over_ranks(elapsed2, dist, dev)
    elapsed, kt = _timed(args.steps, args.warmup, step, dist, dev, eng=eng)
    t = _max_over_ranks(elapsed, dist, dev)
    k = float(np.mean(kt))
    h2d = B * (L + 8 + 2 + 8)  # key bytes + offsets, cols, values
    tail = slice(args.warmup, None)
    return {"metric": "GCOUNT end-to-end ingest throughput (host batches through the C-ABI)",
            "workload": f"GCOUNT end-to-end ingest: {B} host cells per step (one decoded peer batch; "
                        f"1/16 new keys) into {K} keys x {R} replicas: jy_counter_converge_keys (host key "
                        f"strings interned on the device + COO merge with the device slots, pinned staging)",
            "unit_of_work": "cell ingested", "value": world * B * args.steps / t,
            "ms_per_step": t / args.steps * 1e3,
            "two_calls": {"ms_per_step": t2 / args.steps * 1e3, "value": world * B * args.steps / t2,
                          "host_intern_ms": float(np.mean(times["intern"][tail])) * 1e3,
                          "host_converge_call_ms": float(np.mean(times["converge"][tail])) * 1e3,
                          "note": "jy_keys_intern (slots back to the host) + jy_gcount_converge"},
            "h2d_bytes_per_step": h2d, "h2d_GBps_effective": h2d / (t / args.steps) / 1e9,
            "setup_intern_s": setup_intern_s,
            "roofline": {"bound": "hbm", "achieved": 24 * B / k / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": 24 * B / k / 1e9 / HBM_PEAK_GBS, "kernel": "k_coo_max_keyed (merge only)",
                         "kernel_ms_avg": k * 1e3, "bytes_per_unit": 24,
                         "note": "random 8-B cells: each touches a whole 64-B line; the step is interning- "
                                 "and PCIe-bound, the merge is a small part"}}


# ---- batched read path at scale -------------------------------------------------

def bench_read(args, eng, dev, dist, rank, world):
    """PNCOUNT GET over every key of a 16M-key x 64-replica shard in one call
    (jy_pncount_get, device slots -> device i64: the reference's
    repo_pncount.pony:55-57 value() per key), plus the RESP-sized host
    readback of the same answers."""
    import torch
    from jylis_amd import synth as S
    K, R = args.keys or (1 << 24), 64
    seed = S.BASE_SEED + 12
    kb, ko = S.counter_keys(K, prefix=f"s{rank}:r".encode(), width=8)
    eng.reserve(1, K)
    eng.intern(1, (kb, ko))
    cols = eng.replica_cols(S.replica_ids(R, seed).tolist())
    st = torch.empty((2, R, K), dtype=torch.int64, device=dev)
    S.counter_rows_torch(st, seed, wrap_frac=False)
    eng.pncount_converge_block(cols, 0, st[0], st[1])
    del st
    slots = torch.arange(K, dtype=torch.int32, device=dev)
    out = {}

    def step(i):
        out["v"] = eng.pncount_get(slots)

    elapsed, kt = _timed(args.steps, args.warmup, step, dist, dev)
    t = _max_over_ranks(elapsed, dist, dev)
    k = float(np.mean(kt))
    bytes_per_key = 2 * R * 8 + 4 + 8  # both slabs' columns + slot + answer
    # verification: a sampled key's sum recomputed from an export of its columns
    v = out["v"].cpu().numpy()
    sample = np.random.default_rng(1).integers(0, K, 64)
    ok = True
    for s in sample.tolist():
        ex = eng.counter_export(1, R, int(s), 1).reshape(2, R)
        d = (sum(int(x) for x in ex[0]) - sum(int(x) for x in ex[1])) % (1 << 64)  # wrapping, as GCounter
        ok = ok and int(v[s]) == (d - (1 << 64) if d >= 1 << 63 else d)
    t1 = time.perf_counter()
    host = out["v"].cpu().numpy()
    d2h_s = time.perf_counter() - t1
    return {"metric": "PNCOUNT GET throughput (batched read path, SURVEY 8f rank 4)",
            "workload": f"PNCOUNT GET of every key: {K} keys x {R} replicas x {{P,N}} per GPU in one "
                        f"jy_pncount_get (device slots -> device answers)",
            "unit_of_work": "key read", "value": world * K * args.steps / t, "ms_per_step": t / args.steps * 1e3,
            "verified_sampled_keys": bool(ok), "d2h_all_answers_ms": d2h_s * 1e3, "answers": int(len(host)),
            "roofline": {"bound": "hbm", "achieved": bytes_per_key * K / k / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": bytes_per_key * K / k / 1e9 / HBM_PEAK_GBS,
                         "kernel": "k_sum (pncount)", "kernel_ms_avg": k * 1e3, "bytes_per_unit": bytes_per_key}}


def _uj_doc(t, i):
    """row i of a UJSON table -> ({(id, seq): elem}, {id: n}, {(id, seq)})"""
    eo, vo, co = (np.asarray(t[k], np.int64) for k in ("el_offs", "vv_offs", "cloud_offs"))
    m = {(int(t["dot_ids"][j]), int(t["dot_seqs"][j])): int(t["elems"][j]) for j in range(eo[i], eo[i + 1])}
    vv = {int(t["vv_ids"][j]): int(t["vv_seqs"][j]) for j in range(vo[i], vo[i + 1])}
    cl = {(int(t["cloud_ids"][j]), int(t["cloud_seqs"][j])) for j in range(co[i], co[i + 1])}
    return m, vv, cl


def _uj_join(a, b):
    """the dot-kernel join restated independently (ujson.md:176-182): keep a's
    dots b's context has not seen or b also holds; add b's dots a has not
    seen; contexts united and compacted"""
    (am, avv, acl), (bm, bvv, bcl) = a, b

    def seen(vv, cl, d):
        return d[1] <= vv.get(d[0], 0) or d in cl
    m = {d: e for d, e in am.items() if d in bm or not seen(bvv, bcl, d)}
    for d, e in bm.items():
        if not seen(avv, acl, d):
            m[d] = e
    vv = dict(avv)
    for r, n in bvv.items():
        vv[r] = max(vv.get(r, 0), n)
    cl = acl | bcl
    for r in {d[0] for d in cl}:
        while (r, vv.get(r, 0) + 1) in cl:
            vv[r] = vv.get(r, 0) + 1
    cl = {d for d in cl if d[1] > vv.get(d[0], 0)}
    return m, vv, cl


def _verify_ujson(eng, repo, st, applied, D, nsample=96, locate=None, ask=None):
    """sampled docs (the hottest delta docs and random ones) recomputed from
    the tables with _uj_join and compared with the owner's documents
    (locate / ask as in _verify_tlog; by default a lookup on this engine)"""
    width = len(st["key_offs"]) and int(st["key_offs"][1] - st["key_offs"][0])

    def docs_of(t):
        kb, ko = np.asarray(t["key_bytes"], np.uint8), np.asarray(t["key_offs"], np.int64)
        return [int(bytes(kb[ko[i]:ko[i + 1]])[width - 8:]) for i in range(len(ko) - 1)]
    rows = [dict((d, i) for i, d in enumerate(docs_of(t))) for t in applied]
    hot = {}
    for t, r in zip(applied, rows):
        eo = np.diff(np.asarray(t["el_offs"], np.int64))
        for d, i in r.items():
            hot[d] = hot.get(d, 0) + int(eo[i])
    pick = sorted(hot, key=hot.get, reverse=True)[:nsample // 2]
    pick += np.random.default_rng(9).integers(0, D, nsample - len(pick)).tolist()
    from jylis_amd import engine as E

    def answer(slots):
        eo, dots, elems, vv, co, cloud = eng.ujson_read(np.asarray(slots, np.uint32))
        ids = [eng.replica_id(c) for c in range(eng.replica_count())]
        out = []
        for i in range(len(slots)):
            c, q = E.unpack_dot(dots[eo[i]:eo[i + 1]])
            gm = {(ids[int(x)], int(y)): int(e) for x, y, e in zip(c, q, elems[eo[i]:eo[i + 1]])}
            gvv = {ids[j]: int(n) for j, n in enumerate(vv[i]) if n}
            c, q = E.unpack_dot(cloud[co[i]:co[i + 1]])
            out.append((gm, gvv, {(ids[int(x)], int(y)) for x, y in zip(c, q)}))
        return out
    if locate is None:
        slots = eng.lookup(4, [bytes(np.asarray(st["key_bytes"], np.uint8)[
            int(st["key_offs"][d]):int(st["key_offs"][d + 1])]) for d in pick])
        got = answer(slots)
    else:
        got = ask([locate(d) for d in pick], answer)
    for d, g in zip(pick, got):
        want = _uj_doc(st, d)
        for t, r in zip(applied, rows):
            if d in r:
                want = _uj_join(want, _uj_doc(t, r[d]))
        if g != want:
            return False
    return True


MODES = {"gcount": bench_gcount, "treg": bench_treg, "tlog": bench_tlog, "ujson": bench_ujson, "e2e": bench_e2e,
         "read": bench_read}
