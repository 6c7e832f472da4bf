#!/usr/bin/env python3
"""bench.py -- CRDT delta merges/s and HBM roofline (BASELINE.json metric).

Workload (BASELINE.json configs[1]): PNCOUNT,
16M keys x 64 replicas x {P, N} per GPU shard.  One step = converge one full
delta batch: 64 flushed peer batches (one per replica column, each covering
every key, both signs) = 2^31 cell merges per shard, HBM-resident input.

Keys are hash-sharded over the N GPUs (weak scaling: 16M keys per GPU).  A
step is ONE engine call per shard (jy_pncount_converge_block) over the 64
peer columns of that shard's keys: peers that run the same key sharding
flush shard by shard, so each shard's part of a peer batch arrives at its
owner and no collective sits on the data path (`value`, `roofline`).

At N > 1 the line also carries `routed`: the same converge with the peer
batches arriving MIXED (north_star) -- rank r ingests the 64/N
peer columns c with c % N == r for the keys of every owner and
route.CounterRouter moves each owner's part to it with equal-split RCCL
all-to-alls over xGMI, double-buffered so chunk c+1 is in flight while the
owners merge chunk c.  (N - 1)/N of every batch then crosses xGMI, as many
bytes as the merge reads from HBM, so that step is bound by the links; it
reports its exchange GB/s against the links it uses.

Inputs: seeded splitmix64 streams generated in HBM (jylis_amd/synth.py); the
state starts from a synthetic full state and `--batches` distinct delta
batches (a monotone chain, 75% of cells advanced / 25% stale) are cycled.
After the first cycle the state already dominates every batch, so later
steps change no cell -- the kernel's traffic is the same (it reads both
operands and stores the max unconditionally), and `first_cycle_changes`
reports how many cells the first application changed.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import time

import numpy as np

METRIC = "CRDT delta merges/sec (keys×replicas) + achieved HBM GB/s vs peak, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_CELL = 24    # 8 delta read + 8 state read + 8 state write


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--keys", type=int, default=16 * 1024 * 1024, help="keys per GPU shard")
    ap.add_argument("--replicas", type=int, default=64)
    ap.add_argument("--batches", type=int, default=4, help="distinct delta batches held in HBM")
    ap.add_argument("--cpu-keys", type=int, default=65536, help="cpu_baseline sample: keys (x replicas x 2)")
    ap.add_argument("--cpu-rounds", type=int, default=6, help="cpu_baseline sample: peer-batch rounds")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="key-partitioned CPU baseline threads; 0 = every CPU this process may run on "
                         "(cpu_share()); 1 = off")
    ap.add_argument("--cpu-keys-per-thread", type=int, default=8192)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-file", default=None, help="per-launch HBM bytes from a PMC run (json)")
    ap.add_argument("--type", default="pncount", choices=["pncount", "gcount", "treg", "tlog", "ujson", "e2e", "read"],
                    help="pncount = the BASELINE metric line; the others measure SURVEY 8d configs 1,3,4,5")
    ap.add_argument("--route", action="store_true", help="treg / tlog / ujson: run the routing path even on 1 GPU")
    ap.add_argument("--overlap", type=float, default=None,
                    help="treg --route: S local shards on one GPU whose sources share this fraction of their keys "
                         "in every step (timed beside the same run with no overlap)")
    ap.add_argument("--shards", type=int, default=2, help="--overlap: local shards (engines) on the GPU")
    ap.add_argument("--resolve", action="store_true",
                    help="treg --route: every timed step first resolves its batch's key strings on the GPU "
                         "(route.KeyResolver), 1/16 of them new to the node")
    ap.add_argument("--node", action="store_true",
                    help="treg: every step is one jy_node_treg_converge of key strings (the node C-ABI)")
    ap.add_argument("--node-shards", type=int, default=1,
                    help="--node at N = 1: shards on this GPU (1: RCCL; more: the copy fabric)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1 collectives: nccl (RCCL over xGMI); gloo only rehearses the routed path "
                         "with several ranks on one GPU")
    return ap.parse_args()


def other_mode(args, rank, world, local, dist):
    """bench_modes.py: one JSON line for a non-default CRDT type"""
    import torch

    import bench_modes
    from jylis_amd.engine import Engine
    dev = torch.device("cuda", local)
    eng = Engine(device=local, counter_columns=16)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    if args.keys == 16 * 1024 * 1024:
        args.keys = 0  # per-mode default size
    res = bench_modes.MODES[args.type](args, eng, dev, dist, rank, world)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = bench_modes.cpu_baseline(args.type)
        if cb is not None:
            res["cpu_baseline"] = cb
    if rank == 0:
        line = {"metric": res.pop("metric", f"{args.type.upper()} delta converge throughput (SURVEY 8d)"),
                "value": res.pop("value"),
                "unit": res.pop("unit_of_work") + "s/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": res.pop("ms_per_step"), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic (jylis_amd/synth.py)",
                "config": {"workload": res.pop("workload")}, **res}
        print(json.dumps(line), flush=True)
    eng.close()


def cpu_baseline(args, seed):
    """The oracle (a C++ restatement of the reference's per-key converge loop,
    repo_manager.pony:92-93 over Map[String, PNCounter]) timed single-threaded
    on a bounded sample of the same stream: cpu_keys keys x R replicas x 2
    signs, `cpu_rounds` rounds of R peer batches."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle"))
    import oracle as O
    from jylis_amd import synth as S
    K, R = args.cpu_keys, args.replicas
    kb, ko = S.counter_keys(K, prefix=b"c")
    rids = S.replica_ids(R, seed)
    st = S.counter_state_np(K, R, 2, seed)
    repo = O.Repo(O.PNCOUNT, 1)
    for t in S.counter_batch_tables(st, rids, (kb, ko)):
        repo.converge(t)
    dt = 0.0
    cur = st
    for r in range(args.cpu_rounds):
        # decode (untimed) one round of R peer batches, then time the converge loop
        cur = S.counter_delta_np(cur, r, seed)
        batches = [O.Batch(O.PNCOUNT, t) for t in S.counter_batch_tables(cur, rids, (kb, ko))]
        t0 = time.perf_counter()
        for b in batches:
            repo.converge(b)
        dt += time.perf_counter() - t0
        del batches
    cells = K * R * 2 * args.cpu_rounds
    return {"value": cells / dt, "unit": "merges/s", "cores": 1, "kind": "port",
            "sample": f"PNCOUNT {K} keys x {R} replicas x 2 signs x {args.cpu_rounds} rounds of {R} peer batches "
                      f"({cells} cell merges, {dt:.2f} s, oracle/jy_oracle.cpp unordered_map path, 1 thread)",
            "host_cpus": os.cpu_count()}


def cpu_share():
    """CPUs this process may really use: its affinity set, capped by a cgroup
    CPU quota if one is set (a GPU box shares its host: os.cpu_count() there
    reports the whole machine) -> (threads, how it was found)"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    how = f"sched_getaffinity {n} of os.cpu_count() {os.cpu_count()}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) / int(period)))
            if q < n:
                n, how = q, how + f", cgroup cpu.max quota {quota}/{period}"
    except (OSError, ValueError):
        pass
    return n, how


def cpu_baseline_parallel(args, seed):
    """The stronger CPU baseline of SURVEY 8d: the oracle key-partitioned over
    `cpu_threads` threads, each converging its own partition's peer batches
    into its own Repo (one unordered_map per thread, no sharing; the ctypes
    calls release the GIL).  Same stream shape as cpu_baseline."""
    import sys
    import threading
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle"))
    import oracle as O
    from jylis_amd import synth as S
    T, kt, R, rounds = args.cpu_threads, args.cpu_keys_per_thread, args.replicas, 2
    how = "--cpu-threads"
    if T <= 0:
        T, how = cpu_share()
    rids = S.replica_ids(R, seed)
    repos, batches = [], []
    for t in range(T):
        keys = S.counter_keys(kt, prefix=b"c", start=t * kt)
        st = S.counter_state_np(kt, R, 2, seed + t)
        repo = O.Repo(O.PNCOUNT, 1)
        for tab in S.counter_batch_tables(st, rids, keys):
            repo.converge(tab)
        mine = []
        cur = st
        for r in range(rounds):
            cur = S.counter_delta_np(cur, r, seed + t)
            mine += [O.Batch(O.PNCOUNT, tab) for tab in S.counter_batch_tables(cur, rids, keys)]
        repos.append(repo)
        batches.append(mine)

    def work(t):
        for b in batches[t]:
            repos[t].converge(b)

    threads = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    t0 = time.perf_counter()
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    dt = time.perf_counter() - t0
    cells = T * kt * R * 2 * rounds
    return {"value": cells / dt, "unit": "merges/s", "cores": T, "kind": "port",
            "sample": f"PNCOUNT {T} key partitions x {kt} keys x {R} replicas x 2 signs x {rounds} rounds of {R} "
                      f"peer batches ({cells} cell merges, {dt:.2f} s, oracle/jy_oracle.cpp, {T} threads)",
            "threads_from": how, "host_cpus": os.cpu_count()}


def _owner_seed(seed, owner):
    return seed + owner * 7919  # owner 0 keeps the single-GPU stream


LAUNCH_FAIL_EXIT = 2


def visible_devices():
    """GPUs this process would see, counted in a CHILD process: the launching
    parent never touches the GPU (it starts torch.distributed.run as a child,
    and a process that initialised HIP must not fork-exec GPU programs)"""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def launch_cmd(argv, n, port):
    """the torch.distributed.run command of an N-rank run (one process per GPU,
    rendezvous on 127.0.0.1), re-running this file with the same arguments"""
    import sys
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args, argv):
    """`--gpus N > 1` without a torch.distributed environment: start N ranks as
    a child torch.distributed.run and exit with its code (rank 0 prints the
    line).  Refuses (exit LAUNCH_FAIL_EXIT) when fewer than N GPUs are
    visible: an N-GPU line must never come from fewer GPUs."""
    import subprocess
    import sys
    if args.backend == "nccl":
        have = visible_devices()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but {have} GPU(s) visible", file=sys.stderr, flush=True)
            return LAUNCH_FAIL_EXIT
    return subprocess.run(launch_cmd(argv, args.gpus, free_port())).returncode


def world_check(args, world, ndev):
    """None if this rank's environment fits --gpus, else the reason"""
    if world != args.gpus:
        return f"WORLD_SIZE {world} but --gpus {args.gpus}"
    if args.backend == "nccl" and ndev < world:
        return f"{world} ranks over RCCL but {ndev} GPU(s) visible"
    return None


def main():
    import sys
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args, sys.argv[1:]))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:  # before torch: a mismatched launch fails at once
        print(f"bench.py: {world_check(args, world, world)}", file=sys.stderr, flush=True)
        sys.exit(LAUNCH_FAIL_EXIT)
    import torch
    why = world_check(args, world, torch.cuda.device_count())
    if why:
        print(f"bench.py: {why}", file=sys.stderr, flush=True)
        sys.exit(LAUNCH_FAIL_EXIT)
    if args.backend == "gloo":  # rehearsal: several ranks may share one GPU
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dist = cpu_group = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        cpu_group = dist.new_group(backend="gloo")
    if args.type != "pncount":
        other_mode(args, rank, world, local, dist)
        if dist:
            dist.destroy_process_group()
        return

    from jylis_amd import synth as S
    from jylis_amd._lib import PNCOUNT
    from jylis_amd.engine import Engine
    K, R = args.keys, args.replicas
    assert R % world == 0, "the replica columns are split evenly over the ranks"
    Cn = R // world  # peer columns ingested per rank
    seed = S.BASE_SEED + 2  # config 2
    seed_me = _owner_seed(seed, rank)
    dev = torch.device("cuda", local)
    routed_on = world > 1 or args.route
    # the headline runs on a plain engine; the routed phase (N > 1, --route)
    # makes its node -- an RCCL communicator over every rank -- only after the
    # headline is measured, under its watchdog, with a shard of its own
    eng = Engine(device=local, counter_columns=R, key_capacity=[1024, K, 1024, 1024, 1024])
    # one non-default stream shared by torch (generation, collectives, timing
    # events) and the engine, so the HIP events bracket the engine's launches
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)

    def load_shard(e):
        """this rank's key shard interned on the host like any key
        (s<rank>:p########) and its initial state generated in HBM and loaded
        (max(0, s) = s)"""
        kb, ko = S.counter_keys(K, prefix=f"s{rank}:p".encode())
        slots = e.intern(PNCOUNT, (kb, ko))
        assert slots[0] == 0 and slots[-1] == K - 1
        del kb, ko, slots
        cols = e.replica_cols(S.replica_ids(R, seed).tolist())
        assert (cols == np.arange(R)).all()
        tmp = torch.empty((2, R, K), dtype=torch.int64, device=dev)
        S.counter_rows_torch(tmp, seed_me)
        e.pncount_converge_block(cols, 0, tmp[0], tmp[1])
        del tmp
        return cols

    cols = load_shard(eng)
    peer = [[r + c * world for c in range(Cn)] for r in range(world)]  # global column of rank r's c-th peer
    nb = max(1, args.batches)

    def chain_into(seed_d, g, outs):
        """column g of owner d's delta chain: outs[j][sign][K] <- round j"""
        prev = torch.empty((2, 1, K), dtype=torch.int64, device=dev)
        S.counter_rows_torch(prev, seed_d, col_offset=g, col_total=R)
        for j, o in enumerate(outs):
            cur = torch.empty_like(prev)
            S.counter_rows_torch(cur, seed_d, rnd=j, prev=prev, col_offset=g, col_total=R)
            o.copy_(cur[:, 0])
            prev = cur

    # sharded ingest: every peer batch of this rank's keys, [sign][R][K] per
    # round -- peers that run the same key sharding flush shard by shard, so
    # each shard's part of a peer batch arrives at its owner
    shard = [torch.empty((2, R, K), dtype=torch.int64, device=dev) for _ in range(nb)]
    for g in range(R):
        chain_into(seed_me, g, [shard[j][:, g] for j in range(nb)])
    all_cols = np.arange(R, dtype=np.uint16)
    # routed ingest (N > 1): rank r holds the Cn peer columns c % N == r for
    # the keys of EVERY owner, [sign][c][owner][K] per round, and routes them
    nbr = min(nb, 2)
    routed = []
    if routed_on:
        routed = [torch.empty((2, Cn, world, K), dtype=torch.int64, device=dev) for _ in range(nbr)]
        for d in range(world):
            for c in range(Cn):
                chain_into(_owner_seed(seed, d), peer[rank][c], [routed[j][:, c, d] for j in range(nbr)])
    torch.cuda.synchronize(dev)

    def step(i):
        eng.pncount_converge_block(all_cols, 0, shard[i % nb][0], shard[i % nb][1])

    changed = None
    for i in range(args.warmup):
        if i == 0:
            before = eng.counter_export(PNCOUNT, R, 0, min(K, 1 << 16))
        step(i)
        if i == 0:
            changed = int((eng.counter_export(PNCOUNT, R, 0, min(K, 1 << 16)) != before).sum())
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    eng.timing(True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    calls = eng.timing_read(cap=1 << 16)
    eng.timing(False)
    merge_ms_per_step = float(np.sum(calls)) / args.steps

    # correctness spot-check on sampled cells of this shard: state == max(initial, applied rounds)
    rng = np.random.default_rng(rank)
    s0 = int(rng.integers(0, K - 64))
    cells = (np.arange(2)[:, None, None] * R * K + np.arange(R)[None, :, None] * K
             + (s0 + np.arange(64))[None, None, :]).astype(np.uint64)

    def verify(applied, e=None):
        e = e or eng
        exp = S.counter_state_np(K, R, 2, seed_me, cells=cells)
        chain, best = exp.copy(), exp.copy()
        for j in range(max(applied) + 1):
            chain = S.counter_delta_np(chain, j, seed_me, cells=cells)
            if j in applied:
                best = np.maximum(best, chain)
        ok = bool((e.counter_export(PNCOUNT, R, s0, 64) == best).all())
        sums = e.pncount_get(np.arange(s0, s0 + 64, dtype=np.uint32))
        exp_sum = (best[0].sum(axis=0, dtype=np.uint64) - best[1].sum(axis=0, dtype=np.uint64)).view(np.int64)
        ok = ok and bool((sums == exp_sum).all())
        if dist:
            t = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ok = float(t[0]) == 0.0
        return ok

    applied = {i % nb for i in range(args.warmup + args.steps)}
    ok = verify(applied)

    t_max = elapsed
    if dist:
        tt = torch.tensor([elapsed, merge_ms_per_step], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max, merge_ms_per_step = float(tt[0]), float(tt[1])
    cells_per_step = 2 * R * K
    value = world * cells_per_step * args.steps / t_max
    avg_kern_s = merge_ms_per_step / 1e3
    achieved = BYTES_PER_CELL * cells_per_step / avg_kern_s / 1e9

    traffic = None
    tf = args.traffic_file or os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            with open(tf) as f:
                tj = json.load(f)
            if tj.get("workload_cells_per_launch") == cells_per_step:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = cpu_par = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, seed)
        cpu_par = cpu_baseline_parallel(args, seed) if args.cpu_threads != 1 else None

    line = {
        "metric": METRIC,
        "value": value,
        "unit": "merges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded splitmix64 in HBM; SURVEY.md 8d config 2)",
        "config": {"workload": f"PNCOUNT converge: {K // (1 << 20)}M keys x {R} replicas x {{P,N}} per GPU shard, "
                               f"one full delta batch ({R} peer batches) per step, each shard's part of every peer "
                               f"batch converged on its owner",
                   "keys_per_gpu": K, "replicas": R, "signs": 2, "cells_per_step_per_gpu": cells_per_step,
                   "parallelism": f"key-sharded x{world}", "distinct_batches": nb},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "k_block_max<true>", "kernel_ms_avg": avg_kern_s * 1e3,
                     "merge_launches_per_step": len(calls) // max(args.steps, 1),
                     "bytes_per_cell": BYTES_PER_CELL},
        "cpu_baseline": cpu,
        "cpu_baseline_parallel": cpu_par,
        "first_cycle_changes": {"cells_changed": changed, "cells_sampled": 2 * R * min(K, 1 << 16)},
        "verified": ok,
    }
    eng.close()
    del shard
    if routed_on:
        try:
            routed_phase(args, load_shard, dev, dist, rank, world, routed, peer, fabric_of(dist, cpu_group, world),
                         cells_per_step, line, verify)
        except Exception as e:  # the headline stands; the routed phase's failure is reported in the line
            line["routed_error"] = f"{type(e).__name__}: {e}"
        r = line.get("routed")
        if isinstance(r, dict) and "value" in r:
            # the end-to-end figure beside the key-sharded `value`: peer batches
            # arriving mixed, each owner's part moved by the node's native RCCL
            line["value_routed"] = r["value"]
            line["value_routed_note"] = ("end-to-end merges/s with peer batches arriving mixed and routed to "
                                         "their owners over RCCL (jy_node_counter_converge_block); `value` is "
                                         "the key-sharded converge")
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


WATCHDOG_EXIT = 3


def watchdog(limit, line, rank, key="routed"):
    """A phase that may hang in a collective: after `limit` seconds rank 0
    prints the line with an error under `key`, and every rank exits with
    WATCHDOG_EXIT -- a hang is a failure, never a clean exit.  Cancel the
    returned timer when the phase finished."""
    import threading

    def fire():
        if rank == 0:
            line[key] = {"error": f"{key} phase did not finish within {limit:.0f} s"}
            print(json.dumps(line), flush=True)
        os._exit(WATCHDOG_EXIT)

    dog = threading.Timer(limit, fire)
    dog.daemon = True
    dog.start()
    return dog


XGMI_LINK_GBPS = 153.0  # per xGMI link and direction, nominal (MI355X: 7 links per GPU)


def fabric_of(dist, cpu_group, world):
    from jylis_amd.route import DistFabric, LocalFabric
    return DistFabric(dist, cpu_group=cpu_group) if world > 1 else LocalFabric(1)


def routed_phase(args, load_shard, dev, dist, rank, world, routed, peer, fabric, cells_per_step, line, verify):
    """The same converge with the peer batches arriving MIXED: rank r holds
    whole peer columns (the keys of every owner) and each owner's part moves
    to it over xGMI, double-buffered against the owner's merge.
    Every cell a shard merges then crosses xGMI once unless the ingesting rank
    owns it: (N - 1) / N of the batch, as many bytes as the merge reads, so the
    step is bound by the links, not by HBM.  Timed twice, apart from `value`,
    with a few steps each:
      routed        the node C-ABI (jy_node_counter_converge_block): native
                    RCCL ncclSend / ncclRecv per column on a second stream,
                    the engine's block merge of column c while c + 1 moves
      routed_torch  route.CounterRouter: the same exchange as torch
                    all_to_all_single calls (DistFabric) from Python
    The node is made here, after the headline (its communicator's setup is
    inside the watchdog too), with this rank's shard loaded into its engine.
    A watchdog exits non-zero (printing the line with an error) if a
    collective hangs; an exception is reported in the line (`routed_error`),
    the headline standing.  At N = 1 (--route) both run against one shard."""
    limit = float(os.environ.get("JY_ROUTED_LIMIT_S", "240"))
    dog = watchdog(limit, line, rank)
    try:
        _routed_phase(args, load_shard, dev, dist, rank, world, routed, peer, fabric, cells_per_step, line, verify)
    finally:
        dog.cancel()


def _routed_phase(args, load_shard, dev, dist, rank, world, routed, peer, fabric, cells_per_step, line, verify):
    import torch
    from bench_modes import node_for
    from jylis_amd._lib import PNCOUNT
    from jylis_amd.route import CounterRouter
    R = routed[0].shape[1] * world
    K = routed[0].shape[3]
    # a gloo rehearsal may put several ranks on one GPU: RCCL takes one rank
    # per device, so the native node is left out there
    shared = world > 1 and args.backend == "gloo" and world > torch.cuda.device_count()
    node = None
    if shared:
        from jylis_amd.engine import Engine
        eng = Engine(device=dev.index, counter_columns=R, key_capacity=[1024, K, 1024, 1024, 1024])
    else:
        node, _ = node_for(args, dev, dist, rank, world, counter_columns=R, key_capacity=[1024, K, 1024, 1024, 1024])
        eng = node.engines[0]
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    load_shard(eng)
    applied = set()
    nbr = len(routed)
    warm, steps = 1, max(1, min(args.steps, 4))
    _, Cn, _, K = routed[0].shape
    xbytes = 2 * Cn * (world - 1) * K * 8  # sent (= received) per rank per step

    def run(step_fn, k0):
        for i in range(warm):
            step_fn(routed[(k0 + i) % nbr])
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(steps):
            step_fn(routed[(k0 + warm + i) % nbr])
        if node is not None:
            node.sync()
        eng.sync()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if dist:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt[0])
        ms = el / steps * 1e3
        res = {"value": world * cells_per_step * steps / el, "unit": "merges/s", "steps": steps, "warmup": warm,
               "ms_per_step": ms, "exchange_bytes_per_gpu_per_step": xbytes,
               "exchange_GBps_per_gpu": xbytes / (ms / 1e3) / 1e9, "xgmi_links_used": world - 1,
               "xgmi_link_GBps_nominal": XGMI_LINK_GBPS}
        if world > 1:
            res["exchange_frac_of_links"] = xbytes / (ms / 1e3) / 1e9 / ((world - 1) * XGMI_LINK_GBPS)
        return res

    cols_all = np.array(peer, np.uint16)  # [rank][c]: the column of rank r's c-th peer
    if node is not None:
        native = run(lambda b: node.counter_converge_block(PNCOUNT, cols_all, 0, K, b[0], b[1]), 0)
        native["verified"] = verify(applied | {i % nbr for i in range(warm + steps)}, eng)
        native["note"] = ("peer batches ingested mixed: rank r holds peer columns c % N == r for every owner; "
                          "jy_node_counter_converge_block moves each column to its owners with native RCCL "
                          "send/recv and block-merges it, column c + 1 in flight on a second stream")
        line["routed"] = native
    else:
        line["routed"] = {"skipped": "gloo rehearsal with ranks sharing one GPU: RCCL takes one rank per device"}
    router = CounterRouter([eng], fabric, PNCOUNT)
    tor = run(lambda b: router.step([b], peer), 1)
    tor["verified"] = verify(applied | {i % nbr for i in range(2 * (warm + steps) + 1)}, eng)
    tor["note"] = "the same exchange through route.CounterRouter (torch all_to_all_single, RCCL, from Python)"
    line["routed_torch"] = tor
    eng.close()
    if node is not None:
        node.close()


if __name__ == "__main__":
    main()
