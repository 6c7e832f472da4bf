"""Key-hash sharding of one node's GPUs and the delta-routing exchange step.

SURVEY.md section 8e: every merge is per key, so a shard converges without any
collective; the one real exchange is routing an ingested peer batch to the
shards that own its keys.  The reference has no counterpart (every Jylis node
holds every key); this is the intra-node analogue of Cluster.broadcast_deltas
(jylis/cluster.pony:209-213).

Control plane (host): a key's slot lives on its owner.  The first time a rank
ingests a key owned elsewhere, it sends the key bytes to the owner, which
interns it and answers with the slot (`ShardRouter.resolve`); the answer is
cached.

Data plane (device): runs of a FIXED capacity per destination, so every
all-to-all is an equal-split collective (RCCL over xGMI) and the per-run
counts travel as a small device header beside the data -- the host never
reads a count back per batch.  What does not fit a run (a skewed batch) is
listed on the device and sent in a drain round, decided one step later from
an asynchronously read global maximum, so no step waits for the GPU.

`Fabric` is the medium: `DistFabric` (one rank per process: RCCL for CUDA
tensors, or gloo through host memory) or `LocalFabric` (S engines in one
process, for single-GPU tests).  Routers take lists of per-rank engines and
batches: one per process with a DistFabric, S with a LocalFabric.
"""
import ctypes as C

import numpy as np

from . import _lib

# run capacity: the expected share of a balanced hash partition plus slack
CAP_SLACK = 1.125
CAP_MARGIN = 256
BYTE_SLACK = 1.25
BYTE_MARGIN = 4096


def owners(kb, ko, nshards):
    """owner shard of every key (jy_keys_owner: FNV-1a-64 + splitmix finaliser mod S)"""
    kb = np.ascontiguousarray(kb, np.uint8)
    ko = np.ascontiguousarray(ko, np.uint64)
    n = len(ko) - 1
    out = np.empty(n, np.uint32)
    _lib.load().jy_keys_owner(n, kb.ctypes.data, ko.ctypes.data, nshards, out.ctypes.data)
    return out


def run_caps(n_max, bytes_max, world):
    """(records, value bytes) per destination run for batches of at most
    n_max entries / bytes_max long-value bytes per rank"""
    if world == 1:
        return max(n_max, 1), round8(max(bytes_max, 1))
    cap = min(max(n_max, 1), int(np.ceil(n_max / world * CAP_SLACK)) + CAP_MARGIN)
    capb = min(max(bytes_max, 1), int(np.ceil(bytes_max / world * BYTE_SLACK)) + BYTE_MARGIN)
    return cap, round8(capb)


# ---- fabrics ------------------------------------------------------------------

class _Done:
    def wait(self):
        pass


class _Pending:
    """an in-flight transfer: wait() orders the current stream after it
    (what RCCL's Work.wait() does for an async collective)"""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        import torch
        torch.cuda.current_stream().wait_event(self.ev)


class LocalFabric:
    """S shards hosted by one process (tests on one GPU): the all-to-all is a
    set of device copies.  With `async_copies`, an async all-to-all runs its
    copies on a side stream (after the current stream's work, optionally
    behind a spin delay) and returns pending work whose wait() orders the
    current stream after them -- the ordering contract of an async RCCL
    collective, so the routers' works / wait() / chunk pipelining is exercised
    with transfers genuinely in flight."""

    def __init__(self, world, async_copies=False, delay_cycles=0):
        self.world = world
        self.ranks = list(range(world))
        self.async_copies = async_copies
        self.delay_cycles = delay_cycles
        self._side = None

    def _copies(self, outs, ins):
        S = self.world
        for r in range(S):
            cr = outs[r].numel() // S
            for s in range(S):
                cs = ins[s].numel() // S
                assert cs == cr, "equal-split all-to-all: every rank sends the same chunk size"
                outs[r].view(-1)[s * cr:(s + 1) * cr].copy_(ins[s].view(-1)[r * cs:(r + 1) * cs])

    def a2a(self, outs, ins, async_op=False):
        if not (async_op and self.async_copies):
            self._copies(outs, ins)
            return _Done()
        import torch
        cur = torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream(cur.device)
        self._side.wait_stream(cur)
        with torch.cuda.stream(self._side):
            if self.delay_cycles:
                torch.cuda._sleep(self.delay_cycles)  # a slow link: a missing wait() reads stale runs
            self._copies(outs, ins)
            for t in list(outs) + list(ins):
                t.record_stream(self._side)
            ev = torch.cuda.Event()
            ev.record(self._side)
        return _Pending(ev)

    def max_all(self, ts):
        """in place: every tensor becomes the max over ranks"""
        import torch
        if len(ts) == 1:
            return _Done()  # the max over one rank is its own value
        m = torch.stack([t.view(-1) for t in ts]).max(0).values
        for t in ts:
            t.view(-1).copy_(m)
        return _Done()

    def host_max(self, vals):
        m = np.max(np.asarray(vals, np.int64), axis=0)
        return [m.copy() for _ in vals]

    def host_a2a(self, vals):
        """vals[s][r]: what rank s sends rank r (host ints) -> out[r][s]"""
        v = np.asarray(vals, np.int64)
        return [v[:, r].copy() for r in range(self.world)]

    def a2a_v(self, outs, ins, out_splits, in_splits):
        """variable all-to-all: rank s's segment r (in_splits[s][r] items) lands
        as rank r's segment s (out_splits[r][s])"""
        S = self.world
        ioff = [np.concatenate([[0], np.cumsum(np.asarray(x, np.int64))]) for x in in_splits]
        ooff = [np.concatenate([[0], np.cumsum(np.asarray(x, np.int64))]) for x in out_splits]
        for r in range(S):
            for s_ in range(S):
                k = int(in_splits[s_][r])
                assert k == int(out_splits[r][s_])
                if k:
                    outs[r].view(-1)[int(ooff[r][s_]):int(ooff[r][s_]) + k].copy_(
                        ins[s_].view(-1)[int(ioff[s_][r]):int(ioff[s_][r]) + k])


class DistFabric:
    """One rank per process over torch.distributed.  With the nccl backend
    (RCCL on ROCm) CUDA tensors move GPU to GPU over xGMI; with gloo they go
    through host memory (multi-process tests on one GPU).  `cpu_group` (gloo)
    carries the host-side control values."""

    def __init__(self, dist, group=None, cpu_group=None):
        self.dist = dist
        self.group = group
        self.cpu_group = cpu_group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.ranks = [self.rank]
        self.staged = dist.get_backend(group) == "gloo"

    def a2a(self, outs, ins, async_op=False):
        (out,), (inp,) = outs, ins
        if self.staged:
            o = out.view(-1).cpu()
            self.dist.all_to_all_single(o, inp.view(-1).cpu(), group=self.group)
            out.view(-1).copy_(o)
            return _Done()
        w = self.dist.all_to_all_single(out.view(-1), inp.view(-1), group=self.group, async_op=async_op)
        return w if async_op else _Done()

    def max_all(self, ts):
        (t,) = ts
        if self.staged:
            c = t.cpu()
            self.dist.all_reduce(c, op=self.dist.ReduceOp.MAX, group=self.group)
            t.copy_(c)
            return _Done()
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return _Done()

    def host_max(self, vals):
        import torch
        (v,) = vals
        t = torch.tensor(np.asarray(v, np.int64))
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.cpu_group)
        return [t.numpy()]

    def host_a2a(self, vals):
        """this rank's host ints per destination -> what every rank sends this one"""
        import torch
        (v,) = vals
        t = torch.tensor(np.asarray(v, np.int64))
        out = torch.empty_like(t)
        self.dist.all_to_all_single(out, t, group=self.cpu_group)
        return [out.numpy()]

    def a2a_v(self, outs, ins, out_splits, in_splits):
        """variable all-to-all (RCCL for CUDA tensors; gloo through host memory)"""
        (out,), (inp,), (osp,), (isp,) = outs, ins, out_splits, in_splits
        osp, isp = [int(x) for x in osp], [int(x) for x in isp]
        if self.staged:
            o = out.view(-1).cpu()
            self.dist.all_to_all_single(o, inp.view(-1).cpu(), osp, isp, group=self.group)
            out.view(-1).copy_(o)
            return
        self.dist.all_to_all_single(out.view(-1), inp.view(-1), osp, isp, group=self.group)


def _bind_streams(engines):
    """every engine enqueues on torch's current stream of its device, so the
    collectives (issued by torch against that stream) and the engine's
    launches are ordered, and tensors the caching allocator recycles are
    stream-ordered with the engine's reads of them.  The engine cannot name
    the legacy default stream (NULL selects its own stream), so a router
    bound while torch is on the default stream moves torch to a new stream."""
    import torch
    for e in engines:
        dev = torch.device("cuda", e.device)
        if torch.cuda.current_stream(dev).cuda_stream == 0:
            torch.cuda.synchronize(dev)
            torch.cuda.set_stream(torch.cuda.Stream(dev))
        cur = torch.cuda.current_stream(dev).cuda_stream
        if e.stream() != cur:
            e.set_stream(cur)


def _check_streams(engines):
    import torch
    for e in engines:
        if e.stream() != torch.cuda.current_stream(e.device).cuda_stream:
            raise RuntimeError("the engine stream is not torch's current stream: call router.bind() after "
                               "switching streams")


# ---- fixed-capacity runs (TREG records, TLOG logs, UJSON documents) ------------

def round8(x):
    return (int(x) + 7) // 8 * 8


class _CudaBytes:
    """__cuda_array_interface__ of `n` bytes of device memory the engine owns"""
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 2,
                                         "strides": None}


def _device_bytes(ptr, n, device):
    """a uint8 tensor over engine-owned device memory (no copy, not owned by torch)"""
    import torch
    if n == 0:
        return torch.empty(0, dtype=torch.uint8, device=torch.device("cuda", device))
    t = torch.as_tensor(_CudaBytes(ptr, n), device=torch.device("cuda", device))
    assert t.data_ptr() == ptr and t.dtype == torch.uint8
    return t


def long_bytes(lr):
    """padded bytes of the values longer than 8 bytes among value handles
    `lr` (numpy uint64 or CUDA int64 tensor): what their runs' byte sections take"""
    if isinstance(lr, np.ndarray):
        lens = (lr & np.uint64((1 << 24) - 1)).astype(np.int64)
        return int(((lens[lens > 8] + 7) // 8 * 8).sum())
    import torch
    lens = lr & ((1 << 24) - 1)
    pad = (lens + 7) // 8 * 8
    return int(torch.where(lens > 8, pad, torch.zeros_like(pad)).sum())


def _csr_pick(offs, idx, cols):
    """sub-batch of the keys `idx` of a CSR on the device: (offsets, columns)"""
    import torch
    lo, hi = offs[idx], offs[idx + 1]
    cnt = hi - lo
    noffs = torch.zeros(len(idx) + 1, dtype=torch.int64, device=offs.device)
    noffs[1:] = torch.cumsum(cnt, 0)
    total = int(noffs[-1])
    ent = (torch.repeat_interleave(lo - noffs[:-1], cnt, output_size=total)
           + torch.arange(total, dtype=torch.int64, device=offs.device))
    return noffs, [c.index_select(0, ent) for c in cols]


class _RunRouter:
    """Common driver of the routers: partition into fixed-capacity runs,
    exchange (one equal-split all-to-all per buffer), merge every received
    run; overflow goes out in a drain round decided one step later from an
    asynchronously read global maximum.  Subclasses give the batch sizes,
    capacities, partition, merge and the overflow sub-batch."""

    # rounds in flight before the host reads the oldest one's overflow: with
    # 2, step i + 1 is enqueued while step i still runs (with 1 the host waited
    # for every step before enqueuing the next, and the GPU idled through the
    # host's enqueue).  A drain round merges after a later step's runs, which
    # is exact: every join is commutative, associative and idempotent.  The
    # caller keeps a step's batches alive until `depth` steps later (or drain()).
    depth = 2

    def __init__(self, engines, fabric):
        import collections
        self.engs = list(engines)
        self.fabric = fabric
        self.S = fabric.world
        assert len(self.engs) == len(fabric.ranks)
        self.pending = collections.deque()  # (batches, ovf tensors, pinned pairs, event), oldest first
        self._pin_pool = []  # pinned (global max, own count) pairs per engine, reused
        self.routed = 0
        self.drains = 0
        self.bind()

    def bind(self):
        _bind_streams(self.engs)

    def step(self, batches):
        _check_streams(self.engs)
        while len(self.pending) >= self.depth:
            self._settle()
        ovfs = self._round(batches)
        self._publish(batches, ovfs)

    arena_type = None  # the value arena the sending batches' handles point into (TREG / TLOG)

    def drain(self, collect=False):
        """route everything still pending (a collective: every rank calls it).
        With `collect`, then reclaim the engines' value arenas when dead bytes
        pass twice the live ones: the receivers append every run's byte
        section, and collection is refused while rounds are in flight (the
        pending batches' handles are read again by a drain round)."""
        _check_streams(self.engs)
        while self.pending:
            self._settle()
        if collect and self.arena_type is not None:
            for e in self.engs:
                n, _ = e.arena_usage(self.arena_type)
                live = getattr(e, "_arena_live", {}).get(self.arena_type, 0)
                if n > 2 * live + (1 << 20):
                    e.__dict__.setdefault("_arena_live", {})[self.arena_type] = e.arena_collect(self.arena_type)

    def _hold(self, on):
        for e in self.engs:
            holds = e.__dict__.setdefault("_route_holds", set())
            (holds.add if on else holds.discard)(id(self))

    chunks = 1  # key-range chunks per round (CSR routers pipeline the exchange over them)

    def _round(self, batches, caps=None):
        """one exchange round.  The batches are cut into `chunks` key ranges;
        chunk c + 1's all-to-alls are in flight while the owners merge chunk c
        (RCCL runs on its own stream; the engine's merge kernels on the
        compute stream).  Drain rounds (caps given) go in one chunk."""
        import torch
        S, fab = self.S, self.fabric
        nch = self.chunks if (caps is None and S > 1) else 1
        if caps is None:
            m = fab.host_max([np.array(self._sizes(b), np.int64) for b in batches])[0]
            caps = self._caps([int(x) for x in m], nch)
        ovfs = [torch.empty(int(b[0].numel()) + 1, dtype=torch.int32, device=torch.device("cuda", e.device))
                for e, b in zip(self.engs, batches)]
        for o in ovfs:
            o[:1].zero_()  # the count; the list is written as it grows
        sends = []  # [chunk][local rank]
        for c in range(nch):
            per = []
            for eng, b, ovf in zip(self.engs, batches, ovfs):
                n = int(b[0].numel())
                per.append(self._part(eng, b, caps, c * n // nch, (c + 1) * n // nch, ovf))
            sends.append(per)
        if S == 1:
            for per in sends:
                for eng, snd in zip(self.engs, per):
                    self._merge(eng, snd, caps)
        else:
            def issue(c):
                recv = [self._recv_bufs(eng, snd, caps) for eng, snd in zip(self.engs, sends[c])]
                works = [fab.a2a([r[k] for r in recv], [s_[k] for s_ in sends[c]], async_op=True)
                         for k in range(len(sends[c][0]))]
                return recv, works

            cur = issue(0)
            for c in range(nch):
                recv, works = cur
                for w in works:
                    w.wait()
                if c + 1 < nch:
                    cur = issue(c + 1)
                for eng, rcv in zip(self.engs, recv):
                    self._merge(eng, rcv, caps)
        self.routed += 1
        return ovfs

    def _recv_bufs(self, eng, snd, caps):
        """the receive buffers of one local rank (shaped like its send buffers)"""
        import torch
        return tuple(torch.empty_like(x) for x in snd)

    def _publish(self, batches, ovfs):
        """global max of the overflow counts, copied to pinned memory behind an event"""
        import torch
        # a pinned pair per engine for this round, back in the pool once settled
        pins = self._pin_pool.pop() if self._pin_pool else [torch.empty(2, dtype=torch.int32, pin_memory=True)
                                                            for _ in ovfs]
        if self.S == 1 and len(ovfs) == 1:
            # one rank: the global max is the own count (one copy, no reduction)
            pins[0][0:1].copy_(ovfs[0][:1], non_blocking=True)
        else:
            gm = [o[:1].clone() for o in ovfs]
            self.fabric.max_all(gm)
            for g, o, p in zip(gm, ovfs, pins):
                p[0:1].copy_(g, non_blocking=True)
                p[1:2].copy_(o[:1], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((batches, ovfs, pins, ev))
        self._hold(True)

    def _settle(self):
        """check the oldest pending round's overflow; run a drain round if any rank overflowed"""
        if not self.pending:
            return
        batches, ovfs, pins, ev = self.pending.popleft()
        if not self.pending:
            self._hold(False)  # a drain round below holds them again
        ev.synchronize()
        gmax = int(pins[0][0])
        counts = [gmax] if (self.S == 1 and len(pins) == 1) else [int(p[1]) for p in pins]
        self._pin_pool.append(pins)
        if gmax == 0:
            return
        sub = [self._subset(b, o[1:1 + k].long()) for b, o, k in zip(batches, ovfs, counts)]
        m = self.fabric.host_max([np.array(self._sizes(s), np.int64) for s in sub])[0]
        # capacity = the whole overflow of the largest sender: nothing can overflow again
        ovfs2 = self._round(sub, caps=self._drain_caps([int(x) for x in m]))
        self.drains += 1
        self._publish(sub, ovfs2)

    @staticmethod
    def _ptr(t):
        return C.c_void_p(t.data_ptr())


# ---- TREG ---------------------------------------------------------------------

class TregRouter(_RunRouter):
    """Routes TREG delta batches between the shards of one node.

    `step(batches)`: batches[i] = (owner, slot, ts, pre, lr, long_bytes) for
    local rank i (CUDA tensors; owner/slot int32, the rest int64 bits;
    long_bytes = `long_bytes(lr)`, a host int).  Partition -> header +
    records + bytes all-to-all -> one merge of every received run.

    `self_direct`: a shard's own entries never enter a run; the partition
    merges them where they lie (jy_treg_route_part_self), so run `self` stays
    empty and one shard alone exchanges and merges nothing.  That costs one
    more read of the whole batch (~28 B per entry: the own entries are spread
    over every line) and saves the own share's record write + read (64 B per
    own entry, 1/S of them), so it pays for S <= 2 only -- the default."""
    arena_type = _lib.TREG

    def __init__(self, engines, fabric, self_direct=None):
        self.self_direct = fabric.world <= 2 if self_direct is None else bool(self_direct)
        super().__init__(engines, fabric)

    def _sizes(self, b):
        return (int(b[0].numel()), int(b[5]))

    def _caps(self, m, nch):
        return run_caps(m[0], m[1], self.S)

    def _drain_caps(self, m):
        return (max(m[0], 1), round8(max(m[1], 8)))

    # The receivers' byte runs land straight in their TREG arenas
    # (jy_arena_reserve): one shard sends to itself by writing there from the
    # partition, several receive there through the exchange, and the merge
    # (jy_treg_converge_routed_at) addresses them in place -- no append copy.
    def _arena_bytes(self, eng, nbytes):
        """this engine's arena tail for `nbytes` received bytes: (uint8 tensor over it, rebase);
        the rebase waits in `_rebase` for the engine's merge of this round"""
        dst, rebase = eng.arena_reserve(_lib.TREG, nbytes)
        self.__dict__.setdefault("_rebase", {})[id(eng)] = rebase
        return _device_bytes(dst, nbytes, eng.device), rebase

    def _recv_bufs(self, eng, snd, caps):
        import torch
        hdr, recs, _ = snd
        byts, _ = self._arena_bytes(eng, self.S * caps[1])
        return (torch.empty_like(hdr), torch.empty_like(recs), byts)

    def _part(self, eng, b, caps, a, e, ovf):
        import torch
        S = self.S
        cap, capb = caps
        own, slot, ts, pre, lr = b[:5]
        n = int(own.numel())
        assert (a, e) == (0, n), "TREG rounds are not chunked"
        dev = torch.device("cuda", eng.device)
        alone = S == 1 and self.self_direct
        # one shard merging its own entries where they lie: the runs stay
        # empty -- token buffers instead of S * cap records
        recs = torch.empty((1 if alone else S * cap, 4), dtype=torch.int64, device=dev)
        if alone:
            byts = torch.empty(8, dtype=torch.uint8, device=dev)
        elif S == 1:  # its own receiver: the run's bytes go to the arena directly
            byts, _ = self._arena_bytes(eng, capb)
        else:
            byts = torch.empty(S * capb, dtype=torch.uint8, device=dev)
        hdr = torch.empty((S, 2), dtype=torch.int64, device=dev)
        if n:
            for t in (own, slot, ts, pre, lr):
                assert t.is_cuda and t.is_contiguous() and t.numel() == n
            ptrs = (eng.h, n, own.data_ptr(), slot.data_ptr(), ts.data_ptr(), pre.data_ptr(), lr.data_ptr(), S)
            outs = (_lib.DEVICE, self._ptr(recs), self._ptr(byts), self._ptr(hdr), self._ptr(ovf))
            if self.self_direct:
                me = self.fabric.ranks[self.engs.index(eng)]
                eng._check(eng.lib.jy_treg_route_part_self(*ptrs, me, 1 if alone else cap, 8 if alone else capb,
                                                           *outs))
            else:
                eng._check(eng.lib.jy_treg_route_part(*ptrs, cap, capb, *outs))
        else:
            hdr.zero_()
        return (hdr, recs, byts)

    def _merge(self, eng, rcv, caps):
        if self.S == 1 and self.self_direct:
            return  # the partition merged every entry where it lay: no run holds a record
        hdr, recs, byts = rcv
        eng._check(eng.lib.jy_treg_converge_routed_at(eng.h, self.S, caps[0], caps[1], self._ptr(recs),
                                                      self._ptr(hdr), self._rebase.pop(id(eng))))

    def _subset(self, b, idx):
        own, slot, ts, pre, lr = (t.index_select(0, idx).contiguous() for t in b[:5])
        return (own, slot, ts, pre, lr, long_bytes(lr))


# ---- TLOG / UJSON (CSR runs, k_route_csr.hip) ------------------------------------

ENT_SLACK = 1.25
ENT_MARGIN = 1024


def _cap_of(m, world, slack, margin):
    if world == 1:
        return max(m, 1)
    return min(max(m, 1), int(np.ceil(m / world * slack)) + margin)


class TlogRouter(_RunRouter):
    """Routes TLOG delta batches (a key with its whole log) between shards.

    batches[i] = (owner, slot, cutoff, ent_offs, ts, pre, lr, long_bytes):
    per key owner / owner-side slot (int32), cutoff (int64 bits) and CSR
    offsets (int64, n + 1); per entry ts, value handle pre / lr (int64 bits,
    packed on the sending engine); long_bytes = `long_bytes(lr)`.  Each
    owner merges the received runs one source at a time."""
    arena_type = _lib.TLOG

    def _sizes(self, b):
        return (int(b[0].numel()), int(b[4].numel()), int(b[7]))

    chunks = 4

    def _caps(self, m, nch):
        S = self.S
        m = [-(-x // nch) for x in m]
        return (_cap_of(m[0], S, CAP_SLACK, CAP_MARGIN), _cap_of(m[1], S, ENT_SLACK, ENT_MARGIN),
                round8(_cap_of(m[2], S, BYTE_SLACK, BYTE_MARGIN)))

    def _drain_caps(self, m):
        return (max(m[0], 1), max(m[1], 1), round8(max(m[2], 8)))

    def _part(self, eng, b, caps, a, e, ovf):
        import torch
        S = self.S
        cap_k, cap_e, capb = caps
        own, slot, cut, offs, ts, pre, lr = b[:7]
        n, nent = int(own.numel()), int(ts.numel())
        assert int(offs.numel()) == n + 1
        W = int(eng.lib.jy_route_words(_lib.TLOG, cap_k, (C.c_uint64 * 1)(cap_e)))
        dev = torch.device("cuda", eng.device)
        runs = torch.empty(S * W, dtype=torch.int64, device=dev)
        byts = torch.empty(S * capb, dtype=torch.uint8, device=dev)
        hdr = torch.empty(S * 8, dtype=torch.int64, device=dev)
        eng._check(eng.lib.jy_tlog_route_part(
            eng.h, e - a, own[a:].data_ptr(), slot[a:].data_ptr(), cut[a:].data_ptr(), offs[a:].data_ptr(), nent,
            ts.data_ptr(), pre.data_ptr(), lr.data_ptr(), S, cap_k, cap_e, capb, a, _lib.DEVICE, self._ptr(runs),
            self._ptr(byts), self._ptr(hdr), self._ptr(ovf)))
        self.last_hdr = hdr
        return (runs, byts)

    def _merge(self, eng, rcv, caps):
        runs, byts = rcv
        eng._check(eng.lib.jy_tlog_converge_routed(eng.h, self.S, caps[0], caps[1], caps[2], self._ptr(runs),
                                                   self._ptr(byts)))

    def _subset(self, b, idx):
        own, slot, cut, offs, ts, pre, lr = b[:7]
        noffs, (ts2, pre2, lr2) = _csr_pick(offs, idx, [ts, pre, lr])
        return (own.index_select(0, idx), slot.index_select(0, idx), cut.index_select(0, idx), noffs, ts2, pre2,
                lr2, long_bytes(lr2))


class UjsonRouter(_RunRouter):
    """Routes UJSON delta batches (a document with its elements, vv entries
    and cloud dots) between shards.

    batches[i] = (owner, slot, el_offs, dots, elems, vv_offs, vv, cloud_offs,
    cloud): int32 per-doc owner / owner-side slot, int64 CSR offsets and
    packed dots (column << 48 | seq).  Dots carry engine columns, so every
    shard must register the cluster's replica ids in one order
    (`Engine.replica_cols` with the same list on every shard)."""

    def _sizes(self, b):
        return (int(b[0].numel()), int(b[3].numel()), int(b[6].numel()), int(b[8].numel()))

    chunks = 4

    def _caps(self, m, nch):
        S = self.S
        m = [-(-x // nch) for x in m]
        return (_cap_of(m[0], S, CAP_SLACK, CAP_MARGIN) + 1, _cap_of(m[1], S, ENT_SLACK, ENT_MARGIN),
                _cap_of(m[2], S, ENT_SLACK, ENT_MARGIN), _cap_of(m[3], S, ENT_SLACK, ENT_MARGIN))

    def _drain_caps(self, m):
        return (max(m[0], 1) + 1, max(m[1], 1), max(m[2], 1), max(m[3], 1))

    def _part(self, eng, b, caps, a, e, ovf):
        import torch
        S = self.S
        cap_k, cap_e, cap_v, cap_c = caps
        own, slot, eo, dots, elems, vo, vv, co, cloud = b[:9]
        W = int(eng.lib.jy_route_words(_lib.UJSON, cap_k, (C.c_uint64 * 3)(cap_e, cap_v, cap_c)))
        dev = torch.device("cuda", eng.device)
        runs = torch.empty(S * W, dtype=torch.int64, device=dev)
        hdr = torch.empty(S * 8, dtype=torch.int64, device=dev)
        eng._check(eng.lib.jy_ujson_route_part(
            eng.h, e - a, own[a:].data_ptr(), slot[a:].data_ptr(), eo[a:].data_ptr(), int(dots.numel()),
            dots.data_ptr(), elems.data_ptr(), vo[a:].data_ptr(), int(vv.numel()), vv.data_ptr(), co[a:].data_ptr(),
            int(cloud.numel()), cloud.data_ptr(), S, cap_k, cap_e, cap_v, cap_c, a, _lib.DEVICE, self._ptr(runs),
            self._ptr(hdr), self._ptr(ovf)))
        self.last_hdr = hdr
        return (runs,)

    def _merge(self, eng, rcv, caps):
        (runs,) = rcv
        eng._check(eng.lib.jy_ujson_converge_routed(eng.h, self.S, *caps, self._ptr(runs)))

    def _subset(self, b, idx):
        own, slot, eo, dots, elems, vo, vv, co, cloud = b[:9]
        eo2, (dots2, elems2) = _csr_pick(eo, idx, [dots, elems])
        vo2, (vv2,) = _csr_pick(vo, idx, [vv])
        co2, (cloud2,) = _csr_pick(co, idx, [cloud])
        return (own.index_select(0, idx), slot.index_select(0, idx), eo2, dots2, elems2, vo2, vv2, co2, cloud2)


# ---- counters (dense column blocks) --------------------------------------------

class CounterRouter:
    """Routes dense GCOUNT / PNCOUNT peer batches between the shards of a node.

    A peer replica that runs the same sharding flushes shard by shard, so
    its batch for one replica column arrives grouped by owner: K slots for
    owner 0, then owner 1, ... (each owner's run in that owner's slot
    order).  Rank r ingests C peer columns: `ingest` is an int64 CUDA tensor
    [nsigns][C][S][K] and `cols[r]` the engine columns of r's peers.  Chunk c
    of the exchange moves column c of every rank to its owners (an
    equal-split all-to-all); the owner merges the S received columns with one
    block converge while chunk c + 1 is in flight (double-buffered)."""

    def __init__(self, engines, fabric, ctype):
        self.engs = list(engines)
        self.fabric = fabric
        self.S = fabric.world
        self.ctype = ctype
        self.bind()

    def bind(self):
        _bind_streams(self.engs)

    def step(self, ingests, cols):
        """ingests[i]: local rank i's [nsigns][C][S][K] batch; cols[r][c]: the
        engine column of rank r's c-th peer (every rank knows every rank's)"""
        import torch
        _check_streams(self.engs)
        S, fab = self.S, self.fabric
        nsigns, Cn, S_, K = ingests[0].shape
        assert S_ == S
        merge = [self._merge_fn(e) for e in self.engs]
        if S == 1:
            for eng, m, ing in zip(self.engs, merge, ingests):
                m(np.asarray(cols[0], np.uint16), ing[:, :, 0])
            return
        bufs = [[torch.empty((nsigns, S, K), dtype=torch.int64, device=ing.device) for _ in range(2)]
                for ing in ingests]
        works = [None, None]

        def issue(c):
            b = c & 1
            works[b] = [fab.a2a([bf[b][g] for bf in bufs], [ing[g, c] for ing in ingests], async_op=True)
                        for g in range(nsigns)]

        issue(0)
        for c in range(Cn):
            for w in works[c & 1]:
                w.wait()
            if c + 1 < Cn:
                issue(c + 1)
            colc = np.array([cols[s][c] for s in range(S)], np.uint16)
            for m, bf in zip(merge, bufs):
                m(colc, bf[c & 1])

    def _merge_fn(self, eng):
        if self.ctype == _lib.PNCOUNT:
            return lambda cols, v: eng.pncount_converge_block(cols, 0, v[0], v[1])
        return lambda cols, v: eng.gcount_converge_block(cols, 0, v[0])


# ---- cross-shard key resolution on the GPU ----------------------------------------

class KeyResolver:
    """Owner and owner-side slot of every key of ingested batches, on the GPU
    (k_keyroute.hip): the reference's `_data_for(key)` (repo_treg.pony:37-42,
    every repo_*.pony) when the key's slot lives on another shard.

    `resolve(keysets)`: keysets[i] = (key bytes uint8, key offsets int64) CUDA
    tensors of local rank i -> [(owner int32, slot int32)] CUDA tensors.
    Per call: the senders regroup their keys by owner (jy_keys_route_part),
    the per-owner counts cross the host (one small readback + a host
    all-to-all), the key lengths and bytes go to their owners (variable
    all-to-alls: RCCL over xGMI with nccl), every owner interns what it
    received in its device directory (jy_keys_intern_lens, create on miss),
    and the slots come back the same way (jy_keys_route_back puts them in
    input order).  Keys are never walked by the host."""

    def __init__(self, engines, fabric, ctype):
        self.engs = list(engines)
        self.fabric = fabric
        self.S = fabric.world
        self.ctype = ctype
        assert len(self.engs) == len(fabric.ranks)
        _bind_streams(self.engs)

    def resolve(self, keysets):
        import torch
        _check_streams(self.engs)
        S, fab = self.S, self.fabric
        parts = [e.keys_route_part(kb, ko, S) for e, (kb, ko) in zip(self.engs, keysets)]
        cnt = [p[4].cpu().numpy() for p in parts]  # [keys per owner, bytes per owner]
        send_k = [c[:S] for c in cnt]
        send_b = [c[S:] for c in cnt]
        recv_k = fab.host_a2a(send_k)
        recv_b = fab.host_a2a(send_b)
        dev = [torch.device("cuda", e.device) for e in self.engs]
        lens = [torch.empty(max(int(k.sum()), 1), dtype=torch.int64, device=d) for k, d in zip(recv_k, dev)]
        byts = [torch.empty(max(int(b.sum()), 1), dtype=torch.uint8, device=d) for b, d in zip(recv_b, dev)]
        fab.a2a_v(lens, [p[2] for p in parts], recv_k, send_k)
        fab.a2a_v(byts, [p[3] for p in parts], recv_b, send_b)
        answers = [e.keys_intern_lens(self.ctype, b, l[:int(k.sum())])
                   for e, b, l, k in zip(self.engs, byts, lens, recv_k)]
        back = [torch.empty(max(int(p[0].numel()), 1), dtype=torch.int32, device=d) for p, d in zip(parts, dev)]
        fab.a2a_v(back, [a if a.numel() else torch.empty(1, dtype=torch.int32, device=a.device) for a in answers],
                  send_k, recv_k)
        return [(p[0], e.keys_route_back(p[1], b)) for e, p, b in zip(self.engs, parts, back)]


# ---- control plane ----------------------------------------------------------------

def _a2a_host(dist, group, send, send_counts):
    """variable all-to-all of a 1-D int64 / uint8 numpy array over `group` (host)"""
    import torch
    world = dist.get_world_size(group)
    sc = torch.tensor(np.asarray(send_counts, np.int64))
    rc = torch.empty(world, dtype=torch.int64)
    dist.all_to_all_single(rc, sc, group=group)
    t = torch.from_numpy(np.ascontiguousarray(send))
    out = torch.empty(int(rc.sum()), dtype=t.dtype)
    dist.all_to_all_single(out, t, rc.tolist(), list(map(int, send_counts)), group=group)
    return out.numpy(), rc.numpy()


class ShardRouter:
    """Owner-slot directory of one rank, on the host: the reference the GPU
    path (KeyResolver) is checked against, and the resolver of the CPU-only
    gloo tests (an oracle stand-in interns there).

    `intern_local(keys_table) -> slots` interns keys on this rank's engine
    (or, in CPU tests, on an oracle stand-in)."""

    def __init__(self, rank, world, intern_local, dist=None, group=None):
        self.rank, self.world = rank, world
        self.intern_local = intern_local
        self.dist, self.group = dist, group
        self.directory = {}  # key bytes -> slot on its owner

    def resolve(self, kb, ko):
        """owner and owner-side slot of every key of a batch (collective)"""
        kb = np.ascontiguousarray(kb, np.uint8)
        ko = np.ascontiguousarray(ko, np.uint64)
        n = len(ko) - 1
        own = owners(kb, ko, self.world)
        slot = np.full(n, _lib.JY_NO_SLOT, np.uint32)
        keys = [bytes(kb[ko[i]:ko[i + 1]]) for i in range(n)]
        mine = np.nonzero(own == self.rank)[0]
        if len(mine):
            sub_b, sub_o = _pick_keys(kb, ko, mine)
            slot[mine] = self.intern_local((sub_b, sub_o))
        ask = [[] for _ in range(self.world)]
        for i in np.nonzero(own != self.rank)[0]:
            s = self.directory.get(keys[i])
            if s is None:
                ask[own[i]].append(i)
            else:
                slot[i] = s
        if self.world > 1:
            self._exchange(keys, ask, slot)
        for i in np.nonzero(own != self.rank)[0]:
            self.directory[keys[i]] = int(slot[i])
        return own, slot

    def _exchange(self, keys, ask, slot):
        dist, g = self.dist, self.group
        # requests: key bytes + lengths per owner
        req_bytes, req_lens, nbytes, nkeys = [], [], [], []
        for d in range(self.world):
            bs = [keys[i] for i in ask[d]]
            req_bytes.append(np.frombuffer(b"".join(bs), np.uint8))
            req_lens.append(np.array([len(b) for b in bs], np.int64))
            nbytes.append(len(req_bytes[-1]))
            nkeys.append(len(bs))
        got_bytes, _ = _a2a_host(dist, g, np.concatenate(req_bytes), nbytes)
        got_lens, got_nkeys = _a2a_host(dist, g, np.concatenate(req_lens), nkeys)
        # intern what others asked of us, answer with the slots (same order)
        offs = np.zeros(len(got_lens) + 1, np.uint64)
        offs[1:] = np.cumsum(got_lens, dtype=np.uint64)
        answer = (self.intern_local((got_bytes.astype(np.uint8), offs)).astype(np.int64)
                  if len(got_lens) else np.zeros(0, np.int64))
        back, _ = _a2a_host(dist, g, answer, got_nkeys)
        at = 0
        for d in range(self.world):
            for i in ask[d]:
                slot[i] = back[at]
                at += 1


def _pick_keys(kb, ko, idx):
    lens = (ko[idx + 1] - ko[idx]).astype(np.int64)
    offs = np.zeros(len(idx) + 1, np.uint64)
    offs[1:] = np.cumsum(lens, dtype=np.uint64)
    total = int(offs[-1])
    pos = np.repeat(ko[idx].astype(np.int64) - offs[:-1].astype(np.int64), lens) + np.arange(total)
    return kb[pos], offs
