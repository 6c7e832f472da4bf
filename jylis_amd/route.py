"""Key-hash sharding of one node's GPUs and the delta-routing exchange step.

SURVEY.md section 8e: every merge is per key, so a shard converges without any
collective; the one real exchange is routing an ingested peer batch to the
shards that own its keys.  The reference has no counterpart (every Jylis node
holds every key); this is the intra-node analogue of Cluster.broadcast_deltas
(jylis/cluster.pony:209-213).

Control plane (host, gloo): a key's slot lives on its owner.  The first time
a rank ingests a key owned elsewhere, it sends the key bytes to the owner,
which interns it and answers with the slot (`ShardRouter.resolve`); the
answer is cached.  Data plane (device, RCCL over xGMI): records and long
value bytes move with two all_to_all_single calls per batch.

Everything here runs in every rank (collective calls).
"""
import ctypes as C

import numpy as np

from . import _lib


def owners(kb, ko, nshards):
    """owner shard of every key (jy_keys_owner: FNV-1a-64 + splitmix finaliser mod S)"""
    kb = np.ascontiguousarray(kb, np.uint8)
    ko = np.ascontiguousarray(ko, np.uint64)
    n = len(ko) - 1
    out = np.empty(n, np.uint32)
    _lib.load().jy_keys_owner(n, kb.ctypes.data, ko.ctypes.data, nshards, out.ctypes.data)
    return out


def _a2a_host(dist, group, send, send_counts):
    """variable all-to-all of a 1-D int64 / uint8 numpy array over `group`"""
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
    """Owner-slot directory of one rank.

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


# ---- data plane -------------------------------------------------------------

def partition_counts_np(owner, lr, world):
    """records and long-value bytes per destination (numpy restatement of k_route_count)"""
    lens = np.asarray(lr, np.uint64) & np.uint64((1 << 24) - 1)
    rec = np.bincount(owner, minlength=world).astype(np.uint64)
    byt = np.bincount(owner, weights=np.where(lens > 8, lens, 0).astype(np.float64), minlength=world)
    return rec, byt.astype(np.uint64)


class TregRouter:
    """Routes TREG delta batches between the engines of one node (RCCL)."""

    def __init__(self, eng, dist, group=None):
        self.eng = eng
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist else 1

    def exchange_and_converge(self, owner, slot, ts, pre, lr):
        """one routed converge: partition -> all-to-all(v) -> converge each source run.
        Arguments are CUDA tensors (or numpy) of one ingested batch; every rank calls."""
        import torch
        eng, S = self.eng, self.world
        lib = eng.lib
        from .engine import _arg, _same_mem
        args = [_arg(owner, np.uint32), _arg(slot, np.uint32), _arg(ts, np.uint64), _arg(pre, np.uint64),
                _arg(lr, np.uint64)]
        mem = _same_mem(*[m for (_, _, m) in args])
        n = len(args[0][0])
        rc = np.zeros(S, np.uint64)
        bc = np.zeros(S, np.uint64)
        eng._check(lib.jy_treg_route_count(eng.h, n, args[0][1], args[4][1], S, mem, rc.ctypes.data, bc.ctypes.data))
        dev = torch.device("cuda", eng.device)
        recs = torch.empty((max(n, 1), 4), dtype=torch.int64, device=dev)
        byts = torch.empty(max(int(bc.sum()), 1), dtype=torch.uint8, device=dev)
        eng._check(lib.jy_treg_route_scatter(eng.h, n, args[0][1], args[1][1], args[2][1], args[3][1], args[4][1],
                                             S, rc.ctypes.data, bc.ctypes.data, mem,
                                             C.c_void_p(recs.data_ptr()), C.c_void_p(byts.data_ptr())))
        if S > 1:
            cnt = torch.tensor(np.concatenate([rc, bc]).astype(np.int64), device=dev).view(2, S).t().contiguous()
            rcnt = torch.empty_like(cnt)
            self.dist.all_to_all_single(rcnt, cnt, group=self.group)
            rcnt = rcnt.cpu().numpy()
            rrc, rbc = rcnt[:, 0].astype(np.uint64), rcnt[:, 1].astype(np.uint64)
            rrecs = torch.empty((max(int(rrc.sum()), 1), 4), dtype=torch.int64, device=dev)
            rbyts = torch.empty(max(int(rbc.sum()), 1), dtype=torch.uint8, device=dev)
            self.dist.all_to_all_single(rrecs[:int(rrc.sum())], recs[:n], rrc.astype(np.int64).tolist(),
                                        rc.astype(np.int64).tolist(), group=self.group)
            self.dist.all_to_all_single(rbyts[:int(rbc.sum())], byts[:int(bc.sum())], rbc.astype(np.int64).tolist(),
                                        bc.astype(np.int64).tolist(), group=self.group)
        else:
            rrc, rbc, rrecs, rbyts = rc, bc, recs, byts
        eng._check(lib.jy_treg_converge_routed(eng.h, S, rrc.ctypes.data, rbc.ctypes.data,
                                               C.c_void_p(rrecs.data_ptr()), C.c_void_p(rbyts.data_ptr())))
        return int(rrc.sum())
