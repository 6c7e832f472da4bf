// k_tlog.hip -- TLOG segmented sorted-merge with cutoff trim, gfx950.
//
// Semantics (oracle/jy_oracle.cpp TLog; tlog.md:116-133, repo_tlog.pony:66-67):
//   cutoff' = max(cutoff_s, cutoff_d)
//   entries' = dedupe(state U delta) restricted to ts >= cutoff', ordered with
//              the later timestamp first, then the greater value first
//              (Pony String order); (ts, value) duplicates collapse.
//
// HBM layout: per type, CSR over slots -- off[kcap+1] (u64); entries are
// 32-B records {ts, pre, lr, seg} (value handle as in TREG: 8-byte big-endian
// prefix + arena offset/length; seg = slot of the entry), so the streaming
// passes move them with 16-B accesses; cutoff[kcap].  Entries are
// double-buffered: a converge rewrites the CSR into the other buffer.
//
// Parallel shape: one thread per ENTRY (state or delta), coalesced, with
// merge-path positions -- no per-key loops, so long or skewed logs cost the
// same per entry as short ones:
//   keep(state e)  = ts >= cutoff'
//   keep(delta e)  = ts >= cutoff' and no equal entry in the state segment
//   pos(e) = new_off[key] + #kept own-side entries before e
//                         + #kept other-side entries ordered before e
// the counts coming from an exclusive scan of the delta keep flags and one
// binary search per delta entry (entry order, value bytes compared only on
// (ts, prefix) ties) into the state segment.  That search's result (the
// entry's state rank, prel) is kept, so the state side finds its count by a
// search over small integers and the delta side needs no second search.  A delta segment that is not strictly
// ordered is not a TLog: its key is left untouched and counted (the
// reference swallows converge errors, repo_tlog.pony:67).
//
// Roofline: HBM.  Per state entry 32 B read; per delta entry 24 B read;
// 32 B written per output entry; per key 16 B offsets + 16 B cutoff; delta
// keep flags, their scan and prel add ~28 B per delta entry; see DESIGN.md.

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr u32 kNone = 0xFFFFFFFFu;

__device__ __forceinline__ u64 gid() { return (u64)blockIdx.x * kThreads + threadIdx.x; }

// > 0 if (ta, pa, la) is ordered before (tb, pb, lb): later ts, then greater value
__device__ __forceinline__ int entry_cmp(u64 ta, u64 pa, u64 la, u64 tb, u64 pb, u64 lb,
                                         const uint8_t* __restrict__ arena) {
  if (ta != tb) return ta > tb ? 1 : -1;
  return jy_value_cmp(pa, la, pb, lb, arena);
}

struct Ent {
  u64 t, p, l;
};

// > 0 if log entry m is ordered before x; value handles are read only on a
// timestamp tie
__device__ __forceinline__ int cmp_at(const TRec* __restrict__ rec, u64 m, const Ent& x,
                                      const uint8_t* __restrict__ arena) {
  const u64 t = rec[m].ts;
  if (t != x.t) return t > x.t ? 1 : -1;
  return jy_value_cmp(rec[m].pre, rec[m].lr, x.p, x.l, arena);
}

// first index in [lo, hi) of a sorted log whose entry is NOT ordered before x
__device__ __forceinline__ u64 lower_bound_entry(const TRec* __restrict__ rec, u64 lo, u64 hi, const Ent& x,
                                                 const uint8_t* __restrict__ arena) {
  while (lo < hi) {
    const u64 m = (lo + hi) >> 1;
    if (cmp_at(rec, m, x, arena) > 0) lo = m + 1;
    else hi = m;
  }
  return lo;
}

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ TRec load_rec(const TRec* __restrict__ p) {
  const u64x2* q = reinterpret_cast<const u64x2*>(p);
  const u64x2 a = __builtin_nontemporal_load(q), b = __builtin_nontemporal_load(q + 1);
  TRec r;
  r.ts = a.x;
  r.pre = a.y;
  r.lr = b.x;
  r.seg = (u32)b.y;
  r.pad = (u32)(b.y >> 32);
  return r;
}

__device__ __forceinline__ void store_rec(TRec* __restrict__ p, u64 ts, u64 pre, u64 lr, u32 seg) {
  u64x2* q = reinterpret_cast<u64x2*>(p);
  u64x2 a, b;
  a.x = ts;
  a.y = pre;
  b.x = lr;
  b.y = seg;
  __builtin_nontemporal_store(a, q);
  __builtin_nontemporal_store(b, q + 1);
}

// per-key record for the state-side scatter: one line instead of six
// scattered per-key arrays
struct KeyInfo {
  u64 lo;        // off[s]: the state segment (its surviving prefix is what the output holds)
  u64 blo, bhi;  // delta segment (empty if none)
  u32 scan_lo;   // scan_b[blo]
  u32 front;     // every delta entry is kept and precedes the whole state
};

// per delta key: its state segment, merged cutoff and whether it merges
struct DInfo {
  u64 lo, hi;  // state segment [off[s], off[s+1])
  u64 cut;     // max(state cutoff, delta cutoff)
  u64 newest;  // ts of the state's first (newest) entry (any value if empty)
  u32 s;       // slot
  u32 raised;  // the delta raises the cutoff (else no state entry drops:
               // every state entry already has ts >= the state cutoff)
};

struct TlogArgs {
  // state (current buffer)
  const u64* off;
  const TRec* rec;
  u64* cutoff;
  u64* newest;
  u64 nkeys, na;
  // delta batch
  u64 nd, nb;
  const u32* slot;
  u32* dptr;
  const u64* dcut;
  const u64* doff;
  const u64* dts;
  const u64* dpre;
  const u64* dlr;
  const uint8_t* arena;
  const u32* dseg;  // [nb] delta key of each delta entry
  // temporaries
  u32* bad;     // [nd]
  DInfo* dinfo;  // [nd]
  u64* keep_a;  // [nkeys] surviving state entries: a prefix of every log
  u32* flag_b;  // [nb + 1]
  u32* scan_b;  // [nb + 1]
  u32* prel;    // [nb] state entries of the key ordered before the delta entry
  u32* slow;       // [nb] 1: the delta entry needs the full search
  u32* slow_list;  // [nb] those entries, compacted (count at slow_n)
  u32* slow_n;
  KeyInfo* info;  // [nkeys]
};

// per delta key.  A slot named twice in one device batch breaks the
// one-delta-per-key contract: both deltas are skipped (counted), the key is
// left untouched.  bad[] and dptr[] are cleared before this launch.
__global__ __launch_bounds__(kThreads) void k_tlog_prep(TlogArgs A) {
  const u64 k = gid();
  if (k >= A.nd) return;
  const u64 s = A.slot[k];
  const u32 prev = atomicCAS(A.dptr + s, kNone, (u32)k);
  if (prev != kNone) {
    A.bad[k] = 1;
    A.bad[prev] = 1;
  }
  const u64 cs = A.cutoff[s], cd = A.dcut[k];
  DInfo D;
  D.lo = A.off[s];
  D.hi = A.off[s + 1];
  D.cut = cs > cd ? cs : cd;
  D.newest = A.newest[s];
  D.s = (u32)s;
  D.raised = cd > cs;
  A.dinfo[k] = D;
}

__global__ __launch_bounds__(kThreads) void k_tlog_validate(TlogArgs A) {
  const u64 j = gid();
  if (j >= A.nb) return;
  const u32 k = A.dseg[j];
  if (j > A.doff[k] &&
      entry_cmp(A.dts[j - 1], A.dpre[j - 1], A.dlr[j - 1], A.dts[j], A.dpre[j], A.dlr[j], A.arena) <= 0)
    A.bad[k] = 1;
}

// the delta key that merges into slot s, or kNone (no delta, or a malformed
// one: the reference swallows the error and leaves the key untouched)
__device__ __forceinline__ u32 merging_key(const TlogArgs& A, u64 s) {
  const u32 k = A.dptr[s];
  return (k != kNone && !A.bad[k]) ? k : kNone;
}

// keep flag of every delta entry and its rank among the state entries.
// prel is non-decreasing along a delta segment: entries dropped by the
// cutoff are its tail and take the segment length.
// keep flag and state rank of every delta entry.  The usual entry is newer
// than its whole log: rank 0, kept, no search.  Entries that need the full
// search (ties with the newest entry, older entries, duplicates) go to a
// worklist so waves of the common case never wait on a searching lane.
__global__ __launch_bounds__(kThreads) void k_tlog_flag_b(TlogArgs A) {
  const u64 j = gid();
  if (j > A.nb) return;
  if (j == A.nb) {
    A.flag_b[j] = 0;
    return;
  }
  const u32 k = A.dseg[j];
  const DInfo D = A.dinfo[k];
  const u64 t = A.dts[j];
  bool slow = false;
  u32 keep = 0;
  u64 p = D.hi;
  if (t >= D.cut && !A.bad[k]) {
    if (D.lo == D.hi || t > D.newest) {
      p = D.lo;
      keep = 1;
    } else {
      slow = true;
    }
  }
  A.slow[j] = slow;  // compacted into the worklist by DeviceSelect
  if (!slow) {
    A.flag_b[j] = keep;
    A.prel[j] = (u32)(p - D.lo);
  }
}

__global__ __launch_bounds__(kThreads) void k_tlog_flag_slow(TlogArgs A) {
  const u32 n = *A.slow_n;
  for (u64 w = gid(); w < n; w += (u64)gridDim.x * kThreads) {
    const u32 j = A.slow_list[w];
    const DInfo D = A.dinfo[A.dseg[j]];
    const Ent x{A.dts[j], A.dpre[j], A.dlr[j]};
    const u64 p = lower_bound_entry(A.rec, D.lo, D.hi, x, A.arena);
    A.flag_b[j] = !(p < D.hi && cmp_at(A.rec, p, x, A.arena) == 0);
    A.prel[j] = (u32)(p - D.lo);
  }
}

__global__ __launch_bounds__(kThreads) void k_tlog_sizes_out(TlogArgs A, u64* __restrict__ cnt) {
  const u64 s = gid();
  if (s > A.nkeys) return;
  if (s == A.nkeys) {
    cnt[s] = 0;
    return;
  }
  const u32 k = merging_key(A, s);
  const u64 lo = A.off[s];
  u64 hi = A.off[s + 1];
  if (k != kNone && A.dinfo[k].raised && lo < hi && A.rec[hi - 1].ts < A.dinfo[k].cut) {
    // entries are in non-increasing ts order: the cutoff drops a suffix
    const u64 c = A.dinfo[k].cut;
    u64 a = lo;
    while (a < hi) {
      const u64 m = (a + hi) >> 1;
      if (A.rec[m].ts >= c) a = m + 1;
      else hi = m;
    }
    hi = a;
  }
  A.keep_a[s] = hi - lo;
  u64 n = hi - lo;
  if (k != kNone) n += A.scan_b[A.doff[k + 1]] - A.scan_b[A.doff[k]];
  cnt[s] = n;
}

// per slot: the state-side scatter record; merged cutoff stored; malformed
// deltas counted
__global__ __launch_bounds__(kThreads) void k_tlog_info(TlogArgs A, unsigned long long* __restrict__ skipped) {
  const u64 s = gid();
  if (s >= A.nkeys) return;
  u32 k = A.dptr[s];
  if (k != kNone) {
    if (A.bad[k]) {
      atomicAdd(skipped, 1ull);
      k = kNone;
    } else {
      A.cutoff[s] = A.dinfo[k].cut;
    }
  }
  KeyInfo I;
  I.lo = A.off[s];
  I.blo = k == kNone ? 0 : A.doff[k];
  I.bhi = k == kNone ? 0 : A.doff[k + 1];
  I.scan_lo = A.scan_b[I.blo];
  I.front = I.bhi > I.blo && A.prel[I.bhi - 1] == 0 && A.scan_b[I.bhi] - I.scan_lo == I.bhi - I.blo;
  A.info[s] = I;
}

// Output-parallel write of the merged logs.  A workgroup owns a fixed range
// of kTileOut output positions (so a skewed log costs its size, never a
// straggler), finds the keys of its range once (noff staged in LDS), and
// every lane resolves its output position r of key s to its source:
//   o_j = (kept deltas before j) + prel_j is non-decreasing over the key's
//   delta segment; c = #kept deltas with o_j <= r.  Position r holds the
//   kept delta of kept-rank c-1 if that one has o == r, else state entry
//   r - c (always inside the surviving prefix).
// Writes are one contiguous 32-B record stream per workgroup.
constexpr u32 kTileOut = 4096;
constexpr u32 kTileKeys = 2048;

__global__ __launch_bounds__(kThreads) void k_tlog_gather_out(TlogArgs A, const u64* __restrict__ noff,
                                                              TRec* __restrict__ out) {
  __shared__ u64 loff[kTileKeys + 2];
  __shared__ u64 sb_sh, se_sh;
  const u64 nk = A.nkeys;
  const u64 total = noff[nk];
  const u64 t0 = (u64)blockIdx.x * kTileOut;
  if (t0 >= total) return;
  const u64 t1 = t0 + kTileOut < total ? t0 + kTileOut : total;
  if (threadIdx.x == 0) {
    // last s with noff[s] <= x, over [0, nk]
    u64 lo = 0, hi = nk + 1;
    while (lo < hi) {
      const u64 m = (lo + hi) >> 1;
      if (noff[m] <= t0) lo = m + 1;
      else hi = m;
    }
    sb_sh = lo - 1;
    hi = nk + 1;
    while (lo < hi) {
      const u64 m = (lo + hi) >> 1;
      if (noff[m] <= t1 - 1) lo = m + 1;
      else hi = m;
    }
    se_sh = lo - 1;
  }
  __syncthreads();
  const u64 sb = sb_sh, se = se_sh;
  const bool local = se - sb + 2 <= kTileKeys + 2;
  if (local)
    for (u64 q = threadIdx.x; q < se - sb + 2; q += kThreads) loff[q] = noff[sb + q];
  __syncthreads();
  for (u64 t = t0 + threadIdx.x; t < t1; t += kThreads) {
    u64 lo = 0, hi = se - sb + 1;  // last q in [0, se-sb] with off(q) <= t
    while (lo < hi) {
      const u64 m = (lo + hi + 1) >> 1;
      const u64 v = local ? loff[m] : noff[sb + m];
      if (v <= t) lo = m;
      else hi = m - 1;
    }
    const u64 s = sb + lo;
    const u64 r = t - (local ? loff[lo] : noff[s]);
    const KeyInfo I = A.info[s];
    u64 a = r;
    if (I.front) {
      // every delta entry kept, all before the state: deltas, then the state
      const u64 K = I.bhi - I.blo;
      if (r < K) {
        const u64 j = I.blo + r;
        if (r == 0) A.newest[s] = A.dts[j];
        store_rec(out + t, A.dts[j], A.dpre[j], A.dlr[j], (u32)s);
        continue;
      }
      a = r - K;
    } else if (I.bhi > I.blo) {
      u64 l = I.blo, h = I.bhi;  // jj: first j with o_j > r
      while (l < h) {
        const u64 m = (l + h) >> 1;
        if ((u64)(A.scan_b[m] - (u32)I.scan_lo) + A.prel[m] <= r) l = m + 1;
        else h = m;
      }
      const u64 jj = l;
      const u64 c = A.scan_b[jj] - (u32)I.scan_lo;
      if (c > 0) {
        // the kept delta of kept-rank c-1: last j in [blo, jj) with scan_b[j] < scan_lo + c
        l = I.blo;
        h = jj;
        while (l < h) {
          const u64 m = (l + h) >> 1;
          if ((u64)(A.scan_b[m] - (u32)I.scan_lo) < c) l = m + 1;
          else h = m;
        }
        const u64 jk = l - 1;
        if (c - 1 + A.prel[jk] == r) {
          if (r == 0) A.newest[s] = A.dts[jk];
          store_rec(out + t, A.dts[jk], A.dpre[jk], A.dlr[jk], (u32)s);
          continue;
        }
      }
      a = r - c;
    }
    const TRec x = load_rec(A.rec + I.lo + a);
    if (r == 0) A.newest[s] = x.ts;
    store_rec(out + t, x.ts, x.pre, x.lr, (u32)s);
  }
}

__global__ __launch_bounds__(kThreads) void k_fill_tail(u64* __restrict__ off, u64 from, u64 to) {
  // off[from+1 .. to] = off[from]  (new, empty slots)
  const u64 i = from + 1 + gid();
  if (i <= to) off[i] = off[from];
}

__global__ __launch_bounds__(kThreads) void k_tlog_sizes(const u64* __restrict__ off, const u64* __restrict__ cutoff,
                                                         const u32* __restrict__ slots, u64 n, u64* __restrict__ len,
                                                         u64* __restrict__ cut) {
  const u64 i = gid();
  if (i >= n) return;
  const u64 s = slots[i];
  len[i] = off[s + 1] - off[s];
  cut[i] = cutoff[s];
}

__global__ __launch_bounds__(kThreads) void k_tlog_gather(const u64* __restrict__ off, const TRec* __restrict__ rec,
                                                          const u32* __restrict__ slots, const u64* __restrict__ ooff,
                                                          u64 n, u64* __restrict__ ots, u64* __restrict__ opre,
                                                          u64* __restrict__ olr) {
  const u64 i = gid();
  if (i >= n) return;
  const u64 s = slots[i];
  u64 o = ooff[i];
  for (u64 j = off[s]; j < off[s + 1]; j++, o++) {
    ots[o] = rec[j].ts;
    opre[o] = rec[j].pre;
    olr[o] = rec[j].lr;
  }
}

__global__ __launch_bounds__(kThreads) void k_seg_starts(const u64* __restrict__ offs, u64 nseg, u32* __restrict__ out) {
  const u64 k = gid();
  if (k < nseg && offs[k] < offs[k + 1]) out[offs[k]] = (u32)k;
}

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

#define LAUNCH(k, n, ...)                                                                          \
  do {                                                                                             \
    hipLaunchKernelGGL(k, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, __VA_ARGS__);     \
    JY_HIP(eng, hipGetLastError());                                                                \
  } while (0)

int32_t realloc_dead(jy_engine* eng, void** p, u64 bytes) {
  // the buffer's contents are dead (it is rewritten): stream-ordered free
  JY_TRACE("tlog entries realloc %llu bytes", (unsigned long long)bytes);
  jy_dev_free(eng, *p);
  *p = nullptr;
  return jy_dev_alloc(eng, p, bytes, "tlog entries");
}

}  // namespace

// ---------------------------------------------------------------------------
// device exclusive scan: out[0..n] with out[n] = total (in[n] must be 0)
int32_t jy_scan_u64(jy_engine* eng, const u64* in, u64* out, u64 n) {
  size_t tmp = 0;
  JY_HIP(eng, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, (int)(n + 1), eng->stream));
  void* t;
  JY_TRY(jy_scratch(eng, 15, tmp, &t));
  JY_HIP(eng, hipcub::DeviceScan::ExclusiveSum(t, tmp, in, out, (int)(n + 1), eng->stream));
  return JY_OK;
}

// segment id of every item of a CSR (offs[0..nseg], n items): mark each
// non-empty segment's first item, then an inclusive max-scan carries it on
int32_t jy_seg_ids(jy_engine* eng, const u64* offs, u64 nseg, u64 n, u32* out) {
  if (n == 0) return JY_OK;
  JY_HIP(eng, hipMemsetAsync(out, 0, n * 4, eng->stream));
  LAUNCH(k_seg_starts, nseg, offs, nseg, out);
  size_t tmp = 0;
  JY_HIP(eng, hipcub::DeviceScan::InclusiveScan(nullptr, tmp, out, out, hipcub::Max(), (int)n, eng->stream));
  void* t;
  JY_TRY(jy_scratch(eng, 15, tmp, &t));
  JY_HIP(eng, hipcub::DeviceScan::InclusiveScan(t, tmp, out, out, hipcub::Max(), (int)n, eng->stream));
  return JY_OK;
}

static int32_t ensure_entries(jy_engine* eng, int buf, u64 need) {
  TlogState& t = eng->tlog;
  if (need <= t.ecap[buf] && t.rec[buf]) return JY_OK;
  const u64 nc = std::max<u64>(std::max<u64>(need + need / 2, eng->cfg.entry_capacity[JY_TLOG]), 1024);
  JY_TRY(realloc_dead(eng, reinterpret_cast<void**>(&t.rec[buf]), nc * sizeof(TRec)));
  t.ecap[buf] = nc;
  return JY_OK;
}

int32_t jy_tlog_grow(jy_engine* eng, u64 need) {
  TlogState& t = eng->tlog;
  if (need <= t.kcap && t.cutoff) return JY_OK;
  u64 nk = std::max<u64>(need, t.kcap ? t.kcap * 2 : need);
  nk = std::max<u64>((nk + 63) & ~63ull, 64);
  void* c = t.cutoff;
  JY_TRY(jy_realloc(eng, &c, t.kcap * 8, nk * 8, true));
  t.cutoff = static_cast<u64*>(c);
  void* w = t.newest;
  JY_TRY(jy_realloc(eng, &w, t.kcap * 8, nk * 8, true));
  t.newest = static_cast<u64*>(w);
  for (int b = 0; b < 2; b++) {
    void* o = t.off[b];
    JY_TRY(jy_realloc(eng, &o, t.kcap ? (t.kcap + 1) * 8 : 0, (nk + 1) * 8, true));
    t.off[b] = static_cast<u64*>(o);
  }
  t.kcap = nk;
  for (int b = 0; b < 2; b++) JY_TRY(ensure_entries(eng, b, 1));
  return JY_OK;
}

// new slots [from, to) start as empty logs: off[from+1..to] = off[from]
int32_t jy_tlog_extend(jy_engine* eng, u64 from, u64 to) {
  if (to <= from) return JY_OK;
  TlogState& t = eng->tlog;
  LAUNCH(k_fill_tail, to - from, t.off[t.cur], from, to);
  return JY_OK;
}

int32_t jy_tlog_merge(jy_engine* eng, u64 nd, const u32* slot, const u64* dcut, const u64* doff, u64 nent,
                      const u64* dts, const u64* dpre, const u64* dlr) {
  JyTimed tm(eng);
  TlogState& t = eng->tlog;
  const u64 nk = eng->nkeys[JY_TLOG];
  if (nd == 0 || nk == 0) return JY_OK;
  if (nent >= (1ull << 31)) return eng->fail(JY_ERANGE, "tlog converge: more than 2^31 entries in one call");
  // live entries of the current buffer: exact when the previous merge's
  // total has landed (non-blocking query), else the host upper bound; the
  // kernels take the exact count from off[nkeys] in HBM.  The host never
  // waits for the GPU here, so merges queue back to back.
  const double t_enter = jy_tracing() ? jy_now_us() : 0;
  u64 na = 0;
  if (t.nent_known) {
    const hipError_t q = hipEventQuery(eng->total_ready);
    if (q == hipSuccess) na = eng->pin_total[0];
    else if (q == hipErrorNotReady) na = t.nent_bound;
    else JY_HIP(eng, q);
  }
  const double t_synced = jy_tracing() ? jy_now_us() : 0;
  const int cur = t.cur, nxt = 1 - cur;
  JY_TRY(ensure_entries(eng, nxt, na + nent));

  TlogArgs A{};
  A.off = t.off[cur];
  A.rec = t.rec[cur];
  A.cutoff = t.cutoff;
  A.newest = t.newest;
  A.nkeys = nk;
  A.na = na;
  A.nd = nd;
  A.nb = nent;
  A.slot = slot;
  A.dcut = dcut;
  A.doff = doff;
  A.dts = dts;
  A.dpre = dpre;
  A.dlr = dlr;
  A.arena = eng->arena[JY_TLOG].p;
  void* p;
  JY_TRY(jy_scratch(eng, 8, nk * 4, &p));
  A.dptr = static_cast<u32*>(p);
  JY_TRY(jy_scratch(eng, 9, nd * (sizeof(DInfo) + 4), &p));
  A.dinfo = static_cast<DInfo*>(p);
  A.bad = reinterpret_cast<u32*>(A.dinfo + nd);
  JY_TRY(jy_scratch(eng, 11, nk * 8, &p));
  A.keep_a = static_cast<u64*>(p);
  JY_TRY(jy_scratch(eng, 12, (nent + 1) * 20 + 16, &p));
  A.flag_b = static_cast<u32*>(p);
  A.scan_b = A.flag_b + nent + 1;
  A.prel = A.scan_b + nent + 1;
  A.slow = A.prel + nent + 1;
  A.slow_list = A.slow + nent + 1;
  A.slow_n = A.slow_list + nent + 1;
  JY_TRY(jy_scratch(eng, 16, (nk + 1) * 8, &p));
  u64* cnt = static_cast<u64*>(p);
  JY_TRY(jy_scratch(eng, 18, nk * sizeof(KeyInfo), &p));
  A.info = static_cast<KeyInfo*>(p);
  JY_TRY(jy_scratch(eng, 17, std::max<u64>(nent, 1) * 4, &p));
  A.dseg = static_cast<const u32*>(p);
  JY_TRY(jy_seg_ids(eng, doff, nd, nent, static_cast<u32*>(p)));

  JY_HIP(eng, hipMemsetAsync(A.dptr, 0xFF, nk * 4, eng->stream));
  JY_HIP(eng, hipMemsetAsync(A.bad, 0, nd * 4, eng->stream));
  LAUNCH(k_tlog_prep, nd, A);
  if (nent) LAUNCH(k_tlog_validate, nent, A);
  LAUNCH(k_tlog_flag_b, nent + 1, A);
  if (nent) {
    size_t tmp = 0;
    hipcub::CountingInputIterator<u32> idx(0);
    JY_HIP(eng, hipcub::DeviceSelect::Flagged(nullptr, tmp, idx, A.slow, A.slow_list, A.slow_n, (int)nent,
                                              eng->stream));
    JY_TRY(jy_scratch(eng, 15, tmp, &p));
    JY_HIP(eng, hipcub::DeviceSelect::Flagged(p, tmp, idx, A.slow, A.slow_list, A.slow_n, (int)nent, eng->stream));
    const u32 g = (u32)std::min<u64>(2048, (nent + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(k_tlog_flag_slow, dim3(g), dim3(kThreads), 0, eng->stream, A);
    JY_HIP(eng, hipGetLastError());
  }
  {
    size_t tmp = 0;
    JY_HIP(eng, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, A.flag_b, A.scan_b, (int)(nent + 1), eng->stream));
    JY_TRY(jy_scratch(eng, 15, tmp, &p));
    JY_HIP(eng, hipcub::DeviceScan::ExclusiveSum(p, tmp, A.flag_b, A.scan_b, (int)(nent + 1), eng->stream));
  }
  LAUNCH(k_tlog_sizes_out, nk + 1, A, cnt);
  JY_TRY(jy_scan_u64(eng, cnt, t.off[nxt], nk));
  LAUNCH(k_tlog_info, nk, A, reinterpret_cast<unsigned long long*>(eng->skipped_dev));
  {
    // output size bound: surviving state + kept delta <= na + nent
    const u64 nout = na + nent;
    const u32 tiles = (u32)std::max<u64>(1, (nout + kTileOut - 1) / kTileOut);
    hipLaunchKernelGGL(k_tlog_gather_out, dim3(tiles), dim3(kThreads), 0, eng->stream, A, t.off[nxt], t.rec[nxt]);
    JY_HIP(eng, hipGetLastError());
  }
  // publish the new total for the next call (read back asynchronously)
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, t.off[nxt] + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipEventRecord(eng->total_ready, eng->stream));
  if (jy_tracing()) JY_TRACE("tlog merge host: wait %.1f us, issue %.1f us", t_synced - t_enter, jy_now_us() - t_synced);
  t.nent_known = true;
  t.nent_bound = na + nent;
  t.cur = nxt;
  return JY_OK;
}

int32_t jy_tlog_sizes(jy_engine* eng, u64 n, const u32* slots, u64* len, u64* cut) {
  TlogState& t = eng->tlog;
  LAUNCH(k_tlog_sizes, n, t.off[t.cur], t.cutoff, slots, n, len, cut);
  return JY_OK;
}

int32_t jy_tlog_gather(jy_engine* eng, u64 n, const u32* slots, const u64* ooff, u64* ts, u64* pre, u64* lr) {
  TlogState& t = eng->tlog;
  const int c = t.cur;
  LAUNCH(k_tlog_gather, n, t.off[c], t.rec[c], slots, ooff, n, ts, pre, lr);
  return JY_OK;
}
