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
  u64 shift;     // new_off[s] - off[s]
  u64 keep_end;  // off[s] + surviving prefix length
  u64 lo;        // off[s]
  u64 blo, bhi;  // delta segment (empty if none)
  u64 scan_lo;   // scan_b[blo]
};

// per delta key: its state segment, merged cutoff and whether it merges
struct DInfo {
  u64 lo, hi;  // state segment [off[s], off[s+1])
  u64 cut;     // max(state cutoff, delta cutoff)
  u32 s;       // slot
  u32 raised;  // the delta raises the cutoff (else no state entry drops:
               // every state entry already has ts >= the state cutoff)
};

struct TlogArgs {
  // state (current buffer)
  const u64* off;
  const TRec* rec;
  u64* cutoff;
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
  u64* flag_b;  // [nb + 1]
  u64* scan_b;  // [nb + 1]
  u32* prel;    // [nb] state entries of the key ordered before the delta entry
  KeyInfo* info;  // [nkeys]
};

__global__ __launch_bounds__(kThreads) void k_tlog_prep(TlogArgs A) {
  const u64 k = gid();
  if (k >= A.nd) return;
  const u64 s = A.slot[k];
  A.dptr[s] = (u32)k;
  A.bad[k] = 0;
  const u64 cs = A.cutoff[s], cd = A.dcut[k];
  DInfo D;
  D.lo = A.off[s];
  D.hi = A.off[s + 1];
  D.cut = cs > cd ? cs : cd;
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
__global__ __launch_bounds__(kThreads) void k_tlog_flag_b(TlogArgs A) {
  const u64 j = gid();
  if (j > A.nb) return;
  if (j == A.nb) {
    A.flag_b[j] = 0;
    return;
  }
  const u32 k = A.dseg[j];
  const DInfo D = A.dinfo[k];
  u64 keep = 0;
  const u64 lo = D.lo, hi = D.hi;
  u64 p = hi;
  const u64 t = A.dts[j];
  if (t >= D.cut && !A.bad[k] && A.dptr[D.s] == k) {
    const Ent x{t, A.dpre[j], A.dlr[j]};
    // fast path: new log entries are usually newer than the whole state
    const int c0 = lo < hi ? cmp_at(A.rec, lo, x, A.arena) : -1;
    if (c0 < 0) {
      p = lo;
      keep = 1;
    } else if (c0 == 0) {
      p = lo;
    } else {
      p = lower_bound_entry(A.rec, lo + 1, hi, x, A.arena);
      keep = !(p < hi && cmp_at(A.rec, p, x, A.arena) == 0);
    }
  }
  A.flag_b[j] = keep;
  A.prel[j] = (u32)(p - lo);
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
__global__ __launch_bounds__(kThreads) void k_tlog_info(TlogArgs A, const u64* __restrict__ noff,
                                                        unsigned long long* __restrict__ skipped) {
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
  I.shift = noff[s] - I.lo;
  I.keep_end = I.lo + A.keep_a[s];
  I.blo = k == kNone ? 0 : A.doff[k];
  I.bhi = k == kNone ? 0 : A.doff[k + 1];
  I.scan_lo = A.scan_b[I.blo];
  A.info[s] = I;
}

// every surviving state entry: new position = old + key shift + kept delta
// entries ordered before it (those whose state rank is <= its own)
__global__ __launch_bounds__(kThreads) void k_tlog_scatter_a(TlogArgs A, TRec* __restrict__ out) {
  const u64 i = gid();
  if (i >= A.na) return;
  const TRec r = load_rec(A.rec + i);
  const KeyInfo I = A.info[r.seg];
  if (i >= I.keep_end) return;
  u64 pos = i + I.shift;
  if (I.bhi > I.blo) {
    const u32 rr = (u32)(i - I.lo);
    u64 lo = I.blo, hi = I.bhi;
    while (lo < hi) {
      const u64 m = (lo + hi) >> 1;
      if (A.prel[m] <= rr) lo = m + 1;
      else hi = m;
    }
    pos += A.scan_b[lo] - I.scan_lo;
  }
  store_rec(out + pos, r.ts, r.pre, r.lr, r.seg);
}

__global__ __launch_bounds__(kThreads) void k_tlog_scatter_b(TlogArgs A, const u64* __restrict__ noff,
                                                             TRec* __restrict__ out) {
  const u64 j = gid();
  if (j >= A.nb || !A.flag_b[j]) return;
  const u32 k = A.dseg[j];
  const u32 s = A.dinfo[k].s;
  const u64 pos = noff[s] + (A.scan_b[j] - A.scan_b[A.doff[k]]) + A.prel[j];
  store_rec(out + pos, A.dts[j], A.dpre[j], A.dlr[j], s);
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
  if (*p) {
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
    JY_HIP(eng, hipFree(*p));
    *p = nullptr;
  }
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return eng->fail(JY_ENOMEM, std::string("tlog entries: ") + hipGetErrorString(e));
  return JY_OK;
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
  TlogState& t = eng->tlog;
  const u64 nk = eng->nkeys[JY_TLOG];
  if (nd == 0 || nk == 0) return JY_OK;
  // exact live entry count of the current buffer: the previous merge's total
  JY_HIP(eng, hipEventSynchronize(eng->total_ready));
  const u64 na = t.nent_known ? eng->pin_total[0] : 0;
  const int cur = t.cur, nxt = 1 - cur;
  JY_TRY(ensure_entries(eng, nxt, na + nent));

  TlogArgs A{};
  A.off = t.off[cur];
  A.rec = t.rec[cur];
  A.cutoff = t.cutoff;
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
  JY_TRY(jy_scratch(eng, 12, (nent + 1) * 20, &p));
  A.flag_b = static_cast<u64*>(p);
  A.scan_b = A.flag_b + nent + 1;
  A.prel = reinterpret_cast<u32*>(A.scan_b + nent + 1);
  JY_TRY(jy_scratch(eng, 16, (nk + 1) * 8, &p));
  u64* cnt = static_cast<u64*>(p);
  JY_TRY(jy_scratch(eng, 18, nk * sizeof(KeyInfo), &p));
  A.info = static_cast<KeyInfo*>(p);
  JY_TRY(jy_scratch(eng, 17, std::max<u64>(nent, 1) * 4, &p));
  A.dseg = static_cast<const u32*>(p);
  JY_TRY(jy_seg_ids(eng, doff, nd, nent, static_cast<u32*>(p)));

  JY_HIP(eng, hipMemsetAsync(A.dptr, 0xFF, nk * 4, eng->stream));
  LAUNCH(k_tlog_prep, nd, A);
  if (nent) LAUNCH(k_tlog_validate, nent, A);
  LAUNCH(k_tlog_flag_b, nent + 1, A);
  JY_TRY(jy_scan_u64(eng, A.flag_b, A.scan_b, nent));
  LAUNCH(k_tlog_sizes_out, nk + 1, A, cnt);
  JY_TRY(jy_scan_u64(eng, cnt, t.off[nxt], nk));
  LAUNCH(k_tlog_info, nk, A, t.off[nxt], reinterpret_cast<unsigned long long*>(eng->skipped_dev));
  if (na) LAUNCH(k_tlog_scatter_a, na, A, t.rec[nxt]);
  if (nent) LAUNCH(k_tlog_scatter_b, nent, A, t.off[nxt], t.rec[nxt]);
  // publish the new total for the next call (read back asynchronously)
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, t.off[nxt] + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipEventRecord(eng->total_ready, eng->stream));
  t.nent_known = true;
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
