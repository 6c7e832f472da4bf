// k_tlog.hip -- TLOG segmented sorted-merge with cutoff trim, gfx950.
//
// Semantics (oracle/jy_oracle.cpp TLog; tlog.md:116-133, repo_tlog.pony:66-67):
//   cutoff' = max(cutoff_s, cutoff_d)
//   entries' = dedupe(state U delta) restricted to ts >= cutoff', ordered with
//              the later timestamp first, then the greater value first
//              (Pony String order); (ts, value) duplicates collapse.
//
// HBM layout: per type, CSR over slots -- off[kcap+1] (u64); entries SoA
// ts / pre / lr (u64 each; value handle as in TREG: 8-byte big-endian prefix
// + arena offset/length) and seg (u32 slot of the entry); cutoff[kcap].
// Entries are double-buffered: a converge rewrites the CSR into the other
// buffer.
//
// Parallel shape: one thread per ENTRY (state or delta), coalesced, with
// merge-path positions -- no per-key loops, so long or skewed logs cost the
// same per entry as short ones:
//   keep(state e)  = ts >= cutoff'
//   keep(delta e)  = ts >= cutoff' and no equal entry in the state segment
//   pos(e) = new_off[key] + #kept own-side entries before e
//                         + #kept other-side entries ordered before e
// the counts coming from exclusive scans of the keep flags and one binary
// search (entry order, value bytes compared only on (ts, prefix) ties) into
// the other side's sorted segment.  A delta segment that is not strictly
// ordered is not a TLog: its key is left untouched and counted (the
// reference swallows converge errors, repo_tlog.pony:67).
//
// Roofline: HBM.  Per input entry: 24 B read (+4 B seg, state side) and
// 28 B written per output entry; per key 16 B offsets + 16 B cutoff; keep
// flags and their scans add 24 B per input entry (u64 flag, scan write +
// read); see DESIGN.md.

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
__device__ __forceinline__ int cmp_at(const u64* __restrict__ ts, const u64* __restrict__ pre,
                                      const u64* __restrict__ lr, u64 m, const Ent& x,
                                      const uint8_t* __restrict__ arena) {
  const u64 t = ts[m];
  if (t != x.t) return t > x.t ? 1 : -1;
  return jy_value_cmp(pre[m], lr[m], x.p, x.l, arena);
}

// first index in [lo, hi) of a sorted log whose entry is NOT ordered before x
__device__ __forceinline__ u64 lower_bound_entry(const u64* __restrict__ ts, const u64* __restrict__ pre,
                                                 const u64* __restrict__ lr, u64 lo, u64 hi, const Ent& x,
                                                 const uint8_t* __restrict__ arena) {
  while (lo < hi) {
    const u64 m = (lo + hi) >> 1;
    if (cmp_at(ts, pre, lr, m, x, arena) > 0) lo = m + 1;
    else hi = m;
  }
  return lo;
}

// per-key record for the state-side scatter: one cache line instead of six
// scattered per-key arrays
struct KeyInfo {
  u64 shift;     // new_off[s] - off[s]
  u64 keep_end;  // off[s] + surviving prefix length
  u64 blo, bhi;  // delta segment (empty if none)
  u64 scan_lo;   // scan_b[blo]
  u64 pad;
};

struct TlogArgs {
  // state (current buffer)
  const u64* off;
  const u64* ts;
  const u64* pre;
  const u64* lr;
  const u32* seg;
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
  u64* cut;     // [nd] merged cutoff
  u64* keep_a;  // [nkeys] surviving state entries: a prefix of every log
  u64* flag_b;
  u64* scan_b;
  KeyInfo* info;  // [nkeys]
};

__global__ __launch_bounds__(kThreads) void k_tlog_prep(TlogArgs A) {
  const u64 k = gid();
  if (k >= A.nd) return;
  const u64 s = A.slot[k];
  A.dptr[s] = (u32)k;
  A.bad[k] = 0;
  const u64 cs = A.cutoff[s], cd = A.dcut[k];
  A.cut[k] = cs > cd ? cs : cd;
}

__global__ __launch_bounds__(kThreads) void k_tlog_validate(TlogArgs A) {
  const u64 j = gid();
  if (j >= A.nb) return;
  const u32 k = A.dseg[j];
  if (j > A.doff[k] &&
      entry_cmp(A.dts[j - 1], A.dpre[j - 1], A.dlr[j - 1], A.dts[j], A.dpre[j], A.dlr[j], A.arena) <= 0)
    A.bad[k] = 1;
}

__global__ __launch_bounds__(kThreads) void k_tlog_drop_bad(TlogArgs A, unsigned long long* __restrict__ skipped) {
  const u64 k = gid();
  if (k >= A.nd) return;
  if (A.bad[k]) {
    A.dptr[A.slot[k]] = kNone;
    atomicAdd(skipped, 1ull);
  }
}

__global__ __launch_bounds__(kThreads) void k_tlog_flag_b(TlogArgs A) {
  const u64 j = gid();
  if (j > A.nb) return;
  if (j == A.nb) {
    A.flag_b[j] = 0;
    return;
  }
  const u32 k = A.dseg[j];
  const u64 s = A.slot[k];
  u64 keep = 0;
  if (A.dptr[s] == k && A.dts[j] >= A.cut[k]) {
    const Ent x{A.dts[j], A.dpre[j], A.dlr[j]};
    const u64 hi = A.off[s + 1];
    const u64 p = lower_bound_entry(A.ts, A.pre, A.lr, A.off[s], hi, x, A.arena);
    keep = !(p < hi && cmp_at(A.ts, A.pre, A.lr, p, x, A.arena) == 0);
  }
  A.flag_b[j] = keep;
}

__global__ __launch_bounds__(kThreads) void k_tlog_sizes_out(TlogArgs A, u64* __restrict__ cnt) {
  const u64 s = gid();
  if (s > A.nkeys) return;
  if (s == A.nkeys) {
    cnt[s] = 0;
    return;
  }
  const u32 k = A.dptr[s];
  const u64 lo = A.off[s];
  u64 hi = A.off[s + 1];
  if (k != kNone) {
    // entries are in non-increasing ts order: the cutoff drops a suffix
    const u64 c = A.cut[k];
    u64 a = lo;
    while (a < hi) {
      const u64 m = (a + hi) >> 1;
      if (A.ts[m] >= c) a = m + 1;
      else hi = m;
    }
    hi = a;
  }
  A.keep_a[s] = hi - lo;
  u64 n = hi - lo;
  if (k != kNone) n += A.scan_b[A.doff[k + 1]] - A.scan_b[A.doff[k]];
  cnt[s] = n;
}

__global__ __launch_bounds__(kThreads) void k_tlog_info(TlogArgs A, const u64* __restrict__ noff) {
  const u64 s = gid();
  if (s >= A.nkeys) return;
  const u32 k = A.dptr[s];
  KeyInfo I;
  I.shift = noff[s] - A.off[s];
  I.keep_end = A.off[s] + A.keep_a[s];
  I.blo = k == kNone ? 0 : A.doff[k];
  I.bhi = k == kNone ? 0 : A.doff[k + 1];
  I.scan_lo = A.scan_b[I.blo];
  I.pad = 0;
  A.info[s] = I;
}

__global__ __launch_bounds__(kThreads) void k_tlog_scatter_a(TlogArgs A, const u64* __restrict__ noff,
                                                             u64* __restrict__ ots, u64* __restrict__ opre,
                                                             u64* __restrict__ olr, u32* __restrict__ oseg) {
  const u64 i = gid();
  if (i >= A.na) return;
  const u32 s = A.seg[i];
  const KeyInfo I = A.info[s];
  if (i >= I.keep_end) return;
  const Ent x{A.ts[i], A.pre[i], A.lr[i]};
  u64 pos = i + I.shift;
  if (I.bhi > I.blo) pos += A.scan_b[lower_bound_entry(A.dts, A.dpre, A.dlr, I.blo, I.bhi, x, A.arena)] - I.scan_lo;
  (void)noff;
  ots[pos] = x.t;
  opre[pos] = x.p;
  olr[pos] = x.l;
  oseg[pos] = (u32)s;
}

__global__ __launch_bounds__(kThreads) void k_tlog_scatter_b(TlogArgs A, const u64* __restrict__ noff,
                                                             u64* __restrict__ ots, u64* __restrict__ opre,
                                                             u64* __restrict__ olr, u32* __restrict__ oseg) {
  const u64 j = gid();
  if (j >= A.nb || !A.flag_b[j]) return;
  const u32 k = A.dseg[j];
  const u64 s = A.slot[k];
  const Ent x{A.dts[j], A.dpre[j], A.dlr[j]};
  const u64 lo = A.off[s];
  // state entries ordered before x all survive the cutoff (x itself does)
  const u64 p = lower_bound_entry(A.ts, A.pre, A.lr, lo, A.off[s + 1], x, A.arena);
  const u64 pos = noff[s] + (A.scan_b[j] - A.scan_b[A.doff[k]]) + (p - lo);
  ots[pos] = x.t;
  opre[pos] = x.p;
  olr[pos] = x.l;
  oseg[pos] = (u32)s;
}

__global__ __launch_bounds__(kThreads) void k_tlog_cut_store(TlogArgs A) {
  const u64 k = gid();
  if (k >= A.nd || A.bad[k]) return;
  A.cutoff[A.slot[k]] = A.cut[k];
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

__global__ __launch_bounds__(kThreads) void k_tlog_gather(const u64* __restrict__ off, const u64* __restrict__ ts,
                                                          const u64* __restrict__ pre, const u64* __restrict__ lr,
                                                          const u32* __restrict__ slots, const u64* __restrict__ ooff,
                                                          u64 n, u64* __restrict__ ots, u64* __restrict__ opre,
                                                          u64* __restrict__ olr) {
  const u64 i = gid();
  if (i >= n) return;
  const u64 s = slots[i];
  u64 o = ooff[i];
  for (u64 j = off[s]; j < off[s + 1]; j++, o++) {
    ots[o] = ts[j];
    opre[o] = pre[j];
    olr[o] = lr[j];
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
  if (need <= t.ecap[buf] && t.ts[buf]) return JY_OK;
  const u64 nc = std::max<u64>(std::max<u64>(need + need / 2, eng->cfg.entry_capacity[JY_TLOG]), 1024);
  for (u64** p : {&t.ts[buf], &t.pre[buf], &t.lr[buf]}) JY_TRY(realloc_dead(eng, reinterpret_cast<void**>(p), nc * 8));
  JY_TRY(realloc_dead(eng, reinterpret_cast<void**>(&t.seg[buf]), nc * 4));
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
  A.ts = t.ts[cur];
  A.pre = t.pre[cur];
  A.lr = t.lr[cur];
  A.seg = t.seg[cur];
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
  JY_TRY(jy_scratch(eng, 9, nd * 12, &p));
  A.cut = static_cast<u64*>(p);
  A.bad = reinterpret_cast<u32*>(A.cut + nd);
  JY_TRY(jy_scratch(eng, 11, nk * 8, &p));
  A.keep_a = static_cast<u64*>(p);
  JY_TRY(jy_scratch(eng, 12, (nent + 1) * 16, &p));
  A.flag_b = static_cast<u64*>(p);
  A.scan_b = A.flag_b + nent + 1;
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
  LAUNCH(k_tlog_drop_bad, nd, A, reinterpret_cast<unsigned long long*>(eng->skipped_dev));
  LAUNCH(k_tlog_flag_b, nent + 1, A);
  JY_TRY(jy_scan_u64(eng, A.flag_b, A.scan_b, nent));
  LAUNCH(k_tlog_sizes_out, nk + 1, A, cnt);
  JY_TRY(jy_scan_u64(eng, cnt, t.off[nxt], nk));
  LAUNCH(k_tlog_info, nk, A, t.off[nxt]);
  if (na) LAUNCH(k_tlog_scatter_a, na, A, t.off[nxt], t.ts[nxt], t.pre[nxt], t.lr[nxt], t.seg[nxt]);
  if (nent) LAUNCH(k_tlog_scatter_b, nent, A, t.off[nxt], t.ts[nxt], t.pre[nxt], t.lr[nxt], t.seg[nxt]);
  LAUNCH(k_tlog_cut_store, nd, A);
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
  LAUNCH(k_tlog_gather, n, t.off[c], t.ts[c], t.pre[c], t.lr[c], slots, ooff, n, ts, pre, lr);
  return JY_OK;
}
