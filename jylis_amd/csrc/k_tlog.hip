// k_tlog.hip -- TLOG segmented sorted-merge with cutoff trim, gfx950.
//
// Semantics (oracle/jy_oracle.cpp TLog; tlog.md:116-133, repo_tlog.pony:66-67):
//   cutoff' = max(cutoff_s, cutoff_d)
//   entries' = dedupe(state U delta) restricted to ts >= cutoff', sorted with
//              the later timestamp first, then the greater value first
//              (Pony String order); (ts, value) duplicates collapse.
//
// HBM layout: per type, CSR over slots -- off[kcap+1] (u64), entries SoA
// ts / pre / lr (u64 each, value handle as in TREG: 8-byte big-endian prefix
// + arena offset/length), cutoff[kcap].  Entries are double-buffered: a
// converge rewrites the whole CSR into the other buffer in three passes
//   1. count  : per slot, size of the merged log       (thread per slot)
//   2. scan   : exclusive prefix sum -> new offsets     (hipcub)
//   3. write  : per slot, merge into the new buffer     (thread per slot)
// Slots without a delta in the batch are copied.  Delta segments must be
// canonical (strictly descending); a malformed segment leaves its key
// untouched and is counted in jy_skipped (the reference swallows converge
// errors, repo_tlog.pony:67).
//
// Roofline: HBM.  Per batch: 24 B read per input entry (state + delta;
// count pass re-reads 8 B ts per entry), 24 B written per output entry,
// plus 8 B offset + 8 B cutoff read/write per slot.

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr u32 kNone = 0xFFFFFFFFu;

struct Seg {  // a view of one sorted log
  const u64* ts;
  const u64* pre;
  const u64* lr;
  u64 lo, hi;
};

// > 0 if entry (ta, pa, la) sorts before (tb, pb, lb)
__device__ __forceinline__ int entry_cmp(u64 ta, u64 pa, u64 la, u64 tb, u64 pb, u64 lb,
                                         const uint8_t* __restrict__ arena) {
  if (ta != tb) return ta > tb ? 1 : -1;
  return jy_value_cmp(pa, la, pb, lb, arena);
}

__device__ __forceinline__ bool seg_canonical(const Seg& s, const uint8_t* __restrict__ arena) {
  for (u64 j = s.lo + 1; j < s.hi; j++)
    if (entry_cmp(s.ts[j - 1], s.pre[j - 1], s.lr[j - 1], s.ts[j], s.pre[j], s.lr[j], arena) <= 0) return false;
  return true;
}

// drop the tail below the cutoff (entries are in non-increasing ts order)
__device__ __forceinline__ void seg_cut(Seg& s, u64 c) {
  while (s.hi > s.lo && s.ts[s.hi - 1] < c) s.hi--;
}

// Merge two canonical logs; emit(ts, pre, lr) for each output entry in order.
template <class Emit>
__device__ __forceinline__ void merge_logs(Seg a, Seg b, const uint8_t* __restrict__ arena, Emit emit) {
  u64 i = a.lo, j = b.lo;
  while (i < a.hi && j < b.hi) {
    const u64 ta = a.ts[i], tb = b.ts[j];
    int c;
    if (ta != tb) {
      c = ta > tb ? 1 : -1;
    } else {
      c = jy_value_cmp(a.pre[i], a.lr[i], b.pre[j], b.lr[j], arena);
    }
    if (c > 0) {
      emit(ta, a.pre[i], a.lr[i]);
      i++;
    } else if (c < 0) {
      emit(tb, b.pre[j], b.lr[j]);
      j++;
    } else {  // (ts, value) duplicate: keep the state's copy
      emit(ta, a.pre[i], a.lr[i]);
      i++;
      j++;
    }
  }
  for (; i < a.hi; i++) emit(a.ts[i], a.pre[i], a.lr[i]);
  for (; j < b.hi; j++) emit(b.ts[j], b.pre[j], b.lr[j]);
}

__global__ __launch_bounds__(kThreads) void k_scatter_ptr(u32* __restrict__ dptr, const u32* __restrict__ slot, u64 n) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) dptr[slot[i]] = (u32)i;
}

struct TlogArgs {
  // state (current buffer)
  const u64* off;
  const u64* ts;
  const u64* pre;
  const u64* lr;
  u64* cutoff;
  // delta batch
  const u32* dptr;
  const u64* dcut;
  const u64* doff;
  const u64* dts;
  const u64* dpre;
  const u64* dlr;
  const uint8_t* arena;
  u64 nkeys;
};

// resolve slot s: its state segment, its delta segment (if any, canonical),
// and the merged cutoff.  Returns false for "copy unchanged".
__device__ __forceinline__ bool tlog_resolve(const TlogArgs& A, u64 s, Seg& a, Seg& b, u64& c, bool& bad) {
  a = Seg{A.ts, A.pre, A.lr, A.off[s], A.off[s + 1]};
  bad = false;
  const u32 i = A.dptr[s];
  if (i == kNone) return false;
  b = Seg{A.dts, A.dpre, A.dlr, A.doff[i], A.doff[i + 1]};
  if (!seg_canonical(b, A.arena)) {
    bad = true;
    return false;
  }
  const u64 cs = A.cutoff[s], cd = A.dcut[i];
  c = cs > cd ? cs : cd;
  seg_cut(a, c);
  seg_cut(b, c);
  return true;
}

__global__ __launch_bounds__(kThreads) void k_tlog_count(TlogArgs A, u64* __restrict__ cnt,
                                                         unsigned long long* __restrict__ skipped) {
  const u64 s = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (s > A.nkeys) return;
  if (s == A.nkeys) {
    cnt[s] = 0;
    return;
  }
  Seg a, b;
  u64 c;
  bool bad;
  if (!tlog_resolve(A, s, a, b, c, bad)) {
    cnt[s] = a.hi - a.lo;
    if (bad) atomicAdd(skipped, 1ull);
    return;
  }
  u64 n = 0;
  merge_logs(a, b, A.arena, [&](u64, u64, u64) { n++; });
  cnt[s] = n;
}

__global__ __launch_bounds__(kThreads) void k_tlog_write(TlogArgs A, const u64* __restrict__ noff,
                                                         u64* __restrict__ ots, u64* __restrict__ opre,
                                                         u64* __restrict__ olr) {
  const u64 s = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (s >= A.nkeys) return;
  Seg a, b;
  u64 c;
  bool bad;
  u64 o = noff[s];
  if (!tlog_resolve(A, s, a, b, c, bad)) {
    for (u64 j = a.lo; j < a.hi; j++, o++) {
      ots[o] = a.ts[j];
      opre[o] = a.pre[j];
      olr[o] = a.lr[j];
    }
    return;
  }
  merge_logs(a, b, A.arena, [&](u64 t, u64 p, u64 l) {
    ots[o] = t;
    opre[o] = p;
    olr[o] = l;
    o++;
  });
  A.cutoff[s] = c;
}

__global__ __launch_bounds__(kThreads) void k_fill_tail(u64* __restrict__ off, u64 from, u64 to) {
  // off[from+1 .. to] = off[from]  (new, empty slots)
  const u64 i = from + 1 + (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i <= to) off[i] = off[from];
}

__global__ __launch_bounds__(kThreads) void k_tlog_sizes(const u64* __restrict__ off, const u64* __restrict__ cutoff,
                                                         const u32* __restrict__ slots, u64 n, u64* __restrict__ len,
                                                         u64* __restrict__ cut) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
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
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u64 s = slots[i];
  u64 o = ooff[i];
  for (u64 j = off[s]; j < off[s + 1]; j++, o++) {
    ots[o] = ts[j];
    opre[o] = pre[j];
    olr[o] = lr[j];
  }
}

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

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

static int32_t ensure_entries(jy_engine* eng, int buf, u64 need) {
  TlogState& t = eng->tlog;
  if (need <= t.ecap[buf] && t.ts[buf]) return JY_OK;
  u64 nc = std::max<u64>(std::max<u64>(need + need / 2, eng->cfg.entry_capacity[JY_TLOG]), 1024);
  // contents of the target buffer are dead (it is rewritten): free, then allocate
  for (u64** p : {&t.ts[buf], &t.pre[buf], &t.lr[buf]}) {
    if (*p) {
      JY_HIP(eng, hipStreamSynchronize(eng->stream));
      JY_HIP(eng, hipFree(*p));
      *p = nullptr;
    }
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), nc * 8);
    if (e != hipSuccess) return eng->fail(JY_ENOMEM, std::string("tlog entries: ") + hipGetErrorString(e));
  }
  t.ecap[buf] = nc;
  return JY_OK;
}

int32_t jy_tlog_grow(jy_engine* eng, u64 need) {
  TlogState& t = eng->tlog;
  if (need <= t.kcap && t.cutoff) return JY_OK;
  u64 nk = std::max<u64>(need, t.kcap ? t.kcap * 2 : need);
  nk = std::max<u64>((nk + 63) & ~63ull, 64);
  const u64 live = eng->nkeys[JY_TLOG];
  void* c = t.cutoff;
  JY_TRY(jy_realloc(eng, &c, t.kcap * 8, nk * 8, true));
  t.cutoff = static_cast<u64*>(c);
  for (int b = 0; b < 2; b++) {
    void* o = t.off[b];
    JY_TRY(jy_realloc(eng, &o, t.kcap ? (t.kcap + 1) * 8 : 0, (nk + 1) * 8, true));
    t.off[b] = static_cast<u64*>(o);
  }
  (void)live;
  t.kcap = nk;
  for (int b = 0; b < 2; b++) JY_TRY(ensure_entries(eng, b, 1));
  return JY_OK;
}

// new slots [from, to) start as empty logs: off[from+1..to] = off[from]
int32_t jy_tlog_extend(jy_engine* eng, u64 from, u64 to) {
  if (to <= from) return JY_OK;
  TlogState& t = eng->tlog;
  hipLaunchKernelGGL(k_fill_tail, dim3(blocks_for(to - from)), dim3(kThreads), 0, eng->stream, t.off[t.cur], from,
                     to);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_tlog_merge(jy_engine* eng, u64 nd, const u32* slot, const u64* dcut, const u64* doff, u64 nent,
                      const u64* dts, const u64* dpre, const u64* dlr) {
  TlogState& t = eng->tlog;
  const u64 nk = eng->nkeys[JY_TLOG];
  if (nd == 0 || nk == 0) return JY_OK;
  // live entry count of the current buffer: the previous merge's total
  JY_HIP(eng, hipEventSynchronize(eng->total_ready));
  const u64 live = t.nent_known ? eng->pin_total[0] : t.nent_bound;
  const int cur = t.cur, nxt = 1 - cur;
  JY_TRY(ensure_entries(eng, nxt, live + nent));

  void *dptr, *cnt;
  JY_TRY(jy_scratch(eng, 8, nk * 4, &dptr));
  JY_TRY(jy_scratch(eng, 9, (nk + 1) * 8, &cnt));
  JY_HIP(eng, hipMemsetAsync(dptr, 0xFF, nk * 4, eng->stream));
  hipLaunchKernelGGL(k_scatter_ptr, dim3(blocks_for(nd)), dim3(kThreads), 0, eng->stream, static_cast<u32*>(dptr),
                     slot, nd);
  TlogArgs A{t.off[cur], t.ts[cur], t.pre[cur], t.lr[cur], t.cutoff, static_cast<const u32*>(dptr), dcut, doff,
             dts, dpre, dlr, eng->arena[JY_TLOG].p, nk};
  hipLaunchKernelGGL(k_tlog_count, dim3(blocks_for(nk + 1)), dim3(kThreads), 0, eng->stream, A,
                     static_cast<u64*>(cnt), reinterpret_cast<unsigned long long*>(eng->skipped_dev));
  JY_HIP(eng, hipGetLastError());
  JY_TRY(jy_scan_u64(eng, static_cast<const u64*>(cnt), t.off[nxt], nk));
  hipLaunchKernelGGL(k_tlog_write, dim3(blocks_for(nk)), dim3(kThreads), 0, eng->stream, A, t.off[nxt], t.ts[nxt],
                     t.pre[nxt], t.lr[nxt]);
  JY_HIP(eng, hipGetLastError());
  // publish the new total for the next call (read back asynchronously)
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, t.off[nxt] + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipEventRecord(eng->total_ready, eng->stream));
  t.nent_known = true;
  t.nent_bound = live + nent;
  t.cur = nxt;
  return JY_OK;
}

int32_t jy_tlog_sizes(jy_engine* eng, u64 n, const u32* slots, u64* len, u64* cut) {
  TlogState& t = eng->tlog;
  hipLaunchKernelGGL(k_tlog_sizes, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, t.off[t.cur], t.cutoff,
                     slots, n, len, cut);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_tlog_gather(jy_engine* eng, u64 n, const u32* slots, const u64* ooff, u64* ts, u64* pre, u64* lr) {
  TlogState& t = eng->tlog;
  const int c = t.cur;
  hipLaunchKernelGGL(k_tlog_gather, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, t.off[c], t.ts[c],
                     t.pre[c], t.lr[c], slots, ooff, n, ts, pre, lr);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}
