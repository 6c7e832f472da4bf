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
// + arena offset/length); cutoff[kcap].  Entries are double-buffered: a
// converge rewrites the CSR into the other buffer.
//
// Parallel shape: a workgroup owns a tile of kTile consecutive slots (one
// lane per slot).  The tile's state entries are one contiguous CSR range:
// the workgroup stages it into LDS with coalesced loads, then every lane
// merges its own log out of LDS against its delta segment (short, read from
// HBM) and streams the result to the new CSR.  Two passes -- count (ts only,
// value bytes on ties) and write -- around a scan of per-slot sizes.  A tile
// whose state range exceeds the LDS budget reads HBM directly (same code).
// Logs are short (state ~Geom(8) capped at 64, deltas ~Geom(2): SURVEY 8d
// config 4), so lanes stay balanced; unbounded skew is UJSON's problem
// (per-element design there).
//
// A delta segment that is not strictly ordered is not a TLog: its key is
// left untouched and counted (the reference swallows converge errors,
// repo_tlog.pony:67).
//
// Roofline: HBM.  Count pass 8 B per input entry; write pass 24 B per input
// entry + 24 B per output entry; per slot 8 B offsets in + 8 B out + 16 B
// cutoff.

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "jy_internal.hpp"

namespace {

constexpr int kTile = 128;      // slots (lanes) per workgroup
constexpr u32 kStage = 2048;    // state entries staged in LDS per tile (48 KiB)
constexpr u32 kNone = 0xFFFFFFFFu;

__device__ __forceinline__ int entry_cmp(u64 ta, u64 pa, u64 la, u64 tb, u64 pb, u64 lb,
                                         const uint8_t* __restrict__ arena) {
  if (ta != tb) return ta > tb ? 1 : -1;
  return jy_value_cmp(pa, la, pb, lb, arena);
}

struct TlogArgs {
  // state (current buffer)
  const u64* off;
  const u64* ts;
  const u64* pre;
  const u64* lr;
  u64* cutoff;
  u64 nkeys;
  // delta batch
  u64 nd;
  const u32* slot;
  const u32* dptr;
  const u64* dcut;
  const u64* doff;
  const u64* dts;
  const u64* dpre;
  const u64* dlr;
  const uint8_t* arena;
  u32* bad;  // [nd] malformed delta segment (set by the count pass)
};

__global__ __launch_bounds__(256) void k_scatter_ptr(u32* __restrict__ dptr, const u32* __restrict__ slot, u64 n) {
  const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dptr[slot[i]] = (u32)i;
}

// kWrite = false: count pass (cnt[s]); true: write pass (entries + cutoff)
template <bool kWrite>
__global__ __launch_bounds__(kTile) void k_tlog_tile(TlogArgs A, u64* __restrict__ cnt, const u64* __restrict__ noff,
                                                     u64* __restrict__ ots, u64* __restrict__ opre,
                                                     u64* __restrict__ olr, unsigned long long* __restrict__ skipped) {
  __shared__ u64 sts[kStage];
  __shared__ u64 spre[kWrite ? kStage : 1];
  __shared__ u64 slr[kWrite ? kStage : 1];
  const u64 s0 = (u64)blockIdx.x * kTile;
  const u64 s = s0 + threadIdx.x;
  const u64 s1 = min(s0 + (u64)kTile, A.nkeys);
  const u64 a0 = A.off[s0], a1 = A.off[s1];
  const bool staged = (a1 - a0) <= kStage;
  if (staged) {
    for (u64 j = threadIdx.x; j < a1 - a0; j += kTile) {
      sts[j] = A.ts[a0 + j];
      if (kWrite) {
        spre[j] = A.pre[a0 + j];
        slr[j] = A.lr[a0 + j];
      }
    }
  }
  __syncthreads();
  if (!kWrite && s == A.nkeys) cnt[s] = 0;  // scan sentinel
  if (s >= A.nkeys) return;
  // this lane's state log: LDS when staged, else HBM
  const u64 lo = A.off[s], hi0 = A.off[s + 1];
  const u64* ta = staged ? sts + (lo - a0) : A.ts + lo;
  const u64* pa = kWrite ? (staged ? spre + (lo - a0) : A.pre + lo) : A.pre + lo;
  const u64* la = kWrite ? (staged ? slr + (lo - a0) : A.lr + lo) : A.lr + lo;
  u64 na = hi0 - lo;
  const u32 k = A.dptr[s];
  u64 b = 0, nb = 0, c = A.cutoff[s];
  bool merge = false;
  if (k != kNone) {
    b = A.doff[k];
    nb = A.doff[k + 1] - b;
    if (!kWrite) {
      bool ok = true;
      for (u64 j = 1; j < nb && ok; j++)
        ok = entry_cmp(A.dts[b + j - 1], A.dpre[b + j - 1], A.dlr[b + j - 1], A.dts[b + j], A.dpre[b + j],
                       A.dlr[b + j], A.arena) > 0;
      if (!ok) {
        A.bad[k] = 1;
        atomicAdd(skipped, 1ull);
      }
      merge = ok;
    } else {
      merge = !A.bad[k];
    }
  }
  if (merge) {
    const u64 cd = A.dcut[k];
    c = c > cd ? c : cd;
    while (na > 0 && ta[na - 1] < c) na--;  // the cutoff drops a suffix
    while (nb > 0 && A.dts[b + nb - 1] < c) nb--;
  } else {
    nb = 0;
  }
  u64 o = kWrite ? noff[s] : 0;
  u64 n = 0;
  u64 i = 0, j = 0;
  while (i < na || j < nb) {
    int cmp;
    if (j >= nb) cmp = 1;
    else if (i >= na) cmp = -1;
    else {
      const u64 x = ta[i], y = A.dts[b + j];
      cmp = x != y ? (x > y ? 1 : -1) : jy_value_cmp(pa[i], la[i], A.dpre[b + j], A.dlr[b + j], A.arena);
    }
    if (kWrite) {
      if (cmp >= 0) {
        ots[o] = ta[i];
        opre[o] = pa[i];
        olr[o] = la[i];
      } else {
        ots[o] = A.dts[b + j];
        opre[o] = A.dpre[b + j];
        olr[o] = A.dlr[b + j];
      }
      o++;
    }
    n++;
    if (cmp > 0) i++;
    else if (cmp < 0) j++;
    else {  // (ts, value) duplicate: the state's copy stays
      i++;
      j++;
    }
  }
  if (!kWrite) cnt[s] = n;
  if (kWrite && merge) A.cutoff[s] = c;
}

__global__ __launch_bounds__(256) void k_fill_tail(u64* __restrict__ off, u64 from, u64 to) {
  // off[from+1 .. to] = off[from]  (new, empty slots)
  const u64 i = from + 1 + (u64)blockIdx.x * 256 + threadIdx.x;
  if (i <= to) off[i] = off[from];
}

__global__ __launch_bounds__(256) void k_tlog_sizes(const u64* __restrict__ off, const u64* __restrict__ cutoff,
                                                    const u32* __restrict__ slots, u64 n, u64* __restrict__ len,
                                                    u64* __restrict__ cut) {
  const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const u64 s = slots[i];
  len[i] = off[s + 1] - off[s];
  cut[i] = cutoff[s];
}

__global__ __launch_bounds__(256) void k_tlog_gather(const u64* __restrict__ off, const u64* __restrict__ ts,
                                                     const u64* __restrict__ pre, const u64* __restrict__ lr,
                                                     const u32* __restrict__ slots, const u64* __restrict__ ooff,
                                                     u64 n, u64* __restrict__ ots, u64* __restrict__ opre,
                                                     u64* __restrict__ olr) {
  const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const u64 s = slots[i];
  u64 o = ooff[i];
  for (u64 j = off[s]; j < off[s + 1]; j++, o++) {
    ots[o] = ts[j];
    opre[o] = pre[j];
    olr[o] = lr[j];
  }
}

__global__ __launch_bounds__(256) void k_seg_starts(const u64* __restrict__ offs, u64 nseg, u32* __restrict__ out) {
  const u64 k = (u64)blockIdx.x * 256 + threadIdx.x;
  if (k < nseg && offs[k] < offs[k + 1]) out[offs[k]] = (u32)k;
}

u32 blocks_for(u64 n, u64 per = 256) { return (u32)std::max<u64>(1, (n + per - 1) / per); }

#define LAUNCH(k, n, ...)                                                                          \
  do {                                                                                             \
    hipLaunchKernelGGL(k, dim3(blocks_for(n)), dim3(256), 0, eng->stream, __VA_ARGS__);          \
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
  t.ecap[buf] = nc;
  return JY_OK;
}

int32_t jy_tlog_grow(jy_engine* eng, u64 need) {
  TlogState& t = eng->tlog;
  if (need <= t.kcap && t.cutoff) return JY_OK;
  u64 nk = std::max<u64>(need, t.kcap ? t.kcap * 2 : need);
  nk = std::max<u64>((nk + 127) & ~127ull, 128);  // whole tiles
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
  A.cutoff = t.cutoff;
  A.nkeys = nk;
  A.nd = nd;
  A.slot = slot;
  A.dcut = dcut;
  A.doff = doff;
  A.dts = dts;
  A.dpre = dpre;
  A.dlr = dlr;
  A.arena = eng->arena[JY_TLOG].p;
  void *dptr, *bad, *cnt;
  JY_TRY(jy_scratch(eng, 8, nk * 4, &dptr));
  JY_TRY(jy_scratch(eng, 9, nd * 4, &bad));
  JY_TRY(jy_scratch(eng, 16, (nk + 1) * 8, &cnt));
  A.dptr = static_cast<const u32*>(dptr);
  A.bad = static_cast<u32*>(bad);
  JY_HIP(eng, hipMemsetAsync(dptr, 0xFF, nk * 4, eng->stream));
  JY_HIP(eng, hipMemsetAsync(bad, 0, nd * 4, eng->stream));
  LAUNCH(k_scatter_ptr, nd, static_cast<u32*>(dptr), slot, nd);
  auto* skipped = reinterpret_cast<unsigned long long*>(eng->skipped_dev);
  const u32 tiles = blocks_for(nk + 1, kTile);  // +1: the scan sentinel lane
  hipLaunchKernelGGL(k_tlog_tile<false>, dim3(tiles), dim3(kTile), 0, eng->stream, A, static_cast<u64*>(cnt),
                     (const u64*)nullptr, (u64*)nullptr, (u64*)nullptr, (u64*)nullptr, skipped);
  JY_HIP(eng, hipGetLastError());
  JY_TRY(jy_scan_u64(eng, static_cast<const u64*>(cnt), t.off[nxt], nk));
  hipLaunchKernelGGL(k_tlog_tile<true>, dim3(blocks_for(nk, kTile)), dim3(kTile), 0, eng->stream, A,
                     static_cast<u64*>(cnt), t.off[nxt], t.ts[nxt], t.pre[nxt], t.lr[nxt], skipped);
  JY_HIP(eng, hipGetLastError());
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
