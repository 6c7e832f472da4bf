// jy_dscan.hpp -- device-wide scans and selects for the engine (gfx950): one
// launch each, a single pass with a decoupled look-back over ticketed tiles
// (jy_scan.hpp).  Replaces the CUB-compatible DeviceScan / DeviceSelect of
// round 1 on the product path (flush, key interning, log compaction, segment
// ids).
//
// Status words are epoch-tagged (no reset between launches); the ticket
// counter is reset by the workgroup that draws the launch's last ticket (every
// other ticket is drawn by then).  Each launch takes a fresh epoch from the
// engine (jy_dscan_ctx).
#pragma once

#include "jy_internal.hpp"
#include "jy_scan.hpp"

namespace jydscan {

constexpr int kThreads = 256;
constexpr int kPer = 8;
constexpr u64 kTileItems = (u64)kThreads * kPer;  // 2048 items per tile

struct Ctx {
  u64* status;
  u32* tick;
  u32 epoch;
};

struct OpSum {
  __device__ __forceinline__ u64 operator()(u64 a, u64 b) const { return a + b; }
  static constexpr u64 kId = 0;
};
struct OpMax {
  __device__ __forceinline__ u64 operator()(u64 a, u64 b) const { return a > b ? a : b; }
  static constexpr u64 kId = 0;
};

template <class Op>
__device__ __forceinline__ u64 wave_reduce(u64 x) {
  Op op;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = op(x, __shfl_xor(x, o));
  return x;
}
template <class Op>
__device__ __forceinline__ u64 wave_incl(u64 x) {
  Op op;
  const int lane = __lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u64 y = __shfl_up(x, o);
    if (lane >= o) x = op(x, y);
  }
  return x;
}
// exclusive scan over the workgroup (identity for thread 0) and the total
template <class Op>
__device__ __forceinline__ u64 block_excl(u64 x, u64* lds, u64& total) {
  Op op;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const u64 inc = wave_incl<Op>(x);
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  u64 off = Op::kId, tot = Op::kId;
#pragma unroll
  for (int i = 0; i < kThreads / 64; i++) {
    const u64 v = lds[i];
    if (i < w) off = op(off, v);
    tot = op(tot, v);
  }
  __syncthreads();
  total = tot;
  const u64 ex = __shfl_up(inc, 1);
  return op(off, lane == 0 ? Op::kId : ex);
}

// sum over the workgroup (every thread calls; every thread gets it)
__device__ __forceinline__ u64 block_total(u64 x, u64* lds) {
  u64 tot;
  block_excl<OpSum>(x, lds, tot);
  return tot;
}

// the look-back of jy_scan.hpp, generic over the operator (values < 2^40)
template <class Op>
__device__ __forceinline__ u64 lookback(const Ctx& c, u32 tile, u64 agg, u64* lds) {
  using namespace jyscan;
  Op op;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const u64 ep = (u64)(c.epoch & ((1u << kEpochBits) - 1));
    if (lane == 0)
      __hip_atomic_store(c.status + tile, lb_word(c.epoch, tile == 0 ? 2 : 1, agg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    u64 excl = Op::kId;
    if (tile > 0) {
      long long top = (long long)tile - 1;
      for (;;) {
        const long long j = top - lane;
        u64 w;
        for (;;) {
          w = j >= 0 ? __hip_atomic_load(c.status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : lb_word(c.epoch, 2, Op::kId);
          if ((w >> 42) == ep && ((w >> 40) & 3u) != 0) break;
          __builtin_amdgcn_s_sleep(1);
        }
        const u64 incl = __ballot(((w >> 40) & 3u) == 2);
        if (incl) {
          const int L = __ffsll((unsigned long long)incl) - 1;
          excl = op(excl, wave_reduce<Op>(lane <= L ? (w & kValMask) : Op::kId));
          break;
        }
        excl = op(excl, wave_reduce<Op>(w & kValMask));
        top -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(c.status + tile, lb_word(c.epoch, 2, op(excl, agg)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) *lds = excl;
  }
  __syncthreads();
  const u64 r = *lds;
  __syncthreads();
  return r;
}

// (k_select) Tiles of kTileItems items; a workgroup takes ONE ticket for G consecutive
// tiles (G = 1 up to kMaxTickets tiles): a ticket is a same-address atomic,
// and those serialise at ~11 ns each (tools/mb_ticket.hip: 4096 tickets
// 48 us, 32768 tickets 373 us), so an 8M-item scan spent half its time
// drawing them.  With G > 1 the workgroup first reduces its G tiles (its
// look-back aggregate), then scans them again from the top (the re-read is
// its own recent loads, mostly still in the caches).
// (Round 4 tried the reduce sweep with four tiles' loads in flight and the
// rescan loading tile s + 1 before tile s's block scan: in-box A/B of the
// key-resolving TREG step, 2 runs each, and the TLOG step -- no difference.)
constexpr u64 kMaxTickets = 1024;

// indices i < n with pred(i), in order, into out; the count into *count
template <class Pred>
__global__ __launch_bounds__(kThreads) void k_select(Ctx c, u64 n, u64 ntiles, u64 G, Pred pred,
                                                     u32* __restrict__ out, u32* __restrict__ count) {
  __shared__ u64 red[kThreads / 64];
  __shared__ u64 pre;
  __shared__ u32 tk;
  const u32 t = jyscan::ticket(c.tick, &tk);
  if (t == gridDim.x - 1 && threadIdx.x == 0) *c.tick = 0;
  const u64 s0 = (u64)t * G, s1 = s0 + G < ntiles ? s0 + G : ntiles;
  u64 agg = 0;  // several tiles: their count first (the look-back aggregate)
  if (s1 - s0 > 1) {
    u64 acc = 0;
    for (u64 s = s0; s < s1; s++) {
      const u64 i0 = s * kTileItems + (u64)threadIdx.x * kPer;
#pragma unroll
      for (int u = 0; u < kPer; u++) acc += i0 + u < n && pred(i0 + u);
    }
    agg = block_total(acc, red);
  }
  u64 base = 0;
  for (u64 s = s0; s < s1; s++) {
    const u64 i0 = s * kTileItems + (u64)threadIdx.x * kPer;
    u32 f = 0;
    u64 a = 0;
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const bool sel = i0 + u < n && pred(i0 + u);
      f |= (u32)sel << u;
      a += sel;
    }
    u64 ts;
    const u64 off = block_excl<OpSum>(a, red, ts);
    if (s == s0) base = lookback<OpSum>(c, t, s1 - s0 > 1 ? agg : ts, &pre);
    u64 pos = base + off;
#pragma unroll
    for (int u = 0; u < kPer; u++)
      if (f >> u & 1) out[pos++] = (u32)(i0 + u);
    base += ts;
  }
  if (t == gridDim.x - 1 && threadIdx.x == 0) *count = (u32)base;
}

inline u64 tiles_of(u64 n) { return n == 0 ? 1 : (n + kTileItems - 1) / kTileItems; }

// tiles per workgroup (one ticket each workgroup) and the workgroups
inline u64 group_of(u64 nt) { return (nt + kMaxTickets - 1) / kMaxTickets; }

// ---- reduce-then-scan (round 5): three launches, no look-back, no tickets.
// A tile is kRows rows of kThreads items; lane t of a row holds item
// row * kThreads + t, so every load and store is coalesced (the look-back
// form above gave each thread 8 consecutive items: 64-B lane strides).  A
// chunk is T consecutive tiles, at most kMaxChunks chunks per scan:
//   k_scan_part   each chunk's reduction           (reads the input once)
//   k_scan_mid    one workgroup: exclusive scan of the chunk totals
//   k_scan_down   each chunk scanned from its base (reads it again: mostly
//                 the caches' -- a chunk is 4-64 KB, read moments before)
// The look-back scan of an 8M-item u64 column took 80-97 us on MI355X (node
// TREG trace, round 5): one ticket per workgroup, 1024 workgroups of 4 tiles,
// strided lanes.  Values are full 64-bit (no 40-bit look-back words).
constexpr int kRows = kPer;
constexpr u64 kMaxChunks = kThreads * kRows;  // k_scan_mid scans them as one tile

// one tile's rows, scanned in place: x[u] (row u's item of this lane) becomes
// its exclusive (or inclusive) prefix from `carry`; returns the tile total
template <class Op, bool kIncl>
__device__ __forceinline__ u64 tile_rows(u64 (&x)[kRows], u64 carry, u64 (*wt)[kThreads / 64]) {
  Op op;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  u64 inc[kRows];
#pragma unroll
  for (int u = 0; u < kRows; u++) {
    inc[u] = wave_incl<Op>(x[u]);
    if (lane == 63) wt[u][w] = inc[u];
  }
  __syncthreads();
  u64 base = carry;
#pragma unroll
  for (int u = 0; u < kRows; u++) {
    u64 off = base, row = Op::kId;
#pragma unroll
    for (int q = 0; q < kThreads / 64; q++) {
      const u64 v = wt[u][q];
      if (q < w) off = op(off, v);
      row = op(row, v);
    }
    const u64 ex = __shfl_up(inc[u], 1);
    x[u] = kIncl ? op(off, inc[u]) : op(off, lane == 0 ? Op::kId : ex);
    base = op(base, row);
  }
  __syncthreads();  // wt is reused by the next tile
  return base;
}

template <class Op, class Ld>
__global__ __launch_bounds__(kThreads) void k_scan_part(u64 n, u64 T, Ld ld, u64* __restrict__ part) {
  __shared__ u64 red[kThreads / 64];
  Op op;
  const u64 i0 = (u64)blockIdx.x * T * kTileItems;
  const u64 i1 = i0 + T * kTileItems < n ? i0 + T * kTileItems : n;
  u64 acc = Op::kId;
  for (u64 b = i0; b < i1; b += kTileItems) {
    u64 v[kRows];
#pragma unroll
    for (int u = 0; u < kRows; u++) {
      const u64 i = b + (u64)u * kThreads + threadIdx.x;
      v[u] = i < i1 ? ld(i) : Op::kId;
    }
#pragma unroll
    for (int u = 0; u < kRows; u++) acc = op(acc, v[u]);
  }
  acc = wave_reduce<Op>(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 t = Op::kId;
#pragma unroll
    for (int q = 0; q < kThreads / 64; q++) t = op(t, red[q]);
    part[blockIdx.x] = t;
  }
}

// the nc chunk totals -> their exclusive prefixes (in place; part[nc] = all)
template <class Op>
__global__ __launch_bounds__(kThreads) void k_scan_mid(u64 nc, u64* __restrict__ part) {
  __shared__ u64 wt[kRows][kThreads / 64];
  u64 x[kRows];
#pragma unroll
  for (int u = 0; u < kRows; u++) {
    const u64 i = (u64)u * kThreads + threadIdx.x;
    x[u] = i < nc ? part[i] : Op::kId;
  }
  const u64 tot = tile_rows<Op, false>(x, Op::kId, wt);
#pragma unroll
  for (int u = 0; u < kRows; u++) {
    const u64 i = (u64)u * kThreads + threadIdx.x;
    if (i < nc) part[i] = x[u];
  }
  if (threadIdx.x == 0) part[nc] = tot;
}

// chunk blockIdx.x scanned from part[blockIdx.x] (nullptr: from the identity,
// the one-workgroup form of a small scan)
template <class Op, bool kIncl, class Ld, class St>
__global__ __launch_bounds__(kThreads) void k_scan_down(u64 n, u64 T, Ld ld, St st, const u64* __restrict__ part) {
  __shared__ u64 wt[kRows][kThreads / 64];
  const u64 i0 = (u64)blockIdx.x * T * kTileItems;
  const u64 i1 = i0 + T * kTileItems < n ? i0 + T * kTileItems : n;
  u64 carry = part ? part[blockIdx.x] : Op::kId;
  for (u64 b = i0; b < i1; b += kTileItems) {
    u64 x[kRows];
#pragma unroll
    for (int u = 0; u < kRows; u++) {
      const u64 i = b + (u64)u * kThreads + threadIdx.x;
      x[u] = i < i1 ? ld(i) : Op::kId;
    }
    carry = tile_rows<Op, kIncl>(x, carry, wt);
#pragma unroll
    for (int u = 0; u < kRows; u++) {
      const u64 i = b + (u64)u * kThreads + threadIdx.x;
      if (i < i1) st(i, x[u]);
    }
  }
}

// small scans stay in one workgroup (one launch): up to this many tiles
constexpr u64 kOneGroupTiles = 8;

// a scan over n items: ld(i) -> u64, st(i, prefix).  In place (st writing
// what ld reads) is allowed: every item is read before it is written.
template <class Op, bool kIncl, class Ld, class St>
int32_t scan(jy_engine* eng, u64 n, Ld ld, St st) {
  if (n == 0) return JY_OK;
  const u64 nt = tiles_of(n);
  if (nt <= kOneGroupTiles) {
    hipLaunchKernelGGL((k_scan_down<Op, kIncl, Ld, St>), dim3(1), dim3(kThreads), 0, eng->stream, n, nt, ld, st,
                       (const u64*)nullptr);
    JY_HIP(eng, hipGetLastError());
    return JY_OK;
  }
  const u64 T = (nt + kMaxChunks - 1) / kMaxChunks, nc = (nt + T - 1) / T;
  void* p;
  JY_TRY(jy_scratch(eng, 31, (nc + 1) * 8, &p));
  u64* part = static_cast<u64*>(p);
  hipLaunchKernelGGL((k_scan_part<Op, Ld>), dim3((u32)nc), dim3(kThreads), 0, eng->stream, n, T, ld, part);
  hipLaunchKernelGGL((k_scan_mid<Op>), dim3(1), dim3(kThreads), 0, eng->stream, nc, part);
  hipLaunchKernelGGL((k_scan_down<Op, kIncl, Ld, St>), dim3((u32)nc), dim3(kThreads), 0, eng->stream, n, T, ld, st,
                     (const u64*)part);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}
template <class Pred>
int32_t select(jy_engine* eng, u64 n, Pred pred, u32* out, u32* count) {
  const u64 nt = tiles_of(n), G = group_of(nt), nwg = (nt + G - 1) / G;
  Ctx c;
  JY_TRY(jy_dscan_ctx(eng, nwg, &c.status, &c.tick, &c.epoch));
  hipLaunchKernelGGL((k_select<Pred>), dim3((u32)nwg), dim3(kThreads), 0, eng->stream, c, n, nt, G, pred, out,
                     count);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

// loaders / storers
template <class T>
struct LdArr {
  const T* a;
  __device__ __forceinline__ u64 operator()(u64 i) const { return (u64)a[i]; }
};
template <class T>
struct StArr {
  T* a;
  __device__ __forceinline__ void operator()(u64 i, u64 v) const { a[i] = (T)v; }
};

// a row-major [rows][W] matrix scanned column after column (column c's rows
// are contiguous in the scan order); scan index rows * W is one extra word
// after the matrix (the grand total of an exclusive scan)
struct LdColMajor {
  const u64* a;
  u64 rows, W;
  __device__ __forceinline__ u64 operator()(u64 f) const {
    if (f >= rows * W) return 0;
    const u64 c = f / rows;
    return a[(f - c * rows) * W + c];
  }
};
struct StColMajor {
  u64* a;
  u64 rows, W;
  __device__ __forceinline__ void operator()(u64 f, u64 v) const {
    if (f >= rows * W) {
      a[rows * W] = v;
      return;
    }
    const u64 c = f / rows;
    a[(f - c * rows) * W + c] = v;
  }
};

}  // namespace jydscan
