// jy_scan.hpp -- wave / workgroup scans and single-pass decoupled look-back
// scans for gfx950 (64-wide waves).  Used by the variable-length merges
// (UJSON, TLOG) and the flush compaction; replaces the CUB-compatible
// device scans of round 1.
//
// Look-back: a launch's tiles are numbered by a ticket (one atomicAdd per
// workgroup), so a tile only ever waits for tiles whose workgroups took a
// ticket earlier and are running or done -- the wait always ends.  Each tile
// publishes its aggregate, then walks back over its predecessors' published
// words until it meets an inclusive prefix, and publishes its own inclusive
// prefix.  Status words carry the launch's epoch, so status arrays need no
// reset between launches.  Value and state share one 64-bit word, so the
// words are written and read with RELAXED agent-scope atomics: an acquire /
// release pair would invalidate L1 / write back the XCD's L2 on every word
// (measured: 0.7 us per tile, the whole scan serialised).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace jyscan {

typedef uint64_t u64;
typedef uint32_t u32;

template <typename T>
__device__ __forceinline__ T wave_incl(T x) {
  const int lane = __lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  return x;
}

// exclusive sum over the workgroup (kThreads a multiple of 64); `lds` holds
// kThreads / 64 values; every thread calls it; returns the thread's prefix
// and the workgroup total
template <int kThreads, typename T>
__device__ __forceinline__ T block_excl(T x, T* lds, T& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const T inc = wave_incl(x);
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  T off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kThreads / 64; i++) {
    const T v = lds[i];
    if (i < w) off += v;
    tot += v;
  }
  __syncthreads();
  total = tot;
  return off + inc - x;
}

// status word: epoch (22 bits) | state (2 bits: 1 aggregate, 2 inclusive) | value (40 bits)
constexpr u32 kEpochBits = 22;
constexpr u64 kValMask = (1ull << 40) - 1;
__device__ __forceinline__ u64 lb_word(u32 epoch, u32 st, u64 v) {
  return ((u64)(epoch & ((1u << kEpochBits) - 1)) << 42) | ((u64)st << 40) | (v & kValMask);
}

// one workgroup-wide ticket; `lds` is one shared u32
__device__ __forceinline__ u32 ticket(u32* counter, u32* lds) {
  if (threadIdx.x == 0) *lds = atomicAdd(counter, 1u);
  __syncthreads();
  const u32 t = *lds;
  __syncthreads();
  return t;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// exclusive prefix (< 2^40) of tile `tile` whose sum is `agg` (every thread
// calls; the first wave does the walk); `lds` is one shared u64.  The walk
// reads 64 predecessors per step, one per lane, waits until each has
// published something, and stops at the nearest inclusive prefix: with the
// predecessors' aggregates published early, a tile waits about one load.
__device__ __forceinline__ u64 lookback(u64* status, u32 tile, u32 epoch, u64 agg, u64* lds) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const u64 ep = (u64)(epoch & ((1u << kEpochBits) - 1));
    if (lane == 0)
      __hip_atomic_store(status + tile, lb_word(epoch, tile == 0 ? 2 : 1, agg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    u64 excl = 0;
    if (tile > 0) {
      long long top = (long long)tile - 1;
      for (;;) {
        const long long j = top - lane;
        u64 w;
        for (;;) {  // predecessors with lower tickets are running or done: they publish
          w = j >= 0 ? __hip_atomic_load(status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : lb_word(epoch, 2, 0);
          if ((w >> 42) == ep && ((w >> 40) & 3u) != 0) break;
          __builtin_amdgcn_s_sleep(1);
        }
        const u64 incl = __ballot(((w >> 40) & 3u) == 2);
        if (incl) {
          const int L = __ffsll((unsigned long long)incl) - 1;  // the nearest inclusive prefix
          excl += wave_sum<u64>(lane <= L ? (w & kValMask) : 0);
          break;
        }
        excl += wave_sum<u64>(w & kValMask);
        top -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(status + tile, lb_word(epoch, 2, excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) *lds = excl;
  }
  __syncthreads();
  const u64 r = *lds;
  __syncthreads();
  return r;
}

// the first wave finds the last k in [0, n] with offs[k] <= x (offs non-
// decreasing, offs[0] <= x): a 64-ary search, one dependent load per level
__device__ __forceinline__ u64 wave_last_le(const u64* offs, u64 n, u64 x) {
  const u32 lane = __lane_id();
  u64 lo = 0, hi = n;
  while (lo < hi) {
    const u64 step = (hi - lo + 63) / 64;
    const u64 c = lo + (u64)(lane + 1) * step;
    const u64 pass = __ballot(c <= hi && offs[c] <= x);  // a prefix of the lanes
    const u64 nlo = lo + (u64)__popcll(pass) * step;
    hi = nlo + step - 1 < hi ? nlo + step - 1 : hi;
    lo = nlo;
  }
  return lo;
}

}  // namespace jyscan
