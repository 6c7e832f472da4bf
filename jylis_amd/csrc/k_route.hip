// k_route.hip -- routing delta batches to owner shards (the exchange step).
//
// Keys are hash-sharded over S engines (jy_key_owner).  A peer batch that
// lands on one GPU is partitioned by owner into per-destination runs of a
// FIXED capacity, exchanged with one equal-split all-to-all (RCCL over
// xGMI; the host side drives it) together with a small header of counts,
// and each owner converges every received run in one launch, reading the
// counts from device memory -- no host round trip per batch.  Entries that
// do not fit their run are listed for a later round (jylis_amd/route.py).
// This is the intra-node analogue of Cluster.broadcast_deltas
// (jylis/cluster.pony:209-213); the reference replicates instead.
//
// TREG record: u64[4] = {slot on owner, ts, pre, lr'}, lr' = (byte offset
// inside the destination's byte run << 24 | length) for values > 8 bytes,
// whose bytes travel in a second run.
//
// Roofline: HBM.  Partition reads 4+4+24 B per entry (+ long value bytes),
// writes 32 B per record; the receiver reads 32 B per record + state.

#include <algorithm>

#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr int kPer = 8;  // entries per lane: one tile of 2048 entries per workgroup
constexpr u64 kTile = (u64)kThreads * kPer;
constexpr u32 kMaxShards = 64;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u64 round_up8(u64 x) { return (x + kArenaAlign - 1) & ~(kArenaAlign - 1); }

// Per-owner counts without same-address atomics per lane: a wave walks the
// distinct owners among its lanes (one ballot each), and its leader adds the
// wave's count and long-value bytes to the workgroup's LDS counters once.
// `rank`/`brank` (scatter only) receive each lane's position inside the
// workgroup's run for its owner.  All lanes of the wave call this together.
template <bool kRanks>
__device__ __forceinline__ void wave_aggregate(bool valid, u32 o, u32 blen, unsigned long long* lrec,
                                               unsigned long long* lbyte, u64* rank, u64* brank) {
  const int lane = __lane_id();
  const u64 lt = (1ull << lane) - 1;
  u64 pending = __ballot(valid);
  while (pending) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const u32 d = __shfl(o, leader);
    const bool mine = valid && o == d;
    const u64 m = __ballot(mine);
    // inclusive scan of the long-value bytes of this owner's lanes (a value
    // is < 2^24 bytes, so a wave's sum fits 32 bits); skipped when none is long
    u32 x = mine ? blen : 0;
    u32 bsum = 0;
    if (__ballot(x != 0)) {
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const u32 y = __shfl_up(x, off);
        if (lane >= off) x += y;
      }
      bsum = __shfl(x, 63);
    }
    unsigned long long rb = 0, bb = 0;
    if (lane == leader) {
      rb = atomicAdd(&lrec[d], (unsigned long long)__popcll(m));
      if (bsum) bb = atomicAdd(&lbyte[d], (unsigned long long)bsum);
    }
    if (kRanks) {
      rb = __shfl(rb, leader);
      bb = __shfl(bb, leader);
      if (mine) {
        *rank = rb + __popcll(m & lt);
        *brank = bb + x - blen;
      }
    }
    pending &= ~m;
  }
}

// One pass: per-owner ranks inside the workgroup (wave_aggregate), one
// global reservation per (workgroup, owner) on the header cursors, then
// every entry that fits its owner's run is written there.  An entry past
// the run's record capacity, or whose long value would pass the run's byte
// capacity, is listed in ovf (input index) -- a record slot it took is left
// as a hole (slot ~0) the receiver skips.  hdr[2d] / hdr[2d + 1] end as the
// records / bytes reserved for owner d, which may pass the capacities; the
// receiver clamps.
__global__ __launch_bounds__(kThreads) void k_route_part_treg(
    const u32* __restrict__ owner, const u32* __restrict__ slot, const u64* __restrict__ ts,
    const u64* __restrict__ pre, const u64* __restrict__ lr, const uint8_t* __restrict__ arena, u64 n, u32 S, u64 cap,
    u64 cap_byte, unsigned long long* __restrict__ hdr, u64* __restrict__ recs, uint8_t* __restrict__ bytes,
    u32* __restrict__ ovf) {
  __shared__ unsigned long long lrec[kMaxShards], lbyte[kMaxShards], grec[kMaxShards], gbyte[kMaxShards];
  for (u32 d = threadIdx.x; d < S; d += kThreads) lrec[d] = lbyte[d] = 0;
  __syncthreads();
  const u64 base = (u64)blockIdx.x * kTile + threadIdx.x;
  u32 o[kPer], sl[kPer];
  u64 l[kPer], t[kPer], p[kPer], rk[kPer], brk[kPer];
#pragma unroll
  for (int u = 0; u < kPer; u++) {  // every load in flight before the first ballot
    const u64 i = base + (u64)u * kThreads;
    const bool valid = i < n;
    o[u] = valid ? owner[i] : 0;
    l[u] = valid ? lr[i] : 0;
    sl[u] = valid ? slot[i] : 0;
    t[u] = valid ? ts[i] : 0;
    p[u] = valid ? pre[i] : 0;
  }
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const u64 len = l[u] & JY_LR_LEN_MASK;
    rk[u] = brk[u] = 0;
    // long values keep the arena's 8-byte granules (jy_arena_collect)
    wave_aggregate<true>(base + (u64)u * kThreads < n, o[u], len > 8 ? (u32)round_up8(len) : 0u, lrec, lbyte, &rk[u],
                         &brk[u]);
  }
  __syncthreads();
  for (u32 d = threadIdx.x; d < S; d += kThreads) {
    grec[d] = lrec[d] ? atomicAdd(&hdr[2 * d], lrec[d]) : 0;
    gbyte[d] = lbyte[d] ? atomicAdd(&hdr[2 * d + 1], lbyte[d]) : 0;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const u64 i = base + (u64)u * kThreads;
    if (i >= n) continue;
    const u64 pos = grec[o[u]] + rk[u];
    const u64 len = l[u] & JY_LR_LEN_MASK;
    const u64 bpos = gbyte[o[u]] + brk[u];
    const bool long_v = len > 8;
    const bool fits = pos < cap && (!long_v || bpos + round_up8(len) <= cap_byte);
    u64x2* r = reinterpret_cast<u64x2*>(recs + ((u64)o[u] * cap + pos) * 4);  // 32-B records, two 16-B stores
    if (!fits) {
      ovf[1 + atomicAdd(ovf, 1u)] = (u32)i;
      if (pos < cap) r[0] = u64x2{~0ull, 0};  // hole
      continue;
    }
    u64 out_lr = l[u];
    if (long_v) {
      uint8_t* dst = bytes + (u64)o[u] * cap_byte + bpos;
      const uint8_t* src = arena + (l[u] >> JY_LR_LEN_BITS);
      for (u64 j = 0; j < len; j++) dst[j] = src[j];
      out_lr = (bpos << JY_LR_LEN_BITS) | len;
    }
    r[0] = u64x2{(u64)sl[u], t[u]};
    r[1] = u64x2{p[u], out_lr};
  }
}

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kTile - 1) / kTile); }

}  // namespace

extern "C" {

void jy_keys_owner(uint64_t n, const uint8_t* kb, const uint64_t* ko, uint32_t nshards, uint32_t* out) {
  for (u64 i = 0; i < n; i++) out[i] = jy_key_owner(kb + ko[i], ko[i + 1] - ko[i], nshards);
}

int32_t jy_treg_route_part(jy_engine* eng, uint64_t n, const uint32_t* owner, const uint32_t* slot, const uint64_t* ts,
                           const uint64_t* pre, const uint64_t* lr, uint32_t nshards, uint64_t cap, uint64_t cap_byte,
                           int32_t mem, uint64_t* recs_dev, uint8_t* bytes_dev, uint64_t* hdr_dev,
                           uint32_t* ovf_dev) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (nshards == 0 || nshards > kMaxShards) return eng->fail(JY_ERANGE, "nshards must be in [1, 64]");
  if (n == 0) return JY_OK;
  if (n >= 0xFFFFFFFFull) return eng->fail(JY_ERANGE, "more than 2^32 - 1 entries in one call");
  if (reinterpret_cast<uintptr_t>(recs_dev) % 16) return eng->fail(JY_EINVAL, "recs_dev must be 16-B aligned");
  if (cap_byte % kArenaAlign) return eng->fail(JY_EINVAL, "cap_byte must be a multiple of 8");
  if (mem == JY_HOST)
    for (u64 i = 0; i < n; i++)
      if (owner[i] >= nshards) return eng->fail(JY_ERANGE, "owner outside [0, nshards)");
  const void *dow, *dsl, *dts, *dpre, *dlr;
  JY_TRY(jy_stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, owner, n * 4, mem, &dow));
  JY_TRY(jy_stage(eng, 1, slot, n * 4, mem, &dsl));
  JY_TRY(jy_stage(eng, 2, ts, n * 8, mem, &dts));
  JY_TRY(jy_stage(eng, 3, pre, n * 8, mem, &dpre));
  JY_TRY(jy_stage(eng, 4, lr, n * 8, mem, &dlr));
  JY_TRY(jy_stage_end(eng));
  hipLaunchKernelGGL(k_route_part_treg, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream,
                     static_cast<const u32*>(dow), static_cast<const u32*>(dsl), static_cast<const u64*>(dts),
                     static_cast<const u64*>(dpre), static_cast<const u64*>(dlr), eng->arena[JY_TREG].p, n, nshards,
                     cap, cap_byte, reinterpret_cast<unsigned long long*>(hdr_dev), recs_dev, bytes_dev, ovf_dev);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_treg_converge_routed(jy_engine* eng, uint32_t nsrc, uint64_t cap, uint64_t cap_byte,
                                const uint64_t* recs_dev, const uint8_t* bytes_dev, const uint64_t* hdr_dev) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (nsrc == 0 || cap == 0) return JY_OK;
  if (cap_byte % kArenaAlign) return eng->fail(JY_EINVAL, "cap_byte must be a multiple of 8");
  // the sources' byte runs go to the arena whole (nsrc x cap_byte); the
  // records address them relative to their run
  u64 rebase;
  JY_TRY(jy_arena_append_dev(eng, JY_TREG, bytes_dev, (u64)nsrc * cap_byte, &rebase));
  return jy_treg_merge_routed(eng, nsrc, cap, cap_byte, recs_dev, hdr_dev, rebase);
}

}  // extern "C"
