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
#include "jy_dscan.hpp"
#include "jy_scan.hpp"

namespace {

constexpr u32 kMaxShards = 64;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u64 round_up8(u64 x) { return (x + kArenaAlign - 1) & ~(kArenaAlign - 1); }

// Three passes, no same-address global atomics (one reservation atomic per
// workgroup and owner serialised ~4k workgroups on one header word):
//   k_rt_count  per tile of 256 entries: records and long-value bytes per owner
//   scan        every (owner, quantity) column of tile counts in one
//               device-wide scan taken column after column (jy_dscan.hpp);
//               k_rt_hdr takes the grand totals to the header
//   k_rt_place  per entry: its place in its owner's run = tile base + the
//               waves before it + its rank among its wave's entries for the
//               same owner (one ballot per distinct owner, masked scans);
//               an entry that fits is written, else listed in ovf -- and the
//               first entry of an owner that does not fit writes the header
//               (the placed entries are the prefix before it: the ends grow
//               along an owner's sequence)
// The count is ONE WAVE per tile (4 entries per lane, slice u = entries
// u*64 + lane): owner d's counts live in lane d's registers (S <= 64), no LDS
// and no barrier (45 -> 29 us at 8M entries against a 256-thread workgroup
// with LDS counts per wave).
// Measured and dropped in round 4 (routed TREG step at 8M entries, kernel
// trace): ONE pass with a decoupled look-back over ticketed tiles -- 0.41-
// 0.54 ms for the pass, the tickets (one same-address atomic per workgroup,
// 32K of them) serialise; 1024-entry tiles, four per ticket, chained every
// workgroup behind the previous one's last tile (60 ms); block sums added
// atomically by the count instead of the scan -- the count went 29 -> 120 us
// (the block rows share a few lines) and the placement's base sums cost 18 us.
constexpr int kSlices = 4;        // 64-entry slices per count tile (one wave)
constexpr int kT = 64 * kSlices;  // entries per tile (count and place)
constexpr int kWG = 256;          // count: threads per workgroup = 4 tiles

// `self`: entries owned by this shard are merged where they lie
// (jy_treg_route_part_self) and neither counted nor placed; S = none
__global__ __launch_bounds__(kWG) void k_rt_count(const u32* __restrict__ owner, const u64* __restrict__ lr, u64 n,
                                                  u32 S, u32 self, u64* __restrict__ tcnt) {
  const u64 tile = (u64)blockIdx.x * (kWG / 64) + (threadIdx.x >> 6);
  if (tile * kT >= n) return;  // a whole wave
  const u32 lane = __lane_id();
  u32 o[kSlices];
  u64 b[kSlices];
#pragma unroll
  for (int u = 0; u < kSlices; u++) {
    const u64 i = tile * kT + (u64)u * 64 + lane;
    o[u] = S;
    b[u] = 0;
    if (i < n) {
      o[u] = owner[i];
      if (o[u] == self) {
        o[u] = S;
      } else {
        const u64 len = __builtin_nontemporal_load(lr + i) & JY_LR_LEN_MASK;
        b[u] = len > 8 ? round_up8(len) : 0;
      }
    }
  }
  u64 c = 0, cb = 0;  // lane d: owner d's records and bytes in this tile
#pragma unroll
  for (int u = 0; u < kSlices; u++) {
    const bool anyb = __ballot(b[u] != 0) != 0;
    u64 pending = __ballot(o[u] < S);
    while (pending) {
      const u32 d = __builtin_amdgcn_readlane(o[u], __ffsll((unsigned long long)pending) - 1);
      const u64 m = __ballot(o[u] == d);
      pending &= ~m;
      const u64 bs = anyb ? jyscan::wave_sum<u64>(o[u] == d ? b[u] : 0ull) : 0ull;
      if (lane == d) {
        c += __popcll(m);
        cb += bs;
      }
    }
  }
  if (lane < S) {
    u64* row = tcnt + tile * S * 2;
    row[lane * 2] = c;
    row[lane * 2 + 1] = cb;
  }
}


// after the column-major device scan of tcnt (every column's prefix offset by
// the columns before it): the header's totals per (owner, quantity)
__global__ void k_rt_hdr(const u64* __restrict__ tcnt, u64 ntiles, u32 W, unsigned long long* __restrict__ hdr) {
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= W) return;
  const u64 hi = c + 1 < W ? tcnt[c + 1] : tcnt[ntiles * W];
  hdr[c] = hi - tcnt[c];
}

// placement: a 256-thread workgroup per tile, one entry per thread, per-wave
// counts in LDS.  (A one-wave-per-tile form with four entries per lane and
// the running bases in lane registers, like k_rt_count, measured slower:
// in-box A/B of the routed TREG step 0.358 vs 0.341 ms.)
__global__ __launch_bounds__(256) void k_rt_place(const u32* __restrict__ owner, const u32* __restrict__ slot,
                                                 const u64* __restrict__ ts, const u64* __restrict__ pre,
                                                 const u64* __restrict__ lr, const uint8_t* __restrict__ arena, u64 n,
                                                 u32 S, u32 self, u64 cap, u64 cap_byte, const u64* __restrict__ tcnt,
                                                 unsigned long long* __restrict__ hdr, u64* __restrict__ recs,
                                                 uint8_t* __restrict__ bytes, u32* __restrict__ ovf,
                                                 unsigned long long* __restrict__ skipped) {
  constexpr int kW = 256 / 64;
  __shared__ u64 wt[kW][kMaxShards * 2];
  __shared__ u64 tbase[kMaxShards * 2];
  for (u32 j = threadIdx.x; j < S * 2; j += kT) {
#pragma unroll
    for (int w = 0; w < kW; w++) wt[w][j] = 0;
    // the tile's base per column (less the column's base, row 0): loaded
    // before the entries' ranks are known, in flight with their loads
    tbase[j] = tcnt[(u64)blockIdx.x * S * 2 + j] - tcnt[j];
  }
  __syncthreads();
  const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
  const int lane = __lane_id(), wv = threadIdx.x >> 6;
  const u64 lt = (1ull << lane) - 1;
  u32 o = 0xFFFFFFFFu, sl = 0;
  u64 t = 0, p = 0, l = 0, b = 0;
  u64 g0 = 0, g1 = 0;  // a long value's first two 8-B granules, loaded early
  if (i < n) o = owner[i];
  if (i < n && o != self) {  // this shard's own entries are merged where they lie
    sl = slot[i];
    t = ts[i];
    p = pre[i];
    l = lr[i];
    const u64 len = l & JY_LR_LEN_MASK;
    b = len > 8 ? round_up8(len) : 0;
    if (b) {
      const u64* src = reinterpret_cast<const u64*>(arena + (l >> JY_LR_LEN_BITS));
      g0 = src[0];
      g1 = src[1];
    }
  }
  const bool valid = i < n && o < S && o != self;
  if (i < n && o >= S) atomicAdd(skipped, 1ull);  // an owner outside [0, S): dropped, counted
  u64 rk = 0, bk = 0;
  u64 pending = __ballot(valid);
  while (pending) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const u32 d = __shfl(o, leader);
    const bool mine = valid && o == d;
    const u64 m = __ballot(mine);
    const u64 x = mine ? b : 0;
    const u64 inc = jyscan::wave_incl<u64>(x);
    if (mine) {
      rk = __popcll(m & lt);
      bk = inc - x;
    }
    const u64 tot = __shfl(inc, 63);
    if (lane == leader) {
      wt[wv][d * 2] = __popcll(m);
      wt[wv][d * 2 + 1] = tot;
    }
    pending &= ~m;
  }
  __syncthreads();
  if (!valid) return;
  u64 pos = tbase[o * 2] + rk, bpos = tbase[o * 2 + 1] + bk;
  for (int w = 0; w < wv; w++) {
    pos += wt[w][o * 2];
    bpos += wt[w][o * 2 + 1];
  }
  const bool fits = pos < cap && bpos + b <= cap_byte;
  if (!fits) {
    ovf[1 + atomicAdd(ovf, 1u)] = (u32)i;
    if (pos == 0 || (pos - 1 < cap && bpos <= cap_byte)) {  // the first of its owner that does not fit
      hdr[2 * o] = pos;
      hdr[2 * o + 1] = bpos;
    }
    return;
  }
  u64 out_lr = l;
  if (b) {  // the value's 8-B granules into the run's byte section
    const u64* src = reinterpret_cast<const u64*>(arena + (l >> JY_LR_LEN_BITS));
    u64* dst = reinterpret_cast<u64*>(bytes + (u64)o * cap_byte + bpos);
    dst[0] = g0;  // b >= 16: a long value has two granules at least
    dst[1] = g1;
    for (u64 w = 2; w < b / 8; w++) dst[w] = src[w];
    out_lr = (bpos << JY_LR_LEN_BITS) | (l & JY_LR_LEN_MASK);
  }
  u64x2* r = reinterpret_cast<u64x2*>(recs + ((u64)o * cap + pos) * 4);  // 32-B records, two 16-B stores
  r[0] = u64x2{(u64)sl, t};
  r[1] = u64x2{p, out_lr};
}


}  // namespace

extern "C" {

void jy_keys_owner(uint64_t n, const uint8_t* kb, const uint64_t* ko, uint32_t nshards, uint32_t* out) {
  for (u64 i = 0; i < n; i++) out[i] = jy_key_owner(kb + ko[i], ko[i + 1] - ko[i], nshards);
}

}  // extern "C"

namespace {

int32_t route_part(jy_engine* eng, uint64_t n, const uint32_t* owner, const uint32_t* slot, const uint64_t* ts,
                   const uint64_t* pre, const uint64_t* lr, uint32_t nshards, uint32_t self, uint64_t cap,
                   uint64_t cap_byte, int32_t mem, uint64_t* recs_dev, uint8_t* bytes_dev, uint64_t* hdr_dev,
                   uint32_t* ovf_dev) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (nshards == 0 || nshards > kMaxShards) return eng->fail(JY_ERANGE, "nshards must be in [1, 64]");
  if (self != nshards && self >= nshards) return eng->fail(JY_ERANGE, "self must be in [0, nshards)");
  if (n == 0) {
    JY_HIP(eng, hipMemsetAsync(hdr_dev, 0, (u64)nshards * 16, eng->stream));
    return JY_OK;
  }
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
  const u64 ntiles = (n + kT - 1) / kT;
  void* p;
  JY_TRY(jy_scratch(eng, 24, ntiles * nshards * 2 * 8 + 64, &p));
  u64* tcnt = static_cast<u64*>(p);
  const u32* own = static_cast<const u32*>(dow);
  const u64* l = static_cast<const u64*>(dlr);
  const u32 nwg = (u32)((ntiles + kWG / 64 - 1) / (kWG / 64));
  if (self < nshards)  // this shard's share first: the partition below leaves it out
    JY_TRY(jy_treg_merge_owned(eng, n, own, self, static_cast<const u32*>(dsl), static_cast<const u64*>(dts),
                               static_cast<const u64*>(dpre), l));
  hipLaunchKernelGGL(k_rt_count, dim3(nwg), dim3(kWG), 0, eng->stream, own, l, n, nshards, self, tcnt);
  JY_HIP(eng, hipGetLastError());
  {
    // the tile counts of every (owner, quantity) column in ONE device-wide
    // scan taken column after column (a workgroup per column walking its
    // tiles took 35 us at 8M entries); each column's base is its row-0 entry
    const u64 W = (u64)nshards * 2;
    JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, ntiles * W + 1, jydscan::LdColMajor{tcnt, ntiles, W},
                                                  jydscan::StColMajor{tcnt, ntiles, W})));
    hipLaunchKernelGGL(k_rt_hdr, dim3(1), dim3(128), 0, eng->stream, tcnt, ntiles, (u32)W,
                       reinterpret_cast<unsigned long long*>(hdr_dev));
    JY_HIP(eng, hipGetLastError());
  }
  static_assert(kT == 256, "the workgroup placement takes 256-entry tiles");
  hipLaunchKernelGGL(k_rt_place, dim3((u32)ntiles), dim3(256), 0, eng->stream, own, static_cast<const u32*>(dsl),
                     static_cast<const u64*>(dts), static_cast<const u64*>(dpre), l, eng->arena[JY_TREG].p, n, nshards,
                     self, cap, cap_byte, tcnt, reinterpret_cast<unsigned long long*>(hdr_dev), recs_dev, bytes_dev, ovf_dev,
                     reinterpret_cast<unsigned long long*>(eng->skipped_dev));
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

}  // namespace

extern "C" {

int32_t jy_treg_route_part(jy_engine* eng, uint64_t n, const uint32_t* owner, const uint32_t* slot, const uint64_t* ts,
                           const uint64_t* pre, const uint64_t* lr, uint32_t nshards, uint64_t cap, uint64_t cap_byte,
                           int32_t mem, uint64_t* recs_dev, uint8_t* bytes_dev, uint64_t* hdr_dev,
                           uint32_t* ovf_dev) {
  return route_part(eng, n, owner, slot, ts, pre, lr, nshards, nshards, cap, cap_byte, mem, recs_dev, bytes_dev,
                    hdr_dev, ovf_dev);
}

int32_t jy_treg_route_part_self(jy_engine* eng, uint64_t n, const uint32_t* owner, const uint32_t* slot,
                                const uint64_t* ts, const uint64_t* pre, const uint64_t* lr, uint32_t nshards,
                                uint32_t self, uint64_t cap, uint64_t cap_byte, int32_t mem, uint64_t* recs_dev,
                                uint8_t* bytes_dev, uint64_t* hdr_dev, uint32_t* ovf_dev) {
  if (self >= nshards) return eng->fail(JY_ERANGE, "self must be in [0, nshards)");
  return route_part(eng, n, owner, slot, ts, pre, lr, nshards, self, cap, cap_byte, mem, recs_dev, bytes_dev, hdr_dev,
                    ovf_dev);
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

// the received byte runs already sit in this engine's TREG arena at `rebase`
// (jy_arena_reserve; the exchange landed them there): no append copy
int32_t jy_treg_converge_routed_at(jy_engine* eng, uint32_t nsrc, uint64_t cap, uint64_t cap_byte,
                                   const uint64_t* recs_dev, const uint64_t* hdr_dev, uint64_t rebase) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (nsrc == 0 || cap == 0) return JY_OK;
  if (cap_byte % kArenaAlign || rebase % kArenaAlign) return eng->fail(JY_EINVAL, "cap_byte and rebase: multiples of 8");
  if (rebase + (u64)nsrc * cap_byte > eng->arena[JY_TREG].len)
    return eng->fail(JY_ERANGE, "the byte runs lie outside the arena's reserved bytes");
  return jy_treg_merge_routed(eng, nsrc, cap, cap_byte, recs_dev, hdr_dev, rebase);
}

}  // extern "C"
