// k_keyroute.hip -- cross-shard key resolution on the GPU (SURVEY 8f #1 at S > 1).
//
// On a node whose keys are hash-sharded over S engines, a key's slot lives
// on its owner.  An ingested batch names its keys as strings; before its
// entries can be routed (k_route.hip) every key needs (owner, slot on the
// owner) -- the reference's `_data_for(key)` (repo_treg.pony:37-42, the same
// in every repo_*.pony), create on miss, but on another GPU.  Three device
// steps and two variable all-to-alls (jylis_amd/route.py KeyResolver):
//
//   jy_keys_route_part   sender: owner of every key (jy_key_owner's hash on
//                        the device), the keys regrouped by owner -- lengths
//                        and bytes in owner order, the count of keys / bytes
//                        per owner, and each key's index in that order
//   (exchange)           lengths and bytes to their owners
//   jy_keys_intern_lens  owner: the received keys interned in its device
//                        directory (k_keys.hip: create on miss)
//   (exchange back)      the slots, in the senders' owner order
//   jy_keys_route_back   sender: slot of every input key = answer[index]
//
// Regrouping is the routers' three-pass partition (no same-address global
// atomics): per-tile counts of keys and bytes per owner, one column-major
// device scan whose column order [keys of owner 0..S-1, bytes of owner
// 0..S-1] makes every prefix directly an offset in owner order, then a
// placement pass (tile base + waves before + rank in the wave's ballot).
//
// Roofline: HBM / latency.  Per key: its bytes read twice (hash, copy) and
// written once, 8 B length + 4 B index + 4 B owner written; the directory
// probe on the owner (k_keys.hip) dominates.

#include <algorithm>

#include "jy_dscan.hpp"
#include "jy_internal.hpp"
#include "jy_scan.hpp"

namespace {

constexpr int kT = 256;
constexpr u32 kMaxShards = 64;

__device__ __forceinline__ u32 owner_of(const uint8_t* __restrict__ p, u64 len, u32 S) {
  return jy_dev_key_owner(p, len, S);
}

// per tile: keys and bytes per owner, one LDS atomic per (wave, owner, quantity)
__global__ __launch_bounds__(kT) void k_kr_count(const uint8_t* __restrict__ kb, const u64* __restrict__ ko, u64 n,
                                                 u32 S, u32* __restrict__ owner, u64* __restrict__ tcnt) {
  __shared__ unsigned long long lc[2 * kMaxShards];
  for (u32 j = threadIdx.x; j < 2 * S; j += kT) lc[j] = 0;
  __syncthreads();
  const u64 i = (u64)blockIdx.x * kT + threadIdx.x;
  u32 o = S;
  u64 len = 0;
  if (i < n) {
    const u64 a = ko[i];
    len = ko[i + 1] - a;
    o = owner_of(kb + a, len, S);
    owner[i] = o;
  }
  const bool valid = i < n;
  u64 pending = __ballot(valid);
  while (pending) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const u32 d = __shfl(o, leader);
    const bool mine = valid && o == d;
    pending &= ~__ballot(mine);
    const u64 keys = jyscan::wave_sum<u64>(mine ? 1ull : 0ull);
    const u64 byts = jyscan::wave_sum<u64>(mine ? len : 0ull);
    if (__lane_id() == (u32)leader) {
      atomicAdd(&lc[d], (unsigned long long)keys);
      atomicAdd(&lc[S + d], (unsigned long long)byts);
    }
  }
  __syncthreads();
  u64* row = tcnt + (u64)blockIdx.x * 2 * S;
  for (u32 j = threadIdx.x; j < 2 * S; j += kT) row[j] = lc[j];
}

// totals per (quantity, owner) from the scanned columns: counts[c] = prefix of
// column c + 1 (row 0) - prefix of column c (row 0)
__global__ void k_kr_totals(const u64* __restrict__ tcnt, u64 ntiles, u32 W, u64* __restrict__ counts) {
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= W) return;
  const u64 hi = c + 1 < W ? tcnt[c + 1] : tcnt[ntiles * W];
  counts[c] = hi - tcnt[c];
}

__global__ __launch_bounds__(kT) void k_kr_place(const uint8_t* __restrict__ kb, const u64* __restrict__ ko, u64 n,
                                                 u32 S, const u32* __restrict__ owner, const u64* __restrict__ tcnt,
                                                 u32* __restrict__ pos_out, u64* __restrict__ lens,
                                                 uint8_t* __restrict__ bytes) {
  constexpr int kW = kT / 64;
  __shared__ u64 wt[kW][2 * kMaxShards];
  for (u32 j = threadIdx.x; j < 2 * S; j += kT) {
#pragma unroll
    for (int w = 0; w < kW; w++) wt[w][j] = 0;
  }
  __syncthreads();
  const u64 i = (u64)blockIdx.x * kT + threadIdx.x;
  const int lane = __lane_id(), wv = threadIdx.x >> 6;
  const u64 lt = (1ull << lane) - 1;
  const bool valid = i < n;
  u32 o = 0xFFFFFFFFu;
  u64 a = 0, len = 0;
  if (valid) {
    o = owner[i];
    a = ko[i];
    len = ko[i + 1] - a;
  }
  u64 rk = 0, bk = 0;
  u64 pending = __ballot(valid);
  while (pending) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const u32 d = __shfl(o, leader);
    const bool mine = valid && o == d;
    const u64 m = __ballot(mine);
    const u64 x = mine ? len : 0;
    const u64 inc = jyscan::wave_incl<u64>(x);
    if (mine) {
      rk = __popcll(m & lt);
      bk = inc - x;
    }
    const u64 tot = __shfl(inc, 63);
    if (lane == leader) {
      wt[wv][d] = __popcll(m);
      wt[wv][S + d] = tot;
    }
    pending &= ~m;
  }
  __syncthreads();
  if (!valid) return;
  // column-major prefixes: key columns first, so a key column's prefix is the
  // key's offset in owner order; byte columns start after all n keys
  const u64* tb = tcnt + (u64)blockIdx.x * 2 * S;
  u64 p = tb[o] + rk, b = tb[S + o] - tcnt[S] + bk;
  for (int w = 0; w < wv; w++) {
    p += wt[w][o];
    b += wt[w][S + o];
  }
  pos_out[i] = (u32)p;
  lens[p] = len;
  for (u64 q = 0; q < len; q++) bytes[b + q] = kb[a + q];  // (word reads + byte stores measured slower: 111 -> 153 us)
}

__global__ __launch_bounds__(kT) void k_kr_back(u64 n, const u32* __restrict__ pos, const u32* __restrict__ answers,
                                                u32* __restrict__ slots) {
  const u64 i = (u64)blockIdx.x * kT + threadIdx.x;
  if (i < n) slots[i] = answers[pos[i]];
}

__global__ __launch_bounds__(kT) void k_kr_lens(u64 n, const u64* __restrict__ lens, u64* __restrict__ buf) {
  const u64 i = (u64)blockIdx.x * kT + threadIdx.x;
  if (i <= n) buf[i] = i < n ? lens[i] : 0;
}

u32 tiles_of(u64 n) { return (u32)std::max<u64>(1, (n + kT - 1) / kT); }

}  // namespace

extern "C" {

int32_t jy_keys_route_part(jy_engine* eng, uint64_t n, const uint8_t* key_bytes, const uint64_t* key_offs,
                           uint32_t nshards, uint32_t* owner_out, uint32_t* pos_out, uint64_t* send_lens,
                           uint8_t* send_bytes, uint64_t* counts_out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (nshards == 0 || nshards > kMaxShards) return eng->fail(JY_ERANGE, "nshards must be in [1, 64]");
  const u64 W = 2ull * nshards;
  if (n == 0) {
    JY_HIP(eng, hipMemsetAsync(counts_out, 0, W * 8, eng->stream));
    return JY_OK;
  }
  if (n >= 0xFFFFFFFFull) return eng->fail(JY_ERANGE, "more than 2^32 - 1 keys in one call");
  const u64 ntiles = tiles_of(n);
  void* p;
  JY_TRY(jy_scratch(eng, 24, (ntiles * W + 1) * 8 + 64, &p));
  u64* tcnt = static_cast<u64*>(p);
  hipLaunchKernelGGL(k_kr_count, dim3((u32)ntiles), dim3(kT), 0, eng->stream, key_bytes, key_offs, n, nshards,
                     owner_out, tcnt);
  JY_HIP(eng, hipGetLastError());
  JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, ntiles * W + 1, jydscan::LdColMajor{tcnt, ntiles, W},
                                                jydscan::StColMajor{tcnt, ntiles, W})));
  hipLaunchKernelGGL(k_kr_totals, dim3(1), dim3(128), 0, eng->stream, tcnt, ntiles, (u32)W, counts_out);
  JY_HIP(eng, hipGetLastError());
  hipLaunchKernelGGL(k_kr_place, dim3((u32)ntiles), dim3(kT), 0, eng->stream, key_bytes, key_offs, n, nshards,
                     owner_out, tcnt, pos_out, send_lens, send_bytes);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_keys_intern_lens(jy_engine* eng, int32_t type, uint64_t n, const uint8_t* bytes, const uint64_t* lens,
                            uint32_t* slots_out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (type < 0 || type >= JY_NTYPES) return eng->fail(JY_ETYPE, "unknown CRDT type");
  if (n == 0) return JY_OK;
  void* p;
  JY_TRY(jy_scratch(eng, 30, (n + 1) * 16 + 64, &p));
  u64* buf = static_cast<u64*>(p);
  u64* offs = buf + n + 1;
  hipLaunchKernelGGL(k_kr_lens, dim3(tiles_of(n + 1)), dim3(kT), 0, eng->stream, n, lens, buf);
  JY_HIP(eng, hipGetLastError());
  JY_TRY(jy_scan_u64(eng, buf, offs, n));
  return jy_keys_intern_mem(eng, type, n, bytes, offs, slots_out, JY_DEVICE);
}

int32_t jy_keys_route_back(jy_engine* eng, uint64_t n, const uint32_t* pos, const uint32_t* answers,
                           uint32_t* slots_out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  hipLaunchKernelGGL(k_kr_back, dim3(tiles_of(n)), dim3(kT), 0, eng->stream, n, pos, answers, slots_out);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

}  // extern "C"
