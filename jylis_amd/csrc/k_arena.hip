// k_arena.hip -- value-arena reclamation for TREG / TLOG, gfx950.
//
// jy_values_pack only appends: every converge or SET carrying values longer
// than 8 bytes grows the type's arena, while the registers and log entries
// they replace (repo_treg.pony:51-52 replaces a register's value; a TLOG
// cutoff drops entries) leave dead bytes behind.  jy_arena_collect copies the
// live values into a fresh arena back to back and rewrites every handle.
//
// Long values start on 8-byte granules (jy_values_pack pads them), and two
// handles either name the same value range or disjoint ones, so a granule
// map describes the live set exactly:
//   mark     every live handle (state registers / log entries of every slot,
//            the pending deltas) stores its length at its first granule
//            (identical handles store the same length)
//   scan     exclusive sum of the padded lengths over granules -> new offsets
//   copy     each live value to its new offset
//   rewrite  every handle's offset through the granule map
// Handles packed but not yet merged become invalid (the ABI says so).
//
// Roofline: HBM; one pass over the old arena's granule map plus the live
// bytes twice; rare (a repo calls it when dead bytes outnumber live ones).

#include <algorithm>

#include "jy_dscan.hpp"
#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ u64 gid() { return (u64)blockIdx.x * kThreads + threadIdx.x; }

__device__ __forceinline__ void mark(u64 lr, u32* __restrict__ glen) {
  const u64 len = lr & JY_LR_LEN_MASK;
  if (len > 8) glen[(lr >> JY_LR_LEN_BITS) / kArenaAlign] = (u32)len;
}
__device__ __forceinline__ u64 moved(u64 lr, const u64* __restrict__ goff) {
  const u64 len = lr & JY_LR_LEN_MASK;
  if (len <= 8) return lr;
  return (goff[(lr >> JY_LR_LEN_BITS) / kArenaAlign] << JY_LR_LEN_BITS) | len;
}

// TREG: the state register and the pending delta register of every slot
template <bool kRewrite>
__global__ __launch_bounds__(kThreads) void k_arena_treg(TVal* __restrict__ val, TVal* __restrict__ dval,
                                                         const u32* __restrict__ dflag, u64 n, u64 nd,
                                                         u32* __restrict__ glen, const u64* __restrict__ goff) {
  const u64 s = gid();
  if (s >= n) return;
  if (kRewrite) val[s].lr = moved(val[s].lr, goff);
  else mark(val[s].lr, glen);
  if (s < nd && dflag[s]) {
    if (kRewrite) dval[s].lr = moved(dval[s].lr, goff);
    else mark(dval[s].lr, glen);
  }
}

// TLOG: the live entries of every log of one store (state or pending deltas)
template <bool kRewrite>
__global__ __launch_bounds__(kThreads) void k_arena_tlog(const TMeta* __restrict__ meta, TRec* __restrict__ pool,
                                                         u64 n, u32* __restrict__ glen, const u64* __restrict__ goff) {
  const u64 s = gid();
  if (s >= n) return;
  const TMeta m = meta[s];
  const u64 b = tm_base(m);
  for (u64 j = b; j < b + m.len; j++) {
    if (kRewrite) pool[j].lr = moved(pool[j].lr, goff);
    else mark(pool[j].lr, glen);
  }
}

// each live value to its new place (granule g's value: old g * align -> new goff[g])
__global__ __launch_bounds__(kThreads) void k_arena_copy(const u32* __restrict__ glen, const u64* __restrict__ goff,
                                                         u64 ng, const uint8_t* __restrict__ src,
                                                         uint8_t* __restrict__ dst) {
  const u64 g = gid();
  if (g >= ng || glen[g] == 0) return;
  const u64 len = glen[g];
  const uint8_t* a = src + g * kArenaAlign;
  uint8_t* b = dst + goff[g];
  for (u64 i = 0; i < len; i++) b[i] = a[i];
}

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

#define LAUNCH(k, n, ...)                                                                          \
  do {                                                                                             \
    hipLaunchKernelGGL(k, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, __VA_ARGS__);     \
    JY_HIP(eng, hipGetLastError());                                                                \
  } while (0)

// padded length of a granule's value (0: no value starts there)
struct LdPad {
  const u32* glen;
  __device__ u64 operator()(u64 g) const { return (glen[g] + kArenaAlign - 1) / kArenaAlign * kArenaAlign; }
};

}  // namespace

// device bytes appended to a type's arena on its 8-byte granule; *rebase_out
// receives their arena offset (routed runs: k_route.hip, k_route_csr.hip)
int32_t jy_arena_append_dev(jy_engine* eng, int32_t type, const uint8_t* src, u64 bytes, u64* rebase_out) {
  Arena& a = eng->arena[type];
  const u64 at = (a.len + kArenaAlign - 1) / kArenaAlign * kArenaAlign;
  *rebase_out = at;
  if (bytes == 0) return JY_OK;
  if ((at + bytes) >> (64 - JY_LR_LEN_BITS)) return eng->fail(JY_ERANGE, "arena offset overflow");
  if (at + bytes > a.cap) {
    const u64 nc = std::max<u64>(std::max<u64>(a.cap * 2, at + bytes), 1 << 16);
    void* p = a.p;
    JY_TRY(jy_realloc(eng, &p, a.len, nc, false));
    a.p = static_cast<uint8_t*>(p);
    a.cap = nc;
  }
  JY_HIP(eng, hipMemcpyAsync(a.p + at, src, bytes, hipMemcpyDeviceToDevice, eng->stream));
  a.len = at + bytes;
  return JY_OK;
}

// room for `bytes` more at the tail of a type's arena (8-byte granule): the
// device pointer to write them through and their arena offset.  The pointer
// stays valid until the next call that grows this arena (an append, a pack,
// a collection); a routed receiver lands its byte runs there directly
// (jy_treg_converge_routed_at) instead of appending a copy.
extern "C" int32_t jy_arena_reserve(jy_engine* eng, int32_t type, uint64_t bytes, uint8_t** dev_out,
                                    uint64_t* rebase_out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (type != JY_TREG && type != JY_TLOG) return eng->fail(JY_EINVAL, "only TREG and TLOG hold an arena");
  Arena& a = eng->arena[type];
  const u64 at = (a.len + kArenaAlign - 1) / kArenaAlign * kArenaAlign;
  if ((at + bytes) >> (64 - JY_LR_LEN_BITS)) return eng->fail(JY_ERANGE, "arena offset overflow");
  if (at + bytes > a.cap || !a.p) {
    const u64 nc = std::max<u64>(std::max<u64>(a.cap * 2, at + bytes), 1 << 16);
    void* p = a.p;
    JY_TRY(jy_realloc(eng, &p, a.len, nc, false));
    a.p = static_cast<uint8_t*>(p);
    a.cap = nc;
  }
  a.len = at + bytes;
  *dev_out = a.p + at;
  *rebase_out = at;
  return JY_OK;
}

// capacity for `bytes` more (aligned) without moving the arena later: a
// reserve within it only advances the length (the node reserves the long
// values' exact total on its read-back stream, where a reallocation on the
// engine stream would not be ordered before the writes)
int32_t jy_arena_ensure(jy_engine* eng, int32_t type, u64 bytes) {
  if (type != JY_TREG && type != JY_TLOG) return eng->fail(JY_EINVAL, "only TREG and TLOG hold an arena");
  Arena& a = eng->arena[type];
  const u64 at = (a.len + kArenaAlign - 1) / kArenaAlign * kArenaAlign;
  if (at + bytes <= a.cap && a.p) return JY_OK;
  const u64 nc = std::max<u64>(std::max<u64>(a.cap * 2, at + bytes), 1 << 16);
  void* p = a.p;
  JY_TRY(jy_realloc(eng, &p, a.len, nc, false));
  a.p = static_cast<uint8_t*>(p);
  a.cap = nc;
  return JY_OK;
}

extern "C" int32_t jy_arena_usage(jy_engine* eng, int32_t type, uint64_t* len_out, uint64_t* cap_out) {
  if (type < 0 || type >= JY_NTYPES) return eng->fail(JY_EINVAL, "bad type");
  *len_out = eng->arena[type].len;
  *cap_out = eng->arena[type].cap;
  return JY_OK;
}

extern "C" int32_t jy_arena_collect(jy_engine* eng, int32_t type, uint64_t* live_out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (type != JY_TREG && type != JY_TLOG) return eng->fail(JY_EINVAL, "only TREG and TLOG hold an arena");
  if (type == JY_TLOG) JY_TRY(jy_tlog_settle(eng));  // a spilled merge's handles are live too
  Arena& a = eng->arena[type];
  *live_out = 0;
  if (a.len == 0) return JY_OK;
  const u64 ng = (a.len + kArenaAlign - 1) / kArenaAlign;
  void* p;
  JY_TRY(jy_scratch(eng, 23, ng * 4 + 64, &p));
  u32* glen = static_cast<u32*>(p);
  JY_TRY(jy_scratch(eng, 22, (ng + 1) * 8 + 64, &p));
  u64* goff = static_cast<u64*>(p);
  JY_HIP(eng, hipMemsetAsync(glen, 0, (ng + 1) * 4, eng->stream));  // (+1: the scan's total slot)
  const u64 nk = eng->nkeys[type];
  if (type == JY_TREG) {
    TregState& t = eng->treg;
    JY_TRY(jy_treg_fold(eng));  // pending duplicate records hold handles too
    if (nk) LAUNCH((k_arena_treg<false>), nk, t.val, t.dval, t.dflag, nk, std::min<u64>(nk, t.dkcap), glen, goff);
  } else {
    if (nk) LAUNCH((k_arena_tlog<false>), nk, eng->tlog.meta, eng->tlog.pool, nk, glen, goff);
    if (nk && eng->tlog_d.meta) LAUNCH((k_arena_tlog<false>), nk, eng->tlog_d.meta, eng->tlog_d.pool, nk, glen, goff);
  }
  JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, ng + 1, LdPad{glen}, jydscan::StArr<u64>{goff})));
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, goff + ng, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  const u64 live = eng->pin_total[0];
  const u64 cap = std::max<u64>(std::max<u64>(2 * live, 1 << 16), eng->cfg.arena_capacity[type]);
  uint8_t* na = nullptr;
  JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&na), cap, "value arena"));
  LAUNCH(k_arena_copy, ng, glen, goff, ng, a.p, na);
  if (type == JY_TREG) {
    TregState& t = eng->treg;
    if (nk) LAUNCH((k_arena_treg<true>), nk, t.val, t.dval, t.dflag, nk, std::min<u64>(nk, t.dkcap), glen, goff);
  } else {
    if (nk) LAUNCH((k_arena_tlog<true>), nk, eng->tlog.meta, eng->tlog.pool, nk, glen, goff);
    if (nk && eng->tlog_d.meta) LAUNCH((k_arena_tlog<true>), nk, eng->tlog_d.meta, eng->tlog_d.pool, nk, glen, goff);
  }
  JY_HIP(eng, hipStreamSynchronize(eng->stream));  // the old arena is read until here
  jy_dev_free(eng, a.p);
  a.p = na;
  a.len = live;
  a.cap = cap;
  *live_out = live;
  return JY_OK;
}
