// k_treg.hip -- TREG last-writer-wins compare-select for gfx950.
//
// Semantics (oracle/jy_oracle.cpp TReg; treg.md:58-63): the delta (v, t)
// replaces the state (v_s, t_s) iff t > t_s, or t == t_s and v > v_s in
// Pony String order.  A fresh slot is ("", 0) (repo_treg.pony:37-42).
//
// HBM layout per slot: ts u64 in its own array (every merge reads it) and a
// 16-B value handle TVal {pre, lr} (pre = first 8 value bytes big-endian,
// zero padded; lr = arena offset << 24 | length) that only winners and
// timestamp ties touch.  Values longer than 8 bytes also live whole in the
// type's arena; the byte loop runs only on (timestamp, prefix) ties of two
// long values.  tools/mb_treg.hip measured this split against SoA
// ts/pre/lr, a 32-B AoS record, a ts mirror + 32-B record and full
// rewrites: it is the fastest at the bench's winner fractions because a
// winner dirties one 8-B ts word and one 16-B handle instead of three
// scattered 8-B words (DESIGN.md "TREG").
//
// Roofline: HBM.  SURVEY 8d prices a key at 48 B (16 delta + 16 state read
// + 16 state write).  What this kernel moves per delta entry: 28 B delta
// (slot, ts, pre, lr; all coalesced, loaded up front with the state-ts
// gather -- loading the handle lazily for winners only measured slower at
// winner fractions >= 0.2) + 8 B state ts, and per winner 24 B state write.

#include <algorithm>

#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
// keys per lane; lanes on consecutive keys for every unroll step, so all
// delta loads and the dependent state-ts gathers of the kUnroll keys are in
// flight together before any decision
constexpr int kUnroll = 4;

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ bool lww_wins(u64 t, u64 t0, u64 p, u64 l, const TVal* __restrict__ val, u64 s,
                                         const uint8_t* __restrict__ arena) {
  if (t != t0) return t > t0;
  const TVal v0 = val[s];
  return jy_value_cmp(p, l, v0.pre, v0.lr, arena) > 0;
}

__global__ __launch_bounds__(kThreads) void k_treg_lww(u64* __restrict__ ts, TVal* __restrict__ val,
                                                       const uint8_t* __restrict__ arena,
                                                       const u32* __restrict__ slot, const u64* __restrict__ dts,
                                                       const u64* __restrict__ dpre, const u64* __restrict__ dlr,
                                                       u64 n) {
  const u64 base = (u64)blockIdx.x * (kThreads * kUnroll) + threadIdx.x;
  u32 s[kUnroll];
  u64 t[kUnroll], t0[kUnroll], p[kUnroll], l[kUnroll];
#pragma unroll
  for (int u = 0; u < kUnroll; u++) {
    const u64 i = base + (u64)u * kThreads;
    if (i < n) {
      s[u] = __builtin_nontemporal_load(slot + i);
      t[u] = __builtin_nontemporal_load(dts + i);
      p[u] = __builtin_nontemporal_load(dpre + i);
      l[u] = __builtin_nontemporal_load(dlr + i);
    }
  }
#pragma unroll
  for (int u = 0; u < kUnroll; u++)
    if (base + (u64)u * kThreads < n) t0[u] = ts[s[u]];
#pragma unroll
  for (int u = 0; u < kUnroll; u++) {
    const u64 i = base + (u64)u * kThreads;
    if (i >= n || t[u] < t0[u]) continue;
    if (lww_wins(t[u], t0[u], p[u], l[u], val, s[u], arena)) {
      ts[s[u]] = t[u];
      val[s[u]] = TVal{p[u], l[u]};
    }
  }
}

// receiver side of routing: one 32-B record (slot, ts, pre, lr) per entry,
// long values rebased onto the arena region this run's bytes went to
__global__ __launch_bounds__(kThreads) void k_treg_lww_records(u64* __restrict__ ts, TVal* __restrict__ val,
                                                               const uint8_t* __restrict__ arena,
                                                               const u64* __restrict__ recs, u64 n, u64 rebase) {
  constexpr int U = 2;
  const u64 base = (u64)blockIdx.x * (kThreads * U) + threadIdx.x;
  u64x2 a[U], b[U];
  u64 t0[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * kThreads;
    if (i < n) {
      a[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(recs + i * 4));
      b[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(recs + i * 4) + 1);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++)
    if (base + (u64)u * kThreads < n) t0[u] = ts[a[u].x];
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (base + (u64)u * kThreads >= n) continue;
    const u64 s = a[u].x, t = a[u].y, p = b[u].x;
    u64 l = b[u].y;
    if ((l & JY_LR_LEN_MASK) > 8) l = (((l >> JY_LR_LEN_BITS) + rebase) << JY_LR_LEN_BITS) | (l & JY_LR_LEN_MASK);
    if (t >= t0[u] && lww_wins(t, t0[u], p, l, val, s, arena)) {
      ts[s] = t;
      val[s] = TVal{p, l};
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_treg_gather(const u64* __restrict__ ts, const TVal* __restrict__ val,
                                                          const u32* __restrict__ slots, u64 n, u64* __restrict__ ots,
                                                          u64* __restrict__ opre, u64* __restrict__ olr) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u64 s = slots[i];
  const TVal v = val[s];
  ots[i] = ts[s];
  opre[i] = v.pre;
  olr[i] = v.lr;
}

u32 blocks(u64 n, u64 per) { return (u32)std::max<u64>(1, (n + per - 1) / per); }

}  // namespace

int32_t jy_treg_grow(jy_engine* eng, u64 need) {
  TregState& t = eng->treg;
  if (need <= t.kcap && t.ts) return JY_OK;
  u64 nk = std::max<u64>(need, t.kcap ? t.kcap * 2 : need);
  nk = std::max<u64>((nk + 63) & ~63ull, 64);
  void *a = t.ts, *b = t.val;
  JY_TRY(jy_realloc(eng, &a, t.kcap * 8, nk * 8, true));
  JY_TRY(jy_realloc(eng, &b, t.kcap * sizeof(TVal), nk * sizeof(TVal), true));
  t.ts = static_cast<u64*>(a);
  t.val = static_cast<TVal*>(b);
  t.kcap = nk;
  return JY_OK;
}

int32_t jy_treg_merge(jy_engine* eng, u64 n, const u32* slot, const u64* ts, const u64* pre, const u64* lr) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  JyTimed tm(eng);
  hipLaunchKernelGGL(k_treg_lww, dim3(blocks(n, kThreads * kUnroll)), dim3(kThreads), 0, eng->stream, t.ts, t.val,
                     eng->arena[JY_TREG].p, slot, ts, pre, lr, n);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_treg_merge_records(jy_engine* eng, const u64* recs, u64 n, u64 base) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  JyTimed tm(eng);
  hipLaunchKernelGGL(k_treg_lww_records, dim3(blocks(n, kThreads * 2)), dim3(kThreads), 0, eng->stream, t.ts, t.val,
                     eng->arena[JY_TREG].p, recs, n, base);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_treg_gather(jy_engine* eng, u64 n, const u32* slots, u64* ots, u64* opre, u64* olr) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  hipLaunchKernelGGL(k_treg_gather, dim3(blocks(n, kThreads)), dim3(kThreads), 0, eng->stream, t.ts, t.val, slots, n,
                     ots, opre, olr);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}
