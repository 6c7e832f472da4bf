// k_treg.hip -- TREG last-writer-wins compare-select for gfx950.
//
// Semantics (oracle/jy_oracle.cpp TReg; treg.md:58-63): the delta (v, t)
// replaces the state (v_s, t_s) iff t > t_s, or t == t_s and v > v_s in
// Pony String order.  A fresh slot is ("", 0) (repo_treg.pony:37-42).
//
// HBM layout (SoA per slot): ts u64, pre u64 (first 8 value bytes,
// big-endian, zero padded), lr u64 (arena offset << 24 | length).  Values
// longer than 8 bytes also live whole in the type's arena; the byte loop
// runs only on (timestamp, prefix) ties of two long values.
//
// Roofline: HBM.  Per delta entry: 28 B delta read (slot + ts/pre/lr) +
// 8 B state ts read (pre/lr only on timestamp ties) + 24 B winner write.

#include <algorithm>

#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;

// kUnroll keys per lane, lanes on consecutive keys for every unroll step:
// all delta loads (coalesced, nontemporal) and the dependent state-ts
// gathers of the kUnroll keys are in flight together before any decision.
constexpr int kUnroll = 4;

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void lww_one(u64* __restrict__ ts, u64* __restrict__ pre, u64* __restrict__ lr,
                                        const uint8_t* __restrict__ arena, u64 s, u64 t, u64 p, u64 l, u64 t0) {
  bool win = t > t0;
  if (t == t0) win = jy_value_cmp(p, l, pre[s], lr[s], arena) > 0;
  if (win) {
    ts[s] = t;
    pre[s] = p;
    lr[s] = l;
  }
}

// Vector form: every lane owns PAIRS of consecutive delta entries, so the
// delta streams move 16 B per lane per load (8 B for the slot pair).  n is
// even and the delta arrays are 16-B aligned (checked by the launcher).
__global__ __launch_bounds__(kThreads) void k_treg_lww_v2(u64* __restrict__ ts, u64* __restrict__ pre,
                                                          u64* __restrict__ lr, const uint8_t* __restrict__ arena,
                                                          const u32* __restrict__ slot, const u64* __restrict__ dts,
                                                          const u64* __restrict__ dpre,
                                                          const u64* __restrict__ dlr, u64 npairs) {
  constexpr int U = 2;  // pairs per lane
  const u64 base = (u64)blockIdx.x * (kThreads * U) + threadIdx.x;
  u32x2 s[U];
  u64x2 t[U], p[U], l[U], t0[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 q = base + (u64)u * kThreads;
    if (q < npairs) {
      s[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(slot) + q);
      t[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(dts) + q);
      p[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(dpre) + q);
      l[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(dlr) + q);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (base + (u64)u * kThreads < npairs) {
      t0[u].x = ts[s[u].x];
      t0[u].y = ts[s[u].y];
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (base + (u64)u * kThreads >= npairs) continue;
    lww_one(ts, pre, lr, arena, s[u].x, t[u].x, p[u].x, l[u].x, t0[u].x);
    lww_one(ts, pre, lr, arena, s[u].y, t[u].y, p[u].y, l[u].y, t0[u].y);
  }
}

__global__ __launch_bounds__(kThreads) void k_treg_lww(u64* __restrict__ ts, u64* __restrict__ pre,
                                                       u64* __restrict__ lr, const uint8_t* __restrict__ arena,
                                                       const u32* __restrict__ slot, const u64* __restrict__ dts,
                                                       const u64* __restrict__ dpre, const u64* __restrict__ dlr,
                                                       u64 n) {
  const u64 base = (u64)blockIdx.x * (kThreads * kUnroll) + threadIdx.x;
  u64 s[kUnroll], t[kUnroll], p[kUnroll], l[kUnroll], t0[kUnroll];
#pragma unroll
  for (int u = 0; u < kUnroll; u++) {
    const u64 i = base + (u64)u * kThreads;
    if (i < n) {
      s[u] = slot[i];
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
    if (base + (u64)u * kThreads >= n) continue;
    bool win = t[u] > t0[u];
    if (t[u] == t0[u]) win = jy_value_cmp(p[u], l[u], pre[s[u]], lr[s[u]], arena) > 0;
    if (win) {
      ts[s[u]] = t[u];
      pre[s[u]] = p[u];
      lr[s[u]] = l[u];
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_treg_gather(const u64* __restrict__ ts, const u64* __restrict__ pre,
                                                          const u64* __restrict__ lr, const u32* __restrict__ slots,
                                                          u64 n, u64* __restrict__ ots, u64* __restrict__ opre,
                                                          u64* __restrict__ olr) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u64 s = slots[i];
  ots[i] = ts[s];
  opre[i] = pre[s];
  olr[i] = lr[s];
}

}  // namespace

int32_t jy_treg_grow(jy_engine* eng, u64 need) {
  TregState& t = eng->treg;
  if (need <= t.kcap && t.ts) return JY_OK;
  u64 nk = std::max<u64>(need, t.kcap ? t.kcap * 2 : need);
  nk = std::max<u64>((nk + 63) & ~63ull, 64);
  void *a = t.ts, *b = t.pre, *c = t.lr;
  JY_TRY(jy_realloc(eng, &a, t.kcap * 8, nk * 8, true));
  JY_TRY(jy_realloc(eng, &b, t.kcap * 8, nk * 8, true));
  JY_TRY(jy_realloc(eng, &c, t.kcap * 8, nk * 8, true));
  t.ts = static_cast<u64*>(a);
  t.pre = static_cast<u64*>(b);
  t.lr = static_cast<u64*>(c);
  t.kcap = nk;
  return JY_OK;
}

int32_t jy_treg_merge(jy_engine* eng, u64 n, const u32* slot, const u64* ts, const u64* pre, const u64* lr) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  auto al16 = [](const void* q) { return reinterpret_cast<uintptr_t>(q) % 16 == 0; };
  u64 done = 0;
  if (n >= 2 && al16(ts) && al16(pre) && al16(lr) && reinterpret_cast<uintptr_t>(slot) % 8 == 0) {
    const u64 npairs = n / 2;
    const u64 blocks = (npairs + kThreads * 2 - 1) / (kThreads * 2);
    hipLaunchKernelGGL(k_treg_lww_v2, dim3((u32)blocks), dim3(kThreads), 0, eng->stream, t.ts, t.pre, t.lr,
                       eng->arena[JY_TREG].p, slot, ts, pre, lr, npairs);
    done = npairs * 2;
  }
  if (done < n) {
    const u64 rest = n - done;
    const u64 blocks = (rest + kThreads * kUnroll - 1) / (kThreads * kUnroll);
    hipLaunchKernelGGL(k_treg_lww, dim3((u32)blocks), dim3(kThreads), 0, eng->stream, t.ts, t.pre, t.lr,
                       eng->arena[JY_TREG].p, slot + done, ts + done, pre + done, lr + done, rest);
  }
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_treg_gather(jy_engine* eng, u64 n, const u32* slots, u64* ots, u64* opre, u64* olr) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  const u64 blocks = (n + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(k_treg_gather, dim3((u32)blocks), dim3(kThreads), 0, eng->stream, t.ts, t.pre, t.lr, slots, n,
                     ots, opre, olr);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}
