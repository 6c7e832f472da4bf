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
// winner fractions >= 0.2) + 8 B state ts read + 8 B ts rewritten, and per
// winner a 16-B handle write (a state over the MALL also rewrites losers'
// handles, 32 B more per loser: see k_treg_lww).

#include <algorithm>

#include <hipcub/hipcub.hpp>

#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
// keys per lane; lanes on consecutive keys for every unroll step, so all
// delta loads and the dependent state-ts gathers of the kUnroll keys are in
// flight together before any decision
constexpr int kUnroll = 4;
constexpr u64 kMallBytes = 256ull << 20;  // MI355X Infinity Cache (MALL)

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ bool lww_wins(u64 t, u64 t0, u64 p, u64 l, const TVal* __restrict__ val, u64 s,
                                         const uint8_t* __restrict__ arena) {
  if (t != t0) return t > t0;
  const TVal v0 = val[s];
  return jy_value_cmp(p, l, v0.pre, v0.lr, arena) > 0;
}

// kRewriteAll = false: every key rewrites its ts word (a loser writes back
//   the timestamp it read, so ts lines leave L2 whole instead of byte-masked:
//   no extra bytes), winners write their 16-B handle.
// kRewriteAll = true: losers also read and rewrite their handle, so every
//   handle line is written whole.  A byte-masked line that misses the
//   Infinity Cache costs HBM a read-modify-write; when the state outruns the
//   256 MiB MALL the explicit rewrite is cheaper (64M keys: 0.84 vs 0.96 ms),
//   while a cache-resident state prefers the leaner form (8M keys: 84 vs
//   94 us).  jy_treg_merge picks by state size.
// Both need one entry per slot per launch (the C ABI's contract; host
// batches that repeat a key are split into rounds).
template <bool kRewriteAll>
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
    if (i >= n) continue;
    const bool w = t[u] >= t0[u] && lww_wins(t[u], t0[u], p[u], l[u], val, s[u], arena);
    ts[s[u]] = w ? t[u] : t0[u];
    if (kRewriteAll) {
      const TVal old = w ? TVal{0, 0} : val[s[u]];
      val[s[u]] = w ? TVal{p[u], l[u]} : old;
    } else if (w) {
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

// ---- local SET (RepoTREG.set repo_treg.pony:65-68): TReg.update(v, t, delta)
// changes the state and records the write in the key's pending delta only if
// it wins against the state; the delta key exists either way
// (oracle/jy_oracle.cpp or_treg_set).  Run BEFORE the state merge of the same
// batch (one entry per key): an entry that beats the state as it was is
// LWW-merged into the pending delta, which equals the reference's sequence.
__global__ __launch_bounds__(kThreads) void k_treg_set_pending(const u64* __restrict__ ts, const TVal* __restrict__ val,
                                                               u64* __restrict__ dts, TVal* __restrict__ dval,
                                                               u32* __restrict__ dflag, u64* __restrict__ dcount,
                                                               const uint8_t* __restrict__ arena,
                                                               const u32* __restrict__ slot,
                                                               const u64* __restrict__ t, const u64* __restrict__ p,
                                                               const u64* __restrict__ l, u64 n) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u32 s = slot[i];
  const u64 ti = t[i], pi = p[i], li = l[i];
  if (atomicOr(dflag + s, 1u) == 0u) atomicAdd(dcount, 1ull);
  const u64 t0 = ts[s];
  if (ti < t0 || !lww_wins(ti, t0, pi, li, val, s, arena)) return;
  const u64 d0 = dts[s];
  if (ti < d0 || !lww_wins(ti, d0, pi, li, dval, s, arena)) return;
  dts[s] = ti;
  dval[s] = TVal{pi, li};
}

struct TregPendingPred {
  const u32* dflag;
  __device__ bool operator()(u32 s) const { return dflag[s] != 0; }
};

// flush_deltas (repo_treg.pony:18-22): emit each pending key's delta TReg and
// reset it to the fresh ("", 0)
__global__ __launch_bounds__(kThreads) void k_treg_flush(u32* __restrict__ dflag, u64* __restrict__ dts,
                                                         TVal* __restrict__ dval, const u32* __restrict__ slots,
                                                         u64 cnt, u64* __restrict__ ots, u64* __restrict__ opre,
                                                         u64* __restrict__ olr) {
  const u64 j = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (j >= cnt) return;
  const u32 s = slots[j];
  const TVal v = dval[s];
  ots[j] = dts[s];
  opre[j] = v.pre;
  olr[j] = v.lr;
  dts[s] = 0;
  dval[s] = TVal{0, 0};
  dflag[s] = 0;
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
  // state larger than the Infinity Cache: write whole lines (see k_treg_lww)
  const bool whole = t.kcap * (8 + sizeof(TVal)) > kMallBytes;
  if (whole)
    hipLaunchKernelGGL(k_treg_lww<true>, dim3(blocks(n, kThreads * kUnroll)), dim3(kThreads), 0, eng->stream, t.ts,
                       t.val, eng->arena[JY_TREG].p, slot, ts, pre, lr, n);
  else
    hipLaunchKernelGGL(k_treg_lww<false>, dim3(blocks(n, kThreads * kUnroll)), dim3(kThreads), 0, eng->stream,
                       t.ts, t.val, eng->arena[JY_TREG].p, slot, ts, pre, lr, n);
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

static int32_t treg_delta_grow(jy_engine* eng) {
  TregState& t = eng->treg;
  if (!t.dcount) {
    void* p = nullptr;
    JY_TRY(jy_dev_alloc(eng, &p, 8, "treg pending count"));
    JY_HIP(eng, hipMemsetAsync(p, 0, 8, eng->stream));
    t.dcount = static_cast<u64*>(p);
  }
  if (t.dkcap >= t.kcap && t.dflag) return JY_OK;
  void *a = t.dts, *b = t.dval, *f = t.dflag;
  JY_TRY(jy_realloc(eng, &a, t.dkcap * 8, t.kcap * 8, true));
  JY_TRY(jy_realloc(eng, &b, t.dkcap * sizeof(TVal), t.kcap * sizeof(TVal), true));
  JY_TRY(jy_realloc(eng, &f, t.dkcap * 4, t.kcap * 4, true));
  t.dts = static_cast<u64*>(a);
  t.dval = static_cast<TVal*>(b);
  t.dflag = static_cast<u32*>(f);
  t.dkcap = t.kcap;
  return JY_OK;
}

int32_t jy_treg_set_pending(jy_engine* eng, u64 n, const u32* slot, const u64* ts, const u64* pre, const u64* lr) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  JY_TRY(treg_delta_grow(eng));
  hipLaunchKernelGGL(k_treg_set_pending, dim3(blocks(n, kThreads)), dim3(kThreads), 0, eng->stream,
                     (const u64*)t.ts, (const TVal*)t.val, t.dts, t.dval, t.dflag, t.dcount,
                     eng->arena[JY_TREG].p, slot, ts, pre, lr, n);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_treg_pending(jy_engine* eng, u64* count) {
  TregState& t = eng->treg;
  *count = 0;
  if (!t.dcount) return JY_OK;
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, t.dcount, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  *count = eng->pin_total[0];
  return JY_OK;
}

int32_t jy_treg_flush_dev(jy_engine* eng, u64 nkeys, u64 cap, u32* slots, u64* ots, u64* opre, u64* olr, u64* count) {
  TregState& t = eng->treg;
  u64 cnt = 0;
  JY_TRY(jy_treg_pending(eng, &cnt));
  *count = cnt;
  if (cnt == 0) return JY_OK;
  if (cnt > cap) return eng->fail(JY_ERANGE, "flush output capacity is smaller than the pending delta count");
  nkeys = std::min<u64>(nkeys, t.dkcap);
  void *tmp = nullptr, *num = nullptr;
  size_t tb = 0;
  hipcub::CountingInputIterator<u32> it(0);
  TregPendingPred pred{t.dflag};
  JY_HIP(eng, hipcub::DeviceSelect::If(nullptr, tb, it, slots, (u32*)nullptr, (int)nkeys, pred, eng->stream));
  JY_TRY(jy_scratch(eng, 15, tb, &tmp));
  JY_TRY(jy_scratch(eng, 14, 8, &num));
  JY_HIP(eng, hipcub::DeviceSelect::If(tmp, tb, it, slots, static_cast<u32*>(num), (int)nkeys, pred, eng->stream));
  hipLaunchKernelGGL(k_treg_flush, dim3(blocks(cnt, kThreads)), dim3(kThreads), 0, eng->stream, t.dflag, t.dts,
                     t.dval, (const u32*)slots, cnt, ots, opre, olr);
  JY_HIP(eng, hipGetLastError());
  JY_HIP(eng, hipMemsetAsync(t.dcount, 0, 8, eng->stream));
  return JY_OK;
}
