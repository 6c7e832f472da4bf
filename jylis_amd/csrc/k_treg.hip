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
// A slot named twice in one launch (a device batch that breaks the
// one-delta-per-key contract, or routed runs of two sources touching one
// key) is resolved EXACTLY: the first entry of each slot (jy_claim_rows, one
// bit per slot) is merged by the wide kernel; the others are copied into a
// duplicate list that is folded in later -- before the next read or SET of
// the register file, or when the list could fill -- since LWW is a join and
// the fold's timing and order do not change the result.  The fold is a few
// parallel ROUNDS, one ordinary launch each (k_treg_fold_round: each merges
// the first record of every slot in its list and moves the rest to the next
// list), so a key that arrives many times costs one round per extra
// occurrence, not a serial walk; one wave folds whatever the rounds leave
// (unbounded repeats only).  An empty list costs the launches alone: every
// workgroup reads the count from HBM and returns.  No merge records an event
// or waits for the host, so merges run back to back.
// Routed runs are merged one source per launch: keys that several peers
// flushed in the same step never become duplicates.  A dense batch in slot
// order costs the claim one atomic instruction per wave.  Two claim bitmaps
// alternate: each launch clears the other one, slice by slice, so no launch
// is spent on resetting them.
//
// Roofline: HBM.  SURVEY 8d prices a key at 48 B (16 delta + 16 state read
// + 16 state write).  What this kernel moves per delta entry: 28 B delta
// (slot, ts, pre, lr; all coalesced, loaded up front with the state-ts
// gather -- loading the handle lazily for winners only measured slower at
// winner fractions >= 0.2) + 8 B state ts read + 8 B ts rewritten, and per
// winner a 16-B handle write (a state over the MALL also rewrites losers'
// handles, 32 B more per loser: see k_treg_lww).

#include <algorithm>
#include <cstring>


#include "jy_dscan.hpp"
#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
// keys per lane; lanes on consecutive keys for every unroll step, so all
// delta loads and the dependent state-ts gathers of the kUnroll keys are in
// flight together before any decision
#ifndef JY_TREG_UNROLL
#define JY_TREG_UNROLL 4
#endif
constexpr int kUnroll = JY_TREG_UNROLL;
// <true> form: load the old handles with the state timestamps (A/B switch)
#ifndef JY_TREG_PRELOAD
#define JY_TREG_PRELOAD 1
#endif
constexpr u64 kMallBytes = 256ull << 20;  // MI355X Infinity Cache (MALL)

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

// kCoh: loads that bypass the CU's L1 (the one-wave duplicate fold reads
// what other lanes of its wave stored a round earlier)
template <bool kCoh>
__device__ __forceinline__ u64 ld64(const u64* p) {
  return kCoh ? __hip_atomic_load(const_cast<u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
}

template <bool kCoh = false>
__device__ __forceinline__ bool lww_wins(u64 t, u64 t0, u64 p, u64 l, const TVal* __restrict__ val, u64 s,
                                         const uint8_t* __restrict__ arena) {
  if (t != t0) return t > t0;
  const u64 pre0 = ld64<kCoh>(&val[s].pre), lr0 = ld64<kCoh>(&val[s].lr);
  return jy_value_cmp(p, l, pre0, lr0, arena) > 0;
}

// state + (SET path) pending-delta registers + the launch's claim state
struct TregK {
  u64* ts;
  TVal* val;
  const uint8_t* arena;
  u32* seen;     // this launch's claim bitmap
  u32* clear;    // the other bitmap (cleared by this launch), or null
  u64 clear_bytes;
  u32* dupn;     // duplicate list: count, then 32-B records {slot, ts, pre, lr}
  u64* dups;
  u32* dupflag;  // host-mapped: [0] set when a duplicate is pushed, [1] when the list was full
  u64 dup_cap;   // records the list holds
  // RepoTREG._deltas (SET path only)
  u64* pts;
  TVal* pval;
  u32* pflag;
  u64* pcount;
};

// SET semantics of one entry whose slot nobody else touches right now:
// TReg.update(v, t, delta) (repo_treg.pony:65-68) changes the state and
// records the write in the key's pending delta only if it wins against the
// state; the delta key exists either way (oracle/jy_oracle.cpp or_treg_set)
template <bool kCoh = false>
__device__ __forceinline__ void set_one(const TregK& K, u32 s, u64 t, u64 p, u64 l) {
  jy_wave_count(atomicOr(K.pflag + s, 1u) == 0u, reinterpret_cast<unsigned long long*>(K.pcount));
  const u64 t0 = ld64<kCoh>(K.ts + s);
  if (t < t0 || !lww_wins<kCoh>(t, t0, p, l, K.val, s, K.arena)) return;
  K.ts[s] = t;
  K.val[s] = TVal{p, l};
  const u64 d0 = ld64<kCoh>(K.pts + s);
  if (t < d0 || !lww_wins<kCoh>(t, d0, p, l, K.pval, s, K.arena)) return;
  K.pts[s] = t;
  K.pval[s] = TVal{p, l};
}

// (the host's bound keeps the list from filling; a record past its capacity
// is never written, the count may pass the capacity but every reader clamps
// it (fold_count), and the overflow word makes the next call fail loudly --
// the state then misses that duplicate, memory is never touched past the
// list).  Returns 1 if pushed, 2 if it overflowed: the wave publishes both
// through dup_publish.
__device__ __forceinline__ u32 push_dup(const TregK& K, u32 s, u64 t, u64 p, u64 l) {
  const u32 at = atomicAdd(K.dupn, 1u);
  if ((u64)at >= K.dup_cap) return 2u;
  u64x2* r = reinterpret_cast<u64x2*>(K.dups + (u64)at * 4);
  r[0] = u64x2{(u64)s, t};
  r[1] = u64x2{p, l};
  return 1u;
}

// An overflow (a push past the list's capacity: a wrong bound) is published
// to a host-mapped word: ONE lane of a wave that overflowed stores it with
// system scope and waits for the store to be performed at system scope
// before the wave may end, so a completed launch's overflow is visible to
// the host (jy_treg_overflow_check).  Called by every lane of the wave
// together; the fence runs only on that path.
__device__ __forceinline__ void dup_publish(const TregK& K, u32 what) {
  const u32 any = jy_wave_or(what);
  if (!(any & 2u) || !K.dupflag) return;
  if (__lane_id() == 0) {
    __hip_atomic_store(K.dupflag + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope: the store above is performed
  }
}

// records a fold may read: the count clamped to the list's capacity (a count
// past it means records were dropped; the overflow word reports that)
__device__ __forceinline__ u64 fold_count(u32 n, u64 cap) { return (u64)n < cap ? (u64)n : cap; }

// this workgroup's slice of the other claim bitmap (16-B stores)
__device__ __forceinline__ void clear_slice(const TregK& K) {
  if (!K.clear) return;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u64 per = ((K.clear_bytes + gridDim.x - 1) / gridDim.x + 15) & ~15ull;
  const u64 b0 = (u64)blockIdx.x * per, b1 = b0 + per < K.clear_bytes ? b0 + per : K.clear_bytes;
  uint8_t* base = reinterpret_cast<uint8_t*>(K.clear);
  for (u64 o = b0 + threadIdx.x * 16; o < b1; o += blockDim.x * 16) *reinterpret_cast<u32x4*>(base + o) = u32x4{0, 0, 0, 0};
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
// kSet: local SETs (RepoTREG.set): the pending delta is updated with the
//   state (set_one); the wide form is used for cache-friendly batches.
// kDense: a block batch -- entry i is slot slot0 + i (slot == nullptr): no
//   slot stream to read, and no slot can repeat, so no claim and no
//   duplicate list either.
// kOwned: a routed sender's batch merged where it lies (jy_treg_route_part_self):
//   only entries whose owner is this shard (own[i] == self) take part, and a
//   slot this shard never handed out is counted as skipped, as a receiver
//   does for routed records.  The owner words are loaded with the rest of
//   the entry (at S shards 1/S of the entries are this shard's, spread over
//   every line: the lines are fetched either way).
struct Owned {
  const u32* own;
  u32 self;
  u64 nslots;
  unsigned long long* skipped;
};
template <bool kRewriteAll, bool kSet, bool kDense = false, bool kOwned = false>
__global__ __launch_bounds__(kThreads) void k_treg_lww(TregK K, const u32* __restrict__ slot,
                                                       const u64* __restrict__ dts, const u64* __restrict__ dpre,
                                                       const u64* __restrict__ dlr, u64 n, u32 slot0 = 0,
                                                       Owned O = Owned{}) {
  // a wave's rows are kUnroll consecutive runs of 64 entries (jy_claim_rows)
  const u64 base = (u64)blockIdx.x * (kThreads * kUnroll) + (threadIdx.x >> 6) * (64 * kUnroll) + (threadIdx.x & 63);
  u32 s[kUnroll];
  u64 t[kUnroll], t0[kUnroll], p[kUnroll], l[kUnroll];
  bool valid[kUnroll], first[kUnroll];
#pragma unroll
  for (int u = 0; u < kUnroll; u++) {
    const u64 i = base + (u64)u * 64;
    valid[u] = i < n;
    s[u] = 0;
    if (valid[u]) {
      s[u] = kDense ? slot0 + (u32)i : __builtin_nontemporal_load(slot + i);
      if (!kDense && !kOwned && s[u] == JY_NO_SLOT) {  // a key with no slot (yet): skipped
        valid[u] = false;
        s[u] = 0;
        continue;
      }
      t[u] = __builtin_nontemporal_load(dts + i);
      p[u] = __builtin_nontemporal_load(dpre + i);
      l[u] = __builtin_nontemporal_load(dlr + i);
      if (kOwned) valid[u] = __builtin_nontemporal_load(O.own + i) == O.self;
    }
  }
  if (kOwned) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
      if (valid[u] && s[u] >= O.nslots) {
        atomicAdd(O.skipped, 1ull);
        valid[u] = false;
        s[u] = 0;
      }
  }
  // <true> (a state streamed from HBM): the old handles come with the state
  // timestamps, in the same round trip -- a loser rewrites its own, and at
  // ~1/3 losers nearly every 64-B handle line holds one, so those lines were
  // fetched anyway (PMC, profiles/r06_pmc_treg.json: 48 B read per key, not
  // the 37 B of ts + loser handles); the decision no longer waits for a
  // second, dependent load
  TVal h0[kRewriteAll && !kSet && JY_TREG_PRELOAD ? kUnroll : 1];
  if (!kSet) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
      if (valid[u]) {
        t0[u] = K.ts[s[u]];
        if constexpr (kRewriteAll && JY_TREG_PRELOAD) h0[u] = K.val[s[u]];
      }
  }
  if (kDense) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++) first[u] = true;
  } else {
    jy_claim_rows<kUnroll>(valid, s, K.seen, first);
    clear_slice(K);
  }
  u32 pushed = 0;
#pragma unroll
  for (int u = 0; u < kUnroll; u++) {
    if (!valid[u]) continue;
    if (!kDense && !first[u]) {
      pushed |= push_dup(K, s[u], t[u], p[u], l[u]);
      continue;
    }
    if (kSet) {
      set_one(K, s[u], t[u], p[u], l[u]);
      continue;
    }
    if constexpr (kRewriteAll && JY_TREG_PRELOAD) {
      const bool w = t[u] > t0[u] || (t[u] == t0[u] && jy_value_cmp(p[u], l[u], h0[u].pre, h0[u].lr, K.arena) > 0);
      K.ts[s[u]] = w ? t[u] : t0[u];
      K.val[s[u]] = w ? TVal{p[u], l[u]} : h0[u];
      continue;
    }
    const bool w = t[u] >= t0[u] && lww_wins(t[u], t0[u], p[u], l[u], K.val, s[u], K.arena);
    K.ts[s[u]] = w ? t[u] : t0[u];
    if (kRewriteAll) {
      const TVal old = w ? TVal{0, 0} : K.val[s[u]];
      K.val[s[u]] = w ? TVal{p[u], l[u]} : old;
    } else if (w) {
      K.val[s[u]] = TVal{p[u], l[u]};
    }
  }
  if (!kDense) dup_publish(K, pushed);
}

// Routed runs (receiver side of the exchange, k_route.hip): one source's run
// per launch, 32-B records {slot on this owner, ts, pre, lr'} at recs[0 ..],
// hdr[0] of them (counts travel with the data: no host round trip).  A hole
// (slot ~0) is a record whose value bytes overflowed the sender's byte run;
// a slot this shard never handed out is counted as skipped.  lr' offsets are
// relative to the source's byte run, which sits at arena offset `rebase`.
struct RoutedIn {
  const u64* recs;
  const u64* hdr;
  u64 cap, rebase, nslots;
  unsigned long long* skipped;
};

__device__ __forceinline__ bool routed_get(const RoutedIn& R, u64 cnt, u64 i, u32& s, u64& t, u64& p, u64& l) {
  if (i >= cnt) return false;
  const u64x2 a = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(R.recs + i * 4));
  const u64x2 b = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(R.recs + i * 4) + 1);
  if (a.x == ~0ull) return false;  // hole
  if (a.x >= R.nslots) {
    atomicAdd(R.skipped, 1ull);
    return false;
  }
  s = (u32)a.x;
  t = a.y;
  p = b.x;
  l = b.y;
  if ((l & JY_LR_LEN_MASK) > 8) l = (((l >> JY_LR_LEN_BITS) + R.rebase) << JY_LR_LEN_BITS) | (l & JY_LR_LEN_MASK);
  return true;
}

// (Measured and dropped in round 3, in-box A/B of the routed TREG step: four
// records per lane, each record loaded together with its run's count, every
// record rewriting its ts word -- 0.352 vs 0.341 ms together; separately, the
// ts rewrite 0.332 and four records per lane 0.333 vs 0.330 ms.)
#ifndef JY_TREG_ROUTED_U
#define JY_TREG_ROUTED_U 2
#endif
constexpr int kRoutedU = JY_TREG_ROUTED_U;  // records per lane
__global__ __launch_bounds__(kThreads) void k_treg_lww_routed(TregK K, RoutedIn R) {
  constexpr int U = kRoutedU;
  const u64 base = (u64)blockIdx.x * (kThreads * U) + (threadIdx.x >> 6) * (64 * U) + (threadIdx.x & 63);
  const u64 cnt = R.hdr[0] < R.cap ? R.hdr[0] : R.cap;
  u32 s[U];
  u64 t[U], p[U], l[U], t0[U];
  bool valid[U], first[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 64;
    s[u] = 0;
    valid[u] = routed_get(R, cnt, i, s[u], t[u], p[u], l[u]);
  }
#pragma unroll
  for (int u = 0; u < U; u++)
    if (valid[u]) t0[u] = K.ts[s[u]];
  jy_claim_rows<U>(valid, s, K.seen, first);
  clear_slice(K);
  u32 pushed = 0;
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (!valid[u]) continue;
    if (!first[u]) {
      pushed |= push_dup(K, s[u], t[u], p[u], l[u]);
      continue;
    }
    if (t[u] >= t0[u] && lww_wins(t[u], t0[u], p[u], l[u], K.val, s[u], K.arena)) {
      K.ts[s[u]] = t[u];
      K.val[s[u]] = TVal{p[u], l[u]};
    }
  }
  dup_publish(K, pushed);
}

// The rest of a duplicate list, folded in by ONE wave: a chunk of 64 records
// per pass (lane = record); records of one slot inside a chunk run in rounds
// by their rank among the chunk's records of that slot, so no two lanes
// touch a slot at once and chunks run in list order.
template <bool kSet>
__device__ void fold_wave(const TregK& K, const u64* __restrict__ list, u32 n) {
  const int lane = threadIdx.x;
  for (u32 j0 = 0; j0 < n; j0 += 64) {
    const u32 j = j0 + lane;
    const bool live = j < n;
    u32 s = 0xFFFFFFFFu;
    u64 t = 0, p = 0, l = 0;
    if (live) {
      const u64x2 a = reinterpret_cast<const u64x2*>(list + (u64)j * 4)[0];
      const u64x2 b = reinterpret_cast<const u64x2*>(list + (u64)j * 4)[1];
      s = (u32)a.x;
      t = a.y;
      p = b.x;
      l = b.y;
    }
    u32 rank = 0;
    for (int k = 0; k < 64; k++) {
      const u32 sk = __shfl(s, k);
      if (k < lane && sk == s) rank++;
    }
    u32 rounds = live ? rank + 1 : 0;
    for (int o = 32; o > 0; o >>= 1) rounds = max(rounds, (u32)__shfl_xor(rounds, o));
    for (u32 r = 0; r < rounds; r++) {
      if (live && rank == r) {
        if (kSet) {
          set_one<true>(K, s, t, p, l);
        } else {
          const u64 t0 = ld64<true>(K.ts + s);
          if (t >= t0 && lww_wins<true>(t, t0, p, l, K.val, s, K.arena)) {
            K.ts[s] = t;
            K.val[s] = TVal{p, l};
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0);  // this round's stores land before the next round reads
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// The fold: kFoldRounds ordinary launches and a one-wave tail, in stream
// order behind the merges that pushed the records (the kernel boundaries are
// the barriers between rounds).  Round r reads list r's count from the
// device -- an empty list (the usual case) returns in every workgroup at
// once -- merges the first record of every slot and pushes the others to
// list r + 1.  The first record is found with a claim word per slot holding
// the round's epoch (a number the host never reuses until it resets the
// words), so no round clears anything.  Counts: cnt[0] is the pending list's,
// cnt[1..kFoldRounds] the rounds' outputs (all zero between folds; the tail
// zeroes them); the records alternate between the two lists.
constexpr int kFoldRounds = 3;
struct FoldK {
  TregK K;       // state (and the pending registers for kSet)
  u32* cin;      // this round's input count and list
  const u64* lin;
  u32* claim;    // per slot: the epoch of the round that last claimed it
  u32 epoch;
};
template <bool kSet>
__global__ __launch_bounds__(kThreads) void k_treg_fold_round(FoldK F) {
  constexpr int U = 2;
  const u64 n = fold_count(*F.cin, F.K.dup_cap);
  if (n == 0) return;
  const TregK& K = F.K;  // K.dupn / K.dups: the round's output list
  u32 pushed = 0;
  for (u64 b0 = (u64)blockIdx.x * (kThreads * U); b0 < n; b0 += (u64)gridDim.x * (kThreads * U)) {
    const u64 base = b0 + (threadIdx.x >> 6) * (64 * U) + (threadIdx.x & 63);
    u32 s[U];
    u64 t[U], p[U], l[U];
    bool valid[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const u64 i = base + (u64)u * 64;
      valid[u] = i < n;
      s[u] = 0;
      if (valid[u]) {
        const u64x2 a = reinterpret_cast<const u64x2*>(F.lin + i * 4)[0];
        const u64x2 b = reinterpret_cast<const u64x2*>(F.lin + i * 4)[1];
        s[u] = (u32)a.x;
        t[u] = a.y;
        p[u] = b.x;
        l[u] = b.y;
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (!valid[u]) continue;
      if (atomicExch(F.claim + s[u], F.epoch) == F.epoch) {  // not the slot's first record this round
        pushed |= push_dup(K, s[u], t[u], p[u], l[u]);
        continue;
      }
      if (kSet) {
        set_one(K, s[u], t[u], p[u], l[u]);
      } else {
        const u64 t0 = K.ts[s[u]];
        if (t[u] >= t0 && lww_wins(t[u], t0, p[u], l[u], K.val, s[u], K.arena)) {
          K.ts[s[u]] = t[u];
          K.val[s[u]] = TVal{p[u], l[u]};
        }
      }
    }
  }
  dup_publish(K, pushed);
}

// the tail: one wave folds what the rounds left (a slot repeated more than
// kFoldRounds times in the list) and zeroes every count
template <bool kSet>
__global__ __launch_bounds__(64) void k_treg_fold_tail(TregK K, u32* cnt0, u32* rcnt, const u64* list) {
  const u64 n = fold_count(rcnt[kFoldRounds - 1], K.dup_cap);
  if (n) fold_wave<kSet>(K, list, (u32)n);
  if (threadIdx.x == 0) {
    *cnt0 = 0;
    for (int r = 0; r < kFoldRounds; r++) rcnt[r] = 0;
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

struct TregPendingPred {
  const u32* dflag;
  __device__ bool operator()(u64 s) const { return dflag[s] != 0; }
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

TregK state_of(jy_engine* eng) {
  TregState& t = eng->treg;
  TregK K{};
  K.ts = t.ts;
  K.val = t.val;
  K.arena = eng->arena[JY_TREG].p;
  K.dupn = t.dupn;
  K.dups = t.dups;
  K.dupflag = t.dupflag_dev;
  K.dup_cap = t.dup_cap;
  return K;
}

}  // namespace

int32_t jy_treg_overflow_check(jy_engine* eng) {
  const TregState& t = eng->treg;
  if (t.dupflag && __atomic_load_n(t.dupflag + 1, __ATOMIC_ACQUIRE) != 0)
    return eng->fail(JY_ERANGE, "treg duplicate list overflowed (a bound was wrong): state may miss duplicates");
  return JY_OK;
}

namespace {
int32_t overflow_check(jy_engine* eng) { return jy_treg_overflow_check(eng); }

// the host-mapped overflow word (dupflag[1], dup_publish)
int32_t flag_init(jy_engine* eng) {
  TregState& t = eng->treg;
  if (t.dupflag) return JY_OK;
  void* h = nullptr;
  JY_HIP(eng, hipHostMalloc(&h, 64, hipHostMallocMapped));
  std::memset(h, 0, 64);
  void* d = nullptr;
  JY_HIP(eng, hipHostGetDevicePointer(&d, h, 0));
  t.dupflag = static_cast<u32*>(h);
  t.dupflag_dev = static_cast<u32*>(d);
  return JY_OK;
}

// the claim bitmaps of one launch: this launch's (clean) and the other one,
// which the launch clears (or a memset, for a grid too small to clear it)
int32_t claim_bits(jy_engine* eng, u32 nblocks, TregK& K) {
  TregState& t = eng->treg;
  K.seen = t.seen[t.parity];
  const u64 bytes = ((t.seen_words * 4 + 15) & ~15ull);
  if (bytes > (u64)nblocks * 4096) {
    JY_HIP(eng, hipMemsetAsync(t.seen[t.parity ^ 1], 0, bytes, eng->stream));
    K.clear = nullptr;
    K.clear_bytes = 0;
  } else {
    K.clear = t.seen[t.parity ^ 1];
    K.clear_bytes = bytes;
  }
  t.parity ^= 1;
  return JY_OK;
}

// the second list, the rounds' counts and the fold's claim words (one per
// slot of the register file's capacity)
int32_t fold_bufs(jy_engine* eng) {
  TregState& t = eng->treg;
  if (!t.dups_alt) {
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&t.dups_alt), std::max<u64>(t.dup_cap, 1) * 32,
                        "treg duplicate list"));
  }
  if (!t.dupn_alt) {
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&t.dupn_alt), 64, "treg fold counts"));
    JY_HIP(eng, hipMemsetAsync(t.dupn_alt, 0, 64, eng->stream));
  }
  const u64 slots = t.seen_words * 32;
  if (t.fold_slots < slots || !t.fold_claim) {
    jy_dev_free(eng, t.fold_claim);
    t.fold_claim = nullptr;
    t.fold_slots = slots;
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&t.fold_claim), std::max<u64>(slots, 1) * 4,
                        "treg fold claim words"));
    JY_HIP(eng, hipMemsetAsync(t.fold_claim, 0, std::max<u64>(slots, 1) * 4, eng->stream));
    t.fold_epoch = 0;
  }
  return JY_OK;
}

// the fold (stream order): kFoldRounds round launches and the tail; with
// nothing pushed every launch reads a zero count and returns.  Round 0's grid
// covers the records that may be pending (dup_bound); later rounds hold the
// repeats of repeats, a small grid strides over them.
int32_t fold_launch(jy_engine* eng, bool set) {
  TregState& t = eng->treg;
  if (!t.dups) return JY_OK;  // nothing was ever claimed
  JY_TRY(fold_bufs(eng));
  if (t.fold_epoch > 0xFFFFFFF0u) {  // epochs are never reused: reset the words
    JY_HIP(eng, hipMemsetAsync(t.fold_claim, 0, std::max<u64>(t.fold_slots, 1) * 4, eng->stream));
    t.fold_epoch = 0;
  }
  TregK K = state_of(eng);
  if (set) {
    K.pts = t.dts;
    K.pval = t.dval;
    K.pflag = t.dflag;
    K.pcount = t.dcount;
  }
  u32* cnt[kFoldRounds + 1];
  cnt[0] = t.dupn;
  for (int r = 1; r <= kFoldRounds; r++) cnt[r] = t.dupn_alt + (r - 1);
  u64* lst[2] = {t.dups, t.dups_alt};
  const u64 pending = std::min<u64>(t.dup_bound, t.dup_cap);
  for (int r = 0; r < kFoldRounds; r++) {
    FoldK F{};
    F.K = K;
    F.K.dupn = cnt[r + 1];
    F.K.dups = lst[(r + 1) & 1];
    F.cin = cnt[r];
    F.lin = lst[r & 1];
    F.claim = t.fold_claim;
    F.epoch = ++t.fold_epoch;
    // round 0 strides too: an empty round (the usual case) costs its grid's
    // dispatch, ~1 us at 1024 workgroups against ~3.5 us at 4096
    const u32 grid = r == 0 ? std::min<u32>(blocks(pending, kThreads * 2), 1024) : 256;
    if (set)
      hipLaunchKernelGGL(k_treg_fold_round<true>, dim3(grid), dim3(kThreads), 0, eng->stream, F);
    else
      hipLaunchKernelGGL(k_treg_fold_round<false>, dim3(grid), dim3(kThreads), 0, eng->stream, F);
    JY_HIP(eng, hipGetLastError());
  }
  if (set)
    hipLaunchKernelGGL(k_treg_fold_tail<true>, dim3(1), dim3(64), 0, eng->stream, K, t.dupn, t.dupn_alt,
                       lst[kFoldRounds & 1]);
  else
    hipLaunchKernelGGL(k_treg_fold_tail<false>, dim3(1), dim3(64), 0, eng->stream, K, t.dupn, t.dupn_alt,
                       lst[kFoldRounds & 1]);
  JY_HIP(eng, hipGetLastError());
  t.dup_bound = 0;
  return JY_OK;
}

// fold the pending converge duplicates now: before a read, a SET batch
// (whose pending-delta test must see them), an arena move, or when the list
// could fill
int32_t fold_now(jy_engine* eng) {
  TregState& t = eng->treg;
  if (t.dup_bound == 0) return JY_OK;
  return fold_launch(eng, false);
}

// claim state of one launch over n entries: room for n more duplicates
// (folding the list first when the bound says it might overflow), this
// launch's bitmap and the other one to clear
// JY_CFG_TREG_DUP_TEST: a fixed list of this many records that the host
// never folds or grows ahead of time, so a test can overflow it on purpose
constexpr u64 kDupTestCap = 64;

int32_t claim_begin(jy_engine* eng, u64 n, u32 nblocks, TregK& K) {
  TregState& t = eng->treg;
  JY_TRY(flag_init(eng));
  JY_TRY(overflow_check(eng));
  if (eng->cfg.flags & JY_CFG_TREG_DUP_TEST) {
    if (!t.dups) {
      JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&t.dups), kDupTestCap * 32, "treg duplicate list"));
      JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&t.dups_alt), kDupTestCap * 32, "treg duplicate list"));
      t.dup_cap = kDupTestCap;
      JY_TRY(fold_bufs(eng));
    }
    K = state_of(eng);
    JY_TRY(claim_bits(eng, nblocks, K));
    t.dup_bound += n;
    return JY_OK;
  }
  if (t.dup_bound + n > t.dup_cap) {
    // the list could fill: fold it first (one launch; nothing to do on the
    // device when no duplicate was pushed, the usual case)
    JY_TRY(fold_now(eng));
    if (n > t.dup_cap) {
      const u64 cap = std::max<u64>(4 * n, 1 << 16);
      jy_dev_free(eng, t.dups);
      jy_dev_free(eng, t.dups_alt);
      t.dups = t.dups_alt = nullptr;
      t.dup_cap = 0;
      JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&t.dups), cap * 32, "treg duplicate list"));
      JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&t.dups_alt), cap * 32, "treg duplicate list"));
      t.dup_cap = cap;
      JY_TRY(fold_bufs(eng));
    }
  }
  K = state_of(eng);
  JY_TRY(claim_bits(eng, nblocks, K));
  t.dup_bound += n;
  return JY_OK;
}

}  // namespace

// pending duplicates folded in (before an arena collection moves values)
int32_t jy_treg_fold(jy_engine* eng) { return fold_now(eng); }

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
  // the pending duplicates hold slots of the old capacity: fold them first;
  // then two claim bitmaps (one bit per slot), both zero
  JY_TRY(fold_now(eng));
  for (auto& b : t.seen) jy_dev_free(eng, b);
  t.seen_words = (nk + 31) / 32;
  for (auto& b : t.seen) {
    void* sp = nullptr;
    JY_TRY(jy_dev_alloc(eng, &sp, (t.seen_words + 16) * 4, "treg claim bitmap"));
    b = static_cast<u32*>(sp);
    JY_HIP(eng, hipMemsetAsync(b, 0, (t.seen_words + 16) * 4, eng->stream));
  }
  if (!t.dupn) {
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&t.dupn), 64, "treg duplicate count"));
    JY_HIP(eng, hipMemsetAsync(t.dupn, 0, 64, eng->stream));
  }
  return JY_OK;
}

int32_t jy_treg_merge(jy_engine* eng, u64 n, const u32* slot, const u64* ts, const u64* pre, const u64* lr) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  JyTimed tm(eng);
  const u32 grid = blocks(n, kThreads * kUnroll);
  TregK K{};
  JY_TRY(claim_begin(eng, n, grid, K));
  // state larger than the Infinity Cache: write whole lines (see k_treg_lww);
  // config flag JY_CFG_TREG_WHOLE_LINES forces that form (tests)
  const bool whole =
      t.kcap * (8 + sizeof(TVal)) > kMallBytes || (eng->cfg.flags & JY_CFG_TREG_WHOLE_LINES) != 0;
  if (whole)
    hipLaunchKernelGGL((k_treg_lww<true, false>), dim3(grid), dim3(kThreads), 0,
                       eng->stream, K, slot, ts, pre, lr, n);
  else
    hipLaunchKernelGGL((k_treg_lww<false, false>), dim3(grid), dim3(kThreads), 0,
                       eng->stream, K, slot, ts, pre, lr, n);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

// the entries of a routed sender's batch that this shard owns (own[i] ==
// self), merged in place: a shard's share of its own batch never enters a run
int32_t jy_treg_merge_owned(jy_engine* eng, u64 n, const u32* own, u32 self, const u32* slot, const u64* ts,
                            const u64* pre, const u64* lr) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  JyTimed tm(eng);
  const u32 grid = blocks(n, kThreads * kUnroll);
  TregK K{};
  JY_TRY(claim_begin(eng, n, grid, K));
  const Owned O{own, self, eng->nkeys[JY_TREG], reinterpret_cast<unsigned long long*>(eng->skipped_dev)};
  const bool whole =
      t.kcap * (8 + sizeof(TVal)) > kMallBytes || (eng->cfg.flags & JY_CFG_TREG_WHOLE_LINES) != 0;
  if (whole)
    hipLaunchKernelGGL((k_treg_lww<true, false, false, true>), dim3(grid), dim3(kThreads), 0, eng->stream, K, slot,
                       ts, pre, lr, n, 0u, O);
  else
    hipLaunchKernelGGL((k_treg_lww<false, false, false, true>), dim3(grid), dim3(kThreads), 0, eng->stream, K, slot,
                       ts, pre, lr, n, 0u, O);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

// a block batch: entry i merges into slot slot0 + i.  No claim, no duplicate
// list: the claim bitmaps' parity is left as it is (the next keyed launch
// still finds its bitmap clean).
int32_t jy_treg_merge_block(jy_engine* eng, u32 slot0, u64 n, const u64* ts, const u64* pre, const u64* lr) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  JyTimed tm(eng);
  const u32 grid = blocks(n, kThreads * kUnroll);
  JY_TRY(flag_init(eng));
  JY_TRY(overflow_check(eng));
  TregK K = state_of(eng);
  const bool whole =
      t.kcap * (8 + sizeof(TVal)) > kMallBytes || (eng->cfg.flags & JY_CFG_TREG_WHOLE_LINES) != 0;
  if (whole)
    hipLaunchKernelGGL((k_treg_lww<true, false, true>), dim3(grid), dim3(kThreads), 0, eng->stream, K, nullptr, ts,
                       pre, lr, n, slot0);
  else
    hipLaunchKernelGGL((k_treg_lww<false, false, true>), dim3(grid), dim3(kThreads), 0, eng->stream, K, nullptr, ts,
                       pre, lr, n, slot0);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_treg_merge_routed(jy_engine* eng, u32 S, u64 cap, u64 cap_byte, const u64* recs, const u64* hdr,
                             u64 rebase) {
  if ((u64)S * cap == 0) return JY_OK;
  JyTimed tm(eng);
  // one source's run per launch: a key that several peers flushed in the same
  // step is merged launch after launch (stream order), never a duplicate
  const u32 grid = blocks(cap, kThreads * kRoutedU);
  for (u32 src = 0; src < S; src++) {
    TregK K{};
    JY_TRY(claim_begin(eng, cap, grid, K));
    RoutedIn R{recs + (u64)src * cap * 4, hdr + 2 * (u64)src, cap, rebase + (u64)src * cap_byte,
               eng->nkeys[JY_TREG], reinterpret_cast<unsigned long long*>(eng->skipped_dev)};
    hipLaunchKernelGGL(k_treg_lww_routed, dim3(grid), dim3(kThreads), 0, eng->stream, K, R);
    JY_HIP(eng, hipGetLastError());
  }
  return JY_OK;
}

int32_t jy_treg_gather(jy_engine* eng, u64 n, const u32* slots, u64* ots, u64* opre, u64* olr) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  // the fold is memory-safe after an overflow (fold_count); the caller
  // reports the overflow once the launches before it have finished
  // (jy_treg_read after its read-back; a merge's claim_begin)
  JY_TRY(fold_now(eng));
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

// local SET batch (RepoTREG.set repo_treg.pony:65-68): every entry updates
// the state and, if it wins there, the key's pending delta.  A SET's pending
// test must see the state as the reference would, so converge duplicates
// still pending are folded first, and the batch's own repeated keys are
// folded right after it (SET semantics) rather than later.
int32_t jy_treg_set_batch(jy_engine* eng, u64 n, const u32* slot, const u64* ts, const u64* pre, const u64* lr) {
  if (n == 0) return JY_OK;
  TregState& t = eng->treg;
  JY_TRY(treg_delta_grow(eng));
  JyTimed tm(eng);
  JY_TRY(fold_now(eng));
  const u32 grid = blocks(n, kThreads * kUnroll);
  TregK K{};
  JY_TRY(claim_begin(eng, n, grid, K));
  K.pts = t.dts;
  K.pval = t.dval;
  K.pflag = t.dflag;
  K.pcount = t.dcount;
  hipLaunchKernelGGL((k_treg_lww<false, true>), dim3(grid), dim3(kThreads), 0, eng->stream, K, slot, ts, pre, lr, n);
  JY_HIP(eng, hipGetLastError());
  return fold_launch(eng, true);  // the batch's own repeats, with SET semantics
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
  void* num = nullptr;
  JY_TRY(jy_scratch(eng, 14, 8, &num));
  JY_TRY(jydscan::select(eng, nkeys, TregPendingPred{t.dflag}, slots, static_cast<u32*>(num)));
  hipLaunchKernelGGL(k_treg_flush, dim3(blocks(cnt, kThreads)), dim3(kThreads), 0, eng->stream, t.dflag, t.dts,
                     t.dval, (const u32*)slots, cnt, ots, opre, olr);
  JY_HIP(eng, hipGetLastError());
  JY_HIP(eng, hipMemsetAsync(t.dcount, 0, 8, eng->stream));
  return JY_OK;
}
