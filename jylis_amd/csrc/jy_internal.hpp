// jy_internal.hpp -- engine internals shared by the HIP translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/jylis_gpu.h"

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;

#define JY_LR_LEN_BITS 24
#define JY_LR_LEN_MASK ((1ull << JY_LR_LEN_BITS) - 1)
#define JY_MAX_VALUE_LEN JY_LR_LEN_MASK
#define JY_DOT_SEQ_BITS 48
#define JY_DOT_SEQ_MASK ((1ull << JY_DOT_SEQ_BITS) - 1)

// ---------------------------------------------------------------------------
// Device-side helpers

// Pony String order on (prefix, lr) handles: unsigned bytewise, then length.
// prefix = first 8 bytes big-endian zero-padded, so unsigned prefix order is
// bytewise order of the first min(8, len) bytes up to zero padding; the
// arena holds the whole value when len > 8.
// (the arena bytes from `from` on, both values longer than `from`: equal
// before it)
__device__ __forceinline__ int jy_value_cmp_tail(u64 la, u64 lb, const uint8_t* __restrict__ arena, u64 from) {
  const u64 na = la & JY_LR_LEN_MASK, nb = lb & JY_LR_LEN_MASK;
  {
    const uint8_t* a = arena + (la >> JY_LR_LEN_BITS);
    const uint8_t* b = arena + (lb >> JY_LR_LEN_BITS);
    const u64 n = na < nb ? na : nb;
    // 8 bytes per step, all 16 loads of a step issued together (one memory
    // round trip per step instead of one per byte); bytes past n read as 0
    for (u64 i = from; i < n; i += 8) {
      u64 wa = 0, wb = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const bool in = i + q < n;
        const u64 xa = in ? a[i + q] : 0, xb = in ? b[i + q] : 0;
        wa = (wa << 8) | xa;
        wb = (wb << 8) | xb;
      }
      if (wa != wb) return wa < wb ? -1 : 1;
    }
  }
  // equal common bytes: the shorter one is a prefix of the other
  if (na == nb) return 0;
  return na < nb ? -1 : 1;
}
__device__ __forceinline__ int jy_value_cmp(u64 pa, u64 la, u64 pb, u64 lb, const uint8_t* __restrict__ arena) {
  if (pa != pb) return pa < pb ? -1 : 1;
  const u64 na = la & JY_LR_LEN_MASK, nb = lb & JY_LR_LEN_MASK;
  if (na > 8 && nb > 8) return jy_value_cmp_tail(la, lb, arena, 8);
  // equal prefix, one side <= 8 bytes: the shorter one is a prefix of the other
  if (na == nb) return 0;
  return na < nb ? -1 : 1;
}

// a value's second word: bytes 8..15 big-endian, zero-padded (0 for values
// of up to 8 bytes).  Values over 8 bytes start on 8-byte arena granules, so
// this is one aligned load inside the value's own granules.
__device__ __forceinline__ u64 jy_value_w2(u64 lr, const uint8_t* __restrict__ arena) {
  const u64 n = lr & JY_LR_LEN_MASK;
  if (n <= 8) return 0;
  u64 w = *reinterpret_cast<const u64*>(arena + (lr >> JY_LR_LEN_BITS) + 8);
  if (n < 16) w &= (1ull << (8 * (n - 8))) - 1;
  return __builtin_bswap64(w);
}
// the same order with both values' second words at hand (TLOG records
// carry theirs): values of up to 16 bytes never touch the arena
__device__ __forceinline__ int jy_value_cmp_w(u64 pa, u64 wa, u64 la, u64 pb, u64 wb, u64 lb,
                                              const uint8_t* __restrict__ arena) {
  if (pa != pb) return pa < pb ? -1 : 1;
  const u64 na = la & JY_LR_LEN_MASK, nb = lb & JY_LR_LEN_MASK;
  if (na > 8 && nb > 8) {
    if (wa != wb) return wa < wb ? -1 : 1;
    if (na > 16 && nb > 16) return jy_value_cmp_tail(la, lb, arena, 16);
  }
  if (na == nb) return 0;
  return na < nb ? -1 : 1;
}

// include/jylis_gpu.h jy_key_owner on the device: FNV-1a 64 over the key
// bytes, splitmix64 finaliser, mod S (the node's key sharding)
// the first min(8, avail) bytes at p as a little-endian word, zero filled,
// from at most two aligned 8-byte loads (never touching an aligned word that
// holds none of the bytes asked for, so never a page the bytes do not share)
__device__ __forceinline__ u64 jy_ld8u(const uint8_t* p, u64 avail) {
  if (avail == 0) return 0;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const u32 sh = (u32)(a & 7);
  const u64* w = reinterpret_cast<const u64*>(a - sh);
  u64 v = w[0] >> (8 * sh);
  if (sh && avail > 8 - sh) v |= w[1] << (64 - 8 * sh);
  if (avail < 8) v &= (1ull << (8 * avail)) - 1;
  return v;
}

// (the key's bytes read a word at a time: jy_ld8u; the first two words are
// loaded together, before any byte is hashed -- one round trip for keys of
// up to 16 bytes)
__device__ __forceinline__ u32 jy_dev_key_owner(const uint8_t* __restrict__ p, u64 len, u32 S) {
  u64 h = 0xCBF29CE484222325ull;
  const u64 w0 = jy_ld8u(p, len), w1 = len > 8 ? jy_ld8u(p + 8, len - 8) : 0ull;
  for (u64 i = 0; i < len; i += 8) {
    const u64 w = i == 0 ? w0 : i == 8 ? w1 : jy_ld8u(p + i, len - i);
    const u64 m = len - i < 8 ? len - i : 8;
    for (u64 b = 0; b < m; b++) {
      h ^= (w >> (8 * b)) & 0xFFu;
      h *= 0x100000001B3ull;
    }
  }
  h ^= h >> 30;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 27;
  h *= 0x94D049BB133111EBull;
  h ^= h >> 31;
  return (u32)(h % S);
}

// adds the number of active lanes with f to *c: one atomic per wave (a
// same-address atomic per lane serialises at L2, ~15 ns each)
__device__ __forceinline__ void jy_wave_count(bool f, unsigned long long* c) {
  const unsigned long long m = __ballot(f);
  if (m && (unsigned)__lane_id() == (unsigned)(__ffsll(m) - 1)) atomicAdd(c, (unsigned long long)__popcll(m));
}

__device__ __forceinline__ u32 jy_wave_or(u32 x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o);
  return x;
}

// ---- first-occurrence claims: exact handling of a slot named twice in one launch
// `bits` holds one bit per slot and is zero before the launch.  For each of
// the U rows of a wave (one entry per lane per row), first[u] is true iff the
// lane's entry is the FIRST entry of its slot in the whole launch: the one
// whose atomicOr set the slot's bit.  Every lane of the wave calls this
// together.  A batch in slot order (a flush, a routed run) puts a row's 64
// entries on two or three bitmap words, so the row's distinct words are
// walked with ballots (at most kAgg) and each is claimed by ONE atomicOr of
// the OR of its lanes' bits; lanes left over (scattered slots, or two lanes
// of a row on one slot) claim with one atomicOr each -- the memory side
// orders those, so exactly one entry of a slot sees its bit clear.  Every
// atomic of all U rows is issued before any result is consumed.
// JY_CLAIM_MODE (build-time A/B switch, tools/ and DESIGN.md): 2 = walk the
// row's words (default), 1 = one atomicOr per lane, 0 = no claim (UNSAFE:
// measures the claim's cost only; never shipped)
#ifndef JY_CLAIM_MODE
#define JY_CLAIM_MODE 2
#endif
template <int U, int kAgg = 3>
__device__ __forceinline__ void jy_claim_rows(const bool (&valid)[U], const u32 (&s)[U], u32* __restrict__ bits,
                                              bool (&first)[U]) {
  if (JY_CLAIM_MODE == 0) {
#pragma unroll
    for (int u = 0; u < U; u++) first[u] = valid[u];
    return;
  }
  const int lane = __lane_id();
  // Fast path: callers lay a wave's rows out as U consecutive runs of 64
  // entries (row u, lane l = entry wave_base + 64u + l).  When those U * 64
  // entries name the consecutive slots s0 .. s0 + 64U - 1 (a dense batch in
  // slot order: a flush, the bench), their bitmap words and masks follow
  // from s0 alone: one atomicOr instruction with one lane per word.
  {
    const u32 s0 = __shfl(s[0], 0);
    bool contig = true;
#pragma unroll
    for (int u = 0; u < U; u++) contig = contig && valid[u] && s[u] == s0 + (u32)(u * 64 + lane);
    if (__ballot(!contig) == 0) {
      const u32 last = s0 + (u32)(U * 64 - 1), w0 = s0 >> 5;
      u32 old = 0;
      if ((u32)lane <= (last >> 5) - w0) {
        const u32 w = w0 + lane;
        const u32 lo = (s0 > w * 32 ? s0 - w * 32 : 0), hi = (last < w * 32 + 31 ? last - w * 32 : 31);
        const u32 mask = (hi == 31 ? 0xFFFFFFFFu : ((1u << (hi + 1)) - 1)) & ~((1u << lo) - 1);
        old = atomicOr(bits + w, mask);
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const u32 o = __shfl(old, (int)((s[u] >> 5) - w0));
        first[u] = !(o & (1u << (s[u] & 31)));
      }
      return;
    }
  }
  u32 ret[U][kAgg], own[U];
  int grp[U], ldr[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u32 w = s[u] >> 5, b = 1u << (s[u] & 31);
    grp[u] = -1;
    ldr[u] = 0;
    u64 pending = JY_CLAIM_MODE == 2 ? __ballot(valid[u]) : 0;
#pragma unroll
    for (int k = 0; k < kAgg; k++) {
      ret[u][k] = 0;
      if (pending) {  // wave-uniform
        const int leader = __ffsll((unsigned long long)pending) - 1;
        const u32 d = __shfl(w, leader);
        const bool mine = ((pending >> lane) & 1) && w == d;
        const u64 m = __ballot(mine);
        const u32 orv = jy_wave_or(mine ? b : 0u);
        if ((u32)__popc(orv) == (u32)__popcll(m)) {  // no two lanes of the group on one slot
          if (lane == leader) ret[u][k] = atomicOr(bits + d, orv);
          if (mine) {
            grp[u] = k;
            ldr[u] = leader;
          }
        }
        pending &= ~m;
      }
    }
    own[u] = 0;
    if (valid[u] && grp[u] < 0) own[u] = atomicOr(bits + w, b);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    u32 old = own[u];
#pragma unroll
    for (int k = 0; k < kAgg; k++) {
      const u32 v = __shfl(ret[u][k], ldr[u]);
      if (grp[u] == k) old = v;
    }
    first[u] = valid[u] && !(old & (1u << (s[u] & 31)));
  }
}

// ---------------------------------------------------------------------------
// Host-side engine state

struct DevArray {
  void* p = nullptr;
  u64 bytes = 0;
};

// host cache of the device key directory (String -> slot); the device
// directory is authoritative, the cache only saves round trips
struct KeyIndex {
  std::unordered_map<std::string, u32> map;
};

// device key directory (k_keys.hip)
struct KeyDir {
  uint8_t* bytes = nullptr;  // key bytes in slot order
  u64 blen = 0, bcap = 0;
  u64* kref = nullptr;   // [scap] offset << 24 | length
  u64* khash = nullptr;  // [scap] table hash
  u64* kw = nullptr;     // [scap][2] the key's bytes 0..7 and 8..15, zero filled (the probe's compare words)
  u64 n = 0, scap = 0;   // keys, slot capacity
  u64* table = nullptr;  // [tcap] 8-B entries: tag << 32 | slot (~0 empty)
  u64 tcap = 0;
  u32 lg = 0;
};

struct CounterState {  // GCOUNT (nsigns 1) / PNCOUNT (nsigns 2): slab [sign][col][kcap]
  u64* slab = nullptr;
  u32 ccap = 0;  // column capacity
  u64 kcap = 0;  // slot capacity (column pitch, even)
  // pending local deltas (RepoXXX._deltas, repo_gcount.pony:14): per slot a
  // flag word (bit s = sign s written since the last flush) and the recorded
  // post-write totals [sign][dkcap]; dcount = keys with a pending delta
  u32* dflag = nullptr;
  u64* dval = nullptr;
  u64 dkcap = 0;
  u64* dcount = nullptr;
  int32_t dcol = -1;  // the writing replica's column while deltas are pending
};

// TREG value handle of one slot: first 8 value bytes (big-endian) + arena ref
struct alignas(16) TVal {
  u64 pre, lr;
};

struct TregState {  // per slot: ts u64 (read by every merge) + TVal (written by winners)
  u64* ts = nullptr;
  TVal* val = nullptr;
  u64 kcap = 0;
  // pending local deltas (RepoTREG._deltas, repo_treg.pony:14): a TReg per
  // slot (dts, dval: the LWW max of this replica's winning SETs since the
  // last flush), a flag per slot and the pending-key count
  u64* dts = nullptr;
  TVal* dval = nullptr;
  u32* dflag = nullptr;
  u64 dkcap = 0;
  u64* dcount = nullptr;
  // first-occurrence claims (jy_claim_rows): two bitmaps of one bit per slot
  // used by alternate launches (each launch clears the other one), and the
  // list of non-first entries not yet folded in: count (device), 32-B
  // records, host capacity and an upper bound of the records it holds
  u32* seen[2] = {nullptr, nullptr};
  u64 seen_words = 0;
  int parity = 0;
  u32* dupn = nullptr;
  u64* dups = nullptr;
  u32* dupn_alt = nullptr;  // the fold rounds' output counts; dups_alt the other list (k_treg_fold_round)
  u64* dups_alt = nullptr;
  u64 dup_cap = 0;
  u64 dup_bound = 0;
  // host-mapped: [1] set when a push overflowed the list (a wrong bound:
  // the next call fails loudly)
  u32* dupflag = nullptr;
  u32* dupflag_dev = nullptr;
  // the fold's rounds (k_treg_fold_round): a claim word per slot holding the
  // epoch of the round that last claimed it, and the last epoch handed out
  u32* fold_claim = nullptr;
  u64 fold_slots = 0;
  u32 fold_epoch = 0;
};

// one TLOG entry: 32 B so a lane moves it with two 16-B accesses and an
// entry write is one whole 32-B sector; `pad` holds the value's bytes 8..15
// (jy_value_w2), so values of up to 16 bytes compare without the arena
struct alignas(16) TRec {
  u64 ts, pre, lr;
  u64 pad;
};

// per log: a segment of the entry pool, entries OLDEST FIRST (ascending
// (ts, value)), so the usual delta -- entries newer than the whole log --
// is an append at the tail; a raised cutoff drops a prefix (base moves up).
// The segment also keeps FRONT ROOM: free pool entries just below base (a
// rebuild or compaction leaves some, a cutoff drop adds the dropped prefix),
// so an entry inserted near the oldest end moves the short prefix down instead
// of the whole rest of the log up (k_tlog.hip stage 5).
struct alignas(16) TMeta {
  u64 bf;       // base | front << kBaseBits: pool index of the oldest live entry, front room (saturating)
  u32 len;      // live entries
  u32 cap;      // pool entries reserved from base
  u64 cut;      // cutoff
  u64 newest;   // ts of the newest entry (any value when len == 0)
};
constexpr int kBaseBits = 40;  // 2^40 pool entries (32 TB): never the bound
constexpr u64 kBaseMask = (1ull << kBaseBits) - 1;
constexpr u64 kFrontMax = (1ull << (64 - kBaseBits)) - 1;
__host__ __device__ __forceinline__ u64 tm_base(const TMeta& m) { return m.bf & kBaseMask; }
__host__ __device__ __forceinline__ u64 tm_front(const TMeta& m) { return m.bf >> kBaseBits; }
__host__ __device__ __forceinline__ u64 tm_bf(u64 base, u64 front) {
  return base | ((front < kFrontMax ? front : kFrontMax) << kBaseBits);
}

struct TlogState {  // per-slot segments of one entry pool
  TMeta* meta = nullptr;  // [kcap]
  // [kcap] the oldest surviving timestamp of each log, a HINT for the
  // interpolated searches (k_tlog_tile): kept by the merges that know it, never
  // needed for correctness (a stale hint only costs the search a fallback)
  u64* hint = nullptr;
  // [kcap] each log's update history: epoch << 32 | its length when its
  // segment was last made (a rebuild); 0 = none yet.  Sizes the next segment
  // (k_tlog.hip seg_cap): a log that filled its room fast gets room for
  // kHorizon more merges at the rate it grew
  u64* hist = nullptr;
  TRec* pool = nullptr;   // [pcap]
  u64 pcap = 0;
  u64* ctr = nullptr;     // device: [0] pool entries handed out (bump pointer)
  u64* pin = nullptr;     // pinned, mapped: [0..7] compaction readback, [8 + 4 i ..] merge ring slot i
  u64* pin_dev = nullptr; // device view of pin
  u64 kcap = 0;
  // Merges never wait for the host: k_tlog_commit checks ON THE DEVICE that
  // the merge's rebuilt logs fit the pool.  If they do not, it leaves those
  // keys untouched and copies their deltas into the merge's spill buffer;
  // the host re-merges the spill after a compaction once it sees the flag
  // (the next merge call that finds the merge finished, or any call that
  // reads the store, which waits for it).  A spill buffer per merge in
  // flight; [kSpill] serves the re-merges, which settle synchronously.
  static constexpr int kSpill = 2;
  struct Spill {
    DevArray buf;           // slot u32[nd] | cutoff, offsets u64[nd], [nd + 1] | ts, pre, lr u64[nent]
    u64 nd = 0, nent = 0;   // the merge's batch shape
    u64 seq = 0;            // merge number
    bool busy = false;      // issued, not yet settled
    hipEvent_t done = nullptr;
  };
  Spill spill[kSpill + 1];
  u64 seq = 0;          // merges issued
  u64 compact_seq = 0;  // merges issued before the newest compaction (their readback is stale)
  u64 used = 0;         // bump pointer after the newest settled merge
  u64 spills = 0;       // merges whose rebuilt keys were spilled and re-merged (telemetry)
  u64 compactions = 0;
};

// one UJSON element: (dot, element handle), moved with one 16-B access
struct alignas(16) URec {
  u64 dot, elem;
};

// per document: its segments of the element pool (records ascending by dot)
// and of the cloud pool (dots ascending)
struct alignas(16) UMeta {
  u64 ebase;
  u32 elen, ecap;
  u64 cbase;
  u32 clen, ccap;
};

// ---- UJSON in-place layout of long documents (k_ujson.hip, round 6) ----
// A document of at least UjsonState::long_min elements ("long") keeps ONE
// element run and ONE cloud run PER REPLICA COLUMN in the long pools, each
// with room behind it.  Its UMeta then reads {lid, elen total, kLongMark,
// 0, clen total, kLongMark}: ebase is the long-document id, the totals stay
// exact (sizes, reads and compaction use them).  A converge whose delta is
// append-shaped for such a document (every delta dot above the state's
// context in its column, or already covered and removing nothing; the
// delta's vv adding nothing) appends the new dots at the column runs' tails
// and folds the cloud in place: the state's runs are never read or moved.
constexpr u32 kLongMark = 0xFFFFFFFFu;
struct alignas(16) LCol {  // [lid][R]: column c's runs (pool indices of the long pools)
  u64 ebase;
  u32 elen, ecap;
  u64 cbase;
  u32 clen, ccap;
};
struct alignas(16) LPlan {  // [lid][R]: one converge's plan for column c of a long document
  // epoch << 32 | value, written by single items (k_uj_items / k_uj_flags):
  u64 efs, ece;    // delta elements: first fresh one, end of the column's range
  u64 cfs, cce;    // delta cloud: the same
  u64 nfold;       // fresh cloud dots folded into the vv (an empty cloud run only)
  u64 treq;        // live state elements the delta removes, all in the run's first kTrimSpan (k_uj_items)
  u64 tcut;        // how many the trim removed (k_uj_jobs)
  // written by the document's own thread (k_uj_docs) once it is judged in place:
  u64 erun, crun;  // the runs after this converge (moved when they had to grow)
  u64 eapp, capp;  // where the appended items start
  u32 ecap, ccap;  // the runs' capacities after this converge
  u32 cz, pad;     // the cloud run was empty: fresh dots go to crun + rank (fold mode)
};
// a copy job of the in-place layout (k_uj_jobs), one per document: a
// demotion (long column runs -> a regular run at e / c), the column runs of a
// document in place that had to grow (-> LPlan erun / crun), a trim (e = the
// delta doc), a promotion too long for its wave to copy (the regular run at
// e / c -> the new long column runs)
struct alignas(16) UJob {
  u64 e, c;  // the regular run's element / cloud base (demotion: destination, promotion: source); regrowth, trim: e = the delta doc
  u64 n;     // items to copy (elements + cloud dots)
  u32 what;  // UJobWhat
  u32 lid;
};
enum UJobWhat : u32 { UJ_DEMOTE = 0, UJ_REGROW, UJ_PROMOTE, UJ_TRIM };
// a document in place whose delta removes live elements near the start of a
// column run (a vv entry covering the run's first elements, a context dot of
// an old element): the run's first kTrimSpan elements are compacted towards
// its end in one workgroup (k_uj_jobs), the run's start moves up
constexpr u32 kTrimSpan = 256;
// element (kEl) / cloud entry j of a long document, in the order of a regular
// run (ascending dot = column-major): its index in the long pool
template <bool kEl>
__device__ __forceinline__ u64 uj_long_at(const LCol* lc, u32 R, u64 j) {
  for (u32 c = 0; c < R; c++) {
    const LCol L = lc[c];
    const u64 n = kEl ? L.elen : L.clen;
    if (j < n) return (kEl ? L.ebase : L.cbase) + j;
    j -= n;
  }
  return 0;  // j beyond the document's total: not reached by callers
}

struct UjsonState {  // per-document pool segments + dense vv
  UMeta* meta = nullptr;  // [kcap]
  URec* epool = nullptr;  // element pool
  u64 epcap = 0;
  u64* cpool = nullptr;   // cloud pool
  u64 cpcap = 0;
  URec* spare_e = nullptr;  // the pools a compaction wrote out of (reused by the next one)
  u64 spare_ecap = 0;
  u64* spare_c = nullptr;
  u64 spare_ccap = 0;
  u64* ctr = nullptr;     // device: [0] element bump pointer, [1] cloud bump pointer
  u64* pin = nullptr;     // pinned readback
  u64* vv = nullptr;      // [kcap][R]
  u32 R = 0;
  u64 kcap = 0;
  // converge pipeline (k_ujson.hip): epoch-tagged claims and bad marks (no
  // reset between converges), a zero-between-converges dense delta vv, the
  // launches' tickets, and the host's bounds of pool use
  u32 epoch = 0;
  u64* dptr = nullptr;     // [kcap] epoch << 32 | first delta doc of the slot
  u32* bad = nullptr;      // [dcap] == epoch: the delta doc is skipped
  u64* vvd = nullptr;      // [dcap][R], zero between converges
  u64 dcap = 0;
  u32* tick = nullptr;     // [8] ticket counters of the launches
  u64* pin_dev = nullptr;  // device view of pin: [8 + 2j ..] bump pointers after converge j (mod kRing)
  // converges in flight: converge j records ready[j % kRing] and its worst-
  // case pool use; the host absorbs the newest finished one's exact bump
  // pointers, so it waits only when the pools may really be short
  static constexpr int kRing = 4;
  hipEvent_t ready[kRing] = {};
  u64 ring_e[kRing] = {}, ring_c[kRing] = {};
  // touched state elements / cloud dots of the newest finished converge (pin[2j ..]):
  // sizes the item launches' grids (they stride over any excess)
  u64 pred_ta = 0, pred_tc = 0;
  bool has_pred = false;
  u64 seq = 0, done = 0;               // converges issued / absorbed
  u64 used_e = 0, used_c = 0;          // bump pointers after converge done - 1 (exact)
  u64 live_e = 0, live_c = 0;          // upper bounds of live elements / cloud dots
  DevArray st[6];                      // look-back status words of the scans (zeroed once)
  DevArray tmap;                       // epoch-tagged tile -> doc maps of long segments (zeroed once)
  u64* stats = nullptr;                // [16] cumulative converge counters (jy_ujson_stats[_ext])
  // in-place layout of long documents (LCol above).  ctr[2] / ctr[3]: long
  // pool bump pointers, ctr[4]: long ids handed out, ctr[5]: copy jobs of
  // the converge's demotions, regrowths and trims, ctr[6]: documents to
  // promote, ctr[7]: documents in place.  pin[24 + 3 r ..]: ctr[2..4] as
  // converge r saw them.
  bool allow_long = false;  // this store may promote (the state; never the pending deltas)
  u32 long_min = 0;         // promotion threshold in elements (0: none)
  URec* lpe = nullptr;      // long element pool
  u64 lpe_cap = 0;
  u64* lpc = nullptr;       // long cloud pool
  u64 lpc_cap = 0;
  LCol* lcol = nullptr;     // [lcap][R]
  LPlan* lplan = nullptr;   // [lcap][R] (epoch tags: zeroed once)
  u64 lcap = 0;
  UJob* jobs = nullptr;     // [3 jcap]: demotion / regrowth / trim jobs (two per delta doc at most), promotions (plist order)
  u64 jcap = 0;
  u32* fast = nullptr;      // [dcap] == epoch: the delta doc converges in place
  u32* nf = nullptr;        // [dcap] == epoch: a long doc whose delta is not append-shaped
  u32* plist = nullptr;     // [dcap] delta docs whose merged document is promoted
  u32* flist = nullptr;     // [dcap] delta docs converged in place (ctr[7] of them; U5 commits them)
  u64 long_used_e = 0, long_used_c = 0, long_ids = 0;  // the newest readback of ctr[2..4]
};

struct Arena {
  uint8_t* p = nullptr;
  u64 len = 0, cap = 0;
};

struct jy_engine {
  jy_config cfg;
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own_stream = nullptr;
  hipMemPool_t pool = nullptr;  // the engine's stream-ordered pool (jy_dev_alloc)
  std::string err;
  u64 skipped_host = 0;
  u64* skipped_dev = nullptr;  // device counter of skipped entries

  std::unordered_map<u64, u32> rep_col;
  std::vector<u64> rep_id;

  KeyIndex keys[JY_NTYPES];
  KeyDir kdir[JY_NTYPES];
  u64 nkeys[JY_NTYPES] = {0, 0, 0, 0, 0};
  Arena arena[JY_NTYPES];

  CounterState cnt[2];  // [0] GCOUNT, [1] PNCOUNT
  TregState treg;
  TlogState tlog;
  // TLOG write path: the pending delta logs (repo_tlog.pony _deltas) are a
  // second store of the same layout; tl_dflag marks the keys _delta_for
  // touched since the last flush
  TlogState tlog_d;
  // UJSON write path: pending delta documents (repo_ujson.pony _deltas), a
  // second store of the same layout; uj_dflag marks the docs _delta_for touched
  UjsonState ujson_d;
  u32* uj_dflag = nullptr;
  u64 uj_dkcap = 0;
  u64* uj_dcount = nullptr;
  u32* tl_dflag = nullptr;
  u64 tl_dkcap = 0;
  u64* tl_dcount = nullptr;
  UjsonState ujson;

  // scratch (device) reused across calls, stream-ordered
  // 0-7 staged inputs, 8-14 and 16-23 merge temporaries, 15 scan temp storage
  DevArray scratch[32];
  // TLOG merge: the delta key claiming each slot (kNone between merges; a
  // merge resets only its batch's slots, so no per-merge memset over all keys)
  DevArray tl_claim;    // TLOG slot claims: u64 epoch << 32 | delta key (k_tlog_prep)
  u32 tl_epoch = 0;      // the claims' epoch, one per TLOG merge launch
  DevArray tl_bad;       // TLOG: per delta key, the epoch of the merge that found its slot repeated
  // device-wide scans / selects (jy_dscan.hpp): epoch-tagged look-back words
  DevArray dscan_st;
  u32* dscan_tick = nullptr;
  u32 dscan_epoch = 0;
  // column lists of block merges, kept resident: a routed step cycles
  // through a few lists, and uploading one must not stall the stream
  struct ColList {
    u16* dev = nullptr;
    u16* pin = nullptr;  // the pinned source of the async upload, kept with it
  };
  std::map<std::vector<u16>, ColList> cols_cache;
  // pinned host staging: a ring of regions, so a call only waits for the
  // copies of the call kRing calls ago
  static constexpr int kPinRing = 4;
  struct PinSlot {
    void* p = nullptr;
    u64 bytes = 0;
    hipEvent_t ready = nullptr;  // the region may be overwritten once this fired
  };
  PinSlot pins[kPinRing];
  int pin_slot = 0;
  u64 pin_cursor = 0;
  bool pin_used = false;
  u64* pin_total = nullptr;        // pinned u64[4] for async totals
  // pinned landing area of large device -> host results (slots of a host key
  // batch): DMA here, then a parallel host copy out (host_copy.hip)
  void* pin_rb = nullptr;
  u64* kd_words = nullptr;      // mapped pinned: the key probe's partial sums, written by the GPU
  u64* kd_words_dev = nullptr;  // the same memory as the device addresses it
  u32* kd_done = nullptr;       // device: workgroups of the probe sums that have published theirs
  u64 kd_seq = 0;               // the last probe's completion number (written to kd_words by the GPU)
  u64 pin_rb_bytes = 0;
  hipEvent_t total_ready = nullptr;

  // jy_timing_enable: event pairs around the device work of merge calls
  bool timing = false;
  int tm_depth = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> tm_ev;
  size_t tm_used = 0;

  int32_t fail(int32_t code, const std::string& msg) {
    err = msg;
    return code;
  }
};

// scope guard: records the start/stop events of one timed merge call (the
// outermost guard of nested ones wins)
struct JyTimed {
  jy_engine* eng;
  bool on = false;
  explicit JyTimed(jy_engine* e) : eng(e) {
    if (!eng->timing || eng->tm_depth++ > 0) return;
    if (eng->tm_used == eng->tm_ev.size()) {
      std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
      // timing-only events: no system-scope fence on record (that fence writes
      // back and invalidates the caches, ~19 us between two TREG merges)
      if (hipEventCreateWithFlags(&ev.first, hipEventDisableSystemFence) != hipSuccess ||
          hipEventCreateWithFlags(&ev.second, hipEventDisableSystemFence) != hipSuccess)
        return;
      eng->tm_ev.push_back(ev);
    }
    on = hipEventRecord(eng->tm_ev[eng->tm_used].first, eng->stream) == hipSuccess;
  }
  ~JyTimed() {
    if (!eng->timing) return;
    eng->tm_depth--;
    if (on && hipEventRecord(eng->tm_ev[eng->tm_used].second, eng->stream) == hipSuccess) eng->tm_used++;
  }
};

// JY_TRACE=1 in the environment: host-side timing lines on stderr
// (allocation and synchronisation points of the merge paths)
#include <chrono>
#include <cstdio>
#include <cstdlib>
inline bool jy_tracing() {
  static const bool on = std::getenv("JY_TRACE") != nullptr;
  return on;
}
inline double jy_now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define JY_TRACE(...)                            \
  do {                                           \
    if (jy_tracing()) {                          \
      std::fprintf(stderr, "[jy] " __VA_ARGS__); \
      std::fputc('\n', stderr);                  \
    }                                            \
  } while (0)

#define JY_HIP(eng, call)                                                                       \
  do {                                                                                          \
    hipError_t e_ = (call);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return (eng)->fail(JY_EHIP, std::string(#call) + ": " + hipGetErrorString(e_));        \
  } while (0)

#define JY_TRY(expr)            \
  do {                          \
    int32_t rc_ = (expr);       \
    if (rc_ != JY_OK) return rc_; \
  } while (0)

// engine.hip helpers used by the kernel translation units
int32_t jy_scratch(jy_engine* eng, int idx, u64 bytes, void** out);
int32_t jy_treg_fold(jy_engine* eng);
// long values start on 8-byte granules (an arena collection maps granules)
constexpr u64 kArenaAlign = 8;
int32_t jy_arena_append_dev(jy_engine* eng, int32_t type, const uint8_t* src, u64 bytes, u64* rebase_out);
int32_t jy_arena_ensure(jy_engine* eng, int32_t type, u64 bytes);  // room for `bytes` more, without moving later
// look-back status words for `ntiles` tiles, the ticket counter and a fresh epoch
int32_t jy_dscan_ctx(jy_engine* eng, u64 ntiles, u64** status, u32** tick, u32* epoch);
// copy a borrowed input into device memory if it is on the host; returns a
// device pointer valid in stream order (scratch slot `idx`)
int32_t jy_stage(jy_engine* eng, int idx, const void* src, u64 bytes, int32_t mem, const void** dev_out);
// bracket the jy_stage calls of one API call (pinned staging reuse)
int32_t jy_stage_begin(jy_engine* eng);
int32_t jy_stage_end(jy_engine* eng);
int32_t jy_slots_check(jy_engine* eng, int32_t type, u64 n, const u32* slot, int32_t mem);
int32_t jy_ensure_slots(jy_engine* eng, int32_t type, u64 nkeys);
int32_t jy_realloc(jy_engine* eng, void** p, u64 old_bytes, u64 new_bytes, bool zero_tail);

// kernel-side entry points (k_*.hip)
int32_t jy_counter_grow(jy_engine* eng, int which, u32 need_cols, u64 need_slots);
int32_t jy_counter_coo(jy_engine* eng, int which, int sign, u64 n, const u32* slot, const u16* col, const u64* val);
int32_t jy_counter_coo_keyed(jy_engine* eng, int which, u64 n, u64 nkeys, const u32* kslot, const u32* cell_key,
                             const uint8_t* sign, const u16* col, const u64* val);
int32_t jy_counter_block(jy_engine* eng, int which, u32 ncols, const u16* cols_dev, u32 slot0, u32 nslots,
                         const u64* vals_p, const u64* vals_n);
int32_t jy_counter_sum(jy_engine* eng, int which, u64 n, const u32* slots_dev, u64* out_dev);
int32_t jy_cnt_write(jy_engine* eng, int which, int sign, u16 col, u64 n, const u32* slot_dev,
                         const u64* val_dev);
int32_t jy_cnt_flush(jy_engine* eng, int which, u64 nkeys, u64 cap, u32* slot_dev, u64* vals_dev,
                         u32* mask_dev, u64* count_host);
int32_t jy_cnt_pending(jy_engine* eng, int which, u64* count_host);

int32_t jy_treg_grow(jy_engine* eng, u64 need_slots);
int32_t jy_treg_merge(jy_engine* eng, u64 n, const u32* slot, const u64* ts, const u64* pre, const u64* lr);
int32_t jy_treg_gather(jy_engine* eng, u64 n, const u32* slots, u64* ts, u64* pre, u64* lr);
// JY_ERANGE once a duplicate list overflowed (sticky: the state may miss an update)
int32_t jy_treg_overflow_check(jy_engine* eng);
// routed runs: S sources x cap records (slot, ts, pre, lr'), counts in hdr
// (device, 2 u64 per source); source src's value bytes at arena offset
// rebase + src * cap_byte
int32_t jy_treg_merge_block(jy_engine* eng, u32 slot0, u64 n, const u64* ts, const u64* pre, const u64* lr);
int32_t jy_treg_merge_owned(jy_engine* eng, u64 n, const u32* own, u32 self, const u32* slot, const u64* ts,
                            const u64* pre, const u64* lr);
int32_t jy_treg_merge_routed(jy_engine* eng, u32 S, u64 cap, u64 cap_byte, const u64* recs, const u64* hdr,
                             u64 rebase);
// local SETs: state LWW + pending delta, repeated keys exact
int32_t jy_treg_set_batch(jy_engine* eng, u64 n, const u32* slot, const u64* ts, const u64* pre, const u64* lr);
int32_t jy_treg_pending(jy_engine* eng, u64* count_host);
int32_t jy_treg_flush_dev(jy_engine* eng, u64 nkeys, u64 cap, u32* slot_dev, u64* ts_dev, u64* pre_dev, u64* lr_dev,
                      u64* count_host);

int32_t jy_tlog_grow(jy_engine* eng, u64 need_slots);
int32_t jy_tlog_extend(jy_engine* eng, u64 from, u64 to);
int32_t jy_tlog_sizes(jy_engine* eng, u64 n, const u32* slots, u64* len, u64* cut);
int32_t jy_tlog_gather(jy_engine* eng, u64 n, const u32* slots, const u64* ooff, u64* ts, u64* pre, u64* lr);
int32_t jy_tlog_merge(jy_engine* eng, u64 nkeys, const u32* slot, const u64* cutoff, const u64* offs, u64 nent,
                      const u64* ts, const u64* pre, const u64* lr);
struct TlogState;
int32_t jy_tlog_merge_into(jy_engine* eng, TlogState& t, u64 nd, const u32* slot, const u64* dcut, const u64* doff,
                           u64 nent, const u64* dts, const u64* dpre, const u64* dlr);
// wait for every TLOG merge in flight (state and pending stores) and re-merge
// any spilled rebuilds: every call that reads a TLOG store goes through this
int32_t jy_tlog_settle(jy_engine* eng);
// TLOG write path (k_tlog.hip): one command per key (device arrays)
int32_t jy_tlog_write_batch(jy_engine* eng, u64 n, const uint8_t* op, const u32* slot, const u64* ts, const u64* arg,
                            const u64* pre, const u64* lr);
int32_t jy_tlog_pending(jy_engine* eng, u64* count);
// flush: pending slots, their delta logs; nkeys / nent: sizes (first call with caps 0 to size)
int32_t jy_tlog_flush_dev(jy_engine* eng, u64 cap_keys, u64 cap_ent, u32* slots, u64* cut, u64* offs, u64* ts,
                          u64* pre, u64* lr, u64* nkeys, u64* nent);

int32_t jy_dev_alloc(jy_engine* eng, void** p, u64 bytes, const char* what);
void jy_dev_free(jy_engine* eng, void* p);
int32_t jy_keydir_reserve(jy_engine* eng, int32_t type, u64 cap);
void jy_keydir_free(jy_engine* eng, KeyDir& K);
int32_t jy_keydir_run(jy_engine* eng, int32_t type, u64 n, const uint8_t* kb, const u64* ko, u32* slots, bool create,
                      u64* created, int32_t (*after_probe)(void*) = nullptr, void* arg = nullptr);
int32_t jy_keys_intern_dev(jy_engine* eng, int32_t type, u64 n, const uint8_t* kb, const u64* ko, u32* slots,
                           int32_t (*after)(void*), void* arg, u64* created_out = nullptr);
int32_t jy_ujson_grow(jy_engine* eng, u64 need_slots);
int32_t jy_ujson_extend(jy_engine* eng, u64 from, u64 to);
int32_t jy_ujson_sizes(jy_engine* eng, u64 n, const u32* slots, u64* ne, u64* nc);
int32_t jy_ujson_gather(jy_engine* eng, u64 n, const u32* slots, const u64* oeoff, const u64* ocoff, u64 nel, u64 ncl,
                        u64* odots, u64* oelems, u64* ovv, u64* ocloud);
int32_t jy_ujson_merge(jy_engine* eng, u64 ndocs, const u32* slot, const u64* eoffs, u64 nel, const u64* dots,
                       const u64* elems, const u64* vvoffs, u64 nvv, const u64* vv, const u64* coffs, u64 ncloud,
                       const u64* cloud);
struct UjsonState;
int32_t jy_ujson_merge_into(jy_engine* eng, UjsonState& u, u64 nd, const u32* slot, const u64* deoff, u64 nel,
                            const u64* ddots, const u64* delems, const u64* dvoff, u64 nvv, const u64* dvv,
                            const u64* dcoff, u64 ncloud, const u64* dcloud, bool keep_all = false);
int32_t jy_ujson_sizes_of(jy_engine* eng, const UjsonState& u, u64 n, const u32* slots, u64* ne, u64* nc);
int32_t jy_ujson_gather_of(jy_engine* eng, const UjsonState& u, u64 n, const u32* slots, const u64* oeoff,
                           const u64* ocoff, u64 nel, u64 ncl, u64* odots, u64* oelems, u64* ovv, u64* ocloud);
int32_t ujson_grow_store(jy_engine* eng, UjsonState& u, u64 need, u64 init_cap);
// UJSON write path (k_uj_write.hip): one command per doc (device arrays)
int32_t jy_ujson_write_batch(jy_engine* eng, u64 n, const uint8_t* op, const u32* slot, const u64* elem, u32 col);
int32_t jy_ujson_pending(jy_engine* eng, u64* count);
int32_t jy_ujson_flush_dev(jy_engine* eng, u64 cap_docs, u64 cap_el, u64 cap_cl, u32* slots, u64* eoff, u64* dots,
                           u64* elems, u64* vv, u64* coff, u64* cloud, u64* ndocs, u64* nel, u64* ncl);

// device exclusive scan of n u64 counts into out[0..n] (out[n] = total)
int32_t jy_scan_u64(jy_engine* eng, const u64* in, u64* out, u64 n);
// segment id (u32) of each of the n items of a CSR offs[0..nseg]
int32_t jy_seg_ids(jy_engine* eng, const u64* offs, u64 nseg, u64 n, u32* out);

// host_copy.hip: chunked parallel host copies of the staging paths
int32_t jy_copy_h2d_staged(jy_engine* eng, void* dev, uint8_t* pinned, const void* src, u64 bytes);
void jy_copy_host(void* dst, const void* src, u64 bytes);
// device -> pageable host through the pinned landing area (synchronises the stream)
int32_t jy_readback(jy_engine* eng, void* dst, const void* dev, u64 bytes);
