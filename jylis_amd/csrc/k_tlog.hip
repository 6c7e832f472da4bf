// k_tlog.hip -- TLOG segmented sorted-merge with cutoff trim, gfx950.
//
// Semantics (oracle/jy_oracle.cpp TLog; tlog.md:116-133, repo_tlog.pony:66-67):
//   cutoff' = max(cutoff_s, cutoff_d)
//   entries' = dedupe(state U delta) restricted to ts >= cutoff', ordered with
//              the later timestamp first, then the greater value first
//              (Pony String order); (ts, value) duplicates collapse.
//
// HBM layout: one entry pool of 32-B records {ts, pre, lr, w2} (value
// handle as in TREG: 8-byte big-endian prefix + arena offset/length, and
// since round 6 the value's second 8 bytes, so comparing values of up to 16
// bytes -- a duplicate, a timestamp tie -- never reads the arena) and a
// 32-B TMeta per slot {base | front room, len, cap, cutoff, newest}.  A log is
// the pool segment [base, base + len), stored OLDEST FIRST, with room up to
// cap and `front` free entries below base.
// Reads reverse it into the reference's newest-first order.
//
// Why this layout: a peer's delta is almost always entries newer than the
// whole log (writes carry the current time).  Oldest-first, those are an
// APPEND at the segment's tail -- the merge writes only the new entries and
// the key's 32-B meta; the rest of the log is never read or moved.  A raised
// cutoff drops a prefix: base moves up, nothing is copied.  Only a key whose
// delta interleaves with its log (an older entry, a timestamp tie) or whose
// segment is full is REBUILT into fresh pool space (bump allocation,
// capacity rounded to a power of two) by a merge of the two sorted runs;
// one that interleaves but fits is rewritten in place, moving the shorter
// side of the log: the suffix up into the tail room, or the prefix down into
// the front room (round 6: an entry inserted near the oldest end no longer
// moves the whole log).
// The pool is compacted (every log rewritten back to back) when its free
// space cannot cover the worst case of the next merge.
//
// Per merge, KEY TILES: a wave owns 64 consecutive delta keys and
// their delta entries (contiguous), keys staged in LDS, entries walked in
// coalesced chunks with lanes on consecutive entries:
//   k_tlog_prep    repeated slots in the batch (both copies skipped)
//   k_tlog_tile    validate (strictly newest first), cutoff drop, kept flag
//                  and state rank per entry (no search for the usual entry,
//                  newer than the log), append / insert / rebuild per key;
//                  appends are written at the tail and in-place inserts
//                  moved here
//   k_tlog_commit  rebuilt keys are written into the fresh space the scan of
//                  their sizes gave them, one lane per output entry
//                  (merge-path positions from the ranks), metas published
// Pool space for rebuilt keys is only known on the device after that scan,
// so the host never waits for it: k_tlog_commit checks on the device that the
// rebuilt logs fit the pool.  If they do not, those keys are left untouched
// and their deltas are copied into the merge's spill buffer; the host sees
// the flag once the merge has finished (the next merge call, or any call
// that reads the store), compacts the pool and re-merges the spill -- exact,
// since the join is commutative, associative and idempotent.  Appends and
// in-place inserts are published by the tile / commit passes themselves, so
// a call that fails midway may have applied part of its batch (retrying it
// is safe for the same reason).
//
// Roofline: HBM.  An append-path delta entry costs 24 B read + 32 B written;
// per delta key 32 B meta read + 32 B written + a 48-B plan record written
// and read back.  Rebuilt keys add 32 B read + 32 B written per surviving
// entry.  See DESIGN.md "TLOG".


#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "jy_dscan.hpp"
#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ u64 gid() { return (u64)blockIdx.x * kThreads + threadIdx.x; }

struct Ent {
  u64 t, p, l;
};

// sign of (pool[m] - x) in age order; value handles are read only on a tie
__device__ __forceinline__ int cmp_at(const TRec* __restrict__ pool, u64 m, const Ent& x,
                                      const uint8_t* __restrict__ arena) {
  const u64 t = pool[m].ts;
  if (t != x.t) return t > x.t ? 1 : -1;
  return jy_value_cmp(pool[m].pre, pool[m].lr, x.p, x.l, arena);
}

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

// JY_TLOG_W2 (A/B): records carry the value's second word (1) or 0 (0: a
// tie compares through the arena)
#ifndef JY_TLOG_W2
#define JY_TLOG_W2 0
#endif
__device__ __forceinline__ u64 rec_w2(u64 lr, const uint8_t* __restrict__ arena) {
  return JY_TLOG_W2 ? jy_value_w2(lr, arena) : 0ull;
}

__device__ __forceinline__ void store_rec(TRec* __restrict__ p, u64 ts, u64 pre, u64 lr, u64 w2) {
  u64x2* q = reinterpret_cast<u64x2*>(p);
  u64x2 a, b;
  a.x = ts;
  a.y = pre;
  b.x = lr;
  b.y = w2;
  __builtin_nontemporal_store(a, q);
  __builtin_nontemporal_store(b, q + 1);
}

__device__ __forceinline__ TRec load_rec(const TRec* __restrict__ p) {
  const u64x2* q = reinterpret_cast<const u64x2*>(p);
  const u64x2 a = __builtin_nontemporal_load(q), b = __builtin_nontemporal_load(q + 1);
  TRec r;
  r.ts = a.x;
  r.pre = a.y;
  r.lr = b.x;
  r.pad = b.y;
  return r;
}

// kInsert moves the log's suffix from the smallest inserted rank up into the
// tail room; kInsertDn moves its prefix below the largest inserted rank down
// into the front room (an entry inserted near the oldest end)
enum : u32 { kSkip = 0, kAppend = 1, kRebuild = 2, kFast = 3, kInsert = 4, kInsertDn = 5 };

// per REBUILT key: what k_tlog_tile decided; the log's current base is read
// from its meta at commit
struct alignas(16) PInfo {
  u64 newest;  // newest ts after the merge
  u64 cut;     // merged cutoff
  u32 k;       // delta key
  u32 s;       // slot
  u32 len;     // old length
  u32 drop;    // state entries dropped by the cutoff (a prefix)
  u32 newlen;  // entries after the merge
  u32 cap;     // the new segment's capacity
};

struct TlogArgs {
  TMeta* meta;
  u64* hint;  // [nkeys] oldest-timestamp hints (TlogState::hint)
  u64* hist;  // [nkeys] update histories (TlogState::hist)
  const TRec* pool;
  const uint8_t* arena;
  // delta batch
  u64 nd;
  const u32* slot;
  const u64* dcut;
  const u64* doff;
  const u64* dts;
  const u64* dpre;
  const u64* dlr;
  // temporaries
  u64* dptr;      // [nkeys] epoch << 32 | the delta key merging into each slot (last claimer)
  u32 epoch;      // this merge's claim epoch (never 0)
  u32* bad;       // [nd] == epoch: the key's slot is repeated in the batch (no reset between merges)
  PInfo* pinfo;   // [nd] written for rebuilt and inserted keys only
  u32* rz;        // [nd + 1] pool entries a rebuilt key takes (0 otherwise)
  u64* rsum;      // [tiles + 1] rebuilt pool entries per key tile (scanned in place before k_tlog_commit)
  unsigned long long* skipped;
  // the device-side pool check: when the rebuilt logs do not fit pcap, the
  // rebuilt keys' deltas go to the spill (the batch's shape: slot JY_NO_SLOT
  // for every other key, the same offsets, only the rebuilt keys' entries)
  u64 pcap;
  u32* sp_slot;
  u64 *sp_cut, *sp_off, *sp_ts, *sp_pre, *sp_lr;
};

// A slot named twice in one device batch breaks the one-delta-per-key
// contract: both deltas are skipped (counted once), the key is left untouched.
// The claims carry the merge's epoch, so nothing resets them: a claimer that
// finds this epoch's tag marks itself and the key it displaced (with three or
// more copies every copy is marked by the next one).  The marks carry the
// epoch too: bad[k] == epoch.
__global__ __launch_bounds__(kThreads) void k_tlog_prep(TlogArgs A) {
  const u64 k = gid();
  if (k >= A.nd) return;
  const u32 s = A.slot[k];
  if (s == JY_NO_SLOT) return;  // a hole of a routed run (k_route_csr.hip)
  const u64 tag = (u64)A.epoch << 32;
  const u64 prev = atomicExch(reinterpret_cast<unsigned long long*>(A.dptr + s), (unsigned long long)(tag | k));
  if ((prev & ~0xFFFFFFFFull) == tag) {
    A.bad[k] = A.epoch;
    A.bad[(u32)prev] = A.epoch;
  }
}

// first position in [lo, hi) of a log whose timestamps ascend, with
// timestamp >= x (hi if none); tlo < x is a lower bound of the timestamps
// before lo, thi >= x an upper bound from hi - 1 on (the log's oldest and
// newest timestamps to start with).  Timestamps follow wall time, so an
// interpolated guess usually lands close: each round loads the ALIGNED
// 128-B line of records around it (kWin = 4 timestamps for one line), which
// either brackets x or narrows [lo, hi) to one side of the line, the next
// guess interpolating between the timestamps just read; a range of at most
// kWin entries is settled by one load of all of it.  Round 6: kWin 2
// unaligned (two lines half the time) and a binary search after the first
// miss took ~5 dependent probes per search at config 4 (the searches were
// ~55% of a key tile's lifetime, profiles/r06_tlog_tile_probe.txt).
constexpr u32 kWin = 4;
constexpr int kInterpRounds = 3;
__device__ __forceinline__ u32 ts_interp(const TRec* __restrict__ pool, u64 base, u32 lo, u32 hi, u64 tlo, u64 thi,
                                         u64 x) {
#pragma unroll 1
  for (int it = 0; it < kInterpRounds; it++) {
    if (hi - lo <= kWin) {  // all of it at once
      u64 w[kWin];
#pragma unroll
      for (u32 i = 0; i < kWin; i++) w[i] = lo + i < hi ? pool[base + lo + i].ts : ~0ull;
      u32 c = 0;
#pragma unroll
      for (u32 i = 0; i < kWin; i++) c += w[i] < x;
      return lo + c;
    }
    u64 g;
    if (x > tlo && x <= thi && thi > tlo) {
      const double f = (double)(x - tlo) / (double)(thi - tlo);
      g = lo + (u64)(f * (double)(hi - 1 - lo));
    } else {
      g = lo + ((hi - lo) >> 1);
    }
    u64 ga = ((base + g) & ~(u64)(kWin - 1)) - base;  // the line holding the guess
    if (ga < lo) ga = lo;
    if (ga > hi - kWin) ga = hi - kWin;
    u64 w[kWin];
#pragma unroll
    for (u32 i = 0; i < kWin; i++) w[i] = pool[base + ga + i].ts;
    u32 c = 0;
#pragma unroll
    for (u32 i = 0; i < kWin; i++) c += w[i] < x;
    if (c == 0) {
      if (ga == lo) return lo;
      hi = (u32)ga;  // at or before ga
      thi = w[0];
    } else if (c == kWin) {
      lo = (u32)ga + kWin;  // after the line
      tlo = w[kWin - 1];
    } else {
      return (u32)ga + c;
    }
  }
  while (lo < hi) {
    const u32 m = (lo + hi) >> 1;
    if (pool[base + m].ts < x) lo = m + 1;
    else hi = m;
  }
  return lo;
}

// capacity of a rebuilt segment, a power of two: room to grow 4x by appends
// (HBM is plentiful; every rebuild copies the whole log, so they should be
// rare) -- and, driven by the log's update history, room for kHorizon more
// merges at the rate it grew since its last segment was made: a short log
// that is appended to on every merge would otherwise be rebuilt again within
// a few merges (round 6)
constexpr u64 kGrow = 4;
constexpr u64 kHorizon = 16;
__device__ __forceinline__ u64 hist_room(u64 h, u32 n, u32 epoch) {
  if (h == 0) return 0;  // no history yet
  const u32 age = epoch - (u32)h, n0 = (u32)(h >> 32);
  if (age == 0 || age > 1024 || n <= n0) return 0;
  return ((u64)(n - n0) * kHorizon + age - 1) / age;
}
__device__ __forceinline__ u32 pow2_cap(u32 n, u64 room = 0) {
  u64 want = kGrow * (u64)n + kGrow;
  if ((u64)n + room > want) want = (u64)n + room;
  u64 c = 4;
  while (c < want) c <<= 1;
  return c > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)c;
}

// front room of a rebuilt segment (cap entries for n): an eighth of its free
// room, for entries inserted near the log's oldest end (stage 5, kInsertDn)
__device__ __forceinline__ u32 rebuild_front(u32 cap, u32 n) { return (cap - n) / 8; }
// and of a compacted one
__device__ __forceinline__ u32 cmp_front(u32 n) { return n ? n / 8 + 2 : 0; }

// last idx in [0, n] with a[idx] <= x (a non-decreasing, a[0] <= x)
template <class T>
__device__ __forceinline__ u32 lds_last_le(const T* a, u32 n, u64 x) {
  u32 lo = 0, hi = n;
  while (lo < hi) {
    const u32 m = (lo + hi + 1) >> 1;
    if (a[m] <= x) lo = m;
    else hi = m - 1;
  }
  return lo;
}

// key tiles are one wave: no cross-wave barriers, many tiles in flight per CU
constexpr int kTile = 64;
#ifndef JY_TLOG_FASTENT
#define JY_TLOG_FASTENT 4
#endif
constexpr int kFastEnt = JY_TLOG_FASTENT;  // delta entries a key may have for the lane-per-key fast path
#ifndef JY_TLOG_KCACHE
#define JY_TLOG_KCACHE 1
#endif
// (a next-pass prefetch of stage 2's entry measured no gain in round 4: 0.837
// / 0.841 ms without, 0.865 with at 6 waves per SIMD (spills), 0.834 / 0.836
// at 5 waves; removed)
constexpr int kCache = JY_TLOG_KCACHE;  // passes of slow entries kept in registers for the append stores

#ifdef JY_TLOG_PROBE  // A/B only: per-stage wall-clock latency of the key tiles (100 MHz), summed
constexpr int kProbeSlots = 64, kProbeN = 16;
__device__ unsigned long long g_tprobe[kProbeSlots][kProbeN];
#define JY_TCLK(v) const u64 v = wall_clock64()
#define JY_TCLKV(v) v = wall_clock64()
#define JY_TPROBE(i, v) \
  if (threadIdx.x == 0) atomicAdd(&g_tprobe[blockIdx.x % kProbeSlots][i], (unsigned long long)(v))
#else
#define JY_TCLK(v)
#define JY_TCLKV(v)
#define JY_TPROBE(i, v)
#endif

constexpr u32 kKept = 0x80000000u;  // eqx: kept flag | # kept entries of the key before this one

// KEY TILES: a workgroup (one wave) owns kTile consecutive delta keys.
//   1. per key (lane = key): meta, merged cutoff; the FAST PATH -- a delta of
//      at most kFastEnt entries, strictly newest first, every kept entry
//      newer than the log, room in the segment, no cutoff raise -- is
//      appended and its meta published right here, its entries loaded by
//      the key's own lane together with the meta (one round trip)
//   2. the other keys' entries, flattened (LDS prefix of their counts), lanes
//      on consecutive entries: order check against the previous entry; kept
//      flag and rank (# state entries older than it: len for an entry newer
//      than the log, else a binary search, duplicates dropped); q = kept
//      entries of the key before it (ballot with carry)
//   3. per key: append (every kept entry has rank len, room left) -> meta
//      published; rebuild -> its plan and size for k_tlog_commit; skip
//   4. appends: kept entries to the tail, oldest first (the first kCache
//      passes from registers)
// rank / q of the slow entries go to HBM for the rebuild in k_tlog_commit.
#ifndef JY_TLOG_WAVES
// 80 VGPRs: 6 waves per SIMD (one cached pass; 2 cached passes took 90 VGPRs / 5 waves)
#define JY_TLOG_WAVES 6
#endif
#ifndef JY_TLOG_TILE_ATTR
#define JY_TLOG_TILE_ATTR __attribute__((amdgpu_waves_per_eu(JY_TLOG_WAVES)))
#endif
__global__ __launch_bounds__(kTile) JY_TLOG_TILE_ATTR void k_tlog_tile(TlogArgs A, TRec* __restrict__ pool,
                                                                        u32* __restrict__ erank,
                                                                        u32* __restrict__ eqx) {
  // u32 offsets inside the tile (its entries are < 2^32): 5.9 -> 4.9 KB of LDS
  // per one-wave tile, under 160 KB / 32 waves per CU
  __shared__ u32 l_soff[kTile + 1];  // flattened offsets of the slow keys' entries
  __shared__ u32 l_gb[kTile];        // first delta entry of each key, less the tile's first (gb0)
  __shared__ u32 l_slot[kTile];
  __shared__ u64 l_oldest[kTile];  // oldest surviving timestamp of a slow key's log
  __shared__ u64 l_base[kTile], l_newest[kTile], l_cut[kTile], l_tn[kTile], l_to[kTile];
  __shared__ u32 l_len[kTile], l_cap[kTile], l_drop[kTile], l_M[kTile], l_minrank[kTile], l_bad[kTile],
      l_gstart[kTile], l_mode[kTile];
  __shared__ u32 l_Mi[kTile], l_mx[kTile];  // kept entries inside the log (rank < len), their largest rank
  const u32 tid = threadIdx.x;
  const u64 lanelt = (1ull << tid) - 1;
  const u64 k0 = (u64)blockIdx.x * kTile;
  const u32 nt = (u32)(A.nd - k0 < kTile ? A.nd - k0 : kTile);
  JY_TCLK(ck0);
  const u64 gb0 = A.doff[k0];  // the tile's first delta entry
  // 1. keys
  u64 sc = 0;      // slow entries of this lane's key
  u32 front = 0;   // its front room (stage 3 is this lane's again)
  bool raise = false;  // its cutoff rises over part of its log: a drop search
  if (tid < nt) {
    const u64 k = k0 + tid;
    const u32 s = A.slot[k];
    const u64 b0 = A.doff[k], b1 = A.doff[k + 1];
    const u64 ne = b1 - b0;
    u64 ft[kFastEnt], fp[kFastEnt], fl[kFastEnt];
#pragma unroll
    for (int u = 0; u < kFastEnt; u++) {  // issued with the meta load
      ft[u] = fp[u] = fl[u] = 0;
      if ((u64)u < ne) {
        ft[u] = A.dts[b0 + u];
        fp[u] = A.dpre[b0 + u];
        fl[u] = A.dlr[b0 + u];
      }
    }
    const bool hole = s == JY_NO_SLOT;  // a routed run's unused record: skipped, not counted
    const TMeta m = hole ? TMeta{0, 0, 0, 0, 0} : A.meta[s];
    const u64 mb = tm_base(m);
    const u64 hv = hole ? 0 : A.hint[s];  // with the meta: no dependent load of the log's first record
    const u64 cd = A.dcut[k];
    const u32 bad = hole ? 4u : (A.bad[k] == A.epoch ? 1u : 0u);
    const u64 cut = m.cut > cd ? m.cut : cd;
    bool fast = !bad && ne <= kFastEnt && cd <= m.cut;
    u32 M = 0;  // kept entries newer than the log: a prefix (strictly newest first)
#pragma unroll
    for (int u = 0; u < kFastEnt; u++) {
      if ((u64)u >= ne) continue;
      if (u > 0) fast = fast && ft[u - 1] > ft[u];  // equal timestamps need the value order
      if (ft[u] >= cut) {
        if (m.len == 0 || ft[u] > m.newest) M++;
        else fast = false;  // not newer than the log: a search (stage 2)
      }
    }
    fast = fast && m.len + M <= m.cap;
    if (fast) {
#pragma unroll
      for (int u = 0; u < kFastEnt; u++)
        if ((u32)u < M)
          store_rec(pool + mb + m.len + (M - 1 - u), ft[u], fp[u], fl[u], rec_w2(fl[u], A.arena));
      if (M) A.meta[s] = TMeta{m.bf, m.len + M, m.cap, m.cut, (m.len == 0 || ft[0] > m.newest) ? ft[0] : m.newest};
      if (M && m.len == 0) {  // an empty log's oldest entry: the oldest appended one (kept entries are a prefix)
        u64 o = ft[0];
#pragma unroll
        for (int u = 1; u < kFastEnt; u++)
          if ((u32)u < M) o = ft[u];
        A.hint[s] = o;
      }
    } else {
      // a raised cutoff's dropped prefix is searched in stage 2, in the same
      // search passes as the entries (round 6: searched here, it was a
      // dependent chain of its own that the whole tile waited for)
      raise = cd > m.cut && m.len > 0;
      // the oldest timestamp (hint: no dependent load of the log's first
      // record) -- the lower bound of every search; the drop search replaces
      // it by the oldest surviving one, for the hint stage 3 publishes
      l_oldest[tid] = m.len > 0 ? hv : 0;
      sc = hole ? 0 : ne;  // a hole's entries (a spill's unspilled keys) are never walked
      l_base[tid] = mb;
      front = (u32)tm_front(m);
      l_newest[tid] = m.newest;
      l_cut[tid] = cut;
      l_len[tid] = m.len;
      l_cap[tid] = m.cap;
      l_drop[tid] = 0;
      l_bad[tid] = bad;
      l_M[tid] = 0;
      l_Mi[tid] = 0;
      l_mx[tid] = 0;
      l_minrank[tid] = 0xFFFFFFFFu;
      l_tn[tid] = 0;
      l_to[tid] = ~0ull;
    }
    l_gb[tid] = (u32)(b0 - A.doff[k0]);
    l_slot[tid] = s;
    l_mode[tid] = fast ? kFast : kSkip;
  }
  {
    const u64 inc = jyscan::wave_incl<u64>(sc);
    const u64 tot = __shfl(inc, 63);  // every lane: a shuffle reads only active lanes
    if (tid < nt) l_soff[tid] = (u32)(inc - sc);
    if (tid == 0) l_soff[nt] = (u32)tot;
  }
  __syncthreads();
  const u64 F = l_soff[nt];
  JY_TCLK(ck1);
#ifdef JY_TLOG_PROBE
  u64 pl = 0, ps = 0, pe = 0, pa = 0, pb = 0;
#endif
  // 2. slow entries.  (a) one per lane per pass: order check, cutoff, and
  //    the rank of an entry newer than the log (its length); an entry that
  //    needs a search joins the tile's SEARCH QUEUE (LDS), with the raised
  //    cutoffs' drop searches.  (b) the queue in passes of 64 searches: the
  //    rank in the log (an aligned-line interpolation search, then the value
  //    order on equal timestamps, duplicates dropped).  A tile's searches run
  //    as ONE chain of dependent loads (two when it has more than 64), not
  //    one per entry pass.  (c) per pass again: kept flags from (a) / (b),
  //    q = kept entries of the key before it (ballot with carry), the keys'
  //    counts and bounds.  erank / eqx carry the ranks and states between
  //    them (eqx: 0 dropped, 1 kept, until (c) writes the final word).
  __shared__ u32 l_q[kTile];   // queued items: entry index f, or kDropItem | key
  __shared__ u64 l_qx[kTile];  // their timestamps (the value searched for)
  constexpr u32 kDropItem = 0x80000000u;
  u32 nq = 0;  // wave-uniform
  {
    const u64 m = __ballot(raise);
    if (raise) {
      const u32 at = (u32)__popcll(m & lanelt);
      l_q[at] = kDropItem | tid;
      l_qx[at] = l_cut[tid];
    }
    nq = (u32)__popcll(m);
  }
  // the n queued searches, lane = item
  auto run_searches = [&](u32 n) {
    __syncthreads();  // the queue's writes
    u32 item = 0, idx = 0, r = 0;
    u64 x = 0, j = 0;
    bool live = tid < n;
    if (live) {
      item = l_q[tid];
      x = l_qx[tid];
      idx = (item & kDropItem) ? (item & (kTile - 1)) : lds_last_le(l_soff, nt - 1, item);
      const u64 base = l_base[idx];
      const u32 len = l_len[idx];
      u64 pp = 0, ll = 0;
      if (!(item & kDropItem)) {
        j = gb0 + l_gb[idx] + (item - l_soff[idx]);
        pp = A.dpre[j];  // in flight with the search
        ll = A.dlr[j];
      }
      r = ts_interp(A.pool, base, 0, len, l_oldest[idx], l_newest[idx], x);
      if (item & kDropItem) {
        l_drop[idx] = r;  // oldest first: the dropped prefix
        l_oldest[idx] = r < len ? A.pool[base + r].ts : 0;
      } else {
        int c = 1;
        u32 e = r;
        for (; e < len; e++) {
          const TRec y = A.pool[base + e];
          if (y.ts != x) break;
          c = jy_value_cmp(y.pre, y.lr, pp, ll, A.arena);
          if (c >= 0) break;
        }
        erank[j] = e;
        eqx[j] = c != 0 ? 1u : 0u;  // c == 0: a duplicate of entry e
      }
    }
    __syncthreads();  // l_oldest / l_drop / erank / eqx
  };
  // the drop searches read l_oldest / l_newest of their own key only, and the
  // entry searches of a raise key run in the same pass or later: their lower
  // bound may already be the surviving oldest, a tighter one -- either is a
  // valid bound (every timestamp searched is >= the cutoff)
  u32 carry = 0;
  constexpr int kCacheN = kCache > 0 ? kCache : 1;
  u64 c_t[kCacheN], c_p[kCacheN], c_l[kCacheN];
  u32 c_q[kCacheN], c_i[kCacheN];
#pragma unroll
  for (int c = 0; c < kCache; c++) c_q[c] = c_i[c] = 0, c_t[c] = c_p[c] = c_l[c] = 0;
  // (a)
  int pass = 0;
  for (u64 c0 = 0; c0 < F; c0 += kTile, pass++) {
    const u64 f = c0 + tid;
    u32 idx = 0, st = 0;
    u64 t = 0, pp = 0, ll = 0, j = 0;
    if (f < F) {
      idx = lds_last_le(l_soff, nt - 1, f);
      j = gb0 + l_gb[idx] + (f - l_soff[idx]);
      t = A.dts[j];
      pp = A.dpre[j];
      ll = A.dlr[j];
      const u64 pt = f > l_soff[idx] ? A.dts[j - 1] : ~0ull;
      // strictly newest first; the previous value is read only on a ts tie
      if (f > l_soff[idx] && (pt < t || (pt == t && jy_value_cmp(A.dpre[j - 1], A.dlr[j - 1], pp, ll, A.arena) <= 0)))
        atomicOr(&l_bad[idx], 2u);
      const u32 len = l_len[idx];
      if (t >= l_cut[idx]) {
        if (len == 0 || t > l_newest[idx]) {
          st = 1;
          erank[j] = len;
          eqx[j] = 1u;
        } else {
          st = 2;  // a search; every state entry below the cutoff is older than t, so [0, len) does
        }
      } else {
        erank[j] = 0u;  // (below the cutoff: the oldest entries, rank 0 keeps the ranks non-increasing)
        eqx[j] = 0u;
      }
    }
    const u64 m = __ballot(st == 2);
    if (nq + (u32)__popcll(m) > kTile) {  // no room: the queue's searches first
      run_searches(nq);
      nq = 0;
    }
    if (st == 2) {
      const u32 at = nq + (u32)__popcll(m & lanelt);
      l_q[at] = (u32)f;
      l_qx[at] = t;
    }
    nq += (u32)__popcll(m);
#pragma unroll
    for (int c = 0; c < kCache; c++)
      if (c == pass) c_t[c] = t, c_p[c] = pp, c_l[c] = ll, c_i[c] = idx;
  }
  if (nq) run_searches(nq);
  else __syncthreads();  // (a)'s global stores, for (c)
#ifdef JY_TLOG_PROBE
  __builtin_amdgcn_s_waitcnt(0);
  JY_TCLKV(pa);
  pl = pa - ck1;
#endif
  // (c)
  pass = 0;
  for (u64 c0 = 0; c0 < F; c0 += kTile, pass++) {
    const u64 f = c0 + tid;
    u32 idx = 0, kept = 0, rank = 0;
    u64 t = 0, j = 0;
    if (f < F) {
      if (pass < kCache) {
        idx = c_i[0], t = c_t[0];
#pragma unroll
        for (int c = 1; c < kCache; c++)
          if (c == pass) idx = c_i[c], t = c_t[c];
      } else {
        idx = lds_last_le(l_soff, nt - 1, f);
      }
      j = gb0 + l_gb[idx] + (f - l_soff[idx]);
      if (pass >= kCache) t = A.dts[j];
      kept = eqx[j];
      rank = kept ? erank[j] : 0u;
    }
    // kept ranks in entry order (a wave ballot per pass)
    const u64 mask = __ballot(kept != 0);
    const u32 g = carry + (u32)__popcll(mask & lanelt);
    carry += (u32)__popcll(mask);
    if (f < F && f == l_soff[idx]) l_gstart[idx] = g;
    __syncthreads();
    u32 qx = 0;
    if (f < F) {
      qx = (g - l_gstart[idx]) | (kept ? kKept : 0u);
      eqx[j] = qx;
      if (kept) {
        atomicAdd(&l_M[idx], 1u);
        atomicMin(&l_minrank[idx], rank);
        atomicMax((unsigned long long*)&l_tn[idx], (unsigned long long)t);  // newest kept
        atomicMin((unsigned long long*)&l_to[idx], (unsigned long long)t);  // oldest kept (the hint)
        if (rank < l_len[idx]) {
          atomicAdd(&l_Mi[idx], 1u);
          atomicMax(&l_mx[idx], rank);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < kCache; c++)
      if (c == pass) c_q[c] = qx;
    __syncthreads();  // l_gstart reuse
  }
#ifdef JY_TLOG_PROBE
  __builtin_amdgcn_s_waitcnt(0);
  JY_TCLKV(pb);
  ps = 0;
  pe = pb - pa;
#endif
  JY_TCLK(ck2);
  // 3. per slow key: append (meta published here), rebuild (planned) or skip
  u32 mode = kFast;
  PInfo P{};
  if (blockIdx.x == 0 && tid == 0) A.rz[A.nd] = 0;
  if (tid < nt && l_mode[tid] != kFast) {
    const u64 k = k0 + tid;
    P.k = (u32)k;
    P.s = l_slot[tid];
    if (l_bad[tid]) {
      mode = kSkip;
      // once per slot: the last claimer counts it
      if (P.s != JY_NO_SLOT && A.dptr[P.s] == (((u64)A.epoch << 32) | k)) atomicAdd(A.skipped, 1ull);
    } else {
      const u32 len = l_len[tid], drop = l_drop[tid], M = l_M[tid];
      const u32 surv = len - drop;
      const u64 newest = l_newest[tid];
      u64 nn = newest;
      if (M > 0) {
        const u64 tn = l_tn[tid];
        nn = (surv == 0 || tn > newest) ? tn : newest;
      }
      P.len = len;
      P.drop = drop;
      P.newlen = surv + M;
      P.cut = l_cut[tid];
      P.newest = nn;
      // the merged log's oldest entry, as a hint for later searches (a
      // spilled rebuild leaves it ahead of the state until its re-merge)
      if (P.newlen > 0) {
        const u64 so = l_oldest[tid], dlo = l_to[tid];
        A.hint[P.s] = surv == 0 ? dlo : (M > 0 && dlo < so ? dlo : so);
      }
      const u64 base = l_base[tid], fr = (u64)front + drop;  // front room once the dropped prefix is free
      const u32 cap = l_cap[tid], Mi = l_Mi[tid];
      const bool up_ok = (u64)len + M <= cap;
      if ((M == 0 || l_minrank[tid] == len) && up_ok) {
        mode = kAppend;
        A.meta[P.s] = TMeta{tm_bf(base + drop, fr), P.newlen, cap - drop, P.cut, nn};
      } else {
        // interleaves: if the segment has room the log is rewritten in place
        // (stage 5) -- its suffix from the smallest inserted rank moves up
        // into the tail room, or its prefix below the largest inserted rank
        // moves down into the front room, whichever moves fewer entries
        const bool dn_ok = Mi <= fr && (u64)len + (M - Mi) <= cap;
        const u32 up = len - l_minrank[tid], dn = l_mx[tid] - drop;
        if (dn_ok && (!up_ok || dn < up)) {
          mode = kInsertDn;
          const u64 nc = (u64)cap - drop + Mi;
          A.meta[P.s] = TMeta{tm_bf(base + drop - Mi, fr - Mi), P.newlen, nc < 0xFFFFFFFFull ? (u32)nc : 0xFFFFFFFFu,
                              P.cut, nn};
        } else if (up_ok) {
          mode = kInsert;
          A.meta[P.s] = TMeta{tm_bf(base + drop, fr), P.newlen, cap - drop, P.cut, nn};
        } else {
          mode = kRebuild;
          P.cap = pow2_cap(surv + M, hist_room(A.hist[P.s], surv + M, A.epoch));
          A.pinfo[k] = P;
        }
      }
    }
    l_mode[tid] = mode;
  }
  if (tid < nt) {
    A.rz[k0 + tid] = mode == kRebuild ? P.cap : 0u;
  }
  {  // the tile's rebuilt space: k_tlog_commit offsets its keys from the scan of these
    const u64 r = jyscan::wave_sum<u64>(tid < nt && mode == kRebuild ? (u64)P.cap : 0ull);
    if (tid == 0) A.rsum[blockIdx.x] = r;
  }
  __syncthreads();
  JY_TCLK(ck3);
  // 4. appends: kept entries of append keys go to the tail, oldest first
  pass = 0;
  for (u64 c0 = 0; c0 < F; c0 += kTile, pass++) {
    const u64 f = c0 + tid;
    if (f >= F) continue;
    u32 idx, qx;
    u64 t, pp, ll;
    if (pass < kCache) {
      idx = c_i[0], qx = c_q[0], t = c_t[0], pp = c_p[0], ll = c_l[0];
#pragma unroll
      for (int c = 1; c < kCache; c++)
        if (c == pass) idx = c_i[c], qx = c_q[c], t = c_t[c], pp = c_p[c], ll = c_l[c];
      if (l_mode[idx] != kAppend || !(qx & kKept)) continue;
    } else {
      idx = lds_last_le(l_soff, nt - 1, f);
      if (l_mode[idx] != kAppend) continue;
      const u64 j = gb0 + l_gb[idx] + (f - l_soff[idx]);
      qx = eqx[j];
      if (!(qx & kKept)) continue;
      t = A.dts[j], pp = A.dpre[j], ll = A.dlr[j];
    }
    const u64 tail = l_base[idx] + l_len[idx] + l_M[idx] - 1;
    store_rec(pool + tail - (qx & ~kKept), t, pp, ll, rec_w2(ll, A.arena));
  }
  JY_TCLK(ck4);
  u32 s5items = 0;
  // 5. in-place inserts: each insert key's delta entries, then its state
  //    entries from minrank, flattened (a wave scan of their counts) and
  //    moved from the last item down -- one wave, so a pass's loads all
  //    return before its stores, and a state entry only moves up: every
  //    entry is read before anything is written over it (as k_tlog_commit
  //    did it for these keys).  The key's ranks and q words are this pass's
  //    own stage-2 stores, read back after the workgroup barrier.
  //      delta entry j: (rank_j - drop) + (M - 1 - q_j), if kept
  //      state entry i: (i - drop) + #kept deltas with rank <= i
  //    relative to the log's new base (base + drop).  Reads and writes both
  //    go through `pool`.
  //    A kInsertDn key numbers its moved state entries from the largest
  //    index down (so the passes, last item first, move them lowest first:
  //    entries only move down, so every one is read before anything is
  //    written over it), and its new base is base + drop - Mi.
  {
    u32 w = 0, ne = 0;
    if (tid < nt && (l_mode[tid] == kInsert || l_mode[tid] == kInsertDn)) {
      ne = l_soff[tid + 1] - l_soff[tid];  // an insert key walked every entry (stage 2)
      w = ne + (l_mode[tid] == kInsert ? l_len[tid] - l_minrank[tid] : l_mx[tid] - l_drop[tid]);
    }
    const u32 winc = jyscan::wave_incl<u32>(w);
    const u32 wtot = __shfl(winc, 63);
    __syncthreads();  // stage 4's reads of l_soff are done
    if (tid < nt) {
      l_soff[tid] = winc - w;  // reused: the keys' first items
      l_gstart[tid] = ne;      // reused: their delta entry counts
    }
    if (tid == 0) l_soff[nt] = wtot;
    __syncthreads();
    s5items = wtot;
    for (long long c0 = wtot ? (long long)((wtot - 1) / kTile) * kTile : -1; c0 >= 0; c0 -= kTile) {
      const u32 item = (u32)c0 + tid;
      bool write = false;
      u64 at = 0;
      TRec x{};
      if (item < wtot) {
        const u32 a = lds_last_le(l_soff, nt - 1, item);
        const u32 r = item - l_soff[a], nek = l_gstart[a], drop = l_drop[a], M = l_M[a];
        const bool dn = l_mode[a] == kInsertDn;
        const u64 jb = gb0 + l_gb[a], dst = l_base[a] + drop - (dn ? l_Mi[a] : 0u);
        if (r < nek) {
          const u64 j = jb + r;
          const u32 qx = eqx[j], rank = erank[j];
          x.ts = A.dts[j];
          x.pre = A.dpre[j];
          x.lr = A.dlr[j];
          x.pad = rec_w2(x.lr, A.arena);
          write = (qx & kKept) != 0;
          at = dst + (u64)(rank - drop) + (M - 1 - (qx & ~kKept));
        } else {
          const u64 i = dn ? l_mx[a] - 1 - (r - nek) : l_minrank[a] + (r - nek);
          x = load_rec(pool + l_base[a] + i);
          // the first delta entry with rank <= i (ranks fall along the
          // newest-first segment): a short segment counted at once, a long
          // one bisected
          u64 lo = jb, hi = jb + nek;
          u32 q = 0;  // kept delta entries before lo (segment order)
          if (hi - lo <= 4) {
            // a short segment: its ranks and kept flags in one round trip
            u32 rk[4], kq[4];
#pragma unroll
            for (u64 e = 0; e < 4; e++) {
              rk[e] = lo + e < hi ? erank[lo + e] : 0u;
              kq[e] = lo + e < hi ? eqx[lo + e] : 0u;
            }
            u64 c = 0;
#pragma unroll
            for (u64 e = 0; e < 4; e++) {
              const bool above = (lo + e < hi) & (rk[e] > i);
              c += above;
              q += above & ((kq[e] & kKept) != 0);
            }
            lo += c;
          } else {
            while (lo < hi) {
              const u64 m = (lo + hi) >> 1;
              if (erank[m] <= i) hi = m;
              else lo = m + 1;
            }
            q = lo < jb + nek ? (eqx[lo] & ~kKept) : 0u;
          }
          write = true;
          at = dst + (i - drop) + (lo < jb + nek ? M - q : 0u);
        }
      }
      if (write) store_rec(pool + at, x.ts, x.pre, x.lr, x.pad);
    }
  }
#ifdef JY_TLOG_PROBE
  __builtin_amdgcn_s_waitcnt(0);
#endif
  JY_TCLK(ck5);
  JY_TPROBE(0, 1);
  JY_TPROBE(1, ck1 - ck0);
  JY_TPROBE(2, ck2 - ck1);
  JY_TPROBE(3, ck3 - ck2);
  JY_TPROBE(4, ck4 - ck3);
  JY_TPROBE(5, ck5 - ck4);
  JY_TPROBE(6, F);
  JY_TPROBE(7, (F + kTile - 1) / kTile);
  JY_TPROBE(8, s5items);
  JY_TPROBE(9, (s5items + kTile - 1) / kTile);
#ifdef JY_TLOG_PROBE
  JY_TPROBE(10, pl);
  JY_TPROBE(11, ps);
  JY_TPROBE(12, pe);
#endif
  (void)s5items;
}

// KEY TILES again, after the scan of rebuilt sizes (tiles without a rebuilt
// or inserted key exit after one load), one lane per output entry (state
// entries and delta entries of the tile's keys, flattened by a wave scan):
//   state entry i: (i - drop) + #kept deltas with rank <= i; ranks fall along
//     the newest-first delta segment, so that is M - q of the first entry
//     with rank <= i (binary search)
//   kept delta entry j: (rank_j - drop) + (M - 1 - q_j)
// relative to the log's new base: every survivor of a REBUILT key into fresh
// space.  (In-place inserts are k_tlog_tile's stage 5 since round 5: the
// commit re-loaded each insert key's plan, meta, delta entries and ranks,
// and nearly every 64-key tile of config 4 has one.)
__global__ __launch_bounds__(kTile) void k_tlog_commit(TlogArgs A, const u64* __restrict__ rtile,
                                                       const u64* __restrict__ ctr, TRec* __restrict__ pool,
                                                       const u32* __restrict__ erank, const u32* __restrict__ eqx) {
  __shared__ u64 l_woff[kTile + 1];
  __shared__ u64 l_src[kTile], l_dst[kTile], l_blo[kTile], l_bhi[kTile];
  __shared__ u32 l_drop[kTile], l_s0[kTile], l_ns[kTile], l_M[kTile];
  const u32 tid = threadIdx.x;
  const u64 k0 = (u64)blockIdx.x * kTile;
  const u32 nt = (u32)(A.nd - k0 < kTile ? A.nd - k0 : kTile);
  u32 cap = tid < nt ? A.rz[k0 + tid] : 0u;
  // the pool check (uniform: k_tlog_bump moves ctr only after every tile)
  if (ctr[0] + rtile[gridDim.x] > A.pcap) {
    // no room for this merge's rebuilt logs: they stay as they are and their
    // deltas go to the spill, which the host re-merges after a compaction
    if (tid < nt) {
      const u64 k = k0 + tid;
      const u64 b0 = A.doff[k], b1 = A.doff[k + 1];
      A.sp_slot[k] = cap ? A.slot[k] : JY_NO_SLOT;
      A.sp_cut[k] = A.dcut[k];
      A.sp_off[k] = b0;
      if (k + 1 == A.nd) A.sp_off[A.nd] = b1;
      if (cap)
        for (u64 j = b0; j < b1; j++) {
          A.sp_ts[j] = A.dts[j];
          A.sp_pre[j] = A.dpre[j];
          A.sp_lr[j] = A.dlr[j];
        }
    }
    cap = 0;
  }
  if (__ballot(cap != 0) == 0) return;
  const u64 roff_k = rtile[blockIdx.x] + jyscan::wave_incl<u64>(cap) - cap;  // the key's rebuilt space
  u32 w = 0;
  if (cap) {
    const u64 k = k0 + tid;
    const PInfo P = A.pinfo[k];
    const u64 src = tm_base(A.meta[P.s]);
    const u32 f = rebuild_front(P.cap, P.newlen);
    const u64 dst = ctr[0] + roff_k + f;
    A.meta[P.s] = TMeta{tm_bf(dst, f), P.newlen, P.cap - f, P.cut, P.newest};
    A.hist[P.s] = (u64)P.newlen << 32 | A.epoch;
    const u64 blo = A.doff[k], bhi = A.doff[k + 1];
    l_src[tid] = src;
    l_dst[tid] = dst;
    l_blo[tid] = blo;
    l_bhi[tid] = bhi;
    l_drop[tid] = P.drop;
    l_s0[tid] = P.drop;
    l_ns[tid] = P.len - P.drop;
    l_M[tid] = P.newlen - (P.len - P.drop);
    w = l_ns[tid] + (u32)(bhi - blo);
  }
  const u32 winc = jyscan::wave_incl<u32>(w);  // a key tile is one wave
  const u32 wo = winc - w, wtot = __shfl(winc, 63);
  if (tid < nt) l_woff[tid] = wo;
  if (tid == 0) l_woff[nt] = wtot;
  __syncthreads();
  if (wtot == 0) return;
  // one pass per kTile items, from the last item down.  The next (lower)
  // pass's item and record loads are issued before this pass's stores: a
  // lower pass reads only positions below this pass's lowest item of the
  // same key, and this pass writes at or above it (entries only move up), so
  // the prefetch never reads what this pass writes; every pass still reads
  // before the passes above it have stored.
  struct CItem {
    bool live, st;
    u32 a, qx, rank;
    u64 i, j;
    TRec x;
  };
  auto fetch = [&](long long c0) {
    CItem c{};
    const u32 item = (u32)c0 + tid;
    c.live = item < wtot;
    if (c.live) {
      u32 h = nt - 1;  // last idx with woff <= item (a key with items)
      u32 a = 0;
      while (a < h) {
        const u32 m = (a + h + 1) >> 1;
        if (l_woff[m] <= item) a = m;
        else h = m - 1;
      }
      c.a = a;
      const u32 r = item - (u32)l_woff[a];
      c.st = r < l_ns[a];
      c.i = l_s0[a] + r;
      c.j = l_blo[a] + (r - l_ns[a]);
      if (c.st) {
        c.x = load_rec(A.pool + l_src[a] + c.i);
      } else {
        c.qx = eqx[c.j];
        c.x.ts = A.dts[c.j];
        c.x.pre = A.dpre[c.j];
        c.x.lr = A.dlr[c.j];
        c.rank = erank[c.j];
        c.x.pad = rec_w2(c.x.lr, A.arena);
      }
    }
    return c;
  };
  long long c0 = (long long)((wtot - 1) / kTile) * kTile;
  CItem cur = fetch(c0);
  for (; c0 >= 0; c0 -= kTile) {
    CItem nxt{};
    if (c0 >= kTile) nxt = fetch(c0 - kTile);
    const u32 a = cur.a;
    u32 qx = cur.qx;
    u64 lo = 0;
    if (cur.live && cur.st) {
      // first delta entry with rank <= i: the ranks do not increase along
      // the (newest-first) delta segment, so the entries ranked above i are
      // a prefix.  A short segment is counted with its ranks loaded at once
      // (one round trip), a long one bisected.
      const u64 i = cur.i;
      lo = l_blo[a];
      u64 hi = l_bhi[a];
      constexpr u64 kLin = 4;
      if (hi - lo <= kLin) {
        // a short segment: its ranks and kept flags in one round trip; qx
        // gets the kept count before lo (what eqx[lo] would hold)
        u32 rk[kLin], kq[kLin];
#pragma unroll
        for (u64 e = 0; e < kLin; e++) {
          rk[e] = lo + e < hi ? erank[lo + e] : 0u;
          kq[e] = lo + e < hi ? eqx[lo + e] : 0u;
        }
        u64 c = 0;
        u32 q = 0;
#pragma unroll
        for (u64 e = 0; e < kLin; e++) {
          const bool above = (lo + e < hi) & (rk[e] > i);
          c += above;
          q += above & ((kq[e] & kKept) != 0);
        }
        lo += c;
        qx = q;
      } else {
        while (lo < hi) {
          const u64 m = (lo + hi) >> 1;
          if (erank[m] <= i) hi = m;
          else lo = m + 1;
        }
        qx = lo < l_bhi[a] ? eqx[lo] : 0u;
      }
    }
    if (cur.live) {
      const u32 M = l_M[a];
      u64 pos;
      bool write = true;
      if (cur.st) {
        pos = (cur.i - l_drop[a]) + (lo < l_bhi[a] ? M - (qx & ~kKept) : 0u);
      } else {
        write = (qx & kKept) != 0;
        pos = (u64)(cur.rank - l_drop[a]) + (M - 1 - (qx & ~kKept));
      }
      if (write) store_rec(pool + l_dst[a] + pos, cur.x.ts, cur.x.pre, cur.x.lr, cur.x.pad);
    }
    cur = nxt;
  }
}

// the bump pointer moves only if the rebuilt logs were written (the same
// check as k_tlog_commit's); the outcome goes to the merge's words of mapped
// host memory: bump pointer after it, rebuilt entries, 1 if spilled
__global__ void k_tlog_bump(u64* __restrict__ ctr, const u64* __restrict__ roff, u64 tiles, u64 pcap,
                            u64* __restrict__ pin) {
  const u64 total = roff[tiles];
  const bool over = ctr[0] + total > pcap;
  if (!over) ctr[0] += total;
  __hip_atomic_store(pin, ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(pin + 1, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(pin + 2, (u64)over, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr u32 kTileOut = 2048;

// ---- compaction: every log rewritten back to back into a fresh pool ----
__global__ __launch_bounds__(kThreads) void k_cmp_size(const TMeta* __restrict__ meta, const u64* __restrict__ hist,
                                                       u32 epoch, u64 nk, u64* __restrict__ sz,
                                                       u64* __restrict__ lens) {
  const u64 s = gid();
  if (s > nk) return;
  if (s == nk) {
    sz[s] = lens[s] = 0;
    return;
  }
  const TMeta m = meta[s];
  const u32 n = m.len;
  // headroom for appends: as long again, and never less than the segment had
  // (a merge between its tile and commit pass may have planned an in-place
  // insert against that capacity)
  // (and front room below the log); a log with an update history gets room
  // for kHorizon merges at its rate, as a rebuild does
  const u64 hr = hist_room(hist[s], n, epoch);
  u64 want = (u64)n + (n > 4 ? n : 4);
  if ((u64)n + hr > want) want = (u64)n + hr;
  sz[s] = n ? (want > m.cap ? want : m.cap) + cmp_front(n) : 0;
  lens[s] = n;
}

// a tile of kTileOut output entries: its first and last logs found by two
// wave searches, their offsets and segments staged in LDS (per-entry search
// there), then the live entries copied (coalesced stores)
constexpr u32 kCmpLds = 1024;
__global__ __launch_bounds__(kThreads) void k_cmp_copy(const TMeta* __restrict__ meta, u64 nk,
                                                       const u64* __restrict__ roff, const TRec* __restrict__ src,
                                                       TRec* __restrict__ dst) {
  __shared__ u64 l_off[kCmpLds + 1], l_base[kCmpLds];
  __shared__ u32 l_len[kCmpLds];
  __shared__ u64 sh[2];
  const u64 total = roff[nk];
  const u64 t0 = (u64)blockIdx.x * kTileOut;
  if (t0 >= total) return;
  const u64 t1 = t0 + kTileOut < total ? t0 + kTileOut : total;
  if (threadIdx.x < 128) {
    const u64 k = jyscan::wave_last_le(roff, nk, threadIdx.x < 64 ? t0 : t1 - 1);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = k;
  }
  __syncthreads();
  const u64 k0 = sh[0], cnt = sh[1] - sh[0] + 1;
  const bool lds = cnt <= kCmpLds;
  if (lds) {
    for (u64 j = threadIdx.x; j < cnt; j += kThreads) {
      const TMeta m = meta[k0 + j];
      l_off[j] = roff[k0 + j] + cmp_front(m.len);  // the log's first entry
      l_base[j] = tm_base(m);
      l_len[j] = m.len;
    }
  }
  __syncthreads();
  for (u64 t = t0 + threadIdx.x; t < t1; t += kThreads) {
    u64 base, r;
    u32 len;
    if (lds) {
      u32 lo = 0, hi = (u32)cnt - 1;
      while (lo < hi) {
        const u32 m = (lo + hi + 1) >> 1;
        if (l_off[m] <= t) lo = m;
        else hi = m - 1;
      }
      base = l_base[lo], len = l_len[lo], r = t - l_off[lo];  // wraps below the log: skipped
    } else {
      u64 lo = k0, hi = k0 + cnt - 1;
      while (lo < hi) {
        const u64 m = (lo + hi + 1) >> 1;
        if (roff[m] <= t) lo = m;
        else hi = m - 1;
      }
      const TMeta m = meta[lo];
      base = tm_base(m), len = m.len, r = t - roff[lo] - cmp_front(m.len);
    }
    if (r >= len) continue;  // headroom
    const TRec x = load_rec(src + base + r);
    store_rec(dst + t, x.ts, x.pre, x.lr, x.pad);
  }
}

__global__ __launch_bounds__(kThreads) void k_cmp_meta(TMeta* __restrict__ meta, u64 nk, const u64* __restrict__ roff) {
  const u64 s = gid();
  if (s >= nk) return;
  const u32 f = cmp_front(meta[s].len);
  meta[s].bf = tm_bf(roff[s] + f, f);
  meta[s].cap = (u32)(roff[s + 1] - roff[s] - f);
}

// ---- reads ----
__global__ __launch_bounds__(kThreads) void k_tlog_sizes(const TMeta* __restrict__ meta, const u32* __restrict__ slots,
                                                         u64 n, u64* __restrict__ len, u64* __restrict__ cut) {
  const u64 i = gid();
  if (i >= n) return;
  const TMeta m = meta[slots[i]];
  len[i] = m.len;
  cut[i] = m.cut;
}

// newest first, as GET shows it (repo_tlog.pony:69-83)
__global__ __launch_bounds__(kThreads) void k_tlog_gather(const TMeta* __restrict__ meta,
                                                          const TRec* __restrict__ pool,
                                                          const u32* __restrict__ slots, const u64* __restrict__ ooff,
                                                          u64 n, u64* __restrict__ ots, u64* __restrict__ opre,
                                                          u64* __restrict__ olr) {
  const u64 i = gid();
  if (i >= n) return;
  const TMeta m = meta[slots[i]];
  u64 o = ooff[i];
  for (u64 q = m.len; q-- > 0; o++) {
    const TRec& x = pool[tm_base(m) + q];
    ots[o] = x.ts;
    opre[o] = x.pre;
    olr[o] = x.lr;
  }
}

__global__ __launch_bounds__(kThreads) void k_seg_starts(const u64* __restrict__ offs, u64 nseg, u32* __restrict__ out) {
  const u64 k = gid();
  if (k < nseg && offs[k] < offs[k + 1]) out[offs[k]] = (u32)k;
}

// ---- write path: RepoTLOG.ins / trimat / trim / clr (repo_tlog.pony:85-111) ----
// Each command (one per key here) becomes a delta log for the state -- at
// most one entry, and a cutoff -- judged against the state as it is:
//   INS     the entry (ts, value); changes the state iff ts >= cutoff and the
//           entry is new (TLog.write)
//   TRIMAT  cutoff ts; changes iff ts > cutoff (raise_cutoff)
//   TRIM n  cutoff = ts of the n-th newest entry (n == 0: CLR; past the end:
//           nothing, as the reference's try swallows the bounds error)
//   CLR     cutoff = newest ts + 1 (U64 wraps), nothing on an empty log
// and, where the state changed, the same delta goes to the key's pending
// delta log (d.write / d.raise_cutoff(l.cutoff) of the reference).  Every
// command marks its key pending (_delta_for runs either way).
struct WCmd {
  const uint8_t* op;
  const u32* slot;
  const u64* ts;
  const u64* arg;
  const u64* pre;
  const u64* lr;
};
__global__ __launch_bounds__(kThreads) void k_tlog_wprep(WCmd W, u64 n, const TMeta* __restrict__ meta,
                                                         const TRec* __restrict__ pool,
                                                         const uint8_t* __restrict__ arena, u64* __restrict__ scut,
                                                         u64* __restrict__ sflag, u64* __restrict__ dcut,
                                                         u64* __restrict__ dflag, u32* __restrict__ pend,
                                                         u64* __restrict__ pcount) {
  const u64 i = gid();
  if (i >= n) return;
  const u32 s = W.slot[i];
  const TMeta m = meta[s];
  u64 raise = 0;
  bool ent = false, changed = false;
  const uint8_t op = W.op[i];
  if (op == JY_TLOG_INS) {
    ent = true;
    const Ent x{W.ts[i], W.pre[i], W.lr[i]};
    if (x.t >= m.cut) {  // present? the log is ascending (ts, value) from base
      u64 lo = tm_base(m), hi = tm_base(m) + m.len;
      while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (cmp_at(pool, mid, x, arena) < 0) lo = mid + 1;
        else hi = mid;
      }
      changed = !(lo < tm_base(m) + m.len && cmp_at(pool, lo, x, arena) == 0);
    }
  } else if (op == JY_TLOG_TRIMAT) {
    raise = W.ts[i];
    changed = raise > m.cut;
  } else {
    const u64 cnt = op == JY_TLOG_CLR ? 0 : W.arg[i];
    if (cnt == 0) {
      if (m.len) {
        raise = m.newest + 1;
        changed = raise > m.cut;
      }
    } else if (cnt - 1 < m.len) {
      raise = pool[tm_base(m) + m.len - cnt].ts;
      changed = raise > m.cut;
    }
    if (!changed) raise = 0;
  }
  scut[i] = raise;
  sflag[i] = ent;
  dcut[i] = changed ? raise : 0;
  dflag[i] = ent && changed;
  jy_wave_count(atomicExch(pend + s, 1u) == 0, (unsigned long long*)pcount);
}

// the entries of the INS commands, packed for the state's delta (positions
// from the scan of sflag) and for the pending deltas (scan of dflag)
__global__ __launch_bounds__(kThreads) void k_tlog_wpack(WCmd W, u64 n, const u64* __restrict__ soff,
                                                         const u64* __restrict__ doff, u64* __restrict__ sts,
                                                         u64* __restrict__ spre, u64* __restrict__ slr,
                                                         u64* __restrict__ dts, u64* __restrict__ dpre,
                                                         u64* __restrict__ dlr) {
  const u64 i = gid();
  if (i >= n) return;
  if (soff[i + 1] != soff[i]) {
    const u64 o = soff[i];
    sts[o] = W.ts[i];
    spre[o] = W.pre[i];
    slr[o] = W.lr[i];
  }
  if (doff[i + 1] != doff[i]) {
    const u64 o = doff[i];
    dts[o] = W.ts[i];
    dpre[o] = W.pre[i];
    dlr[o] = W.lr[i];
  }
}

// flush: the pending keys' delta logs are emptied (their pool space is
// released wholesale: every pending key is flushed at once)
__global__ __launch_bounds__(kThreads) void k_tlog_wreset(TMeta* __restrict__ dmeta, u32* __restrict__ pend,
                                                          const u32* __restrict__ slots, u64 n) {
  const u64 i = gid();
  if (i >= n) return;
  const u32 s = slots[i];
  dmeta[s] = TMeta{0, 0, 0, 0, 0};
  pend[s] = 0;
}

struct PendPred {
  const u32* pend;
  __device__ bool operator()(u64 s) const { return pend[s] != 0; }
};

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

#define LAUNCH(k, n, ...)                                                                          \
  do {                                                                                             \
    hipLaunchKernelGGL(k, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, __VA_ARGS__);     \
    JY_HIP(eng, hipGetLastError());                                                                \
  } while (0)

int32_t scan_excl_u64(jy_engine* eng, const u64* in, u64* out, u64 n_plus_1) {
  return jydscan::scan<jydscan::OpSum, false>(eng, n_plus_1, jydscan::LdArr<u64>{in}, jydscan::StArr<u64>{out});
}

// rewrite every log back to back into a fresh pool with `room` free entries
// after them; synchronises (the new size is read back)
int32_t tlog_compact(jy_engine* eng, TlogState& t, u64 room) {
  const u64 nk = eng->nkeys[JY_TLOG];
  const double t_enter = jy_tracing() ? jy_now_us() : 0;
  void* p;
  JY_TRY(jy_scratch(eng, 17, (nk + 1) * 32, &p));
  u64* sz = static_cast<u64*>(p);
  u64* roff = sz + nk + 1;
  u64* lens = roff + nk + 1;
  u64* loff = lens + nk + 1;
  LAUNCH(k_cmp_size, nk + 1, t.meta, t.hist, eng->tl_epoch, nk, sz, lens);
  JY_TRY(scan_excl_u64(eng, sz, roff, nk + 1));
  JY_TRY(scan_excl_u64(eng, lens, loff, nk + 1));
  JY_HIP(eng, hipMemcpyAsync(t.pin, roff + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(t.pin + 1, loff + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  const u64 total = t.pin[0], live = t.pin[1];
  // the next merges' worst case fits several times over before the next sync
  // 6x the live entries: a compaction costs a copy of the pool, so they
  // should be rare (HBM is plentiful: 4M logs of ~15 entries -> ~12 GB)
  const u64 ncap = std::max<u64>({total + room, 6 * total, eng->cfg.entry_capacity[JY_TLOG], 1024});
  TRec* np = nullptr;
  JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&np), ncap * sizeof(TRec), "tlog pool"));
  if (total) {
    const u32 tiles = (u32)std::max<u64>(1, (total + kTileOut - 1) / kTileOut);
    hipLaunchKernelGGL(k_cmp_copy, dim3(tiles), dim3(kThreads), 0, eng->stream, t.meta, nk, roff, t.pool, np);
    JY_HIP(eng, hipGetLastError());
  }
  if (nk) LAUNCH(k_cmp_meta, nk, t.meta, nk, roff);
  jy_dev_free(eng, t.pool);
  t.pool = np;
  t.pcap = ncap;
  *t.pin = total;
  JY_HIP(eng, hipMemcpyAsync(t.ctr, t.pin, 8, hipMemcpyHostToDevice, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));  // pin is reused right away
  t.used = total;
  t.compact_seq = t.seq;
  t.compactions++;
  (void)live;
  JY_TRACE("tlog compact: %llu entries, pool %llu, %.1f us", (unsigned long long)total, (unsigned long long)ncap,
           jy_now_us() - t_enter);
  return JY_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// device exclusive scan: out[0..n] with out[n] = total (in[n] must be 0)
int32_t jy_scan_u64(jy_engine* eng, const u64* in, u64* out, u64 n) { return scan_excl_u64(eng, in, out, n + 1); }

// segment id of every item of a CSR (offs[0..nseg], n items): mark each
// non-empty segment's first item, then an inclusive max-scan carries it on
int32_t jy_seg_ids(jy_engine* eng, const u64* offs, u64 nseg, u64 n, u32* out) {
  if (n == 0) return JY_OK;
  JY_HIP(eng, hipMemsetAsync(out, 0, n * 4, eng->stream));
  LAUNCH(k_seg_starts, nseg, offs, nseg, out);
  // in place: a tile loads its items before it stores them, and no other tile reads them
  return jydscan::scan<jydscan::OpMax, true>(eng, n, jydscan::LdArr<u32>{out}, jydscan::StArr<u32>{out});
}

int32_t tlog_grow_store(jy_engine* eng, TlogState& t, u64 need) {
  if (!t.ctr) {
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&t.ctr), 64, "tlog counters"));
    JY_HIP(eng, hipMemsetAsync(t.ctr, 0, 64, eng->stream));
    JY_HIP(eng, hipHostMalloc(reinterpret_cast<void**>(&t.pin), 8 * (8 + 4 * (TlogState::kSpill + 1)),
                              hipHostMallocMapped));
    std::memset(t.pin, 0, 8 * (8 + 4 * (TlogState::kSpill + 1)));
    JY_HIP(eng, hipHostGetDevicePointer(reinterpret_cast<void**>(&t.pin_dev), t.pin, 0));
    for (auto& sp : t.spill) JY_HIP(eng, hipEventCreateWithFlags(&sp.done, hipEventDisableTiming));
    t.pcap = std::max<u64>(eng->cfg.entry_capacity[JY_TLOG], 1024);
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&t.pool), t.pcap * sizeof(TRec), "tlog pool"));
  }
  if (need <= t.kcap && t.meta) return JY_OK;
  u64 nk = std::max<u64>(need, t.kcap ? t.kcap * 2 : need);
  nk = std::max<u64>((nk + 63) & ~63ull, 64);
  void* m = t.meta;
  JY_TRY(jy_realloc(eng, &m, t.kcap * sizeof(TMeta), nk * sizeof(TMeta), true));  // empty logs
  t.meta = static_cast<TMeta*>(m);
  void* hs = t.hist;
  JY_TRY(jy_realloc(eng, &hs, t.kcap * 8, nk * 8, true));
  t.hist = static_cast<u64*>(hs);
  void* h = t.hint;
  JY_TRY(jy_realloc(eng, &h, t.kcap * 8, nk * 8, true));
  t.hint = static_cast<u64*>(h);
  t.kcap = nk;
  return JY_OK;
}

int32_t jy_tlog_grow(jy_engine* eng, u64 need) {
  JY_TRY(tlog_grow_store(eng, eng->tlog, need));
  if (eng->tlog_d.ctr) JY_TRY(tlog_grow_store(eng, eng->tlog_d, eng->tlog.kcap));
  return JY_OK;
}

// new slots start as empty logs: their meta is zeroed when it is allocated
int32_t jy_tlog_extend(jy_engine*, u64, u64) { return JY_OK; }

int32_t jy_tlog_merge(jy_engine* eng, u64 nd, const u32* slot, const u64* dcut, const u64* doff, u64 nent,
                      const u64* dts, const u64* dpre, const u64* dlr) {
  JyTimed tm(eng);
  return jy_tlog_merge_into(eng, eng->tlog, nd, slot, dcut, doff, nent, dts, dpre, dlr);
}

namespace {

// spill buffer views of ring slot r sized for (nd, nent)
int32_t spill_reserve(jy_engine* eng, TlogState::Spill& sp, u64 nd, u64 nent) {
  const u64 bytes = ((nd * 4 + 15) & ~15ull) + (2 * nd + 1) * 8 + 3 * std::max<u64>(nent, 1) * 8 + 64;
  if (sp.buf.bytes < bytes) {
    jy_dev_free(eng, sp.buf.p);
    sp.buf.p = nullptr;
    sp.buf.bytes = 0;
    const u64 nb = std::max<u64>(bytes, sp.buf.bytes * 2);
    JY_TRY(jy_dev_alloc(eng, &sp.buf.p, nb, "tlog spill"));
    sp.buf.bytes = nb;
  }
  sp.nd = nd;
  sp.nent = nent;
  return JY_OK;
}

struct SpillView {
  u32* slot;
  u64 *cut, *off, *ts, *pre, *lr;
};
SpillView spill_view(const TlogState::Spill& sp) {
  SpillView v;
  v.slot = static_cast<u32*>(sp.buf.p);
  v.cut = reinterpret_cast<u64*>(static_cast<char*>(sp.buf.p) + ((sp.nd * 4 + 15) & ~15ull));
  v.off = v.cut + sp.nd;
  v.ts = v.off + sp.nd + 1;
  v.pre = v.ts + std::max<u64>(sp.nent, 1);
  v.lr = v.pre + std::max<u64>(sp.nent, 1);
  return v;
}

// enqueue one merge of a device batch into store t; spill ring slot r
// receives its rebuilt keys if they do not fit the pool.  Never waits.
int32_t tlog_launch(jy_engine* eng, TlogState& t, int r, u64 nd, const u32* slot, const u64* dcut, const u64* doff,
                    u64 nent, const u64* dts, const u64* dpre, const u64* dlr) {
  const u64 nk = eng->nkeys[JY_TLOG];
  TlogState::Spill& sp = t.spill[r];
  JY_TRY(spill_reserve(eng, sp, nd, nent));
  const SpillView v = spill_view(sp);
  TlogArgs A{};
  A.arena = eng->arena[JY_TLOG].p;
  A.nd = nd;
  A.slot = slot;
  A.dcut = dcut;
  A.doff = doff;
  A.dts = dts;
  A.dpre = dpre;
  A.dlr = dlr;
  A.skipped = reinterpret_cast<unsigned long long*>(eng->skipped_dev);
  A.pcap = t.pcap;
  A.sp_slot = v.slot;
  A.sp_cut = v.cut;
  A.sp_off = v.off;
  A.sp_ts = v.ts;
  A.sp_pre = v.pre;
  A.sp_lr = v.lr;
  void* p;
  {
    DevArray& c = eng->tl_claim;
    if (c.bytes < nk * 8) {  // grows rarely: the whole array (re)set to epoch 0 once
      const u64 nb = std::max<u64>(nk * 8, c.bytes * 2);
      jy_dev_free(eng, c.p);
      c.p = nullptr;
      c.bytes = 0;
      JY_TRY(jy_dev_alloc(eng, &c.p, nb, "tlog slot claims"));
      c.bytes = nb;
      JY_HIP(eng, hipMemsetAsync(c.p, 0, nb, eng->stream));
    }
    DevArray& b = eng->tl_bad;
    if (b.bytes < nd * 4) {  // grows rarely: zero (epoch 0) once
      const u64 nb = std::max<u64>(nd * 4, b.bytes * 2);
      jy_dev_free(eng, b.p);
      b.p = nullptr;
      b.bytes = 0;
      JY_TRY(jy_dev_alloc(eng, &b.p, nb, "tlog repeated-slot marks"));
      b.bytes = nb;
      JY_HIP(eng, hipMemsetAsync(b.p, 0, nb, eng->stream));
    }
    if (++eng->tl_epoch == 0) {  // wrapped: no old tag may match a new epoch
      JY_HIP(eng, hipMemsetAsync(c.p, 0, c.bytes, eng->stream));
      JY_HIP(eng, hipMemsetAsync(b.p, 0, b.bytes, eng->stream));
      eng->tl_epoch = 1;
    }
    A.bad = static_cast<u32*>(b.p);
    A.dptr = static_cast<u64*>(c.p);
    A.epoch = eng->tl_epoch;
  }
  JY_TRY(jy_scratch(eng, 9, nd * (sizeof(PInfo) + 12) + 64, &p));
  A.pinfo = static_cast<PInfo*>(p);
  A.rz = reinterpret_cast<u32*>(A.pinfo + nd);
  const u32 tiles = (u32)((nd + kTile - 1) / kTile);
  JY_TRY(jy_scratch(eng, 16, ((u64)tiles + 1) * 8, &p));
  A.rsum = static_cast<u64*>(p);  // per key tile, then (scanned in place) each tile's offset; [tiles] = total
  JY_TRY(jy_scratch(eng, 12, std::max<u64>(nent, 1) * 8, &p));
  u32* erank = static_cast<u32*>(p);
  u32* eqx = erank + std::max<u64>(nent, 1);
  JY_HIP(eng, hipMemsetAsync(A.rsum + tiles, 0, 8, eng->stream));
  LAUNCH(k_tlog_prep, nd, A);
  A.meta = t.meta;
  A.hint = t.hint;
  A.hist = t.hist;
  A.pool = t.pool;
  hipLaunchKernelGGL(k_tlog_tile, dim3(tiles), dim3(kTile), 0, eng->stream, A, t.pool, erank, eqx);
  JY_HIP(eng, hipGetLastError());
  // one offset per 64-key tile (a key's own offset is a wave prefix in k_tlog_commit): 64x fewer
  // items than a scan over every key (61 -> a few us at 4M keys)
  JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, (u64)tiles + 1, jydscan::LdArr<u64>{A.rsum},
                                                jydscan::StArr<u64>{A.rsum})));
  hipLaunchKernelGGL(k_tlog_commit, dim3(tiles), dim3(kTile), 0, eng->stream, A, A.rsum, t.ctr, t.pool, erank, eqx);
  JY_HIP(eng, hipGetLastError());
  hipLaunchKernelGGL(k_tlog_bump, dim3(1), dim3(1), 0, eng->stream, t.ctr, A.rsum, (u64)tiles, t.pcap,
                     t.pin_dev + 8 + 4 * r);
  JY_HIP(eng, hipGetLastError());
#ifdef JY_TLOG_PROBE
  if (const char* path = getenv("JY_TLOG_PROBE_OUT")) {
    static unsigned long long buf[kProbeSlots][kProbeN];
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
    JY_HIP(eng, hipMemcpyFromSymbol(buf, HIP_SYMBOL(g_tprobe), sizeof(buf)));
    unsigned long long tot[kProbeN] = {};
    for (int i = 0; i < kProbeSlots; i++)
      for (int j = 0; j < kProbeN; j++) tot[j] += buf[i][j];
    if (FILE* f = fopen(path, "a")) {
      const double n = tot[0] ? (double)tot[0] : 1.0;
      fprintf(f, "merge %llu tiles %llu | per tile (us): s1 %.2f s2 %.2f [load %.2f search %.2f end %.2f] s3 %.2f s4 %.2f "
              "s5 %.2f | slow ent %.1f passes %.2f s5 items %.1f s5 passes %.2f\n", (unsigned long long)t.seq, tot[0],
              tot[1] / n / 100, tot[2] / n / 100, tot[10] / n / 100, tot[11] / n / 100, tot[12] / n / 100,
              tot[3] / n / 100, tot[4] / n / 100, tot[5] / n / 100, tot[6] / n, tot[7] / n, tot[8] / n, tot[9] / n);
      fclose(f);
    }
    std::memset(buf, 0, sizeof(buf));
    JY_HIP(eng, hipMemcpyToSymbol(HIP_SYMBOL(g_tprobe), buf, sizeof(buf)));
  }
#endif
  JY_HIP(eng, hipEventRecord(sp.done, eng->stream));
  sp.seq = ++t.seq;
  sp.busy = true;
  return JY_OK;
}

// absorb the outcome of ring slot r's merge (waits for it); a spilled merge
// is re-merged after a compaction sized for it
int32_t tlog_absorb(jy_engine* eng, TlogState& t, int r) {
  TlogState::Spill& sp = t.spill[r];
  JY_HIP(eng, hipEventSynchronize(sp.done));
  sp.busy = false;
  const u64* w = t.pin + 8 + 4 * r;
  const u64 used = __atomic_load_n(w, __ATOMIC_ACQUIRE), rebuilt = w[1], over = w[2];
  if (sp.seq > t.compact_seq) t.used = used;
  if (!over) return JY_OK;
  // room for the spilled rebuilds several times over
  t.spills++;
  JY_TRACE("tlog: merge %llu spilled %llu rebuilt entries (pool %llu of %llu used)", (unsigned long long)sp.seq,
           (unsigned long long)rebuilt, (unsigned long long)used, (unsigned long long)t.pcap);
  JY_TRY(tlog_compact(eng, t, 4 * (rebuilt + sp.nent) + 1024));
  const SpillView v = spill_view(sp);
  constexpr int R = TlogState::kSpill;
  JY_TRY(tlog_launch(eng, t, R, sp.nd, v.slot, v.cut, v.off, sp.nent, v.ts, v.pre, v.lr));
  JY_HIP(eng, hipEventSynchronize(t.spill[R].done));
  t.spill[R].busy = false;
  const u64* w2 = t.pin + 8 + 4 * R;
  if (w2[2]) return eng->fail(JY_ENOMEM, "tlog pool: no room for a spilled merge after compaction");
  t.used = w2[0];
  return JY_OK;
}

// absorb finished merges, oldest first; with `block`, every merge in flight
int32_t tlog_reap(jy_engine* eng, TlogState& t, bool block) {
  for (;;) {
    int r = -1;
    for (int i = 0; i < TlogState::kSpill; i++)
      if (t.spill[i].busy && (r < 0 || t.spill[i].seq < t.spill[r].seq)) r = i;
    if (r < 0) return JY_OK;
    if (!block && hipEventQuery(t.spill[r].done) == hipErrorNotReady) return JY_OK;
    JY_TRY(tlog_absorb(eng, t, r));
  }
}

}  // namespace

extern "C" int32_t jy_tlog_stats(jy_engine* eng, uint64_t* out4) {
  JY_HIP(eng, hipSetDevice(eng->device));
  const TlogState& t = eng->tlog;
  out4[0] = t.seq;
  out4[1] = t.spills;
  out4[2] = t.compactions;
  out4[3] = t.pcap;
  return JY_OK;
}

int32_t jy_tlog_settle(jy_engine* eng) {
  if (eng->tlog.ctr) JY_TRY(tlog_reap(eng, eng->tlog, true));
  if (eng->tlog_d.ctr) JY_TRY(tlog_reap(eng, eng->tlog_d, true));
  return JY_OK;
}

// the merge into one store: the state, or the pending deltas of the write path.
// Only enqueues: no host wait unless every spill buffer is still in flight
// (kSpill merges ahead of the GPU), when it waits for the oldest.
int32_t jy_tlog_merge_into(jy_engine* eng, TlogState& t, u64 nd, const u32* slot, const u64* dcut, const u64* doff,
                           u64 nent, const u64* dts, const u64* dpre, const u64* dlr) {
  const u64 nk = eng->nkeys[JY_TLOG];
  if (nd == 0 || nk == 0) return JY_OK;
  JY_TRY(tlog_reap(eng, t, false));
  int r = -1;
  for (int i = 0; i < TlogState::kSpill && r < 0; i++)
    if (!t.spill[i].busy) r = i;
  if (r < 0) {  // every ring slot in flight: settle the oldest
    r = 0;
    for (int i = 1; i < TlogState::kSpill; i++)
      if (t.spill[i].seq < t.spill[r].seq) r = i;
    JY_TRY(tlog_absorb(eng, t, r));
  }
  return tlog_launch(eng, t, r, nd, slot, dcut, doff, nent, dts, dpre, dlr);
}

int32_t jy_tlog_sizes(jy_engine* eng, u64 n, const u32* slots, u64* len, u64* cut) {
  JY_TRY(jy_tlog_settle(eng));
  TlogState& t = eng->tlog;
  LAUNCH(k_tlog_sizes, n, t.meta, slots, n, len, cut);
  return JY_OK;
}

int32_t jy_tlog_gather(jy_engine* eng, u64 n, const u32* slots, const u64* ooff, u64* ts, u64* pre, u64* lr) {
  JY_TRY(jy_tlog_settle(eng));
  TlogState& t = eng->tlog;
  LAUNCH(k_tlog_gather, n, t.meta, t.pool, slots, ooff, n, ts, pre, lr);
  return JY_OK;
}

// ---- TLOG write path --------------------------------------------------------
namespace {
int32_t tlog_pending_grow(jy_engine* eng) {
  TlogState& d = eng->tlog_d;
  JY_TRY(tlog_grow_store(eng, d, eng->tlog.kcap));
  if (!eng->tl_dcount) {
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&eng->tl_dcount), 8, "tlog pending count"));
    JY_HIP(eng, hipMemsetAsync(eng->tl_dcount, 0, 8, eng->stream));
  }
  if (eng->tl_dkcap < d.kcap || !eng->tl_dflag) {
    void* f = eng->tl_dflag;
    JY_TRY(jy_realloc(eng, &f, eng->tl_dkcap * 4, d.kcap * 4, true));
    eng->tl_dflag = static_cast<u32*>(f);
    eng->tl_dkcap = d.kcap;
  }
  return JY_OK;
}
}  // namespace

int32_t jy_tlog_write_batch(jy_engine* eng, u64 n, const uint8_t* op, const u32* slot, const u64* ts, const u64* arg,
                            const u64* pre, const u64* lr) {
  if (n == 0) return JY_OK;
  JY_TRY(tlog_pending_grow(eng));
  // every command is judged against the state as it is: no merge may still be pending
  JY_TRY(jy_tlog_settle(eng));
  void* p;
  // (scratch 0..7 hold the staged commands; the merges use 8, 9, 12, 16)
  JY_TRY(jy_scratch(eng, 10, (n + 1) * 8 * 8 + 64, &p));
  u64* scut = static_cast<u64*>(p);
  u64* sflag = scut + (n + 1);
  u64* dcut = sflag + (n + 1);
  u64* dflag = dcut + (n + 1);
  u64* soff = dflag + (n + 1);
  u64* doff = soff + (n + 1);
  JY_TRY(jy_scratch(eng, 11, n * 8 * 6 + 64, &p));
  u64* sts = static_cast<u64*>(p);
  u64 *spre = sts + n, *slr = spre + n, *dts = slr + n, *dpre = dts + n, *dlr = dpre + n;
  const WCmd W{op, slot, ts, arg, pre, lr};
  TlogState& t = eng->tlog;
  JY_HIP(eng, hipMemsetAsync(sflag + n, 0, 8, eng->stream));
  JY_HIP(eng, hipMemsetAsync(dflag + n, 0, 8, eng->stream));
  LAUNCH(k_tlog_wprep, n, W, n, t.meta, t.pool, eng->arena[JY_TLOG].p, scut, sflag, dcut, dflag, eng->tl_dflag,
         eng->tl_dcount);
  JY_TRY(scan_excl_u64(eng, sflag, soff, n + 1));
  JY_TRY(scan_excl_u64(eng, dflag, doff, n + 1));
  LAUNCH(k_tlog_wpack, n, W, n, soff, doff, sts, spre, slr, dts, dpre, dlr);
  // n bounds the entry counts (the merges size from the device offsets)
  JY_TRY(jy_tlog_merge_into(eng, t, n, slot, scut, soff, n, sts, spre, slr));
  JY_TRY(jy_tlog_merge_into(eng, eng->tlog_d, n, slot, dcut, doff, n, dts, dpre, dlr));
  return JY_OK;
}

int32_t jy_tlog_pending(jy_engine* eng, u64* count) {
  *count = 0;
  if (!eng->tl_dcount) return JY_OK;
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, eng->tl_dcount, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  *count = eng->pin_total[0];
  return JY_OK;
}

// two calls: with caps too small (e.g. 0) it only reports the sizes; with
// room for both it writes (device arrays) and clears the pending deltas
int32_t jy_tlog_flush_dev(jy_engine* eng, u64 cap_keys, u64 cap_ent, u32* slots, u64* cut, u64* offs, u64* ts,
                          u64* pre, u64* lr, u64* nkeys, u64* nent) {
  u64 k = 0;
  JY_TRY(jy_tlog_settle(eng));
  JY_TRY(jy_tlog_pending(eng, &k));
  *nkeys = k;
  *nent = 0;
  if (k == 0) return JY_OK;
  TlogState& d = eng->tlog_d;
  void* p;
  JY_TRY(jy_scratch(eng, 13, k * 4 + (k + 1) * 24 + 64, &p));
  u32* sl = static_cast<u32*>(p);
  u64* lens = reinterpret_cast<u64*>((reinterpret_cast<uintptr_t>(sl + k) + 15) & ~uintptr_t(15));
  u64* cuts = lens + (k + 1);
  u64* loff = cuts + (k + 1);
  void* num;
  JY_TRY(jy_scratch(eng, 14, 8, &num));
  JY_TRY(jydscan::select(eng, std::min<u64>(eng->nkeys[JY_TLOG], eng->tl_dkcap), PendPred{eng->tl_dflag}, sl,
                         static_cast<u32*>(num)));
  JY_HIP(eng, hipMemsetAsync(lens + k, 0, 8, eng->stream));
  LAUNCH(k_tlog_sizes, k, d.meta, sl, k, lens, cuts);
  JY_TRY(scan_excl_u64(eng, lens, loff, k + 1));
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, loff + k, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  const u64 m = eng->pin_total[0];
  *nent = m;
  if (cap_keys < k || cap_ent < m) return JY_OK;  // sizes only
  JY_HIP(eng, hipMemcpyAsync(slots, sl, k * 4, hipMemcpyDeviceToDevice, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(cut, cuts, k * 8, hipMemcpyDeviceToDevice, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(offs, loff, (k + 1) * 8, hipMemcpyDeviceToDevice, eng->stream));
  if (m) LAUNCH(k_tlog_gather, k, d.meta, d.pool, sl, loff, k, ts, pre, lr);
  LAUNCH(k_tlog_wreset, k, d.meta, eng->tl_dflag, sl, k);
  JY_HIP(eng, hipMemsetAsync(eng->tl_dcount, 0, 8, eng->stream));
  // every pending key was flushed: the delta pool is empty again
  JY_HIP(eng, hipMemsetAsync(d.ctr, 0, 8, eng->stream));
  d.used = 0;
  d.compact_seq = d.seq;
  return JY_OK;
}
