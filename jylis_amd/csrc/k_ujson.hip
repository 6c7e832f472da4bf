// k_ujson.hip -- UJSON observed-remove dot-set union and tombstone filter, gfx950.
//
// Semantics (oracle/jy_oracle.cpp UJSON / CausalContext; ujson.md:172-182,
// repo_ujson.pony:65-66): a document is a set of (dot, element) pairs inside
// a causal context (version vector vv + dot cloud).  Join of state A with
// delta B:
//   keep (d, e) of A unless B's context saw d and B's map lacks d
//   add  (d, e) of B whose d A's context has not seen
//   equal dots: B's element replaces A's only if A's context lacks d
//   context := vv max + cloud union, compacted (cloud dots contiguous with
//              their column's vv are folded into the vv)
// Elements are opaque handles (interned (path, value) leaves).
//
// HBM layout per type: dots packed (column << 48 | seq); per document a
// UMeta naming its segment of the element pool (16-B records (dot, elem),
// ascending by dot) and of the cloud pool (dots ascending); dense vv
// [kcap][R].
//
// A converge touches ONLY the documents of its batch; every merged document
// is written as one fresh run at the pools' bump pointers and its UMeta
// repointed.  Untouched documents are never read or moved.
//
// Parallel shape: ONE THREAD PER ELEMENT / CLOUD DOT (the Zipf config-5
// stream puts tens of thousands of dots on its hottest documents, so a
// thread- or wave-per-document join serialises on them).  Every decision is
// local to one item given binary searches into the other side's sorted
// segment; output positions come from merge-path ranks,
//   pos(x) = out_off[doc] + #kept own-side before x + #kept other-side < x,
// with the kept counts from scans of keep flags.  A cloud dot x of column c
// above the merged vv v folds into the vv iff seq(x) == v + 1 + |union dots
// of c in (v, seq(x))|.
//
// FIVE item launches (+ two one-workgroup tile scans) per converge and no
// host round trip:
//   U1 k_uj_docs     per delta doc: slot claim, meta, scans of the touched-
//                    state sizes, the doc of every item (ids, or a tile map
//                    inside long segments); per delta item: validation and
//                    the dense delta vv
//   U2 k_uj_flags    keep flags and cross ranks of state / delta elements and
//                    delta cloud dedupe, tile-scanned
//   U3 k_uj_compact  cloud compaction against the merged vv (the state rows,
//                    raised in place by the folds, max the delta vv),
//                    tile-scanned
//   U4 k_uj_sizes    per-document output sizes, scanned; the pools' bump
//                    pointers move on the device
//   U5 k_uj_scatter  every kept item to its merge-path position; the delta's
//                    sparse vv entries into the state rows; metas; the dense
//                    delta vv back to zero
// No [docs][R] working rows: the state rows are read in place and only the
// delta's sparse vv entries are written back.  Doc scans are single-pass
// (jy_scan.hpp: tickets + decoupled look-back); item launches are persistent
// grids that read their sizes from device memory.  Claims (a slot named
// twice in one batch: both copies skipped) and bad marks carry the
// converge's epoch, so nothing is reset with a memset.  The host reads pool
// use back only through a mapped pinned word written by U4 and checks it
// when a later converge's worst case might not fit (then it compacts).
//
// Roofline: HBM.  Per touched element: 16 B read + 16 B written (+ 4 B
// scan value, written and read); per touched cloud dot 8 B read + 8 B
// written (+ 4 B); the delta's vv entries and the metas of delta docs.

#include <algorithm>
#include <cstring>

#include "jy_internal.hpp"
#include "jy_scan.hpp"

namespace {

// (in-box A/B, round 4, ms per config-5 converge: 128 threads 0.528, 256
// 0.494, 512 0.525 -- tiles, doc tiles and U1 item tiles all follow it)
#ifndef JY_UJ_THREADS
#define JY_UJ_THREADS 256
#endif
constexpr int kThreads = JY_UJ_THREADS;
// U1 items per thread (round 6, in-box A/B, ms per config-5 step: 4 items
// 0.495 / 0.495 / 0.494, 2 items 0.509 / 0.481 / 0.477, 1 item 0.469 /
// 0.478 / 0.468 -- a thread's items ran one after another: each item's
// stores kept the next item's loads behind them)
#ifndef JY_UJ_PER
#define JY_UJ_PER 1
#endif
constexpr int kPer = JY_UJ_PER;                 // items per thread in U1 item tiles
constexpr u64 kTile1 = (u64)kThreads * kPer;    // U1 item tiles
constexpr u64 kTile = kThreads;                 // U2 / U3 / U5 item tiles: one item per thread
constexpr u64 kDocTile = kThreads;              // docs per doc tile
constexpr u64 kLdsDocs = 1023;                  // docs a tile stages in LDS for its search

enum { T_U1 = 0, T_U2, T_U3, T_U4, T_U5 };  // ticket counters

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u32 dcol(u64 d) { return (u32)(d >> JY_DOT_SEQ_BITS); }
__device__ __forceinline__ u64 dseq(u64 d) { return d & JY_DOT_SEQ_MASK; }
__device__ __forceinline__ u64 mkdot(u64 c, u64 q) { return (c << JY_DOT_SEQ_BITS) | q; }

// first index in [lo, hi) with a[i] >= x (a sorted): bisect down to 8
// candidates, then load those at once and count -- one round trip for the
// short segments of a typical document instead of one per level
template <bool kRec>
__device__ __forceinline__ u64 dot_at(const void* src, u64 i) {
  return kRec ? static_cast<const URec*>(src)[i].dot : static_cast<const u64*>(src)[i];
}
template <bool kRec>
__device__ __forceinline__ u64 lb_g(const void* src, u64 lo, u64 hi, u64 x) {
  while (hi - lo > 8) {
    const u64 m = (lo + hi) >> 1;
    if (dot_at<kRec>(src, m) < x) lo = m + 1;
    else hi = m;
  }
  if (lo >= hi) return lo;
  const u64 n = hi - lo;
  u32 c = 0;
#pragma unroll
  for (u32 j = 0; j < 8; j++) {
    const u64 v = dot_at<kRec>(src, lo + (j < n ? j : 0));
    c += (j < n) & (v < x);
  }
  return lo + c;
}
__device__ __forceinline__ u64 lower_bound(const u64* __restrict__ a, u64 lo, u64 hi, u64 x) {
  return lb_g<false>(a, lo, hi, x);
}

// ---- wave-cooperative lower bounds (every lane of a wave calls with the
// same searches): 64-ary probes per round, so a segment of n sorted dots
// costs ceil(log64 n) dependent round trips instead of ~log2 n; the N
// searches advance together (each round issues all their probes at once).
// A wave whose 64 items lie in ONE long document bounds every item's search
// this way (the other side's range between its first and last dot), and the
// items then search only those few entries.
struct WSearch {
  const u64* a;  // dots at a[i * stride]
  u32 stride;
  u64 lo, hi, x;  // in: range and key; out: lo = hi = first index with a >= x
};
template <int N>
__device__ __forceinline__ void wave_lbs(WSearch (&s)[N]) {
  const u64 lane = __lane_id();
  for (;;) {  // wave-uniform: lo / hi come from ballots
    bool more = false;
    u64 v[N], step[N];
#pragma unroll
    for (int q = 0; q < N; q++) {
      step[q] = s[q].hi > s[q].lo ? (s[q].hi - s[q].lo + 63) / 64 : 0;
      const u64 at = s[q].lo + (lane + 1) * step[q] - 1;
      v[q] = step[q] && at < s[q].hi ? s[q].a[at * s[q].stride] : ~0ull;
    }
#pragma unroll
    for (int q = 0; q < N; q++) {
      if (!step[q]) continue;
      const u64 at = s[q].lo + (lane + 1) * step[q] - 1;
      const u64 c = __popcll(__ballot(at < s[q].hi && v[q] < s[q].x));  // blocks wholly below x (a prefix)
      const u64 nlo = s[q].lo + c * step[q];
      s[q].lo = nlo;
      if (step[q] == 1) {
        s[q].hi = nlo;
      } else {
        // block c's last entry is >= x (or past hi): the bound is at or before it
        s[q].hi = nlo + step[q] - 1 < s[q].hi ? nlo + step[q] - 1 : s[q].hi;
        more = true;
      }
    }
    if (!more) return;
  }
}

// A short segment's lower bound + membership with the final window's loads
// issued up front (win_load) and consumed later (win_rank): an item issues
// the windows of all its lookups at once -- one round trip for the short
// segments of a small document -- instead of one search after another.
// Segments of W or more are first bisected down to W - 1 (dependent loads).
template <int W>
struct Win {
  u64 lo, hi;
  u64 v[W];
};
// The lower bound lies in [lo, hi] after bisecting, so the window spans
// [lo, lo + W) clipped to the segment's end (w.hi), which includes position
// hi itself: an equal dot found there is a member.
template <bool kRec, int W>
__device__ __forceinline__ void win_load(Win<W>& w, const void* src, u64 lo, u64 hi, u64 x) {
  const u64 end = hi;
  while (hi - lo >= W) {
    const u64 m = (lo + hi) >> 1;
    if (dot_at<kRec>(src, m) < x) lo = m + 1;
    else hi = m;
  }
  w.lo = lo;
  w.hi = end;
#pragma unroll
  for (int j = 0; j < W; j++) w.v[j] = lo + j < end ? dot_at<kRec>(src, lo + j) : ~0ull;
}
template <int W>
__device__ __forceinline__ u64 win_rank(const Win<W>& w, u64 x, bool& eq) {
  u32 c = 0;
  eq = false;
#pragma unroll
  for (int j = 0; j < W; j++) {
    c += w.v[j] < x;
    eq = eq || (w.v[j] == x && w.lo + j < w.hi);
  }
  return w.lo + c;
}

__device__ __forceinline__ URec load_rec(const URec* p) {
  const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(p));
  return URec{v.x, v.y};
}
__device__ __forceinline__ void store_rec(URec* p, u64 d, u64 e) {
  u64x2 v;
  v.x = d;
  v.y = e;
  __builtin_nontemporal_store(v, reinterpret_cast<u64x2*>(p));
}

struct UjArgs {
  // state
  UMeta* meta;
  const URec* rec;   // element pool
  const u64* cloud;  // cloud pool
  u64* vv;
  URec* epool_out;
  u64* cpool_out;
  u64* ctr;          // bump pointers (device)
  u64* pin;          // mapped pinned: bump pointers after this converge
  u64* pin_t;        // mapped pinned: this converge's touched state elements / cloud dots
  u64* pin_l;        // mapped pinned: the long pools' bump pointers and ids handed out
  u32 R;
  u32 epoch;
  u32 keep_all;      // context-only join: every state element stays (the write path's pending deltas)
  u64* dptr;         // [kcap] epoch << 32 | first delta doc of the slot
  u32* bad;          // [nd] == epoch: skipped
  unsigned long long* skipped;
  u32* tick;
  // delta batch
  u64 nd, nb, cb, nvv;
  const u32* slot;
  const u64* deoff;
  const u64* ddots;
  const u64* delems;
  const u64* dvoff;
  const u64* dvv;
  const u64* dcoff;
  const u64* dcloud;
  // per delta doc
  u64* abase;  // [nd] state element segment base
  u64* cbs;    // [nd] state cloud segment base
  u64* ao;     // [nd + 1] exclusive scan of the touched state element counts (ao[nd] = ta)
  u64* co;     // [nd + 1] ... of the touched state cloud counts (co[nd] = tc)
  u64* neo;    // [nd + 1] output offsets (elements)
  u64* nco;    // [nd + 1] output offsets (cloud)
  u64* base;   // [2] this converge's pool bases
  u64* vvd;    // [nd][R] the delta's vv, dense (zero between converges)
  u32* sidV;   // [nvv] the doc of every sparse delta vv entry (U1 -> U5)
  // scans: sc over [state elements | delta elements | delta cloud], ksc over
  // [state cloud | delta cloud]; tile-local exclusive prefixes (see ScanSp)
  u32* sc;
  u32* ksc;
  // cross ranks (U2 / U3 -> U5): each item's merge position on the other
  // side, relative to that side's segment start, so U5 needs no search
  u32* xr;  // over the sc space
  u32* kr;  // over the ksc space
  // look-back status words
  u64* st_ao;
  u64* st_co;
  // the doc of every item, per item space (written by U1's doc tiles):
  // state elements, delta elements, state cloud, delta cloud
  u32* sidA;
  u32* sidB;
  u32* sidC;
  u32* sidD;
  // ... except inside long segments: there a tile lying wholly in one doc
  // finds it in its space's tile map (epoch << 32 | doc)
  u64* tmA;
  u64* tmB;
  u64* tmC;
  u64* tmD;
  u64* stats;
  u64* tp;   // [tiles + 1] sc tile aggregates -> exclusive tile prefixes (U2 -> k_uj_tscan)
  u64* ktp;  // ... of ksc
  u64* st_ne;
  u64* st_nc;
  // in-place layout of long documents (jy_internal.hpp LCol); lcol ==
  // nullptr: the store has none and never promotes
  LCol* lcol;
  LPlan* lplan;
  URec* lpe;
  u64* lpc;
  u64 lpe_cap, lpc_cap, lcap;
  UJob* jobs;  // [2][jcap]
  u64 jcap;
  u32* fast;
  u32* nf;
  u32* plist;
  u32* flist;    // the delta docs converging in place (ctr[7] of them)
  u32 long_min;  // promotion threshold (0: none this converge)
};

__device__ __forceinline__ bool is_bad(const UjArgs& A, u64 k) { return A.bad[k] == A.epoch; }
// the delta doc converges in place (k_uj_docs judged it append-shaped)
__device__ __forceinline__ bool is_fast(const UjArgs& A, u64 k) { return A.lcol && A.fast[k] == A.epoch; }
__device__ __forceinline__ u64 tag(const UjArgs& A, u64 v) { return ((u64)A.epoch << 32) | (u32)v; }
__device__ __forceinline__ bool tagged(const UjArgs& A, u64 w) { return (u32)(w >> 32) == A.epoch; }
// the long id of delta doc k's document, or ~0u (a regular document or a hole)
__device__ __forceinline__ u32 long_id(const UjArgs& A, u64 k) {
  const u32 s = A.slot[k];
  if (s == JY_NO_SLOT) return ~0u;
  const UMeta m = A.meta[s];
  return m.ecap == kLongMark ? (u32)m.ebase : ~0u;
}
// capacity of a column run that must hold n: room for as many again
__device__ __forceinline__ u32 roomy(u64 n) { return (u32)(2 * n + 16); }
__device__ __forceinline__ void mark_bad(const UjArgs& A, u64 k) { A.bad[k] = A.epoch; }  // same value from every writer
__device__ __forceinline__ u64 doc_at(const UjArgs& A, const u64* tm, u64 tile, const u32* sid, u64 i) {
  const u64 v = tm[tile];
  return (u32)(v >> 32) == A.epoch ? (u32)v : sid[i];
}

// A scan space of up to three kinds laid back to back, each cut into kTile
// tiles from its own start.  U2 / U3 write each item's exclusive prefix
// WITHIN its tile (loc) and each tile's total (tp); k_uj_tscan turns tp into
// exclusive tile prefixes.  No tile waits for another (a decoupled look-back
// would make every tile wait for its slowest predecessor's searches).
__device__ __forceinline__ u64 cdiv(u64 a) { return (a + kTile - 1) / kTile; }
struct ScanSp {
  const u32* loc;
  const u64* tp;
  u64 b1, b2, n;   // kinds [0, b1) [b1, b2) [b2, n)
  u64 t1, t2, tn;  // their first tiles; tile count
  __device__ __forceinline__ u64 at(u64 j) const {  // global exclusive prefix at j (j <= n)
    if (j >= n) return tp[tn];
    const u64 t = j < b1 ? j / kTile : j < b2 ? t1 + (j - b1) / kTile : t2 + (j - b2) / kTile;
    return tp[t] + loc[j];
  }
};
__device__ __forceinline__ ScanSp sc_space(const UjArgs& A) {
  const u64 ta = A.ao[A.nd];
  const u64 t1 = cdiv(ta), t2 = t1 + cdiv(A.nb);
  return ScanSp{A.sc, A.tp, ta, ta + A.nb, ta + A.nb + A.cb, t1, t2, t2 + cdiv(A.cb)};
}
__device__ __forceinline__ ScanSp ksc_space(const UjArgs& A) {
  const u64 tc = A.co[A.nd];
  const u64 t1 = cdiv(tc), tn = t1 + cdiv(A.cb);
  return ScanSp{A.ksc, A.ktp, tc, tc + A.cb, tc + A.cb, t1, tn, tn};
}

// the state's vv entry of delta doc k: the state rows are read in place
// (only U5 writes them, after U3's folds raised them with atomics)
__device__ __forceinline__ u64 state_vv(const UjArgs& A, u64 k, u32 c) { return A.vv[(u64)A.slot[k] * A.R + c]; }
// the merged vv entry max(state, delta) of delta doc k for U3.  U3's folds
// raise the state rows in place while other items read them: any value read
// is the merged entry raised by a run of folded dots that starts at it, and
// "seq(x) == v + 1 + |union dots in (v, seq(x))|" decides the same for every
// such v (a value at or past seq(x) means x itself is folded: dropped)
__device__ __forceinline__ u64 merged_vv(const UjArgs& A, u64 k, u32 c) {
  const u64 s = state_vv(A, k, c), d = A.vvd[k * A.R + c];
  return s > d ? s : d;
}


// ---- tiles: the documents of an item range [i0, i1) of a CSR offs[0..nd],
// staged in LDS (first wave searches; everyone loads); doc_of() per item
struct TileDocs {
  u64 k0, cnt;  // docs k0 .. k0 + cnt - 1 cover the range
  bool lds;     // their offsets are staged in LDS
};
// waves 0 and 1 search the first and the last doc at once
template <u64 kCap>
__device__ __forceinline__ TileDocs tile_docs(const u64* offs, u64 nd, u64 i0, u64 i1, u64* lds, u64* sh) {
  if (threadIdx.x < 128) {
    const u64 k = jyscan::wave_last_le(offs, nd, threadIdx.x < 64 ? i0 : i1 - 1);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = k;
  }
  __syncthreads();
  TileDocs T{sh[0], sh[1] - sh[0] + 1, sh[1] - sh[0] + 1 <= kCap};
  if (T.lds)
    for (u64 j = threadIdx.x; j <= T.cnt; j += kThreads) lds[j] = offs[T.k0 + j];
  __syncthreads();
  return T;
}
__device__ __forceinline__ u64 doc_of(const TileDocs& T, const u64* offs, const u64* lds, u64 i) {
  if (T.lds) {
    u32 lo = 0, hi = (u32)T.cnt - 1;
    while (lo < hi) {
      const u32 m = (lo + hi + 1) >> 1;
      if (lds[m] <= i) lo = m;
      else hi = m - 1;
    }
    return T.k0 + lo;
  }
  u64 lo = T.k0, hi = T.k0 + T.cnt - 1;
  while (lo < hi) {
    const u64 m = (lo + hi + 1) >> 1;
    if (offs[m] <= i) lo = m;
    else hi = m - 1;
  }
  return lo;
}

struct Shared {
  u64 offs[kLdsDocs + 1];  // the CSR offsets of a tile's docs
  u64 rng[8];
  u64 sh[2];
  u64 red[kThreads / 64];
  u64 pre;
  u32 tk;
};


// ---- U1a classification of one delta item of a LONG document (lid):
// whether the delta is append-shaped in the item's column, and where the
// column's fresh run of delta dots starts and ends (single writers: the first
// fresh item, the column's last item).  Fresh = above everything the state's
// column holds (vv, element and cloud runs).  A dot that is not fresh must
// change nothing: a delta element already in the state's context (dropped, or
// the state's own copy kept); a delta cloud dot in the state's context that
// removes no live state element (none there, or the delta keeps it).  A vv
// entry must not raise the state's and must lie below the column's first
// element.  Anything else marks the doc: it is demoted (k_uj_docs).
__device__ void uj_item_long(const UjArgs& A, int kind, u64 k, u64 i, u32 lid, u64 x) {
  const u32 c = dcol(x);
  if (c >= A.R) return;  // malformed: U1a marks the doc bad
  const u32 s = A.slot[k];
  const u64 li = (u64)lid * A.R + c;
  const LCol L = A.lcol[li];
  const u64 vs = A.vv[(u64)s * A.R + c], q = dseq(x);
  if (kind == 2) {  // a vv entry of the delta: it must not raise the state's
    if (q > vs) {
      A.nf[k] = A.epoch;
      return;
    }
    // the elements it covers (the run's prefix of seq <= q) go unless the
    // delta holds them: a prefix within kTrimSpan is trimmed in place
    if (L.elen) {  // the run's first 8 elements at once (old elements sit there); a search past them
      u64 cut = 0;
#pragma unroll
      for (u32 j = 0; j < 8; j++) cut += j < L.elen && dseq(A.lpe[L.ebase + j].dot) <= q;
      if (cut == 8 && L.elen > 8) cut = lb_g<true>(A.lpe, L.ebase + 8, L.ebase + L.elen, mkdot(c, q + 1)) - L.ebase;
      if (cut > kTrimSpan) A.nf[k] = A.epoch;
      else if (cut) atomicMax((unsigned long long*)&A.lplan[li].treq, (unsigned long long)tag(A, cut));
    }
    return;
  }
  const u64 te = L.elen ? dseq(A.lpe[L.ebase + L.elen - 1].dot) : 0;
  const u64 tc = L.clen ? dseq(A.lpc[L.cbase + L.clen - 1]) : 0;
  const u64 F = vs > te ? (vs > tc ? vs : tc) : (te > tc ? te : tc);
  const u64* a = kind == 0 ? A.ddots : A.dcloud;
  const u64* offs = kind == 0 ? A.deoff : A.dcoff;
  const u64 lo = offs[k], hi = offs[k + 1];
  const u64 prev = i > lo ? a[i - 1] : 0, next = i + 1 < hi ? a[i + 1] : ~0ull;
  const bool fresh = q > F;
  LPlan& P = A.lplan[li];
  if (fresh && (i == lo || dcol(prev) != c || dseq(prev) <= F)) (kind == 0 ? P.efs : P.cfs) = tag(A, i);
  if (i + 1 == hi || dcol(next) != c) (kind == 0 ? P.ece : P.cce) = tag(A, i + 1);
  if (fresh) return;
  // the state's cloud run (seen?), and for a context dot the state's element
  // run (a live element?) and the delta's elements (kept?): the three
  // searches in lockstep, one dependent round per level
  const bool el = kind == 1;
  u64 clo = L.cbase, chi = q <= vs ? clo : L.cbase + L.clen;  // (covered by the vv: no cloud search)
  u64 elo = L.ebase, ehi = el ? L.ebase + L.elen : elo;
  u64 dlo = A.deoff[k], dhi = el ? A.deoff[k + 1] : dlo;
  while (clo < chi || elo < ehi || dlo < dhi) {
    const u64 cm = (clo + chi) >> 1, em = (elo + ehi) >> 1, dm = (dlo + dhi) >> 1;
    const u64 cv = clo < chi ? A.lpc[cm] : 0, ev = elo < ehi ? A.lpe[em].dot : 0, dv = dlo < dhi ? A.ddots[dm] : 0;
    if (clo < chi) (cv < x ? clo = cm + 1 : chi = cm);
    if (elo < ehi) (ev < x ? elo = em + 1 : ehi = em);
    if (dlo < dhi) (dv < x ? dlo = dm + 1 : dhi = dm);
  }
  const bool seen = q <= vs || (clo < L.cbase + L.clen && A.lpc[clo] == x);
  if (!seen) {
    A.nf[k] = A.epoch;
    return;
  }
  if (el && elo < L.ebase + L.elen && A.lpe[elo].dot == x && !(dlo < A.deoff[k + 1] && A.ddots[dlo] == x)) {
    // a context dot removes a live state element the delta does not hold
    if (elo - L.ebase >= kTrimSpan) A.nf[k] = A.epoch;  // too far in: the regular path
    else atomicMax((unsigned long long*)&P.treq, (unsigned long long)tag(A, elo - L.ebase + 1));
  }
}

// ---- U1b decision for a long document, one WAVE per document (lane c =
// column c): in place when the delta is append-shaped; a column run that
// overflows moves to a larger run of the long pool (a copy job, k_uj_jobs);
// when the long pool is short, or the delta is not append-shaped, the
// document is DEMOTED: a copy job lays its column runs out as one regular
// run at the pools' bump pointers and the regular merge path takes it.
// Returns (lane 0) the doc's touched state sizes for the scans (0 in place).
// the tile's copy jobs are gathered in LDS and reserved with one atomic per
// tile (a same-address atomic per document serialised ~1.5K of them)
struct JobBuf {
  static constexpr u32 kCap = 128;
  UJob j[kCap];
  u32 n;
  __device__ void push(const UjArgs& A, const UJob& x) {  // (one lane)
    const u32 q = atomicAdd(&n, 1u);
    if (q < kCap) j[q] = x;
    else A.jobs[atomicAdd((unsigned long long*)(A.ctr + 5), 1ull)] = x;  // overflow: directly
  }
};
__device__ void uj_docs_long(const UjArgs& A, u64 k, u32 lid, u32 melen, u32 mclen, u64& asz, u64& csz, JobBuf& jb,
                             bool& in_place) {
  const u32 lane = threadIdx.x & 63, R = A.R;
  const UMeta m{lid, melen, kLongMark, 0, mclen, kLongMark};
  const u64 b = (u64)lid * R;
  const bool act = lane < R;
  LCol L{};
  u64 efs = 0, ece = 0, cfs = 0, cce = 0, treq = 0;
  if (act) {
    L = A.lcol[b + lane];
    const LPlan& P = A.lplan[b + lane];
    efs = P.efs, ece = P.ece, cfs = P.cfs, cce = P.cce, treq = P.treq;
  }
  const bool tr = act && tagged(A, treq);
  const u64 ne = tagged(A, efs) ? (u32)ece - (u32)efs : 0, nc = tagged(A, cfs) ? (u32)cce - (u32)cfs : 0;
  const bool ge = act && L.elen + ne > L.ecap, gc = act && (L.clen ? L.clen + nc : nc) > L.ccap;
  const bool broken = act && ((tagged(A, efs) && !tagged(A, ece)) || (tagged(A, cfs) && !tagged(A, cce)));
  // (a run that moves is not trimmed in place as well)
  bool fast = A.nf[k] != A.epoch && !__ballot(broken || (ge && tr));
  const u64 ne_e = ge ? roomy(L.elen + ne) : 0, ne_c = gc ? roomy(L.clen + nc) : 0;
  const u64 oe = jyscan::wave_incl<u64>(ne_e) - ne_e, oc = jyscan::wave_incl<u64>(ne_c) - ne_c;
  const u64 NE = __shfl(oe + ne_e, 63), NC = __shfl(oc + ne_c, 63);
  const u64 moved = jyscan::wave_sum<u64>((ge ? L.elen : 0) + (gc ? L.clen : 0));
  u64 eb = 0, cb = 0, ok = fast;
  if (lane == 0 && fast) {
    // (a refused request wastes its reservation until the next compaction:
    // the host keeps the long pools at 4x the live entries)
    if (NE) eb = atomicAdd((unsigned long long*)(A.ctr + 2), (unsigned long long)NE), ok = eb + NE <= A.lpe_cap;
    if (ok && NC) cb = atomicAdd((unsigned long long*)(A.ctr + 3), (unsigned long long)NC), ok = cb + NC <= A.lpc_cap;
  }
  fast = __shfl(ok, 0);
  if (fast) {
    eb = __shfl(eb, 0);
    cb = __shfl(cb, 0);
    if (act && (ne || nc || tr)) {
      LPlan& P = A.lplan[b + lane];
      const u64 erun = ge ? eb + oe : L.ebase, crun = gc ? cb + oc : L.cbase;
      P.erun = erun;
      P.crun = crun;
      P.eapp = erun + L.elen;
      P.capp = crun + L.clen;
      P.ecap = ge ? (u32)ne_e : L.ecap;
      P.ccap = gc ? (u32)ne_c : L.ccap;
      P.cz = L.clen == 0;
    }
    const u64 trims = __popcll(__ballot(tr));
    if (lane == 0) {
      // the runs that grew are copied, the trims done, before any append
      // (k_uj_jobs, then U2); a repeated doc's jobs are skipped there
      if (moved) jb.push(A, UJob{k, 0, moved, UJ_REGROW, lid});
      if (trims) jb.push(A, UJob{k, 0, R, UJ_TRIM, lid});
      A.fast[k] = A.epoch;
      A.abase[k] = lid;
      asz = csz = 0;
      in_place = true;
    }
    return;
  }
  // demote: one regular run (the host's pool plan budgets it); U5 writes the
  // merged document as usual, the long runs are left behind
  if (lane == 0) {
    eb = m.elen ? atomicAdd((unsigned long long*)A.ctr, (unsigned long long)m.elen) : 0;
    cb = m.clen ? atomicAdd((unsigned long long*)(A.ctr + 1), (unsigned long long)m.clen) : 0;
    if (m.elen + m.clen) jb.push(A, UJob{eb, cb, (u64)m.elen + m.clen, UJ_DEMOTE, lid});
    A.abase[k] = eb;
    A.cbs[k] = cb;
    asz = m.elen;
    csz = m.clen;
    atomicAdd((unsigned long long*)(A.stats + 15), 1ull);
  }
}

// ---- copy jobs of the in-place layout (demotions, regrowths, promotions),
// one per document: its up to 2R column segments (elements, then cloud dots)
// are laid out in LDS and copied in kJobChunk-item chunks dealt round-robin
// over a persistent grid.  An empty list costs one load.
constexpr u64 kJobChunk = 2048;
constexpr int kMaxR = 64;  // the in-place layout needs R <= 64 (a lane per column)

// the trim of column c of delta doc k (one workgroup): the run's first
// min(elen, kTrimSpan) elements are staged in LDS, each keeps unless the
// delta's context covers it (vv entry, cloud dot) and its map lacks it, and
// the kept ones are written back right-aligned -- the run now starts
// `removed` further up and ends where it did (appends are unaffected)
__device__ void uj_trim_column(const UjArgs& A, u64 k, u32 lid, u32 c) {
  __shared__ URec l_rec[kTrimSpan];
  __shared__ u64 l_red[kThreads / 64];
  __syncthreads();  // (the workgroup's previous trim is done with l_rec)
  LPlan& P = A.lplan[(u64)lid * A.R + c];
  if (!tagged(A, P.treq)) return;  // (uniform: every thread reads the same word)
  const LCol L = A.lcol[(u64)lid * A.R + c];
  const u32 span = (u32)P.treq;  // (the furthest element a removal can reach, +1)
  const u32 nb = L.elen < span ? L.elen : span;
  const u64 vd = A.vvd[k * A.R + c];
  const u32 t = threadIdx.x;
  u64 keep = 0;
  if (t < nb) {
    const URec r = A.lpe[L.ebase + t];
    l_rec[t] = r;
    const u64 x = r.dot;
    // the delta's cloud (covered?) and elements (kept?), searched in lockstep
    u64 clo = A.dcoff[k], chi = dseq(x) <= vd ? clo : A.dcoff[k + 1], dlo = A.deoff[k], dhi = A.deoff[k + 1];
    while (clo < chi || dlo < dhi) {
      const u64 cm = (clo + chi) >> 1, dm = (dlo + dhi) >> 1;
      const u64 cv = clo < chi ? A.dcloud[cm] : 0, dv = dlo < dhi ? A.ddots[dm] : 0;
      if (clo < chi) (cv < x ? clo = cm + 1 : chi = cm);
      if (dlo < dhi) (dv < x ? dlo = dm + 1 : dhi = dm);
    }
    const bool covered = dseq(x) <= vd || (clo < A.dcoff[k + 1] && A.dcloud[clo] == x);
    keep = !covered || (dlo < A.deoff[k + 1] && A.ddots[dlo] == x);
  }
  u64 kept;
  const u64 rank = jyscan::block_excl<kThreads, u64>(keep, l_red, kept);  // (syncs: l_rec is complete)
  const u64 cut = nb - kept;
  if (keep) A.lpe[L.ebase + cut + rank] = l_rec[t];
  if (t == 0) P.tcut = tag(A, cut);
}
// one chunk of a copy job: its up to 2R column segments (elements, then
// cloud dots) laid out in LDS, then the chunk's items copied
__device__ void uj_job_chunk(const UjArgs& A, const UJob& J, u64 q) {
  __shared__ u64 l_src[2 * kMaxR], l_dst[2 * kMaxR], l_pre[2 * kMaxR + 1];
  const u32 R = A.R;
  __syncthreads();  // (the workgroup's previous chunk is done with the table)
  if (threadIdx.x < R) {  // lane c: column c's element and cloud segment
    const u32 c = threadIdx.x;
    const LCol L = A.lcol[(u64)J.lid * R + c];
    u64 se = 0, de = 0, ne = 0, sc = 0, dc = 0, nc = 0;
    if (J.what == UJ_REGROW) {
      const LPlan& P = A.lplan[(u64)J.lid * R + c];
      if (tagged(A, P.efs) || tagged(A, P.cfs)) {
        if (P.erun != L.ebase) se = L.ebase, de = P.erun, ne = L.elen;
        if (P.crun != L.cbase) sc = L.cbase, dc = P.crun, nc = L.clen;
      }
    } else {
      ne = L.elen;
      nc = L.clen;
      se = de = L.ebase;  // the regular side is filled in below
      sc = dc = L.cbase;
    }
    l_src[c] = se, l_dst[c] = de, l_pre[c] = ne;
    l_src[R + c] = sc, l_dst[R + c] = dc, l_pre[R + c] = nc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // exclusive prefix over the 2R segments; the regular run's places
    u64 acc = 0, oe = 0, oc = 0;
    for (u32 g = 0; g < 2 * R; g++) {
      const u64 len = l_pre[g];
      if (J.what == UJ_DEMOTE) l_dst[g] = g < R ? J.e + oe : J.c + oc;
      if (J.what == UJ_PROMOTE) l_src[g] = g < R ? J.e + oe : J.c + oc;
      (g < R ? oe : oc) += len;
      l_pre[g] = acc;
      acc += len;
    }
    l_pre[2 * R] = acc;
  }
  __syncthreads();
  // every item's load first, then the stores: a copy's source and destination
  // never overlap (regrowth moves into fresh room), and with one load-store
  // pair per iteration each of the kPerT rounds waited a whole memory round
  // trip (the loop could not move a load above the previous store)
  static_assert(kJobChunk % kThreads == 0, "a chunk is whole rounds of the workgroup");
  constexpr u32 kPerT = (u32)(kJobChunk / kThreads);
  const u64 i0 = q * kJobChunk, i1 = i0 + kJobChunk < J.n ? i0 + kJobChunk : J.n;
  const URec* es = J.what == UJ_PROMOTE ? A.epool_out : A.lpe;
  const u64* cs = J.what == UJ_PROMOTE ? A.cpool_out : A.lpc;
  URec* ed = J.what == UJ_DEMOTE ? A.epool_out : A.lpe;
  u64* cd = J.what == UJ_DEMOTE ? A.cpool_out : A.lpc;
  URec v[kPerT];
  u64 di[kPerT];
  u32 sg[kPerT];
#pragma unroll
  for (u32 u = 0; u < kPerT; u++) {
    const u64 t = i0 + (u64)u * kThreads + threadIdx.x;
    sg[u] = ~0u;
    if (t >= i1) continue;
    u32 lo = 0, hi = 2 * R - 1;  // the last segment g with l_pre[g] <= t
    while (lo < hi) {
      const u32 mid = (lo + hi + 1) >> 1;
      if (l_pre[mid] <= t) lo = mid;
      else hi = mid - 1;
    }
    const u64 o = t - l_pre[lo];
    const u64 si = l_src[lo] + o;
    di[u] = l_dst[lo] + o;
    sg[u] = lo;
    if (lo < R) v[u] = es[si];
    else v[u].dot = cs[si];
  }
#pragma unroll
  for (u32 u = 0; u < kPerT; u++) {
    if (sg[u] == ~0u) continue;
    if (sg[u] < R) ed[di[u]] = v[u];
    else cd[di[u]] = v[u].dot;
  }
}

// The job list's chunks (kJobChunk items of a copy job; one column of a
// trim) dealt round-robin over a persistent grid: the workgroups read a
// block of job headers together, scan their chunk counts in LDS and find a
// chunk's job by a search there (no walk over the list).  An empty list
// costs one load.
constexpr u32 kJobBlock = 2048;
__global__ __launch_bounds__(kThreads) void k_uj_jobs(UjArgs A, const UJob* __restrict__ jobs,
                                                     const u64* __restrict__ cnt, u64 cap) {
  __shared__ u32 l_pre[kJobBlock + 1];
  __shared__ u64 l_red[kThreads / 64];
  const u64 n = *cnt < cap ? *cnt : cap;
  const u64 G = gridDim.x;
  constexpr u32 kPerT = kJobBlock / kThreads;
  u64 base = 0;  // chunks of the blocks before
  for (u64 j0 = 0; j0 < n; j0 += kJobBlock) {
    const u32 m = (u32)(n - j0 < kJobBlock ? n - j0 : kJobBlock);
    u32 v[kPerT];
    u64 sum = 0;
#pragma unroll
    for (u32 u = 0; u < kPerT; u++) {  // thread t: jobs t * kPerT .. (contiguous)
      const u32 i = threadIdx.x * kPerT + u;
      u32 c = 0;
      if (i < m) {
        const UJob J = jobs[j0 + i];
        // (a repeated doc's regrowth / trim: its runs stay; k_uj_docs' claims are final)
        const bool skip = (J.what == UJ_REGROW || J.what == UJ_TRIM) && is_bad(A, J.e);
        c = skip ? 0 : J.what == UJ_TRIM ? (u32)J.n : (u32)((J.n + kJobChunk - 1) / kJobChunk);
      }
      v[u] = c;
      sum += c;
    }
    u64 tot;
    u64 off = jyscan::block_excl<kThreads, u64>(sum, l_red, tot);
#pragma unroll
    for (u32 u = 0; u < kPerT; u++) {
      const u32 i = threadIdx.x * kPerT + u;
      if (i < m) l_pre[i] = (u32)off;
      off += v[u];
    }
    if (threadIdx.x == 0) l_pre[m] = (u32)tot;
    __syncthreads();
    for (u64 g = (blockIdx.x + G - base % G) % G; g < tot; g += G) {  // (uniform over the workgroup)
      u32 lo = 0, hi = m - 1;  // the last job i with l_pre[i] <= g
      while (lo < hi) {
        const u32 mid = (lo + hi + 1) >> 1;
        if (l_pre[mid] <= g) lo = mid;
        else hi = mid - 1;
      }
      const UJob J = jobs[j0 + lo];
      const u64 q = g - l_pre[lo];
      if (J.what == UJ_TRIM) uj_trim_column(A, J.e, J.lid, (u32)q);
      else uj_job_chunk(A, J, q);
    }
    base += tot;
    __syncthreads();  // (l_pre is rewritten by the next block)
  }
}

// item kernels U2 / U3 / U5: one item per thread, a tile of kTile items per
// workgroup, nothing staged -- full occupancy hides the searches' latency
constexpr int kItemThreads = (int)kTile;

// tile-local exclusive scan of one flag per thread; returns the tile total
__device__ __forceinline__ u64 item_scan(u64 f, u64* red, u64& tot) {
  return jyscan::block_excl<kItemThreads, u64>(f, red, tot);
}

// exclusive scan of the tile totals of U2 (`which` 0) or U3 (1), in place,
// total appended; one workgroup of 1024
__global__ __launch_bounds__(1024) void k_uj_tscan(UjArgs A, int which) {
  __shared__ u64 red[16];
  const ScanSp sp = which == 0 ? sc_space(A) : ksc_space(A);
  u64* tp = which == 0 ? A.tp : A.ktp;
  const u64 n = sp.tn;
  u64 carry = 0;
  for (u64 c0 = 0; c0 < n; c0 += 1024 * 4) {
    u64 v[4], sum = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const u64 j = c0 + threadIdx.x * 4 + u;
      v[u] = j < n ? tp[j] : 0;
      sum += v[u];
    }
    u64 tot;
    u64 off = jyscan::block_excl<1024, u64>(sum, red, tot) + carry;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const u64 j = c0 + threadIdx.x * 4 + u;
      if (j < n) tp[j] = off;
      off += v[u];
    }
    carry += tot;
  }
  if (threadIdx.x == 0) tp[n] = carry;
}

#ifdef JY_UJ_PROBE  // A/B only: per-tile clocks of U2..U4 (wall clock, 100 MHz)
constexpr u32 kProbe = 65536;
__device__ u64 g_probe[kProbe][6];
__device__ u32 g_probe_n;
__device__ __forceinline__ void probe(u32 kern, u32 kind, u32 t, u64 c0, u64 c1, u64 c2, u64 ca = 0, u64 cb = 0) {
  if (threadIdx.x != 0) return;
  const u32 j = atomicAdd(&g_probe_n, 1u);
  if (j < kProbe) {
    g_probe[j][0] = ((u64)kern << 56) | ((u64)kind << 48) | t;
    g_probe[j][1] = c0;
    g_probe[j][2] = c1;
    g_probe[j][3] = c2;
    g_probe[j][4] = ca;
    g_probe[j][5] = cb;
  }
}
#define JY_CLK(v) const u64 v = wall_clock64()
#define JY_PROBE(...) probe(__VA_ARGS__)
#else
#define JY_CLK(v)
#define JY_PROBE(...)
#endif

constexpr u64 kLongSeg = 2 * kTile;  // longer segments use the tile maps
struct LongRun {
  u32 f0, f1, k, sp;  // whole tiles [f0, f1) of space sp lie in doc k
};

// ---- U1a: per delta item: validation (strictly ascending dots per doc, col
// < R, seq >= 1; vv entries ascending by column), the dense delta vv, and
// the classification of the items of long documents (uj_item_long) --------
__global__ __launch_bounds__(kThreads) void k_uj_items(UjArgs A, u64 t_el, u64 t_cl, u64 t_vv) {
  __shared__ Shared S;
  __shared__ u32 l_lid[kLdsDocs + 1];  // the tile's docs' long ids (~0u: regular)
  if (A.lcol && blockIdx.x == 0 && threadIdx.x == 0) {
    A.ctr[6] = 0;  // the previous converge's promotions and commits are done (stream order)
    A.ctr[7] = 0;
  }
  u64 tt = blockIdx.x;
  const u64* offs;
  u64 n;
  int kind;
  if (tt < t_el) {
    kind = 0;
    offs = A.deoff;
    n = A.nb;
  } else if ((tt -= t_el) < t_cl) {
    kind = 1;
    offs = A.dcoff;
    n = A.cb;
  } else if ((tt -= t_cl) < t_vv) {
    kind = 2;
    offs = A.dvoff;
    n = A.nvv;
  } else {
    return;
  }
  JY_CLK(c0);
  const u64 i0 = tt * kTile1, i1 = i0 + kTile1 < n ? i0 + kTile1 : n;
  const TileDocs T = tile_docs<kLdsDocs>(offs, A.nd, i0, i1, S.offs, S.sh);
  if (A.lcol) {
    if (T.lds)
      for (u64 j = threadIdx.x; j < T.cnt; j += kThreads) l_lid[j] = long_id(A, T.k0 + j);
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const u64 i = i0 + (u64)u * kThreads + threadIdx.x;
    if (i >= i1) continue;
    const u64 k = doc_of(T, offs, S.offs, i);
    u64 x;
    if (kind == 2) {
      x = A.dvv[i];
      const u32 c = dcol(x);
      A.sidV[i] = (u32)k;
      if (c >= A.R || (i > A.dvoff[k] && dcol(A.dvv[i - 1]) >= c)) {
        mark_bad(A, k);
        continue;
      }
      A.vvd[k * A.R + c] = dseq(x);
    } else {
      const u64* a = kind == 0 ? A.ddots : A.dcloud;
      x = a[i];
      if (dcol(x) >= A.R || dseq(x) < 1 || (i > offs[k] && a[i - 1] >= x)) {
        mark_bad(A, k);
        continue;
      }
    }
    if (A.lcol) {
      const u32 lid = T.lds ? l_lid[k - T.k0] : long_id(A, k);
      if (lid != ~0u) uj_item_long(A, kind, k, i, lid, x);
    }
  }
  JY_CLK(c2);
  JY_PROBE(1, 1 + kind, (u32)tt, c0, c2, c2);
}

// ---- U1b: per delta doc (ticketed doc tiles, for the look-back): slot
// claim, meta, the long documents' in-place / demote decision, scans of the
// touched state sizes, the doc of every item (ids, or a tile map inside long
// segments) -----------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_uj_docs(UjArgs A, u64 ndt) {
  __shared__ Shared S;
  // Every long run of the tile staged (16 KB).  (Round 3 tried 64 staged
  // runs, 1 KB, owners filling the rest themselves: no speed-up.)
#ifndef JY_UJ_LONG_CAP
#define JY_UJ_LONG_CAP (4 * kDocTile)
#endif
  constexpr u32 kLongCap = JY_UJ_LONG_CAP;
  __shared__ LongRun l_long[kLongCap];
  __shared__ u32 l_nlong;
  __shared__ u32 l_lq[kThreads], l_nlq;  // the tile's long documents (thread indices)
  __shared__ u64 l_sz[kThreads][2];
  __shared__ JobBuf l_jb;
  __shared__ u64 l_jbase, l_fbase;
  __shared__ u32 l_lw[kThreads][3];  // a long document's id and totals, for its wave
  __shared__ u32 l_fq[kThreads], l_nfq;  // the tile's documents in place
  if (threadIdx.x == 0) l_nlong = l_nlq = l_jb.n = l_nfq = 0;
  const u32 t = jyscan::ticket(A.tick + T_U1, &S.tk);
  if (t >= ndt) return;
  JY_CLK(c0);
  const u64 k = (u64)t * kDocTile + threadIdx.x;
  u64 asz = 0, csz = 0;
  bool lg = false;  // a long document (decided by a wave below)
  if (k < A.nd) {
    const u32 s = A.slot[k];
    const bool hole = s == JY_NO_SLOT;  // a routed run's unused record (k_route_csr.hip)
    const UMeta m = hole ? UMeta{} : A.meta[s];
    A.abase[k] = m.ebase;
    A.cbs[k] = m.cbase;
    asz = m.elen;
    csz = m.clen;
    // claim the slot for this converge (one delta per doc per call): a
    // later copy marks both bad and does not count its size
    const u64 mine = ((u64)A.epoch << 32) | (u32)k;
    u64 old = hole ? 0 : A.dptr[s];
    if (hole) mark_bad(A, k);
    for (; !hole;) {
      if ((u32)(old >> 32) == A.epoch) {
        mark_bad(A, k);
        mark_bad(A, (u32)old);
        break;
      }
      const u64 seen = atomicCAS((unsigned long long*)(A.dptr + s), (unsigned long long)old,
                                 (unsigned long long)mine);
      if (seen == old) break;
      old = seen;
    }
    // a bad doc (malformed: U1a; repeated) is skipped: nothing of it is touched
    if (is_bad(A, k)) asz = csz = 0;
    else if (m.ecap == kLongMark && A.lcol) {
      l_lq[atomicAdd(&l_nlq, 1u)] = threadIdx.x, lg = true;
      l_lw[threadIdx.x][0] = (u32)m.ebase, l_lw[threadIdx.x][1] = m.elen, l_lw[threadIdx.x][2] = m.clen;
    }
  }
  if (A.lcol) {  // the long documents, a wave each
    __syncthreads();
    for (u32 q = threadIdx.x >> 6; q < l_nlq; q += kThreads / 64) {
      const u32 i = l_lq[q];
      u64 a = 0, c = 0;
      bool ip = false;
      uj_docs_long(A, (u64)t * kDocTile + i, l_lw[i][0], l_lw[i][1], l_lw[i][2], a, c, l_jb, ip);
      if ((threadIdx.x & 63) == 0) {
        l_sz[i][0] = a, l_sz[i][1] = c;
        if (ip) l_fq[atomicAdd(&l_nfq, 1u)] = (u32)((u64)t * kDocTile + i);
      }
    }
    __syncthreads();
    const u32 nj = min(l_jb.n, JobBuf::kCap), nfq = l_nfq;
    if (nj || nfq) {  // one reservation per tile: the copy jobs, the documents in place
      if (threadIdx.x == 0 && nj) l_jbase = atomicAdd((unsigned long long*)(A.ctr + 5), (unsigned long long)nj);
      if (threadIdx.x == 64 && nfq) l_fbase = atomicAdd((unsigned long long*)(A.ctr + 7), (unsigned long long)nfq);
      __syncthreads();
      for (u32 q = threadIdx.x; q < nj; q += kThreads) A.jobs[l_jbase + q] = l_jb.j[q];
      for (u32 q = threadIdx.x; q < nfq; q += kThreads) A.flist[l_fbase + q] = l_fq[q];
    }
    if (lg) {
      asz = l_sz[threadIdx.x][0];
      csz = l_sz[threadIdx.x][1];
    }
  }
  u64 tot;
  const u64 xa = jyscan::block_excl<kThreads, u64>(asz, S.red, tot);
  const u64 pa = jyscan::lookback(A.st_ao, t, A.epoch, tot, &S.pre);
  if (k < A.nd) A.ao[k] = pa + xa;
  if (t == ndt - 1 && threadIdx.x == 0) {
    A.ao[A.nd] = pa + tot;
  }
  const u64 xc = jyscan::block_excl<kThreads, u64>(csz, S.red, tot);
  const u64 pc = jyscan::lookback(A.st_co, t, A.epoch, tot, &S.pre);
  JY_CLK(c1);
  if (k < A.nd) A.co[k] = pc + xc;
  {
    // per-item doc ids.  A short segment's ids are written by its wave
    // together: pass p of the wave covers items [64p, 64p + 64) of the wave's
    // short segments laid end to end, each lane finding its segment by a
    // search over the lanes' run offsets (round 6: one lane per document
    // looping over its items waited for the wave's longest segment, ~13 us
    // of the tile).  A long segment names its doc once per whole tile in the
    // tile map, and its lane writes ids only in its partial end tiles.
    const bool live = k < A.nd;
    const u32 lane = threadIdx.x & 63;
    const u64 kw = (u64)t * kDocTile + (threadIdx.x & ~63u);  // the wave's first doc
    auto ids = [&](u32* sid, u64* tm, u64 off, u64 sz) {
      const u64 f0 = (off + kTile - 1) / kTile, f1 = (off + sz) / kTile;  // whole tiles [f0, f1)
      const bool shrt = sz <= kLongSeg || f0 >= f1;
      const u32 cs = live && shrt ? (u32)sz : 0u;
      u32 inc = cs;
      for (u32 d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(inc, d);
        if (lane >= d) inc += y;
      }
      const u32 lo = inc - cs, W = __shfl(inc, 63);
      for (u32 j0 = 0; j0 < W; j0 += 64) {  // wave-uniform
        const u32 j = j0 + lane;
        u32 r = 0;  // the last lane whose run starts at or before j (its run holds j)
        for (u32 s = 32; s; s >>= 1)
          if (__shfl(lo, (int)(r + s)) <= j) r += s;
        const u32 ro = __shfl(lo, (int)r);
        const u64 roff = __shfl(off, (int)r);
        if (j < W) sid[roff + (j - ro)] = (u32)(kw + r);
      }
      if (!live || shrt) return;
      for (u64 j = off; j < f0 * kTile; j++) sid[j] = (u32)k;
      for (u64 j = f1 * kTile; j < off + sz; j++) sid[j] = (u32)k;
      const u32 q = atomicAdd(&l_nlong, 1u);  // the workgroup fills its tile-map run
      if (q < kLongCap) {
        l_long[q] = LongRun{(u32)f0, (u32)f1, (u32)k, (u32)(tm == A.tmA ? 0 : tm == A.tmB ? 1 : tm == A.tmC ? 2 : 3)};
      } else {
        for (u64 m = f0; m < f1; m++) tm[m] = ((u64)A.epoch << 32) | k;
      }
    };
    ids(A.sidA, A.tmA, pa + xa, asz);
    ids(A.sidC, A.tmC, pc + xc, csz);
    const u64 b0 = live ? A.deoff[k] : 0, d0 = live ? A.dcoff[k] : 0;
    ids(A.sidB, A.tmB, b0, live ? A.deoff[k + 1] - b0 : 0);
    ids(A.sidD, A.tmD, d0, live ? A.dcoff[k + 1] - d0 : 0);
  }
  if (t == ndt - 1 && threadIdx.x == 0) {
    A.co[A.nd] = pc + tot;
  }
  __syncthreads();
  for (u32 q = 0; q < min(l_nlong, kLongCap); q++) {
    const LongRun g = l_long[q];
    u64* tm = g.sp == 0 ? A.tmA : g.sp == 1 ? A.tmB : g.sp == 2 ? A.tmC : A.tmD;
    for (u64 m = g.f0 + threadIdx.x; m < g.f1; m += kThreads) tm[m] = ((u64)A.epoch << 32) | g.k;
  }
  JY_CLK(c2);
  JY_PROBE(1, 0, t, c0, c1, c2);
}

// ---- U2: keep flags + cross ranks ----------------------------------------------
// kind 0: state elements (kept unless the delta saw them and lacks them);
// kind 1: delta elements (added unless the state holds or saw them); kind 2:
// delta cloud dots (dropped when the state cloud holds them).  The cross
// rank of an item is its merge position on the other side (relative to that
// side's segment of the doc); bit 31 of a state element's rank: U5 takes the
// delta's element for it.
// U2 for a wave of items inside long document k (wave-uniform): the keep
// flag and cross rank of item i (as uj_flags_tile), every search bounded by
// the wave's cooperative searches of the other side(s)
__device__ __forceinline__ void uj_flags_long(const UjArgs& A, int kind, u64 k, u64 i, u64 n, u64 gbase, u64& f) {
  const bool live = i < n;
  const u64 lm = __ballot(live);
  if (lm == 0) return;  // a wave past the space's end
  const u64 lastl = (u64)__popcll(lm) - 1;  // the wave's items are a prefix of its lanes
  const u64 clo = A.cbs[k], chi = clo + (A.co[k + 1] - A.co[k]);
  u64 d = 0;
  if (kind == 0) {
    if (live) d = A.rec[A.abase[k] + (i - A.ao[k])].dot;
  } else if (kind == 1) {
    if (live) d = A.ddots[i];
  } else {
    if (live) d = A.dcloud[i];
  }
  const u64 d0 = __shfl(d, 0), d1 = __shfl(d, (int)lastl) + 1;  // the wave's dots lie in [d0, d1)
  if (kind == 0) {
    // the delta's elements and the delta's cloud over [d0, d1)
    const u64 lo = A.deoff[k], hi = A.deoff[k + 1], blo = A.dcoff[k], bhi = A.dcoff[k + 1];
    WSearch s[4] = {{A.ddots, 1, lo, hi, d0}, {A.ddots, 1, lo, hi, d1}, {A.dcloud, 1, blo, bhi, d0},
                    {A.dcloud, 1, blo, bhi, d1}};
    wave_lbs<4>(s);
    if (s[0].lo == s[1].lo && s[2].lo == s[3].lo) {
      // (round 5) no delta element and no delta cloud dot falls in the
      // wave's range -- the usual wave of a long document, far from the
      // delta's few insertion points: no item has its dot in the delta's map
      // or cloud, so only the delta vv can drop it, its merge position on the
      // delta side is the range's, and the state cloud is never searched
      // (~4 dependent 64-ary rounds over a hot document's cloud)
      if (!live) return;
      f = A.keep_all || !(dseq(d) <= A.vvd[k * A.R + dcol(d)]);
      A.xr[gbase + i] = (u32)(s[0].lo - lo);
      return;
    }
    // the item's delta lookups inside the wave's bounds, issued together
    // with its vv entries (the bounds hold every dot of [d0, d1), so a dot
    // equal to d lies inside them)
    Win<8> wb;
    Win<4> wdc;
    u64 vd = 0, vs = 0, p = 0;
    bool eqb = false, indc = false, insc = false;
    if (live) {
      win_load<false>(wb, A.ddots, s[0].lo, s[1].lo, d);
      win_load<false>(wdc, A.dcloud, s[2].lo, s[3].lo, d);
      vd = A.vvd[k * A.R + dcol(d)];
      vs = state_vv(A, k, dcol(d));
      p = win_rank(wb, d, eqb);
      win_rank(wdc, d, indc);
    }
    // the state cloud decides only for a dot the delta also holds, above the
    // state vv: searched by the waves that have one
    const bool need = live && eqb && !(dseq(d) <= vs);
    if (__ballot(need)) {
      WSearch sc[2] = {{A.cloud, 1, clo, chi, d0}, {A.cloud, 1, clo, chi, d1}};
      wave_lbs<2>(sc);
      if (need) {
        Win<4> wsc;
        win_load<false>(wsc, A.cloud, sc[0].lo, sc[1].lo, d);
        win_rank(wsc, d, insc);
      }
    }
    if (!live) return;
    u32 xr = (u32)(p - lo);
    if (eqb) {
      f = 1;
      if (!(dseq(d) <= vs || insc)) xr |= 1u << 31;
    } else {
      f = A.keep_all || !(dseq(d) <= vd || indc);
    }
    A.xr[gbase + i] = xr;
  } else if (kind == 1) {
    // the state's elements and cloud over [d0, d1)
    const u64 lo = A.abase[k], hi = lo + (A.ao[k + 1] - A.ao[k]);
    WSearch s[4] = {{&A.rec[0].dot, 2, lo, hi, d0}, {&A.rec[0].dot, 2, lo, hi, d1}, {A.cloud, 1, clo, chi, d0},
                    {A.cloud, 1, clo, chi, d1}};
    wave_lbs<4>(s);
    if (!live) return;
    Win<8> wa;
    Win<4> wsc;
    win_load<true>(wa, A.rec, s[0].lo, s[1].lo, d);
    win_load<false>(wsc, A.cloud, s[2].lo, s[3].lo, d);
    const u64 vs = state_vv(A, k, dcol(d));
    bool eqa, insc;
    const u64 p = win_rank(wa, d, eqa);
    win_rank(wsc, d, insc);
    f = !eqa && !(dseq(d) <= vs || insc);
    A.xr[gbase + i] = (u32)(p - lo);
  } else {
    WSearch s[2] = {{A.cloud, 1, clo, chi, d0}, {A.cloud, 1, clo, chi, d1}};
    wave_lbs<2>(s);
    if (!live) return;
    Win<8> wsc;
    win_load<false>(wsc, A.cloud, s[0].lo, s[1].lo, d);
    bool insc;
    const u64 p = win_rank(wsc, d, insc);
    f = !insc;
    A.xr[gbase + i] = (u32)(p - clo);
  }
}

// U2 for an item of a delta doc converging IN PLACE (kind 1: a delta
// element, 2: a delta cloud dot; k_uj_docs planned the doc's columns): a
// fresh element goes to its column run's tail; a fresh cloud dot too, unless
// the column's cloud was empty and the dot extends the vv's run (folded: the
// run's last dot tells U5 how many folded -- the ones that do not fold were
// written at crun + rank, so U5 moves the run's start past the folded
// prefix).  Dots that are not fresh change nothing (k_uj_items checked).
__device__ __forceinline__ void uj_fast_item(const UjArgs& A, int kind, u64 k, u64 i) {
  const u32 lid = (u32)A.abase[k];
  if (kind == 1) {
    const u64 x = A.ddots[i];
    LPlan& P = A.lplan[(u64)lid * A.R + dcol(x)];
    const u64 fs = P.efs;
    if (!tagged(A, fs) || i < (u32)fs) return;
    store_rec(A.lpe + P.eapp + (i - (u32)fs), x, A.delems[i]);
    return;
  }
  const u64 x = A.dcloud[i];
  const u32 c = dcol(x);
  LPlan& P = A.lplan[(u64)lid * A.R + c];
  const u64 fs = P.cfs;
  if (!tagged(A, fs) || i < (u32)fs) return;
  const u64 r = i - (u32)fs;
  if (P.cz) {
    const u64 v = A.vv[(u64)A.slot[k] * A.R + c];
    if (dseq(x) == v + 1 + r) {
      if (i + 1 == (u32)P.cce || dseq(A.dcloud[i + 1]) != v + 2 + r) P.nfold = tag(A, r + 1);
      return;
    }
  }
  A.lpc[P.capp + r] = x;
}

__device__ __forceinline__ void uj_flags_tile(const UjArgs& A, const u64 t, u64* red) {
  const u64 ta = A.ao[A.nd];
  const u64 tA = cdiv(ta), tB = cdiv(A.nb);
  JY_CLK(c0);
  int kind;
  u64 lt, n, gbase;
  const u32* sid;
  const u64* tm;
  if (t < tA) {
    kind = 0, lt = t, n = ta, gbase = 0, sid = A.sidA, tm = A.tmA;
  } else if (t < tA + tB) {
    kind = 1, lt = t - tA, n = A.nb, gbase = ta, sid = A.sidB, tm = A.tmB;
  } else {
    kind = 2, lt = t - tA - tB, n = A.cb, gbase = ta + A.nb, sid = A.sidD, tm = A.tmD;
  }
  const u64 i = lt * kTile + threadIdx.x;
  u64 f = 0;
  // a tile wholly inside one long document: its waves bound every item's
  // search with wave-cooperative searches between their first and last dot
  const u64 tmv = tm[lt];
  if ((u32)(tmv >> 32) == A.epoch) {
    const u64 k = (u32)tmv;
    if (is_bad(A, k)) {
    } else if (is_fast(A, k)) {
      if (kind && i < n) uj_fast_item(A, kind, k, i);
    } else {
      uj_flags_long(A, kind, k, i, n, gbase, f);
    }
  } else if (i < n) {
    // small documents: every lookup of the item issued at once (the doc's
    // words, then the item's dot, then all its windows): ~4 round trips
    const u64 k = (u32)(tmv >> 32) == A.epoch ? (u32)tmv : sid[i];
    const bool bad = is_bad(A, k);
    const u64 clo = A.cbs[k], chi = clo + (A.co[k + 1] - A.co[k]);
    const u32 sl = A.slot[k];
    if (!bad && is_fast(A, k)) {
      if (kind) uj_fast_item(A, kind, k, i);  // (a doc in place has no state items here)
    } else if (!bad) {
      u32 xr;
      if (kind == 0) {
        const u64 lo = A.deoff[k], hi = A.deoff[k + 1], blo = A.dcoff[k], bhi = A.dcoff[k + 1];
        const u64 d = A.rec[A.abase[k] + (i - A.ao[k])].dot;
        Win<8> wb;
        Win<4> wdc, wsc;
        win_load<false>(wb, A.ddots, lo, hi, d);
        win_load<false>(wdc, A.dcloud, blo, bhi, d);
        win_load<false>(wsc, A.cloud, clo, chi, d);
        const u64 vd = A.vvd[k * A.R + dcol(d)], vs = A.vv[(u64)sl * A.R + dcol(d)];
        bool eqb, indc, insc;
        const u64 p = win_rank(wb, d, eqb);
        win_rank(wdc, d, indc);
        win_rank(wsc, d, insc);
        xr = (u32)(p - lo);
        if (eqb) {
          f = 1;
          if (!(dseq(d) <= vs || insc)) xr |= 1u << 31;
        } else {
          f = A.keep_all || !(dseq(d) <= vd || indc);
        }
      } else if (kind == 1) {
        const u64 lo = A.abase[k], hi = lo + (A.ao[k + 1] - A.ao[k]);
        const u64 d = A.ddots[i];
        Win<8> wa;
        Win<4> wsc;
        win_load<true>(wa, A.rec, lo, hi, d);
        win_load<false>(wsc, A.cloud, clo, chi, d);
        const u64 vs = A.vv[(u64)sl * A.R + dcol(d)];
        bool eqa, insc;
        const u64 p = win_rank(wa, d, eqa);
        win_rank(wsc, d, insc);
        xr = (u32)(p - lo);
        f = !eqa && !(dseq(d) <= vs || insc);
      } else {
        const u64 x = A.dcloud[i];
        Win<8> wsc;
        win_load<false>(wsc, A.cloud, clo, chi, x);
        bool insc;
        const u64 p = win_rank(wsc, x, insc);
        xr = (u32)(p - clo);
        f = !insc;
      }
      A.xr[gbase + i] = xr;
    }
  }
  JY_CLK(c1);
  u64 tot;
  const u64 x = item_scan(f, red, tot);
  JY_CLK(c2);
  JY_PROBE(2, kind + ((u32)(tmv >> 32) == A.epoch ? 8 : 0), (u32)t, c0, c1, c2);
  if (i < n) A.sc[gbase + i] = (u32)x;
  if (threadIdx.x == 0) A.tp[t] = tot;
}

// item launches: the grid comes from the newest finished converge's touched
// sizes (a prediction, not a bound); the workgroups stride over the tiles this
// converge really has (read on the device), so a short grid stays exact.  The
// host's safe bound (the live-element count) launched ~4x the real tiles,
// and every surplus workgroup paid a dispatch and a dependent load to exit.
__global__ __launch_bounds__(kItemThreads) void k_uj_flags(UjArgs A) {
  __shared__ u64 red[kItemThreads / 64];
  if (A.lcol && blockIdx.x == 0 && threadIdx.x == 0) A.ctr[5] = 0;  // k_uj_jobs (demotions, regrowths) is done
  const u64 T = cdiv(A.ao[A.nd]) + cdiv(A.nb) + cdiv(A.cb);
  for (u64 t = blockIdx.x; t < T; t += gridDim.x) uj_flags_tile(A, t, red);
}

// ---- U3: cloud compaction against the merged vv ---------------------------------
// union rank of x (column c, seq q) above v: state dots of c in (v, q) plus
// de-duplicated delta dots of c in (v, q) (U2's kind-2 flags); x folds into
// the vv when the run from v + 1 reaches it unbroken
// U3 for a wave of cloud items inside long document k (wave-uniform; sa:
// state cloud, else delta cloud): as uj_compact_tile, with the run starts of
// the wave's first and last column and the bounds of its dot range found by
// wave-cooperative searches (a wave of a long cloud spans one or two columns)
__device__ __forceinline__ void uj_compact_long(const UjArgs& A, bool sa, u64 k, u64 i, u64 n, u64& f) {
  const bool live = i < n;
  const u64 lm = __ballot(live);
  if (lm == 0) return;
  const int lastl = __popcll(lm) - 1;
  const u64 ta = A.ao[A.nd], tc = A.co[A.nd];
  const ScanSp sp = sc_space(A);
  const u64 cb0 = ta + A.nb;
  const u64 alo = A.cbs[k], ahi = alo + (A.co[k + 1] - A.co[k]);
  const u64 blo = A.dcoff[k], bhi = A.dcoff[k + 1];
  const u64 pi = alo + (i - A.co[k]);
  u64 x = 0;
  if (live) x = sa ? A.cloud[pi] : A.dcloud[i];
  const u64 x0 = __shfl(x, 0), x1 = __shfl(x, lastl) + 1;
  const u32 cf = dcol(x0), cl = dcol(x1 - 1);
  // the merged vv of the wave's first and last column, read ONCE: the run
  // starts below are searched from them, and an item of those columns must
  // test its fold against the same value.  (Other waves' folds raise the row
  // meanwhile; the fold test is exact for any value the row takes, but only
  // with its run start and its count taken from that same value -- re-reading
  // the row here made config-5 converges nondeterministic in round 3.)
  const u64 vf = merged_vv(A, k, cf), vl = cl == cf ? vf : merged_vv(A, k, cl);
  const u64 lof = mkdot(cf, vf + 1), lol = mkdot(cl, vl + 1);
  // [0, 1]: run starts on the state side, [2, 3]: on the delta side, [4, 5]:
  // the other side's bounds of the wave's dots
  WSearch s[6] = {{A.cloud, 1, alo, ahi, lof},  {A.cloud, 1, alo, ahi, lol}, {A.dcloud, 1, blo, bhi, lof},
                  {A.dcloud, 1, blo, bhi, lol}, {sa ? A.dcloud : A.cloud, 1, sa ? blo : alo, sa ? bhi : ahi, x0},
                  {sa ? A.dcloud : A.cloud, 1, sa ? blo : alo, sa ? bhi : ahi, x1}};
  wave_lbs<6>(s);
  if (!live) return;
  const u32 c = dcol(x);
  const u64 q = dseq(x), v = c == cf ? vf : c == cl ? vl : merged_vv(A, k, c);
  if (q <= v) return;
  const u64 lo = mkdot(c, v + 1);
  const u64 ra0 = c == cf ? s[0].lo : c == cl ? s[1].lo : lower_bound(A.cloud, alo, ahi, lo);
  const u64 b0 = c == cf ? s[2].lo : c == cl ? s[3].lo : lower_bound(A.dcloud, blo, bhi, lo);
  if (sa) {
    const u64 ra = pi - ra0;
    const u64 b1 = lower_bound(A.dcloud, s[4].lo, s[5].lo, x);
    const u64 rb = sp.at(cb0 + b1) - sp.at(cb0 + b0);
    if (q == v + 1 + ra + rb) {
      __hip_atomic_fetch_max(&A.vv[(u64)A.slot[k] * A.R + c], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      f = 1;
      A.kr[i] = (u32)(b1 - blo);
    }
  } else {
    const u64 s0 = sp.at(cb0 + i);
    if (sp.at(cb0 + i + 1) == s0) return;  // held by the state cloud
    const u64 a1 = lower_bound(A.cloud, s[4].lo, s[5].lo, x);
    const u64 rb = s0 - sp.at(cb0 + b0);
    if (q == v + 1 + (a1 - ra0) + rb) {
      __hip_atomic_fetch_max(&A.vv[(u64)A.slot[k] * A.R + c], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      f = 1;
      A.kr[tc + i] = (u32)(a1 - alo);
    }
  }
}

__device__ __forceinline__ void uj_compact_tile(const UjArgs& A, const u64 t, u64* red) {
  const u64 ta = A.ao[A.nd], tc = A.co[A.nd];
  const ScanSp sp = sc_space(A);
  const u64 cb0 = ta + A.nb;  // the delta cloud dedupe prefix: sp.at(cb0 + b)
  const u64 tA = cdiv(tc);
  JY_CLK(c0);
  const bool sa = t < tA;  // state cloud items, else delta cloud items
  const u64 lt = sa ? t : t - tA, n = sa ? tc : A.cb, gbase = sa ? 0 : tc;
  const u64 i = lt * kTile + threadIdx.x;
  u64 f = 0;
  const u64 tmv = sa ? A.tmC[lt] : A.tmD[lt];
  if ((u32)(tmv >> 32) == A.epoch) {  // a tile inside one long document
    const u64 k = (u32)tmv;
    if (!is_bad(A, k) && !is_fast(A, k)) uj_compact_long(A, sa, k, i, n, f);
  } else if (i < n) {
    // small documents: the item's independent lookups issued together
    const u64 k = (u32)(tmv >> 32) == A.epoch ? (u32)tmv : (sa ? A.sidC[i] : A.sidD[i]);
    const bool bad = is_bad(A, k) || is_fast(A, k);
    const u64 alo = A.cbs[k], co0 = A.co[k], ahi = alo + (A.co[k + 1] - co0);
    const u64 blo = A.dcoff[k], bhi = A.dcoff[k + 1];
    const u32 sl = A.slot[k];
    if (sa) {
      const u64 pi = alo + (i - co0);
      const u64 x = bad ? 0 : A.cloud[pi];
      const u32 c = dcol(x);
      const u64 q = dseq(x);
      Win<4> w1;
      if (!bad) win_load<false>(w1, A.dcloud, blo, bhi, x);  // b1 needs only x
      const u64 v = bad ? ~0ull : merged_vv(A, k, c);
      if (q > v) {
        const u64 lo = mkdot(c, v + 1);
        Win<4> wa, w0;
        win_load<false>(wa, A.cloud, alo, pi, lo);
        win_load<false>(w0, A.dcloud, blo, bhi, lo);
        bool e;
        const u64 b1 = win_rank(w1, x, e);
        const u64 ra = pi - win_rank(wa, lo, e);
        const u64 b0 = win_rank(w0, lo, e);
        const u64 rb = sp.at(cb0 + b1) - sp.at(cb0 + b0);
        if (q == v + 1 + ra + rb) {
          __hip_atomic_fetch_max(&A.vv[(u64)sl * A.R + c], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          f = 1;
          A.kr[i] = (u32)(b1 - blo);
        }
      }
    } else {
      // the dedupe prefix and the dot need no document
      const u64 s0 = sp.at(cb0 + i), s1 = sp.at(cb0 + i + 1);
      const u64 x = A.dcloud[i];
      const u32 c = dcol(x);
      const u64 q = dseq(x);
      if (!bad && s1 != s0) {  // not held by the state cloud
        Win<4> w1;
        win_load<false>(w1, A.cloud, alo, ahi, x);  // a1 needs only x
        const u64 v = merged_vv(A, k, c);
        if (q > v) {
          const u64 lo = mkdot(c, v + 1);
          Win<4> wa, wb;
          win_load<false>(wa, A.cloud, alo, ahi, lo);
          win_load<false>(wb, A.dcloud, blo, i, lo);
          bool e;
          const u64 a1 = win_rank(w1, x, e);
          const u64 a0 = win_rank(wa, lo, e);
          const u64 b0 = win_rank(wb, lo, e);
          const u64 rb = s0 - sp.at(cb0 + b0);
          if (q == v + 1 + (a1 - a0) + rb) {
            __hip_atomic_fetch_max(&A.vv[(u64)sl * A.R + c], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            f = 1;
            A.kr[tc + i] = (u32)(a1 - alo);
          }
        }
      }
    }
  }
  JY_CLK(c1);
  u64 tot;
  const u64 x = item_scan(f, red, tot);
  JY_CLK(c2);
  JY_PROBE(3, (sa ? 0 : 1) + ((u32)(tmv >> 32) == A.epoch ? 8 : 0), (u32)t, c0, c1, c2);
  if (i < n) A.ksc[gbase + i] = (u32)x;
  if (threadIdx.x == 0) A.ktp[t] = tot;
}

__global__ __launch_bounds__(kItemThreads) void k_uj_compact(UjArgs A) {
  __shared__ u64 red[kItemThreads / 64];
  const u64 T = cdiv(A.co[A.nd]) + cdiv(A.cb);
  for (u64 t = blockIdx.x; t < T; t += gridDim.x) uj_compact_tile(A, t, red);
}

// ---- U4: output sizes per delta doc (scanned); the bump pointers move --------------
__global__ __launch_bounds__(kThreads) void k_uj_sizes(UjArgs A, u64 ndt) {
  __shared__ Shared S;
  const u32 t = jyscan::ticket(A.tick + T_U4, &S.tk);
  if (t >= ndt) return;
  const u64 ta = A.ao[A.nd], tc = A.co[A.nd];
  const ScanSp sp = sc_space(A), kp = ksc_space(A);
  const u64 k = (u64)t * kDocTile + threadIdx.x;
  JY_CLK(c0);
  u64 ne = 0, nc = 0;
  if (k < A.nd && is_bad(A, k) && A.slot[k] != JY_NO_SLOT && A.dptr[A.slot[k]] == (((u64)A.epoch << 32) | (u32)k))
    atomicAdd(A.skipped, 1ull);  // a bad doc counted once per slot
  if (k < A.nd && !is_bad(A, k)) {
    ne = (sp.at(A.ao[k + 1]) - sp.at(A.ao[k])) + (sp.at(ta + A.deoff[k + 1]) - sp.at(ta + A.deoff[k]));
    nc = (kp.at(A.co[k + 1]) - kp.at(A.co[k])) + (kp.at(tc + A.dcoff[k + 1]) - kp.at(tc + A.dcoff[k]));
  }
  u64 tot;
  const u64 xe = jyscan::block_excl<kThreads, u64>(ne, S.red, tot);
  const u64 pe = jyscan::lookback(A.st_ne, t, A.epoch, tot, &S.pre);
  const u64 te = pe + tot;
  if (k < A.nd) A.neo[k] = pe + xe;
  const u64 xc = jyscan::block_excl<kThreads, u64>(nc, S.red, tot);
  const u64 pc = jyscan::lookback(A.st_nc, t, A.epoch, tot, &S.pre);
  if (k < A.nd) A.nco[k] = pc + xc;
  JY_CLK(c2);
  JY_PROBE(4, 0, t, c0, c0, c2);
  if (t == ndt - 1 && threadIdx.x == 0) {
    const u64 tcl = pc + tot;
    A.neo[A.nd] = te;
    A.nco[A.nd] = tcl;
    u64* st = A.stats;  // stream-ordered: one writer per converge
    st[0] += A.ao[A.nd];
    st[1] += A.co[A.nd];
    st[2] += te;
    st[3] += tcl;
    st[4] += A.nb;
    st[5] += A.cb;
    st[6] += A.nd;
    st[7] += 1;
    const u64 eb = A.ctr[0], cbb = A.ctr[1];
    A.base[0] = eb;
    A.base[1] = cbb;
    A.ctr[0] = eb + te;
    A.ctr[1] = cbb + tcl;
    A.pin[0] = eb + te;  // mapped host memory: the host's exact pool use once the converge is done
    A.pin[1] = cbb + tcl;
    A.pin_t[0] = A.ao[A.nd];
    A.pin_t[1] = A.co[A.nd];
    if (A.lcol) {
      A.pin_l[0] = A.ctr[2];
      A.pin_l[1] = A.ctr[3];
      A.pin_l[2] = A.ctr[4];
    }
  }
}

// ---- U5: scatter into the fresh runs; vv rows, metas; zero state for the next converge
// (no scan.)  A workgroup of kScatterThreads lanes takes a tile of kTile
// items, kScatterU items per lane: a lane first issues the dependent loads of
// all its items (scatter_prep: loads only), then stores them.  (Round 5,
// in-box A/B, ms per config-5 converge, 2 runs each: 1 item per lane 0.380 /
// 0.382, 2 items 0.381 / 0.381, 4 items 0.382 / 0.382 -- more chains in
// flight per wave do not help: 1.)
constexpr int kScatterU = 1;  // (the loop form below is kept: the compiler's code for it measured faster)
constexpr int kScatterThreads = (int)kTile / kScatterU;

struct ScOut {
  u32 what;  // 0 nothing, 1 an element record, 2 a cloud dot
  u64 at;    // pool index
  u64 a, b;  // dot, element
};

// an element / cloud item's destination and payload (kinds 0..3; loads only)
__device__ __forceinline__ ScOut scatter_prep(const UjArgs& A, int kind, u64 lt, u64 i, u64 ta, u64 tc,
                                              const ScanSp& sp, const ScanSp& kp, const u32* xrb, const u32* krb) {
  const u64 eb0 = A.base[0], cb0 = A.base[1];
  ScOut o{0, 0, 0, 0};
  if (kind == 0) {  // state element
    if (i >= ta) return o;
    const u64 si = sp.at(i);
    if (sp.at(i + 1) == si) return o;
    const u64 k = doc_at(A, A.tmA, lt, A.sidA, i);
    const URec x = load_rec(A.rec + A.abase[k] + (i - A.ao[k]));
    const u32 xv = A.xr[i];
    const u64 lo = A.deoff[k], p = lo + (xv & 0x7FFFFFFFu);
    o = ScOut{1, eb0 + A.neo[k] + (si - sp.at(A.ao[k])) + (sp.at(ta + p) - sp.at(ta + lo)), x.dot,
              (xv >> 31) ? A.delems[p] : x.elem};
  } else if (kind == 1) {  // delta element
    if (i >= A.nb) return o;
    const u64 si = sp.at(ta + i);
    if (sp.at(ta + i + 1) == si) return o;
    const u64 k = doc_at(A, A.tmB, lt, A.sidB, i);
    const u64 pa = A.ao[k] + xrb[i];
    o = ScOut{1, eb0 + A.neo[k] + (si - sp.at(ta + A.deoff[k])) + (sp.at(pa) - sp.at(A.ao[k])), A.ddots[i],
              A.delems[i]};
  } else if (kind == 2) {  // state cloud dot
    if (i >= tc) return o;
    const u64 si = kp.at(i);
    if (kp.at(i + 1) == si) return o;
    const u64 k = doc_at(A, A.tmC, lt, A.sidC, i);
    const u64 x = A.cloud[A.cbs[k] + (i - A.co[k])];
    const u64 lo = A.dcoff[k];
    o = ScOut{2, cb0 + A.nco[k] + (si - kp.at(A.co[k])) + (kp.at(tc + lo + A.kr[i]) - kp.at(tc + lo)), x, 0};
  } else {  // delta cloud dot
    if (i >= A.cb) return o;
    const u64 si = kp.at(tc + i);
    if (kp.at(tc + i + 1) == si) return o;
    const u64 k = doc_at(A, A.tmD, lt, A.sidD, i);
    const u64 pa = A.co[k] + krb[i];
    o = ScOut{2, cb0 + A.nco[k] + (si - kp.at(tc + A.dcoff[k])) + (kp.at(pa) - kp.at(A.co[k])), A.dcloud[i], 0};
  }
  return o;
}

// U5 for a delta doc converged in place: the column runs take their new
// lengths (and the runs that grew, their new places), a cloud run that was
// empty starts past its folded prefix, the vv takes the folds, the meta its
// new totals
// U5 for a delta doc converged in place, one WAVE per document (lane c =
// column c): the column runs take their new lengths (and the runs that grew,
// their new places; a trimmed run starts `cut` further up), a cloud run that
// was empty starts past its folded prefix, the vv takes the folds, the meta
// its new totals.  Lane 0 returns the in-place counters (jy_ujson_stats_ext).
struct CommitStats {
  u64 v[6];  // docs, their state elements / cloud dots, appended elements / cloud dots, folded
};
__device__ void uj_commit_long(const UjArgs& A, u64 i, CommitStats& cs) {
  const u32 lane = threadIdx.x & 63, R = A.R, s = A.slot[i], lid = (u32)A.abase[i];
  const u64 b = (u64)lid * R;
  const UMeta m = A.meta[s];
  u64 ne = 0, nc = 0, cut = 0, nf = 0;
  if (lane < R) {
    const LPlan& P = A.lplan[b + lane];
    const u64 efs = P.efs, ece = P.ece, cfs = P.cfs, cce = P.cce, nfw = P.nfold, tcw = P.tcut;
    ne = tagged(A, efs) ? (u32)ece - (u32)efs : 0;
    nc = tagged(A, cfs) ? (u32)cce - (u32)cfs : 0;
    cut = tagged(A, tcw) ? (u32)tcw : 0;
    if (ne || nc || cut) {
      nf = tagged(A, nfw) ? (u32)nfw : 0;
      const LCol L = A.lcol[b + lane];
      // (a trimmed run never moved: erun is its old start, now `cut` further up)
      LCol N{P.erun + cut, (u32)(L.elen - cut + ne), (u32)(P.ecap - cut), P.crun, (u32)(L.clen + nc), P.ccap};
      if (P.cz) {
        N.clen = (u32)(nc - nf);
        if (nf < nc) {
          N.cbase = P.crun + nf;
          N.ccap = (u32)(P.ccap - nf);
        }
      }
      A.lcol[b + lane] = N;
      if (nf) A.vv[(u64)s * R + lane] += nf;
    }
  }
  const u64 app = jyscan::wave_sum<u64>(ne), cuts = jyscan::wave_sum<u64>(cut);
  const u64 dC = jyscan::wave_sum<u64>(nc - nf), nfs = jyscan::wave_sum<u64>(nf);
  if (lane == 0) {
    A.meta[s] = UMeta{lid, (u32)(m.elen + app - cuts), kLongMark, 0, (u32)(m.clen + dC), kLongMark};
    cs = CommitStats{{1, m.elen, m.clen, app, dC, nfs}};
  }
}

// U5's document tiles: regular docs get their metas (and are listed for
// promotion when they are long enough); docs in place are committed by the
// commit tiles (a wave per document, flist)
__device__ void uj_meta_tile(const UjArgs& A, u64 lt) {
  const u64 eb0 = A.base[0], cb0 = A.base[1];
  const u64 i = lt * kTile + threadIdx.x;
  if (i >= A.nd || is_bad(A, i) || is_fast(A, i)) return;
  const u32 ne = (u32)(A.neo[i + 1] - A.neo[i]), nc = (u32)(A.nco[i + 1] - A.nco[i]);
  A.meta[A.slot[i]] = UMeta{eb0 + A.neo[i], ne, ne, cb0 + A.nco[i], nc, nc};
  if (A.long_min && ne >= A.long_min) A.plist[atomicAdd((unsigned long long*)(A.ctr + 6), 1ull)] = (u32)i;
}

__device__ __forceinline__ void scatter_small(const UjArgs& A, int kind, u64 i) {
  const u64 nv = A.nvv;
  if (kind == 4) {  // the delta's sparse vv entries into the state rows; the dense delta vv back to zero
    if (i >= nv) return;
    const u64 x = A.dvv[i];
    const u32 c = dcol(x);
    if (c >= A.R) return;  // never written (the doc is bad)
    const u64 k = A.sidV[i];
    // the state rows already hold U3's folds; elsewhere max(state, delta) is
    // the state (one entry per (doc, column) unless the doc is bad; a doc in
    // place has no entry above the state's)
    if (!is_bad(A, k) && !is_fast(A, k)) {
      u64* r = A.vv + (u64)A.slot[k] * A.R + c;
      const u64 q = dseq(x);
      if (q > *r) *r = q;
    }
    A.vvd[k * A.R + c] = 0;
    return;
  }
}

__device__ __forceinline__ void uj_scatter_tile(const UjArgs& A, const u64 t, const u64 nfast) {
  const u64 ta = A.ao[A.nd], tc = A.co[A.nd];
  const ScanSp sp = sc_space(A), kp = ksc_space(A);
  const u32* xrb = A.xr + ta;
  const u32* krb = A.kr + tc;
  const u64 nv = A.nvv;
  constexpr u64 kWpT = kScatterThreads / 64;  // commit tiles: a wave per document in place
  const u64 tl[7] = {cdiv(ta), cdiv(A.nb), cdiv(tc), cdiv(A.cb), cdiv(nv), cdiv(A.nd), (nfast + kWpT - 1) / kWpT};
  int kind = 0;
  u64 lt = t;
  while (kind < 7 && lt >= tl[kind]) lt -= tl[kind++];
  if (kind == 7) return;
  JY_CLK(c0);
  if (kind == 6) {
    const u64 q = lt * kWpT + (threadIdx.x >> 6);
    CommitStats cs{};
    if (q < nfast) uj_commit_long(A, A.flist[q], cs);
    if ((threadIdx.x & 63) == 0 && cs.v[0]) {
#pragma unroll
      for (int x = 0; x < 6; x++) atomicAdd((unsigned long long*)(A.stats + 8 + x), (unsigned long long)cs.v[x]);
    }
  } else if (kind == 5) {
    uj_meta_tile(A, lt);
  } else if (kind == 4) {
#pragma unroll
    for (int u = 0; u < kScatterU; u++) scatter_small(A, kind, lt * kTile + (u64)u * kScatterThreads + threadIdx.x);
  } else {
    ScOut o[kScatterU];
#pragma unroll
    for (int u = 0; u < kScatterU; u++)
      o[u] = scatter_prep(A, kind, lt, lt * kTile + (u64)u * kScatterThreads + threadIdx.x, ta, tc, sp, kp, xrb, krb);
#pragma unroll
    for (int u = 0; u < kScatterU; u++) {
      if (o[u].what == 1) store_rec(A.epool_out + o[u].at, o[u].a, o[u].b);
      else if (o[u].what == 2) A.cpool_out[o[u].at] = o[u].a;
    }
  }
  JY_CLK(c2);
#ifdef JY_UJ_PROBE
  const u64* tmk = kind == 0 ? A.tmA : kind == 1 ? A.tmB : kind == 2 ? A.tmC : A.tmD;
  const bool lng = kind < 4 && (u32)(tmk[lt] >> 32) == A.epoch;
#endif
  JY_PROBE(5, kind + (lng ? 8 : 0), (u32)lt, c0, c2, c2);
}

__global__ __launch_bounds__(kScatterThreads) void k_uj_scatter(UjArgs A) {
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int c = T_U1; c <= T_U4; c++) A.tick[c] = 0;  // U1..U4 of this converge are done
  const u64 nf = A.lcol ? A.ctr[7] : 0;
  const u64 T = cdiv(A.ao[A.nd]) + cdiv(A.nb) + cdiv(A.co[A.nd]) + cdiv(A.cb) + cdiv(A.nvv) + cdiv(A.nd) +
                (nf + kScatterThreads / 64 - 1) / (kScatterThreads / 64);
  for (u64 t = blockIdx.x; t < T; t += gridDim.x) uj_scatter_tile(A, t, nf);
}

// ---- P: promotion of the merged documents U5 listed (>= long_min elements):
// one wave per document finds its column boundaries in the fresh regular run
// (lane c: the first dot of column c), takes a long id and room in the long
// pools (2n + 16 per column run), writes the column table and the copy jobs
// (k_uj_jobs runs them next) and marks the meta long.  Optional: without
// room the document simply stays regular.
constexpr u64 kSelfCopy = 4096;  // entries a promoting wave copies itself
__global__ __launch_bounds__(kThreads) void k_uj_promote(UjArgs A) {
  const u64 n = A.ctr[6];
  UJob* jobs = A.jobs + 2 * A.jcap;  // the promotion region: job j <-> plist entry j (n = 0: copied here)
  const u32 lane = threadIdx.x & 63, R = A.R;
  const u64 W = (u64)gridDim.x * (kThreads / 64);
  for (u64 j = (u64)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); j < n; j += W) {
    const u64 i = A.plist[j];
    const u32 s = A.slot[i];
    const UMeta m = A.meta[s];
    const bool act = lane < R;
    u64 e0 = m.elen, c0 = m.clen;
    if (act) {  // lane c: the first element / cloud dot of column c (the two searches in lockstep)
      const u64 x = mkdot(lane, 0);
      u64 elo = m.ebase, ehi = m.ebase + m.elen, clo = m.cbase, chi = m.cbase + m.clen;
      while (elo < ehi || clo < chi) {
        const u64 em = (elo + ehi) >> 1, cm = (clo + chi) >> 1;
        const u64 ev = elo < ehi ? A.rec[em].dot : 0, cv = clo < chi ? A.cloud[cm] : 0;
        if (elo < ehi) (ev < x ? elo = em + 1 : ehi = em);
        if (clo < chi) (cv < x ? clo = cm + 1 : chi = cm);
      }
      e0 = elo - m.ebase;
      c0 = clo - m.cbase;
    }
    u64 e1 = __shfl(e0, (int)((lane + 1) & 63)), c1 = __shfl(c0, (int)((lane + 1) & 63));
    if (lane + 1 >= R) e1 = m.elen, c1 = m.clen;
    const u64 ne = act ? e1 - e0 : 0, nc = act ? c1 - c0 : 0;
    const u64 ecap = act ? roomy(ne) : 0, ccap = act ? roomy(nc) : 0;
    const u64 oe = jyscan::wave_incl<u64>(ecap) - ecap, oc = jyscan::wave_incl<u64>(ccap) - ccap;
    const u64 TE = __shfl(oe + ecap, 63), TC = __shfl(oc + ccap, 63);
    u64 lid = 0, eb = 0, cb = 0, ok = 0;
    if (lane == 0) {  // (a refused promotion wastes its reservations until the next compaction)
      lid = atomicAdd((unsigned long long*)(A.ctr + 4), 1ull);
      eb = atomicAdd((unsigned long long*)(A.ctr + 2), (unsigned long long)TE);
      cb = atomicAdd((unsigned long long*)(A.ctr + 3), (unsigned long long)TC);
      ok = lid < A.lcap && eb + TE <= A.lpe_cap && cb + TC <= A.lpc_cap;
    }
    ok = __shfl(ok, 0);
    if (!ok) {
      if (lane == 0) jobs[j] = UJob{0, 0, 0, UJ_PROMOTE, 0};
      continue;
    }
    lid = __shfl(lid, 0);
    eb = __shfl(eb, 0);
    cb = __shfl(cb, 0);
    if (act) A.lcol[lid * R + lane] = LCol{eb + oe, (u32)ne, (u32)ecap, cb + oc, (u32)nc, (u32)ccap};
    // the copy: a short document (the usual promotion: one the regular path
    // just rewrote past the threshold) by this wave, column after column; a
    // long one (a demoted hot document coming back) by the copy grid
    const bool self = (u64)m.elen + m.clen <= kSelfCopy;
    if (self) {
      for (u32 c = 0; c < R; c++) {
        const u64 e0c = __shfl(e0, (int)c), nec = __shfl(ne, (int)c), dstc = eb + __shfl(oe, (int)c);
        for (u64 x = lane; x < nec; x += 64) A.lpe[dstc + x] = A.rec[m.ebase + e0c + x];
        const u64 c0c = __shfl(c0, (int)c), ncc = __shfl(nc, (int)c), dcc = cb + __shfl(oc, (int)c);
        for (u64 x = lane; x < ncc; x += 64) A.lpc[dcc + x] = A.cloud[m.cbase + c0c + x];
      }
    }
    if (lane == 0) {
      jobs[j] = UJob{m.ebase, m.cbase, self ? 0 : (u64)m.elen + m.clen, UJ_PROMOTE, (u32)lid};
      A.meta[s] = UMeta{lid, m.elen, kLongMark, 0, m.clen, kLongMark};
      atomicAdd((unsigned long long*)(A.stats + 14), 1ull);
    }
  }
}

// ---- compaction: every document rewritten back to back into fresh pools ------------
__global__ __launch_bounds__(kThreads) void k_uj_cmp_size(const UMeta* __restrict__ meta, u64 nk,
                                                          u64* __restrict__ se, u64* __restrict__ sc) {
  const u64 s = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (s > nk) return;
  se[s] = s == nk ? 0 : meta[s].elen;
  sc[s] = s == nk ? 0 : meta[s].clen;
}
constexpr u32 kTileOut = 2048;
// (long documents are laid out regular again: compaction empties the long pools)
template <bool kElems, typename T>
__global__ __launch_bounds__(kThreads) void k_uj_cmp_copy(const UMeta* __restrict__ meta, u64 nk,
                                                          const u64* __restrict__ off, const T* __restrict__ src,
                                                          T* __restrict__ dst, const LCol* __restrict__ lcol,
                                                          const T* __restrict__ lsrc, u32 R) {
  __shared__ Shared S;
  const u64 total = off[nk];
  const u64 t0 = (u64)blockIdx.x * kTileOut;  // the grid is the host's bound
  if (t0 >= total) return;
  const u64 t1 = t0 + kTileOut < total ? t0 + kTileOut : total;
  const TileDocs D = tile_docs<kLdsDocs>(off, nk, t0, t1, S.offs, S.sh);
  for (u64 t = t0 + threadIdx.x; t < t1; t += kThreads) {
    const u64 k = doc_of(D, off, S.offs, t);
    const UMeta m = meta[k];
    if (m.ecap == kLongMark) dst[t] = lsrc[uj_long_at<kElems>(lcol + m.ebase * R, R, t - off[k])];
    else dst[t] = src[(kElems ? m.ebase : m.cbase) + (t - off[k])];
  }
}
__global__ __launch_bounds__(kThreads) void k_uj_cmp_meta(UMeta* __restrict__ meta, u64 nk, const u64* __restrict__ eo,
                                                          const u64* __restrict__ co) {
  const u64 s = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (s >= nk) return;
  UMeta m = meta[s];
  m.ebase = eo[s];
  m.ecap = m.elen;
  m.cbase = co[s];
  m.ccap = m.clen;
  meta[s] = m;
}

// ---- reads ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_uj_sizes_read(const UMeta* __restrict__ meta, const u32* __restrict__ slots,
                                                       u64 n, u64* __restrict__ ne, u64* __restrict__ nc) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const UMeta m = meta[slots[i]];
  ne[i] = m.elen;
  nc[i] = m.clen;
}

// reads, flattened over the output: a tile of kThreads output items finds
// its documents with two wave searches of the output offsets (a hot document
// of 10^5 elements is spread over many tiles instead of one thread's loop)
template <bool kEl>
__global__ __launch_bounds__(kThreads) void k_uj_gather_items(const UMeta* __restrict__ meta,
                                                              const URec* __restrict__ rec,
                                                              const u64* __restrict__ cloud,
                                                              const u32* __restrict__ slots, u64 n,
                                                              const u64* __restrict__ ooff, u64 total,
                                                              u64* __restrict__ oa, u64* __restrict__ ob,
                                                              const LCol* __restrict__ lcol,
                                                              const URec* __restrict__ lpe,
                                                              const u64* __restrict__ lpc, u32 R) {
  __shared__ u64 sh[2];
  const u64 t0 = (u64)blockIdx.x * kThreads;
  if (t0 >= total) return;
  const u64 t1 = t0 + kThreads < total ? t0 + kThreads : total;
  if (threadIdx.x < 128) {
    const u64 k = jyscan::wave_last_le(ooff, n, threadIdx.x < 64 ? t0 : t1 - 1);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = k;
  }
  __syncthreads();
  const u64 t = t0 + threadIdx.x;
  if (t >= t1) return;
  u64 lo = sh[0], hi = sh[1];
  while (lo < hi) {
    const u64 m = (lo + hi + 1) >> 1;
    if (ooff[m] <= t) lo = m;
    else hi = m - 1;
  }
  const UMeta m = meta[slots[lo]];
  const u64 j = t - ooff[lo];
  const bool lg = m.ecap == kLongMark;
  if (kEl) {
    const URec r = lg ? lpe[uj_long_at<true>(lcol + m.ebase * R, R, j)] : rec[m.ebase + j];
    oa[t] = r.dot;
    ob[t] = r.elem;
  } else {
    oa[t] = lg ? lpc[uj_long_at<false>(lcol + m.ebase * R, R, j)] : cloud[m.cbase + j];
  }
}

__global__ __launch_bounds__(kThreads) void k_uj_gather_vv(const u64* __restrict__ vv, u32 R,
                                                           const u32* __restrict__ slots, u64 n,
                                                           u64* __restrict__ ovv) {
  const u64 g = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (g >= n * R) return;
  const u64 i = g / R, c = g - i * R;
  ovv[g] = vv[(u64)slots[i] * R + c];
}

u64 cdiv_h(u64 a) { return (a + kTile - 1) / kTile; }
u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

#define LAUNCH(k, n, ...)                                                                          \
  do {                                                                                             \
    hipLaunchKernelGGL(k, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, __VA_ARGS__);     \
    JY_HIP(eng, hipGetLastError());                                                                \
  } while (0)

void ujson_absorb(UjsonState& u);
int32_t ujson_long_grow(jy_engine* eng, UjsonState& u);

// the compacted pools' bump pointers: on the device, and into the host's
// mapped ring slot
__global__ void k_uj_cmp_ctr(const u64* __restrict__ te, const u64* __restrict__ tc, u64* __restrict__ ctr,
                             u64* __restrict__ pin, u64* __restrict__ pin_l) {
  ctr[0] = pin[0] = *te;
  ctr[1] = pin[1] = *tc;
  // every long document is regular again: the long pools are empty
  ctr[2] = ctr[3] = ctr[4] = 0;
  pin_l[0] = pin_l[1] = pin_l[2] = 0;
}

// rewrite every document back to back into the spare pools, sized for the
// host's bound of live entries plus `room_e` / `room_c` several times over,
// then swap.  Asynchronous: the exact compacted sizes reach the host through
// the converge ring like a converge's bump pointers (the spare pools are
// reallocated -- a synchronising hipMalloc -- only when they are too small).
int32_t ujson_compact(jy_engine* eng, UjsonState& u, u64 room_e, u64 room_c) {
  const u64 nk = eng->nkeys[JY_UJSON];
  if (u.seq - u.done == UjsonState::kRing) {  // its ring slot
    JY_HIP(eng, hipEventSynchronize(u.ready[u.done % UjsonState::kRing]));
    ujson_absorb(u);
  }
  void* p;
  JY_TRY(jy_scratch(eng, 20, (nk + 1) * 32, &p));
  u64* se = static_cast<u64*>(p);
  u64* sc = se + nk + 1;
  u64* eo = sc + nk + 1;
  u64* co = eo + nk + 1;
  LAUNCH(k_uj_cmp_size, nk + 1, u.meta, nk, se, sc);
  JY_TRY(jy_scan_u64(eng, se, eo, nk));
  JY_TRY(jy_scan_u64(eng, sc, co, nk));
  const u64 be = u.live_e, bc = u.live_c;  // >= the compacted sizes
  // Headroom: `room` is one converge's WORST case (every live entry touched),
  // so the element pool's 16x lasts ~70 config-5 converges.  The cloud pool
  // is small but every converge rewrites its touched documents' clouds
  // (~0.7M dots against ~1.3M worst case), so 8x lasted ~10 converges and a
  // compaction (~0.25 ms + a host wait) landed every few bench steps; 64x
  // is ~0.7 GB at config 5 -- HBM is plentiful, compactions are not free.
#ifndef JY_UJ_ROOM_E
#define JY_UJ_ROOM_E 16
#endif
#ifndef JY_UJ_ROOM_C
#define JY_UJ_ROOM_C 64
#endif
  constexpr u64 kRoomE = JY_UJ_ROOM_E, kRoomC = JY_UJ_ROOM_C;
  const u64 ecap = std::max<u64>({be + kRoomE * room_e, 3 * be, eng->cfg.entry_capacity[JY_UJSON], 1024});
  const u64 ccap = std::max<u64>({bc + kRoomC * room_c, 3 * bc, eng->cfg.entry_capacity[JY_UJSON], 1024});
  JY_TRACE("ujson compact: <= %llu elements, <= %llu cloud dots -> pools %llu / %llu", (unsigned long long)be,
           (unsigned long long)bc, (unsigned long long)ecap, (unsigned long long)ccap);
  if (u.spare_ecap < ecap) {
    jy_dev_free(eng, u.spare_e);
    u.spare_e = nullptr;
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.spare_e), ecap * sizeof(URec), "ujson element pool"));
    u.spare_ecap = ecap;
  }
  if (u.spare_ccap < ccap) {
    jy_dev_free(eng, u.spare_c);
    u.spare_c = nullptr;
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.spare_c), ccap * 8, "ujson cloud pool"));
    u.spare_ccap = ccap;
  }
  if (be)
    hipLaunchKernelGGL((k_uj_cmp_copy<true, URec>), dim3((u32)((be + kTileOut - 1) / kTileOut)), dim3(kThreads), 0,
                       eng->stream, u.meta, nk, eo, u.epool, u.spare_e, u.lcol, u.lpe, u.R);
  if (bc)
    hipLaunchKernelGGL((k_uj_cmp_copy<false, u64>), dim3((u32)((bc + kTileOut - 1) / kTileOut)), dim3(kThreads), 0,
                       eng->stream, u.meta, nk, co, u.cpool, u.spare_c, u.lcol, u.lpc, u.R);
  JY_HIP(eng, hipGetLastError());
  if (nk) LAUNCH(k_uj_cmp_meta, nk, u.meta, nk, eo, co);
  const int r = (int)(u.seq % UjsonState::kRing);
  hipLaunchKernelGGL(k_uj_cmp_ctr, dim3(1), dim3(1), 0, eng->stream, eo + nk, co + nk, u.ctr, u.pin_dev + 8 + 2 * r,
                     u.pin_dev + 24 + 3 * r);
  JY_HIP(eng, hipGetLastError());
  std::swap(u.epool, u.spare_e);
  std::swap(u.epcap, u.spare_ecap);
  std::swap(u.cpool, u.spare_c);
  std::swap(u.cpcap, u.spare_ccap);
  // the long pools are empty now (k_uj_cmp_ctr)
  u.long_used_e = u.long_used_c = u.long_ids = 0;
  // every earlier converge is compacted in; this one's sizes are bounded by be / bc
  u.used_e = u.used_c = 0;
  u.done = u.seq;
  u.ring_e[r] = be;
  u.ring_c[r] = bc;
  JY_HIP(eng, hipEventRecord(u.ready[r], eng->stream));
  u.seq++;
  return JY_OK;
}

// Pool plan of one converge: the worst case (every live element touched,
// every delta item kept) must fit after the bump pointers the host knows --
// exact once the last converge's mapped readback has landed, an upper bound
// before.  Only when it may not fit does the host wait for the GPU; only
// when the pools are really short does it compact.
// the newest finished converge's exact bump pointers (mapped readback)
void ujson_absorb(UjsonState& u) {
  for (u64 j = u.seq; j > u.done; j--) {
    const int r = (int)((j - 1) % UjsonState::kRing);
    if (hipEventQuery(u.ready[r]) == hipSuccess) {
      u.used_e = u.pin[8 + 2 * r];
      u.used_c = u.pin[9 + 2 * r];
      u.pred_ta = u.pin[2 * r];
      u.pred_tc = u.pin[1 + 2 * r];
      u.long_used_e = u.pin[24 + 3 * r];
      u.long_used_c = u.pin[25 + 3 * r];
      u.long_ids = u.pin[26 + 3 * r];
      u.has_pred = true;
      u.done = j;
      return;
    }
  }
}
// (we / wc: the converge's worst case -- with long documents it includes a
// demotion of every live entry; room_e / room_c: one converge's worst case
// without it, which sizes a compaction's headroom)
int32_t ujson_plan(jy_engine* eng, UjsonState& u, u64 we, u64 wc, u64 room_e, u64 room_c) {
  ujson_absorb(u);
  if (u.seq - u.done == UjsonState::kRing) {  // the ring slot is still in use: wait for its converge
    JY_HIP(eng, hipEventSynchronize(u.ready[u.done % UjsonState::kRing]));
    ujson_absorb(u);
  }
  // the long pools or ids past half used (by the newest readback, which lags
  // the converges in flight): they double, contents kept.  Until then the
  // device refuses what does not fit -- a promotion is skipped, a document
  // whose run cannot grow goes the regular path -- so nothing overflows.
  if (u.lcol) JY_TRY(ujson_long_grow(eng, u));
  auto fits = [&]() {
    u64 be = u.used_e + we, bc = u.used_c + wc;
    for (u64 j = u.done; j < u.seq; j++) {
      be += u.ring_e[j % UjsonState::kRing];
      bc += u.ring_c[j % UjsonState::kRing];
    }
    return be <= u.epcap && bc <= u.cpcap;
  };
  if (!fits()) {
    if (u.seq > u.done) {
      JY_HIP(eng, hipEventSynchronize(u.ready[(u.seq - 1) % UjsonState::kRing]));
      ujson_absorb(u);
    }
    if (!fits()) JY_TRY(ujson_compact(eng, u, room_e, room_c));
  }
  return JY_OK;
}

// a zeroed device buffer that only grows (contents kept when `keep`)
int32_t grow_zero(jy_engine* eng, void** p, u64* cap_bytes, u64 need_bytes) {
  if (need_bytes <= *cap_bytes && *p) return JY_OK;
  const u64 nb = std::max<u64>(need_bytes, *cap_bytes * 2);
  JY_TRY(jy_realloc(eng, p, *cap_bytes, nb, true));
  *cap_bytes = nb;
  return JY_OK;
}

// the long layout's tables and pools, at first use: ids 4096, pools 1M
// entries each; a compaction doubles what was more than half used
int32_t ujson_long_init(jy_engine* eng, UjsonState& u) {
  u.lcap = 4096;
  u.lpe_cap = u.lpc_cap = 1ull << 20;
  JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.lcol), u.lcap * u.R * sizeof(LCol), "ujson long columns"));
  JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.lplan), u.lcap * u.R * sizeof(LPlan), "ujson long plans"));
  JY_HIP(eng, hipMemsetAsync(u.lplan, 0, u.lcap * u.R * sizeof(LPlan), eng->stream));
  JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.lpe), u.lpe_cap * sizeof(URec), "ujson long element pool"));
  JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.lpc), u.lpc_cap * 8, "ujson long cloud pool"));
  return JY_OK;
}

// The long pools hold every long document's runs with room (2n + 16 a run)
// plus the runs regrowth left behind, so they are sized from the store's
// live-entry bound (4x: HBM is plentiful, a refused regrowth demotes a hot
// document) and from the newest readback (more than half used: double).
// Growth keeps the contents (a stream-ordered copy).
int32_t ujson_long_grow(jy_engine* eng, UjsonState& u) {
  const u64 te = std::max<u64>(4 * u.live_e, 2 * u.long_used_e), tc = std::max<u64>(4 * u.live_c, 2 * u.long_used_c);
  if (te > u.lpe_cap) {
    const u64 nc = std::max<u64>(te, 2 * u.lpe_cap);
    void* q = u.lpe;
    JY_TRY(jy_realloc(eng, &q, u.lpe_cap * sizeof(URec), nc * sizeof(URec), false));
    u.lpe = static_cast<URec*>(q);
    u.lpe_cap = nc;
  }
  if (tc > u.lpc_cap) {
    const u64 nc = std::max<u64>(tc, 2 * u.lpc_cap);
    void* q = u.lpc;
    JY_TRY(jy_realloc(eng, &q, u.lpc_cap * 8, nc * 8, false));
    u.lpc = static_cast<u64*>(q);
    u.lpc_cap = nc;
  }
  if (2 * u.long_ids > u.lcap) {
    void* q = u.lcol;
    JY_TRY(jy_realloc(eng, &q, u.lcap * u.R * sizeof(LCol), 2 * u.lcap * u.R * sizeof(LCol), false));
    u.lcol = static_cast<LCol*>(q);
    q = u.lplan;
    JY_TRY(jy_realloc(eng, &q, u.lcap * u.R * sizeof(LPlan), 2 * u.lcap * u.R * sizeof(LPlan), true));
    u.lplan = static_cast<LPlan*>(q);
    u.lcap *= 2;
  }
  return JY_OK;
}

}  // namespace

int32_t ujson_grow_store(jy_engine* eng, UjsonState& u, u64 need, u64 init_cap) {
  if (u.R == 0) u.R = eng->cfg.ujson_columns;
  if (!u.ctr) {
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.ctr), 64, "ujson counters"));
    JY_HIP(eng, hipMemsetAsync(u.ctr, 0, 64, eng->stream));
    JY_HIP(eng, hipHostMalloc(reinterpret_cast<void**>(&u.pin), 512, hipHostMallocMapped));
    std::memset(u.pin, 0, 512);
    JY_HIP(eng, hipHostGetDevicePointer(reinterpret_cast<void**>(&u.pin_dev), u.pin, 0));
    for (hipEvent_t& e : u.ready) JY_HIP(eng, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.tick), 64, "ujson tickets"));
    JY_HIP(eng, hipMemsetAsync(u.tick, 0, 64, eng->stream));
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.stats), 128, "ujson stats"));
    JY_HIP(eng, hipMemsetAsync(u.stats, 0, 128, eng->stream));
    u.epcap = u.cpcap = std::max<u64>(init_cap, 1024);
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.epool), u.epcap * sizeof(URec), "ujson element pool"));
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.cpool), u.cpcap * 8, "ujson cloud pool"));
  }
  if (need <= u.kcap && u.vv) return JY_OK;
  u64 nk = std::max<u64>(need, u.kcap ? u.kcap * 2 : need);
  nk = std::max<u64>((nk + 63) & ~63ull, 64);
  void* v = u.vv;
  JY_TRY(jy_realloc(eng, &v, u.kcap * u.R * 8, nk * u.R * 8, true));
  u.vv = static_cast<u64*>(v);
  void* m = u.meta;
  JY_TRY(jy_realloc(eng, &m, u.kcap * sizeof(UMeta), nk * sizeof(UMeta), true));  // empty docs
  u.meta = static_cast<UMeta*>(m);
  void* d = u.dptr;
  JY_TRY(jy_realloc(eng, &d, u.kcap * 8, nk * 8, true));  // epoch 0: never claimed
  u.dptr = static_cast<u64*>(d);
  u.kcap = nk;
  return JY_OK;
}

// default promotion threshold of the state store (JY_UJ_LONG_MIN overrides;
// 0 disables the in-place layout); jy_ujson_set_inplace changes it
u32 ujson_default_long_min() {
  if (const char* e = getenv("JY_UJ_LONG_MIN")) return (u32)strtoul(e, nullptr, 10);
  // (config 5, ms per converge at --warmup 2 / 6 / 20, one box: 128 ->
  // 0.50 / 0.55 / 0.65, 512 -> 0.47 / 0.50 / 0.55; 32: 0.81 at warmup 6 --
  // every promotion is a pass over its document, so only hot ones pay back)
  return 512;
}

int32_t jy_ujson_grow(jy_engine* eng, u64 need) {
  if (!eng->ujson.allow_long) {  // (jy_ujson_set_inplace before the first UJSON key keeps its choice)
    eng->ujson.allow_long = true;
    eng->ujson.long_min = ujson_default_long_min();
  }
  JY_TRY(ujson_grow_store(eng, eng->ujson, need, eng->cfg.entry_capacity[JY_UJSON]));
  if (eng->ujson_d.ctr) JY_TRY(ujson_grow_store(eng, eng->ujson_d, eng->ujson.kcap, 0));
  return JY_OK;
}

// new documents are empty: their meta is zeroed when it is allocated
int32_t jy_ujson_extend(jy_engine*, u64, u64) { return JY_OK; }

int32_t jy_ujson_merge(jy_engine* eng, u64 nd, const u32* slot, const u64* deoff, u64 nel, const u64* ddots,
                       const u64* delems, const u64* dvoff, u64 nvv, const u64* dvv, const u64* dcoff, u64 ncloud,
                       const u64* dcloud) {
  JyTimed tm(eng);
  return jy_ujson_merge_into(eng, eng->ujson, nd, slot, deoff, nel, ddots, delems, dvoff, nvv, dvv, dcoff, ncloud,
                             dcloud);
}

// the converge into one store: the state, or the pending deltas of the write path
int32_t jy_ujson_merge_into(jy_engine* eng, UjsonState& u, u64 nd, const u32* slot, const u64* deoff, u64 nel,
                            const u64* ddots, const u64* delems, const u64* dvoff, u64 nvv, const u64* dvv,
                            const u64* dcoff, u64 ncloud, const u64* dcloud, bool keep_all) {
  const u64 nk = eng->nkeys[JY_UJSON];
  if (nd == 0 || nk == 0) return JY_OK;
  if (nd >= 0xFFFFFFFFull) return eng->fail(JY_ERANGE, "ujson converge: more than 2^32 - 1 documents in one call");
  const u32 R = u.R;
  // the in-place layout of long documents: the state store, R <= 64 (a lane per column)
  if (!u.lcol && u.allow_long && u.long_min && !keep_all && R <= (u32)kMaxR) JY_TRY(ujson_long_init(eng, u));
  const bool lng = u.lcol != nullptr;
  const u64 live_e = u.live_e, live_c = u.live_c;  // bounds of the touched state, before this converge
  const double th0 = jy_tracing() ? jy_now_us() : 0;
  // worst case: every live entry touched (and, with long documents, demoted first)
  JY_TRY(ujson_plan(eng, u, (lng ? 2 : 1) * u.live_e + nel, (lng ? 2 : 1) * u.live_c + ncloud, u.live_e + nel,
                    u.live_c + ncloud));
  const double th1 = jy_tracing() ? jy_now_us() : 0;
  const u64 le = std::min(u.live_e, live_e), lc = std::min(u.live_c, live_c);  // (a compaction makes them exact)
  if (le + nel + ncloud + 2 >= (1ull << 32) || lc + ncloud + 2 >= (1ull << 32))
    return eng->fail(JY_ERANGE, "ujson converge: more than 2^32 touched items");

  // persistent per-delta-doc state: bad / in-place / not-append-shaped
  // marks, the dense delta vv (zero), the promotion list, the copy jobs
  if (nd > u.dcap) {
    u64 bcap = u.dcap * 4, vcap = u.dcap * R * 8, fcap = u.dcap * 4, ncap = u.dcap * 4;
    void* bp = u.bad;
    void* v = u.vvd;
    void* f = u.fast;
    void* g = u.nf;
    const u64 dcap = std::max<u64>(nd, 2 * u.dcap);
    JY_TRY(grow_zero(eng, &bp, &bcap, dcap * 4));
    JY_TRY(grow_zero(eng, &v, &vcap, dcap * R * 8));
    JY_TRY(grow_zero(eng, &f, &fcap, dcap * 4));
    JY_TRY(grow_zero(eng, &g, &ncap, dcap * 4));
    u.bad = static_cast<u32*>(bp);
    u.vvd = static_cast<u64*>(v);
    u.fast = static_cast<u32*>(f);
    u.nf = static_cast<u32*>(g);
    u.dcap = dcap;
  }
  if (lng && u.jcap < u.dcap) {  // (contents never kept: a converge's jobs are its own)
    jy_dev_free(eng, u.jobs);
    jy_dev_free(eng, u.plist);
    jy_dev_free(eng, u.flist);
    u.jobs = nullptr;
    u.plist = nullptr;
    u.flist = nullptr;
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.jobs), 3 * u.dcap * sizeof(UJob), "ujson copy jobs"));
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.plist), u.dcap * 4, "ujson promotions"));
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.flist), u.dcap * 4, "ujson docs in place"));
    u.jcap = u.dcap;
  }

  // epoch: tags claims, bad marks and look-back words (no per-converge reset)
  u.epoch++;
  if ((u.epoch & ((1u << jyscan::kEpochBits) - 1)) == 0 || u.epoch == 0) {
    // wrap: clear everything the tags protect
    u.epoch = 1;
    JY_HIP(eng, hipMemsetAsync(u.dptr, 0, u.kcap * 8, eng->stream));
    if (u.bad) JY_HIP(eng, hipMemsetAsync(u.bad, 0, u.dcap * 4, eng->stream));
    if (u.fast) JY_HIP(eng, hipMemsetAsync(u.fast, 0, u.dcap * 4, eng->stream));
    if (u.nf) JY_HIP(eng, hipMemsetAsync(u.nf, 0, u.dcap * 4, eng->stream));
    if (u.lplan) JY_HIP(eng, hipMemsetAsync(u.lplan, 0, u.lcap * R * sizeof(LPlan), eng->stream));
    for (int i = 0; i < 6; i++)
      if (u.st[i].p)
        JY_HIP(eng, hipMemsetAsync(u.st[i].p, 0, u.st[i].bytes, eng->stream));
    if (u.tmap.p) JY_HIP(eng, hipMemsetAsync(u.tmap.p, 0, u.tmap.bytes, eng->stream));
  }
  const u64 ndt = (nd + kDocTile - 1) / kDocTile;
  const u64 tf = (le + kTile - 1) / kTile + (nel + kTile - 1) / kTile + (ncloud + kTile - 1) / kTile + 2;
  const u64 tk = (lc + kTile - 1) / kTile + (ncloud + kTile - 1) / kTile + 2;
  const u64 st_need[6] = {ndt, ndt, tf, tk, ndt, ndt};
  u64* st[6];
  for (int i = 0; i < 6; i++) {
    JY_TRY(grow_zero(eng, &u.st[i].p, &u.st[i].bytes, st_need[i] * 8));
    st[i] = static_cast<u64*>(u.st[i].p);
  }

  UjArgs A{};
  A.meta = u.meta;
  A.rec = u.epool;
  A.cloud = u.cpool;
  A.vv = u.vv;
  A.epool_out = u.epool;
  A.cpool_out = u.cpool;
  A.ctr = u.ctr;
  const int slot_r = (int)(u.seq % UjsonState::kRing);
  A.pin = u.pin_dev + 8 + 2 * slot_r;
  A.pin_t = u.pin_dev + 2 * slot_r;
  A.pin_l = u.pin_dev + 24 + 3 * slot_r;
  A.R = R;
  A.epoch = u.epoch;
  A.keep_all = keep_all;
  A.dptr = u.dptr;
  A.bad = u.bad;
  A.skipped = reinterpret_cast<unsigned long long*>(eng->skipped_dev);
  A.tick = u.tick;
  A.nd = nd;
  A.nb = nel;
  A.cb = ncloud;
  A.nvv = nvv;
  A.slot = slot;
  A.deoff = deoff;
  A.ddots = ddots;
  A.delems = delems;
  A.dvoff = dvoff;
  A.dvv = dvv;
  A.dcoff = dcoff;
  A.dcloud = dcloud;
  if (lng) {
    A.lcol = u.lcol;
    A.lplan = u.lplan;
    A.lpe = u.lpe;
    A.lpc = u.lpc;
    A.lpe_cap = u.lpe_cap;
    A.lpc_cap = u.lpc_cap;
    A.lcap = u.lcap;
    A.jobs = u.jobs;
    A.jcap = u.jcap;
    A.fast = u.fast;
    A.nf = u.nf;
    A.plist = u.plist;
    A.flist = u.flist;
    A.long_min = keep_all ? 0 : u.long_min;
  }
  void* p;
  JY_TRY(jy_scratch(eng, 18, (nd + 1) * 8 * 6 + 64, &p));
  u64* tb = static_cast<u64*>(p);
  A.abase = tb;
  A.cbs = tb + (nd + 1);
  A.ao = tb + 2 * (nd + 1);
  A.co = tb + 3 * (nd + 1);
  A.neo = tb + 4 * (nd + 1);
  A.nco = tb + 5 * (nd + 1);
  A.base = tb + 6 * (nd + 1);
  JY_TRY(jy_scratch(eng, 10, nvv * 4 + 64, &p));
  A.sidV = static_cast<u32*>(p);
  A.vvd = u.vvd;
  JY_TRY(jy_scratch(eng, 11, (le + nel + ncloud + 2) * 4, &p));
  A.sc = static_cast<u32*>(p);
  JY_TRY(jy_scratch(eng, 14, (lc + ncloud + 2) * 4, &p));
  A.ksc = static_cast<u32*>(p);
  JY_TRY(jy_scratch(eng, 12, (le + nel + ncloud + 2) * 4, &p));
  A.xr = static_cast<u32*>(p);
  JY_TRY(jy_scratch(eng, 13, (lc + ncloud + 2) * 4, &p));
  A.kr = static_cast<u32*>(p);
  JY_TRY(jy_scratch(eng, 19, (le + nel + lc + ncloud + 4) * 4, &p));
  A.sidA = static_cast<u32*>(p);
  A.sidB = A.sidA + le + 1;
  A.sidC = A.sidB + nel + 1;
  A.sidD = A.sidC + lc + 1;
  {
    const u64 nA = cdiv_h(le) + 1, nB = cdiv_h(nel) + 1, nC = cdiv_h(lc) + 1, nD = cdiv_h(ncloud) + 1;
    JY_TRY(grow_zero(eng, &u.tmap.p, &u.tmap.bytes, (nA + nB + nC + nD) * 8));
    A.tmA = static_cast<u64*>(u.tmap.p);
    A.tmB = A.tmA + nA;
    A.tmC = A.tmB + nB;
    A.tmD = A.tmC + nC;
  }
  A.stats = u.stats;
  JY_TRY(jy_scratch(eng, 17, (tf + tk + 2) * 8, &p));
  A.tp = static_cast<u64*>(p);
  A.ktp = A.tp + tf + 1;
  A.st_ao = st[0];
  A.st_co = st[1];
  A.st_ne = st[4];
  A.st_nc = st[5];

  // U1a items (validation, dense vv, the long documents' items), U1b doc
  // tiles (claims, in place / demote, size scans, item docs), the copy jobs
  // of demotions and regrowths, U2 .. U5, then promotions and their copies
  const u64 t_el = (nel + kTile1 - 1) / kTile1, t_cl = (ncloud + kTile1 - 1) / kTile1,
            t_vv = (nvv + kTile1 - 1) / kTile1;
  hipLaunchKernelGGL(k_uj_items, dim3((u32)std::max<u64>(1, t_el + t_cl + t_vv)), dim3(kThreads), 0, eng->stream, A,
                     t_el, t_cl, t_vv);
  hipLaunchKernelGGL(k_uj_docs, dim3((u32)ndt), dim3(kThreads), 0, eng->stream, A, ndt);
  constexpr u32 kJobGrid = 1024;
  if (lng)
    hipLaunchKernelGGL(k_uj_jobs, dim3(kJobGrid), dim3(kThreads), 0, eng->stream, A, u.jobs, u.ctr + 5, 2 * u.jcap);
  // grids from the newest finished converge's touched sizes (+25 %), never above the safe bound
  const u64 pa = u.has_pred ? std::min(le, u.pred_ta + u.pred_ta / 4 + 4096) : le;
  const u64 pc = u.has_pred ? std::min(lc, u.pred_tc + u.pred_tc / 4 + 4096) : lc;
  const u64 gf = cdiv_h(pa) + cdiv_h(nel) + cdiv_h(ncloud) + 2;
  const u64 gk = cdiv_h(pc) + cdiv_h(ncloud) + 2;
  hipLaunchKernelGGL(k_uj_flags, dim3((u32)gf), dim3(kItemThreads), 0, eng->stream, A);
  hipLaunchKernelGGL(k_uj_tscan, dim3(1), dim3(1024), 0, eng->stream, A, 0);
  hipLaunchKernelGGL(k_uj_compact, dim3((u32)gk), dim3(kItemThreads), 0, eng->stream, A);
  hipLaunchKernelGGL(k_uj_tscan, dim3(1), dim3(1024), 0, eng->stream, A, 1);
  hipLaunchKernelGGL(k_uj_sizes, dim3((u32)ndt), dim3(kThreads), 0, eng->stream, A, ndt);
  const u64 g5 = gf + gk + (nvv + kTile - 1) / kTile + (nd + kTile - 1) / kTile + 2;
  hipLaunchKernelGGL(k_uj_scatter, dim3((u32)g5), dim3(kScatterThreads), 0, eng->stream, A);
  if (lng && A.long_min) {
    hipLaunchKernelGGL(k_uj_promote, dim3(256), dim3(kThreads), 0, eng->stream, A);
    hipLaunchKernelGGL(k_uj_jobs, dim3(kJobGrid), dim3(kThreads), 0, eng->stream, A, u.jobs + 2 * u.jcap, u.ctr + 6,
                       u.jcap);
  }
  JY_HIP(eng, hipGetLastError());
  JY_TRACE("ujson merge %llu docs: plan %.1f us, rest of the host side %.1f us", (unsigned long long)nd, th1 - th0,
           jy_now_us() - th1);
#ifdef JY_UJ_PROBE
  if (const char* path = getenv("JY_UJ_PROBE_OUT")) {
    static std::vector<u64> buf(kProbe * 6);
    u32 n = 0;
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
    JY_HIP(eng, hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_probe_n), 4));
    n = std::min(n, kProbe);
    JY_HIP(eng, hipMemcpyFromSymbol(buf.data(), HIP_SYMBOL(g_probe), (size_t)n * 48));
    if (FILE* f = fopen(path, "ab")) {
      const u64 hdr[4] = {~0ull, n, tf, tk};
      fwrite(hdr, 8, 4, f);
      fwrite(buf.data(), 48, n, f);
      fclose(f);
    }
    const u32 zero = 0;
    JY_HIP(eng, hipMemcpyToSymbol(HIP_SYMBOL(g_probe_n), &zero, 4));
  }
#endif
  // the host's pool bounds: the worst case until the mapped readback lands
  u.ring_e[slot_r] = (lng ? 2 : 1) * le + nel;
  u.ring_c[slot_r] = (lng ? 2 : 1) * lc + ncloud;
  u.live_e += nel;
  u.live_c += ncloud;
  JY_HIP(eng, hipEventRecord(u.ready[slot_r], eng->stream));
  u.seq++;
  return JY_OK;
}

int32_t jy_ujson_stats_ext(jy_engine* eng, u64* out16) {
  JY_HIP(eng, hipSetDevice(eng->device));
  UjsonState& u = eng->ujson;
  if (!u.stats) {
    std::memset(out16, 0, 128);
    return JY_OK;
  }
  JY_HIP(eng, hipMemcpyAsync(out16, u.stats, 128, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  return JY_OK;
}

int32_t jy_ujson_set_inplace(jy_engine* eng, uint32_t min_elems) {
  eng->ujson.allow_long = true;
  eng->ujson.long_min = min_elems;
  return JY_OK;
}

int32_t jy_ujson_stats(jy_engine* eng, u64* out8) {
  JY_HIP(eng, hipSetDevice(eng->device));
  UjsonState& u = eng->ujson;
  if (!u.stats) {
    std::memset(out8, 0, 64);
    return JY_OK;
  }
  JY_HIP(eng, hipMemcpyAsync(out8, u.stats, 64, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  return JY_OK;
}

int32_t jy_ujson_sizes(jy_engine* eng, u64 n, const u32* slots, u64* ne, u64* nc) {
  return jy_ujson_sizes_of(eng, eng->ujson, n, slots, ne, nc);
}
int32_t jy_ujson_sizes_of(jy_engine* eng, const UjsonState& u, u64 n, const u32* slots, u64* ne, u64* nc) {
  LAUNCH(k_uj_sizes_read, n, u.meta, slots, n, ne, nc);
  return JY_OK;
}

int32_t jy_ujson_gather(jy_engine* eng, u64 n, const u32* slots, const u64* oeoff, const u64* ocoff, u64 nel, u64 ncl,
                        u64* odots, u64* oelems, u64* ovv, u64* ocloud) {
  return jy_ujson_gather_of(eng, eng->ujson, n, slots, oeoff, ocoff, nel, ncl, odots, oelems, ovv, ocloud);
}
int32_t jy_ujson_gather_of(jy_engine* eng, const UjsonState& u, u64 n, const u32* slots, const u64* oeoff,
                           const u64* ocoff, u64 nel, u64 ncl, u64* odots, u64* oelems, u64* ovv, u64* ocloud) {
  if (nel)
    LAUNCH(k_uj_gather_items<true>, nel, u.meta, u.epool, u.cpool, slots, n, oeoff, nel, odots, oelems, u.lcol,
           u.lpe, u.lpc, u.R);
  if (ncl)
    LAUNCH(k_uj_gather_items<false>, ncl, u.meta, u.epool, u.cpool, slots, n, ocoff, ncl, ocloud, ocloud, u.lcol,
           u.lpe, u.lpc, u.R);
  LAUNCH(k_uj_gather_vv, n * u.R, u.vv, u.R, slots, n, ovv);
  return JY_OK;
}
