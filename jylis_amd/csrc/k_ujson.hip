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
// A converge touches ONLY the documents of its batch.  Their state segments
// form the "touched state": flat index spaces over the delta documents (ao /
// co = exclusive scans of their sizes), merged with the delta by the
// per-element merge path below; every merged document is written as one
// fresh run at the pools' bump pointers and its UMeta repointed.  Untouched
// documents are never read or moved (the Zipf config-5 stream touches ~17 %
// of them).  The host reads the touched sizes and the bump pointers back once
// per converge (they size the launches); when a pool cannot hold the touched
// state plus the delta, every document is first compacted into a new pool.
//
// Parallel shape: ONE THREAD PER ELEMENT / CLOUD DOT, not per document.
// Delta documents follow a Zipf(1.1) popularity: the
// hottest document of a batch carries tens of thousands of dots, and a
// thread-per-document join serialises on it (measured: 415 ms for 1M docs).
// Every decision is local to one element given binary searches into the
// other side's sorted segment; output positions come from merge-path ranks:
//   pos(x) = out_off[doc] + #kept own-side before x + #kept other-side < x
// with the kept counts from exclusive scans of keep flags.  Compaction of a
// cloud dot x of column c above the merged vv v: x folds into the vv iff
// seq(x) == v + 1 + |union dots of c in (v, seq(x))|, the union rank being
// two lower_bounds (state side) plus a scan over de-duplicated delta dots.
//
// Launch shape: independent per-item jobs of one phase share ONE launch
// (block-uniform ranges: e.g. state-side scatter, delta-side scatter, both
// cloud scatters and the vv store), and the keep flags of all sides are
// concatenated so one scan serves them (positions only ever use differences
// of scan values inside one side).  A converge is ~20 launches.
//
// Roofline: HBM.  Per touched element: 16 B read + 16 B written (+ 4 B
// flag, 4 B scan, 4 B doc id); per touched cloud dot 8 B read + 8 B written;
// vv rows and metas of delta docs.

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr u32 kNone = 0xFFFFFFFFu;
constexpr u32 kSegBits = 28;  // seg-id encoding (range << 28 | doc)
constexpr u32 kSegMask = (1u << kSegBits) - 1;  // readers strip the range bits

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u32 dcol(u64 d) { return (u32)(d >> JY_DOT_SEQ_BITS); }
__device__ __forceinline__ u64 dseq(u64 d) { return d & JY_DOT_SEQ_MASK; }
__device__ __forceinline__ u64 mkdot(u64 c, u64 q) { return (c << JY_DOT_SEQ_BITS) | q; }

// first index in [lo, hi) with a[i] >= x
__device__ __forceinline__ u64 lower_bound(const u64* __restrict__ a, u64 lo, u64 hi, u64 x) {
  while (lo < hi) {
    const u64 m = (lo + hi) >> 1;
    if (a[m] < x) lo = m + 1;
    else hi = m;
  }
  return lo;
}
__device__ __forceinline__ bool contains(const u64* __restrict__ a, u64 lo, u64 hi, u64 x) {
  const u64 i = lower_bound(a, lo, hi, x);
  return i < hi && a[i] == x;
}
// the same over the dots of element records
__device__ __forceinline__ u64 lower_bound_rec(const URec* __restrict__ a, u64 lo, u64 hi, u64 x) {
  while (lo < hi) {
    const u64 m = (lo + hi) >> 1;
    if (a[m].dot < x) lo = m + 1;
    else hi = m;
  }
  return lo;
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
  const UMeta* meta;
  const URec* rec;    // element pool
  const u64* cloud;   // cloud pool
  u64* vv;
  u32 R;
  // touched state: per delta doc its pool segments and flat offsets
  u64* abase;
  u64* asz;    // [nd + 1]
  u64* ao;     // [nd + 1] exclusive scan of asz
  u64* cbs;
  u64* csz;    // [nd + 1]
  u64* co;     // [nd + 1]
  const u32* aseg;   // [ta] delta doc of each touched state element
  const u32* acseg;  // [tc] delta doc of each touched state cloud dot
  u64 ta, tc;
  // delta batch
  u64 nd, nb, cb, nvv;
  const u32* slot;
  u32* dptr;
  const u64* deoff;
  const u64* ddots;
  const u64* delems;
  const u64* dvoff;
  const u64* dvv;
  const u64* dcoff;
  const u64* dcloud;
  const u32* dseg;   // [nb] delta doc of each delta element
  const u32* dcseg;  // [cb] delta doc of each delta cloud dot
  const u32* vseg;   // [nvv] delta doc of each delta vv entry
  // merge temporaries
  u32* bad;  // [nd] malformed delta or repeated slot: the doc is left untouched
  u64* vvs;  // [nd][R] the state's vv rows as they were before this converge
  u64* vvd;  // [nd][R] the delta's own vv, dense
  u64* vvm;  // [nd][R] max(vv_A, vv_B)
  u64* vvn;  // [nd][R] after compaction
  // keep flags, concatenated [flag_a (ta+1) | flag_b (nb+1) | cflag_b (cb+1)]
  // and their exclusive scan in the same layout
  u32* flag_a;
  u32* flag_b;
  u32* cflag_b;
  const u32* scan_a;
  const u32* scan_b;
  const u32* cscan_b;
  // cloud compaction survivors [keep_ca (tc+1) | keep_cb (cb+1)] + scan
  u32* keep_ca;
  u32* keep_cb;
  const u32* kscan_a;
  const u32* kscan_b;
  unsigned long long* skipped;
};

__device__ __forceinline__ bool in_state_ctx(const UjArgs& A, u32 k, u64 d) {
  if (dseq(d) <= A.vvs[(u64)k * A.R + dcol(d)]) return true;
  return contains(A.cloud, A.cbs[k], A.cbs[k] + A.csz[k], d);
}
__device__ __forceinline__ bool in_delta_ctx(const UjArgs& A, u32 k, u64 d) {
  if (dseq(d) <= A.vvd[(u64)k * A.R + dcol(d)]) return true;
  return contains(A.dcloud, A.dcoff[k], A.dcoff[k + 1], d);
}

// ---- multi-range launches ---------------------------------------------------------
// Up to 6 independent item ranges in one grid; each block belongs to one
// range (block-uniform branch).
struct Ranges {
  u64 n[6];
  u32 b0[7];  // first block of each range; b0[cnt] = grid size
  int cnt;
};

__device__ __forceinline__ int range_of(const Ranges& G, u64& i) {
  const u32 b = blockIdx.x;
  int r = 0;
  while (r + 1 < G.cnt && b >= G.b0[r + 1]) r++;
  i = (u64)(b - G.b0[r]) * kThreads + threadIdx.x;
  return r;
}

// ---- P0: per (doc, column): repeated slots, touched-state sizes, vv rows ----------
// dptr[] and bad[] are cleared before this launch.
__global__ __launch_bounds__(kThreads) void k_uj_prep(UjArgs A) {
  const u64 t = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (t >= A.nd * A.R) return;
  const u64 k = t / A.R;
  const u32 c = (u32)(t - k * A.R);
  const u64 s = A.slot[k];
  // the vv row and the meta are loaded before the claim's atomic round trip
  const u64 v = A.vv[s * A.R + c];
  A.vvs[t] = v;  // k_uj_scatter overwrites vv while it still tests the state context
  A.vvm[t] = v;
  A.vvd[t] = 0;
  if (c == 0) {
    const UMeta m = A.meta[s];
    A.abase[k] = m.ebase;
    A.asz[k] = m.elen;
    A.cbs[k] = m.cbase;
    A.csz[k] = m.clen;
    const u32 prev = atomicCAS(A.dptr + s, kNone, (u32)k);
    if (prev != kNone) {  // one delta per doc per call: both copies are skipped
      A.bad[k] = 1;
      A.bad[prev] = 1;
    }
  }
  if (t == 0) {
    A.asz[A.nd] = 0;
    A.csz[A.nd] = 0;
  }
}

// ---- P1: delta vv scattered dense + validation of vv / dots / cloud ---------------
__device__ __forceinline__ void vv_delta(const UjArgs& A, u64 j) {
  const u32 k = A.vseg[j] & kSegMask;
  const u64 x = A.dvv[j];
  const u32 c = dcol(x);
  if (c >= A.R || (j > A.dvoff[k] && dcol(A.dvv[j - 1]) >= c)) {
    A.bad[k] = 1;
    return;
  }
  A.vvd[(u64)k * A.R + c] = dseq(x);  // columns are unique in a well-formed doc
}
// strictly ascending, col < R, seq >= 1
__device__ __forceinline__ void validate(const UjArgs& A, const u32* seg, const u64* offs, const u64* a, u64 j) {
  const u32 k = seg[j] & kSegMask;
  const u64 x = a[j];
  bool ok = dcol(x) < A.R && dseq(x) >= 1;
  if (j > offs[k] && a[j - 1] >= x) ok = false;
  if (!ok) A.bad[k] = 1;
}
__global__ __launch_bounds__(kThreads) void k_uj_check(UjArgs A, Ranges G) {
  u64 i;
  const int r = range_of(G, i);
  if (i >= G.n[r]) return;
  if (r == 0) vv_delta(A, i);
  else if (r == 1) validate(A, A.dseg, A.deoff, A.ddots, i);
  else validate(A, A.dcseg, A.dcoff, A.dcloud, i);
}

// ---- P2: vv max; a malformed delta doc is counted (once per slot) ------------------
__global__ __launch_bounds__(kThreads) void k_uj_drop_bad(UjArgs A) {
  const u64 t = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (t >= A.nd * A.R) return;
  const u64 a = A.vvm[t], b = A.vvd[t];
  const u64 m = a > b ? a : b;
  A.vvm[t] = m;
  A.vvn[t] = m;
  const u64 k = t / A.R;
  if (t - k * A.R == 0 && A.bad[k] && A.dptr[A.slot[k]] == (u32)k) atomicAdd(A.skipped, 1ull);
}

// ---- P3: keep flags: touched state elements, delta elements, delta cloud dedupe ----
__device__ __forceinline__ void flag_a(const UjArgs& A, u64 i) {
  if (i == A.ta) {
    A.flag_a[i] = 0;
    return;
  }
  const u32 k = A.aseg[i] & kSegMask;
  u32 keep = 0;
  if (!A.bad[k]) {
    const u64 d = A.rec[A.abase[k] + (i - A.ao[k])].dot;
    keep = contains(A.ddots, A.deoff[k], A.deoff[k + 1], d) || !in_delta_ctx(A, k, d);
  }
  A.flag_a[i] = keep;
}
__device__ __forceinline__ void flag_b(const UjArgs& A, u64 j) {
  if (j == A.nb) {
    A.flag_b[j] = 0;
    return;
  }
  const u32 k = A.dseg[j] & kSegMask;
  u32 keep = 0;
  if (!A.bad[k]) {
    const u64 d = A.ddots[j];
    const u64 lo = A.abase[k], hi = lo + A.asz[k];
    const u64 p = lower_bound_rec(A.rec, lo, hi, d);
    keep = !(p < hi && A.rec[p].dot == d) && !in_state_ctx(A, k, d);
  }
  A.flag_b[j] = keep;
}
// delta cloud dots that the state cloud also holds are dropped
__device__ __forceinline__ void cloud_dedupe(const UjArgs& A, u64 j) {
  if (j == A.cb) {
    A.cflag_b[j] = 0;
    return;
  }
  const u32 k = A.dcseg[j] & kSegMask;
  u32 f = 0;
  if (!A.bad[k]) f = !contains(A.cloud, A.cbs[k], A.cbs[k] + A.csz[k], A.dcloud[j]);
  A.cflag_b[j] = f;
}
__global__ __launch_bounds__(kThreads) void k_uj_flags(UjArgs A, Ranges G) {
  u64 i;
  const int r = range_of(G, i);
  if (i >= G.n[r]) return;
  if (r == 0) flag_a(A, i);
  else if (r == 1) flag_b(A, i);
  else cloud_dedupe(A, i);
}

// ---- P4: compaction against the merged vv ------------------------------------------
// union rank of x (column c, seq q) above v: state dots of c in (v, q) plus
// de-duplicated delta dots of c in (v, q)
__device__ __forceinline__ void compact_a(const UjArgs& A, u64 i) {
  if (i == A.tc) {
    A.keep_ca[i] = 0;
    return;
  }
  const u32 k = A.acseg[i] & kSegMask;
  if (A.bad[k]) {
    A.keep_ca[i] = 0;
    return;
  }
  const u64 lo0 = A.cbs[k];
  const u64 pi = lo0 + (i - A.co[k]);
  const u64 x = A.cloud[pi];
  const u32 c = dcol(x);
  const u64 q = dseq(x), v = A.vvm[(u64)k * A.R + c];
  u32 keep = 0;
  if (q > v) {
    const u64 lo = mkdot(c, v + 1);
    const u64 ra = pi - lower_bound(A.cloud, lo0, pi, lo);
    const u64 blo = A.dcoff[k], bhi = A.dcoff[k + 1];
    const u64 b0 = lower_bound(A.dcloud, blo, bhi, lo);
    const u64 b1 = lower_bound(A.dcloud, b0, bhi, x);
    const u64 rb = A.cscan_b[b1] - A.cscan_b[b0];
    if (q == v + 1 + ra + rb) {
      __hip_atomic_fetch_max(&A.vvn[(u64)k * A.R + c], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      keep = 1;
    }
  }
  A.keep_ca[i] = keep;
}
__device__ __forceinline__ void compact_b(const UjArgs& A, u64 j) {
  if (j == A.cb) {
    A.keep_cb[j] = 0;
    return;
  }
  u32 keep = 0;
  if (A.cflag_b[j]) {  // (0 for malformed docs)
    const u32 k = A.dcseg[j] & kSegMask;
    const u64 x = A.dcloud[j];
    const u32 c = dcol(x);
    const u64 q = dseq(x), v = A.vvm[(u64)k * A.R + c];
    if (q > v) {
      const u64 lo = mkdot(c, v + 1);
      const u64 alo = A.cbs[k], ahi = alo + A.csz[k];
      const u64 a0 = lower_bound(A.cloud, alo, ahi, lo);
      const u64 ra = lower_bound(A.cloud, a0, ahi, x) - a0;
      const u64 b0 = lower_bound(A.dcloud, A.dcoff[k], j, lo);
      const u64 rb = A.cscan_b[j] - A.cscan_b[b0];
      if (q == v + 1 + ra + rb) {
        __hip_atomic_fetch_max(&A.vvn[(u64)k * A.R + c], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        keep = 1;
      }
    }
  }
  A.keep_cb[j] = keep;
}
__global__ __launch_bounds__(kThreads) void k_uj_compact(UjArgs A, Ranges G) {
  u64 i;
  const int r = range_of(G, i);
  if (i >= G.n[r]) return;
  if (r == 0) compact_a(A, i);
  else compact_b(A, i);
}

// ---- P5: per delta doc output sizes ------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_uj_sizes_out(UjArgs A, u64* __restrict__ ne, u64* __restrict__ nc) {
  const u64 k = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (k > A.nd) return;
  if (k == A.nd || A.bad[k]) {
    ne[k] = 0;
    nc[k] = 0;
    return;
  }
  ne[k] = (A.scan_a[A.ao[k + 1]] - A.scan_a[A.ao[k]]) + (A.scan_b[A.deoff[k + 1]] - A.scan_b[A.deoff[k]]);
  nc[k] = (A.kscan_a[A.co[k + 1]] - A.kscan_a[A.co[k]]) + (A.kscan_b[A.dcoff[k + 1]] - A.kscan_b[A.dcoff[k]]);
}

// ---- P6: scatter into fresh pool runs (merge-path positions) + vv / meta store -----
struct Out {
  const u64* neo;  // exclusive scans of the per-doc output sizes
  const u64* nco;
  URec* epool;
  u64* cpool;
  UMeta* meta;
  u64 eb0, cb0;  // bump pointers: this converge's runs start here
};

__device__ __forceinline__ void scatter_a(const UjArgs& A, const Out& O, u64 i) {
  if (!A.flag_a[i]) return;
  const u32 k = A.aseg[i] & kSegMask;
  const URec x = load_rec(A.rec + A.abase[k] + (i - A.ao[k]));
  u64 e = x.elem;
  u64 pos = O.neo[k] + (A.scan_a[i] - A.scan_a[A.ao[k]]);
  const u64 lo = A.deoff[k], hi = A.deoff[k + 1];
  const u64 p = lower_bound(A.ddots, lo, hi, x.dot);
  pos += A.scan_b[p] - A.scan_b[lo];
  if (p < hi && A.ddots[p] == x.dot && !in_state_ctx(A, k, x.dot)) e = A.delems[p];
  store_rec(O.epool + O.eb0 + pos, x.dot, e);
}
__device__ __forceinline__ void scatter_b(const UjArgs& A, const Out& O, u64 j) {
  if (!A.flag_b[j]) return;
  const u32 k = A.dseg[j] & kSegMask;
  const u64 d = A.ddots[j];
  const u64 lo = A.abase[k];
  const u64 pa = A.ao[k] + (lower_bound_rec(A.rec, lo, lo + A.asz[k], d) - lo);
  const u64 pos = O.neo[k] + (A.scan_b[j] - A.scan_b[A.deoff[k]]) + (A.scan_a[pa] - A.scan_a[A.ao[k]]);
  store_rec(O.epool + O.eb0 + pos, d, A.delems[j]);
}
__device__ __forceinline__ void cscatter_a(const UjArgs& A, const Out& O, u64 i) {
  if (!A.keep_ca[i]) return;
  const u32 k = A.acseg[i] & kSegMask;
  const u64 x = A.cloud[A.cbs[k] + (i - A.co[k])];
  const u64 lo = A.dcoff[k];
  const u64 pos = O.nco[k] + (A.kscan_a[i] - A.kscan_a[A.co[k]]) +
                  (A.kscan_b[lower_bound(A.dcloud, lo, A.dcoff[k + 1], x)] - A.kscan_b[lo]);
  O.cpool[O.cb0 + pos] = x;
}
__device__ __forceinline__ void cscatter_b(const UjArgs& A, const Out& O, u64 j) {
  if (!A.keep_cb[j]) return;
  const u32 k = A.dcseg[j] & kSegMask;
  const u64 x = A.dcloud[j];
  const u64 lo = A.cbs[k];
  const u64 pa = A.co[k] + (lower_bound(A.cloud, lo, lo + A.csz[k], x) - lo);
  const u64 pos = O.nco[k] + (A.kscan_b[j] - A.kscan_b[A.dcoff[k]]) + (A.kscan_a[pa] - A.kscan_a[A.co[k]]);
  O.cpool[O.cb0 + pos] = x;
}
// merged + compacted vv rows back into the state; column 0 repoints the doc
__device__ __forceinline__ void vv_store(const UjArgs& A, const Out& O, u64 t) {
  const u64 k = t / A.R;
  const u32 c = (u32)(t - k * A.R);
  if (A.bad[k]) return;
  const u64 s = A.slot[k];
  A.vv[s * A.R + c] = A.vvn[t];
  if (c == 0) {
    const u32 ne = (u32)(O.neo[k + 1] - O.neo[k]), nc = (u32)(O.nco[k + 1] - O.nco[k]);
    O.meta[s] = UMeta{O.eb0 + O.neo[k], ne, ne, O.cb0 + O.nco[k], nc, nc};
  }
}
__global__ __launch_bounds__(kThreads) void k_uj_scatter(UjArgs A, Out O, Ranges G) {
  u64 i;
  const int r = range_of(G, i);
  if (i >= G.n[r]) return;
  switch (r) {
    case 0: vv_store(A, O, i); break;
    case 1: scatter_a(A, O, i); break;
    case 2: scatter_b(A, O, i); break;
    case 3: cscatter_a(A, O, i); break;
    default: cscatter_b(A, O, i); break;
  }
}

__global__ void k_uj_bump(u64* __restrict__ ctr, const u64* __restrict__ neo, const u64* __restrict__ nco, u64 nd,
                          u64 eb0, u64 cb0) {
  ctr[0] = eb0 + neo[nd];
  ctr[1] = cb0 + nco[nd];
}

// ---- segment ids of up to 5 CSRs over the same docs, one scan ----------------------
// mark the first item of every non-empty segment with (range << 28 | doc);
// an inclusive max-scan carries it on (each range starts with a mark, and
// marks grow with the range)
struct SegSrc {
  const u64* o[5];
  u64 base[5];  // first item of each range in the concatenation
};
__global__ __launch_bounds__(kThreads) void k_uj_seg_starts(SegSrc S, u64 nseg, u32* __restrict__ out) {
  const u64 k = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (k >= nseg) return;
#pragma unroll
  for (u32 r = 0; r < 5; r++)
    if (S.o[r][k] < S.o[r][k + 1]) out[S.base[r] + S.o[r][k]] = (r << kSegBits) | (u32)k;
}

// The max-scan that carries the marks on, one 4096-item tile per workgroup
// with no inter-tile pass: a tile's carry-in is the segment of its first
// item, found by one binary search over that range's offsets (the last
// document whose segment starts at or before it), so every tile scans alone.
constexpr int kFillPer = 16;
constexpr u64 kFillTile = (u64)kThreads * kFillPer;
__global__ __launch_bounds__(kThreads) void k_uj_seg_fill(SegSrc S, u64 nseg, u32* __restrict__ a, u64 n) {
  typedef hipcub::BlockScan<u32, kThreads> Scan;
  typedef hipcub::BlockLoad<u32, kThreads, kFillPer, hipcub::BLOCK_LOAD_WARP_TRANSPOSE> Load;
  typedef hipcub::BlockStore<u32, kThreads, kFillPer, hipcub::BLOCK_STORE_WARP_TRANSPOSE> Store;
  __shared__ union {
    typename Scan::TempStorage scan;
    typename Load::TempStorage load;
    typename Store::TempStorage store;
  } tmp;
  __shared__ u32 carry;
  const u64 t0 = (u64)blockIdx.x * kFillTile;
  if (threadIdx.x < 64) {
    // 64-ary search by the first wave: each round every lane tests one
    // candidate and a ballot keeps the last one that passes (3 dependent
    // loads for 2^18 documents instead of 18)
    u32 r = 4;
    while (r > 0 && S.base[r] > t0) r--;
    const u64 local = t0 - S.base[r];
    const u64* o = S.o[r];
    const u32 lane = threadIdx.x;
    u64 lo = 0, hi = nseg;  // the last doc k with o[k] <= local lies in [lo, hi]
    while (lo < hi) {
      const u64 step = (hi - lo + 63) / 64;
      const u64 c = lo + (u64)(lane + 1) * step;
      const u64 pass = __ballot(c <= hi && o[c] <= local);  // a prefix of the lanes
      const u64 nlo = lo + (u64)__popcll(pass) * step;
      hi = nlo + step - 1 < hi ? nlo + step - 1 : hi;
      lo = nlo;
    }
    if (lane == 0) carry = (r << kSegBits) | (u32)lo;
  }
  // coalesced tile load, transposed through LDS into a blocked arrangement
  u32 v[kFillPer];
  const int valid = (int)(n - t0 < kFillTile ? n - t0 : kFillTile);
  Load(tmp.load).Load(a + t0, v, valid, 0u);
  __syncthreads();
  Scan(tmp.scan).InclusiveScan(v, v, hipcub::Max());
  __syncthreads();
  const u32 c = carry;
#pragma unroll
  for (int u = 0; u < kFillPer; u++) v[u] = v[u] > c ? v[u] : c;
  Store(tmp.store).Store(a + t0, v, valid);
}

// ---- exclusive scans by tiles (the per-document size pairs, the keep flags) ---------
// reduce-then-scan: k_tile_sums sums each 4096-item tile of every array;
// k_tile_scan adds up the sums of the tiles before its own (a few hundred at
// most for these batches) and scans its tile.  Two launches for up to two
// arrays, against two rocprim launches per array.
template <typename T>
struct ScanJob {
  const T* in[2];
  T* out[2];
};
template <typename T, int NA>
__global__ __launch_bounds__(kThreads) void k_tile_sums(ScanJob<T> J, u64 n, T* __restrict__ sums) {
  typedef hipcub::BlockReduce<T, kThreads> Red;
  __shared__ typename Red::TempStorage tmp;
  const u64 t0 = (u64)blockIdx.x * kFillTile;
#pragma unroll
  for (int x = 0; x < NA; x++) {
    T acc = 0;
#pragma unroll 4
    for (u64 i = t0 + threadIdx.x; i < t0 + kFillTile && i < n; i += kThreads) acc += J.in[x][i];
    acc = Red(tmp).Sum(acc);
    if (threadIdx.x == 0) sums[(u64)NA * blockIdx.x + x] = acc;
    __syncthreads();
  }
}
template <typename T, int NA>
__global__ __launch_bounds__(kThreads) void k_tile_scan(ScanJob<T> J, u64 n, const T* __restrict__ sums) {
  typedef hipcub::BlockReduce<T, kThreads> Red;
  typedef hipcub::BlockScan<T, kThreads> Scan;
  typedef hipcub::BlockLoad<T, kThreads, kFillPer, hipcub::BLOCK_LOAD_WARP_TRANSPOSE> Load;
  typedef hipcub::BlockStore<T, kThreads, kFillPer, hipcub::BLOCK_STORE_WARP_TRANSPOSE> Store;
  __shared__ union {
    typename Red::TempStorage red;
    typename Scan::TempStorage scan;
    typename Load::TempStorage load;
    typename Store::TempStorage store;
  } tmp;
  __shared__ T carry;
  const u64 t0 = (u64)blockIdx.x * kFillTile;
  const int valid = (int)(n - t0 < kFillTile ? n - t0 : kFillTile);
#pragma unroll
  for (int x = 0; x < NA; x++) {
    T c = 0;
    for (u32 j = threadIdx.x; j < blockIdx.x; j += kThreads) c += sums[(u64)NA * j + x];
    c = Red(tmp.red).Sum(c);
    if (threadIdx.x == 0) carry = c;
    __syncthreads();
    c = carry;
    T v[kFillPer];
    Load(tmp.load).Load(J.in[x] + t0, v, valid, (T)0);
    __syncthreads();
    Scan(tmp.scan).ExclusiveSum(v, v);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kFillPer; u++) v[u] += c;
    Store(tmp.store).Store(J.out[x] + t0, v, valid);
    __syncthreads();
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
template <bool kElems, typename T>
__global__ __launch_bounds__(kThreads) void k_uj_cmp_copy(const UMeta* __restrict__ meta, u64 nk,
                                                          const u64* __restrict__ off, const T* __restrict__ src,
                                                          T* __restrict__ dst) {
  const u64 total = off[nk];
  const u64 t0 = (u64)blockIdx.x * kTileOut;
  if (t0 >= total) return;
  const u64 t1 = t0 + kTileOut < total ? t0 + kTileOut : total;
  for (u64 t = t0 + threadIdx.x; t < t1; t += kThreads) {
    u64 lo = 0, hi = nk;  // last slot with off <= t
    while (lo < hi) {
      const u64 m = (lo + hi + 1) >> 1;
      if (off[m] <= t) lo = m;
      else hi = m - 1;
    }
    const UMeta m = meta[lo];
    dst[t] = src[(kElems ? m.ebase : m.cbase) + (t - off[lo])];
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
__global__ __launch_bounds__(kThreads) void k_uj_sizes(const UMeta* __restrict__ meta, const u32* __restrict__ slots,
                                                       u64 n, u64* __restrict__ ne, u64* __restrict__ nc) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const UMeta m = meta[slots[i]];
  ne[i] = m.elen;
  nc[i] = m.clen;
}

__global__ __launch_bounds__(kThreads) void k_uj_gather(const UMeta* __restrict__ meta, const URec* __restrict__ rec,
                                                        const u64* __restrict__ cloud, const u64* __restrict__ vv,
                                                        u32 R, const u32* __restrict__ slots, u64 n,
                                                        const u64* __restrict__ oeoff, const u64* __restrict__ ocoff,
                                                        u64* __restrict__ odots, u64* __restrict__ oelems,
                                                        u64* __restrict__ ovv, u64* __restrict__ ocloud) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u64 s = slots[i];
  const UMeta m = meta[s];
  u64 o = oeoff[i];
  for (u64 j = 0; j < m.elen; j++, o++) {
    odots[o] = rec[m.ebase + j].dot;
    oelems[o] = rec[m.ebase + j].elem;
  }
  o = ocoff[i];
  for (u64 j = 0; j < m.clen; j++, o++) ocloud[o] = cloud[m.cbase + j];
  for (u32 c = 0; c < R; c++) ovv[i * R + c] = vv[s * R + c];
}

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

#define LAUNCH(k, n, ...)                                                                          \
  do {                                                                                             \
    hipLaunchKernelGGL(k, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, __VA_ARGS__);     \
    JY_HIP(eng, hipGetLastError());                                                                \
  } while (0)

// rewrite every document back to back into new pools with `room_e` / `room_c`
// free entries after them; synchronises (the new sizes are read back)
// exclusive scans of n items of one or two arrays (in -> out, not in place)
template <typename T, int NA>
static int32_t uj_tile_scan(jy_engine* eng, ScanJob<T> J, u64 n) {
  if (n == 0) return JY_OK;
  const u32 tiles = (u32)((n + kFillTile - 1) / kFillTile);
  void* p;
  JY_TRY(jy_scratch(eng, 19, (u64)tiles * NA * sizeof(T), &p));
  T* sums = static_cast<T*>(p);
  hipLaunchKernelGGL((k_tile_sums<T, NA>), dim3(tiles), dim3(kThreads), 0, eng->stream, J, n, sums);
  hipLaunchKernelGGL((k_tile_scan<T, NA>), dim3(tiles), dim3(kThreads), 0, eng->stream, J, n, (const T*)sums);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}
// a[0..n] -> oa and b[0..n] -> ob (oa[n], ob[n] = the totals)
static int32_t uj_scan2(jy_engine* eng, const u64* a, u64* oa, const u64* b, u64* ob, u64 n) {
  return uj_tile_scan<u64, 2>(eng, ScanJob<u64>{{a, b}, {oa, ob}}, n + 1);
}

int32_t ujson_compact(jy_engine* eng, u64 room_e, u64 room_c) {
  UjsonState& u = eng->ujson;
  const u64 nk = eng->nkeys[JY_UJSON];
  void* p;
  JY_TRY(jy_scratch(eng, 20, (nk + 1) * 32, &p));
  u64* se = static_cast<u64*>(p);
  u64* sc = se + nk + 1;
  u64* eo = sc + nk + 1;
  u64* co = eo + nk + 1;
  LAUNCH(k_uj_cmp_size, nk + 1, u.meta, nk, se, sc);
  JY_TRY(jy_scan_u64(eng, se, eo, nk));
  JY_TRY(jy_scan_u64(eng, sc, co, nk));
  JY_HIP(eng, hipMemcpyAsync(u.pin, eo + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(u.pin + 1, co + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  const u64 te = u.pin[0], tc = u.pin[1];
  // room for many merges like this one before the next compaction
  const u64 ecap = std::max<u64>({te + 16 * room_e, 3 * te, eng->cfg.entry_capacity[JY_UJSON], 1024});
  const u64 ccap = std::max<u64>({tc + 16 * room_c, 3 * tc, eng->cfg.entry_capacity[JY_UJSON], 1024});
  JY_TRACE("ujson compact: %llu elements, %llu cloud dots -> pools %llu / %llu", (unsigned long long)te,
           (unsigned long long)tc, (unsigned long long)ecap, (unsigned long long)ccap);
  URec* ne = nullptr;
  u64* nc = nullptr;
  JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&ne), ecap * sizeof(URec), "ujson element pool"));
  JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&nc), ccap * 8, "ujson cloud pool"));
  if (te)
    hipLaunchKernelGGL((k_uj_cmp_copy<true, URec>), dim3((u32)((te + kTileOut - 1) / kTileOut)), dim3(kThreads), 0,
                       eng->stream, u.meta, nk, eo, u.epool, ne);
  if (tc)
    hipLaunchKernelGGL((k_uj_cmp_copy<false, u64>), dim3((u32)((tc + kTileOut - 1) / kTileOut)), dim3(kThreads), 0,
                       eng->stream, u.meta, nk, co, u.cpool, nc);
  JY_HIP(eng, hipGetLastError());
  if (nk) LAUNCH(k_uj_cmp_meta, nk, u.meta, nk, eo, co);
  jy_dev_free(eng, u.epool);
  jy_dev_free(eng, u.cpool);
  u.epool = ne;
  u.cpool = nc;
  u.epcap = ecap;
  u.cpcap = ccap;
  u.pin[0] = te;
  u.pin[1] = tc;
  JY_HIP(eng, hipMemcpyAsync(u.ctr, u.pin, 16, hipMemcpyHostToDevice, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));  // pin is reused right away
  return JY_OK;
}

}  // namespace

int32_t jy_ujson_grow(jy_engine* eng, u64 need) {
  UjsonState& u = eng->ujson;
  if (u.R == 0) u.R = eng->cfg.ujson_columns;
  if (!u.ctr) {
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&u.ctr), 64, "ujson counters"));
    JY_HIP(eng, hipMemsetAsync(u.ctr, 0, 64, eng->stream));
    JY_HIP(eng, hipHostMalloc(reinterpret_cast<void**>(&u.pin), 64, hipHostMallocDefault));
    u.epcap = u.cpcap = std::max<u64>(eng->cfg.entry_capacity[JY_UJSON], 1024);
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
  u.kcap = nk;
  return JY_OK;
}

// new documents are empty: their meta is zeroed when it is allocated
int32_t jy_ujson_extend(jy_engine*, u64, u64) { return JY_OK; }

int32_t jy_ujson_merge(jy_engine* eng, u64 nd, const u32* slot, const u64* deoff, u64 nel, const u64* ddots,
                       const u64* delems, const u64* dvoff, u64 nvv, const u64* dvv, const u64* dcoff, u64 ncloud,
                       const u64* dcloud) {
  JyTimed tm(eng);
  UjsonState& u = eng->ujson;
  const u64 nk = eng->nkeys[JY_UJSON];
  if (nd == 0 || nk == 0) return JY_OK;
  if (nd >= (1ull << kSegBits)) return eng->fail(JY_ERANGE, "ujson converge: more than 2^28 documents in one call");
  const u32 R = u.R;

  UjArgs A{};
  A.R = R;
  A.vv = u.vv;
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
  A.skipped = reinterpret_cast<unsigned long long*>(eng->skipped_dev);
  void* p;
  JY_TRY(jy_scratch(eng, 8, nk * 4, &p));
  A.dptr = static_cast<u32*>(p);
  JY_TRY(jy_scratch(eng, 9, nd * 4 + 16, &p));
  A.bad = static_cast<u32*>(p);
  JY_TRY(jy_scratch(eng, 10, nd * R * 32, &p));
  A.vvm = static_cast<u64*>(p);
  A.vvn = A.vvm + nd * R;
  A.vvd = A.vvn + nd * R;
  A.vvs = A.vvd + nd * R;
  JY_TRY(jy_scratch(eng, 18, (nd + 1) * 48, &p));
  u64* tb = static_cast<u64*>(p);
  A.abase = tb;
  A.asz = tb + (nd + 1);
  A.ao = tb + 2 * (nd + 1);
  A.cbs = tb + 3 * (nd + 1);
  A.csz = tb + 4 * (nd + 1);
  A.co = tb + 5 * (nd + 1);

  // touched-state sizes and the bump pointers: the one readback of a converge
  u64 ta = 0, tc = 0, eb0 = 0, cb0 = 0;
  for (int attempt = 0;; attempt++) {
    A.meta = u.meta;
    A.rec = u.epool;
    A.cloud = u.cpool;
    JY_HIP(eng, hipMemsetAsync(A.dptr, 0xFF, nk * 4, eng->stream));
    JY_HIP(eng, hipMemsetAsync(A.bad, 0, nd * 4, eng->stream));
    LAUNCH(k_uj_prep, nd * R, A);
    JY_TRY(uj_scan2(eng, A.asz, A.ao, A.csz, A.co, nd));
    JY_HIP(eng, hipMemcpyAsync(u.pin, A.ao + nd, 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(u.pin + 1, A.co + nd, 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(u.pin + 2, u.ctr, 16, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
    ta = u.pin[0];
    tc = u.pin[1];
    eb0 = u.pin[2];
    cb0 = u.pin[3];
    if (eb0 + ta + nel <= u.epcap && cb0 + tc + ncloud <= u.cpcap) break;
    if (attempt == 1) return eng->fail(JY_ENOMEM, "ujson pools: no room after compaction");
    JY_TRY(ujson_compact(eng, ta + nel, tc + ncloud));  // moves every doc: plan again
  }
  if (ta + nel + 3 >= (1ull << 31) || tc + ncloud + 2 >= (1ull << 31))
    return eng->fail(JY_ERANGE, "ujson converge: more than 2^31 touched elements");
  A.ta = ta;
  A.tc = tc;

  const u64 nf = (ta + 1) + (nel + 1) + (ncloud + 1);
  JY_TRY(jy_scratch(eng, 11, nf * 8, &p));
  A.flag_a = static_cast<u32*>(p);
  A.flag_b = A.flag_a + ta + 1;
  A.cflag_b = A.flag_b + nel + 1;
  A.scan_a = A.flag_a + nf;
  A.scan_b = A.scan_a + ta + 1;
  A.cscan_b = A.scan_b + nel + 1;
  const u64 nkp = (tc + 1) + (ncloud + 1);
  JY_TRY(jy_scratch(eng, 14, nkp * 8, &p));
  A.keep_ca = static_cast<u32*>(p);
  A.keep_cb = A.keep_ca + tc + 1;
  A.kscan_a = A.keep_ca + nkp;
  A.kscan_b = A.kscan_a + tc + 1;
  JY_TRY(jy_scratch(eng, 16, (nd + 1) * 32, &p));
  u64* ne = static_cast<u64*>(p);
  u64* nc = ne + nd + 1;
  u64* neo = nc + nd + 1;
  u64* nco = neo + nd + 1;
  // segment ids of delta elements, cloud dots, vv entries and the touched
  // state's elements and cloud dots: one buffer, one scan
  const u64 nsg = nel + ncloud + nvv + ta + tc;
  JY_TRY(jy_scratch(eng, 17, std::max<u64>(nsg, 1) * 4, &p));
  u32* sg = static_cast<u32*>(p);
  A.dseg = sg;
  A.dcseg = sg + nel;
  A.vseg = sg + nel + ncloud;
  A.aseg = sg + nel + ncloud + nvv;
  A.acseg = sg + nel + ncloud + nvv + ta;

  auto ranges = [](std::initializer_list<u64> ns) {
    Ranges G{};
    G.cnt = 0;
    u32 b = 0;
    for (u64 n : ns) {
      G.n[G.cnt] = n;
      G.b0[G.cnt] = b;
      b += (u32)((n + kThreads - 1) / kThreads);
      G.cnt++;
    }
    G.b0[G.cnt] = b;
    return G;
  };
  auto launch_ranges = [&](auto kern, const Ranges& G, auto... args) -> int32_t {
    if (G.b0[G.cnt] == 0) return JY_OK;
    hipLaunchKernelGGL(kern, dim3(G.b0[G.cnt]), dim3(kThreads), 0, eng->stream, args..., G);
    JY_HIP(eng, hipGetLastError());
    return JY_OK;
  };

  if (nsg) {
    SegSrc S{{deoff, dcoff, dvoff, A.ao, A.co}, {0, nel, nel + ncloud, nel + ncloud + nvv, nel + ncloud + nvv + ta}};
    JY_HIP(eng, hipMemsetAsync(sg, 0, nsg * 4, eng->stream));
    LAUNCH(k_uj_seg_starts, nd, S, nd, sg);
    hipLaunchKernelGGL(k_uj_seg_fill, dim3((u32)((nsg + kFillTile - 1) / kFillTile)), dim3(kThreads), 0, eng->stream,
                       S, nd, sg, nsg);
    JY_HIP(eng, hipGetLastError());
  }
  JY_TRY(launch_ranges(k_uj_check, ranges({nvv, nel, ncloud}), A));
  LAUNCH(k_uj_drop_bad, nd * R, A);
  JY_TRY(launch_ranges(k_uj_flags, ranges({ta + 1, nel + 1, ncloud + 1}), A));
  JY_TRY((uj_tile_scan<u32, 1>(eng, ScanJob<u32>{{A.flag_a, nullptr}, {A.flag_a + nf, nullptr}}, nf)));
  JY_TRY(launch_ranges(k_uj_compact, ranges({tc + 1, ncloud + 1}), A));
  JY_TRY((uj_tile_scan<u32, 1>(eng, ScanJob<u32>{{A.keep_ca, nullptr}, {A.keep_ca + nkp, nullptr}}, nkp)));
  LAUNCH(k_uj_sizes_out, nd + 1, A, ne, nc);
  JY_TRY(uj_scan2(eng, ne, neo, nc, nco, nd));
  Out O{neo, nco, u.epool, u.cpool, u.meta, eb0, cb0};
  JY_TRY(launch_ranges(k_uj_scatter, ranges({nd * R, ta, nel, tc, ncloud}), A, O));
  hipLaunchKernelGGL(k_uj_bump, dim3(1), dim3(1), 0, eng->stream, u.ctr, neo, nco, nd, eb0, cb0);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_ujson_sizes(jy_engine* eng, u64 n, const u32* slots, u64* ne, u64* nc) {
  UjsonState& u = eng->ujson;
  LAUNCH(k_uj_sizes, n, u.meta, slots, n, ne, nc);
  return JY_OK;
}

int32_t jy_ujson_gather(jy_engine* eng, u64 n, const u32* slots, const u64* oeoff, const u64* ocoff, u64* odots,
                        u64* oelems, u64* ovv, u64* ocloud) {
  UjsonState& u = eng->ujson;
  LAUNCH(k_uj_gather, n, u.meta, u.epool, u.cpool, u.vv, u.R, slots, n, oeoff, ocoff, odots, oelems, ovv, ocloud);
  return JY_OK;
}
