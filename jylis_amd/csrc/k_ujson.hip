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
// HBM layout per type: dots packed (column << 48 | seq); per slot CSR of
// 16-B element records (dot ascending, elem) + slot-of-element; per slot CSR
// of cloud dots ascending (+ slot-of-dot); dense vv [kcap][R].
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
// Roofline: HBM.  Per element: 16 B read + 20 B written (+ 4 B flag, 4 B
// scan); per cloud dot 8 B read + 12 B written; vv rows of delta docs.

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr u32 kNone = 0xFFFFFFFFu;
constexpr u32 kSegBits = 28;  // seg-id encoding (range << 28 | doc)

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
  // state (current buffers)
  const u64* eoff;
  const URec* rec;
  const u32* eseg;
  const u64* coff;
  const u64* cloud;
  const u32* cseg;
  u64* vv;
  u32 R;
  u64 nkeys, na, ca;  // slots, live elements, live cloud dots
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
  u32* bad;  // [nd]
  u64* vvd;  // [nd][R] the delta's own vv, dense
  u64* vvm;  // [nd][R] max(vv_A, vv_B)
  u64* vvn;  // [nd][R] after compaction
  // keep flags, concatenated [flag_a (na+1) | flag_b (nb+1) | cflag_b (cb+1)]
  // and their exclusive scan in the same layout
  u32* flag_a;
  u32* flag_b;
  u32* cflag_b;
  const u32* scan_a;
  const u32* scan_b;
  const u32* cscan_b;
  // cloud compaction survivors [keep_ca (ca+1) | keep_cb (cb+1)] + scan
  u32* keep_ca;
  u32* keep_cb;
  const u32* kscan_a;
  const u32* kscan_b;
  unsigned long long* skipped;
};

__device__ __forceinline__ bool in_state_ctx(const UjArgs& A, u64 s, u64 d) {
  if (dseq(d) <= A.vv[s * A.R + dcol(d)]) return true;
  return contains(A.cloud, A.coff[s], A.coff[s + 1], d);
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

// ---- P0: per (doc, column): dptr, bad, state vv gather, delta vv cleared ---------
__global__ __launch_bounds__(kThreads) void k_uj_prep(UjArgs A) {
  const u64 t = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (t >= A.nd * A.R) return;
  const u64 k = t / A.R;
  const u32 c = (u32)(t - k * A.R);
  const u64 s = A.slot[k];
  if (c == 0) {
    A.dptr[s] = (u32)k;
    A.bad[k] = 0;
  }
  A.vvm[t] = A.vv[s * A.R + c];
  A.vvd[t] = 0;
}

// ---- P1: delta vv scattered dense + validation of vv / dots / cloud ---------------
__device__ __forceinline__ void vv_delta(const UjArgs& A, u64 j) {
  const u32 k = A.vseg[j];
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
  const u32 k = seg[j];
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

// ---- P2: a malformed delta doc leaves its key untouched (counted); vv max ---------
__global__ __launch_bounds__(kThreads) void k_uj_drop_bad(UjArgs A) {
  const u64 t = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (t >= A.nd * A.R) return;
  const u64 a = A.vvm[t], b = A.vvd[t];
  const u64 m = a > b ? a : b;
  A.vvm[t] = m;
  A.vvn[t] = m;
  const u64 k = t / A.R;
  if (t - k * A.R == 0 && A.bad[k]) {
    A.dptr[A.slot[k]] = kNone;
    atomicAdd(A.skipped, 1ull);
  }
}

// ---- P3: keep flags: state elements, delta elements, delta cloud dedupe ------------
__device__ __forceinline__ void flag_a(const UjArgs& A, u64 i) {
  if (i >= A.eoff[A.nkeys]) {  // A.na is a host bound; eoff[nkeys] is exact
    A.flag_a[i] = 0;
    return;
  }
  const u64 s = A.eseg[i];
  const u32 k = A.dptr[s];
  u32 keep = 1;
  if (k != kNone) {
    const u64 d = A.rec[i].dot;
    keep = contains(A.ddots, A.deoff[k], A.deoff[k + 1], d) || !in_delta_ctx(A, k, d);
  }
  A.flag_a[i] = keep;
}
__device__ __forceinline__ void flag_b(const UjArgs& A, u64 j) {
  if (j == A.nb) {
    A.flag_b[j] = 0;
    return;
  }
  const u32 k = A.dseg[j];
  const u64 s = A.slot[k];
  u32 keep = 0;
  if (A.dptr[s] == k) {
    const u64 d = A.ddots[j];
    const u64 lo = A.eoff[s], hi = A.eoff[s + 1];
    const u64 p = lower_bound_rec(A.rec, lo, hi, d);
    keep = !(p < hi && A.rec[p].dot == d) && !in_state_ctx(A, s, d);
  }
  A.flag_b[j] = keep;
}
// delta cloud dots that the state cloud also holds are dropped
__device__ __forceinline__ void cloud_dedupe(const UjArgs& A, u64 j) {
  if (j == A.cb) {
    A.cflag_b[j] = 0;
    return;
  }
  const u32 k = A.dcseg[j];
  const u64 s = A.slot[k];
  u32 f = 0;
  if (A.dptr[s] == k) f = !contains(A.cloud, A.coff[s], A.coff[s + 1], A.dcloud[j]);
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
  if (i >= A.coff[A.nkeys]) {  // A.ca is a host bound; coff[nkeys] is exact
    A.keep_ca[i] = 0;
    return;
  }
  const u64 s = A.cseg[i];
  const u32 k = A.dptr[s];
  if (k == kNone) {
    A.keep_ca[i] = 1;
    return;
  }
  const u64 x = A.cloud[i];
  const u32 c = dcol(x);
  const u64 q = dseq(x), v = A.vvm[(u64)k * A.R + c];
  u32 keep = 0;
  if (q > v) {
    const u64 lo = mkdot(c, v + 1);
    const u64 ra = i - lower_bound(A.cloud, A.coff[s], i, lo);
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
  if (A.cflag_b[j]) {
    const u32 k = A.dcseg[j];
    const u64 s = A.slot[k];
    const u64 x = A.dcloud[j];
    const u32 c = dcol(x);
    const u64 q = dseq(x), v = A.vvm[(u64)k * A.R + c];
    if (q > v) {
      const u64 lo = mkdot(c, v + 1);
      const u64 alo = A.coff[s], ahi = A.coff[s + 1];
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

// ---- P5: per-slot output sizes ------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_uj_sizes_out(UjArgs A, u64* __restrict__ ne, u64* __restrict__ nc) {
  const u64 s = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (s > A.nkeys) return;
  if (s == A.nkeys) {
    ne[s] = 0;
    nc[s] = 0;
    return;
  }
  const u32 k = A.dptr[s];
  u64 e = A.scan_a[A.eoff[s + 1]] - A.scan_a[A.eoff[s]];
  u64 c = A.kscan_a[A.coff[s + 1]] - A.kscan_a[A.coff[s]];
  if (k != kNone) {
    e += A.scan_b[A.deoff[k + 1]] - A.scan_b[A.deoff[k]];
    c += A.kscan_b[A.dcoff[k + 1]] - A.kscan_b[A.dcoff[k]];
  }
  ne[s] = e;
  nc[s] = c;
}

// ---- P6: scatter (merge-path positions) + vv store + live totals --------------------
struct Out {
  const u64* eoff;  // new offsets
  const u64* coff;
  URec* rec;
  u32* eseg;
  u64* cloud;
  u32* cseg;
  u64* totals;  // [2] live elements, live cloud dots
};

__device__ __forceinline__ void scatter_a(const UjArgs& A, const Out& O, u64 i) {
  if (!A.flag_a[i]) return;
  const u64 s = A.eseg[i];
  const u32 k = A.dptr[s];
  const URec x = load_rec(A.rec + i);
  u64 e = x.elem;
  u64 pos = O.eoff[s] + (A.scan_a[i] - A.scan_a[A.eoff[s]]);
  if (k != kNone) {
    const u64 lo = A.deoff[k], hi = A.deoff[k + 1];
    const u64 p = lower_bound(A.ddots, lo, hi, x.dot);
    pos += A.scan_b[p] - A.scan_b[lo];
    if (p < hi && A.ddots[p] == x.dot && !in_state_ctx(A, s, x.dot)) e = A.delems[p];
  }
  store_rec(O.rec + pos, x.dot, e);
  O.eseg[pos] = (u32)s;
}
__device__ __forceinline__ void scatter_b(const UjArgs& A, const Out& O, u64 j) {
  if (!A.flag_b[j]) return;
  const u32 k = A.dseg[j];
  const u64 s = A.slot[k];
  const u64 d = A.ddots[j];
  const u64 lo = A.eoff[s];
  const u64 p = lower_bound_rec(A.rec, lo, A.eoff[s + 1], d);
  const u64 pos = O.eoff[s] + (A.scan_b[j] - A.scan_b[A.deoff[k]]) + (A.scan_a[p] - A.scan_a[lo]);
  store_rec(O.rec + pos, d, A.delems[j]);
  O.eseg[pos] = (u32)s;
}
__device__ __forceinline__ void cscatter_a(const UjArgs& A, const Out& O, u64 i) {
  if (!A.keep_ca[i]) return;
  const u64 s = A.cseg[i];
  const u32 k = A.dptr[s];
  const u64 x = A.cloud[i];
  u64 pos = O.coff[s] + (A.kscan_a[i] - A.kscan_a[A.coff[s]]);
  if (k != kNone) {
    const u64 lo = A.dcoff[k];
    pos += A.kscan_b[lower_bound(A.dcloud, lo, A.dcoff[k + 1], x)] - A.kscan_b[lo];
  }
  O.cloud[pos] = x;
  O.cseg[pos] = (u32)s;
}
__device__ __forceinline__ void cscatter_b(const UjArgs& A, const Out& O, u64 j) {
  if (!A.keep_cb[j]) return;
  const u32 k = A.dcseg[j];
  const u64 s = A.slot[k];
  const u64 x = A.dcloud[j];
  const u64 lo = A.coff[s];
  const u64 pos = O.coff[s] + (A.kscan_b[j] - A.kscan_b[A.dcoff[k]]) +
                  (A.kscan_a[lower_bound(A.cloud, lo, A.coff[s + 1], x)] - A.kscan_a[lo]);
  O.cloud[pos] = x;
  O.cseg[pos] = (u32)s;
}
// merged + compacted vv rows back into the state; thread 0 publishes totals
__device__ __forceinline__ void vv_store(const UjArgs& A, const Out& O, u64 t) {
  if (t == 0) {
    O.totals[0] = O.eoff[A.nkeys];
    O.totals[1] = O.coff[A.nkeys];
  }
  const u64 k = t / A.R;
  const u32 c = (u32)(t - k * A.R);
  if (A.bad[k]) return;
  A.vv[(u64)A.slot[k] * A.R + c] = A.vvn[t];
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

// ---- segment ids of up to 3 CSRs over the same docs, one scan ----------------------
// mark the first item of every non-empty segment with (range << 28 | doc);
// an inclusive max-scan carries it on (each range starts with a mark, and
// marks grow with the range)
__global__ __launch_bounds__(kThreads) void k_uj_seg_starts(const u64* __restrict__ o0, const u64* __restrict__ o1,
                                                            const u64* __restrict__ o2, u64 nseg, u64 n0, u64 n1,
                                                            u32* __restrict__ out) {
  const u64 k = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (k >= nseg) return;
  if (o0[k] < o0[k + 1]) out[o0[k]] = (u32)k;
  if (o1[k] < o1[k + 1]) out[n0 + o1[k]] = (1u << kSegBits) | (u32)k;
  if (o2[k] < o2[k + 1]) out[n0 + n1 + o2[k]] = (2u << kSegBits) | (u32)k;
}
__global__ __launch_bounds__(kThreads) void k_uj_seg_strip(u32* __restrict__ a, u64 n) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) a[i] &= (1u << kSegBits) - 1;
}

__global__ __launch_bounds__(kThreads) void k_fill_tail(u64* __restrict__ off, u64 from, u64 to) {
  const u64 i = from + 1 + (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i <= to) off[i] = off[from];
}

__global__ __launch_bounds__(kThreads) void k_uj_sizes(const u64* __restrict__ eoff, const u64* __restrict__ coff,
                                                       const u32* __restrict__ slots, u64 n, u64* __restrict__ ne,
                                                       u64* __restrict__ nc) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u64 s = slots[i];
  ne[i] = eoff[s + 1] - eoff[s];
  nc[i] = coff[s + 1] - coff[s];
}

__global__ __launch_bounds__(kThreads) void k_uj_gather(const u64* __restrict__ eoff, const URec* __restrict__ rec,
                                                        const u64* __restrict__ coff,
                                                        const u64* __restrict__ cloud, const u64* __restrict__ vv,
                                                        u32 R, const u32* __restrict__ slots, u64 n,
                                                        const u64* __restrict__ oeoff, const u64* __restrict__ ocoff,
                                                        u64* __restrict__ odots, u64* __restrict__ oelems,
                                                        u64* __restrict__ ovv, u64* __restrict__ ocloud) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u64 s = slots[i];
  u64 o = oeoff[i];
  for (u64 j = eoff[s]; j < eoff[s + 1]; j++, o++) {
    odots[o] = rec[j].dot;
    oelems[o] = rec[j].elem;
  }
  o = ocoff[i];
  for (u64 j = coff[s]; j < coff[s + 1]; j++, o++) ocloud[o] = cloud[j];
  for (u32 c = 0; c < R; c++) ovv[i * R + c] = vv[s * R + c];
}

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

int32_t realloc_dead(jy_engine* eng, void** p, u64 bytes) {
  // the buffer's contents are dead (it is rewritten): stream-ordered free
  JY_TRACE("ujson buffers realloc %llu bytes", (unsigned long long)bytes);
  jy_dev_free(eng, *p);
  *p = nullptr;
  return jy_dev_alloc(eng, p, bytes, "ujson buffers");
}

int32_t ensure_elems(jy_engine* eng, int b, u64 need) {
  UjsonState& u = eng->ujson;
  if (need <= u.ecap[b] && u.rec[b]) return JY_OK;
  const u64 nc = std::max<u64>(std::max<u64>(need + need / 2, eng->cfg.entry_capacity[JY_UJSON]), 1024);
  JY_TRY(realloc_dead(eng, reinterpret_cast<void**>(&u.rec[b]), nc * sizeof(URec)));
  JY_TRY(realloc_dead(eng, reinterpret_cast<void**>(&u.eseg[b]), nc * 4));
  u.ecap[b] = nc;
  return JY_OK;
}

int32_t ensure_cloud(jy_engine* eng, int b, u64 need) {
  UjsonState& u = eng->ujson;
  if (need <= u.ccap[b] && u.cloud[b]) return JY_OK;
  const u64 nc = std::max<u64>(need + need / 2, 1024);
  JY_TRY(realloc_dead(eng, reinterpret_cast<void**>(&u.cloud[b]), nc * 8));
  JY_TRY(realloc_dead(eng, reinterpret_cast<void**>(&u.cseg[b]), nc * 4));
  u.ccap[b] = nc;
  return JY_OK;
}

UjArgs state_args(jy_engine* eng) {
  UjsonState& u = eng->ujson;
  const int c = u.cur;
  UjArgs A{};
  A.eoff = u.eoff[c];
  A.rec = u.rec[c];
  A.eseg = u.eseg[c];
  A.coff = u.coff[c];
  A.cloud = u.cloud[c];
  A.cseg = u.cseg[c];
  A.vv = u.vv;
  A.R = u.R;
  A.nkeys = eng->nkeys[JY_UJSON];
  return A;
}

#define LAUNCH(k, n, ...)                                                                          \
  do {                                                                                             \
    hipLaunchKernelGGL(k, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, __VA_ARGS__);     \
    JY_HIP(eng, hipGetLastError());                                                                \
  } while (0)

}  // namespace

int32_t jy_ujson_grow(jy_engine* eng, u64 need) {
  UjsonState& u = eng->ujson;
  if (need <= u.kcap && u.vv) return JY_OK;
  if (u.R == 0) u.R = eng->cfg.ujson_columns;
  u64 nk = std::max<u64>(need, u.kcap ? u.kcap * 2 : need);
  nk = std::max<u64>((nk + 63) & ~63ull, 64);
  void* v = u.vv;
  JY_TRY(jy_realloc(eng, &v, u.kcap * u.R * 8, nk * u.R * 8, true));
  u.vv = static_cast<u64*>(v);
  for (int b = 0; b < 2; b++) {
    void* e = u.eoff[b];
    JY_TRY(jy_realloc(eng, &e, u.kcap ? (u.kcap + 1) * 8 : 0, (nk + 1) * 8, true));
    u.eoff[b] = static_cast<u64*>(e);
    void* c = u.coff[b];
    JY_TRY(jy_realloc(eng, &c, u.kcap ? (u.kcap + 1) * 8 : 0, (nk + 1) * 8, true));
    u.coff[b] = static_cast<u64*>(c);
    JY_TRY(ensure_elems(eng, b, 1));
    JY_TRY(ensure_cloud(eng, b, 1));
  }
  u.kcap = nk;
  return JY_OK;
}

int32_t jy_ujson_extend(jy_engine* eng, u64 from, u64 to) {
  if (to <= from) return JY_OK;
  UjsonState& u = eng->ujson;
  LAUNCH(k_fill_tail, to - from, u.eoff[u.cur], from, to);
  LAUNCH(k_fill_tail, to - from, u.coff[u.cur], from, to);
  return JY_OK;
}

int32_t jy_ujson_merge(jy_engine* eng, u64 nd, const u32* slot, const u64* deoff, u64 nel, const u64* ddots,
                       const u64* delems, const u64* dvoff, u64 nvv, const u64* dvv, const u64* dcoff, u64 ncloud,
                       const u64* dcloud) {
  JyTimed tm(eng);
  UjsonState& u = eng->ujson;
  const u64 nk = eng->nkeys[JY_UJSON];
  if (nd == 0 || nk == 0) return JY_OK;
  if (nd >= (1ull << kSegBits)) return eng->fail(JY_ERANGE, "ujson converge: more than 2^28 documents in one call");
  // live sizes of the current buffers: exact when the previous merge's
  // totals have landed (non-blocking query), else host upper bounds; the
  // kernels take the exact counts from eoff/coff[nkeys] in HBM, so the host
  // never waits for the GPU here
  const double t_enter = jy_tracing() ? jy_now_us() : 0;
  u64 na = 0, ca = 0;
  if (u.known) {
    const hipError_t q = hipEventQuery(eng->total_ready);
    if (q == hipSuccess) {
      na = eng->pin_total[1];
      ca = eng->pin_total[2];
    } else if (q == hipErrorNotReady) {
      na = u.nel_bound;
      ca = u.ncloud_bound;
    } else {
      JY_HIP(eng, q);
    }
  }
  const double t_synced = jy_tracing() ? jy_now_us() : 0;
  if (na + nel + ncloud + 3 >= (1ull << 31) || ca + ncloud + 2 >= (1ull << 31))
    return eng->fail(JY_ERANGE, "ujson converge: more than 2^31 elements in one shard");
  const int cur = u.cur, nxt = 1 - cur;
  JY_TRY(ensure_elems(eng, nxt, na + nel));
  JY_TRY(ensure_cloud(eng, nxt, ca + ncloud));
  const u32 R = u.R;

  UjArgs A = state_args(eng);
  A.na = na;
  A.ca = ca;
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
  u64* totals_dev = reinterpret_cast<u64*>((reinterpret_cast<uintptr_t>(A.bad + nd) + 7) & ~uintptr_t(7));
  JY_TRY(jy_scratch(eng, 10, nd * R * 24, &p));
  A.vvm = static_cast<u64*>(p);
  A.vvn = A.vvm + nd * R;
  A.vvd = A.vvn + nd * R;
  const u64 nf = (na + 1) + (nel + 1) + (ncloud + 1);
  JY_TRY(jy_scratch(eng, 11, nf * 8, &p));
  A.flag_a = static_cast<u32*>(p);
  A.flag_b = A.flag_a + na + 1;
  A.cflag_b = A.flag_b + nel + 1;
  A.scan_a = A.flag_a + nf;
  A.scan_b = A.scan_a + na + 1;
  A.cscan_b = A.scan_b + nel + 1;
  const u64 nkp = (ca + 1) + (ncloud + 1);
  JY_TRY(jy_scratch(eng, 14, nkp * 8, &p));
  A.keep_ca = static_cast<u32*>(p);
  A.keep_cb = A.keep_ca + ca + 1;
  A.kscan_a = A.keep_ca + nkp;
  A.kscan_b = A.kscan_a + ca + 1;
  JY_TRY(jy_scratch(eng, 16, (nk + 1) * 16, &p));
  u64* ne = static_cast<u64*>(p);
  u64* nc = ne + nk + 1;
  // segment ids of delta elements, cloud dots and vv entries: one buffer
  const u64 nsg = nel + ncloud + nvv;
  JY_TRY(jy_scratch(eng, 17, std::max<u64>(nsg, 1) * 4, &p));
  u32* sg = static_cast<u32*>(p);
  A.dseg = sg;
  A.dcseg = sg + nel;
  A.vseg = sg + nel + ncloud;

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
    JY_HIP(eng, hipMemsetAsync(sg, 0, nsg * 4, eng->stream));
    LAUNCH(k_uj_seg_starts, nd, deoff, dcoff, dvoff, nd, nel, ncloud, sg);
    size_t tmp = 0;
    JY_HIP(eng, hipcub::DeviceScan::InclusiveScan(nullptr, tmp, sg, sg, hipcub::Max(), (int)nsg, eng->stream));
    JY_TRY(jy_scratch(eng, 15, tmp, &p));
    JY_HIP(eng, hipcub::DeviceScan::InclusiveScan(p, tmp, sg, sg, hipcub::Max(), (int)nsg, eng->stream));
    LAUNCH(k_uj_seg_strip, nsg, sg, nsg);
  }
  JY_HIP(eng, hipMemsetAsync(A.dptr, 0xFF, nk * 4, eng->stream));
  LAUNCH(k_uj_prep, nd * R, A);
  JY_TRY(launch_ranges(k_uj_check, ranges({nvv, nel, ncloud}), A));
  LAUNCH(k_uj_drop_bad, nd * R, A);
  JY_TRY(launch_ranges(k_uj_flags, ranges({na + 1, nel + 1, ncloud + 1}), A));
  {
    size_t tmp = 0;
    JY_HIP(eng, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, A.flag_a, A.flag_a + nf, (int)nf, eng->stream));
    JY_TRY(jy_scratch(eng, 15, tmp, &p));
    JY_HIP(eng, hipcub::DeviceScan::ExclusiveSum(p, tmp, A.flag_a, A.flag_a + nf, (int)nf, eng->stream));
  }
  JY_TRY(launch_ranges(k_uj_compact, ranges({ca + 1, ncloud + 1}), A));
  {
    size_t tmp = 0;
    JY_HIP(eng, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, A.keep_ca, A.keep_ca + nkp, (int)nkp, eng->stream));
    JY_TRY(jy_scratch(eng, 15, tmp, &p));
    JY_HIP(eng, hipcub::DeviceScan::ExclusiveSum(p, tmp, A.keep_ca, A.keep_ca + nkp, (int)nkp, eng->stream));
  }
  LAUNCH(k_uj_sizes_out, nk + 1, A, ne, nc);
  JY_TRY(jy_scan_u64(eng, ne, u.eoff[nxt], nk));
  JY_TRY(jy_scan_u64(eng, nc, u.coff[nxt], nk));
  Out O{u.eoff[nxt], u.coff[nxt], u.rec[nxt], u.eseg[nxt], u.cloud[nxt], u.cseg[nxt], totals_dev};
  JY_TRY(launch_ranges(k_uj_scatter, ranges({nd * R, na, nel, ca, ncloud}), A, O));
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total + 1, totals_dev, 16, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipEventRecord(eng->total_ready, eng->stream));
  if (jy_tracing()) JY_TRACE("ujson merge host: wait %.1f us, issue %.1f us", t_synced - t_enter, jy_now_us() - t_synced);
  u.known = true;
  u.nel_bound = na + nel;
  u.ncloud_bound = ca + ncloud;
  u.cur = nxt;
  return JY_OK;
}

int32_t jy_ujson_sizes(jy_engine* eng, u64 n, const u32* slots, u64* ne, u64* nc) {
  UjsonState& u = eng->ujson;
  LAUNCH(k_uj_sizes, n, u.eoff[u.cur], u.coff[u.cur], slots, n, ne, nc);
  return JY_OK;
}

int32_t jy_ujson_gather(jy_engine* eng, u64 n, const u32* slots, const u64* oeoff, const u64* ocoff, u64* odots,
                        u64* oelems, u64* ovv, u64* ocloud) {
  UjsonState& u = eng->ujson;
  const int c = u.cur;
  LAUNCH(k_uj_gather, n, u.eoff[c], u.rec[c], u.coff[c], u.cloud[c], u.vv, u.R, slots, n, oeoff, ocoff,
         odots, oelems, ovv, ocloud);
  return JY_OK;
}
