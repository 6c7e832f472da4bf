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
// (dots ascending, elems, slot-of-element); per slot CSR of cloud dots
// ascending (+ slot-of-dot); dense vv [kcap][R].
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
// Roofline: HBM.  Per element: 16 B read + 20 B written (+ flag/scan
// traffic); per cloud dot 8 B read + 12 B written; vv rows of delta docs.

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr u32 kNone = 0xFFFFFFFFu;

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
struct UjArgs {
  // state (current buffers)
  const u64* eoff;
  const u64* dots;
  const u64* elems;
  const u32* eseg;
  const u64* coff;
  const u64* cloud;
  const u32* cseg;
  u64* vv;
  u32 R;
  u64 nkeys, na, ca;  // slots, live elements, live cloud dots
  // delta batch
  u64 nd, nb, cb;
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
  // merge temporaries
  u32* bad;     // [nd]
  u64* vvm;     // [nd][R] max(vv_A, vv_B)
  u64* vvn;     // [nd][R] after compaction
  u64* flag_a;  // [na+1] element keep flags, then their exclusive scan in scan_a
  u64* scan_a;
  u64* flag_b;  // [nb+1]
  u64* scan_b;
  u64* cflag_b;  // [cb+1] delta cloud dot not a duplicate of a state cloud dot
  u64* cscan_b;
  u64* keep_ca;  // [ca+1] state cloud dot survives compaction
  u64* kscan_a;
  u64* keep_cb;  // [cb+1]
  u64* kscan_b;
};

__device__ __forceinline__ u64 delta_vv(const UjArgs& A, u32 k, u32 col) {
  for (u64 j = A.dvoff[k]; j < A.dvoff[k + 1]; j++) {
    const u64 x = A.dvv[j];
    const u32 c = dcol(x);
    if (c == col) return dseq(x);
    if (c > col) break;
  }
  return 0;
}
__device__ __forceinline__ bool in_state_ctx(const UjArgs& A, u64 s, u64 d) {
  if (dseq(d) <= A.vv[s * A.R + dcol(d)]) return true;
  return contains(A.cloud, A.coff[s], A.coff[s + 1], d);
}
__device__ __forceinline__ bool in_delta_ctx(const UjArgs& A, u32 k, u64 d) {
  if (dseq(d) <= delta_vv(A, k, dcol(d))) return true;
  return contains(A.dcloud, A.dcoff[k], A.dcoff[k + 1], d);
}

__device__ __forceinline__ u64 gid() { return (u64)blockIdx.x * kThreads + threadIdx.x; }

// ---- P0: per delta doc scatter; per (doc, column) vv init; per delta vv entry max
__global__ __launch_bounds__(kThreads) void k_uj_prep(UjArgs A) {
  const u64 k = gid();
  if (k >= A.nd) return;
  A.dptr[A.slot[k]] = (u32)k;
  A.bad[k] = 0;
}

__global__ __launch_bounds__(kThreads) void k_uj_vv_init(UjArgs A) {
  const u64 t = gid();
  if (t >= A.nd * A.R) return;
  const u64 k = t / A.R;
  const u32 c = (u32)(t - k * A.R);
  A.vvm[t] = A.vv[(u64)A.slot[k] * A.R + c];
}

// delta vv entries (col << 48 | n), strictly ascending columns per doc
__global__ __launch_bounds__(kThreads) void k_uj_vv_delta(UjArgs A, const u32* __restrict__ vseg, u64 nvv) {
  const u64 j = gid();
  if (j >= nvv) return;
  const u32 k = vseg[j];
  const u64 x = A.dvv[j];
  const u32 c = dcol(x);
  if (c >= A.R || (j > A.dvoff[k] && dcol(A.dvv[j - 1]) >= c)) {
    A.bad[k] = 1;
    return;
  }
  __hip_atomic_fetch_max(&A.vvm[(u64)k * A.R + c], dseq(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- P1: validate delta dots / cloud (strictly ascending, col < R, seq >= 1)
__global__ __launch_bounds__(kThreads) void k_uj_validate(UjArgs A, const u32* __restrict__ seg,
                                                          const u64* __restrict__ offs, const u64* __restrict__ a,
                                                          u64 n) {
  const u64 j = gid();
  if (j >= n) return;
  const u32 k = seg[j];
  const u64 x = a[j];
  bool ok = dcol(x) < A.R && dseq(x) >= 1;
  if (j > offs[k] && a[j - 1] >= x) ok = false;
  if (!ok) A.bad[k] = 1;
}

// ---- P2: a malformed delta doc leaves its key untouched (counted) -------------
__global__ __launch_bounds__(kThreads) void k_uj_drop_bad(UjArgs A, unsigned long long* __restrict__ skipped) {
  const u64 k = gid();
  if (k >= A.nd) return;
  if (A.bad[k]) {
    A.dptr[A.slot[k]] = kNone;
    atomicAdd(skipped, 1ull);
  }
}

// ---- P3: element keep flags ---------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_uj_flag_a(UjArgs A) {
  const u64 i = gid();
  if (i > A.na) return;
  if (i == A.na) {
    A.flag_a[i] = 0;
    return;
  }
  const u64 s = A.eseg[i];
  const u32 k = A.dptr[s];
  u64 keep = 1;
  if (k != kNone) {
    const u64 d = A.dots[i];
    keep = contains(A.ddots, A.deoff[k], A.deoff[k + 1], d) || !in_delta_ctx(A, k, d);
  }
  A.flag_a[i] = keep;
}

__global__ __launch_bounds__(kThreads) void k_uj_flag_b(UjArgs A) {
  const u64 j = gid();
  if (j > A.nb) return;
  if (j == A.nb) {
    A.flag_b[j] = 0;
    return;
  }
  const u32 k = A.dseg[j];
  const u64 s = A.slot[k];
  u64 keep = 0;
  if (A.dptr[s] == k) {
    const u64 d = A.ddots[j];
    keep = !contains(A.dots, A.eoff[s], A.eoff[s + 1], d) && !in_state_ctx(A, s, d);
  }
  A.flag_b[j] = keep;
}

// ---- P5/P11: per-slot output sizes --------------------------------------------
__global__ __launch_bounds__(kThreads) void k_uj_sizes_out(UjArgs A, u64* __restrict__ ne, u64* __restrict__ nc) {
  const u64 s = gid();
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

// ---- P6: element scatter (merge-path positions) -------------------------------
__global__ __launch_bounds__(kThreads) void k_uj_scatter_a(UjArgs A, const u64* __restrict__ neoff,
                                                           u64* __restrict__ odots, u64* __restrict__ oelems,
                                                           u32* __restrict__ oseg) {
  const u64 i = gid();
  if (i >= A.na || !A.flag_a[i]) return;
  const u64 s = A.eseg[i];
  const u32 k = A.dptr[s];
  const u64 d = A.dots[i];
  u64 e = A.elems[i];
  u64 pos = neoff[s] + (A.scan_a[i] - A.scan_a[A.eoff[s]]);
  if (k != kNone) {
    const u64 lo = A.deoff[k], hi = A.deoff[k + 1];
    const u64 p = lower_bound(A.ddots, lo, hi, d);
    pos += A.scan_b[p] - A.scan_b[lo];
    if (p < hi && A.ddots[p] == d && !in_state_ctx(A, s, d)) e = A.delems[p];
  }
  odots[pos] = d;
  oelems[pos] = e;
  oseg[pos] = (u32)s;
}

__global__ __launch_bounds__(kThreads) void k_uj_scatter_b(UjArgs A, const u64* __restrict__ neoff,
                                                           u64* __restrict__ odots, u64* __restrict__ oelems,
                                                           u32* __restrict__ oseg) {
  const u64 j = gid();
  if (j >= A.nb || !A.flag_b[j]) return;
  const u32 k = A.dseg[j];
  const u64 s = A.slot[k];
  const u64 d = A.ddots[j];
  const u64 lo = A.eoff[s];
  const u64 p = lower_bound(A.dots, lo, A.eoff[s + 1], d);
  const u64 pos = neoff[s] + (A.scan_b[j] - A.scan_b[A.deoff[k]]) + (A.scan_a[p] - A.scan_a[lo]);
  odots[pos] = d;
  oelems[pos] = A.delems[j];
  oseg[pos] = (u32)s;
}

// ---- P7: delta cloud dots that the state cloud also holds are dropped ---------
__global__ __launch_bounds__(kThreads) void k_uj_cloud_dedupe(UjArgs A) {
  const u64 j = gid();
  if (j > A.cb) return;
  if (j == A.cb) {
    A.cflag_b[j] = 0;
    return;
  }
  const u32 k = A.dcseg[j];
  const u64 s = A.slot[k];
  u64 f = 0;
  if (A.dptr[s] == k) f = !contains(A.cloud, A.coff[s], A.coff[s + 1], A.dcloud[j]);
  A.cflag_b[j] = f;
}

// ---- P9: compaction against the merged vv --------------------------------------
// union rank of x (column c, seq q) above v: state dots of c in (v, q) plus
// de-duplicated delta dots of c in (v, q)
__global__ __launch_bounds__(kThreads) void k_uj_compact_a(UjArgs A) {
  const u64 i = gid();
  if (i > A.ca) return;
  if (i == A.ca) {
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
  u64 keep = 0;
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

__global__ __launch_bounds__(kThreads) void k_uj_compact_b(UjArgs A) {
  const u64 j = gid();
  if (j > A.cb) return;
  if (j == A.cb) {
    A.keep_cb[j] = 0;
    return;
  }
  u64 keep = 0;
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

// ---- P12: cloud scatter ---------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_uj_cscatter_a(UjArgs A, const u64* __restrict__ ncoff,
                                                            u64* __restrict__ ocloud, u32* __restrict__ oseg) {
  const u64 i = gid();
  if (i >= A.ca || !A.keep_ca[i]) return;
  const u64 s = A.cseg[i];
  const u32 k = A.dptr[s];
  const u64 x = A.cloud[i];
  u64 pos = ncoff[s] + (A.kscan_a[i] - A.kscan_a[A.coff[s]]);
  if (k != kNone) {
    const u64 lo = A.dcoff[k];
    pos += A.kscan_b[lower_bound(A.dcloud, lo, A.dcoff[k + 1], x)] - A.kscan_b[lo];
  }
  ocloud[pos] = x;
  oseg[pos] = (u32)s;
}

__global__ __launch_bounds__(kThreads) void k_uj_cscatter_b(UjArgs A, const u64* __restrict__ ncoff,
                                                            u64* __restrict__ ocloud, u32* __restrict__ oseg) {
  const u64 j = gid();
  if (j >= A.cb || !A.keep_cb[j]) return;
  const u32 k = A.dcseg[j];
  const u64 s = A.slot[k];
  const u64 x = A.dcloud[j];
  const u64 lo = A.coff[s];
  const u64 pos = ncoff[s] + (A.kscan_b[j] - A.kscan_b[A.dcoff[k]]) +
                  (A.kscan_a[lower_bound(A.cloud, lo, A.coff[s + 1], x)] - A.kscan_a[lo]);
  ocloud[pos] = x;
  oseg[pos] = (u32)s;
}

// ---- P13: merged + compacted vv rows back into the state -----------------------
__global__ __launch_bounds__(kThreads) void k_uj_vv_store(UjArgs A) {
  const u64 t = gid();
  if (t >= A.nd * A.R) return;
  const u64 k = t / A.R;
  const u32 c = (u32)(t - k * A.R);
  if (A.bad[k]) return;
  A.vv[(u64)A.slot[k] * A.R + c] = A.vvn[t];
}

__global__ __launch_bounds__(kThreads) void k_fill_tail(u64* __restrict__ off, u64 from, u64 to) {
  const u64 i = from + 1 + gid();
  if (i <= to) off[i] = off[from];
}

__global__ __launch_bounds__(kThreads) void k_uj_sizes(const u64* __restrict__ eoff, const u64* __restrict__ coff,
                                                       const u32* __restrict__ slots, u64 n, u64* __restrict__ ne,
                                                       u64* __restrict__ nc) {
  const u64 i = gid();
  if (i >= n) return;
  const u64 s = slots[i];
  ne[i] = eoff[s + 1] - eoff[s];
  nc[i] = coff[s + 1] - coff[s];
}

__global__ __launch_bounds__(kThreads) void k_uj_gather(const u64* __restrict__ eoff, const u64* __restrict__ dots,
                                                        const u64* __restrict__ elems, const u64* __restrict__ coff,
                                                        const u64* __restrict__ cloud, const u64* __restrict__ vv,
                                                        u32 R, const u32* __restrict__ slots, u64 n,
                                                        const u64* __restrict__ oeoff, const u64* __restrict__ ocoff,
                                                        u64* __restrict__ odots, u64* __restrict__ oelems,
                                                        u64* __restrict__ ovv, u64* __restrict__ ocloud) {
  const u64 i = gid();
  if (i >= n) return;
  const u64 s = slots[i];
  u64 o = oeoff[i];
  for (u64 j = eoff[s]; j < eoff[s + 1]; j++, o++) {
    odots[o] = dots[j];
    oelems[o] = elems[j];
  }
  o = ocoff[i];
  for (u64 j = coff[s]; j < coff[s + 1]; j++, o++) ocloud[o] = cloud[j];
  for (u32 c = 0; c < R; c++) ovv[i * R + c] = vv[s * R + c];
}

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

int32_t realloc_dead(jy_engine* eng, void** p, u64 bytes) {
  // the target buffer's contents are dead (it is rewritten)
  if (*p) {
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
    JY_HIP(eng, hipFree(*p));
    *p = nullptr;
  }
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return eng->fail(JY_ENOMEM, std::string("ujson buffers: ") + hipGetErrorString(e));
  return JY_OK;
}

int32_t ensure_elems(jy_engine* eng, int b, u64 need) {
  UjsonState& u = eng->ujson;
  if (need <= u.ecap[b] && u.dots[b]) return JY_OK;
  const u64 nc = std::max<u64>(std::max<u64>(need + need / 2, eng->cfg.entry_capacity[JY_UJSON]), 1024);
  JY_TRY(realloc_dead(eng, reinterpret_cast<void**>(&u.dots[b]), nc * 8));
  JY_TRY(realloc_dead(eng, reinterpret_cast<void**>(&u.elems[b]), nc * 8));
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
  A.dots = u.dots[c];
  A.elems = u.elems[c];
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
  UjsonState& u = eng->ujson;
  const u64 nk = eng->nkeys[JY_UJSON];
  if (nd == 0 || nk == 0) return JY_OK;
  (void)nvv;
  // exact live sizes of the current buffers (the previous merge's totals)
  JY_HIP(eng, hipEventSynchronize(eng->total_ready));
  const u64 na = u.known ? eng->pin_total[1] : 0;
  const u64 ca = u.known ? eng->pin_total[2] : 0;
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
  A.slot = slot;
  A.deoff = deoff;
  A.ddots = ddots;
  A.delems = delems;
  A.dvoff = dvoff;
  A.dvv = dvv;
  A.dcoff = dcoff;
  A.dcloud = dcloud;
  void* p;
  JY_TRY(jy_scratch(eng, 8, nk * 4, &p));
  A.dptr = static_cast<u32*>(p);
  JY_TRY(jy_scratch(eng, 9, nd * 4, &p));
  A.bad = static_cast<u32*>(p);
  JY_TRY(jy_scratch(eng, 10, nd * R * 16, &p));
  A.vvm = static_cast<u64*>(p);
  A.vvn = A.vvm + nd * R;
  JY_TRY(jy_scratch(eng, 11, (na + 1) * 16, &p));
  A.flag_a = static_cast<u64*>(p);
  A.scan_a = A.flag_a + na + 1;
  JY_TRY(jy_scratch(eng, 12, (nel + 1) * 16, &p));
  A.flag_b = static_cast<u64*>(p);
  A.scan_b = A.flag_b + nel + 1;
  JY_TRY(jy_scratch(eng, 13, (ncloud + 1) * 48, &p));
  A.cflag_b = static_cast<u64*>(p);
  A.cscan_b = A.cflag_b + ncloud + 1;
  A.keep_cb = A.cscan_b + ncloud + 1;
  A.kscan_b = A.keep_cb + ncloud + 1;
  JY_TRY(jy_scratch(eng, 14, (ca + 1) * 16, &p));
  A.keep_ca = static_cast<u64*>(p);
  A.kscan_a = A.keep_ca + ca + 1;
  JY_TRY(jy_scratch(eng, 16, (nk + 1) * 16, &p));
  u64* ne = static_cast<u64*>(p);
  u64* nc = ne + nk + 1;

  JY_TRY(jy_scratch(eng, 17, std::max<u64>(nel, 1) * 4, &p));
  A.dseg = static_cast<const u32*>(p);
  JY_TRY(jy_seg_ids(eng, deoff, nd, nel, static_cast<u32*>(p)));
  JY_TRY(jy_scratch(eng, 18, std::max<u64>(ncloud, 1) * 4, &p));
  A.dcseg = static_cast<const u32*>(p);
  JY_TRY(jy_seg_ids(eng, dcoff, nd, ncloud, static_cast<u32*>(p)));

  JY_TRY(jy_scratch(eng, 19, std::max<u64>(nvv, 1) * 4, &p));
  const u32* vseg = static_cast<const u32*>(p);
  JY_TRY(jy_seg_ids(eng, dvoff, nd, nvv, static_cast<u32*>(p)));

  JY_HIP(eng, hipMemsetAsync(A.dptr, 0xFF, nk * 4, eng->stream));
  LAUNCH(k_uj_prep, nd, A);
  LAUNCH(k_uj_vv_init, nd * R, A);
  if (nvv) LAUNCH(k_uj_vv_delta, nvv, A, vseg, nvv);
  JY_HIP(eng, hipMemcpyAsync(A.vvn, A.vvm, nd * R * 8, hipMemcpyDeviceToDevice, eng->stream));
  if (nel) LAUNCH(k_uj_validate, nel, A, A.dseg, deoff, ddots, nel);
  if (ncloud) LAUNCH(k_uj_validate, ncloud, A, A.dcseg, dcoff, dcloud, ncloud);
  LAUNCH(k_uj_drop_bad, nd, A, reinterpret_cast<unsigned long long*>(eng->skipped_dev));
  // elements
  LAUNCH(k_uj_flag_a, na + 1, A);
  LAUNCH(k_uj_flag_b, nel + 1, A);
  JY_TRY(jy_scan_u64(eng, A.flag_a, A.scan_a, na));
  JY_TRY(jy_scan_u64(eng, A.flag_b, A.scan_b, nel));
  // cloud
  LAUNCH(k_uj_cloud_dedupe, ncloud + 1, A);
  JY_TRY(jy_scan_u64(eng, A.cflag_b, A.cscan_b, ncloud));
  LAUNCH(k_uj_compact_a, ca + 1, A);
  LAUNCH(k_uj_compact_b, ncloud + 1, A);
  JY_TRY(jy_scan_u64(eng, A.keep_ca, A.kscan_a, ca));
  JY_TRY(jy_scan_u64(eng, A.keep_cb, A.kscan_b, ncloud));
  // per-slot sizes -> new offsets
  LAUNCH(k_uj_sizes_out, nk + 1, A, ne, nc);
  JY_TRY(jy_scan_u64(eng, ne, u.eoff[nxt], nk));
  JY_TRY(jy_scan_u64(eng, nc, u.coff[nxt], nk));
  if (na) LAUNCH(k_uj_scatter_a, na, A, u.eoff[nxt], u.dots[nxt], u.elems[nxt], u.eseg[nxt]);
  if (nel) LAUNCH(k_uj_scatter_b, nel, A, u.eoff[nxt], u.dots[nxt], u.elems[nxt], u.eseg[nxt]);
  if (ca) LAUNCH(k_uj_cscatter_a, ca, A, u.coff[nxt], u.cloud[nxt], u.cseg[nxt]);
  if (ncloud) LAUNCH(k_uj_cscatter_b, ncloud, A, u.coff[nxt], u.cloud[nxt], u.cseg[nxt]);
  LAUNCH(k_uj_vv_store, nd * R, A);
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total + 1, u.eoff[nxt] + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total + 2, u.coff[nxt] + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipEventRecord(eng->total_ready, eng->stream));
  u.known = true;
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
  LAUNCH(k_uj_gather, n, u.eoff[c], u.dots[c], u.elems[c], u.coff[c], u.cloud[c], u.vv, u.R, slots, n, oeoff, ocoff,
         odots, oelems, ovv, ocloud);
  return JY_OK;
}
