// k_ujson.hip -- UJSON observed-remove dot-set union and tombstone filter, gfx950.
//
// Semantics (oracle/jy_oracle.cpp UJSON / CausalContext; ujson.md:172-182,
// repo_ujson.pony:65-66): a document is a set of (dot, element) pairs inside
// a causal context (version vector vv + dot cloud).  Join of state A with
// delta B:
//   keep (d, e) of A unless B's context saw d and B's map lacks d
//   add  (d, e) of B whose d A's context has not seen
//   equal dots: B's element replaces A's only if A's context lacks d
//   context := vv max + cloud union, compacted (a cloud dot contiguous with
//              its column's vv is folded into the vv)
// Elements are opaque handles (interned (path, value) leaves); merge never
// reads them.
//
// HBM layout per type: dots packed (column << 48 | seq); per slot CSR of
// (dots ascending, elems); per slot CSR of cloud dots ascending; dense vv
// [kcap][R] (R = jy_config.ujson_columns).  Three passes as TLOG: count,
// scan (elements and cloud), write; the vv row is updated in place.
//
// Roofline: HBM.  Per doc: 16 B per element read (state + delta) and per
// element written, 8 B per cloud dot read / written, 8*R B vv read + write.

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr u32 kNone = 0xFFFFFFFFu;

__device__ __forceinline__ u32 dcol(u64 d) { return (u32)(d >> JY_DOT_SEQ_BITS); }
__device__ __forceinline__ u64 dseq(u64 d) { return d & JY_DOT_SEQ_MASK; }

__device__ __forceinline__ bool bsearch_u64(const u64* __restrict__ a, u64 lo, u64 hi, u64 x) {
  while (lo < hi) {
    const u64 m = (lo + hi) >> 1;
    const u64 v = a[m];
    if (v == x) return true;
    if (v < x) lo = m + 1;
    else hi = m;
  }
  return false;
}

struct UjArgs {
  // state (current buffers)
  const u64* eoff;
  const u64* dots;
  const u64* elems;
  const u64* coff;
  const u64* cloud;
  u64* vv;
  u32 R;
  // delta batch
  const u32* dptr;
  const u64* deoff;
  const u64* ddots;
  const u64* delems;
  const u64* dvoff;
  const u64* dvv;
  const u64* dcoff;
  const u64* dcloud;
  u64 nkeys;
};

struct Doc {  // one resolved (state slot, delta doc) pair
  u64 s, k;
  u64 ea, eae, eb, ebe;  // element ranges
  u64 ca, cae, cb, cbe;  // cloud ranges
  u64 va, vae;           // delta vv range (sparse)
};

__device__ __forceinline__ u64 delta_vv(const UjArgs& A, const Doc& d, u32 col) {
  for (u64 j = d.va; j < d.vae; j++) {
    const u64 x = A.dvv[j];
    const u32 c = dcol(x);
    if (c == col) return dseq(x);
    if (c > col) break;
  }
  return 0;
}
__device__ __forceinline__ bool in_state_ctx(const UjArgs& A, const Doc& d, u64 dot) {
  if (dseq(dot) <= A.vv[d.s * A.R + dcol(dot)]) return true;
  return bsearch_u64(A.cloud, d.ca, d.cae, dot);
}
__device__ __forceinline__ bool in_delta_ctx(const UjArgs& A, const Doc& d, u64 dot) {
  if (dseq(dot) <= delta_vv(A, d, dcol(dot))) return true;
  return bsearch_u64(A.dcloud, d.cb, d.cbe, dot);
}

__device__ __forceinline__ bool strictly_ascending(const u64* __restrict__ a, u64 lo, u64 hi, u32 R, bool seq_pos) {
  for (u64 j = lo; j < hi; j++) {
    const u64 x = a[j];
    if (dcol(x) >= R || (seq_pos && dseq(x) == 0)) return false;
    if (j > lo && a[j - 1] >= x) return false;
  }
  return true;
}
__device__ __forceinline__ bool vv_ascending(const u64* __restrict__ a, u64 lo, u64 hi, u32 R) {
  for (u64 j = lo; j < hi; j++) {
    if (dcol(a[j]) >= R) return false;
    if (j > lo && dcol(a[j - 1]) >= dcol(a[j])) return false;
  }
  return true;
}

// false: copy the slot unchanged (no delta, or a malformed delta -> bad)
__device__ __forceinline__ bool uj_resolve(const UjArgs& A, u64 s, Doc& d, bool& bad) {
  d.s = s;
  d.ea = A.eoff[s];
  d.eae = A.eoff[s + 1];
  d.ca = A.coff[s];
  d.cae = A.coff[s + 1];
  bad = false;
  const u32 k = A.dptr[s];
  if (k == kNone) return false;
  d.k = k;
  d.eb = A.deoff[k];
  d.ebe = A.deoff[k + 1];
  d.cb = A.dcoff[k];
  d.cbe = A.dcoff[k + 1];
  d.va = A.dvoff[k];
  d.vae = A.dvoff[k + 1];
  if (!strictly_ascending(A.ddots, d.eb, d.ebe, A.R, true) || !strictly_ascending(A.dcloud, d.cb, d.cbe, A.R, true) ||
      !vv_ascending(A.dvv, d.va, d.vae, A.R)) {
    bad = true;
    return false;
  }
  return true;
}

// element join; emit(dot, elem) in ascending dot order
template <class Emit>
__device__ __forceinline__ void join_elements(const UjArgs& A, const Doc& d, Emit emit) {
  u64 i = d.ea, j = d.eb;
  while (i < d.eae && j < d.ebe) {
    const u64 a = A.dots[i], b = A.ddots[j];
    if (a == b) {
      emit(a, in_state_ctx(A, d, a) ? A.elems[i] : A.delems[j]);
      i++;
      j++;
    } else if (a < b) {
      if (!in_delta_ctx(A, d, a)) emit(a, A.elems[i]);
      i++;
    } else {
      if (!in_state_ctx(A, d, b)) emit(b, A.delems[j]);
      j++;
    }
  }
  for (; i < d.eae; i++)
    if (!in_delta_ctx(A, d, A.dots[i])) emit(A.dots[i], A.elems[i]);
  for (; j < d.ebe; j++)
    if (!in_state_ctx(A, d, A.ddots[j])) emit(A.ddots[j], A.delems[j]);
}

// context join: union of the clouds (ascending, deduped) compacted against
// the merged version vector.  keep(dot) for surviving cloud dots;
// setvv(col, n) for every column whose vv advanced past max(vvA, vvB).
template <class Keep, class SetVV>
__device__ __forceinline__ void join_context(const UjArgs& A, const Doc& d, Keep keep, SetVV setvv) {
  u64 i = d.ca, j = d.cb;
  u32 col = 0xFFFFFFFFu;
  u64 v = 0, v0 = 0;
  auto visit = [&](u64 x) {
    const u32 c = dcol(x);
    if (c != col) {
      if (col != 0xFFFFFFFFu && v != v0) setvv(col, v);
      col = c;
      const u64 va = A.vv[d.s * A.R + c], vb = delta_vv(A, d, c);
      v = v0 = va > vb ? va : vb;
    }
    const u64 q = dseq(x);
    if (q <= v) return;
    if (q == v + 1) {
      v = q;
      return;
    }
    keep(x);
  };
  while (i < d.cae || j < d.cbe) {
    u64 x;
    if (j >= d.cbe || (i < d.cae && A.cloud[i] < A.dcloud[j])) {
      x = A.cloud[i++];
    } else if (i >= d.cae || A.dcloud[j] < A.cloud[i]) {
      x = A.dcloud[j++];
    } else {
      x = A.cloud[i++];
      j++;
    }
    visit(x);
  }
  if (col != 0xFFFFFFFFu && v != v0) setvv(col, v);
}

__global__ __launch_bounds__(kThreads) void k_scatter_ptr(u32* __restrict__ dptr, const u32* __restrict__ slot, u64 n) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) dptr[slot[i]] = (u32)i;
}

__global__ __launch_bounds__(kThreads) void k_uj_count(UjArgs A, u64* __restrict__ ne, u64* __restrict__ nc,
                                                       unsigned long long* __restrict__ skipped) {
  const u64 s = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (s > A.nkeys) return;
  if (s == A.nkeys) {
    ne[s] = 0;
    nc[s] = 0;
    return;
  }
  Doc d;
  bool bad;
  if (!uj_resolve(A, s, d, bad)) {
    ne[s] = d.eae - d.ea;
    nc[s] = d.cae - d.ca;
    if (bad) atomicAdd(skipped, 1ull);
    return;
  }
  u64 a = 0, b = 0;
  join_elements(A, d, [&](u64, u64) { a++; });
  join_context(A, d, [&](u64) { b++; }, [&](u32, u64) {});
  ne[s] = a;
  nc[s] = b;
}

__global__ __launch_bounds__(kThreads) void k_uj_write(UjArgs A, const u64* __restrict__ neoff,
                                                       const u64* __restrict__ ncoff, u64* __restrict__ odots,
                                                       u64* __restrict__ oelems, u64* __restrict__ ocloud) {
  const u64 s = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (s >= A.nkeys) return;
  Doc d;
  bool bad;
  u64 oe = neoff[s], oc = ncoff[s];
  if (!uj_resolve(A, s, d, bad)) {
    for (u64 j = d.ea; j < d.eae; j++, oe++) {
      odots[oe] = A.dots[j];
      oelems[oe] = A.elems[j];
    }
    for (u64 j = d.ca; j < d.cae; j++, oc++) ocloud[oc] = A.cloud[j];
    return;
  }
  join_elements(A, d, [&](u64 dot, u64 e) {
    odots[oe] = dot;
    oelems[oe] = e;
    oe++;
  });
  // context: the cloud pass reads the state vv, so collect vv advances first
  // and apply them (and the plain max with the delta vv) afterwards
  join_context(A, d, [&](u64 x) { ocloud[oc++] = x; }, [&](u32, u64) {});
  u64* row = A.vv + s * A.R;
  for (u64 j = d.va; j < d.vae; j++) {
    const u64 x = A.dvv[j];
    const u32 c = dcol(x);
    if (dseq(x) > row[c]) row[c] = dseq(x);
  }
  // replay the compaction against the (now max-merged) row: identical walk
  // to join_context with vv = max(vvA, vvB)
  u64 i = d.ca, j = d.cb;
  u32 col = 0xFFFFFFFFu;
  u64 v = 0;
  const u64* cl = A.cloud;
  const u64* dcl = A.dcloud;
  while (i < d.cae || j < d.cbe) {
    u64 x;
    if (j >= d.cbe || (i < d.cae && cl[i] < dcl[j])) {
      x = cl[i++];
    } else if (i >= d.cae || dcl[j] < cl[i]) {
      x = dcl[j++];
    } else {
      x = cl[i++];
      j++;
    }
    const u32 c = dcol(x);
    if (c != col) {
      if (col != 0xFFFFFFFFu) row[col] = v;
      col = c;
      v = row[c];
    }
    if (dseq(x) == v + 1) v = dseq(x);
  }
  if (col != 0xFFFFFFFFu) row[col] = v;
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

__global__ __launch_bounds__(kThreads) void k_uj_gather(UjArgs A, const u32* __restrict__ slots, u64 n,
                                                        const u64* __restrict__ oeoff, const u64* __restrict__ ocoff,
                                                        u64* __restrict__ odots, u64* __restrict__ oelems,
                                                        u64* __restrict__ ovv, u64* __restrict__ ocloud) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u64 s = slots[i];
  u64 o = oeoff[i];
  for (u64 j = A.eoff[s]; j < A.eoff[s + 1]; j++, o++) {
    odots[o] = A.dots[j];
    oelems[o] = A.elems[j];
  }
  o = ocoff[i];
  for (u64 j = A.coff[s]; j < A.coff[s + 1]; j++, o++) ocloud[o] = A.cloud[j];
  for (u32 c = 0; c < A.R; c++) ovv[i * A.R + c] = A.vv[s * A.R + c];
}

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

int32_t ensure_buf(jy_engine* eng, u64** a, u64** b, u64& cap, u64 need, u64 floor) {
  if (need <= cap && *a) return JY_OK;
  u64 nc = std::max<u64>(std::max<u64>(need + need / 2, floor), 1024);
  for (u64** p : {a, b}) {
    if (!p) continue;
    if (*p) {
      JY_HIP(eng, hipStreamSynchronize(eng->stream));
      JY_HIP(eng, hipFree(*p));
      *p = nullptr;
    }
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), nc * 8);
    if (e != hipSuccess) return eng->fail(JY_ENOMEM, std::string("ujson buffers: ") + hipGetErrorString(e));
  }
  cap = nc;
  return JY_OK;
}

UjArgs state_args(jy_engine* eng) {
  UjsonState& u = eng->ujson;
  const int c = u.cur;
  UjArgs A{};
  A.eoff = u.eoff[c];
  A.dots = u.dots[c];
  A.elems = u.elems[c];
  A.coff = u.coff[c];
  A.cloud = u.cloud[c];
  A.vv = u.vv;
  A.R = u.R;
  A.nkeys = eng->nkeys[JY_UJSON];
  return A;
}

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
    JY_TRY(ensure_buf(eng, &u.dots[b], &u.elems[b], u.ecap[b], 1, eng->cfg.entry_capacity[JY_UJSON]));
    JY_TRY(ensure_buf(eng, &u.cloud[b], nullptr, u.ccap[b], 1, 1024));
  }
  u.kcap = nk;
  return JY_OK;
}

int32_t jy_ujson_extend(jy_engine* eng, u64 from, u64 to) {
  if (to <= from) return JY_OK;
  UjsonState& u = eng->ujson;
  hipLaunchKernelGGL(k_fill_tail, dim3(blocks_for(to - from)), dim3(kThreads), 0, eng->stream, u.eoff[u.cur], from,
                     to);
  hipLaunchKernelGGL(k_fill_tail, dim3(blocks_for(to - from)), dim3(kThreads), 0, eng->stream, u.coff[u.cur], from,
                     to);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_ujson_merge(jy_engine* eng, u64 nd, const u32* slot, const u64* deoff, u64 nel, const u64* ddots,
                       const u64* delems, const u64* dvoff, u64 nvv, const u64* dvv, const u64* dcoff, u64 ncloud,
                       const u64* dcloud) {
  UjsonState& u = eng->ujson;
  const u64 nk = eng->nkeys[JY_UJSON];
  if (nd == 0 || nk == 0) return JY_OK;
  (void)nvv;
  JY_HIP(eng, hipEventSynchronize(eng->total_ready));
  const u64 live_e = u.known ? eng->pin_total[1] : u.nel_bound;
  const u64 live_c = u.known ? eng->pin_total[2] : u.ncloud_bound;
  const int cur = u.cur, nxt = 1 - cur;
  JY_TRY(ensure_buf(eng, &u.dots[nxt], &u.elems[nxt], u.ecap[nxt], live_e + nel, eng->cfg.entry_capacity[JY_UJSON]));
  JY_TRY(ensure_buf(eng, &u.cloud[nxt], nullptr, u.ccap[nxt], live_c + ncloud, 1024));

  void *dptr, *ne, *nc;
  JY_TRY(jy_scratch(eng, 8, nk * 4, &dptr));
  JY_TRY(jy_scratch(eng, 9, (nk + 1) * 8, &ne));
  JY_TRY(jy_scratch(eng, 10, (nk + 1) * 8, &nc));
  JY_HIP(eng, hipMemsetAsync(dptr, 0xFF, nk * 4, eng->stream));
  hipLaunchKernelGGL(k_scatter_ptr, dim3(blocks_for(nd)), dim3(kThreads), 0, eng->stream, static_cast<u32*>(dptr),
                     slot, nd);
  UjArgs A = state_args(eng);
  A.dptr = static_cast<const u32*>(dptr);
  A.deoff = deoff;
  A.ddots = ddots;
  A.delems = delems;
  A.dvoff = dvoff;
  A.dvv = dvv;
  A.dcoff = dcoff;
  A.dcloud = dcloud;
  hipLaunchKernelGGL(k_uj_count, dim3(blocks_for(nk + 1)), dim3(kThreads), 0, eng->stream, A,
                     static_cast<u64*>(ne), static_cast<u64*>(nc),
                     reinterpret_cast<unsigned long long*>(eng->skipped_dev));
  JY_HIP(eng, hipGetLastError());
  JY_TRY(jy_scan_u64(eng, static_cast<const u64*>(ne), u.eoff[nxt], nk));
  JY_TRY(jy_scan_u64(eng, static_cast<const u64*>(nc), u.coff[nxt], nk));
  hipLaunchKernelGGL(k_uj_write, dim3(blocks_for(nk)), dim3(kThreads), 0, eng->stream, A, u.eoff[nxt], u.coff[nxt],
                     u.dots[nxt], u.elems[nxt], u.cloud[nxt]);
  JY_HIP(eng, hipGetLastError());
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total + 1, u.eoff[nxt] + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total + 2, u.coff[nxt] + nk, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipEventRecord(eng->total_ready, eng->stream));
  u.known = true;
  u.nel_bound = live_e + nel;
  u.ncloud_bound = live_c + ncloud;
  u.cur = nxt;
  return JY_OK;
}

int32_t jy_ujson_sizes(jy_engine* eng, u64 n, const u32* slots, u64* ne, u64* nc) {
  UjsonState& u = eng->ujson;
  hipLaunchKernelGGL(k_uj_sizes, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, u.eoff[u.cur], u.coff[u.cur],
                     slots, n, ne, nc);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_ujson_gather(jy_engine* eng, u64 n, const u32* slots, const u64* oeoff, const u64* ocoff, u64* odots,
                        u64* oelems, u64* ovv, u64* ocloud) {
  UjArgs A = state_args(eng);
  hipLaunchKernelGGL(k_uj_gather, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, A, slots, n, oeoff, ocoff,
                     odots, oelems, ovv, ocloud);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}
