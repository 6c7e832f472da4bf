// k_uj_write.hip -- UJSON write path on the engine, gfx950: RepoUJSON.ins /
// rm / clr (repo_ujson.pony:74-110) over opaque element handles, plus
// flush_deltas (repo_ujson.pony:22-26).
//
// A write is a delta document of the dot kernel, built on the device from the
// state as it is, then converged into the state AND into the key's pending
// delta (a second store of the same layout, ujson_d) -- the reference's
// (state, delta) argument pairs; the pending delta takes RM / CLR dots into
// its context only (context-only join: elements it holds stay):
//   INS h   a fresh dot (col, vv[col] + 1) carrying h; context = that dot
//   RM h    no element; context = the dots of every element equal to h
//           (observed remove: concurrent inserts elsewhere survive)
//   CLR     no element; context = the dots of every element of the doc
// Path-scoped CLR / SET are host compositions of these (jylis_amd/ujson_doc.py).
// Every command marks its doc pending (_delta_for); the host does not issue
// RM / CLR for a key that does not exist (repo_ujson.pony:86,108 create
// nothing).  One command per doc per call here; the C-ABI runs host batches
// with repeated docs in rounds.
//
// Roofline: not a hot path (local writes); one pass over each touched doc's
// element segment plus two converges of tiny deltas.

#include <algorithm>

#include "jy_dscan.hpp"
#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ u64 gid() { return (u64)blockIdx.x * kThreads + threadIdx.x; }

struct WArgs {
  const uint8_t* op;
  const u32* slot;
  const u64* elem;
  u64 n;
  u32 col, R;
  const UMeta* meta;
  const URec* rec;
  const u64* vv;
  const LCol* lcol;  // the in-place layout's column runs (k_ujson.hip), or nullptr
  const URec* lpe;
};

// the element records of the doc of meta m in dot order: a regular run, or
// a long document's column runs one after another
template <typename Fn>
__device__ __forceinline__ void for_each_rec(const WArgs& W, const UMeta& m, Fn&& fn) {
  if (m.ecap == kLongMark) {
    for (u32 c = 0; c < W.R; c++) {
      const LCol L = W.lcol[m.ebase * W.R + c];
      for (u64 j = 0; j < L.elen; j++) fn(W.lpe[L.ebase + j]);
    }
    return;
  }
  for (u64 j = 0; j < m.elen; j++) fn(W.rec[m.ebase + j]);
}

// delta sizes per command; every doc becomes pending
__global__ __launch_bounds__(kThreads) void k_ujw_count(WArgs W, u64* __restrict__ ne, u64* __restrict__ nc,
                                                        u32* __restrict__ pend, u64* __restrict__ pcount) {
  const u64 i = gid();
  if (i >= W.n) return;
  const u32 s = W.slot[i];
  const uint8_t op = W.op[i];
  u64 e = 0, c = 0;
  if (op == JY_UJSON_INS) {
    e = c = 1;
  } else {
    const UMeta m = W.meta[s];
    if (op == JY_UJSON_CLR) {
      c = m.elen;
    } else {
      const u64 h = W.elem[i];
      for_each_rec(W, m, [&](const URec& r) { c += r.elem == h; });
    }
  }
  ne[i] = e;
  nc[i] = c;
  jy_wave_count(atomicExch(pend + s, 1u) == 0, (unsigned long long*)pcount);
}

// the delta documents: elements, cloud (ascending: the state's elements are
// stored ascending by dot), empty version vectors
__global__ __launch_bounds__(kThreads) void k_ujw_fill(WArgs W, const u64* __restrict__ eo, const u64* __restrict__ co,
                                                       u64* __restrict__ dots, u64* __restrict__ elems,
                                                       u64* __restrict__ cloud) {
  const u64 i = gid();
  if (i >= W.n) return;
  const u32 s = W.slot[i];
  const uint8_t op = W.op[i];
  if (op == JY_UJSON_INS) {
    const u64 d = ((u64)W.col << JY_DOT_SEQ_BITS) | (W.vv[(u64)s * W.R + W.col] + 1);
    dots[eo[i]] = d;
    elems[eo[i]] = W.elem[i];
    cloud[co[i]] = d;
    return;
  }
  const UMeta m = W.meta[s];
  const u64 h = W.elem[i];
  u64 o = co[i];
  for_each_rec(W, m, [&](const URec& r) {
    if (op == JY_UJSON_CLR || r.elem == h) cloud[o++] = r.dot;
  });
}

// flush: the pending docs' delta documents are emptied
__global__ __launch_bounds__(kThreads) void k_ujw_reset(UMeta* __restrict__ dmeta, u64* __restrict__ dvv, u32 R,
                                                        u32* __restrict__ pend, const u32* __restrict__ slots, u64 n) {
  const u64 i = gid();
  if (i >= n) return;
  const u32 s = slots[i];
  dmeta[s] = UMeta{0, 0, 0, 0, 0, 0};
  for (u32 c = 0; c < R; c++) dvv[(u64)s * R + c] = 0;
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

int32_t pending_grow(jy_engine* eng) {
  UjsonState& d = eng->ujson_d;
  d.R = eng->ujson.R;
  JY_TRY(ujson_grow_store(eng, d, eng->ujson.kcap, 0));
  if (!eng->uj_dcount) {
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&eng->uj_dcount), 8, "ujson pending count"));
    JY_HIP(eng, hipMemsetAsync(eng->uj_dcount, 0, 8, eng->stream));
  }
  if (eng->uj_dkcap < d.kcap || !eng->uj_dflag) {
    void* f = eng->uj_dflag;
    JY_TRY(jy_realloc(eng, &f, eng->uj_dkcap * 4, d.kcap * 4, true));
    eng->uj_dflag = static_cast<u32*>(f);
    eng->uj_dkcap = d.kcap;
  }
  return JY_OK;
}

}  // namespace

int32_t jy_ujson_write_batch(jy_engine* eng, u64 n, const uint8_t* op, const u32* slot, const u64* elem, u32 col) {
  if (n == 0) return JY_OK;
  UjsonState& u = eng->ujson;
  if (col >= u.R) return eng->fail(JY_ERANGE, "ujson write: replica column outside the version vector");
  JY_TRY(pending_grow(eng));
  // (scratch 0..7 hold the staged commands; the converges use 10..20)
  void* p;
  JY_TRY(jy_scratch(eng, 21, (n + 1) * 8 * 4 + 64, &p));
  u64* ne = static_cast<u64*>(p);
  u64* nc = ne + (n + 1);
  u64* eo = nc + (n + 1);
  u64* co = eo + (n + 1);
  const WArgs W{op, slot, elem, n, col, u.R, u.meta, u.epool, u.vv, u.lcol, u.lpe};
  JY_HIP(eng, hipMemsetAsync(ne + n, 0, 8, eng->stream));
  JY_HIP(eng, hipMemsetAsync(nc + n, 0, 8, eng->stream));
  LAUNCH(k_ujw_count, n, W, ne, nc, eng->uj_dflag, eng->uj_dcount);
  JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, n + 1, jydscan::LdArr<u64>{ne}, jydscan::StArr<u64>{eo})));
  JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, n + 1, jydscan::LdArr<u64>{nc}, jydscan::StArr<u64>{co})));
  // the delta's sizes (a local write waits for them: RM / CLR sizes come from the state)
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, eo + n, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total + 1, co + n, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  const u64 nins = eng->pin_total[0], ncl = eng->pin_total[1];
  JY_TRY(jy_scratch(eng, 22, (2 * n + ncl + 1) * 8 + (n + 1) * 8 + 64, &p));
  u64* dots = static_cast<u64*>(p);
  u64* elems = dots + n;
  u64* cloud = elems + n;
  u64* vvoff = cloud + ncl + 1;  // no version-vector entries
  JY_HIP(eng, hipMemsetAsync(vvoff, 0, (n + 1) * 8, eng->stream));
  LAUNCH(k_ujw_fill, n, W, eo, co, dots, elems, cloud);
  JY_TRY(jy_ujson_merge_into(eng, u, n, slot, eo, nins, dots, elems, vvoff, 0, vvoff, co, ncl, cloud));
  // the pending delta takes the removed dots into its context only: an
  // element it already holds stays (what the reference's delta.ctx insert
  // does, oracle UJSON::remove / clear)
  JY_TRY(jy_ujson_merge_into(eng, eng->ujson_d, n, slot, eo, nins, dots, elems, vvoff, 0, vvoff, co, ncl, cloud,
                             true));
  return JY_OK;
}

int32_t jy_ujson_pending(jy_engine* eng, u64* count) {
  *count = 0;
  if (!eng->uj_dcount) return JY_OK;
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, eng->uj_dcount, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  *count = eng->pin_total[0];
  return JY_OK;
}

// two calls: with caps too small it only reports the sizes; with room it
// writes (device arrays; vv dense [ndocs][R]) and clears the pending deltas
int32_t jy_ujson_flush_dev(jy_engine* eng, u64 cap_docs, u64 cap_el, u64 cap_cl, u32* slots, u64* eoff, u64* dots,
                           u64* elems, u64* vv, u64* coff, u64* cloud, u64* ndocs, u64* nel, u64* ncl) {
  u64 k = 0;
  JY_TRY(jy_ujson_pending(eng, &k));
  *ndocs = k;
  *nel = *ncl = 0;
  if (k == 0) return JY_OK;
  UjsonState& d = eng->ujson_d;
  void* p;
  JY_TRY(jy_scratch(eng, 21, k * 4 + (k + 1) * 32 + 64, &p));
  u32* sl = static_cast<u32*>(p);
  u64* se = reinterpret_cast<u64*>((reinterpret_cast<uintptr_t>(sl + k) + 15) & ~uintptr_t(15));
  u64* sc = se + (k + 1);
  u64* eo = sc + (k + 1);
  u64* co = eo + (k + 1);
  void* num;
  JY_TRY(jy_scratch(eng, 14, 8, &num));
  JY_TRY(jydscan::select(eng, std::min<u64>(eng->nkeys[JY_UJSON], eng->uj_dkcap), PendPred{eng->uj_dflag}, sl,
                         static_cast<u32*>(num)));
  JY_HIP(eng, hipMemsetAsync(se + k, 0, 8, eng->stream));
  JY_HIP(eng, hipMemsetAsync(sc + k, 0, 8, eng->stream));
  JY_TRY(jy_ujson_sizes_of(eng, d, k, sl, se, sc));
  JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, k + 1, jydscan::LdArr<u64>{se}, jydscan::StArr<u64>{eo})));
  JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, k + 1, jydscan::LdArr<u64>{sc}, jydscan::StArr<u64>{co})));
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, eo + k, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total + 1, co + k, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  const u64 me = eng->pin_total[0], mc = eng->pin_total[1];
  *nel = me;
  *ncl = mc;
  if (cap_docs < k || cap_el < me || cap_cl < mc) return JY_OK;  // sizes only
  JY_HIP(eng, hipMemcpyAsync(slots, sl, k * 4, hipMemcpyDeviceToDevice, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(eoff, eo, (k + 1) * 8, hipMemcpyDeviceToDevice, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(coff, co, (k + 1) * 8, hipMemcpyDeviceToDevice, eng->stream));
  JY_TRY(jy_ujson_gather_of(eng, d, k, sl, eo, co, me, mc, dots, elems, vv, cloud));
  LAUNCH(k_ujw_reset, k, d.meta, d.vv, d.R, eng->uj_dflag, sl, k);
  JY_HIP(eng, hipMemsetAsync(eng->uj_dcount, 0, 8, eng->stream));
  // every pending doc was flushed: the delta pools are empty again (in-flight
  // converges of the delta store are stream-ordered before this reset)
  JY_HIP(eng, hipMemsetAsync(d.ctr, 0, 16, eng->stream));
  d.used_e = d.used_c = 0;
  d.live_e = d.live_c = 0;
  d.done = d.seq;
  return JY_OK;
}
