// k_counter.hip -- GCOUNT / PNCOUNT kernels for gfx950.
//
// Semantics (bit-exact with the oracle, oracle/jy_oracle.cpp GCounter):
//   converge: s[slot][col] = max(s[slot][col], v)         gcount.md:45-47,
//             PNCOUNT: P and N separately                  pncount.md:51-55
//   value:    sum_col s[slot][col] mod 2^64;  PNCOUNT sum P - sum N, as i64
//             (repo_gcount.pony:53-55, repo_pncount.pony:55-57)
//
// HBM layout: one slab per type, [sign][column][slot] (replica-major).  A
// flushed peer batch is one replica column, so the dense merge of a peer
// batch streams one contiguous column; the per-key sum reads across
// columns with lanes on consecutive slots (coalesced).  Absent replica
// entries are 0, which is indistinguishable from absent under max and sum.
//
// Roofline: HBM.  Block merge moves 24 B per cell (8 delta read, 8 state
// read, 8 state write); sum-read 8 B per cell + 8 B per key.

#include <algorithm>


#include "jy_dscan.hpp"
#include "jy_internal.hpp"

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

namespace {

#ifndef JY_BLK_THREADS
#define JY_BLK_THREADS 256
#endif
// One 16-B vector per lane, 512-cell tiles (in-box A/B of the PNCOUNT
// headline, round 4, ms per 2^31-cell merge: 4 vectors per lane 8.78-8.80,
// 2 vectors 8.53-8.54, 1 vector 8.19-8.36; 128 threads x 1 or 2 vectors
// 8.20-8.27; 512 threads x 4 vectors 9.18; 64 threads x 2 vectors 9.71):
// more, smaller workgroups keep the 256 CUs fed to the end of each row.
#ifndef JY_BLK_UNROLL
#define JY_BLK_UNROLL 1
#endif
constexpr int kThreads = JY_BLK_THREADS;
constexpr int kUnroll = JY_BLK_UNROLL;              // 16-B vectors in flight per lane
constexpr u64 kTileCells = kThreads * 2 * kUnroll;  // 512 cells per tile

// Dense column-block max-merge.  Grid: x = 512-cell tile of a row, y = row
// (sign, column); one tile per workgroup (the dispatcher keeps 256 CUs fed
// better than a grid-stride loop here: tools/mb_stream.hip).  16 B per lane
// per access, kUnroll independent vectors in flight per lane; every stream
// is touched once, so loads and stores are nontemporal.
template <bool kVec>
__global__ __launch_bounds__(kThreads) void k_block_max(u64* __restrict__ slab, u64 row_pitch, u64 sign_pitch,
                                                        const u16* __restrict__ cols, u32 ncols, u64 slot0,
                                                        u64 nslots, const u64* __restrict__ vp,
                                                        const u64* __restrict__ vn, u64 rows) {
  for (u64 row = blockIdx.y; row < rows; row += gridDim.y) {
    const u32 sign = (u32)(row / ncols);
    const u32 c = (u32)(row - (u64)sign * ncols);
    u64* __restrict__ s = slab + sign * sign_pitch + (u64)cols[c] * row_pitch + slot0;
    const u64* __restrict__ d = (sign ? vn : vp) + (u64)c * nslots;
    if (kVec) {
      const u64 base = (u64)blockIdx.x * kTileCells + (u64)threadIdx.x * 2;
      u64x2 dv[kUnroll], sv[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const u64 i = base + (u64)u * (kThreads * 2);
        if (i < nslots) {
          dv[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(d + i));
          sv[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(s + i));
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const u64 i = base + (u64)u * (kThreads * 2);
        if (i < nslots) {
          u64x2 r;
          r.x = dv[u].x > sv[u].x ? dv[u].x : sv[u].x;
          r.y = dv[u].y > sv[u].y ? dv[u].y : sv[u].y;
          __builtin_nontemporal_store(r, reinterpret_cast<u64x2*>(s + i));
        }
      }
    } else {  // odd slot runs / misaligned inputs
      const u64 base = (u64)blockIdx.x * kTileCells + threadIdx.x;
#pragma unroll
      for (int u = 0; u < 2 * kUnroll; u++) {
        const u64 i = base + (u64)u * kThreads;
        if (i < nslots) {
          const u64 dv = d[i], sv = s[i];
          s[i] = dv > sv ? dv : sv;
        }
      }
    }
  }
}

// Sparse COO max-merge.  Cells of one call may repeat (several deltas for
// one key, or a delta naming a replica twice): the 64-bit atomic max keeps
// the join exact in any order.
__global__ __launch_bounds__(kThreads) void k_coo_max(u64* __restrict__ slab, u64 row_pitch,
                                                      const u32* __restrict__ slot, const u16* __restrict__ col,
                                                      const u64* __restrict__ val, u64 n) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  u64* p = slab + (u64)col[i] * row_pitch + slot[i];
  const u64 v = val[i];
  if (v > *p) __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// COO cells whose slots come from a device key interning of the same call
// (jy_counter_converge_keys): cell i belongs to key cell_key[i] (identity
// when null) and to slab `sign[i]` (P when null).  Device batches are not
// validated on the host: a cell naming no key of the batch, a sign other
// than 0/1, a column past the registered replicas or a key the directory
// could not place is skipped and counted (jy_skipped), like a malformed
// entry of the reference's swallowed converge (repo_gcount.pony:51).
__global__ __launch_bounds__(kThreads) void k_coo_max_keyed(u64* __restrict__ slab, u64 row_pitch, u64 sign_pitch,
                                                            const u32* __restrict__ kslot,
                                                            const u32* __restrict__ cell_key,
                                                            const uint8_t* __restrict__ sign,
                                                            const u16* __restrict__ col,
                                                            const u64* __restrict__ val, u64 n, u64 nkeys,
                                                            u32 nsigns, u32 ncols,
                                                            unsigned long long* __restrict__ skipped) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u64 k = cell_key ? (u64)cell_key[i] : i;
  const u32 g = sign ? (u32)sign[i] : 0u;
  const u32 c = col[i];
  const u32 s = k < nkeys ? kslot[k] : JY_NO_SLOT;
  if (s >= row_pitch || g >= nsigns || c >= ncols) {
    atomicAdd(skipped, 1ull);
    return;
  }
  u64* p = slab + (g ? sign_pitch : 0) + (u64)c * row_pitch + s;
  const u64 v = val[i];
  if (v > *p) __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// value(): wrapping sum over the used replica columns; PNCOUNT subtracts N.
__global__ __launch_bounds__(kThreads) void k_sum(const u64* __restrict__ slab, u64 row_pitch, u64 sign_pitch,
                                                  u32 ncols, u32 nsigns, const u32* __restrict__ slots, u64 n,
                                                  u64* __restrict__ out) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u64 s = slots ? (u64)slots[i] : i;
  u64 acc = 0;
  const u64* p = slab + s;
#pragma unroll 8
  for (u32 c = 0; c < ncols; c++) acc += p[(u64)c * row_pitch];
  if (nsigns == 2) {
    const u64* q = slab + sign_pitch + s;
#pragma unroll 8
    for (u32 c = 0; c < ncols; c++) acc -= q[(u64)c * row_pitch];
  }
  out[i] = acc;
}

// ---- local write path (RepoGCOUNT.inc repo_gcount.pony:57-60, RepoPNCOUNT
// inc/dec repo_pncount.pony:59-67): s[slot][own] += v, wrapping.  Repeated
// keys in one batch add atomically (u64 addition mod 2^64 commutes, so the
// total equals the reference's sequential one).  The first write of a key
// since the last flush bumps the pending count (deltas_size).
__global__ __launch_bounds__(kThreads) void k_cnt_add(u64* __restrict__ cell0, u32* __restrict__ dflag, u64* __restrict__ dcount,
                                                      u32 bit, const u32* __restrict__ slot,
                                                      const u64* __restrict__ val, u64 n) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u32 s = slot[i];
  atomicAdd(cell0 + s, val[i]);
  jy_wave_count(atomicOr(dflag + s, bit) == 0u, reinterpret_cast<unsigned long long*>(dcount));
}

// the delta records the post-write total (GCounter.increment writes
// delta[id] = cur).  Within one batch no merge interleaves, so the cell after
// the whole batch is the total of the key's last write; duplicates store the
// same value.
__global__ __launch_bounds__(kThreads) void k_cnt_record(const u64* __restrict__ cell0, u64* __restrict__ dval,
                                                         u32 nsigns, u32 sign, const u32* __restrict__ slot, u64 n) {
  const u64 i = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const u32 s = slot[i];
  dval[(u64)s * nsigns + sign] = cell0[s];
}

struct PendingPred {
  const u32* dflag;
  __device__ bool operator()(u64 s) const { return dflag[s] != 0; }
};

// flush_deltas (repo_gcount.pony:18-23): emit every pending key, then clear it
__global__ __launch_bounds__(kThreads) void k_cnt_flush(u32* __restrict__ dflag, const u64* __restrict__ dval,
                                                        u32 nsigns, const u32* __restrict__ slots, u64 cnt,
                                                        u64 cap, u64* __restrict__ vals, u32* __restrict__ mask) {
  const u64 j = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (j >= cnt) return;
  const u32 s = slots[j];
  const u32 f = dflag[s];
  mask[j] = f;
  for (u32 g = 0; g < nsigns; g++) vals[(u64)g * cap + j] = (f >> g) & 1u ? dval[(u64)s * nsigns + g] : 0;
  dflag[s] = 0;
}

}  // namespace

int32_t jy_counter_grow(jy_engine* eng, int which, u32 need_cols, u64 need_slots) {
  CounterState& c = eng->cnt[which];
  const u32 nsigns = which + 1;
  u32 ncap = c.ccap;
  u64 nk = c.kcap;
  if (need_cols > ncap) ncap = std::max<u32>(need_cols, ncap ? std::min<u32>(ncap * 2, 0xFFFF) : need_cols);
  if (need_slots > nk) nk = std::max<u64>(need_slots, nk ? nk * 2 : need_slots);
  nk = (nk + 63) & ~63ull;  // 512-B aligned column pitch
  if (ncap == 0) ncap = eng->cfg.counter_columns;
  if (ncap == c.ccap && nk == c.kcap && c.slab) return JY_OK;
  void* p = nullptr;
  const u64 bytes = (u64)nsigns * ncap * nk * 8;
  JY_TRY(jy_dev_alloc(eng, &p, bytes, "counter slab"));
  JY_HIP(eng, hipMemsetAsync(p, 0, bytes, eng->stream));
  if (c.slab) {
    for (u32 s = 0; s < nsigns; s++) {
      u64* dst = static_cast<u64*>(p) + (u64)s * ncap * nk;
      const u64* src = c.slab + (u64)s * c.ccap * c.kcap;
      JY_HIP(eng, hipMemcpy2DAsync(dst, nk * 8, src, c.kcap * 8, c.kcap * 8, c.ccap, hipMemcpyDeviceToDevice,
                                   eng->stream));
    }
    jy_dev_free(eng, c.slab);
  }
  c.slab = static_cast<u64*>(p);
  c.ccap = ncap;
  c.kcap = nk;
  return JY_OK;
}

int32_t jy_counter_coo(jy_engine* eng, int which, int sign, u64 n, const u32* slot, const u16* col, const u64* val) {
  if (n == 0) return JY_OK;
  JyTimed tm(eng);
  CounterState& c = eng->cnt[which];
  u64* base = c.slab + (u64)sign * c.ccap * c.kcap;
  const u64 blocks = (n + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(k_coo_max, dim3((u32)blocks), dim3(kThreads), 0, eng->stream, base, c.kcap, slot, col, val, n);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_counter_coo_keyed(jy_engine* eng, int which, u64 n, u64 nkeys, const u32* kslot, const u32* cell_key,
                             const uint8_t* sign, const u16* col, const u64* val) {
  if (n == 0) return JY_OK;
  JyTimed tm(eng);
  CounterState& c = eng->cnt[which];
  const u64 blocks = (n + kThreads - 1) / kThreads;
  const u32 ncols = std::min<u32>((u32)eng->rep_id.size(), c.ccap);
  hipLaunchKernelGGL(k_coo_max_keyed, dim3((u32)blocks), dim3(kThreads), 0, eng->stream, c.slab, c.kcap,
                     c.ccap * c.kcap, kslot, cell_key, sign, col, val, n, nkeys, (u32)(which + 1), ncols,
                     reinterpret_cast<unsigned long long*>(eng->skipped_dev));
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_counter_block(jy_engine* eng, int which, u32 ncols, const u16* cols_dev, u32 slot0, u32 nslots,
                         const u64* vp, const u64* vn) {
  JyTimed tm(eng);
  CounterState& c = eng->cnt[which];
  const u32 nsigns = which + 1;
  const void* dcols = cols_dev;
  const u64 rows = (u64)nsigns * ncols;
  const u64 tiles_per_row = (nslots + kTileCells - 1) / kTileCells;
  const bool vec = (slot0 % 2 == 0) && (nslots % 2 == 0) && (c.kcap % 2 == 0) &&
                   (reinterpret_cast<uintptr_t>(vp) % 16 == 0) && (!vn || reinterpret_cast<uintptr_t>(vn) % 16 == 0);
  const dim3 grid((u32)tiles_per_row, (u32)std::min<u64>(rows, 65535));
  if (vec)
    hipLaunchKernelGGL(k_block_max<true>, grid, dim3(kThreads), 0, eng->stream, c.slab, c.kcap,
                       (u64)c.ccap * c.kcap, static_cast<const u16*>(dcols), ncols, (u64)slot0, (u64)nslots, vp,
                       vn, rows);
  else
    hipLaunchKernelGGL(k_block_max<false>, grid, dim3(kThreads), 0, eng->stream, c.slab, c.kcap,
                       (u64)c.ccap * c.kcap, static_cast<const u16*>(dcols), ncols, (u64)slot0, (u64)nslots, vp,
                       vn, rows);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_counter_sum(jy_engine* eng, int which, u64 n, const u32* slots_dev, u64* out_dev) {
  if (n == 0) return JY_OK;
  CounterState& c = eng->cnt[which];
  const u32 ncols = std::min<u32>((u32)eng->rep_id.size(), c.ccap);
  const u64 blocks = (n + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(k_sum, dim3((u32)blocks), dim3(kThreads), 0, eng->stream, c.slab, c.kcap,
                     (u64)c.ccap * c.kcap, ncols, (u32)(which + 1), slots_dev, n, out_dev);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

// ---- local write path + flush_deltas ----
static int32_t counter_delta_grow(jy_engine* eng, int which) {
  CounterState& c = eng->cnt[which];
  const u32 nsigns = which + 1;
  if (!c.dcount) {
    void* p = nullptr;
    JY_TRY(jy_dev_alloc(eng, &p, 8, "counter pending count"));
    JY_HIP(eng, hipMemsetAsync(p, 0, 8, eng->stream));
    c.dcount = static_cast<u64*>(p);
  }
  if (c.dkcap >= c.kcap && c.dflag) return JY_OK;
  void *f = c.dflag, *v = c.dval;
  JY_TRY(jy_realloc(eng, &f, c.dkcap * 4, c.kcap * 4, true));
  JY_TRY(jy_realloc(eng, &v, c.dkcap * 8 * nsigns, c.kcap * 8 * nsigns, true));
  c.dflag = static_cast<u32*>(f);
  c.dval = static_cast<u64*>(v);
  c.dkcap = c.kcap;
  return JY_OK;
}

int32_t jy_cnt_write(jy_engine* eng, int which, int sign, u16 col, u64 n, const u32* slot, const u64* val) {
  if (n == 0) return JY_OK;
  CounterState& c = eng->cnt[which];
  if (c.dcol >= 0 && c.dcol != col)
    return eng->fail(JY_EINVAL, "pending deltas were written under another replica column (flush first)");
  JY_TRY(counter_delta_grow(eng, which));
  c.dcol = col;
  JyTimed tm(eng);
  u64* cell0 = c.slab + (u64)sign * c.ccap * c.kcap + (u64)col * c.kcap;
  const u32 blocks = (u32)((n + kThreads - 1) / kThreads);
  hipLaunchKernelGGL(k_cnt_add, dim3(blocks), dim3(kThreads), 0, eng->stream, cell0, c.dflag, c.dcount,
                     1u << sign, slot, val, n);
  hipLaunchKernelGGL(k_cnt_record, dim3(blocks), dim3(kThreads), 0, eng->stream, (const u64*)cell0, c.dval,
                     (u32)(which + 1), (u32)sign, slot, n);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t jy_cnt_pending(jy_engine* eng, int which, u64* count) {
  CounterState& c = eng->cnt[which];
  *count = 0;
  if (!c.dcount) return JY_OK;
  JY_HIP(eng, hipMemcpyAsync(eng->pin_total, c.dcount, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  *count = eng->pin_total[0];
  return JY_OK;
}

int32_t jy_cnt_flush(jy_engine* eng, int which, u64 nkeys, u64 cap, u32* slots, u64* vals, u32* mask,
                         u64* count) {
  CounterState& c = eng->cnt[which];
  u64 cnt = 0;
  JY_TRY(jy_cnt_pending(eng, which, &cnt));
  *count = cnt;
  if (cnt == 0) return JY_OK;
  if (cnt > cap) return eng->fail(JY_ERANGE, "flush output capacity is smaller than the pending delta count");
  nkeys = std::min<u64>(nkeys, c.dkcap);
  void* num = nullptr;
  JY_TRY(jy_scratch(eng, 14, 8, &num));
  JY_TRY(jydscan::select(eng, nkeys, PendingPred{c.dflag}, slots, static_cast<u32*>(num)));
  hipLaunchKernelGGL(k_cnt_flush, dim3((u32)((cnt + kThreads - 1) / kThreads)), dim3(kThreads), 0, eng->stream,
                     c.dflag, (const u64*)c.dval, (u32)(which + 1), (const u32*)slots, cnt, cap, vals, mask);
  JY_HIP(eng, hipGetLastError());
  JY_HIP(eng, hipMemsetAsync(c.dcount, 0, 8, eng->stream));
  c.dcol = -1;
  return JY_OK;
}
