// k_route_csr.hip -- routing CSR delta batches (TLOG logs, UJSON documents)
// to their owner shards, gfx950.
//
// The exchange step of SURVEY.md section 8e for the two CSR types, the
// counterpart of k_route.hip's TREG records.  A key travels with all of its
// entries (a TLOG key's log, a UJSON document's elements, vv entries and
// cloud dots), so the unit of the partition is the key and its CSR ranges.
//
// Sender: the batch is partitioned by owner into one RUN per destination of
// a fixed layout (route_layout below: slots, per-key cutoffs for TLOG, per
// CSR the offsets and the entry columns), so every all-to-all is an
// equal-split collective and each run is a well-formed converge batch on
// its own.  Keys keep their input order inside a run; a key that does not
// fit (record, entry or value-byte capacity) goes to the overflow list and
// so does every later key of that destination -- the placed keys of a run
// are a prefix, and their counts are the run's header.  Unused records are
// HOLES (slot JY_NO_SLOT, empty ranges) that the merge kernels skip; for
// UJSON, whose item kernels cover every entry of a batch, the last record
// is always a hole that spans the run's unused entry capacity.
//   R1 k_rc_count   per key tile: per destination totals (keys, entries per
//                   CSR, long-value bytes)
//   R2 scan         every (destination, quantity) column of tile counts in
//                   one device-wide scan, column after column; k_rc_hdr
//   R3 k_rc_place   per key: its place in its destination's run (tile base
//                   + wave ranks), fit test, key records
//   R4 k_rc_copy    per entry: the entry columns into the key's run range,
//                   long values' bytes into the run's byte section
//   R5 k_rc_finish  holes after each run's placed keys
// Receiver: TLOG value handles are rebased onto the arena (k_rc_rebase) and
// each source's run is merged by the type's own converge kernels, one source
// at a time (a key named by several sources is then exact).
//
// No count crosses to the host: the host reads only the overflow count, one
// step later and asynchronously (jylis_amd/route.py).
//
// Roofline: HBM.  The sender reads each key's offsets twice and its entries
// once and writes each entry once (+ long value bytes); the receiver's
// merge is the type's converge over the run.

#include <algorithm>

#include "jy_internal.hpp"
#include "jy_dscan.hpp"
#include "jy_scan.hpp"

namespace {

constexpr int kThreads = 256;  // keys (or entries) per tile, one per thread
constexpr u32 kMaxShards = 64;
constexpr u32 kNone = 0xFFFFFFFFu;

__device__ __forceinline__ u64 round8(u64 x) { return (x + kArenaAlign - 1) & ~(kArenaAlign - 1); }

struct Csr {
  const u64* offs;
  const u64* col[3];
  u64 nent_host;  // entries of the input (host's bound for the copy grid)
  u64 cap;        // entry capacity of a run
  u64 o_offs;     // run word offset of the offsets [cap_k + 1]
  u64 o_col[3];   // ... of each column [cap]
};

template <int kC>
struct RouteArgs {
  u64 n;
  u64 kbase;  // input index of key 0 (overflow lists name keys of the whole batch)
  u32 S;
  u64 cap_k;  // records per run
  u64 kfit;   // records that may hold a key (cap_k, or cap_k - 1 with a slack hole)
  u32 slack;
  const u32* owner;
  const u32* slot;
  const u64* kx;  // per-key scalar (TLOG cutoff) or null
  Csr c[kC];
  u32 ncol[kC];
  int lr;  // column of c[0] holding value handles (TLOG), -1 for none
  const uint8_t* arena;
  u64 cap_b;
  u64 W, o_slot, o_kx;
  u64* out;
  uint8_t* bytes;
  unsigned long long* hdr;  // [S][8]
  u32* ovf;
  unsigned long long* skipped;
  u64* tcnt;  // [ntiles][S][kQ]
  u64* kb;    // [n] long-value bytes of the key (padded)
  u32* eb;    // [entries of CSR 0] a long value's byte offset inside its key's bytes
  u32* kdst;  // [n] destination, or kNone
  u64* keo;   // [n][kC (+1)] first entry of the key in its run per CSR (+ its first value byte)
};

// layout of one run in u64 words: slots (u32, packed), [per-key scalars],
// per CSR the offsets, then per CSR its columns
template <int kC>
void route_layout(RouteArgs<kC>& A, bool has_kx, const u64* caps, const u32* ncol) {
  u64 w = 0;
  A.o_slot = w;
  w += (A.cap_k + 1) / 2;
  A.o_kx = w;
  if (has_kx) w += A.cap_k;
  for (int c = 0; c < kC; c++) {
    A.c[c].cap = caps[c];
    A.c[c].o_offs = w;
    w += A.cap_k + 1;
  }
  for (int c = 0; c < kC; c++) {
    A.ncol[c] = ncol[c];
    for (u32 j = 0; j < ncol[c]; j++) {
      A.c[c].o_col[j] = w;
      w += caps[c];
    }
  }
  A.W = (w + 1) & ~1ull;  // runs stay 16-B aligned
}

template <int kC, bool kLR>
__device__ __forceinline__ void key_quantities(const RouteArgs<kC>& A, u64 k, u64* v) {
  v[0] = 1;
#pragma unroll
  for (int c = 0; c < kC; c++) v[1 + c] = A.c[c].offs[k + 1] - A.c[c].offs[k];
  if (kLR) v[1 + kC] = A.kb[k];
}

// R1: per tile of keys, per destination totals; the key's long-value bytes
// lanes with the same destination add their quantities with one LDS atomic
// per destination and quantity
template <int kQ>
__device__ __forceinline__ void wave_add_by_owner(u32 o, bool valid, const u64 (&v)[kQ],
                                                  unsigned long long* __restrict__ lc) {
  u64 pending = __ballot(valid);
  while (pending) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const u32 lo = __shfl(o, leader);
    const bool mine = valid && o == lo;
    pending &= ~__ballot(mine);
#pragma unroll
    for (int q = 0; q < kQ; q++) {
      const u64 sum = jyscan::wave_sum<u64>(mine ? v[q] : 0ull);
      if (__lane_id() == (u32)leader && sum) atomicAdd(&lc[lo * kQ + q], (unsigned long long)sum);
    }
  }
}

template <int kC, bool kLR>
__global__ __launch_bounds__(kThreads) void k_rc_count(RouteArgs<kC> A) {
  constexpr int kQ = 1 + kC + (kLR ? 1 : 0);
  __shared__ unsigned long long lc[kMaxShards * kQ];
  for (u32 j = threadIdx.x; j < A.S * kQ; j += kThreads) lc[j] = 0;
  __syncthreads();
  const u64 k = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (k < A.n) {
    if (kLR) {
      const u64* lr = A.c[0].col[A.lr];
      u64 b = 0;
      for (u64 j = A.c[0].offs[k]; j < A.c[0].offs[k + 1]; j++) {
        const u64 len = lr[j] & JY_LR_LEN_MASK;
        if (len > 8) {
          A.eb[j] = (u32)b;
          b += round8(len);
        }
      }
      A.kb[k] = b;
    }
  }
  {
    u32 o = A.S;
    u64 v[kQ] = {};
    if (k < A.n) {
      o = A.owner[k];
      if (o < A.S) key_quantities<kC, kLR>(A, k, v);
    }
    wave_add_by_owner<kQ>(o, o < A.S, v, lc);  // one LDS atomic per (wave, owner, quantity)
  }
  __syncthreads();
  u64* row = A.tcnt + (u64)blockIdx.x * A.S * kQ;
  for (u32 j = threadIdx.x; j < A.S * kQ; j += kThreads) row[j] = lc[j];
}

// R2 (as launched): one device-wide scan of the tile counts column after
// column, then the header's totals from the column bases
__global__ void k_rc_hdr(const u64* __restrict__ tcnt, u64 ntiles, u32 W, u32 kq, unsigned long long* __restrict__ hdr) {
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= W) return;
  const u64 hi = c + 1 < W ? tcnt[c + 1] : tcnt[ntiles * W];
  hdr[(c / kq) * 8 + c % kq] = hi - tcnt[c];
}


// R3: the key's place in its run: tile base (R2) + the waves before it + its
// rank among its wave's keys of the same destination (one ballot per
// distinct destination, masked scans of the quantities)
template <int kC, bool kLR>
__global__ __launch_bounds__(kThreads) void k_rc_place(RouteArgs<kC> A) {
  constexpr int kQ = 1 + kC + (kLR ? 1 : 0);
  constexpr int kW = kThreads / 64;
  __shared__ u64 wt[kW][kMaxShards * kQ];
  for (u32 j = threadIdx.x; j < A.S * kQ; j += kThreads) {
#pragma unroll
    for (int w = 0; w < kW; w++) wt[w][j] = 0;
  }
  __syncthreads();
  const u64 k = (u64)blockIdx.x * kThreads + threadIdx.x;
  const int lane = __lane_id(), wv = threadIdx.x >> 6;
  const u64 lt = (1ull << lane) - 1;
  u32 o = kNone;
  u64 v[kQ], pre[kQ];
  if (k < A.n) {
    o = A.owner[k];
    key_quantities<kC, kLR>(A, k, v);
  }
  const bool valid = k < A.n && o < A.S;
  if (k < A.n && !valid) {
    atomicAdd(A.skipped, 1ull);  // an owner outside [0, S): dropped, counted
    A.kdst[k] = kNone;
  }
#pragma unroll
  for (int q = 0; q < kQ; q++) pre[q] = 0;
  u64 pending = __ballot(valid);
  while (pending) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const u32 d = __shfl(o, leader);
    const bool mine = valid && o == d;
    const u64 m = __ballot(mine);
    if (mine) pre[0] = __popcll(m & lt);
    if (lane == leader) wt[wv][d * kQ] = __popcll(m);
#pragma unroll
    for (int q = 1; q < kQ; q++) {
      const u64 x = mine ? v[q] : 0;
      const u64 inc = jyscan::wave_incl<u64>(x);
      if (mine) pre[q] = inc - x;
      const u64 tot = __shfl(inc, 63);
      if (lane == leader) wt[wv][d * kQ + q] = tot;
    }
    pending &= ~m;
  }
  __syncthreads();
  if (valid) {
    const u64* tb = A.tcnt + (u64)blockIdx.x * A.S * kQ + o * kQ;
    u64 at[kQ];
#pragma unroll
    for (int q = 0; q < kQ; q++) {
      u64 x = tb[q] - A.tcnt[o * kQ + q] + pre[q];  // less the column's base (row 0)
      for (int w = 0; w < wv; w++) x += wt[w][o * kQ + q];
      at[q] = x;
    }
    bool fits = at[0] < A.kfit;
#pragma unroll
    for (int c = 0; c < kC; c++) fits = fits && at[1 + c] + v[1 + c] <= A.c[c].cap;
    if (kLR) fits = fits && at[1 + kC] + v[1 + kC] <= A.cap_b;
    if (!fits) {
      A.kdst[k] = kNone;
      A.ovf[1 + atomicAdd(A.ovf, 1u)] = (u32)(A.kbase + k);
      // the first key of its destination that does not fit (the one before
      // it, whose ends are this key's starts, fits) writes the run's header:
      // the placed keys are exactly the prefix before it (no atomics)
      bool prev = at[0] > 0 && at[0] - 1 < A.kfit;
#pragma unroll
      for (int c = 0; c < kC; c++) prev = prev && at[1 + c] <= A.c[c].cap;
      if (kLR) prev = prev && at[1 + kC] <= A.cap_b;
      if (at[0] == 0 || prev) {
#pragma unroll
        for (int q = 0; q < kQ; q++) A.hdr[o * 8 + q] = at[q];
      }
    } else {
      u64* R = A.out + (u64)o * A.W;
      reinterpret_cast<u32*>(R + A.o_slot)[at[0]] = A.slot[k];
      if (A.kx) R[A.o_kx + at[0]] = A.kx[k];
      constexpr int kE = kC + (kLR ? 1 : 0);
#pragma unroll
      for (int c = 0; c < kC; c++) {
        R[A.c[c].o_offs + at[0] + 1] = at[1 + c] + v[1 + c];
        A.keo[k * kE + c] = at[1 + c];
      }
      if (kLR) A.keo[k * kE + kC] = at[1 + kC];  // the key's values start here in the byte section
      A.kdst[k] = o;
    }
  }
}

// R4: entry columns; a tile of entries of one CSR finds its keys with two
// wave searches and per-thread bisection between them.  The offsets are
// absolute (a chunk of a batch starts at offs[0] > 0); the grid is the
// host's bound, surplus tiles exit
template <int kC, bool kLR>
__global__ __launch_bounds__(kThreads) void k_rc_copy(RouteArgs<kC> A, u64 t1, u64 t2) {
  constexpr u32 kLds = kThreads;  // keys a tile stages (a tile of entries spans at most 256 non-empty keys)
  constexpr int kE = kC + (kLR ? 1 : 0);
  __shared__ u64 sh[2];
  __shared__ u64 l_off[kLds + 1], l_at[kLds], l_bb[kLds];
  __shared__ u32 l_d[kLds];
  u64 t = blockIdx.x;
  const int c = t < t1 ? 0 : t < t2 ? 1 : 2;
  if (c >= kC) return;
  t -= c == 0 ? 0 : c == 1 ? t1 : t2;
  const Csr C = c == 0 ? A.c[0] : c == 1 ? A.c[kC > 1 ? 1 : 0] : A.c[kC > 2 ? 2 : 0];  // uniform: no indexed kernarg
  const u32 ncol = c == 0 ? A.ncol[0] : c == 1 ? A.ncol[kC > 1 ? 1 : 0] : A.ncol[kC > 2 ? 2 : 0];
  const u64 nent = C.offs[A.n];
  const u64 j0 = C.offs[0] + t * kThreads;
  if (j0 >= nent) return;
  const u64 j1 = j0 + kThreads < nent ? j0 + kThreads : nent;
  if (threadIdx.x < 128) {
    const u64 kk = jyscan::wave_last_le(C.offs, A.n, threadIdx.x < 64 ? j0 : j1 - 1);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = kk;
  }
  __syncthreads();
  const u64 k0 = sh[0], cnt = sh[1] - sh[0] + 1;
  const bool lds = cnt <= kLds;  // empty keys between them can make it more
  if (lds && threadIdx.x < cnt) {  // the tile's keys: offsets, destination, first entry in the run
    const u64 k = k0 + threadIdx.x;
    l_off[threadIdx.x] = C.offs[k];
    l_d[threadIdx.x] = A.kdst[k];
    l_at[threadIdx.x] = A.keo[k * kE + c];
    if (kLR && c == 0) l_bb[threadIdx.x] = A.keo[k * kE + kC];
  }
  __syncthreads();
  const u64 j = j0 + threadIdx.x;
  if (j >= j1) return;
  u64 lo, off;
  u32 d;
  u64 at0, bb = 0;
  if (lds) {
    u32 a = 0, h = (u32)cnt - 1;
    while (a < h) {
      const u32 m = (a + h + 1) >> 1;
      if (l_off[m] <= j) a = m;
      else h = m - 1;
    }
    off = l_off[a], d = l_d[a], at0 = l_at[a];
    if (kLR && c == 0) bb = l_bb[a];
  } else {
    lo = k0;
    u64 hi = sh[1];
    while (lo < hi) {
      const u64 m = (lo + hi + 1) >> 1;
      if (C.offs[m] <= j) lo = m;
      else hi = m - 1;
    }
    off = C.offs[lo], d = A.kdst[lo], at0 = d == kNone ? 0 : A.keo[lo * kE + c];
    if (kLR && c == 0 && d != kNone) bb = A.keo[lo * kE + kC];
  }
  if (d == kNone) return;
  u64* R = A.out + (u64)d * A.W;
  const u64 at = at0 + (j - off);
#pragma unroll
  for (u32 q = 0; q < 3; q++) {
    if (q >= ncol) break;
    u64 x = C.col[q][j];
    if (kLR && c == 0 && (int)q == A.lr && (x & JY_LR_LEN_MASK) > 8) {
      // a long value: its 8-B granules into the run's byte section, the handle rewritten
      const u64 len = x & JY_LR_LEN_MASK, b = bb + A.eb[j];
      const u64* src = reinterpret_cast<const u64*>(A.arena + (x >> JY_LR_LEN_BITS));
      u64* dst = reinterpret_cast<u64*>(A.bytes + (u64)d * A.cap_b + b);
      for (u64 w = 0; w < round8(len) / 8; w++) dst[w] = src[w];
      x = (b << JY_LR_LEN_BITS) | len;
    }
    R[C.o_col[q] + at] = x;
  }
}

// R5: holes after the placed keys of every run; offsets[0]
template <int kC>
__global__ __launch_bounds__(kThreads) void k_rc_finish(RouteArgs<kC> A) {
  const u64 g = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (g >= (u64)A.S * A.cap_k) return;
  const u32 d = (u32)(g / A.cap_k);
  const u64 p = g - (u64)d * A.cap_k;
  u64* R = A.out + (u64)d * A.W;
  constexpr int kQ8 = 8;
  const unsigned long long* h = A.hdr + (u64)d * kQ8;
  if (p == 0) {
#pragma unroll
    for (int c = 0; c < kC; c++) R[A.c[c].o_offs] = 0;
  }
  if (p < h[0]) return;
  reinterpret_cast<u32*>(R + A.o_slot)[p] = JY_NO_SLOT;
  if (A.kx) R[A.o_kx + p] = 0;
  const bool last = A.slack && p == A.cap_k - 1;
#pragma unroll
  for (int c = 0; c < kC; c++) R[A.c[c].o_offs + p + 1] = last ? A.c[c].cap : h[1 + c];
}

// receiver: value handles of the runs' long values move onto the arena
__global__ __launch_bounds__(kThreads) void k_rc_rebase(u64* __restrict__ runs, u32 nsrc, u64 W, u64 o_lr, u64 cap_e,
                                                        u64 rebase, u64 cap_b) {
  const u64 g = (u64)blockIdx.x * kThreads + threadIdx.x;
  if (g >= (u64)nsrc * cap_e) return;
  const u64 s = g / cap_e, j = g - s * cap_e;
  u64* p = runs + s * W + o_lr + j;
  const u64 h = *p;
  if ((h & JY_LR_LEN_MASK) > 8) *p = h + ((rebase + s * cap_b) << JY_LR_LEN_BITS);
}

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

bool csr_ok(const u64* offs, u64 n, u64 nent) {
  if (offs[0] != 0 || offs[n] != nent) return false;
  for (u64 i = 0; i < n; i++)
    if (offs[i + 1] < offs[i]) return false;
  return true;
}

// sender: R1..R5 over a staged batch (device pointers)
template <int kC, bool kLR>
int32_t route_part(jy_engine* eng, RouteArgs<kC>& A) {
  const u64 n = A.n;
  constexpr int kQ = 1 + kC + (kLR ? 1 : 0);
  A.skipped = reinterpret_cast<unsigned long long*>(eng->skipped_dev);
  JY_HIP(eng, hipMemsetAsync(A.hdr, 0, (u64)A.S * 8 * 8, eng->stream));
  if (n) {
    const u64 ntiles = (n + kThreads - 1) / kThreads;
    void* p;
    JY_TRY(jy_scratch(eng, 24, ntiles * A.S * kQ * 8 + 64, &p));
    A.tcnt = static_cast<u64*>(p);
    JY_TRY(jy_scratch(eng, 25, n * 8 + (kLR ? A.c[0].nent_host * 4 : 0) + 64, &p));
    A.kb = static_cast<u64*>(p);
    A.eb = reinterpret_cast<u32*>(A.kb + n);
    JY_TRY(jy_scratch(eng, 26, n * 4 + 64, &p));
    A.kdst = static_cast<u32*>(p);
    JY_TRY(jy_scratch(eng, 27, n * (kC + (kLR ? 1 : 0)) * 8 + 64, &p));
    A.keo = static_cast<u64*>(p);
    hipLaunchKernelGGL((k_rc_count<kC, kLR>), dim3((u32)ntiles), dim3(kThreads), 0, eng->stream, A);
    JY_HIP(eng, hipGetLastError());
    {
      // every (destination, quantity) column in ONE device-wide scan taken
      // column after column; each column's base is its row-0 entry
      const u64 W = (u64)A.S * kQ;
      JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, ntiles * W + 1, jydscan::LdColMajor{A.tcnt, ntiles, W},
                                                    jydscan::StColMajor{A.tcnt, ntiles, W})));
      hipLaunchKernelGGL(k_rc_hdr, dim3((u32)((W + 255) / 256)), dim3(256), 0, eng->stream, A.tcnt, ntiles, (u32)W,
                         (u32)kQ, A.hdr);
      JY_HIP(eng, hipGetLastError());
    }
    hipLaunchKernelGGL((k_rc_place<kC, kLR>), dim3((u32)ntiles), dim3(kThreads), 0, eng->stream, A);
    JY_HIP(eng, hipGetLastError());
    // entry tiles per CSR: bounded by the host's totals
    u64 tl[3] = {0, 0, 0};
    for (int c = 0; c < kC; c++) tl[c] = (A.c[c].nent_host + kThreads - 1) / kThreads;
    const u64 g = tl[0] + tl[1] + tl[2];
    if (g)
      hipLaunchKernelGGL((k_rc_copy<kC, kLR>), dim3((u32)g), dim3(kThreads), 0, eng->stream, A, tl[0], tl[0] + tl[1]);
    JY_HIP(eng, hipGetLastError());
  }
  hipLaunchKernelGGL((k_rc_finish<kC>), dim3(blocks_for((u64)A.S * A.cap_k)), dim3(kThreads), 0, eng->stream, A);
  JY_HIP(eng, hipGetLastError());
  return JY_OK;
}

int32_t check_part(jy_engine* eng, u64 n, u32 S, u64 cap_k, const void* out, int32_t mem, const u32* owner) {
  if (S == 0 || S > kMaxShards) return eng->fail(JY_ERANGE, "nshards must be in [1, 64]");
  if (n >= 0xFFFFFFFFull) return eng->fail(JY_ERANGE, "more than 2^32 - 1 keys in one call");
  if (cap_k == 0) return eng->fail(JY_EINVAL, "cap_k must be positive");
  if (reinterpret_cast<uintptr_t>(out) % 16) return eng->fail(JY_EINVAL, "runs_dev must be 16-B aligned");
  if (mem == JY_HOST)
    for (u64 i = 0; i < n; i++)
      if (owner[i] >= S) return eng->fail(JY_ERANGE, "owner outside [0, nshards)");
  return JY_OK;
}

}  // namespace

extern "C" {

uint64_t jy_route_words(int32_t type, uint64_t cap_k, const uint64_t* caps) {
  if (type == JY_TLOG) {
    RouteArgs<1> A{};
    A.cap_k = cap_k;
    const u32 nc[1] = {3};
    route_layout(A, true, caps, nc);
    return A.W;
  }
  if (type == JY_UJSON) {
    RouteArgs<3> A{};
    A.cap_k = cap_k;
    const u32 nc[3] = {2, 1, 1};
    route_layout(A, false, caps, nc);
    return A.W;
  }
  return 0;
}

int32_t jy_tlog_route_part(jy_engine* eng, uint64_t n, const uint32_t* owner, const uint32_t* slot,
                           const uint64_t* cutoff, const uint64_t* ent_offs, uint64_t nent, const uint64_t* ts,
                           const uint64_t* pre, const uint64_t* lr, uint32_t nshards, uint64_t cap_k, uint64_t cap_e,
                           uint64_t cap_byte, uint64_t key_base, int32_t mem, uint64_t* runs_dev, uint8_t* bytes_dev,
                           uint64_t* hdr_dev, uint32_t* ovf_dev) {
  JY_HIP(eng, hipSetDevice(eng->device));
  JY_TRY(check_part(eng, n, nshards, cap_k, runs_dev, mem, owner));
  if (cap_byte % kArenaAlign) return eng->fail(JY_EINVAL, "cap_byte must be a multiple of 8");
  if (mem == JY_HOST && !csr_ok(ent_offs, n, nent))
    return eng->fail(JY_EINVAL, "entry offsets are not a CSR of nent entries");
  RouteArgs<1> A{};
  A.n = n;
  A.kbase = key_base;
  A.S = nshards;
  A.cap_k = cap_k;
  A.kfit = cap_k;
  const u64 caps[1] = {cap_e};
  const u32 nc[1] = {3};
  route_layout(A, true, caps, nc);
  const void *dow = nullptr, *dsl = nullptr, *dcut = nullptr, *doff = nullptr, *dts = nullptr, *dpre = nullptr,
             *dlr = nullptr;
  JY_TRY(jy_stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, owner, n * 4, mem, &dow));
  JY_TRY(jy_stage(eng, 1, slot, n * 4, mem, &dsl));
  JY_TRY(jy_stage(eng, 2, cutoff, n * 8, mem, &dcut));
  JY_TRY(jy_stage(eng, 3, ent_offs, (n + 1) * 8, mem, &doff));
  JY_TRY(jy_stage(eng, 4, ts, nent * 8, mem, &dts));
  JY_TRY(jy_stage(eng, 5, pre, nent * 8, mem, &dpre));
  JY_TRY(jy_stage(eng, 6, lr, nent * 8, mem, &dlr));
  JY_TRY(jy_stage_end(eng));
  A.owner = static_cast<const u32*>(dow);
  A.slot = static_cast<const u32*>(dsl);
  A.kx = static_cast<const u64*>(dcut);
  A.c[0].offs = static_cast<const u64*>(doff);
  A.c[0].nent_host = nent;
  A.c[0].col[0] = static_cast<const u64*>(dts);
  A.c[0].col[1] = static_cast<const u64*>(dpre);
  A.c[0].col[2] = static_cast<const u64*>(dlr);
  A.lr = 2;
  A.arena = eng->arena[JY_TLOG].p;
  A.cap_b = cap_byte;
  A.out = runs_dev;
  A.bytes = bytes_dev;
  A.hdr = reinterpret_cast<unsigned long long*>(hdr_dev);
  A.ovf = ovf_dev;
  return route_part<1, true>(eng, A);
}

int32_t jy_tlog_converge_routed(jy_engine* eng, uint32_t nsrc, uint64_t cap_k, uint64_t cap_e, uint64_t cap_byte,
                                uint64_t* runs_dev, const uint8_t* bytes_dev) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (nsrc == 0 || cap_k == 0) return JY_OK;
  if (cap_byte % kArenaAlign) return eng->fail(JY_EINVAL, "cap_byte must be a multiple of 8");
  RouteArgs<1> A{};
  A.cap_k = cap_k;
  const u64 caps[1] = {cap_e};
  const u32 nc[1] = {3};
  route_layout(A, true, caps, nc);
  u64 rebase;
  JY_TRY(jy_arena_append_dev(eng, JY_TLOG, bytes_dev, (u64)nsrc * cap_byte, &rebase));
  if (cap_e)
    hipLaunchKernelGGL(k_rc_rebase, dim3(blocks_for((u64)nsrc * cap_e)), dim3(kThreads), 0, eng->stream, runs_dev,
                       nsrc, A.W, A.c[0].o_col[2], cap_e, rebase, cap_byte);
  JY_HIP(eng, hipGetLastError());
  for (u32 s = 0; s < nsrc; s++) {
    const u64* R = runs_dev + (u64)s * A.W;
    JY_TRY(jy_tlog_merge(eng, cap_k, reinterpret_cast<const u32*>(R + A.o_slot), R + A.o_kx, R + A.c[0].o_offs, cap_e,
                         R + A.c[0].o_col[0], R + A.c[0].o_col[1], R + A.c[0].o_col[2]));
  }
  return JY_OK;
}

int32_t jy_ujson_route_part(jy_engine* eng, uint64_t n, const uint32_t* owner, const uint32_t* slot,
                            const uint64_t* el_offs, uint64_t nel, const uint64_t* dots, const uint64_t* elems,
                            const uint64_t* vv_offs, uint64_t nvv, const uint64_t* vv, const uint64_t* cloud_offs,
                            uint64_t ncloud, const uint64_t* cloud, uint32_t nshards, uint64_t cap_k, uint64_t cap_e,
                            uint64_t cap_v, uint64_t cap_c, uint64_t key_base, int32_t mem, uint64_t* runs_dev,
                            uint64_t* hdr_dev, uint32_t* ovf_dev) {
  JY_HIP(eng, hipSetDevice(eng->device));
  JY_TRY(check_part(eng, n, nshards, cap_k, runs_dev, mem, owner));
  if (cap_k < 2) return eng->fail(JY_EINVAL, "cap_k must be at least 2 (the last record is a hole)");
  if (mem == JY_HOST && (!csr_ok(el_offs, n, nel) || !csr_ok(vv_offs, n, nvv) || !csr_ok(cloud_offs, n, ncloud)))
    return eng->fail(JY_EINVAL, "element / vv / cloud offsets are not CSRs of their totals");
  RouteArgs<3> A{};
  A.n = n;
  A.kbase = key_base;
  A.S = nshards;
  A.cap_k = cap_k;
  A.kfit = cap_k - 1;
  A.slack = 1;
  const u64 caps[3] = {cap_e, cap_v, cap_c};
  const u32 nc[3] = {2, 1, 1};
  route_layout(A, false, caps, nc);
  const void *dow = nullptr, *dsl = nullptr, *deo = nullptr, *dd = nullptr, *de = nullptr, *dvo = nullptr,
             *dv = nullptr, *dco = nullptr, *dc = nullptr;
  JY_TRY(jy_stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, owner, n * 4, mem, &dow));
  JY_TRY(jy_stage(eng, 1, slot, n * 4, mem, &dsl));
  JY_TRY(jy_stage(eng, 2, el_offs, (n + 1) * 8, mem, &deo));
  JY_TRY(jy_stage(eng, 3, dots, nel * 8, mem, &dd));
  JY_TRY(jy_stage(eng, 4, elems, nel * 8, mem, &de));
  JY_TRY(jy_stage(eng, 5, vv_offs, (n + 1) * 8, mem, &dvo));
  JY_TRY(jy_stage(eng, 6, vv, nvv * 8, mem, &dv));
  JY_TRY(jy_stage(eng, 7, cloud_offs, (n + 1) * 8, mem, &dco));
  JY_TRY(jy_stage(eng, 8, cloud, ncloud * 8, mem, &dc));
  JY_TRY(jy_stage_end(eng));
  A.owner = static_cast<const u32*>(dow);
  A.slot = static_cast<const u32*>(dsl);
  A.c[0].offs = static_cast<const u64*>(deo);
  A.c[0].nent_host = nel;
  A.c[0].col[0] = static_cast<const u64*>(dd);
  A.c[0].col[1] = static_cast<const u64*>(de);
  A.c[1].offs = static_cast<const u64*>(dvo);
  A.c[1].nent_host = nvv;
  A.c[1].col[0] = static_cast<const u64*>(dv);
  A.c[2].offs = static_cast<const u64*>(dco);
  A.c[2].nent_host = ncloud;
  A.c[2].col[0] = static_cast<const u64*>(dc);
  A.lr = -1;
  A.out = runs_dev;
  A.hdr = reinterpret_cast<unsigned long long*>(hdr_dev);
  A.ovf = ovf_dev;
  return route_part<3, false>(eng, A);
}

int32_t jy_ujson_converge_routed(jy_engine* eng, uint32_t nsrc, uint64_t cap_k, uint64_t cap_e, uint64_t cap_v,
                                 uint64_t cap_c, const uint64_t* runs_dev) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (nsrc == 0) return JY_OK;
  if (cap_k < 2) return eng->fail(JY_EINVAL, "cap_k must be at least 2 (the last record is a hole)");
  RouteArgs<3> A{};
  A.cap_k = cap_k;
  const u64 caps[3] = {cap_e, cap_v, cap_c};
  const u32 nc[3] = {2, 1, 1};
  route_layout(A, false, caps, nc);
  for (u32 s = 0; s < nsrc; s++) {
    const u64* R = runs_dev + (u64)s * A.W;
    JY_TRY(jy_ujson_merge(eng, cap_k, reinterpret_cast<const u32*>(R + A.o_slot), R + A.c[0].o_offs, cap_e,
                          R + A.c[0].o_col[0], R + A.c[0].o_col[1], R + A.c[1].o_offs, cap_v, R + A.c[1].o_col[0],
                          R + A.c[2].o_offs, cap_c, R + A.c[2].o_col[0]));
  }
  return JY_OK;
}

}  // extern "C"
