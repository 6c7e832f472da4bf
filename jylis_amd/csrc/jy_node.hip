// jy_node.hip -- the node: every GPU of one Jylis node behind one handle.
//
// Boundary (include/jylis_gpu.h, "the node"): one call per decoded peer batch
// replaces Database.converge_deltas (jylis/database.pony:50-51) ->
// RepoManager.converge_deltas -> RepoManagerCore.converge_deltas
// (jylis/repo_manager.pony:30-31,92-93) for the whole node.  Keys are
// hash-sharded over S engines (owner = jy_key_owner(key, S)); the
// reference holds every key on every node, so the exchange below has no
// counterpart there -- it is the intra-node analogue of
// Cluster.broadcast_deltas (cluster.pony:205-213).
//
// One converge call, per local shard (the batch cut into nlocal key ranges):
//
//   ingest     the shard's key range (staged through pinned memory, or in HBM)
//              is hashed on the device (k_nd_owner), stably partitioned by
//              owner (k_nd_count, a column-major look-back scan, k_nd_place:
//              no same-address global atomics), and every wire column is
//              written in owner order: key lengths and bytes, the per-key
//              columns, and each CSR level of the payload (TLOG entries and
//              their long value bytes, UJSON elements / vv / cloud, counter
//              cells) -- k_nd_seg_lens + scan + k_nd_seg_copy.  A value longer
//              than 8 bytes travels as its bytes in 8-byte granules; its
//              8-byte prefix and length travel as words (k_nd_val_head).
//   counts     per destination and granule (keys, key bytes, level elements),
//              exchanged with grouped ncclSend/ncclRecv (or transposed on the
//              host for the copy fabric) and read back: the one host
//              synchronisation of the exchange.  Sizes are exact: no fixed
//              capacities, no overflow rounds.
//   exchange   grouped ncclSend/ncclRecv of every wire column, source-major
//              into one receive buffer per column (RCCL over xGMI), or
//              device copies (JY_FABRIC_COPY: one process, shards may share a
//              GPU -- the single-GPU tests of the multi-shard path).
//   owner      the received keys are interned in the shard's device directory
//              (_data_for, repo_*.pony: create on miss); the received value
//              bytes are appended to its arena and their handles rebuilt; then
//              the engine's own merge kernels run: TREG (k_treg) and counters
//              (k_coo_max_keyed) over all sources at once -- LWW and max are
//              joins, a key two sources sent is exact -- TLOG (k_tlog) and
//              UJSON (k_ujson) one source after another (their device batches
//              name a key once).
//
// Roofline: the exchange moves (S - 1) / S of the batch over xGMI (7 links x
// ~153 GB/s per GPU at S = 8) and the ingest regroup reads the batch once and
// writes it once in HBM; the merges are the engine's.

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <initializer_list>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <type_traits>
#include <vector>

#include "jy_dscan.hpp"
#include "jy_internal.hpp"

namespace {

constexpr int kT = 256;
constexpr u32 kMaxS = JY_NODE_MAX_SHARDS;
constexpr int kMaxLvl = 3;           // CSR levels of a payload (UJSON: elements, vv, cloud)
constexpr int kMaxW = 2 + kMaxLvl;   // count granules: keys, key bytes, one per level
// read-back words after the counts: [0, 2) read2's, [2] the value-length
// verdict, [3] the long values' total (TotalHook), [8, 16) dev_words'
constexpr int kPinTail = 24;

u32 grid_of(u64 n) { return (u32)std::max<u64>(1, (n + kT - 1) / kT); }
u64 round8(u64 x) { return (x + 7) & ~7ull; }

// ---------------------------------------------------------------------------
// kernels: ingest

__global__ __launch_bounds__(kT) void k_nd_owner(const uint8_t* __restrict__ kb, const u64* __restrict__ ko, u64 obase,
                                                 u64 n, u32 S, u32* __restrict__ owner) {
  const u64 i = (u64)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const u64 a = ko[i];
  owner[i] = jy_dev_key_owner(kb + (a - obase), ko[i + 1] - a, S);
}

// per tile of kT items: items per owner (one LDS atomic per wave and owner)
__global__ __launch_bounds__(kT) void k_nd_count(const u32* __restrict__ owner, u64 n, u32 S, u64* __restrict__ tcnt) {
  __shared__ unsigned long long lc[kMaxS];
  for (u32 j = threadIdx.x; j < S; j += kT) lc[j] = 0;
  __syncthreads();
  const u64 i = (u64)blockIdx.x * kT + threadIdx.x;
  const bool valid = i < n;
  const u32 o = valid ? owner[i] : 0u;
  u64 pending = __ballot(valid);
  while (pending) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const u32 d = __shfl(o, leader);
    const u64 m = __ballot(valid && o == d);
    if (__lane_id() == (u32)leader) atomicAdd(&lc[d], (unsigned long long)__popcll(m));
    pending &= ~m;
  }
  __syncthreads();
  u64* row = tcnt + (u64)blockIdx.x * S;
  for (u32 j = threadIdx.x; j < S; j += kT) row[j] = lc[j];
}

// after the column-major exclusive scan of tcnt: where every owner's items
// begin in owner order (kbeg[S] = n)
__global__ void k_nd_kbeg(const u64* __restrict__ tcnt, u64 ntiles, u32 S, u64* __restrict__ kbeg) {
  const u32 d = threadIdx.x;
  if (d < S) kbeg[d] = tcnt[d];
  if (d == S) kbeg[S] = tcnt[ntiles * S];
}

// stable placement: perm[position in owner order] = input index
__global__ __launch_bounds__(kT) void k_nd_place(const u32* __restrict__ owner, u64 n, u32 S,
                                                 const u64* __restrict__ tcnt, u32* __restrict__ perm) {
  __shared__ u32 wt[kT / 64][kMaxS];
  for (u32 j = threadIdx.x; j < S; j += kT)
#pragma unroll
    for (int w = 0; w < kT / 64; w++) wt[w][j] = 0;
  __syncthreads();
  const u64 i = (u64)blockIdx.x * kT + threadIdx.x;
  const int lane = __lane_id(), wv = threadIdx.x >> 6;
  const bool valid = i < n;
  const u32 o = valid ? owner[i] : 0u;
  u32 rk = 0;
  u64 pending = __ballot(valid);
  while (pending) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const u32 d = __shfl(o, leader);
    const bool mine = valid && o == d;
    const u64 m = __ballot(mine);
    if (mine) rk = (u32)__popcll(m & ((1ull << lane) - 1));
    if (lane == leader) wt[wv][d] = (u32)__popcll(m);
    pending &= ~m;
  }
  __syncthreads();
  if (!valid) return;
  u64 p = tcnt[(u64)blockIdx.x * S + o] + rk;
  for (int w = 0; w < wv; w++) p += wt[w][o];
  perm[p] = (u32)i;
}

// segments of an item: [start, start + len) copied into plen >= len slots
// (the tail zero).  SegCsr: a CSR level (offs indexed by item, minus obase).
// SegLong: a value's bytes when it is longer than 8 (else nothing), padded to
// 8-byte granules (the receiver's arena keeps long values on granules).
struct SegCsr {
  static constexpr bool kGranules = false;
  const u64* offs;
  u64 obase;
  __device__ __forceinline__ void get(u64 i, u64& start, u64& len, u64& plen) const {
    const u64 a = offs[i];
    start = a - obase;
    len = plen = offs[i + 1] - a;
  }
};
struct SegLong {
  static constexpr bool kGranules = true;  // output segments are whole 8-byte granules on 8-byte offsets
  const u64* offs;
  u64 obase;
  __device__ __forceinline__ void get(u64 i, u64& start, u64& len, u64& plen) const {
    const u64 a = offs[i], l = offs[i + 1] - a;
    start = a - obase;
    len = l > 8 ? l : 0;
    plen = l > 8 ? (l + 7) & ~7ull : 0;
  }
};

// output item j's segment length (item perm[j]); lens[n] = 0 for the scan
template <class Seg>
__global__ __launch_bounds__(kT) void k_nd_seg_lens(u64 n, const u32* __restrict__ perm, Seg sg, u64* __restrict__ lens) {
  const u64 j = (u64)blockIdx.x * kT + threadIdx.x;
  if (j > n) return;
  if (j == n) {
    lens[n] = 0;
    return;
  }
  u64 st, len, plen;
  sg.get(perm[j], st, len, plen);
  lens[j] = plen;
}

// column readers of the payload
template <int N>
struct InU64 {
  const u64* p[N];
  __device__ __forceinline__ u64 get(int c, u64 k) const { return p[c][k]; }
};
struct InBytes {
  const uint8_t* p;
};
// counter cells: (sign << 16 | col) and the value, so every column is a word
struct InCells {
  const uint8_t* sign;
  const u16* col;
  const u64* val;
  __device__ __forceinline__ u64 get(int c, u64 k) const {
    if (c == 1) return val[k];
    return ((u64)(sign ? sign[k] : 0) << 16) | col[k];
  }
};

// output item j (thread): its segment copied to newoffs[j]; esrc (optional)
// gets each copied element's source index (the next level's item index)
template <int N, class In, class Seg>
__global__ __launch_bounds__(kT) void k_nd_seg_copy(u64 n, const u32* __restrict__ perm, Seg sg,
                                                    const u64* __restrict__ newoffs, In in, u64* o0, u64* o1, u64* o2,
                                                    u32* __restrict__ esrc) {
  const u64 j = (u64)blockIdx.x * kT + threadIdx.x;
  if (j >= n) return;
  u64 st, len, plen;
  sg.get(perm[j], st, len, plen);
  u64* out[3] = {o0, o1, o2};
  const u64 d = newoffs[j];
  for (u64 r = 0; r < len; r++) {
#pragma unroll
    for (int c = 0; c < N; c++) out[c][d + r] = in.get(c, st + r);
    if (esrc) esrc[d + r] = (u32)(st + r);
  }
}

template <class Seg>
__global__ __launch_bounds__(kT) void k_nd_seg_bytes(u64 n, const u32* __restrict__ perm, Seg sg,
                                                     const u64* __restrict__ newoffs, const uint8_t* __restrict__ in,
                                                     uint8_t* __restrict__ out) {
  const u64 j = (u64)blockIdx.x * kT + threadIdx.x;
  if (j >= n) return;
  u64 st, len, plen;
  sg.get(perm[j], st, len, plen);
  const u64 d = newoffs[j];
  if constexpr (Seg::kGranules) {  // word stores, two aligned word loads per granule at most
    u64* o = reinterpret_cast<u64*>(out + d);
    for (u64 q = 0; q < plen / 8; q++) o[q] = jy_ld8u(in + st + 8 * q, len - 8 * q);
  } else {
    for (u64 r = 0; r < plen; r++) out[d + r] = r < len ? in[st + r] : 0;
  }
}

// per-key word columns in owner order
template <int N>
__global__ __launch_bounds__(kT) void k_nd_perm(u64 n, const u32* __restrict__ perm, InU64<N> in, u64* o0, u64* o1,
                                                u64* o2) {
  const u64 j = (u64)blockIdx.x * kT + threadIdx.x;
  if (j >= n) return;
  const u32 i = perm[j];
  u64* out[3] = {o0, o1, o2};
#pragma unroll
  for (int c = 0; c < N; c++) out[c][j] = in.get(c, i);
}

// a value's 8-byte big-endian prefix (zero padded) and its length, item perm[j]
__global__ __launch_bounds__(kT) void k_nd_val_head(u64 n, const u32* __restrict__ perm, const u64* __restrict__ vo,
                                                    u64 vbase, const uint8_t* __restrict__ vb, u64* __restrict__ pre,
                                                    u64* __restrict__ vlen) {
  const u64 j = (u64)blockIdx.x * kT + threadIdx.x;
  if (j >= n) return;
  const u32 i = perm[j];
  const u64 a = vo[i], l = vo[i + 1] - a;
  pre[j] = __builtin_bswap64(jy_ld8u(vb + (a - vbase), l));  // big-endian: byte 0 most significant
  vlen[j] = l;
}

// per destination d and granule: keys, key bytes, then the elements of each
// level (a level's items are the keys or the elements of its parent level)
struct LvlArgs {
  const u64* offs[kMaxLvl];  // owner-order offsets over the parent's items
  int parent[kMaxLvl];       // -1: keys
  u32 nl;
};
__global__ void k_nd_counts(u32 S, const u64* __restrict__ kbeg, const u64* __restrict__ kofs, LvlArgs L,
                            u64* __restrict__ cnt) {
  const u32 d = threadIdx.x;
  if (d >= S) return;
  const u32 W = 2 + L.nl;
  const u64 klo = kbeg[d], khi = kbeg[d + 1];
  cnt[d * W + 0] = khi - klo;
  cnt[d * W + 1] = kofs[khi] - kofs[klo];
  u64 lo[kMaxLvl], hi[kMaxLvl];
  for (u32 l = 0; l < L.nl; l++) {
    const int p = L.parent[l];
    const u64 plo = p < 0 ? klo : lo[p], phi = p < 0 ? khi : hi[p];
    lo[l] = L.offs[l][plo];
    hi[l] = L.offs[l][phi];
    cnt[d * W + 2 + l] = hi[l] - lo[l];
  }
}

// ---------------------------------------------------------------------------
// kernels: owner side

// per-source local CSR offsets (the engine's merges take batches whose
// offsets start at 0): out[kb[s] + s + j] = offs[kb[s] + j] - offs[kb[s]]
struct SrcRanges {
  u64 kb[kMaxS + 1];
  u32 S;
};
__global__ __launch_bounds__(kT) void k_nd_local_offs(const u64* __restrict__ offs, u64 n, SrcRanges R,
                                                      u64* __restrict__ out) {
  const u64 t = (u64)blockIdx.x * kT + threadIdx.x;
  if (t >= n + R.S) return;
  u32 s = R.S - 1;
  while (s > 0 && t < R.kb[s] + s) s--;
  const u64 j = t - R.kb[s] - s;
  out[t] = offs[R.kb[s] + j] - offs[R.kb[s]];
}

__global__ __launch_bounds__(kT) void k_nd_plen(u64 n, const u64* __restrict__ vlen, u64* __restrict__ plen) {
  const u64 j = (u64)blockIdx.x * kT + threadIdx.x;
  if (j > n) return;
  const u64 l = j < n ? vlen[j] : 0;
  plen[j] = l > 8 ? (l + 7) & ~7ull : 0;
}

// value handles in the owner's arena: long values at rebase + their offset in
// the received byte block (granule aligned), short ones by length alone
__global__ __launch_bounds__(kT) void k_nd_lr(u64 n, const u64* __restrict__ vlen, const u64* __restrict__ voff,
                                              u64 rebase, u64* __restrict__ lr) {
  const u64 j = (u64)blockIdx.x * kT + threadIdx.x;
  if (j >= n) return;
  const u64 l = vlen[j] & JY_LR_LEN_MASK;
  lr[j] = l > 8 ? ((rebase + voff[j]) << JY_LR_LEN_BITS) | l : l;
}

// device inputs: the longest value over 16 MiB, if any (the host form refuses
// such a batch in values_check; a handle's length has 24 bits)
__global__ __launch_bounds__(kT) void k_nd_maxlen(const u64* __restrict__ vo, u64 n, unsigned long long* __restrict__ out) {
  const u64 i = (u64)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const u64 l = vo[i + 1] - vo[i];
  if (l > JY_MAX_VALUE_LEN) atomicMax(out, (unsigned long long)l);
}

// up to kWords device words gathered into pinned host memory by one launch
// (an 8-byte hipMemcpyAsync costs the GPU a ~5-us copy kernel each); the word
// at `reset` (a value-length verdict) is zeroed for the next call once read
constexpr int kWords = 8;
struct Words {
  const u64* src[kWords];
  u32 n;
  int reset;
};
__global__ __launch_bounds__(64) void k_nd_words(Words W, u64* __restrict__ dst) {
  const u32 i = threadIdx.x;
  if (i >= W.n) return;
  const u64 v = *W.src[i];
  __hip_atomic_store(dst + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if ((int)i == W.reset) *const_cast<u64*>(W.src[i]) = 0;
}

__global__ __launch_bounds__(kT) void k_nd_cells(u64 n, const u64* __restrict__ packed, uint8_t* __restrict__ sign,
                                                 u16* __restrict__ col) {
  const u64 j = (u64)blockIdx.x * kT + threadIdx.x;
  if (j >= n) return;
  const u64 w = packed[j];
  sign[j] = (uint8_t)(w >> 16);
  col[j] = (u16)w;
}

// ---------------------------------------------------------------------------
// kernels: one shard (S = 1) -- the owner reads the staged inputs in place

// value heads: the 8-byte big-endian prefix, and the padded length of a long
// value (plen[n] = 0: the scan's last input)
// Values in tiles of kValTile (kValU per lane, lanes on consecutive values of
// a row): k_nd1_head writes each value's big-endian prefix and each tile's
// long-value granule bytes; those few tile sums are scanned; k_nd1_long
// rescans its tile's lengths in the workgroup from the tile's offset.  (A
// scan over every value's length took ~51 us of an 8.39M-key node TREG call
// -- three launches over 8.39M words -- and wrote and re-read 67 MB.)
constexpr int kValU = 4;
constexpr u64 kValTile = (u64)kT * kValU;
__device__ __forceinline__ u64 long_bytes(u64 l) { return l > 8 ? (l + 7) & ~7ull : 0; }

__global__ __launch_bounds__(kT) void k_nd1_head(u64 n, const u64* __restrict__ vo, u64 vbase,
                                                 const uint8_t* __restrict__ vb, u64* __restrict__ pre,
                                                 u64* __restrict__ tsum) {
  __shared__ u64 red[kT / 64];
  const u64 t0 = (u64)blockIdx.x * kValTile;
  u64 acc = 0;
#pragma unroll
  for (int u = 0; u < kValU; u++) {
    const u64 j = t0 + (u64)u * kT + threadIdx.x;
    if (j < n) {
      const u64 a = vo[j], l = vo[j + 1] - a;
      pre[j] = __builtin_bswap64(jy_ld8u(vb + (a - vbase), l));
      acc += long_bytes(l);
    }
  }
  u64 tot;
  jyscan::block_excl<kT, u64>(acc, red, tot);
  if (threadIdx.x == 0) {
    tsum[blockIdx.x] = tot;
    if (blockIdx.x == 0) tsum[gridDim.x] = 0;  // the scan's last input
  }
}

// long values' bytes into the arena (dst = the reserved tail; the tile's
// offset from the scan of the tile sums, each value's within the tile from a
// workgroup scan in value order; 8-byte granules, word stores) and every
// value's handle
__global__ __launch_bounds__(kT) void k_nd1_long(u64 n, const u64* __restrict__ vo, u64 vbase,
                                                 const uint8_t* __restrict__ vb, const u64* __restrict__ toff,
                                                 uint8_t* __restrict__ dst, u64 rebase, u64* __restrict__ lr) {
  __shared__ u64 red[kT / 64];
  const u64 t0 = (u64)blockIdx.x * kValTile;
  u64 carry = toff[blockIdx.x];
#pragma unroll
  for (int u = 0; u < kValU; u++) {
    const u64 j = t0 + (u64)u * kT + threadIdx.x;
    u64 a = 0, l = 0;
    if (j < n) a = vo[j], l = vo[j + 1] - a;
    u64 tot;
    const u64 d = carry + jyscan::block_excl<kT, u64>(long_bytes(l), red, tot);
    carry += tot;
    if (j >= n) continue;
    if (l <= 8) {
      lr[j] = l;
      continue;
    }
    u64* o = reinterpret_cast<u64*>(dst + d);
    const uint8_t* src = vb + (a - vbase);
    for (u64 q = 0; q < (l + 7) / 8; q++) o[q] = jy_ld8u(src + 8 * q, l - 8 * q);
    lr[j] = ((rebase + d) << JY_LR_LEN_BITS) | l;
  }
}

// the value tiles' long-byte sums scanned by one workgroup (toff[j],
// exclusive; toff[nt] the total, also stored to mapped pinned memory for the
// host).  A few thousand tiles per call (8.39M values: 8,192): no look-back.
// Rows of 256 consecutive sums, kTScanU rows' loads issued together.  (A
// 1024-thread workgroup waited up to 245 us for a CU with 16 free wave slots
// beside the key probe's workgroups.)
constexpr int kTScanThreads = 256, kTScanU = 8;
__global__ __launch_bounds__(kTScanThreads) void k_nd1_tscan(const u64* __restrict__ tsum, u64 nt,
                                                             u64* __restrict__ toff, u64* __restrict__ total_pin) {
  __shared__ u64 red[kTScanThreads / 64];
  u64 carry = 0;
  for (u64 c0 = 0; c0 < nt; c0 += (u64)kTScanThreads * kTScanU) {
    u64 v[kTScanU];
#pragma unroll
    for (int u = 0; u < kTScanU; u++) {
      const u64 i = c0 + (u64)u * kTScanThreads + threadIdx.x;
      v[u] = i < nt ? tsum[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < kTScanU; u++) {
      const u64 i = c0 + (u64)u * kTScanThreads + threadIdx.x;
      u64 tot;
      const u64 x = jyscan::block_excl<kTScanThreads, u64>(v[u], red, tot);
      if (i < nt) toff[i] = carry + x;
      carry += tot;
    }
  }
  if (threadIdx.x == 0) {
    toff[nt] = carry;
    __hip_atomic_store(total_pin, carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// a CSR's offsets from 0: out[j] = offs[j] - offs[0], j <= n
__global__ __launch_bounds__(kT) void k_nd1_rebase(u64 n, const u64* __restrict__ offs, u64* __restrict__ out) {
  const u64 j = (u64)blockIdx.x * kT + threadIdx.x;
  if (j <= n) out[j] = offs[j] - offs[0];
}

}  // namespace

// ---------------------------------------------------------------------------
// host side

namespace {

// node-owned device buffers (hipMalloc: RCCL may address them from a peer in
// one process; the engines' stream-ordered pools are not peer-mapped)
enum Buf {
  B_OWNER, B_PERM, B_TCNT, B_KBEG, B_CNT, B_KLEN, B_KOFF, B_KBYTES, B_F0, B_F1, B_F2,
  B_LLEN0, B_LLEN1, B_LLEN2, B_LOFF0, B_LOFF1, B_LOFF2,
  B_LC00, B_LC01, B_LC10, B_LC11, B_LC20, B_LC21, B_ESRC,
  R_KLEN, R_KBYTES, R_F0, R_F1, R_F2, R_LC00, R_LC01, R_LC10, R_LC11, R_LC20, R_LC21,
  R_KOFF, R_SLOTS, R_LOFF0, R_LOFF1, R_LOFF2, R_LOC0, R_LOC1, R_LOC2, R_PLEN, R_VOFF, R_LR, R_AUX0, R_AUX1, R_AUX2,
  X_BUF0, X_BUF1,
  kNumBufs
};

struct NdBuf {
  void* p = nullptr;
  u64 bytes = 0;
};

struct NdShard {
  u32 rank = 0;
  int dev = 0;
  jy_engine* eng = nullptr;
  ncclComm_t comm = nullptr;
  hipStream_t xs = nullptr;    // exchange stream of the block converge
  // read-back stream: the caller's input words (k_nd_words) and the value
  // length check (k_nd_maxlen) need none of the engine stream's earlier work,
  // so a call reads them while the previous call's kernels still run
  hipStream_t rs = nullptr;
  hipEvent_t ev_rs_in = nullptr;   // the engine stream's point the read-back stream's value work starts after
  hipEvent_t ev_rs_out = nullptr;  // the value handles are written (the engine stream waits before the merge)
  hipEvent_t ev_in = nullptr;  // this shard's send columns are ready (copy fabric)
  hipEvent_t ev_out = nullptr; // this shard's receives have landed (copy fabric)
  hipEvent_t ev_x[2] = {nullptr, nullptr}, ev_m[2] = {nullptr, nullptr};
  NdBuf b[kNumBufs];
  u64* pin = nullptr;  // pinned: [2][kMaxS][kMaxW] send / recv counts, then kPinTail words of readbacks
  u64* pin_dev = nullptr;  // the same memory, as the device addresses it (k_nd_words writes there)
  u64* mlw = nullptr;      // a value-length verdict word queued by values_dev_enqueue, not yet read
  u64* mlw_buf = nullptr;  // the verdict word's buffer (zero between calls once set up)
  bool mlw_zero = false;
  // the current call's sizes
  u64 n = 0;                 // keys ingested
  u64 tot[kMaxW] = {};       // elements per granule ingested (send side), upper bounds
  u64 rtot[kMaxW] = {};      // received per granule
};

}  // namespace

// ---- the node's executor (round 5) ----
// A converge call validates its arguments, copies host inputs into a pinned
// block the node owns (parallel host copies) and queues a job; ONE worker
// thread per node runs the jobs in call order.  So a call returns without
// waiting for the GPU (the exchange's count read-back, the key directory's
// miss count and the CSR ends of device inputs are the worker's waits, not
// the caller's), and every call of every CRDT type -- the five RepoManager
// actors of one Jylis process share ONE node -- issues its RCCL groups from
// the same thread in one order: one communicator, no interleaving.
namespace {

constexpr int32_t kPinned = 2;  // internal mem mode: host memory the node owns (pinned), DMA'd in place
constexpr int kJobDepth = 3;    // pinned blocks: jobs queued or running at once (a caller waits beyond)
inline bool on_host(int32_t mem) { return mem != JY_DEVICE; }

enum JobKind { K_COUNTER, K_TREG, K_TLOG, K_UJSON, K_BLOCK };
struct NdJob {
  int kind = 0;
  int32_t type = 0, mem = JY_DEVICE;
  int32_t fty = 0;  // the CRDT type whose state the job changes (per-type fences)
  u64 n = 0;
  const void* a[11] = {};  // the call's arrays (host inputs: rebased into the pinned block)
  int pin = -1;
  u32 ncols = 0, slot0 = 0, nslots = 0;  // K_BLOCK
  std::vector<u16> cols;
};
struct NdPin {
  void* p = nullptr;
  u64 bytes = 0;
  bool busy = false;
  std::vector<hipEvent_t> ev;  // per local shard: the job's DMAs out of this block are done
};

}  // namespace

struct jy_node {
  jy_node_config cfg;
  u32 S = 0, nlocal = 0, rank0 = 0, fabric = JY_FABRIC_RCCL;
  std::vector<NdShard> sh;
  std::string werr;  // the worker's (moved to the reporting caller's when a call reports it)
  u64 stats[5] = {};
  u32 nrep = 0;  // replica columns registered (host-side checks of counter cells)
  // executor
  std::mutex mu;  // held while a job runs, by jy_node_lock holders, and by locked entry points
  std::mutex qmu;
  std::condition_variable qcv, dcv;
  std::deque<NdJob> q;
  u64 submitted = 0, finished = 0;
  u64 sub_t[JY_NTYPES] = {}, fin_t[JY_NTYPES] = {};  // the same per CRDT type (jy_node_lock_type)
  bool arena_gc = false;  // jy_node_arena_gc: the worker reclaims TREG / TLOG arenas after their jobs
  // callers waiting in jy_node_lock[_type]: the worker lets them in before it
  // takes the next job (std::mutex is not fair: a worker with a long queue
  // would otherwise take the lock back every time and starve a reader)
  std::atomic<int> lock_waiters{0};
  std::vector<u64> arena_live;  // [local shard][2]: bytes kept by the last collection (TREG, TLOG)
  // replica columns registered on every shard (jy_node_replica_col): a
  // known id is answered from here, under its own small mutex, without
  // waiting for the worker
  std::mutex rmu;
  std::unordered_map<u64, u32> rep;
  bool stop = false, inline_jobs = false;
  bool regroup_one = false;  // JY_NODE_REGROUP_ONE=1: S = 1 through the regroup + exchange (A/B, tests)
  std::thread worker;
  std::thread::id wid;
  int32_t aerr = JY_OK;  // first failure of a queued job, reported by the next call
  std::string aerr_msg;
  NdPin pins[kJobDepth];
  // callers' errors are per calling thread (errno-like, jy_node_last_error):
  // the five repos of a process call one node from their own threads
  static std::string& caller_err() {
    static thread_local std::string e;
    return e;
  }
  int32_t fail(int32_t code, const std::string& m) {
    (std::this_thread::get_id() == wid ? werr : caller_err()) = m;
    return code;
  }
};

namespace {
void exec_start(jy_node* nd);
void exec_stop(jy_node* nd);
int32_t exec_fence(jy_node* nd);  // every queued job issued; a queued job's failure, if any
int32_t exec_fence_type(jy_node* nd, int32_t type);  // the same for one CRDT type's jobs
int32_t exec_pending(jy_node* nd);                   // a queued job's failure, without waiting
}  // namespace

namespace {

#define ND_HIP(nd, call)                                                                                  \
  do {                                                                                                    \
    hipError_t e_ = (call);                                                                               \
    if (e_ != hipSuccess) return (nd)->fail(JY_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define ND_NCCL(nd, call)                                                                                     \
  do {                                                                                                        \
    ncclResult_t r_ = (call);                                                                                 \
    if (r_ != ncclSuccess) return (nd)->fail(JY_EHIP, std::string(#call) + ": " + ncclGetErrorString(r_)); \
  } while (0)
// an engine call inside a node call: its error becomes the node's
#define ND_ENG(nd, sh, expr)                                                    \
  do {                                                                          \
    int32_t rc_ = (expr);                                                       \
    if (rc_ != JY_OK) return (nd)->fail(rc_, std::string("shard ") +            \
                                                 std::to_string((sh).rank) + ": " + (sh).eng->err); \
  } while (0)

// an RCCL group that is ended on every exit: an error return inside an open
// group would leave this thread's group depth raised, and the next node call's
// sends and receives would pile into a group that never launches
struct NcclGroup {
  bool open = false;
  ncclResult_t start() {
    const ncclResult_t r = ncclGroupStart();
    open = r == ncclSuccess;
    return r;
  }
  ncclResult_t end() {
    open = false;
    return ncclGroupEnd();
  }
  ~NcclGroup() {
    if (open) ncclGroupEnd();
  }
};

int32_t buf(jy_node* nd, NdShard& sh, int idx, u64 bytes, void** out) {
  NdBuf& b = sh.b[idx];
  if (b.bytes < bytes || !b.p) {
    ND_HIP(nd, hipSetDevice(sh.dev));
    // growth: whatever still reads the old buffer has to finish
    ND_HIP(nd, hipStreamSynchronize(sh.eng->stream));
    if (sh.xs) ND_HIP(nd, hipStreamSynchronize(sh.xs));
    if (sh.rs) ND_HIP(nd, hipStreamSynchronize(sh.rs));
    if (b.p) ND_HIP(nd, hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    const u64 nb = std::max<u64>(((bytes + bytes / 4) + 4095) & ~4095ull, 4096);
    ND_HIP(nd, hipMalloc(&b.p, nb));
    b.bytes = nb;
  }
  *out = b.p;
  return JY_OK;
}
template <class T>
int32_t bufT(jy_node* nd, NdShard& sh, int idx, u64 count, T** out) {
  void* p;
  JY_TRY(buf(nd, sh, idx, count * sizeof(T), &p));
  *out = static_cast<T*>(p);
  return JY_OK;
}

// two words read back from device (or host) memory: a CSR's first and last offset
// device words read with one launch and one wait; a queued value-length
// verdict (values_dev_enqueue) rides along into the pinned verdict word
int32_t dev_words(jy_node* nd, NdShard& sh, std::initializer_list<const u64*> src, u64* out) {
  Words W{};
  for (const u64* p : src) {
    if (W.n == (u32)kWords) return nd->fail(JY_EINVAL, "node: too many device words in one read-back");
    W.src[W.n++] = p;
  }
  const u32 nsrc = W.n;
  W.reset = -1;
  if (sh.mlw) {
    if (W.n == (u32)kWords) return nd->fail(JY_EINVAL, "node: too many device words in one read-back");
    W.reset = (int)W.n;
    W.src[W.n++] = sh.mlw;
  }
  u64* pw = sh.pin + 2 * kMaxS * kMaxW + 8;
  hipLaunchKernelGGL(k_nd_words, dim3(1), dim3(64), 0, sh.rs, W, sh.pin_dev + 2 * kMaxS * kMaxW + 8);
  ND_HIP(nd, hipGetLastError());
  ND_HIP(nd, hipStreamSynchronize(sh.rs));
  for (u32 k = 0; k < nsrc; k++) out[k] = pw[k];
  if (sh.mlw) {
    sh.pin[2 * kMaxS * kMaxW + 2] = pw[nsrc];
    sh.mlw = nullptr;
  }
  return JY_OK;
}

int32_t read2(jy_node* nd, NdShard& sh, const u64* a, const u64* b, int32_t mem, u64& x, u64& y) {
  if (on_host(mem)) {
    x = *a;
    y = *b;
    return JY_OK;
  }
  u64 w[2];
  JY_TRY(dev_words(nd, sh, {a, b}, w));
  x = w[0];
  y = w[1];
  return JY_OK;
}

// ---- a CSR level of the ingest: item offsets (n_items + 1, relative to the
// staged elements by obase) and its element columns
struct Level {
  const u64* offs = nullptr;  // device, indexed by item (relative)
  u64 obase = 0;              // subtracted from offs to index the staged columns
  u64 nel = 0;                // elements of this chunk (upper bound for SegLong)
  int parent = -1;            // -1: items are keys; else the level whose elements they are
  bool longval = false;       // items' value bytes (SegLong) instead of a CSR of words
};

struct Ingest {
  // keys of the chunk
  const uint8_t* kb = nullptr;
  const u64* ko = nullptr;
  u64 kobase = 0, nkb = 0;
};

// owners, the stable partition and the key columns (lens, offsets, bytes)
int32_t ingest_keys(jy_node* nd, NdShard& sh, const Ingest& in) {
  jy_engine* eng = sh.eng;
  const u64 n = sh.n, S = nd->S;
  const u64 nt = std::max<u64>(1, (n + kT - 1) / kT);
  u32 *owner, *perm;
  u64 *tcnt, *kbeg, *klen, *koff;
  uint8_t* kbytes;
  JY_TRY(bufT(nd, sh, B_OWNER, std::max<u64>(n, 1), &owner));
  JY_TRY(bufT(nd, sh, B_PERM, std::max<u64>(n, 1), &perm));
  JY_TRY(bufT(nd, sh, B_TCNT, nt * S + 1, &tcnt));
  JY_TRY(bufT(nd, sh, B_KBEG, S + 1, &kbeg));
  JY_TRY(bufT(nd, sh, B_KLEN, n + 1, &klen));
  JY_TRY(bufT(nd, sh, B_KOFF, n + 1, &koff));
  JY_TRY(bufT(nd, sh, B_KBYTES, std::max<u64>(in.nkb, 1), &kbytes));
  if (n == 0) {
    ND_HIP(nd, hipMemsetAsync(kbeg, 0, (S + 1) * 8, eng->stream));
    ND_HIP(nd, hipMemsetAsync(koff, 0, 8, eng->stream));
    return JY_OK;
  }
  hipLaunchKernelGGL(k_nd_owner, dim3(grid_of(n)), dim3(kT), 0, eng->stream, in.kb, in.ko, in.kobase, n, (u32)S, owner);
  hipLaunchKernelGGL(k_nd_count, dim3((u32)nt), dim3(kT), 0, eng->stream, (const u32*)owner, n, (u32)S, tcnt);
  ND_HIP(nd, hipGetLastError());
  ND_ENG(nd, sh, (jydscan::scan<jydscan::OpSum, false>(eng, nt * S + 1, jydscan::LdColMajor{tcnt, nt, S},
                                                       jydscan::StColMajor{tcnt, nt, S})));
  hipLaunchKernelGGL(k_nd_kbeg, dim3(1), dim3(128), 0, eng->stream, (const u64*)tcnt, nt, (u32)S, kbeg);
  hipLaunchKernelGGL(k_nd_place, dim3((u32)nt), dim3(kT), 0, eng->stream, (const u32*)owner, n, (u32)S,
                     (const u64*)tcnt, perm);
  const SegCsr ks{in.ko, in.kobase};
  hipLaunchKernelGGL(k_nd_seg_lens<SegCsr>, dim3(grid_of(n + 1)), dim3(kT), 0, eng->stream, n, (const u32*)perm, ks,
                     klen);
  ND_HIP(nd, hipGetLastError());
  ND_ENG(nd, sh, jy_scan_u64(eng, klen, koff, n));
  hipLaunchKernelGGL(k_nd_seg_bytes<SegCsr>, dim3(grid_of(n)), dim3(kT), 0, eng->stream, n, (const u32*)perm, ks,
                     (const u64*)koff, in.kb, kbytes);
  ND_HIP(nd, hipGetLastError());
  return JY_OK;
}

// the counts of every destination and granule (device [S][W] at B_CNT)
int32_t ingest_counts(jy_node* nd, NdShard& sh, const Level* L, u32 nl) {
  u64* cnt;
  JY_TRY(bufT(nd, sh, B_CNT, 2 * kMaxS * kMaxW, &cnt));
  LvlArgs A{};
  A.nl = nl;
  for (u32 l = 0; l < nl; l++) {
    A.offs[l] = static_cast<const u64*>(sh.b[B_LOFF0 + l].p);
    A.parent[l] = L[l].parent;
  }
  hipLaunchKernelGGL(k_nd_counts, dim3(1), dim3(kMaxS), 0, sh.eng->stream, nd->S,
                     (const u64*)sh.b[B_KBEG].p, (const u64*)sh.b[B_KOFF].p, A, cnt);
  ND_HIP(nd, hipGetLastError());
  return JY_OK;
}

// one level in owner order: lengths, offsets and (for word levels) its
// columns through `in`; `items` = the parent's output items, `perm` maps them
// to input items (keys: B_PERM; a nested level: the parent's element sources)
template <int N, class In>
int32_t ingest_level(jy_node* nd, NdShard& sh, u32 l, const Level& L, u64 items, const u32* perm, const In& in,
                     bool want_src) {
  jy_engine* eng = sh.eng;
  u64 *len, *off;
  JY_TRY(bufT(nd, sh, B_LLEN0 + l, items + 1, &len));
  JY_TRY(bufT(nd, sh, B_LOFF0 + l, items + 1, &off));
  const u64 cap = L.longval ? round8(L.nel) + 8 * items : L.nel;  // padded bytes bound
  sh.tot[2 + l] = cap;
  void* unused;
  if (items == 0) {
    ND_HIP(nd, hipMemsetAsync(off, 0, 8, eng->stream));
    for (int c = 0; c < N; c++) JY_TRY(buf(nd, sh, B_LC00 + 2 * l + c, 8, &unused));
    if (want_src) JY_TRY(buf(nd, sh, B_ESRC, 8, &unused));
    return JY_OK;
  }
  if constexpr (std::is_same<In, InBytes>::value) {
    const SegLong sg{L.offs, L.obase};
    hipLaunchKernelGGL(k_nd_seg_lens<SegLong>, dim3(grid_of(items + 1)), dim3(kT), 0, eng->stream, items, perm, sg, len);
    ND_HIP(nd, hipGetLastError());
    ND_ENG(nd, sh, jy_scan_u64(eng, len, off, items));
    uint8_t* o;
    JY_TRY(bufT(nd, sh, B_LC00 + 2 * l, std::max<u64>(cap, 1), &o));
    hipLaunchKernelGGL(k_nd_seg_bytes<SegLong>, dim3(grid_of(items)), dim3(kT), 0, eng->stream, items, perm, sg,
                       (const u64*)off, in.p, o);
    ND_HIP(nd, hipGetLastError());
    return JY_OK;
  } else {
    const SegCsr sg{L.offs, L.obase};
    hipLaunchKernelGGL(k_nd_seg_lens<SegCsr>, dim3(grid_of(items + 1)), dim3(kT), 0, eng->stream, items, perm, sg,
                       len);
    ND_HIP(nd, hipGetLastError());
    ND_ENG(nd, sh, jy_scan_u64(eng, len, off, items));
    u64* o[3] = {nullptr, nullptr, nullptr};
    for (int c = 0; c < N; c++) JY_TRY(bufT(nd, sh, B_LC00 + 2 * l + c, std::max<u64>(L.nel, 1), &o[c]));
    u32* src = nullptr;
    if (want_src) JY_TRY(bufT(nd, sh, B_ESRC, std::max<u64>(L.nel, 1), &src));
    hipLaunchKernelGGL((k_nd_seg_copy<N, In, SegCsr>), dim3(grid_of(items)), dim3(kT), 0, eng->stream, items, perm,
                       sg, (const u64*)off, in, o[0], o[1], o[2], src);
    ND_HIP(nd, hipGetLastError());
    return JY_OK;
  }
}

// per-key word columns in owner order (B_F0..)
template <int N>
int32_t ingest_fixed(jy_node* nd, NdShard& sh, const InU64<N>& in, int first = 0) {
  u64* o[3] = {nullptr, nullptr, nullptr};
  for (int c = 0; c < N; c++) JY_TRY(bufT(nd, sh, B_F0 + first + c, std::max<u64>(sh.n, 1), &o[c]));
  if (sh.n == 0) return JY_OK;
  hipLaunchKernelGGL((k_nd_perm<N>), dim3(grid_of(sh.n)), dim3(kT), 0, sh.eng->stream, sh.n,
                     (const u32*)sh.b[B_PERM].p, in, o[0], o[1], o[2]);
  ND_HIP(nd, hipGetLastError());
  return JY_OK;
}

// ---- the exchange ----
// a wire column: granule (0 keys, 1 key bytes, 2 + l level l), element size,
// send and receive buffers
struct Wire {
  int gran, esize, sidx, ridx;
};

// The payload schedule of one shard (pure host logic, shared with
// jy_node_exchange_plan, which the CPU tests drive for S = 2..8): per wire
// column, peers in ascending order -- the same order on every rank -- a
// send of this shard's part for the peer and a receive of the peer's part,
// each at its running offset in the source-major columns; the shard's own
// part is a device copy.  sc / rc: [kMaxS][W] element counts sent to /
// received from each peer (rc of shard d from s == sc of shard s for d).
struct XOp {
  u32 kind;  // 0 own part (device copy), 1 send, 2 receive
  u32 wire, peer;
  u64 soff, roff, bytes;
};
void plan_payload(u32 S, u32 rank, u32 W, const std::vector<Wire>& wires, const u64* sc, const u64* rc,
                  std::vector<XOp>& ops) {
  ops.clear();
  for (u32 wi = 0; wi < (u32)wires.size(); wi++) {
    const Wire& w = wires[wi];
    u64 so = 0, ro = 0;
    for (u32 d = 0; d < S; d++) {
      const u64 sn = sc[(u64)d * W + w.gran] * w.esize, rn = rc[(u64)d * W + w.gran] * w.esize;
      if (d == rank) {
        if (sn) ops.push_back(XOp{0, wi, d, so, ro, sn});
      } else {
        if (sn) ops.push_back(XOp{1, wi, d, so, 0, sn});
        if (rn) ops.push_back(XOp{2, wi, d, 0, ro, rn});
      }
      so += sn;
      ro += rn;
    }
  }
}

int32_t exchange(jy_node* nd, u32 W, const std::vector<Wire>& wires, u32 nl) {
  const u32 S = nd->S;
  // 1. counts: per destination and granule -> per source and granule
  if (nd->fabric == JY_FABRIC_RCCL) {
    NcclGroup grp;  // ends the group on every return
    ND_NCCL(nd, grp.start());
    for (NdShard& sh : nd->sh) {
      u64* cnt = static_cast<u64*>(sh.b[B_CNT].p);
      for (u32 d = 0; d < S; d++) {
        ND_NCCL(nd, ncclSend(cnt + (u64)d * W, W, ncclUint64, (int)d, sh.comm, sh.eng->stream));
        ND_NCCL(nd, ncclRecv(cnt + (u64)(kMaxS + d) * W, W, ncclUint64, (int)d, sh.comm, sh.eng->stream));
      }
    }
    ND_NCCL(nd, grp.end());
    for (NdShard& sh : nd->sh) {
      ND_HIP(nd, hipSetDevice(sh.dev));
      ND_HIP(nd, hipMemcpyAsync(sh.pin, sh.b[B_CNT].p, 2 * kMaxS * kMaxW * 8, hipMemcpyDeviceToHost, sh.eng->stream));
    }
    for (NdShard& sh : nd->sh) ND_HIP(nd, hipStreamSynchronize(sh.eng->stream));
  } else {
    for (NdShard& sh : nd->sh) {
      ND_HIP(nd, hipSetDevice(sh.dev));
      ND_HIP(nd, hipMemcpyAsync(sh.pin, sh.b[B_CNT].p, (u64)S * W * 8, hipMemcpyDeviceToHost, sh.eng->stream));
      ND_HIP(nd, hipEventRecord(sh.ev_in, sh.eng->stream));
    }
    for (NdShard& sh : nd->sh) ND_HIP(nd, hipStreamSynchronize(sh.eng->stream));
    for (NdShard& dst : nd->sh)
      for (const NdShard& src : nd->sh)
        std::memcpy(dst.pin + (u64)(kMaxS + src.rank) * W, src.pin + (u64)dst.rank * W, W * 8);
  }
  // 2. receive buffers, source-major per wire column
  for (NdShard& sh : nd->sh) {
    const u64* rc = sh.pin + (u64)kMaxS * W;
    for (u32 g = 0; g < W; g++) {
      u64 t = 0;
      for (u32 s = 0; s < S; s++) t += rc[(u64)s * W + g];
      sh.rtot[g] = t;
    }
    for (const Wire& w : wires) {
      void* p;
      // a key-length column gets one word more (the scan's last input)
      const u64 extra = (w.ridx == R_KLEN) ? 1 : 0;
      JY_TRY(buf(nd, sh, w.ridx, (sh.rtot[w.gran] + extra) * w.esize + 8, &p));
    }
    nd->stats[1] += sh.rtot[0];
    u64 sb = 0, rb = 0;
    for (const Wire& w : wires)
      for (u32 d = 0; d < S; d++) {
        sb += sh.pin[(u64)d * W + w.gran] * w.esize;
        rb += rc[(u64)d * W + w.gran] * w.esize;
      }
    nd->stats[2] += sb;
    nd->stats[3] += rb;
  }
  // 3. payload
  if (nd->fabric == JY_FABRIC_RCCL) {
    NcclGroup grp;  // ends the group on every return
    ND_NCCL(nd, grp.start());
    std::vector<XOp> ops;
    for (NdShard& sh : nd->sh) {
      ND_HIP(nd, hipSetDevice(sh.dev));  // (the self copies below)
      plan_payload(S, sh.rank, W, wires, sh.pin, sh.pin + (u64)kMaxS * W, ops);
      for (const XOp& o : ops) {
        const Wire& w = wires[o.wire];
        const uint8_t* sp = static_cast<const uint8_t*>(sh.b[w.sidx].p);
        uint8_t* rp = static_cast<uint8_t*>(sh.b[w.ridx].p);
        if (o.kind == 0)  // its own part: a device copy on the same stream (through RCCL it
                          // cost ~100 us per column at 8M keys, the whole exchange at S = 1)
          ND_HIP(nd, hipMemcpyAsync(rp + o.roff, sp + o.soff, o.bytes, hipMemcpyDeviceToDevice, sh.eng->stream));
        else if (o.kind == 1)
          ND_NCCL(nd, ncclSend(sp + o.soff, o.bytes, ncclUint8, (int)o.peer, sh.comm, sh.eng->stream));
        else
          ND_NCCL(nd, ncclRecv(rp + o.roff, o.bytes, ncclUint8, (int)o.peer, sh.comm, sh.eng->stream));
      }
    }
    ND_NCCL(nd, grp.end());
  } else {
    // pull: each destination waits for every source's columns, copies its
    // parts on its own stream, and records that its receives landed (the next
    // call's ingest on a source waits for it before rewriting its columns)
    for (NdShard& dst : nd->sh) {
      ND_HIP(nd, hipSetDevice(dst.dev));
      for (NdShard& src : nd->sh) ND_HIP(nd, hipStreamWaitEvent(dst.eng->stream, src.ev_in, 0));
      const u64* rc = dst.pin + (u64)kMaxS * W;
      for (const Wire& w : wires) {
        uint8_t* rp = static_cast<uint8_t*>(dst.b[w.ridx].p);
        u64 ro = 0;
        for (NdShard& src : nd->sh) {
          // where dst's part starts in src's owner-order column
          u64 so = 0;
          for (u32 d = 0; d < dst.rank; d++) so += src.pin[(u64)d * W + w.gran];
          const u64 rn = rc[(u64)src.rank * W + w.gran] * w.esize;
          if (rn) {
            const uint8_t* sp = static_cast<const uint8_t*>(src.b[w.sidx].p) + so * w.esize;
            if (src.dev == dst.dev)
              ND_HIP(nd, hipMemcpyAsync(rp + ro, sp, rn, hipMemcpyDeviceToDevice, dst.eng->stream));
            else
              ND_HIP(nd, hipMemcpyPeerAsync(rp + ro, dst.dev, sp, src.dev, rn, dst.eng->stream));
          }
          ro += rn;
        }
      }
      ND_HIP(nd, hipEventRecord(dst.ev_out, dst.eng->stream));
    }
  }
  nd->stats[4]++;
  (void)nl;
  return JY_OK;
}

// the next ingest rewrites the send columns: with the copy fabric the other
// shards' pulls of the previous call must have happened first
int32_t ingest_begin(jy_node* nd, NdShard& sh) {
  ND_HIP(nd, hipSetDevice(sh.dev));
  if (nd->fabric == JY_FABRIC_COPY)
    for (NdShard& o : nd->sh) ND_HIP(nd, hipStreamWaitEvent(sh.eng->stream, o.ev_out, 0));
  for (auto& t : sh.tot) t = 0;
  return JY_OK;
}

// key ranges per local shard: contiguous, as even as the key count allows
void split(const jy_node* nd, u64 n, std::vector<u64>& at) {
  at.assign(nd->nlocal + 1, 0);
  for (u32 L = 0; L <= nd->nlocal; L++) at[L] = n * L / nd->nlocal;
}

// stage a chunk: host memory through the engine's pinned ring, device
// memory in place
int32_t stage(jy_node* nd, NdShard& sh, int slot, const void* src, u64 bytes, int32_t mem, const void** out) {
  if (mem == kPinned) {  // the node's pinned block: one DMA, no second host copy
    void* d;
    ND_ENG(nd, sh, jy_scratch(sh.eng, slot, std::max<u64>(bytes, 8), &d));
    if (bytes) ND_HIP(nd, hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, sh.eng->stream));
    *out = d;
    return JY_OK;
  }
  ND_ENG(nd, sh, jy_stage(sh.eng, slot, src, bytes, mem, out));
  return JY_OK;
}

// the received keys interned in the owner's directory -> R_SLOTS
int32_t owner_keys(jy_node* nd, NdShard& sh, int32_t type, u32** slots) {
  const u64 n = sh.rtot[0];
  u64* koff;
  JY_TRY(bufT(nd, sh, R_KOFF, n + 1, &koff));
  JY_TRY(bufT(nd, sh, R_SLOTS, std::max<u64>(n, 1), slots));
  if (n == 0) return JY_OK;
  u64* klen = static_cast<u64*>(sh.b[R_KLEN].p);
  ND_HIP(nd, hipMemsetAsync(klen + n, 0, 8, sh.eng->stream));
  ND_ENG(nd, sh, jy_scan_u64(sh.eng, klen, koff, n));
  ND_ENG(nd, sh, jy_keys_intern_mem(sh.eng, type, n, static_cast<const uint8_t*>(sh.b[R_KBYTES].p), koff, *slots,
                                    JY_DEVICE));
  return JY_OK;
}

// a received CSR level: its per-item lengths (received per-key column
// `lens_idx`, n items) -> global offsets (R_LOFF l) and per-source local
// offsets (R_LOC l, n + S words); per-source item and element starts on the host
int32_t owner_level(jy_node* nd, NdShard& sh, u32 l, int lens_idx, u64 n, u32 gran_items, u32 gran_el, u32 W,
                    SrcRanges& R, std::vector<u64>& ebase) {
  const u32 S = nd->S;
  const u64* rc = sh.pin + (u64)kMaxS * W;
  u64 *lens = static_cast<u64*>(sh.b[lens_idx].p), *goff, *loc;
  JY_TRY(bufT(nd, sh, R_LOFF0 + l, n + 1, &goff));
  JY_TRY(bufT(nd, sh, R_LOC0 + l, n + S, &loc));
  R.S = S;
  ebase.assign(S + 1, 0);
  u64 k = 0, e = 0;
  for (u32 s = 0; s < S; s++) {
    R.kb[s] = k;
    ebase[s] = e;
    k += rc[(u64)s * W + gran_items];
    e += rc[(u64)s * W + gran_el];
  }
  R.kb[S] = k;
  ebase[S] = e;
  if (n == 0) return JY_OK;
  // lens has room for one word more (buf() sizes receive columns with + 8 B)
  ND_HIP(nd, hipMemsetAsync(lens + n, 0, 8, sh.eng->stream));
  ND_ENG(nd, sh, jy_scan_u64(sh.eng, lens, goff, n));
  hipLaunchKernelGGL(k_nd_local_offs, dim3(grid_of(n + S)), dim3(kT), 0, sh.eng->stream, (const u64*)goff, n, R, loc);
  ND_HIP(nd, hipGetLastError());
  return JY_OK;
}

// received value bytes (a long-value level) into the owner's arena; handles
// from the lengths column `vlen` (n items) -> R_LR
int32_t owner_values(jy_node* nd, NdShard& sh, int32_t type, const u64* vlen, u64 n, int bytes_idx, u64 nbytes,
                     u64** lr) {
  u64 *plen, *voff;
  JY_TRY(bufT(nd, sh, R_PLEN, n + 1, &plen));
  JY_TRY(bufT(nd, sh, R_VOFF, n + 1, &voff));
  JY_TRY(bufT(nd, sh, R_LR, std::max<u64>(n, 1), lr));
  if (n == 0) return JY_OK;
  u64 rebase = 0;
  ND_ENG(nd, sh, jy_arena_append_dev(sh.eng, type, static_cast<const uint8_t*>(sh.b[bytes_idx].p), nbytes, &rebase));
  hipLaunchKernelGGL(k_nd_plen, dim3(grid_of(n + 1)), dim3(kT), 0, sh.eng->stream, n, vlen, plen);
  ND_HIP(nd, hipGetLastError());
  ND_ENG(nd, sh, jy_scan_u64(sh.eng, plen, voff, n));
  hipLaunchKernelGGL(k_nd_lr, dim3(grid_of(n)), dim3(kT), 0, sh.eng->stream, n, vlen, (const u64*)voff, rebase, *lr);
  ND_HIP(nd, hipGetLastError());
  return JY_OK;
}

int32_t node_check(jy_node* nd, int32_t mem, u64 n) {
  if (!nd) return JY_EINVAL;
  if (mem != JY_HOST && mem != JY_DEVICE) return nd->fail(JY_EINVAL, "mem must be JY_HOST or JY_DEVICE");
  if (n >= 0xFFFFFFFFull) return nd->fail(JY_ERANGE, "more than 2^32 - 1 keys in one call");
  return JY_OK;
}

// host value lengths fit a handle (the device form trusts its caller)
int32_t values_check(jy_node* nd, const u64* vo, u64 a, u64 e, int32_t mem) {
  if (mem != JY_HOST) return JY_OK;
  for (u64 i = a; i < e; i++) {
    if (vo[i + 1] < vo[i]) return nd->fail(JY_EINVAL, "value offsets are not ascending");
    if (vo[i + 1] - vo[i] > JY_MAX_VALUE_LEN) return nd->fail(JY_ERANGE, "value longer than 16 MiB");
  }
  return JY_OK;
}

// device inputs: the n value lengths at vo checked on the device; the
// verdict lands in the pinned read-back area with the next read2's sync
// (values_dev_ok after it)
int32_t values_dev_enqueue(jy_node* nd, NdShard& sh, const u64* vo, u64 n, int32_t mem) {
  if (mem != JY_DEVICE || n == 0) return JY_OK;
  u64* w;
  JY_TRY(bufT(nd, sh, B_CNT, 2 * kMaxS * kMaxW + 1, &w));
  w += 2 * kMaxS * kMaxW;  // (past the counts)
  // the word is zero between calls (dev_words resets it once read); zeroed
  // here only when a verdict was never read (an error path) or on first use
  if (sh.mlw || !sh.mlw_zero || sh.mlw_buf != w) ND_HIP(nd, hipMemsetAsync(w, 0, 8, sh.rs));
  sh.mlw_zero = true;
  sh.mlw_buf = w;
  hipLaunchKernelGGL(k_nd_maxlen, dim3(grid_of(n)), dim3(kT), 0, sh.rs, vo, n,
                     reinterpret_cast<unsigned long long*>(w));
  ND_HIP(nd, hipGetLastError());
  sh.mlw = w;  // read (and reset) by the next dev_words
  return JY_OK;
}
int32_t values_dev_ok(jy_node* nd, NdShard& sh, int32_t mem) {
  if (mem != JY_DEVICE) return JY_OK;
  u64& v = sh.pin[2 * kMaxS * kMaxW + 2];
  const u64 l = v;
  v = 0;
  if (l > JY_MAX_VALUE_LEN) return nd->fail(JY_ERANGE, "value longer than 16 MiB");
  return JY_OK;
}

// per local shard: keys chunk (staged) -> Ingest
int32_t stage_keys(jy_node* nd, NdShard& sh, u64 a, u64 e, const uint8_t* kb, const u64* ko, int32_t mem, Ingest& in) {
  sh.n = e - a;
  const void *dkb, *dko;
  u64 k0, k1;
  JY_TRY(read2(nd, sh, ko + a, ko + e, mem, k0, k1));
  if (k1 < k0) return nd->fail(JY_EINVAL, "key offsets are not ascending");
  JY_TRY(stage(nd, sh, 0, on_host(mem) ? kb + k0 : kb, k1 - k0, mem, &dkb));
  JY_TRY(stage(nd, sh, 1, ko + a, (sh.n + 1) * 8, mem, &dko));
  in.kb = static_cast<const uint8_t*>(dkb);
  in.ko = static_cast<const u64*>(dko);
  in.kobase = on_host(mem) ? k0 : 0;
  in.nkb = k1 - k0;
  sh.tot[0] = sh.n;
  sh.tot[1] = in.nkb;
  return JY_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI

extern "C" {

int32_t jy_node_unique_id(uint8_t* id_out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return JY_EHIP;
  std::memcpy(id_out, &id, sizeof(id));
  return JY_OK;
}

void jy_node_destroy(jy_node* nd) {
  if (!nd) return;
  exec_stop(nd);  // the queued jobs run first
  for (NdShard& sh : nd->sh) {
    hipSetDevice(sh.dev);
    if (sh.eng) hipStreamSynchronize(sh.eng->stream);
    if (sh.xs) hipStreamSynchronize(sh.xs);
    if (sh.rs) hipStreamSynchronize(sh.rs);
  }
  for (NdShard& sh : nd->sh)
    if (sh.comm) ncclCommDestroy(sh.comm);
  for (NdShard& sh : nd->sh) {
    hipSetDevice(sh.dev);
    for (NdBuf& b : sh.b)
      if (b.p) hipFree(b.p);
    if (sh.pin) hipHostFree(sh.pin);
    for (hipEvent_t e : {sh.ev_in, sh.ev_out, sh.ev_x[0], sh.ev_x[1], sh.ev_m[0], sh.ev_m[1], sh.ev_rs_in, sh.ev_rs_out})
      if (e) hipEventDestroy(e);
    if (sh.xs) hipStreamDestroy(sh.xs);
    if (sh.rs) hipStreamDestroy(sh.rs);
    jy_engine_destroy(sh.eng);
  }
  for (NdPin& pb : nd->pins) {
    for (hipEvent_t e : pb.ev)
      if (e) hipEventDestroy(e);
    if (pb.p) hipHostFree(pb.p);
  }
  delete nd;
}

int32_t jy_node_create(const jy_node_config* cfg, jy_node** out) {
  *out = nullptr;
  if (!cfg || cfg->nshards == 0 || cfg->nshards > kMaxS || cfg->nlocal == 0 ||
      cfg->rank0 + cfg->nlocal > cfg->nshards)
    return JY_EINVAL;
  if (cfg->fabric != JY_FABRIC_RCCL && cfg->fabric != JY_FABRIC_COPY) return JY_EINVAL;
  if (cfg->fabric == JY_FABRIC_COPY && cfg->nlocal != cfg->nshards) return JY_EINVAL;  // one process
  jy_node* nd = new jy_node();
  nd->cfg = *cfg;
  nd->S = cfg->nshards;
  nd->nlocal = cfg->nlocal;
  nd->rank0 = cfg->rank0;
  nd->fabric = cfg->fabric;
  nd->sh.resize(nd->nlocal);
  for (u32 L = 0; L < nd->nlocal; L++) {
    NdShard& sh = nd->sh[L];
    sh.rank = nd->rank0 + L;
    sh.dev = cfg->devices[L];
    jy_config ec = cfg->engine;
    ec.device = sh.dev;
    if (jy_engine_create(&ec, &sh.eng) != JY_OK || !sh.eng ||
        hipHostMalloc(reinterpret_cast<void**>(&sh.pin), (2 * kMaxS * kMaxW + kPinTail) * 8, hipHostMallocMapped) !=
            hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&sh.pin_dev), sh.pin, 0) != hipSuccess ||
        hipStreamCreateWithFlags(&sh.xs, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&sh.rs, hipStreamNonBlocking) != hipSuccess) {
      std::fprintf(stderr, "jy_node_create: shard %u on device %d failed\n", sh.rank, sh.dev);
      jy_node_destroy(nd);
      return JY_EHIP;
    }
    for (hipEvent_t* e : {&sh.ev_in, &sh.ev_out, &sh.ev_x[0], &sh.ev_x[1], &sh.ev_m[0], &sh.ev_m[1], &sh.ev_rs_in,
                          &sh.ev_rs_out})
      if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
        jy_node_destroy(nd);
        return JY_EHIP;
      }
    hipEventRecord(sh.ev_out, sh.eng->stream);
  }
  if (nd->fabric == JY_FABRIC_RCCL) {
    ncclUniqueId id;
    std::memcpy(&id, cfg->unique_id, sizeof(id));
    bool zero = true;
    for (u64 i = 0; i < sizeof(id); i++) zero = zero && cfg->unique_id[i] == 0;
    if (zero) {
      if (nd->nlocal != nd->S) {
        std::fprintf(stderr, "jy_node_create: a multi-process node needs the shared unique_id\n");
        jy_node_destroy(nd);
        return JY_EINVAL;
      }
      if (ncclGetUniqueId(&id) != ncclSuccess) {
        jy_node_destroy(nd);
        return JY_EHIP;
      }
    }
    ncclResult_t r = ncclGroupStart();
    for (NdShard& sh : nd->sh) {
      if (r != ncclSuccess) break;
      hipSetDevice(sh.dev);
      r = ncclCommInitRank(&sh.comm, (int)nd->S, id, (int)sh.rank);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess) {
      std::fprintf(stderr, "jy_node_create: ncclCommInitRank: %s\n",
                   ncclGetErrorString(r != ncclSuccess ? r : r2));
      jy_node_destroy(nd);
      return JY_EHIP;
    }
  }
  // one process driving several GPUs: a shard's kernels read JY_DEVICE inputs
  // that live on another local GPU (the header's "readable by every local
  // shard's GPU"), so every local pair gets peer access (over xGMI)
  for (const NdShard& a : nd->sh)
    for (const NdShard& b : nd->sh)
      if (a.dev != b.dev) {
        hipSetDevice(a.dev);
        const hipError_t e = hipDeviceEnablePeerAccess(b.dev, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
          std::fprintf(stderr, "jy_node_create: peer access %d -> %d: %s\n", a.dev, b.dev, hipGetErrorString(e));
          (void)hipGetLastError();
        }
      }
  exec_start(nd);
  *out = nd;
  return JY_OK;
}

int32_t jy_node_create_local(uint32_t nshards, const int32_t* devices, uint32_t fabric, const jy_config* engine,
                             jy_node** out) {
  *out = nullptr;
  if (nshards == 0 || nshards > kMaxS || !devices) return JY_EINVAL;
  jy_node_config cfg;
  std::memset(&cfg, 0, sizeof(cfg));
  cfg.nshards = cfg.nlocal = nshards;
  cfg.rank0 = 0;
  cfg.fabric = fabric;
  for (u32 i = 0; i < nshards; i++) cfg.devices[i] = devices[i];
  if (engine) cfg.engine = *engine;
  else jy_config_default(&cfg.engine);
  return jy_node_create(&cfg, out);
}

// the process's shared node (round 5): the five GPU repos of one Jylis
// process (database.pony:18-22 makes one RepoManager per type) take the same
// node, so one communicator and one engine per GPU serve all five types
namespace {
std::mutex g_shared_mu;
jy_node* g_shared = nullptr;
u64 g_shared_refs = 0;
}  // namespace

int32_t jy_node_acquire_local(const jy_config* engine, jy_node** out) {
  std::lock_guard<std::mutex> lk(g_shared_mu);
  *out = nullptr;
  if (!g_shared) {
    const int32_t n = jy_device_count();
    if (n <= 0) return JY_EHIP;
    int32_t devs[kMaxS];
    const u32 S = std::min<u32>((u32)n, kMaxS);
    for (u32 i = 0; i < S; i++) devs[i] = (int32_t)i;
    JY_TRY(jy_node_create_local(S, devs, JY_FABRIC_RCCL, engine, &g_shared));
  }
  g_shared_refs++;
  *out = g_shared;
  return JY_OK;
}

void jy_node_release(jy_node* nd) {
  std::lock_guard<std::mutex> lk(g_shared_mu);
  if (!nd || nd != g_shared || g_shared_refs == 0) return;
  if (--g_shared_refs == 0) {
    jy_node_destroy(g_shared);
    g_shared = nullptr;
  }
}

int32_t jy_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* jy_node_last_error(const jy_node* nd) { return nd ? jy_node::caller_err().c_str() : "null node"; }
uint32_t jy_node_nshards(const jy_node* nd) { return nd ? nd->S : 0; }

jy_engine* jy_node_engine(jy_node* nd, uint32_t shard) {
  if (!nd || shard < nd->rank0 || shard >= nd->rank0 + nd->nlocal) return nullptr;
  return nd->sh[shard - nd->rank0].eng;
}

uint32_t jy_node_shard_of(const jy_node* nd, const uint8_t* key, uint64_t len) {
  return jy_key_owner(key, len, nd ? nd->S : 1);
}

// A registered id is answered from the node's own map (no wait for the
// worker); a new one is registered on every shard under the node
// mutex -- no fence: no job queued before it can name a column not yet
// registered (callers register before they send cells).
int32_t jy_node_replica_col(jy_node* nd, uint64_t id, uint32_t* col) {
  if (!nd) return JY_EINVAL;
  {
    std::lock_guard<std::mutex> r(nd->rmu);
    auto it = nd->rep.find(id);
    if (it != nd->rep.end()) {
      *col = it->second;
      return JY_OK;
    }
  }
  std::lock_guard<std::mutex> g(nd->mu);
  u32 c0 = 0;
  for (u32 L = 0; L < nd->nlocal; L++) {
    u32 c = 0;
    ND_ENG(nd, nd->sh[L], jy_replica_col(nd->sh[L].eng, id, &c));
    if (L == 0) c0 = c;
    else if (c != c0) return nd->fail(JY_EINVAL, "shards disagree on a replica column (register on the node only)");
  }
  *col = c0;
  nd->nrep = std::max<u32>(nd->nrep, c0 + 1);
  std::lock_guard<std::mutex> r(nd->rmu);
  nd->rep[id] = c0;
  return JY_OK;
}

// every queued job issued and every shard's streams drained, THEN a queued
// job's failure (the streams are synchronised on the error path
// too, so a caller may free its JY_DEVICE inputs once this returns)
int32_t jy_node_sync(jy_node* nd) {
  if (!nd) return JY_EINVAL;
  int32_t rc;
  {
    std::unique_lock<std::mutex> lk(nd->qmu);
    nd->dcv.wait(lk, [&] { return nd->finished == nd->submitted; });
  }
  {
    std::lock_guard<std::mutex> g(nd->mu);
    rc = JY_OK;
    for (NdShard& sh : nd->sh) {  // (every shard, whatever failed first)
      const int32_t re = jy_sync(sh.eng);  // spilled TLOG merges settled, the engine stream drained
      hipSetDevice(sh.dev);
      const hipError_t e1 = hipStreamSynchronize(sh.xs), e2 = hipStreamSynchronize(sh.rs);
      if (rc == JY_OK && re != JY_OK) rc = nd->fail(re, std::string("shard ") + std::to_string(sh.rank) + ": " + sh.eng->err);
      if (rc == JY_OK && (e1 != hipSuccess || e2 != hipSuccess))
        rc = nd->fail(JY_EHIP, "node sync: a shard's stream failed");
    }
  }
  const int32_t pend = exec_pending(nd);
  return pend != JY_OK ? pend : rc;
}

int32_t jy_node_stats(jy_node* nd, uint64_t* out5) {
  if (!nd) return JY_EINVAL;
  JY_TRY(exec_fence(nd));
  std::lock_guard<std::mutex> g(nd->mu);
  std::memcpy(out5, nd->stats, sizeof(nd->stats));
  return JY_OK;
}

}  // extern "C"

namespace {

// ---- one shard (S = 1) ----
// The node's only shard owns every key: no regroup, no exchange, no copy of
// any wire column.  The owner phase reads the staged inputs in place; the
// value work runs beside the key probe (one_keys_values).  (Through the
// regroup + self exchange, an 8.39M-key TREG call
// spent ~0.9 ms of its 1.6 ms before the key probe: profiles/r05_*.)

// up to 8 words of device (or host) memory, one wait
int32_t readn(jy_node* nd, NdShard& sh, int32_t mem, std::initializer_list<const u64*> src, u64* out) {
  int i = 0;
  if (on_host(mem)) {
    for (const u64* p : src) out[i++] = *p;
    return JY_OK;
  }
  return dev_words(nd, sh, src, out);
}

// keys interned on the one shard; with `vals`, the ne values' heads, their
// long bytes in the arena and their handles (pre, lr at R_F1 / R_LR).
// The value work runs on the read-back stream, beside the key probe (the
// probe waits on random table lines, the value kernels stream): heads and
// tile sums first; once the probe is enqueued, the host waits for their total,
// reserves the arena and enqueues the long values; the engine stream waits
// for them before the merge.  (In one stream the 8.39M-key TREG call took
// 0.651 ms, ~70 us heads + scan and ~85 us long values after the probe; side
// by side 0.636: the probe itself slows from 329 to 438 us beside them,
// profiles/r05_node_value_overlap_ab.txt.)
struct OneVals {
  u64 ne = 0;
  const u64* vo = nullptr;  // device, indexed from the first value
  u64 vbase = 0;
  const uint8_t* vb = nullptr;
  u64 vbytes = 0;  // the values' bytes in all (bounds the long values' arena total)
};
struct LongJob;
// what a caller merges right behind the probe (before the host has read the
// miss count): the engine stream already waits for the values
typedef int32_t (*SpecMerge)(void* arg, const LongJob& j);
struct LongJob {
  jy_node* nd;
  NdShard* sh;
  int32_t type;
  const OneVals* vals;
  u64 nvt;
  const u64* toff;
  u64* lr;
  u32* slots = nullptr;
  u64* pre = nullptr;
  SpecMerge spec = nullptr;
  void* spec_arg = nullptr;
};
// on the host while the probe runs: the total, the arena, the long values
int32_t long_values(void* p) {
  LongJob& j = *static_cast<LongJob*>(p);
  NdShard& sh = *j.sh;
  jy_engine* eng = sh.eng;
  if (hipStreamSynchronize(sh.rs) != hipSuccess) return eng->fail(JY_EHIP, "node: value heads");
  const u64 total = sh.pin[2 * kMaxS * kMaxW + 3];
  uint8_t* dst;
  u64 rebase;
  const u64 cap = eng->arena[j.type].cap;
  JY_TRY(jy_arena_reserve(eng, j.type, total, &dst, &rebase));
  if (eng->arena[j.type].cap != cap)  // one_keys_values made room: never reached
    return eng->fail(JY_EINVAL, "node: the arena moved under the read-back stream");
  hipLaunchKernelGGL(k_nd1_long, dim3((u32)j.nvt), dim3(kT), 0, sh.rs, j.vals->ne, j.vals->vo, j.vals->vbase,
                     j.vals->vb, j.toff, dst, rebase, j.lr);
  if (hipGetLastError() != hipSuccess || hipEventRecord(sh.ev_rs_out, sh.rs) != hipSuccess)
    return eng->fail(JY_EHIP, "node: long values");
  if (j.spec) {
    if (hipStreamWaitEvent(eng->stream, sh.ev_rs_out, 0) != hipSuccess) return eng->fail(JY_EHIP, "node: value wait");
    JY_TRY(j.spec(j.spec_arg, j));
  }
  return JY_OK;
}
int32_t one_keys_values(jy_node* nd, NdShard& sh, int32_t type, u64 n, const uint8_t* kbase, const u64* ko,
                        const OneVals* vals, u32** slots, u64** pre, u64** lr, SpecMerge spec = nullptr,
                        void* spec_arg = nullptr, u64* created = nullptr) {
  jy_engine* eng = sh.eng;
  JY_TRY(bufT(nd, sh, R_SLOTS, std::max<u64>(n, 1), slots));
  const u64 ne = vals ? vals->ne : 0;
  u64 *tsum = nullptr, *toff = nullptr;
  const u64 nvt = (ne + kValTile - 1) / kValTile;  // value tiles
  if (vals) {
    JY_TRY(bufT(nd, sh, R_F1, std::max<u64>(ne, 1), pre));
    JY_TRY(bufT(nd, sh, R_PLEN, nvt + 1, &tsum));
    JY_TRY(bufT(nd, sh, R_VOFF, nvt + 1, &toff));
    JY_TRY(bufT(nd, sh, R_LR, std::max<u64>(ne, 1), lr));
  }
  LongJob job{nd, &sh, type, vals, nvt, toff, vals ? *lr : nullptr, *slots, vals ? *pre : nullptr,
              ne ? spec : nullptr, spec_arg};
  if (created) *created = 0;
  if (ne) {
    // the arena holds the long values' total already (at most every value's
    // bytes + a granule's padding each): long_values then only advances its
    // length on the read-back stream -- a growth there would reallocate on
    // the engine stream, past ev_rs_in, while k_nd1_long writes the new tail
    ND_ENG(nd, sh, jy_arena_ensure(eng, type, vals->vbytes + kArenaAlign * ne));
    // after the staged inputs and the previous call's kernels (which read
    // pre / lr / the arena) on the engine stream
    ND_HIP(nd, hipEventRecord(sh.ev_rs_in, eng->stream));
    ND_HIP(nd, hipStreamWaitEvent(sh.rs, sh.ev_rs_in, 0));
    hipLaunchKernelGGL(k_nd1_head, dim3((u32)nvt), dim3(kT), 0, sh.rs, ne, vals->vo, vals->vbase, vals->vb, *pre,
                       tsum);
    ND_HIP(nd, hipGetLastError());
    hipLaunchKernelGGL(k_nd1_tscan, dim3(1), dim3(kTScanThreads), 0, sh.rs, (const u64*)tsum, nvt, toff,
                       sh.pin_dev + 2 * kMaxS * kMaxW + 3);
    ND_HIP(nd, hipGetLastError());
  }
  if (n)
    ND_ENG(nd, sh, jy_keys_intern_dev(eng, type, n, kbase, ko, *slots, ne ? long_values : nullptr, &job, created));
  else if (ne)
    ND_ENG(nd, sh, long_values(&job));
  if (ne) ND_HIP(nd, hipStreamWaitEvent(eng->stream, sh.ev_rs_out, 0));
  return JY_OK;
}

const uint8_t* rebased(const void* p, u64 by) {
  return reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) - by);
}

void one_stats(jy_node* nd, u64 n) {
  nd->stats[0] = nd->stats[1] = n;
  nd->stats[2] = nd->stats[3] = 0;
  nd->stats[4]++;
}

int32_t run_treg_one(jy_node* nd, u64 n, const uint8_t* kb, const u64* ko, const u64* ts, const uint8_t* vb,
                     const u64* vo, int32_t mem) {
  NdShard& sh = nd->sh[0];
  ND_HIP(nd, hipSetDevice(sh.dev));
  one_stats(nd, n);
  if (n == 0) return JY_OK;
  u64 w[4];
  JY_TRY(values_dev_enqueue(nd, sh, vo, n, mem));
  JY_TRY(readn(nd, sh, mem, {ko, ko + n, vo, vo + n}, w));
  JY_TRY(values_dev_ok(nd, sh, mem));
  const u64 k0 = w[0], k1 = w[1], v0 = w[2], v1 = w[3];
  if (k1 < k0 || v1 < v0) return nd->fail(JY_EINVAL, "key or value offsets are not ascending");
  const void *dkb, *dko, *dts, *dvo, *dvb;
  ND_ENG(nd, sh, jy_stage_begin(sh.eng));
  JY_TRY(stage(nd, sh, 0, on_host(mem) ? kb + k0 : kb, k1 - k0, mem, &dkb));
  JY_TRY(stage(nd, sh, 1, ko, (n + 1) * 8, mem, &dko));
  JY_TRY(stage(nd, sh, 2, ts, n * 8, mem, &dts));
  JY_TRY(stage(nd, sh, 3, vo, (n + 1) * 8, mem, &dvo));
  JY_TRY(stage(nd, sh, 4, on_host(mem) ? vb + v0 : vb, v1 - v0, mem, &dvb));
  ND_ENG(nd, sh, jy_stage_end(sh.eng));
  OneVals vals{n, static_cast<const u64*>(dvo), on_host(mem) ? v0 : 0, static_cast<const uint8_t*>(dvb), v1 - v0};
  u32* slots;
  u64 *pre, *lr;
  // The merge goes in right behind the probe, before the host reads the miss
  // count back: the keys found take their LWW with no host round trip between
  // the two (a key still missing has slot JY_NO_SLOT, which the merge skips).
  // New keys then get a second, whole merge once they have slots -- LWW is
  // idempotent, so the keys merged twice are exact.
  struct Spec {
    u64 n;
    const u64* ts;
    bool done;
  } sp{n, static_cast<const u64*>(dts), false};
  const SpecMerge spec = [](void* a, const LongJob& j) -> int32_t {
    Spec& s = *static_cast<Spec*>(a);
    s.done = true;
    return jy_treg_merge(j.sh->eng, s.n, j.slots, s.ts, j.pre, j.lr);
  };
  u64 created = 0;
  JY_TRY(one_keys_values(nd, sh, JY_TREG, n, rebased(dkb, on_host(mem) ? k0 : 0), static_cast<const u64*>(dko),
                         &vals, &slots, &pre, &lr, spec, &sp, &created));
  if (!sp.done || created) ND_ENG(nd, sh, jy_treg_merge(sh.eng, n, slots, static_cast<const u64*>(dts), pre, lr));
  return JY_OK;
}

int32_t run_counter_one(jy_node* nd, int32_t type, u64 n, const uint8_t* kb, const u64* ko, const u64* co,
                        const uint8_t* sign, const u16* col, const u64* val, int32_t mem) {
  NdShard& sh = nd->sh[0];
  jy_engine* eng = sh.eng;
  ND_HIP(nd, hipSetDevice(sh.dev));
  one_stats(nd, n);
  if (n == 0) return JY_OK;
  u64 w[4];
  JY_TRY(readn(nd, sh, mem, {ko, ko + n, co, co + n}, w));
  const u64 k0 = w[0], k1 = w[1], c0 = w[2], c1 = w[3], nc = c1 - c0;
  if (k1 < k0 || c1 < c0) return nd->fail(JY_EINVAL, "key or cell offsets are not ascending");
  if (nc >= 0xFFFFFFFFull) return nd->fail(JY_ERANGE, "more than 2^32 - 1 cells in one call");
  const u64 cb = on_host(mem) ? c0 : 0;  // staged cells start at c0; device cells are indexed from 0
  const void *dkb, *dko, *dco, *dsg = nullptr, *dcol, *dval;
  ND_ENG(nd, sh, jy_stage_begin(eng));
  JY_TRY(stage(nd, sh, 0, on_host(mem) ? kb + k0 : kb, k1 - k0, mem, &dkb));
  JY_TRY(stage(nd, sh, 1, ko, (n + 1) * 8, mem, &dko));
  JY_TRY(stage(nd, sh, 2, co, (n + 1) * 8, mem, &dco));
  if (sign) JY_TRY(stage(nd, sh, 3, sign + cb, nc, mem, &dsg));
  JY_TRY(stage(nd, sh, 4, col + cb, nc * 2, mem, &dcol));
  JY_TRY(stage(nd, sh, 5, val + cb, nc * 8, mem, &dval));
  ND_ENG(nd, sh, jy_stage_end(eng));
  const u64 cel = on_host(mem) ? 0 : c0;  // the batch's first cell in the staged columns
  u64* rel;
  u32* ckey;
  JY_TRY(bufT(nd, sh, R_LOC0, n + 1, &rel));
  JY_TRY(bufT(nd, sh, R_AUX0, std::max<u64>(nc, 1), &ckey));
  hipLaunchKernelGGL(k_nd1_rebase, dim3(grid_of(n + 1)), dim3(kT), 0, eng->stream, n, static_cast<const u64*>(dco),
                     rel);
  ND_HIP(nd, hipGetLastError());
  u32* slots;
  JY_TRY(one_keys_values(nd, sh, type, n, rebased(dkb, on_host(mem) ? k0 : 0), static_cast<const u64*>(dko), nullptr,
                         &slots, nullptr, nullptr));
  if (nc == 0) return JY_OK;
  ND_ENG(nd, sh, jy_seg_ids(eng, rel, n, nc, ckey));
  const int which = type == JY_GCOUNT ? 0 : 1;
  ND_ENG(nd, sh, jy_counter_grow(eng, which, jy_replica_count(eng), 0));
  ND_ENG(nd, sh, jy_counter_coo_keyed(eng, which, nc, n, slots, ckey,
                                      dsg ? static_cast<const uint8_t*>(dsg) + cel : nullptr,
                                      static_cast<const u16*>(dcol) + cel, static_cast<const u64*>(dval) + cel));
  return JY_OK;
}

int32_t run_tlog_one(jy_node* nd, u64 n, const uint8_t* kb, const u64* ko, const u64* cutoff, const u64* eo,
                     const u64* ts, const uint8_t* vb, const u64* vo, int32_t mem) {
  NdShard& sh = nd->sh[0];
  jy_engine* eng = sh.eng;
  ND_HIP(nd, hipSetDevice(sh.dev));
  one_stats(nd, n);
  if (n == 0) return JY_OK;
  u64 w[4], v[2];
  JY_TRY(readn(nd, sh, mem, {ko, ko + n, eo, eo + n}, w));
  const u64 k0 = w[0], k1 = w[1], e0 = w[2], e1 = w[3], ne = e1 - e0;
  if (k1 < k0 || e1 < e0) return nd->fail(JY_EINVAL, "key or entry offsets are not ascending");
  if (ne >= 0xFFFFFFFFull) return nd->fail(JY_ERANGE, "more than 2^32 - 1 entries in one call");
  JY_TRY(values_dev_enqueue(nd, sh, vo + e0, ne, mem));
  JY_TRY(readn(nd, sh, mem, {vo + e0, vo + e1}, v));
  JY_TRY(values_dev_ok(nd, sh, mem));
  const u64 v0 = v[0], v1 = v[1];
  if (v1 < v0) return nd->fail(JY_EINVAL, "value offsets are not ascending");
  const u64 eb = on_host(mem) ? e0 : 0;
  const void *dkb, *dko, *dcut, *deo, *dts, *dvo, *dvb;
  ND_ENG(nd, sh, jy_stage_begin(eng));
  JY_TRY(stage(nd, sh, 0, on_host(mem) ? kb + k0 : kb, k1 - k0, mem, &dkb));
  JY_TRY(stage(nd, sh, 1, ko, (n + 1) * 8, mem, &dko));
  JY_TRY(stage(nd, sh, 2, cutoff, n * 8, mem, &dcut));
  JY_TRY(stage(nd, sh, 3, eo, (n + 1) * 8, mem, &deo));
  JY_TRY(stage(nd, sh, 4, ts + eb, ne * 8, mem, &dts));
  JY_TRY(stage(nd, sh, 5, vo + eb, (ne + 1) * 8, mem, &dvo));
  JY_TRY(stage(nd, sh, 6, on_host(mem) ? vb + v0 : vb, v1 - v0, mem, &dvb));
  ND_ENG(nd, sh, jy_stage_end(eng));
  const u64 ent = on_host(mem) ? 0 : e0;  // the batch's first entry in the staged columns
  u64* rel;
  JY_TRY(bufT(nd, sh, R_LOC0, n + 1, &rel));
  hipLaunchKernelGGL(k_nd1_rebase, dim3(grid_of(n + 1)), dim3(kT), 0, eng->stream, n, static_cast<const u64*>(deo),
                     rel);
  ND_HIP(nd, hipGetLastError());
  OneVals vals{ne, static_cast<const u64*>(dvo) + ent, on_host(mem) ? v0 : 0, static_cast<const uint8_t*>(dvb),
               v1 - v0};
  u32* slots;
  u64 *pre, *lr;
  JY_TRY(one_keys_values(nd, sh, JY_TLOG, n, rebased(dkb, on_host(mem) ? k0 : 0), static_cast<const u64*>(dko),
                         &vals, &slots, &pre, &lr));
  ND_ENG(nd, sh, jy_tlog_merge(eng, n, slots, static_cast<const u64*>(dcut), rel, ne,
                               static_cast<const u64*>(dts) + ent, pre, lr));
  return JY_OK;
}

int32_t run_ujson_one(jy_node* nd, u64 n, const uint8_t* kb, const u64* ko, const u64* eo, const u64* dots,
                      const u64* elems, const u64* vvo, const u64* vv, const u64* clo, const u64* cloud,
                      int32_t mem) {
  NdShard& sh = nd->sh[0];
  jy_engine* eng = sh.eng;
  ND_HIP(nd, hipSetDevice(sh.dev));
  one_stats(nd, n);
  if (n == 0) return JY_OK;
  u64 w[8];
  JY_TRY(readn(nd, sh, mem, {ko, ko + n, eo, eo + n, vvo, vvo + n, clo, clo + n}, w));
  const u64 k0 = w[0], k1 = w[1];
  if (k1 < k0 || w[3] < w[2] || w[5] < w[4] || w[7] < w[6])
    return nd->fail(JY_EINVAL, "key / element / vv / cloud offsets are not ascending");
  const u64 lo[3] = {w[2], w[4], w[6]}, cnt[3] = {w[3] - w[2], w[5] - w[4], w[7] - w[6]};
  const u64 hb[3] = {on_host(mem) ? lo[0] : 0, on_host(mem) ? lo[1] : 0, on_host(mem) ? lo[2] : 0};
  const void *dkb, *dko, *deo, *dd, *de, *dvo, *dv, *dco, *dc;
  ND_ENG(nd, sh, jy_stage_begin(eng));
  JY_TRY(stage(nd, sh, 0, on_host(mem) ? kb + k0 : kb, k1 - k0, mem, &dkb));
  JY_TRY(stage(nd, sh, 1, ko, (n + 1) * 8, mem, &dko));
  JY_TRY(stage(nd, sh, 2, eo, (n + 1) * 8, mem, &deo));
  JY_TRY(stage(nd, sh, 3, dots + hb[0], cnt[0] * 8, mem, &dd));
  JY_TRY(stage(nd, sh, 4, elems + hb[0], cnt[0] * 8, mem, &de));
  JY_TRY(stage(nd, sh, 5, vvo, (n + 1) * 8, mem, &dvo));
  JY_TRY(stage(nd, sh, 6, vv + hb[1], cnt[1] * 8, mem, &dv));
  JY_TRY(stage(nd, sh, 7, clo, (n + 1) * 8, mem, &dco));
  JY_TRY(stage(nd, sh, 8, cloud + hb[2], cnt[2] * 8, mem, &dc));
  ND_ENG(nd, sh, jy_stage_end(eng));
  const void* offs[3] = {deo, dvo, dco};
  u64* rel[3];
  for (int l = 0; l < 3; l++) {
    JY_TRY(bufT(nd, sh, R_LOC0 + l, n + 1, &rel[l]));
    hipLaunchKernelGGL(k_nd1_rebase, dim3(grid_of(n + 1)), dim3(kT), 0, eng->stream, n,
                       static_cast<const u64*>(offs[l]), rel[l]);
  }
  ND_HIP(nd, hipGetLastError());
  u32* slots;
  JY_TRY(one_keys_values(nd, sh, JY_UJSON, n, rebased(dkb, on_host(mem) ? k0 : 0), static_cast<const u64*>(dko),
                         nullptr, &slots, nullptr, nullptr));
  const u64 f[3] = {on_host(mem) ? 0 : lo[0], on_host(mem) ? 0 : lo[1], on_host(mem) ? 0 : lo[2]};
  ND_ENG(nd, sh, jy_ujson_merge(eng, n, slots, rel[0], cnt[0], static_cast<const u64*>(dd) + f[0],
                                static_cast<const u64*>(de) + f[0], rel[1], cnt[1], static_cast<const u64*>(dv) + f[1],
                                rel[2], cnt[2], static_cast<const u64*>(dc) + f[2]));
  return JY_OK;
}

// ---- TREG: key bytes | ts, pre, vlen | long value bytes ----
int32_t run_treg(jy_node* nd, uint64_t n, const uint8_t* kb, const uint64_t* ko, const uint64_t* ts, const uint8_t* vb,
                 const uint64_t* vo, int32_t mem) {
  if (nd->S == 1 && !nd->regroup_one) return run_treg_one(nd, n, kb, ko, ts, vb, vo, mem);
  std::vector<u64> at;
  split(nd, n, at);
  nd->stats[0] = n;
  nd->stats[1] = nd->stats[2] = nd->stats[3] = 0;
  constexpr u32 W = 3;  // keys, key bytes, value bytes
  for (u32 L = 0; L < nd->nlocal; L++) {
    NdShard& sh = nd->sh[L];
    JY_TRY(ingest_begin(nd, sh));
    Ingest in;
    ND_ENG(nd, sh, jy_stage_begin(sh.eng));
    JY_TRY(stage_keys(nd, sh, at[L], at[L + 1], kb, ko, mem, in));
    const u64 a = at[L], m = sh.n;
    u64 v0, v1;
    JY_TRY(values_check(nd, vo, a, at[L + 1], mem));
    JY_TRY(values_dev_enqueue(nd, sh, vo + a, m, mem));
    JY_TRY(read2(nd, sh, vo + a, vo + at[L + 1], mem, v0, v1));
    JY_TRY(values_dev_ok(nd, sh, mem));
    const void *dts, *dvo, *dvb;
    JY_TRY(stage(nd, sh, 2, ts + a, m * 8, mem, &dts));
    JY_TRY(stage(nd, sh, 3, vo + a, (m + 1) * 8, mem, &dvo));
    JY_TRY(stage(nd, sh, 4, on_host(mem) ? vb + v0 : vb, v1 - v0, mem, &dvb));
    ND_ENG(nd, sh, jy_stage_end(sh.eng));
    JY_TRY(ingest_keys(nd, sh, in));
    const u64 vbase = on_host(mem) ? v0 : 0;
    JY_TRY(ingest_fixed<1>(nd, sh, InU64<1>{{static_cast<const u64*>(dts)}}));
    u64 *pre, *vlen;
    JY_TRY(bufT(nd, sh, B_F1, std::max<u64>(m, 1), &pre));
    JY_TRY(bufT(nd, sh, B_F2, std::max<u64>(m, 1), &vlen));
    if (m)
      hipLaunchKernelGGL(k_nd_val_head, dim3(grid_of(m)), dim3(kT), 0, sh.eng->stream, m,
                         (const u32*)sh.b[B_PERM].p, static_cast<const u64*>(dvo), vbase,
                         static_cast<const uint8_t*>(dvb), pre, vlen);
    ND_HIP(nd, hipGetLastError());
    Level lv;
    lv.offs = static_cast<const u64*>(dvo);
    lv.obase = vbase;
    lv.nel = v1 - v0;
    lv.longval = true;
    JY_TRY(ingest_level<1>(nd, sh, 0, lv, m, (const u32*)sh.b[B_PERM].p, InBytes{static_cast<const uint8_t*>(dvb)},
                           false));
    JY_TRY(ingest_counts(nd, sh, &lv, 1));
  }
  const std::vector<Wire> wires = {{0, 8, B_KLEN, R_KLEN}, {1, 1, B_KBYTES, R_KBYTES}, {0, 8, B_F0, R_F0},
                                   {0, 8, B_F1, R_F1},     {0, 8, B_F2, R_F2},         {2, 1, B_LC00, R_LC00}};
  JY_TRY(exchange(nd, W, wires, 1));
  for (NdShard& sh : nd->sh) {
    ND_HIP(nd, hipSetDevice(sh.dev));
    u32* slots;
    JY_TRY(owner_keys(nd, sh, JY_TREG, &slots));
    const u64 m = sh.rtot[0];
    u64* lr;
    JY_TRY(owner_values(nd, sh, JY_TREG, static_cast<const u64*>(sh.b[R_F2].p), m, R_LC00, sh.rtot[2], &lr));
    ND_ENG(nd, sh, jy_treg_merge(sh.eng, m, slots, static_cast<const u64*>(sh.b[R_F0].p),
                                 static_cast<const u64*>(sh.b[R_F1].p), lr));
  }
  return JY_OK;
}

// ---- counters: key bytes | cell count | cells (sign << 16 | col, val) ----
int32_t run_counter(jy_node* nd, int32_t type, uint64_t n, const uint8_t* kb, const uint64_t* ko, const uint64_t* co,
                    const uint8_t* sign, const uint16_t* col, const uint64_t* val, int32_t mem) {
  if (nd->S == 1 && !nd->regroup_one) return run_counter_one(nd, type, n, kb, ko, co, sign, col, val, mem);
  std::vector<u64> at;
  split(nd, n, at);
  nd->stats[0] = n;
  nd->stats[1] = nd->stats[2] = nd->stats[3] = 0;
  constexpr u32 W = 3;  // keys, key bytes, cells
  for (u32 L = 0; L < nd->nlocal; L++) {
    NdShard& sh = nd->sh[L];
    JY_TRY(ingest_begin(nd, sh));
    Ingest in;
    ND_ENG(nd, sh, jy_stage_begin(sh.eng));
    JY_TRY(stage_keys(nd, sh, at[L], at[L + 1], kb, ko, mem, in));
    const u64 a = at[L], m = sh.n;
    u64 c0, c1;
    JY_TRY(read2(nd, sh, co + a, co + at[L + 1], mem, c0, c1));
    if (c1 < c0) return nd->fail(JY_EINVAL, "cell offsets are not ascending");
    if (mem == JY_HOST) {  // (kPinned: checked by the call)
      const u32 nrep = jy_replica_count(sh.eng);
      for (u64 c = c0; c < c1; c++) {
        if (col[c] >= nrep) return nd->fail(JY_ERANGE, "column names no registered replica");
        if (sign && sign[c] > 1) return nd->fail(JY_ERANGE, "sign must be 0 (P) or 1 (N)");
      }
    }
    const u64 cb = on_host(mem) ? c0 : 0;
    const void *dco, *dsg = nullptr, *dcol, *dval;
    JY_TRY(stage(nd, sh, 2, co + a, (m + 1) * 8, mem, &dco));
    if (sign) JY_TRY(stage(nd, sh, 3, sign + cb, c1 - c0, mem, &dsg));
    JY_TRY(stage(nd, sh, 4, col + cb, (c1 - c0) * 2, mem, &dcol));
    JY_TRY(stage(nd, sh, 5, val + cb, (c1 - c0) * 8, mem, &dval));
    ND_ENG(nd, sh, jy_stage_end(sh.eng));
    JY_TRY(ingest_keys(nd, sh, in));
    Level lv;
    lv.offs = static_cast<const u64*>(dco);
    lv.obase = cb;
    lv.nel = c1 - c0;
    const InCells cells{static_cast<const uint8_t*>(dsg), static_cast<const u16*>(dcol), static_cast<const u64*>(dval)};
    JY_TRY(ingest_level<2>(nd, sh, 0, lv, m, (const u32*)sh.b[B_PERM].p, cells, false));
    JY_TRY(ingest_counts(nd, sh, &lv, 1));
  }
  const std::vector<Wire> wires = {{0, 8, B_KLEN, R_KLEN},   {1, 1, B_KBYTES, R_KBYTES}, {0, 8, B_LLEN0, R_F0},
                                   {2, 8, B_LC00, R_LC00}, {2, 8, B_LC01, R_LC01}};
  JY_TRY(exchange(nd, W, wires, 1));
  const int which = type == JY_GCOUNT ? 0 : 1;
  for (NdShard& sh : nd->sh) {
    ND_HIP(nd, hipSetDevice(sh.dev));
    u32* slots;
    JY_TRY(owner_keys(nd, sh, type, &slots));
    const u64 m = sh.rtot[0], nc = sh.rtot[2];
    if (nc == 0) continue;
    u64* off;
    u32* ckey;
    uint8_t* sg;
    u16* cl;
    JY_TRY(bufT(nd, sh, R_LOFF0, m + 1, &off));
    JY_TRY(bufT(nd, sh, R_AUX0, nc, &ckey));
    JY_TRY(bufT(nd, sh, R_AUX1, nc, &sg));
    JY_TRY(bufT(nd, sh, R_AUX2, nc, &cl));
    u64* lens = static_cast<u64*>(sh.b[R_F0].p);
    ND_HIP(nd, hipMemsetAsync(lens + m, 0, 8, sh.eng->stream));
    ND_ENG(nd, sh, jy_scan_u64(sh.eng, lens, off, m));
    ND_ENG(nd, sh, jy_seg_ids(sh.eng, off, m, nc, ckey));
    hipLaunchKernelGGL(k_nd_cells, dim3(grid_of(nc)), dim3(kT), 0, sh.eng->stream, nc,
                       (const u64*)sh.b[R_LC00].p, sg, cl);
    ND_HIP(nd, hipGetLastError());
    ND_ENG(nd, sh, jy_counter_grow(sh.eng, which, jy_replica_count(sh.eng), 0));
    ND_ENG(nd, sh, jy_counter_coo_keyed(sh.eng, which, nc, m, slots, ckey, type == JY_PNCOUNT ? sg : nullptr, cl,
                                        static_cast<const u64*>(sh.b[R_LC01].p)));
  }
  return JY_OK;
}

// ---- TLOG: key bytes | cutoff, entry count | entries (ts, pre, vlen) | long value bytes ----
int32_t run_tlog(jy_node* nd, uint64_t n, const uint8_t* kb, const uint64_t* ko, const uint64_t* cutoff, const uint64_t* eo,
                 const uint64_t* ts, const uint8_t* vb, const uint64_t* vo, int32_t mem) {
  if (nd->S == 1 && !nd->regroup_one) return run_tlog_one(nd, n, kb, ko, cutoff, eo, ts, vb, vo, mem);
  std::vector<u64> at;
  split(nd, n, at);
  nd->stats[0] = n;
  nd->stats[1] = nd->stats[2] = nd->stats[3] = 0;
  constexpr u32 W = 4;  // keys, key bytes, entries, value bytes
  for (u32 L = 0; L < nd->nlocal; L++) {
    NdShard& sh = nd->sh[L];
    JY_TRY(ingest_begin(nd, sh));
    Ingest in;
    ND_ENG(nd, sh, jy_stage_begin(sh.eng));
    JY_TRY(stage_keys(nd, sh, at[L], at[L + 1], kb, ko, mem, in));
    const u64 a = at[L], m = sh.n;
    u64 e0, e1, v0, v1;
    JY_TRY(read2(nd, sh, eo + a, eo + at[L + 1], mem, e0, e1));
    if (e1 < e0) return nd->fail(JY_EINVAL, "entry offsets are not ascending");
    if (e1 - e0 >= 0xFFFFFFFFull) return nd->fail(JY_ERANGE, "more than 2^32 - 1 entries in one shard's range");
    JY_TRY(values_check(nd, vo, e0, e1, mem));
    JY_TRY(values_dev_enqueue(nd, sh, vo + e0, e1 - e0, mem));
    JY_TRY(read2(nd, sh, vo + e0, vo + e1, mem, v0, v1));
    JY_TRY(values_dev_ok(nd, sh, mem));
    if (v1 < v0) return nd->fail(JY_EINVAL, "value offsets are not ascending");
    const u64 eb = on_host(mem) ? e0 : 0, vbase = on_host(mem) ? v0 : 0;
    const void *dcut, *deo, *dts, *dvo, *dvb;
    JY_TRY(stage(nd, sh, 2, cutoff + a, m * 8, mem, &dcut));
    JY_TRY(stage(nd, sh, 3, eo + a, (m + 1) * 8, mem, &deo));
    JY_TRY(stage(nd, sh, 4, ts + eb, (e1 - e0) * 8, mem, &dts));
    JY_TRY(stage(nd, sh, 5, vo + eb, (e1 - e0 + 1) * 8, mem, &dvo));
    JY_TRY(stage(nd, sh, 6, on_host(mem) ? vb + v0 : vb, v1 - v0, mem, &dvb));
    ND_ENG(nd, sh, jy_stage_end(sh.eng));
    JY_TRY(ingest_keys(nd, sh, in));
    JY_TRY(ingest_fixed<1>(nd, sh, InU64<1>{{static_cast<const u64*>(dcut)}}));
    Level lv[2];
    lv[0].offs = static_cast<const u64*>(deo);
    lv[0].obase = eb;
    lv[0].nel = e1 - e0;
    // entries: ts in owner order, element sources for the value level
    JY_TRY(ingest_level<1>(nd, sh, 0, lv[0], m, (const u32*)sh.b[B_PERM].p,
                           InU64<1>{{static_cast<const u64*>(dts)}}, true));
    const u64 ne = e1 - e0;
    u64 *pre, *vlen;
    JY_TRY(bufT(nd, sh, B_LC01, std::max<u64>(ne, 1), &pre));
    // (the value lengths ride in the level-1 slot's second column)
    JY_TRY(bufT(nd, sh, B_LC11, std::max<u64>(ne, 1), &vlen));
    if (ne)
      hipLaunchKernelGGL(k_nd_val_head, dim3(grid_of(ne)), dim3(kT), 0, sh.eng->stream, ne,
                         (const u32*)sh.b[B_ESRC].p, static_cast<const u64*>(dvo), vbase,
                         static_cast<const uint8_t*>(dvb), pre, vlen);
    ND_HIP(nd, hipGetLastError());
    lv[1].offs = static_cast<const u64*>(dvo);
    lv[1].obase = vbase;
    lv[1].nel = v1 - v0;
    lv[1].parent = 0;
    lv[1].longval = true;
    JY_TRY(ingest_level<1>(nd, sh, 1, lv[1], ne, (const u32*)sh.b[B_ESRC].p,
                           InBytes{static_cast<const uint8_t*>(dvb)}, false));
    JY_TRY(ingest_counts(nd, sh, lv, 2));
  }
  const std::vector<Wire> wires = {{0, 8, B_KLEN, R_KLEN}, {1, 1, B_KBYTES, R_KBYTES}, {0, 8, B_F0, R_F0},
                                   {0, 8, B_LLEN0, R_F1},  {2, 8, B_LC00, R_LC00},     {2, 8, B_LC01, R_LC01},
                                   {2, 8, B_LC11, R_LC11}, {3, 1, B_LC10, R_LC10}};
  JY_TRY(exchange(nd, W, wires, 2));
  for (NdShard& sh : nd->sh) {
    ND_HIP(nd, hipSetDevice(sh.dev));
    u32* slots;
    JY_TRY(owner_keys(nd, sh, JY_TLOG, &slots));
    const u64 m = sh.rtot[0], ne = sh.rtot[2];
    SrcRanges R;
    std::vector<u64> ebase;
    JY_TRY(owner_level(nd, sh, 0, R_F1, m, 0, 2, W, R, ebase));
    u64* lr;
    JY_TRY(owner_values(nd, sh, JY_TLOG, static_cast<const u64*>(sh.b[R_LC11].p), ne, R_LC10, sh.rtot[3], &lr));
    const u64* cut = static_cast<const u64*>(sh.b[R_F0].p);
    const u64* loc = static_cast<const u64*>(sh.b[R_LOC0].p);
    const u64* rts = static_cast<const u64*>(sh.b[R_LC00].p);
    const u64* rpre = static_cast<const u64*>(sh.b[R_LC01].p);
    for (u32 s = 0; s < nd->S; s++) {
      const u64 k0 = R.kb[s], nk = R.kb[s + 1] - k0;
      if (nk == 0) continue;
      ND_ENG(nd, sh, jy_tlog_merge(sh.eng, nk, slots + k0, cut + k0, loc + k0 + s, ebase[s + 1] - ebase[s],
                                   rts + ebase[s], rpre + ebase[s], lr + ebase[s]));
    }
  }
  return JY_OK;
}

// ---- UJSON: key bytes | element, vv, cloud counts | (dots, elems), vv, cloud ----
int32_t run_ujson(jy_node* nd, uint64_t n, const uint8_t* kb, const uint64_t* ko, const uint64_t* eo, const uint64_t* dots,
                  const uint64_t* elems, const uint64_t* vvo, const uint64_t* vv, const uint64_t* clo,
                  const uint64_t* cloud, int32_t mem) {
  if (nd->S == 1 && !nd->regroup_one)
    return run_ujson_one(nd, n, kb, ko, eo, dots, elems, vvo, vv, clo, cloud, mem);
  std::vector<u64> at;
  split(nd, n, at);
  nd->stats[0] = n;
  nd->stats[1] = nd->stats[2] = nd->stats[3] = 0;
  constexpr u32 W = 5;  // keys, key bytes, elements, vv entries, cloud dots
  for (u32 L = 0; L < nd->nlocal; L++) {
    NdShard& sh = nd->sh[L];
    JY_TRY(ingest_begin(nd, sh));
    Ingest in;
    ND_ENG(nd, sh, jy_stage_begin(sh.eng));
    JY_TRY(stage_keys(nd, sh, at[L], at[L + 1], kb, ko, mem, in));
    const u64 a = at[L], e = at[L + 1], m = sh.n;
    const u64* offs[3] = {eo, vvo, clo};
    u64 lo[3], hi[3];
    for (int l = 0; l < 3; l++) {
      JY_TRY(read2(nd, sh, offs[l] + a, offs[l] + e, mem, lo[l], hi[l]));
      if (hi[l] < lo[l]) return nd->fail(JY_EINVAL, "element / vv / cloud offsets are not ascending");
    }
    const void *deo, *dd, *de, *dvo, *dv, *dco, *dc;
    const u64 b0 = on_host(mem) ? lo[0] : 0, b1 = on_host(mem) ? lo[1] : 0, b2 = on_host(mem) ? lo[2] : 0;
    JY_TRY(stage(nd, sh, 2, eo + a, (m + 1) * 8, mem, &deo));
    JY_TRY(stage(nd, sh, 3, dots + b0, (hi[0] - lo[0]) * 8, mem, &dd));
    JY_TRY(stage(nd, sh, 4, elems + b0, (hi[0] - lo[0]) * 8, mem, &de));
    JY_TRY(stage(nd, sh, 5, vvo + a, (m + 1) * 8, mem, &dvo));
    JY_TRY(stage(nd, sh, 6, vv + b1, (hi[1] - lo[1]) * 8, mem, &dv));
    JY_TRY(stage(nd, sh, 7, clo + a, (m + 1) * 8, mem, &dco));
    JY_TRY(stage(nd, sh, 8, cloud + b2, (hi[2] - lo[2]) * 8, mem, &dc));
    ND_ENG(nd, sh, jy_stage_end(sh.eng));
    JY_TRY(ingest_keys(nd, sh, in));
    Level lv[3];
    const void* lo_p[3] = {deo, dvo, dco};
    const u64 bases[3] = {b0, b1, b2};
    for (int l = 0; l < 3; l++) {
      lv[l].offs = static_cast<const u64*>(lo_p[l]);
      lv[l].obase = bases[l];
      lv[l].nel = hi[l] - lo[l];
    }
    const u32* perm = static_cast<const u32*>(sh.b[B_PERM].p);
    JY_TRY(ingest_level<2>(nd, sh, 0, lv[0], m, perm,
                           InU64<2>{{static_cast<const u64*>(dd), static_cast<const u64*>(de)}}, false));
    JY_TRY(ingest_level<1>(nd, sh, 1, lv[1], m, perm, InU64<1>{{static_cast<const u64*>(dv)}}, false));
    JY_TRY(ingest_level<1>(nd, sh, 2, lv[2], m, perm, InU64<1>{{static_cast<const u64*>(dc)}}, false));
    JY_TRY(ingest_counts(nd, sh, lv, 3));
  }
  const std::vector<Wire> wires = {{0, 8, B_KLEN, R_KLEN},  {1, 1, B_KBYTES, R_KBYTES}, {0, 8, B_LLEN0, R_F0},
                                   {0, 8, B_LLEN1, R_F1},   {0, 8, B_LLEN2, R_F2},     {2, 8, B_LC00, R_LC00},
                                   {2, 8, B_LC01, R_LC01}, {3, 8, B_LC10, R_LC10},     {4, 8, B_LC20, R_LC20}};
  JY_TRY(exchange(nd, W, wires, 3));
  for (NdShard& sh : nd->sh) {
    ND_HIP(nd, hipSetDevice(sh.dev));
    u32* slots;
    JY_TRY(owner_keys(nd, sh, JY_UJSON, &slots));
    const u64 m = sh.rtot[0];
    SrcRanges R[3];
    std::vector<u64> eb[3];
    JY_TRY(owner_level(nd, sh, 0, R_F0, m, 0, 2, W, R[0], eb[0]));
    JY_TRY(owner_level(nd, sh, 1, R_F1, m, 0, 3, W, R[1], eb[1]));
    JY_TRY(owner_level(nd, sh, 2, R_F2, m, 0, 4, W, R[2], eb[2]));
    const u64* loc[3] = {static_cast<const u64*>(sh.b[R_LOC0].p), static_cast<const u64*>(sh.b[R_LOC1].p),
                         static_cast<const u64*>(sh.b[R_LOC2].p)};
    const u64 *rd = static_cast<const u64*>(sh.b[R_LC00].p), *re = static_cast<const u64*>(sh.b[R_LC01].p),
              *rv = static_cast<const u64*>(sh.b[R_LC10].p), *rcl = static_cast<const u64*>(sh.b[R_LC20].p);
    for (u32 s = 0; s < nd->S; s++) {
      const u64 k0 = R[0].kb[s], nk = R[0].kb[s + 1] - k0;
      if (nk == 0) continue;
      ND_ENG(nd, sh, jy_ujson_merge(sh.eng, nk, slots + k0, loc[0] + k0 + s, eb[0][s + 1] - eb[0][s], rd + eb[0][s],
                                    re + eb[0][s], loc[1] + k0 + s, eb[1][s + 1] - eb[1][s], rv + eb[1][s],
                                    loc[2] + k0 + s, eb[2][s + 1] - eb[2][s], rcl + eb[2][s]));
    }
  }
  return JY_OK;
}

// ---- dense counter blocks arriving mixed ----
int32_t run_block(jy_node* nd, int32_t type, uint32_t ncols, const uint16_t* cols_all, uint32_t slot0, uint32_t nslots,
                  const uint64_t* vals_p, const uint64_t* vals_n) {
  const u32 S = nd->S, G = type == JY_PNCOUNT ? 2 : 1;
  if (ncols == 0 || nslots == 0) return JY_OK;
  const u64 blk = (u64)nslots;                // words of one (column, owner) block
  const u64 per_local = (u64)ncols * S * blk; // words per sign per local shard
  // A shard's block for itself never moves: it is merged straight from the
  // input; only the S - 1 blocks of the other owners travel, landing
  // compacted in the receive buffer ([g][j], j = the other sources in rank
  // order).  (Sent to itself through RCCL, the self block cost a copy of the
  // whole batch at N = 1: 23.5 ms per step against 8.9 for the merge alone.)
  const u32 So = S - 1;
  for (NdShard& sh : nd->sh) {
    ND_HIP(nd, hipSetDevice(sh.dev));
    if (So)
      for (int k = 0; k < 2; k++) {
        void* p;
        JY_TRY(buf(nd, sh, X_BUF0 + k, (u64)G * So * blk * 8, &p));
      }
    // the exchange stream starts after the engine stream's work so far (the
    // inputs were produced there) and after the previous call's merges
    ND_HIP(nd, hipEventRecord(sh.ev_in, sh.eng->stream));
    ND_HIP(nd, hipStreamWaitEvent(sh.xs, sh.ev_in, 0));
  }
  std::vector<u16> cols(S);
  auto input = [&](u32 g, u32 L, u32 c, u32 d) {  // block [g][c][d] of local shard L
    return (g ? vals_n : vals_p) + (u64)L * per_local + ((u64)c * S + d) * blk;
  };
  for (u32 c = 0; c < ncols; c++) {
    const int k = c & 1;
    // column c: block [g][c][d] of local shard L goes to d, lands as [g][j] at d
    if (So && c >= 2)
      for (NdShard& sh : nd->sh) {
        ND_HIP(nd, hipSetDevice(sh.dev));
        ND_HIP(nd, hipStreamWaitEvent(sh.xs, sh.ev_m[k], 0));  // merge c - 2 has read this buffer
      }
    if (So && nd->fabric == JY_FABRIC_RCCL) {
      NcclGroup grp;  // ends the group on every return
      ND_NCCL(nd, grp.start());
      for (u32 L = 0; L < nd->nlocal; L++) {
        NdShard& sh = nd->sh[L];
        u64* rb = static_cast<u64*>(sh.b[X_BUF0 + k].p);
        for (u32 g = 0; g < G; g++) {
          u32 j = 0;
          for (u32 d = 0; d < S; d++) {
            if (d == sh.rank) continue;
            ND_NCCL(nd, ncclSend(input(g, L, c, d), blk, ncclUint64, (int)d, sh.comm, sh.xs));
            ND_NCCL(nd, ncclRecv(rb + ((u64)g * So + j++) * blk, blk, ncclUint64, (int)d, sh.comm, sh.xs));
          }
        }
      }
      ND_NCCL(nd, grp.end());
    } else if (So) {
      // every source's input must be ready before a destination pulls it
      for (NdShard& sh : nd->sh) ND_HIP(nd, hipEventRecord(sh.ev_in, sh.xs));
      for (u32 L = 0; L < nd->nlocal; L++) {
        NdShard& dst = nd->sh[L];
        ND_HIP(nd, hipSetDevice(dst.dev));
        for (NdShard& src : nd->sh) ND_HIP(nd, hipStreamWaitEvent(dst.xs, src.ev_in, 0));
        u64* rb = static_cast<u64*>(dst.b[X_BUF0 + k].p);
        for (u32 g = 0; g < G; g++) {
          u32 j = 0;
          for (u32 s = 0; s < nd->nlocal; s++) {
            if (s == L) continue;
            ND_HIP(nd, hipMemcpyAsync(rb + ((u64)g * So + j++) * blk, input(g, s, c, dst.rank), blk * 8,
                                      hipMemcpyDefault, dst.xs));
          }
        }
      }
    }
    for (u32 L = 0; L < nd->nlocal; L++) {
      NdShard& sh = nd->sh[L];
      ND_HIP(nd, hipSetDevice(sh.dev));
      // the self block first (no wait: its input is ordered on this stream)
      const u16 own_col = cols_all[(u64)sh.rank * ncols + c];
      if (type == JY_PNCOUNT)
        ND_ENG(nd, sh, jy_pncount_converge_block(sh.eng, 1, &own_col, slot0, nslots, input(0, L, c, sh.rank),
                                                 input(1, L, c, sh.rank), JY_DEVICE));
      else
        ND_ENG(nd, sh, jy_gcount_converge_block(sh.eng, 1, &own_col, slot0, nslots, input(0, L, c, sh.rank),
                                                JY_DEVICE));
      if (!So) continue;
      ND_HIP(nd, hipEventRecord(sh.ev_x[k], sh.xs));
      ND_HIP(nd, hipStreamWaitEvent(sh.eng->stream, sh.ev_x[k], 0));
      u32 j = 0;
      for (u32 s = 0; s < S; s++)
        if (s != sh.rank) cols[j++] = cols_all[(u64)s * ncols + c];
      const u64* rb = static_cast<const u64*>(sh.b[X_BUF0 + k].p);
      if (type == JY_PNCOUNT)
        ND_ENG(nd, sh, jy_pncount_converge_block(sh.eng, So, cols.data(), slot0, nslots, rb, rb + (u64)So * blk,
                                                 JY_DEVICE));
      else
        ND_ENG(nd, sh, jy_gcount_converge_block(sh.eng, So, cols.data(), slot0, nslots, rb, JY_DEVICE));
      ND_HIP(nd, hipEventRecord(sh.ev_m[k], sh.eng->stream));
    }
  }
  if (So && nd->fabric == JY_FABRIC_COPY) {
    // a destination's pulls read the other shards' inputs on its exchange
    // stream: every shard's engine stream (the one a caller syncs or reuses
    // its input on) waits for every destination's last pull
    for (NdShard& dst : nd->sh) {
      ND_HIP(nd, hipSetDevice(dst.dev));
      ND_HIP(nd, hipEventRecord(dst.ev_out, dst.xs));
    }
    for (NdShard& src : nd->sh) {
      ND_HIP(nd, hipSetDevice(src.dev));
      for (NdShard& dst : nd->sh) ND_HIP(nd, hipStreamWaitEvent(src.eng->stream, dst.ev_out, 0));
    }
  }
  nd->stats[4] += ncols;
  return JY_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// the executor

namespace {

int32_t run_job(jy_node* nd, const NdJob& j) {
  const int32_t mem = j.mem == JY_HOST ? kPinned : j.mem;
  const auto U8 = [&](int i) { return static_cast<const uint8_t*>(j.a[i]); };
  const auto U64 = [&](int i) { return static_cast<const u64*>(j.a[i]); };
  switch (j.kind) {
    case K_COUNTER:
      return run_counter(nd, j.type, j.n, U8(0), U64(1), U64(2), U8(3), static_cast<const u16*>(j.a[4]), U64(5), mem);
    case K_TREG:
      return run_treg(nd, j.n, U8(0), U64(1), U64(2), U8(3), U64(4), mem);
    case K_TLOG:
      return run_tlog(nd, j.n, U8(0), U64(1), U64(2), U64(3), U64(4), U8(5), U64(6), mem);
    case K_UJSON:
      return run_ujson(nd, j.n, U8(0), U64(1), U64(2), U64(3), U64(4), U64(5), U64(6), U64(7), U64(8), mem);
    case K_BLOCK:
      return run_block(nd, j.type, j.ncols, j.cols.data(), j.slot0, j.nslots, U64(0), U64(1));
  }
  return nd->fail(JY_EINVAL, "unknown node job");
}

// one job, under the node lock: its pinned block is released with events
// that fire once the job's DMAs out of it are done
int32_t run_locked(jy_node* nd, const NdJob& j) {
  int32_t rc = run_job(nd, j);
  if (j.pin >= 0) {
    NdPin& pb = nd->pins[j.pin];
    for (u32 L = 0; L < nd->nlocal; L++) {
      NdShard& sh = nd->sh[L];
      hipSetDevice(sh.dev);
      if (rc != JY_OK) {  // a failed job's staging may be in flight
        hipStreamSynchronize(sh.eng->stream);
        hipStreamSynchronize(sh.rs);
      }
      else if (hipEventRecord(pb.ev[L], sh.eng->stream) != hipSuccess) {
        hipStreamSynchronize(sh.eng->stream);
        hipEventRecord(pb.ev[L], nullptr);
      }
    }
  }
  return rc;
}

void finish(jy_node* nd, const NdJob& j, int32_t rc) {
  std::lock_guard<std::mutex> lk(nd->qmu);
  if (j.pin >= 0) nd->pins[j.pin].busy = false;
  if (rc != JY_OK && nd->aerr == JY_OK) {
    nd->aerr = rc;
    nd->aerr_msg = std::this_thread::get_id() == nd->wid ? nd->werr : jy_node::caller_err();
  }
  nd->finished++;
  nd->fin_t[j.fty]++;
  nd->dcv.notify_all();
}

// the worker's arena policy (jy_node_arena_gc), after a TREG / TLOG job and
// under the node mutex: a shard's arena whose dead bytes pass twice the live
// ones (+ 1 MiB) is collected -- the policy of jylis_amd/repo.py _ArenaGC and
// of the Pony glue's maybe_collect, which the glue's drains no longer run
// (they only enqueue).  Handles callers pack are consumed under the lock, so
// none is outstanding between jobs.
int32_t arena_policy(jy_node* nd, int32_t type) {
  const int t = type == JY_TREG ? 0 : 1;
  nd->arena_live.resize(2 * nd->nlocal, 0);
  for (u32 L = 0; L < nd->nlocal; L++) {
    jy_engine* eng = nd->sh[L].eng;
    u64 len = 0, cap = 0, kept = 0;
    ND_ENG(nd, nd->sh[L], jy_arena_usage(eng, type, &len, &cap));
    if (len <= 2 * nd->arena_live[2 * L + t] + (1ull << 20)) continue;
    ND_ENG(nd, nd->sh[L], jy_arena_collect(eng, type, &kept));
    nd->arena_live[2 * L + t] = kept;
  }
  return JY_OK;
}

void worker_loop(jy_node* nd) {
  for (;;) {
    NdJob j;
    {
      std::unique_lock<std::mutex> lk(nd->qmu);
      nd->qcv.wait(lk, [&] { return nd->stop || !nd->q.empty(); });
      if (nd->q.empty()) return;  // stop, and nothing left
      j = std::move(nd->q.front());
      nd->q.pop_front();
    }
    while (nd->lock_waiters.load(std::memory_order_acquire) > 0) std::this_thread::yield();
    int32_t rc;
    {
      std::lock_guard<std::mutex> g(nd->mu);
      rc = run_locked(nd, j);
      if (rc == JY_OK && nd->arena_gc && (j.fty == JY_TREG || j.fty == JY_TLOG)) rc = arena_policy(nd, j.fty);
    }
    finish(nd, j, rc);
  }
}

void exec_start(jy_node* nd) {
  const char* e = std::getenv("JY_NODE_INLINE");
  nd->inline_jobs = e && *e && *e != '0';
  const char* r = std::getenv("JY_NODE_REGROUP_ONE");
  nd->regroup_one = r && *r && *r != '0';
  if (nd->inline_jobs) return;
  nd->worker = std::thread([nd] { worker_loop(nd); });
  nd->wid = nd->worker.get_id();
}

void exec_stop(jy_node* nd) {
  if (!nd->worker.joinable()) return;
  {
    std::lock_guard<std::mutex> lk(nd->qmu);
    nd->stop = true;
  }
  nd->qcv.notify_all();
  nd->worker.join();
}

// every job queued so far has been issued; then the first failure of a
// queued job since the last report, if any (moved to jy_node_last_error)
int32_t exec_fence(jy_node* nd) {
  std::unique_lock<std::mutex> lk(nd->qmu);
  nd->dcv.wait(lk, [&] { return nd->finished == nd->submitted; });
  if (nd->aerr == JY_OK) return JY_OK;
  const int32_t rc = nd->aerr;
  jy_node::caller_err() = nd->aerr_msg;
  nd->aerr = JY_OK;
  return rc;
}

// every job of CRDT type `type` queued so far has been issued (jobs of other
// types may still be queued: the types' engine states are disjoint and the
// engine stream orders what the caller enqueues next after every issued
// job); then a queued job's failure, as exec_fence
int32_t exec_fence_type(jy_node* nd, int32_t type) {
  std::unique_lock<std::mutex> lk(nd->qmu);
  const u64 target = nd->sub_t[type];
  nd->dcv.wait(lk, [&] { return nd->fin_t[type] >= target; });
  if (nd->aerr == JY_OK) return JY_OK;
  const int32_t rc = nd->aerr;
  jy_node::caller_err() = nd->aerr_msg;
  nd->aerr = JY_OK;
  return rc;
}

// a failure a queued job left behind, reported without waiting
int32_t exec_pending(jy_node* nd) {
  std::lock_guard<std::mutex> lk(nd->qmu);
  if (nd->aerr == JY_OK) return JY_OK;
  const int32_t rc = nd->aerr;
  jy_node::caller_err() = nd->aerr_msg;
  nd->aerr = JY_OK;
  return rc;
}

// ---- packing host inputs into a pinned block ----
struct Pack {
  struct Arr {
    const void* src;  // the caller's array (index 0 = element 0)
    u64 esize, lo, hi;  // elements [lo, hi) are read
    int slot;           // NdJob::a index
  };
  std::vector<Arr> arr;
  void add(int slot, const void* src, u64 esize, u64 lo, u64 hi) { arr.push_back({src, esize, lo, hi, slot}); }
};

// a free pinned block of at least `bytes` (waits while every block is busy,
// then for the DMAs of its previous job)
int32_t pin_acquire(jy_node* nd, u64 bytes, int* out) {
  int b = -1;
  {
    std::unique_lock<std::mutex> lk(nd->qmu);
    nd->dcv.wait(lk, [&] {
      for (int i = 0; i < kJobDepth; i++)
        if (!nd->pins[i].busy) return true;
      return false;
    });
    for (int i = 0; i < kJobDepth && b < 0; i++)
      if (!nd->pins[i].busy) b = i;
    nd->pins[b].busy = true;
  }
  NdPin& pb = nd->pins[b];
  auto release = [&](int32_t rc) {
    std::lock_guard<std::mutex> lk(nd->qmu);
    pb.busy = false;
    nd->dcv.notify_all();
    return rc;
  };
  if (pb.ev.empty()) {
    pb.ev.assign(nd->nlocal, nullptr);
    for (u32 L = 0; L < nd->nlocal; L++) {
      hipSetDevice(nd->sh[L].dev);
      if (hipEventCreateWithFlags(&pb.ev[L], hipEventDisableTiming) != hipSuccess ||
          hipEventRecord(pb.ev[L], nullptr) != hipSuccess)
        return release(nd->fail(JY_EHIP, "node: pinned block events"));
    }
  }
  for (hipEvent_t e : pb.ev)
    if (hipEventSynchronize(e) != hipSuccess) return release(nd->fail(JY_EHIP, "node: pinned block wait"));
  if (pb.bytes < bytes) {
    if (pb.p) hipHostFree(pb.p);
    pb.p = nullptr;
    pb.bytes = 0;
    const u64 nb = std::max<u64>((bytes + bytes / 4 + 4095) & ~4095ull, 1 << 20);
    if (hipHostMalloc(&pb.p, nb, hipHostMallocDefault) != hipSuccess)
      return release(nd->fail(JY_EHIP, "node: hipHostMalloc of the pinned input block"));
    pb.bytes = nb;
  }
  *out = b;
  return JY_OK;
}

// copy every array's read range into one pinned block; the job's pointers
// are rebased so that the original indices (offsets above 0 included) work
int32_t pack_host(jy_node* nd, const Pack& pk, NdJob& j) {
  u64 total = 0;
  for (const Pack::Arr& a : pk.arr) total = round8(total) + (a.hi - a.lo) * a.esize + 8;
  int b;
  JY_TRY(pin_acquire(nd, total, &b));
  j.pin = b;
  uint8_t* base = static_cast<uint8_t*>(nd->pins[b].p);
  u64 at = 0;
  for (const Pack::Arr& a : pk.arr) {
    at = round8(at);
    const u64 nb = (a.hi - a.lo) * a.esize;
    if (nb) jy_copy_host(base + at, static_cast<const uint8_t*>(a.src) + a.lo * a.esize, nb);
    // element lo lives at base + at
    j.a[a.slot] = reinterpret_cast<const void*>(reinterpret_cast<uintptr_t>(base + at) - a.lo * a.esize);
    at += nb + 8;
  }
  return JY_OK;
}

int32_t submit(jy_node* nd, NdJob&& j) {
  j.fty = j.kind == K_TREG ? JY_TREG : j.kind == K_TLOG ? JY_TLOG : j.kind == K_UJSON ? JY_UJSON : j.type;
  if (nd->inline_jobs) {
    int32_t rc;
    {
      std::lock_guard<std::mutex> g(nd->mu);
      rc = run_locked(nd, j);
      if (rc == JY_OK && nd->arena_gc && (j.fty == JY_TREG || j.fty == JY_TLOG)) rc = arena_policy(nd, j.fty);
    }
    {
      std::lock_guard<std::mutex> lk(nd->qmu);
      nd->submitted++;
      nd->sub_t[j.fty]++;
    }
    finish(nd, j, JY_OK);
    return rc;
  }
  {
    std::lock_guard<std::mutex> lk(nd->qmu);
    nd->submitted++;
    nd->sub_t[j.fty]++;
    nd->q.push_back(std::move(j));
  }
  nd->qcv.notify_one();
  return JY_OK;
}

// the public entry's checks common to every converge (a queued job's earlier
// failure is reported here first)
int32_t call_check(jy_node* nd, int32_t mem, u64 n) {
  JY_TRY(node_check(nd, mem, n));
  return exec_pending(nd);
}

}  // namespace

extern "C" {

int32_t jy_node_counter_converge(jy_node* nd, int32_t type, uint64_t n, const uint8_t* kb, const uint64_t* ko,
                                 const uint64_t* co, const uint8_t* sign, const uint16_t* col, const uint64_t* val,
                                 int32_t mem) {
  JY_TRY(call_check(nd, mem, n));
  if (type != JY_GCOUNT && type != JY_PNCOUNT) return nd->fail(JY_EINVAL, "type must be JY_GCOUNT or JY_PNCOUNT");
  if (type == JY_GCOUNT && sign) return nd->fail(JY_EINVAL, "GCOUNT cells have no sign");
  NdJob j;
  j.kind = K_COUNTER;
  j.type = type;
  j.n = n;
  j.mem = mem;
  if (mem == JY_DEVICE) {
    const void* a[6] = {kb, ko, co, sign, col, val};
    std::copy(a, a + 6, j.a);
    return submit(nd, std::move(j));
  }
  if (ko[n] < ko[0]) return nd->fail(JY_EINVAL, "key offsets are not ascending");
  if (co[n] < co[0]) return nd->fail(JY_EINVAL, "cell offsets are not ascending");
  u32 nrep;
  {
    std::lock_guard<std::mutex> g(nd->mu);
    nrep = nd->nrep;
  }
  for (u64 c = co[0]; c < co[n]; c++) {
    if (col[c] >= nrep) return nd->fail(JY_ERANGE, "column names no registered replica");
    if (sign && sign[c] > 1) return nd->fail(JY_ERANGE, "sign must be 0 (P) or 1 (N)");
  }
  Pack pk;
  pk.add(0, kb, 1, ko[0], ko[n]);
  pk.add(1, ko, 8, 0, n + 1);
  pk.add(2, co, 8, 0, n + 1);
  if (sign) pk.add(3, sign, 1, co[0], co[n]);
  pk.add(4, col, 2, co[0], co[n]);
  pk.add(5, val, 8, co[0], co[n]);
  JY_TRY(pack_host(nd, pk, j));
  return submit(nd, std::move(j));
}

int32_t jy_node_treg_converge(jy_node* nd, uint64_t n, const uint8_t* kb, const uint64_t* ko, const uint64_t* ts,
                              const uint8_t* vb, const uint64_t* vo, int32_t mem) {
  JY_TRY(call_check(nd, mem, n));
  NdJob j;
  j.kind = K_TREG;
  j.n = n;
  j.mem = mem;
  if (mem == JY_DEVICE) {
    const void* a[5] = {kb, ko, ts, vb, vo};
    std::copy(a, a + 5, j.a);
    return submit(nd, std::move(j));
  }
  if (ko[n] < ko[0]) return nd->fail(JY_EINVAL, "key offsets are not ascending");
  JY_TRY(values_check(nd, vo, 0, n, JY_HOST));
  Pack pk;
  pk.add(0, kb, 1, ko[0], ko[n]);
  pk.add(1, ko, 8, 0, n + 1);
  pk.add(2, ts, 8, 0, n);
  pk.add(3, vb, 1, vo[0], vo[n]);
  pk.add(4, vo, 8, 0, n + 1);
  JY_TRY(pack_host(nd, pk, j));
  return submit(nd, std::move(j));
}

int32_t jy_node_tlog_converge(jy_node* nd, uint64_t n, const uint8_t* kb, const uint64_t* ko, const uint64_t* cutoff,
                              const uint64_t* eo, const uint64_t* ts, const uint8_t* vb, const uint64_t* vo,
                              int32_t mem) {
  JY_TRY(call_check(nd, mem, n));
  NdJob j;
  j.kind = K_TLOG;
  j.n = n;
  j.mem = mem;
  if (mem == JY_DEVICE) {
    const void* a[7] = {kb, ko, cutoff, eo, ts, vb, vo};
    std::copy(a, a + 7, j.a);
    return submit(nd, std::move(j));
  }
  if (ko[n] < ko[0]) return nd->fail(JY_EINVAL, "key offsets are not ascending");
  if (eo[n] < eo[0]) return nd->fail(JY_EINVAL, "entry offsets are not ascending");
  JY_TRY(values_check(nd, vo, eo[0], eo[n], JY_HOST));
  Pack pk;
  pk.add(0, kb, 1, ko[0], ko[n]);
  pk.add(1, ko, 8, 0, n + 1);
  pk.add(2, cutoff, 8, 0, n);
  pk.add(3, eo, 8, 0, n + 1);
  pk.add(4, ts, 8, eo[0], eo[n]);
  pk.add(5, vb, 1, vo[eo[0]], vo[eo[n]]);
  pk.add(6, vo, 8, eo[0], eo[n] + 1);
  JY_TRY(pack_host(nd, pk, j));
  return submit(nd, std::move(j));
}

int32_t jy_node_ujson_converge(jy_node* nd, uint64_t n, const uint8_t* kb, const uint64_t* ko, const uint64_t* eo,
                               const uint64_t* dots, const uint64_t* elems, const uint64_t* vvo, const uint64_t* vv,
                               const uint64_t* clo, const uint64_t* cloud, int32_t mem) {
  JY_TRY(call_check(nd, mem, n));
  NdJob j;
  j.kind = K_UJSON;
  j.n = n;
  j.mem = mem;
  if (mem == JY_DEVICE) {
    const void* a[9] = {kb, ko, eo, dots, elems, vvo, vv, clo, cloud};
    std::copy(a, a + 9, j.a);
    return submit(nd, std::move(j));
  }
  if (ko[n] < ko[0]) return nd->fail(JY_EINVAL, "key offsets are not ascending");
  if (eo[n] < eo[0] || vvo[n] < vvo[0] || clo[n] < clo[0])
    return nd->fail(JY_EINVAL, "element / vv / cloud offsets are not ascending");
  Pack pk;
  pk.add(0, kb, 1, ko[0], ko[n]);
  pk.add(1, ko, 8, 0, n + 1);
  pk.add(2, eo, 8, 0, n + 1);
  pk.add(3, dots, 8, eo[0], eo[n]);
  pk.add(4, elems, 8, eo[0], eo[n]);
  pk.add(5, vvo, 8, 0, n + 1);
  pk.add(6, vv, 8, vvo[0], vvo[n]);
  pk.add(7, clo, 8, 0, n + 1);
  pk.add(8, cloud, 8, clo[0], clo[n]);
  JY_TRY(pack_host(nd, pk, j));
  return submit(nd, std::move(j));
}

int32_t jy_node_counter_converge_block(jy_node* nd, int32_t type, uint32_t ncols, const uint16_t* cols_all,
                                       uint32_t slot0, uint32_t nslots, const uint64_t* vals_p,
                                       const uint64_t* vals_n) {
  if (!nd) return JY_EINVAL;
  JY_TRY(exec_pending(nd));
  if (type != JY_GCOUNT && type != JY_PNCOUNT) return nd->fail(JY_EINVAL, "type must be JY_GCOUNT or JY_PNCOUNT");
  if ((type == JY_PNCOUNT) != (vals_n != nullptr)) return nd->fail(JY_EINVAL, "vals_n is given iff PNCOUNT");
  if (ncols == 0 || nslots == 0) return JY_OK;
  NdJob j;
  j.kind = K_BLOCK;
  j.type = type;
  j.ncols = ncols;
  j.slot0 = slot0;
  j.nslots = nslots;
  j.cols.assign(cols_all, cols_all + (u64)nd->S * ncols);
  j.a[0] = vals_p;
  j.a[1] = vals_n;
  return submit(nd, std::move(j));
}

int32_t jy_node_fence(jy_node* nd) {
  if (!nd) return JY_EINVAL;
  return exec_fence(nd);
}

// the node mutex for a caller: announced, so the worker steps aside between jobs
static void lock_caller(jy_node* nd) {
  nd->lock_waiters.fetch_add(1, std::memory_order_acq_rel);
  nd->mu.lock();
  nd->lock_waiters.fetch_sub(1, std::memory_order_acq_rel);
}

int32_t jy_node_lock(jy_node* nd) {
  if (!nd) return JY_EINVAL;
  const int32_t rc = exec_fence(nd);
  lock_caller(nd);
  return rc;
}

int32_t jy_node_lock_type(jy_node* nd, int32_t type) {
  if (!nd) return JY_EINVAL;
  if (type != JY_NODE_NOFENCE && (type < 0 || type >= JY_NTYPES)) return nd->fail(JY_EINVAL, "bad type");
  const int32_t rc = type == JY_NODE_NOFENCE ? exec_pending(nd) : exec_fence_type(nd, type);
  lock_caller(nd);
  return rc;
}

int32_t jy_node_pending(jy_node* nd, int32_t type, uint64_t* n_out) {
  if (!nd) return JY_EINVAL;
  if (type >= JY_NTYPES) return nd->fail(JY_EINVAL, "bad type");
  std::lock_guard<std::mutex> lk(nd->qmu);
  *n_out = type < 0 ? nd->submitted - nd->finished : nd->sub_t[type] - nd->fin_t[type];
  return JY_OK;
}

int32_t jy_node_exchange_plan(uint32_t S, uint32_t rank, uint32_t W, uint32_t nwires, const int32_t* wire_gran,
                              const int32_t* wire_esize, const uint64_t* send_cnt, const uint64_t* recv_cnt,
                              uint64_t cap, uint64_t* ops_out, uint64_t* nops_out) {
  if (S == 0 || S > kMaxS || rank >= S || W == 0 || W > kMaxW) return JY_EINVAL;
  std::vector<Wire> wires(nwires);
  for (u32 i = 0; i < nwires; i++) {
    if (wire_gran[i] < 0 || (u32)wire_gran[i] >= W || wire_esize[i] <= 0) return JY_EINVAL;
    wires[i] = Wire{wire_gran[i], wire_esize[i], 0, 0};
  }
  std::vector<u64> sc((u64)kMaxS * W, 0), rc((u64)kMaxS * W, 0);
  std::copy(send_cnt, send_cnt + (u64)S * W, sc.begin());
  std::copy(recv_cnt, recv_cnt + (u64)S * W, rc.begin());
  std::vector<XOp> ops;
  plan_payload(S, rank, W, wires, sc.data(), rc.data(), ops);
  *nops_out = ops.size();
  for (u64 i = 0; i < ops.size() && i < cap; i++) {
    const XOp& o = ops[i];
    const u64 v[6] = {o.kind, o.wire, o.peer, o.soff, o.roff, o.bytes};
    std::copy(v, v + 6, ops_out + 6 * i);
  }
  return JY_OK;
}

int32_t jy_node_arena_gc(jy_node* nd, uint32_t enable) {
  if (!nd) return JY_EINVAL;
  std::lock_guard<std::mutex> g(nd->mu);
  nd->arena_gc = enable != 0;
  return JY_OK;
}

void jy_node_unlock(jy_node* nd) {
  if (nd) nd->mu.unlock();
}

}  // extern "C"
