// k_keys.hip -- device key directory: String key -> dense slot, gfx950.
//
// Replaces the per-type `Map[String, CRDT]` probe of `_data_for(key)`
// (repo_gcount.pony:36-41; same in every repo_*.pony) -- create on miss --
// and `_data(key)?` (repo_gcount.pony:53-55) -- look up only.  SURVEY 8f #1.
//
// HBM layout per type (KeyDir):
//   bytes[]      key bytes, appended in slot order
//   kref[slot]   (byte offset << 24) | length
//   khash[slot]  64-bit table hash (kept for rehashing)
//   kw[slot]     the key's bytes 0..7 and 8..15, zero filled (16 B)
//   table[tcap]  open addressing, linear probing, tcap a power of two kept
//                >= 2x the keys: an 8-B entry tag32 << 32 | slot (EMPTY ~0).
//                The position is the top bits of the hash, the tag its low
//                32 bits.  8 B per entry keeps the table MALL-resident at
//                node scale (2^24 entries: 128 MiB of the 256 MiB Infinity
//                Cache; round 5's 32-B records {entry, length, two key words}
//                made it 512 MiB, and the probe's one random line per key
//                came from HBM: 329-440 us for 8.39M keys).  A tag match is
//                confirmed against the slot's kref (length) and kw (first 16
//                bytes), which a batch in slot order reads as a stream;
//                longer keys compare the rest of their bytes in the
//                directory.
//
// Interning n keys is deterministic and lock-free (no thread ever waits on
// another):
//   K1 probe      every key; found -> its slot; misses counted (+ their bytes)
//   K2 claim      each missing key probes again; at an EMPTY entry it CASes in
//                 a PENDING entry carrying its own input index.  A key that
//                 meets a PENDING entry with its tag compares bytes with that
//                 input key (input bytes, already in HBM) and joins its group.
//   K3 first      atomicMin of the input index per group: slots are handed
//                 out in order of first occurrence in the input, as the host
//                 map would, whatever order the CASes landed in
//   scan          ranks of first occurrences, byte offsets of their keys
//   K4 commit     slot = old count + rank; first occurrences copy their bytes
//                 and fill kref / khash; claimers turn PENDING into final
//
// Roofline: HBM/latency.  Per key: its bytes read once (hash and compare
// words), one table probe chain (32-B records), 4 B slot out; a new key adds
// its bytes + 16 B of kref / khash + its 32-B record written.


#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "jy_dscan.hpp"
#include "jy_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr u64 kEmpty = ~0ull;
constexpr u32 kMiss = 0xFFFFFFFFu;
constexpr u64 kPending = 0x80000000ull;
constexpr u64 kIdxMask = 0x7FFFFFFFull;

__device__ __forceinline__ u64 gid() { return (u64)blockIdx.x * kThreads + threadIdx.x; }

// The table hash is the directory's own (not jy_key_owner's FNV-1a, so the
// table position is independent of the owner shard: owner = h mod S would
// otherwise pin the low bits of every key of a shard).  The bytes come a
// word at a time (jy_ld8u): the key's first two words are loaded together,
// before any byte is hashed, and reused by the comparisons -- a byte loop
// paid one dependent round trip per byte (K1 probe: 460 us for 8.9M keys).
// They are hashed a word at a time as well: a 16-B key costs 4 64-bit
// multiplies instead of FNV-1a's 16 + 4.
struct KeyW {
  u64 w0, w1;  // bytes 0..7 and 8..15, zero filled past the key
};
__device__ __forceinline__ KeyW key_words(const uint8_t* __restrict__ p, u64 len) {
  return KeyW{jy_ld8u(p, len), len > 8 ? jy_ld8u(p + 8, len - 8) : 0ull};
}
// a word folds in with one multiply + xorshift, both bijections of the state,
// so two keys of one length that differ in one word always differ before the
// finaliser (the length seeds the state: "a" and "a\0" differ too)
__device__ __forceinline__ u64 mix_word(u64 h, u64 w) {
  h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
  return h ^ (h >> 31);
}
__device__ __forceinline__ u64 table_hash(const uint8_t* __restrict__ p, u64 len, const KeyW& kw) {
  u64 h = (len * 0x9E3779B97F4A7C15ull) ^ 0xCBF29CE484222325ull;
  h = mix_word(h, kw.w0);
  if (len > 8) h = mix_word(h, kw.w1);
  for (u64 i = 16; i < len; i += 8) h = mix_word(h, jy_ld8u(p + i, len - i));
  h ^= h >> 30;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 27;
  h *= 0x94D049BB133111EBull;
  h ^= h >> 31;
  return h;
}

// the n bytes at a equal the key k whose first words are kw (n = its length)
__device__ __forceinline__ bool key_equal(const uint8_t* __restrict__ a, const uint8_t* __restrict__ k, u64 n,
                                          const KeyW& kw) {
  if (jy_ld8u(a, n) != kw.w0) return false;
  if (n > 8 && jy_ld8u(a + 8, n - 8) != kw.w1) return false;
  for (u64 i = 16; i < n; i += 8)
    if (jy_ld8u(a + i, n - i) != jy_ld8u(k + i, n - i)) return false;
  return true;
}

// bytes 16.. of a key longer than 16 (its record matched its length and
// first 16 bytes).  NOT inlined: inlined into k_key_probe's loop, this
// compiler (ROCm 7.2 clang, gfx950) lost the matched slot on the long-key
// path -- the structurised loop's exit copied the old "miss" value over it --
// so no key over 16 bytes was ever found again and each was re-created on
// every call (tests/test_keys_gpu.py::test_long_keys_found_again)
__device__ __attribute__((noinline)) bool key_tail_equal(const uint8_t* __restrict__ a, const uint8_t* __restrict__ k,
                                                         u64 n) {
  for (u64 i = 16; i < n; i += 8)
    if (jy_ld8u(a + i, n - i) != jy_ld8u(k + i, n - i)) return false;
  return true;
}

// table entries: tag32 << 32 | slot (kPending: a claim of this launch, slot = its input index); EMPTY ~0
struct Dir {
  const uint8_t* bytes;
  u64* kref;
  u64* khash;
  ulonglong2* kw;  // [slot] {w0, w1}
  u64* table;
  u64 mask;
  u32 shift;  // 64 - log2(tcap)
};

struct In {
  const uint8_t* kb;
  const u64* ko;
  u64 n;
};

__device__ __forceinline__ u32 tag_of(u64 t) { return (u32)t; }

// K1: look every key up; misses counted with their bytes.  The counts are
// per-workgroup partials (summed by k_key_sum): one global atomic per miss on
// three shared words serialised ~65K misses per 1M-key batch (~0.6 ms).
// One key per lane.  (Round 5 measured 2, 4 and 8 keys per lane with their
// loads issued together, in-box A/B of the node TREG call, 8.39M keys, ms per
// call: 1 key 0.738 / 0.741, 2 keys 0.742 / 0.747, 4 keys 0.809 / 0.806, 8
// keys 0.968 / 0.962 -- the registers cost more occupancy than the chains in
// flight gain.)
constexpr u64 kProbeKeys = kThreads;  // keys per probe workgroup
__global__ __launch_bounds__(kThreads) void k_key_probe(In I, Dir D, u32* __restrict__ res, u64* __restrict__ th,
                                                        u64* __restrict__ parts) {
  __shared__ u64 red[3][kThreads / 64];
  u64 c[3] = {0, 0, 0};
  const u64 i = gid();
  if (i < I.n) {
    const u64 a = I.ko[i], len = I.ko[i + 1] - a;
    const KeyW kw = key_words(I.kb + a, len);
    const u64 t = table_hash(I.kb + a, len, kw);
    u64 p = t >> D.shift;
    u32 slot = kMiss;
    // at most every entry once: the table always keeps EMPTY entries, so a
    // walk that finds none met a corrupt table -- it ends, and is counted
    for (u64 walk = 0;; walk++) {
      if (walk > D.mask) {
        c[2] |= 1ull << 32;  // counted above the oversized keys: the call fails
        break;
      }
      const u64 e = D.table[p];
      if (e == kEmpty) break;
      if ((u32)(e >> 32) == tag_of(t) && !(e & kPending)) {
        const u32 s = (u32)(e & kIdxMask);
        const u64 kr = D.kref[s];
        const ulonglong2 w = D.kw[s];
        if ((kr & JY_LR_LEN_MASK) == len && w.x == kw.w0 && w.y == kw.w1 &&
            (len <= 16 || key_tail_equal(D.bytes + (kr >> JY_LR_LEN_BITS), I.kb + a, len))) {
          slot = s;
          break;
        }
      }
      p = (p + 1) & D.mask;
    }
    res[i] = slot;
    if (slot == kMiss) {
      th[i] = t;  // read only for misses (claim, commit): a found key writes no hash
      c[0] = 1;
      c[1] = len;
      c[2] |= len > JY_LR_LEN_MASK;
    }
  }
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const u64 v = jyscan::wave_sum<u64>(c[q]);
    if ((threadIdx.x & 63) == 0) red[q][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    u64 v = 0;
#pragma unroll
    for (int j = 0; j < kThreads / 64; j++) v += red[threadIdx.x][j];
    parts[(u64)blockIdx.x * 3 + threadIdx.x] = v;
  }
}

// the probe's [nb][3] partials (misses, their bytes, oversized keys) summed
// by kSumGroups workgroups of 256 into [kSumGroups][3]; the host adds those
// up with its read-back.  (One workgroup of 1024 walking all the rows took 19
// us at 32.8K rows, the node TREG call's 8.39M keys: its loads wait in line.)
// The words land in mapped pinned memory, [kSumGroups][3] and then the
// completion number.  The last
// workgroup to publish writes the completion number (system-scope release
// after every workgroup's system fence), so the host spins on one word of
// its own memory instead of waking from a stream synchronise.
constexpr int kSumThreads = 256;
constexpr u32 kSumGroups = 128;
constexpr u32 kWordDone = kSumGroups * 3, kSumWords = kWordDone + 1;
__global__ __launch_bounds__(kSumThreads) void k_key_sum(const u64* __restrict__ parts, u64 nb,
                                                         u64* __restrict__ counts, u32* __restrict__ done, u64 seq) {
  __shared__ u64 red[3][kSumThreads / 64];
  u64 v[3] = {0, 0, 0};
  for (u64 b = (u64)blockIdx.x * kSumThreads + threadIdx.x; b < nb; b += (u64)gridDim.x * kSumThreads) {
#pragma unroll
    for (int q = 0; q < 3; q++) v[q] += parts[b * 3 + q];
  }
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const u64 w = jyscan::wave_sum<u64>(v[q]);
    if ((threadIdx.x & 63) == 0) red[q][threadIdx.x >> 6] = w;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    u64 t = 0;
    for (int w = 0; w < kSumThreads / 64; w++) t += red[threadIdx.x][w];
    // mapped pinned memory: system-scope vector stores
    __hip_atomic_store(counts + (u64)blockIdx.x * 3 + threadIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x < 3) __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const u32 prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {  // the last: every other workgroup's words are out
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
      __threadfence_system();
      __hip_atomic_store(counts + kWordDone, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// K2: claim an EMPTY entry (PENDING | own index) or join the group of an
// equal key that claimed first
__global__ __launch_bounds__(kThreads) void k_key_claim(In I, Dir D, const u32* __restrict__ res,
                                                        const u64* __restrict__ th, u32* __restrict__ owner,
                                                        u64* __restrict__ pos) {
  const u64 i = gid();
  if (i >= I.n || res[i] != kMiss) return;
  const uint8_t* k = I.kb + I.ko[i];
  const u64 len = I.ko[i + 1] - I.ko[i];
  const u64 t = th[i];
  const KeyW kw = key_words(k, len);
  const u64 mine = ((u64)tag_of(t) << 32) | kPending | i;
  u64 p = t >> D.shift;
  u64 e = D.table[p];
  for (u64 walk = 0; walk <= D.mask; walk++) {  // (an EMPTY entry or the group's claim is always met)
    if (e == kEmpty) {
      const u64 prev = atomicCAS(reinterpret_cast<unsigned long long*>(&D.table[p]), kEmpty, mine);
      if (prev == kEmpty) {
        owner[i] = (u32)i;
        pos[i] = p;
        return;
      }
      e = prev;  // look at what landed here
      continue;
    }
    if ((u32)(e >> 32) == tag_of(t) && (e & kPending)) {
      const u64 j = e & kIdxMask;
      const u64 lj = I.ko[j + 1] - I.ko[j];
      if (lj == len && key_equal(I.kb + I.ko[j], k, len, kw)) {
        owner[i] = (u32)j;
        return;
      }
    }
    p = (p + 1) & D.mask;
    e = D.table[p];
  }
}

// K3: the first input index of every group
__global__ __launch_bounds__(kThreads) void k_key_first(u64 n, const u32* __restrict__ res,
                                                        const u32* __restrict__ owner, u32* __restrict__ first) {
  const u64 i = gid();
  if (i >= n || res[i] != kMiss) return;
  atomicMin(first + owner[i], (u32)i);
}

__global__ __launch_bounds__(kThreads) void k_key_flags(In I, const u32* __restrict__ res,
                                                        const u32* __restrict__ owner, const u32* __restrict__ first,
                                                        u32* __restrict__ flag, u64* __restrict__ blen) {
  const u64 i = gid();
  if (i > I.n) return;
  u32 f = 0;
  u64 b = 0;
  if (i < I.n && res[i] == kMiss && first[owner[i]] == (u32)i) {
    f = 1;
    b = I.ko[i + 1] - I.ko[i];
  }
  flag[i] = f;
  blen[i] = b;
}

// K4: slots out; first occurrences store their key; claimers publish
__global__ __launch_bounds__(kThreads) void k_key_commit(In I, Dir D, uint8_t* __restrict__ dbytes, u64 base_slot,
                                                         u64 base_byte, const u32* res,  // (res aliases slots)
                                                         const u64* __restrict__ th, const u32* __restrict__ owner,
                                                         const u64* __restrict__ pos, const u32* __restrict__ first,
                                                         const u32* __restrict__ rank, const u64* __restrict__ boff,
                                                         u32* slots) {
  const u64 i = gid();
  if (i >= I.n) return;
  if (res[i] != kMiss) return;  // found by the probe, already in slots[i]
  const u32 o = owner[i];
  const u32 f = first[o];
  const u64 slot = base_slot + rank[f];
  slots[i] = (u32)slot;
  if (f == (u32)i) {
    const u64 len = I.ko[i + 1] - I.ko[i];
    const u64 at = base_byte + boff[i];
    const uint8_t* src = I.kb + I.ko[i];
    for (u64 b = 0; b < len; b++) dbytes[at + b] = src[b];  // (word reads + byte stores: 72 -> 79 us)
    D.kref[slot] = (at << JY_LR_LEN_BITS) | len;
    D.khash[slot] = th[i];
    const KeyW kw = key_words(src, len);
    D.kw[slot] = ulonglong2{kw.w0, kw.w1};
  }
  if (o == (u32)i)  // (probes and claims of other keys run in other launches)
    D.table[pos[i]] = ((u64)tag_of(th[i]) << 32) | slot;
}

// rebuild the table from the per-slot hashes
__global__ __launch_bounds__(kThreads) void k_key_rehash(Dir D, u64 nk) {
  const u64 s = gid();
  if (s >= nk) return;
  const u64 t = D.khash[s];
  const u64 e = ((u64)tag_of(t) << 32) | s;
  u64 p = t >> D.shift;
  while (atomicCAS(reinterpret_cast<unsigned long long*>(&D.table[p]), kEmpty, e) != kEmpty) p = (p + 1) & D.mask;
}

// how the host waits for the sums' completion word: a tight spin (pause) for
// as long as a large probe takes (8.39M keys: ~0.3-0.45 ms), then a yielding
// poll -- earlier converges may still be queued ahead of the probe on the
// engine stream, and the core is the other repos' too -- and past kSpinUs a
// stream synchronise (which also reports a launch that never ends)
constexpr double kTightUs = 600.0;
constexpr double kSpinUs = 20000.0;

u32 blocks_for(u64 n) { return (u32)std::max<u64>(1, (n + kThreads - 1) / kThreads); }

#define LAUNCH(k, n, ...)                                                                          \
  do {                                                                                             \
    hipLaunchKernelGGL(k, dim3(blocks_for(n)), dim3(kThreads), 0, eng->stream, __VA_ARGS__);     \
    JY_HIP(eng, hipGetLastError());                                                                \
  } while (0)

Dir dir_of(KeyDir& K) {
  Dir D;
  D.bytes = K.bytes;
  D.kref = K.kref;
  D.khash = K.khash;
  D.kw = reinterpret_cast<ulonglong2*>(K.kw);
  D.table = K.table;
  D.mask = K.tcap - 1;
  D.shift = 64 - K.lg;
  return D;
}

int32_t grow_table(jy_engine* eng, KeyDir& K, u64 need_keys) {
  u64 want = 1024;
  u32 lg = 10;
  while (want < 2 * need_keys) {
    want <<= 1;
    lg++;
  }
  if (K.table && want <= K.tcap) return JY_OK;
  jy_dev_free(eng, K.table);
  K.table = nullptr;
  JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&K.table), want * 8, "key table"));
  K.tcap = want;
  K.lg = lg;
  JY_HIP(eng, hipMemsetAsync(K.table, 0xFF, want * 8, eng->stream));
  if (K.n) LAUNCH(k_key_rehash, K.n, dir_of(K), K.n);
  return JY_OK;
}

int32_t grow_slots(jy_engine* eng, KeyDir& K, u64 need) {
  if (need <= K.scap && K.kref) return JY_OK;
  const u64 nc = std::max<u64>(std::max<u64>(need, K.scap * 2), 1024);
  void* a = K.kref;
  JY_TRY(jy_realloc(eng, &a, K.n * 8, nc * 8, false));
  K.kref = static_cast<u64*>(a);
  void* b = K.khash;
  JY_TRY(jy_realloc(eng, &b, K.n * 8, nc * 8, false));
  K.khash = static_cast<u64*>(b);
  void* c = K.kw;
  JY_TRY(jy_realloc(eng, &c, K.n * 16, nc * 16, false));
  K.kw = static_cast<u64*>(c);
  K.scap = nc;
  return JY_OK;
}

int32_t grow_bytes(jy_engine* eng, KeyDir& K, u64 need) {
  if (need <= K.bcap && K.bytes) return JY_OK;
  const u64 nc = std::max<u64>(std::max<u64>(need, K.bcap * 2), 1 << 16);
  void* a = K.bytes;
  JY_TRY(jy_realloc(eng, &a, K.blen, nc, false));
  K.bytes = static_cast<uint8_t*>(a);
  K.bcap = nc;
  return JY_OK;
}

}  // namespace

int32_t jy_keydir_reserve(jy_engine* eng, int32_t type, u64 cap) {
  KeyDir& K = eng->kdir[type];
  JY_TRY(grow_slots(eng, K, cap));
  return grow_table(eng, K, cap);
}

void jy_keydir_free(jy_engine* eng, KeyDir& K) {
  for (void* p : {static_cast<void*>(K.bytes), static_cast<void*>(K.kref), static_cast<void*>(K.khash),
                  static_cast<void*>(K.kw), static_cast<void*>(K.table)})
    jy_dev_free(eng, p);
  K = KeyDir{};
}

// Device interning / lookup of n keys (device pointers).  Returns the number
// of keys created in *created.  Synchronises (the host must know the new
// key count before any call sizes work by it).
// after_probe (optional) runs on the host once the probe is enqueued and
// before the host waits for its counts: a caller stages its next inputs there
// while the GPU probes
int32_t jy_keydir_run(jy_engine* eng, int32_t type, u64 n, const uint8_t* kb, const u64* ko, u32* slots, bool create,
                      u64* created, int32_t (*after_probe)(void*), void* arg) {
  *created = 0;
  if (n == 0) return JY_OK;
  if (n >= kIdxMask) return eng->fail(JY_ERANGE, "too many keys in one call");
  KeyDir& K = eng->kdir[type];
  JY_TRY(grow_slots(eng, K, std::max<u64>(K.n, 1)));
  JY_TRY(grow_table(eng, K, std::max<u64>(K.n, 1)));
  void* p;
  JY_TRY(jy_scratch(eng, 20, n * 8 + 64, &p));
  if (!eng->kd_words) {  // the probe's partial sums land in mapped pinned memory: no copy back
    void* h = nullptr;
    JY_HIP(eng, hipHostMalloc(&h, kSumWords * 8, hipHostMallocMapped));
    std::memset(h, 0, kSumWords * 8);
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      hipHostFree(h);
      return eng->fail(JY_EHIP, "key directory: mapped pinned words");
    }
    eng->kd_words = static_cast<u64*>(h);
    eng->kd_words_dev = static_cast<u64*>(d);
  }
  if (!eng->kd_done) {
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&eng->kd_done), 64, "key probe sums' counter"));
    JY_HIP(eng, hipMemsetAsync(eng->kd_done, 0, 64, eng->stream));
  }
  // the probe's answers go straight to the caller's slots (a found key's slot
  // or kMiss): every later kernel reads and rewrites index i in the same
  // thread, so a lookup, or an intern that finds every key, is done after the
  // probe (no copy of n words: 19 us at 8.39M keys)
  u32* res = slots;
  u64* th = static_cast<u64*>(p);
  u64* counts = eng->kd_words_dev;  // [sum groups][3] misses, their bytes, oversized keys (mapped)
  In I{kb, ko, n};
  const u64 nb = (n + kProbeKeys - 1) / kProbeKeys;
  void* pp;
  JY_TRY(jy_scratch(eng, 29, nb * 24 + 64, &pp));
  u64* parts = static_cast<u64*>(pp);
  hipLaunchKernelGGL(k_key_probe, dim3((u32)nb), dim3(kThreads), 0, eng->stream, I, dir_of(K), res, th, parts);
  JY_HIP(eng, hipGetLastError());
  const u32 ng = (u32)std::min<u64>(kSumGroups, (nb + kSumThreads - 1) / kSumThreads);
  const u64 seq = ++eng->kd_seq;
  hipLaunchKernelGGL(k_key_sum, dim3(ng), dim3(kSumThreads), 0, eng->stream, parts, nb, counts, eng->kd_done, seq);
  JY_HIP(eng, hipGetLastError());
  if (after_probe) JY_TRY(after_probe(arg));  // (what it enqueues here follows the sums)
  const u64* hg = eng->kd_words;
  const double t0 = jy_now_us();
  // the sums' completion number means every launch before them is done as
  // well (what after_probe enqueued may still run: it is stream-ordered
  // before any use).  A launch that never ends (a fault) leaves the number
  // unwritten: past the spin budget the stream synchronise reports it.
  bool seen = false;
  for (u32 spin = 0;; spin++) {
    if (__atomic_load_n(hg + kWordDone, __ATOMIC_ACQUIRE) == seq) {
      seen = true;
      break;
    }
    if ((spin & 255) == 255) {
      const double w = jy_now_us() - t0;
      if (w > kSpinUs) break;
      if (w > kTightUs) std::this_thread::yield();
    }
    __builtin_ia32_pause();
  }
  if (!seen) JY_HIP(eng, hipStreamSynchronize(eng->stream));
  JY_TRACE("keydir %llu keys: probe counts after %.1f us of waiting (%s)", (unsigned long long)n, jy_now_us() - t0,
           seen ? "spin" : "stream sync");
  u64 hc[3] = {0, 0, 0};
  for (u32 g = 0; g < ng; g++)
    for (int q = 0; q < 3; q++) hc[q] += hg[g * 3 + q];
  const u64 m = hc[0], mbytes = hc[1];
  JY_TRACE("keydir %llu keys: %llu misses (create %d)", (unsigned long long)n, (unsigned long long)m, (int)create);
  if (hc[2] >> 32) return eng->fail(JY_EINVAL, "key directory: a probe walked the whole table (corrupt table)");
  if (!create || m == 0) return JY_OK;  // (a miss's kMiss is JY_NO_SLOT)
  if (hc[2]) return eng->fail(JY_ERANGE, "key longer than 16 MiB");
  if (K.n + m >= kIdxMask) return eng->fail(JY_ERANGE, "slot space exhausted");
  JY_TRY(grow_table(eng, K, K.n + m));
  JY_TRY(grow_slots(eng, K, K.n + m));
  JY_TRY(grow_bytes(eng, K, K.blen + mbytes));
  JY_TRY(jy_scratch(eng, 21, n * 16 + 64, &p));
  u32* owner = static_cast<u32*>(p);
  u32* first = owner + n;
  u64* pos = reinterpret_cast<u64*>((reinterpret_cast<uintptr_t>(first + n) + 15) & ~uintptr_t(15));
  JY_TRY(jy_scratch(eng, 22, (n + 1) * 8 + 64, &p));
  u32* flag = static_cast<u32*>(p);
  u32* rank = flag + n + 1;
  JY_TRY(jy_scratch(eng, 23, (n + 1) * 16 + 64, &p));
  u64* blen = static_cast<u64*>(p);
  u64* boff = blen + n + 1;
  const Dir D = dir_of(K);
  JY_HIP(eng, hipMemsetAsync(first, 0xFF, n * 4, eng->stream));
  LAUNCH(k_key_claim, n, I, D, res, th, owner, pos);
  LAUNCH(k_key_first, n, n, res, owner, first);
  // (rank and byte offset packed into one word for one scan: the look-back
  // status words carry 40-bit values, jy_dscan.hpp -- kept as two scans)
  LAUNCH(k_key_flags, n + 1, I, res, owner, first, flag, blen);
  JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, n + 1, jydscan::LdArr<u32>{flag}, jydscan::StArr<u32>{rank})));
  JY_TRY((jydscan::scan<jydscan::OpSum, false>(eng, n + 1, jydscan::LdArr<u64>{blen}, jydscan::StArr<u64>{boff})));
  LAUNCH(k_key_commit, n, I, D, K.bytes, K.n, K.blen, res, th, owner, pos, first, rank, boff, slots);
  u32 nnew = 0;
  u64 nbytes = 0;
  JY_HIP(eng, hipMemcpyAsync(&nnew, rank + n, 4, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(&nbytes, boff + n, 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  K.n += nnew;
  K.blen += nbytes;
  *created = nnew;
  return JY_OK;
}

// the key strings of slots [slot0, slot0 + n): the directory keeps them in
// slot order, so this is two device-to-host copies (the handles, then one
// byte range).  Blocks.
extern "C" int32_t jy_keys_export(jy_engine* eng, int32_t type, uint64_t slot0, uint64_t n, uint64_t* offs_out,
                                  uint8_t* bytes_out, uint64_t cap_bytes) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (type < 0 || type >= JY_NTYPES) return eng->fail(JY_ETYPE, "unknown CRDT type");
  KeyDir& K = eng->kdir[type];
  if (slot0 + n > K.n) return eng->fail(JY_ERANGE, "slots beyond the interned keys");
  offs_out[0] = 0;
  if (n == 0) return JY_OK;
  std::vector<u64> ref(n);
  JY_HIP(eng, hipMemcpyAsync(ref.data(), K.kref + slot0, n * 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  const u64 b0 = ref[0] >> 24;
  for (u64 i = 0; i < n; i++) {
    if ((ref[i] >> 24) != b0 + offs_out[i]) return eng->fail(JY_EINVAL, "key directory bytes out of slot order");
    offs_out[i + 1] = offs_out[i] + (ref[i] & JY_LR_LEN_MASK);
  }
  if (!bytes_out || cap_bytes < offs_out[n]) return JY_OK;  // sizes only
  if (offs_out[n]) {
    JY_HIP(eng, hipMemcpyAsync(bytes_out, K.bytes + b0, offs_out[n], hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
  }
  return JY_OK;
}
