// mc_keyprobe.hip -- reduced reproducer of the k_key_probe long-key miss
// (round 5, k_keys.hip:102-113): the directory's probe loop -- linear
// probing over 32-B records, a match on (tag, length, first 16 bytes), then
// the bytes past 16 compared in the directory -- built twice, with that tail
// compare inlined into the loop (as round 5 first shipped it) and as a
// noinline call (the fix).  Every key of the directory is looked up; the
// slot found must be the key's own.  Keys of 1..48 bytes.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mc_keyprobe tools/mc_keyprobe.hip
//   ./tools/mc_keyprobe            -> "inline: X misses of N, noinline: Y misses of N"
//
// The kernels restate the shipped loop shape with this file's own helpers
// (the same word loads, the same hash), so a difference between the two
// builds of the SAME source is the compiler's; the host computes the
// expected slots independently.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef uint64_t u64;
typedef uint32_t u32;

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      return 2;                                                                           \
    }                                                                                     \
  } while (0)

constexpr u64 kEmpty = ~0ull;
constexpr u32 kMiss = 0xFFFFFFFFu;

struct alignas(32) Rec {
  u64 e;  // tag32 << 32 | slot
  u64 len, w0, w1;
};

// the first min(8, avail) bytes at p, little endian, zero filled (aligned word loads)
__host__ __device__ inline u64 ld8u(const uint8_t* p, u64 avail) {
  if (avail == 0) return 0;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const u32 sh = (u32)(a & 7);
  const u64* w = reinterpret_cast<const u64*>(a - sh);
  u64 v = w[0] >> (8 * sh);
  if (sh && avail > 8 - sh) v |= w[1] << (64 - 8 * sh);
  if (avail < 8) v &= (1ull << (8 * avail)) - 1;
  return v;
}
__host__ __device__ inline u64 mixw(u64 h, u64 w) {
  h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
  return h ^ (h >> 31);
}
__host__ __device__ inline u64 thash(const uint8_t* p, u64 len) {
  u64 h = (len * 0x9E3779B97F4A7C15ull) ^ 0xCBF29CE484222325ull;
  for (u64 i = 0; i < len; i += 8) h = mixw(h, ld8u(p + i, len - i));
  h ^= h >> 30;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 27;
  h *= 0x94D049BB133111EBull;
  return h ^ (h >> 31);
}

__device__ __forceinline__ bool tail_inline(const uint8_t* __restrict__ a, const uint8_t* __restrict__ k, u64 n) {
  for (u64 i = 16; i < n; i += 8)
    if (ld8u(a + i, n - i) != ld8u(k + i, n - i)) return false;
  return true;
}
__device__ __attribute__((noinline)) bool tail_call(const uint8_t* __restrict__ a, const uint8_t* __restrict__ k,
                                                    u64 n) {
  for (u64 i = 16; i < n; i += 8)
    if (ld8u(a + i, n - i) != ld8u(k + i, n - i)) return false;
  return true;
}

template <bool kInline>
__global__ __launch_bounds__(256) void probe(const uint8_t* kb, const u64* ko, u64 n, const Rec* table, u64 mask,
                                             u32 shift, const uint8_t* dbytes, const u64* dref, u32* res) {
  const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const u64 a = ko[i], len = ko[i + 1] - a;
  const u64 w0 = ld8u(kb + a, len), w1 = len > 8 ? ld8u(kb + a + 8, len - 8) : 0;
  const u64 t = thash(kb + a, len);
  u64 p = t >> shift;
  u32 slot = kMiss;
  for (;;) {
    const Rec r = table[p];
    if (r.e == kEmpty) break;
    if ((u32)(r.e >> 32) == (u32)t && r.len == len && r.w0 == w0 && r.w1 == w1) {
      const u32 s = (u32)r.e;
      const uint8_t* d = dbytes + dref[s];
      if (len <= 16 || (kInline ? tail_inline(d, kb + a, len) : tail_call(d, kb + a, len))) {
        slot = s;
        break;
      }
    }
    p = (p + 1) & mask;
  }
  res[i] = slot;
}

int main(int argc, char** argv) {
  const u64 n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1u << 20);
  std::mt19937_64 rng(7);
  // the directory: n distinct keys of 1..48 bytes (a key index in the first 8 bytes keeps them distinct)
  std::vector<uint8_t> bytes;
  std::vector<u64> ref(n + 1);
  for (u64 k = 0; k < n; k++) {
    ref[k] = bytes.size();
    const u64 len = 9 + rng() % 40;
    u64 id = k;
    for (int b = 0; b < 8; b++, id >>= 8) bytes.push_back((uint8_t)id);
    for (u64 b = 8; b < len; b++) bytes.push_back((uint8_t)rng());
    while (bytes.size() % 8) bytes.push_back(0);  // 8-byte aligned starts, as the directory's words expect
  }
  ref[n] = bytes.size();
  std::vector<u64> klen(n);
  {  // the lengths drawn above (same seed, same draws)
    std::mt19937_64 r2(7);
    for (u64 k = 0; k < n; k++) {
      klen[k] = 9 + r2() % 40;
      for (u64 b = 8; b < klen[k]; b++) r2();
    }
  }
  u64 tcap = 1;
  while (tcap < 2 * n) tcap <<= 1;
  u32 shift = 64;
  for (u64 c = tcap; c > 1; c >>= 1) shift--;
  std::vector<Rec> table(tcap, Rec{kEmpty, 0, 0, 0});
  for (u64 k = 0; k < n; k++) {
    const uint8_t* p = bytes.data() + ref[k];
    const u64 t = thash(p, klen[k]);
    u64 q = t >> shift;
    while (table[q].e != kEmpty) q = (q + 1) & (tcap - 1);
    table[q] = Rec{((u64)(u32)t << 32) | k, klen[k], ld8u(p, klen[k]), klen[k] > 8 ? ld8u(p + 8, klen[k] - 8) : 0};
  }
  uint8_t* d_bytes;
  u64 *d_ref, *d_ko;
  Rec* d_table;
  u32* d_res;
  CHECK(hipMalloc(&d_bytes, bytes.size() + 16));
  CHECK(hipMalloc(&d_ref, (n + 1) * 8));
  CHECK(hipMalloc(&d_ko, (n + 1) * 8));
  CHECK(hipMalloc(&d_table, tcap * sizeof(Rec)));
  CHECK(hipMalloc(&d_res, n * 4));
  CHECK(hipMemcpy(d_bytes, bytes.data(), bytes.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_ref, ref.data(), (n + 1) * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_table, table.data(), tcap * sizeof(Rec), hipMemcpyHostToDevice));
  // the probe input: the keys back to back (a CSR, starts unaligned as a real batch's)
  std::vector<u64> st(n + 1);
  std::vector<uint8_t> packed;
  for (u64 k = 0; k < n; k++) {
    st[k] = packed.size();
    packed.insert(packed.end(), bytes.begin() + ref[k], bytes.begin() + ref[k] + klen[k]);
  }
  st[n] = packed.size();
  uint8_t* d_packed;
  CHECK(hipMalloc(&d_packed, packed.size() + 16));
  CHECK(hipMemcpy(d_packed, packed.data(), packed.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_ko, st.data(), (n + 1) * 8, hipMemcpyHostToDevice));
  std::vector<u32> res(n);
  u64 miss[2] = {0, 0};
  for (int v = 0; v < 2; v++) {
    CHECK(hipMemset(d_res, 0xAB, n * 4));
    if (v == 0)
      hipLaunchKernelGGL(probe<true>, dim3((u32)((n + 255) / 256)), dim3(256), 0, 0, d_packed, d_ko, n, d_table,
                         tcap - 1, shift, d_bytes, d_ref, d_res);
    else
      hipLaunchKernelGGL(probe<false>, dim3((u32)((n + 255) / 256)), dim3(256), 0, 0, d_packed, d_ko, n, d_table,
                         tcap - 1, shift, d_bytes, d_ref, d_res);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(res.data(), d_res, n * 4, hipMemcpyDeviceToHost));
    for (u64 k = 0; k < n; k++) miss[v] += res[k] != (u32)k;
  }
  printf("inline: %llu misses of %llu, noinline: %llu misses of %llu (keys of 9..48 bytes)\n",
         (unsigned long long)miss[0], (unsigned long long)n, (unsigned long long)miss[1], (unsigned long long)n);
  return 0;
}
