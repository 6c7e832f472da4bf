// mb_treg.hip -- microbenchmark of TREG LWW state layouts on gfx950.
// Not part of the product: used to pick the k_treg state layout.
// Winners are decided by timestamp only here (ties are the product's job).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>
typedef unsigned long long u64;
typedef unsigned int u32;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

// A: SoA state (ts, pre, lr), SoA delta, pairs per lane (the round-1 kernel)
template <bool WRITE>
__global__ __launch_bounds__(256) void kA(u64* ts, u64* pre, u64* lr, const u32* slot, const u64* dts,
                                          const u64* dpre, const u64* dlr, u64 npairs) {
  constexpr int U = 2;
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
  u32x2 s[U]; u64x2 t[U], p[U], l[U], t0[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 q = base + (u64)u * 256;
    if (q < npairs) {
      s[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(slot) + q);
      t[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(dts) + q);
      p[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(dpre) + q);
      l[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(dlr) + q);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++)
    if (base + (u64)u * 256 < npairs) { t0[u].x = ts[s[u].x]; t0[u].y = ts[s[u].y]; }
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (base + (u64)u * 256 >= npairs) continue;
    if (t[u].x > t0[u].x && WRITE) { ts[s[u].x] = t[u].x; pre[s[u].x] = p[u].x; lr[s[u].x] = l[u].x; }
    if (t[u].y > t0[u].y && WRITE) { ts[s[u].y] = t[u].y; pre[s[u].y] = p[u].y; lr[s[u].y] = l[u].y; }
    if (!WRITE && (t[u].x + p[u].x + l[u].x == 7 || t[u].y + p[u].y + l[u].y == 7)) ts[0] = 1;
  }
}

// C: AoS 32-B state record {ts, pre, lr, pad}; SoA delta; one key per lane, U keys
struct Rec { u64 ts, pre, lr, pad; };
__global__ __launch_bounds__(256) void kC(Rec* st, const u32* slot, const u64* dts, const u64* dpre,
                                          const u64* dlr, u64 n) {
  constexpr int U = 4;
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
  u32 s[U]; u64 t[U], t0[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) { s[u] = __builtin_nontemporal_load(slot + i); t[u] = __builtin_nontemporal_load(dts + i); }
  }
#pragma unroll
  for (int u = 0; u < U; u++) if (base + (u64)u * 256 < n) t0[u] = st[s[u]].ts;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n && t[u] > t0[u]) {
      u64x2 a; a.x = t[u]; a.y = dpre[i];
      u64x2 b; b.x = dlr[i]; b.y = 0;
      reinterpret_cast<u64x2*>(st + s[u])[0] = a;
      reinterpret_cast<u64x2*>(st + s[u])[1] = b;
    }
  }
}

// D: ts SoA + {pre, lr} 16-B record; delta ts/slot SoA, pre/lr loaded only by winners
__global__ __launch_bounds__(256) void kD(u64* ts, u64x2* pl, const u32* slot, const u64* dts, const u64* dpre,
                                          const u64* dlr, u64 n) {
  constexpr int U = 4;
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
  u32 s[U]; u64 t[U], t0[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) { s[u] = __builtin_nontemporal_load(slot + i); t[u] = __builtin_nontemporal_load(dts + i); }
  }
#pragma unroll
  for (int u = 0; u < U; u++) if (base + (u64)u * 256 < n) t0[u] = ts[s[u]];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n && t[u] > t0[u]) {
      u64x2 a; a.x = dpre[i]; a.y = dlr[i];
      ts[s[u]] = t[u];
      pl[s[u]] = a;
    }
  }
}

// D2: like D but delta pre/lr loaded for all (coalesced) up front
__global__ __launch_bounds__(256) void kD2(u64* ts, u64x2* pl, const u32* slot, const u64* dts, const u64* dpre,
                                           const u64* dlr, u64 n) {
  constexpr int U = 4;
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
  u32 s[U]; u64 t[U], t0[U], p[U], l[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) {
      s[u] = __builtin_nontemporal_load(slot + i); t[u] = __builtin_nontemporal_load(dts + i);
      p[u] = __builtin_nontemporal_load(dpre + i); l[u] = __builtin_nontemporal_load(dlr + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) if (base + (u64)u * 256 < n) t0[u] = ts[s[u]];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n && t[u] > t0[u]) {
      u64x2 a; a.x = p[u]; a.y = l[u];
      ts[s[u]] = t[u];
      pl[s[u]] = a;
    }
  }
}

// D3: like D2 but ts rewritten by every lane (max), so ts lines are written whole
__global__ __launch_bounds__(256) void kD3(u64* ts, u64x2* pl, const u32* slot, const u64* dts, const u64* dpre,
                                           const u64* dlr, u64 n) {
  constexpr int U = 4;
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
  u32 s[U]; u64 t[U], t0[U], p[U], l[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) {
      s[u] = __builtin_nontemporal_load(slot + i); t[u] = __builtin_nontemporal_load(dts + i);
      p[u] = __builtin_nontemporal_load(dpre + i); l[u] = __builtin_nontemporal_load(dlr + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) if (base + (u64)u * 256 < n) t0[u] = ts[s[u]];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) {
      const bool w = t[u] > t0[u];
      ts[s[u]] = w ? t[u] : t0[u];
      if (w) { u64x2 a; a.x = p[u]; a.y = l[u]; pl[s[u]] = a; }
    }
  }
}

// D4: every lane rewrites ts and its 16-B handle (losers re-store the state
// handle they read), so both arrays are written as whole lines
__global__ __launch_bounds__(256) void kD4(u64* ts, u64x2* pl, const u32* slot, const u64* dts, const u64* dpre,
                                           const u64* dlr, u64 n) {
  constexpr int U = 4;
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
  u32 s[U]; u64 t[U], t0[U], p[U], l[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) {
      s[u] = __builtin_nontemporal_load(slot + i); t[u] = __builtin_nontemporal_load(dts + i);
      p[u] = __builtin_nontemporal_load(dpre + i); l[u] = __builtin_nontemporal_load(dlr + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) if (base + (u64)u * 256 < n) t0[u] = ts[s[u]];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) {
      const bool w = t[u] > t0[u];
      u64x2 a;
      if (w) { a.x = p[u]; a.y = l[u]; } else a = pl[s[u]];
      ts[s[u]] = w ? t[u] : t0[u];
      pl[s[u]] = a;
    }
  }
}

// D5: D2 with nontemporal stores
__global__ __launch_bounds__(256) void kD5(u64* ts, u64x2* pl, const u32* slot, const u64* dts, const u64* dpre,
                                           const u64* dlr, u64 n) {
  constexpr int U = 4;
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
  u32 s[U]; u64 t[U], t0[U], p[U], l[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) {
      s[u] = __builtin_nontemporal_load(slot + i); t[u] = __builtin_nontemporal_load(dts + i);
      p[u] = __builtin_nontemporal_load(dpre + i); l[u] = __builtin_nontemporal_load(dlr + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) if (base + (u64)u * 256 < n) t0[u] = ts[s[u]];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n && t[u] > t0[u]) {
      u64x2 a; a.x = p[u]; a.y = l[u];
      __builtin_nontemporal_store(t[u], ts + s[u]);
      __builtin_nontemporal_store(a, pl + s[u]);
    }
  }
}

// D6: D2 with 2 keys per lane and 8 per lane
template <int U>
__global__ __launch_bounds__(256) void kD6(u64* ts, u64x2* pl, const u32* slot, const u64* dts, const u64* dpre,
                                           const u64* dlr, u64 n) {
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
  u32 s[U]; u64 t[U], t0[U], p[U], l[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) {
      s[u] = __builtin_nontemporal_load(slot + i); t[u] = __builtin_nontemporal_load(dts + i);
      p[u] = __builtin_nontemporal_load(dpre + i); l[u] = __builtin_nontemporal_load(dlr + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) if (base + (u64)u * 256 < n) t0[u] = ts[s[u]];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n && t[u] > t0[u]) {
      u64x2 a; a.x = p[u]; a.y = l[u];
      ts[s[u]] = t[u];
      pl[s[u]] = a;
    }
  }
}

// C2: ts mirror (read) + 32-B record written whole by winners
__global__ __launch_bounds__(256) void kC2(u64* ts, Rec* st, const u32* slot, const u64* dts, const u64* dpre,
                                           const u64* dlr, u64 n) {
  constexpr int U = 4;
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
  u32 s[U]; u64 t[U], t0[U], p[U], l[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) {
      s[u] = __builtin_nontemporal_load(slot + i); t[u] = __builtin_nontemporal_load(dts + i);
      p[u] = __builtin_nontemporal_load(dpre + i); l[u] = __builtin_nontemporal_load(dlr + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) if (base + (u64)u * 256 < n) t0[u] = ts[s[u]];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n && t[u] > t0[u]) {
      ts[s[u]] = t[u];
      u64x2 a; a.x = t[u]; a.y = p[u];
      u64x2 b; b.x = l[u]; b.y = 0;
      reinterpret_cast<u64x2*>(st + s[u])[0] = a;
      reinterpret_cast<u64x2*>(st + s[u])[1] = b;
    }
  }
}

// E: SoA, every key's state rewritten (full-line stores), state pre/lr read
__global__ __launch_bounds__(256) void kE(u64* ts, u64* pre, u64* lr, const u32* slot, const u64* dts,
                                          const u64* dpre, const u64* dlr, u64 n) {
  constexpr int U = 4;
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) {
      u32 s = slot[i];
      u64 t = dts[i], t0 = ts[s];
      bool w = t > t0;
      u64 p = w ? dpre[i] : pre[s];
      u64 l = w ? dlr[i] : lr[s];
      ts[s] = w ? t : t0; pre[s] = p; lr[s] = l;
    }
  }
}

// F: ts SoA + 16-B {pre,lr}; delta AoS 32-B record {ts, pre, lr, slot}
__global__ __launch_bounds__(256) void kF(u64* ts, u64x2* pl, const Rec* d, u64 n) {
  constexpr int U = 4;
  const u64 base = (u64)blockIdx.x * (256 * U) + threadIdx.x;
  u64x2 a[U], b[U]; u64 t0[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n) {
      a[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(d + i));
      b[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(d + i) + 1);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) if (base + (u64)u * 256 < n) t0[u] = ts[(u32)b[u].y];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const u64 i = base + (u64)u * 256;
    if (i < n && a[u].x > t0[u]) {
      u64x2 v; v.x = a[u].y; v.y = b[u].x;
      ts[(u32)b[u].y] = a[u].x;
      pl[(u32)b[u].y] = v;
    }
  }
}

static void (*g_reset)() = nullptr;
template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(0);
  CK(hipDeviceSynchronize());
  float tot = 0;
  for (int r = 0; r < reps; r++) {
    g_reset();
    CK(hipEventRecord(a));
    f(r);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  return tot / reps;
}

int main(int argc, char** argv) {
  const u64 n = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 20);
  const double wf = argc > 2 ? atof(argv[2]) : 0.067;
  const int perm = argc > 3 ? atoi(argv[3]) : 0;
  const int NB = 4;  // delta batches cycled, like the bench
  std::mt19937_64 g(42);
  std::vector<u32> hs(n);
  for (u64 i = 0; i < n; i++) hs[i] = (u32)i;
  if (perm) std::shuffle(hs.begin(), hs.end(), g);
  std::vector<u64> h0(n), ht(n * NB), hp(n * NB), hl(n * NB);
  for (u64 i = 0; i < n; i++) h0[i] = (1ull << 40);
  std::uniform_real_distribution<double> U01(0, 1);
  for (int b = 0; b < NB; b++)
    for (u64 i = 0; i < n; i++) {
      // a winner raises ts far above; losers lower -- winners stay ~wf each batch
      ht[b * n + i] = U01(g) < wf ? (1ull << 40) + (u64)(b + 1) * 1000000 + 5 : 1000;
      hp[b * n + i] = g(); hl[b * n + i] = g() & 0xffffff;
    }
  u64 *ts, *pre, *lr, *dts, *dpre, *dlr; u32* slot; Rec *rec, *drec; u64x2* pl;
  CK(hipMalloc(&ts, n * 8)); CK(hipMalloc(&pre, n * 8)); CK(hipMalloc(&lr, n * 8));
  CK(hipMalloc(&rec, n * 32)); CK(hipMalloc(&pl, n * 16)); CK(hipMalloc(&drec, n * 32 * NB));
  CK(hipMalloc(&dts, n * 8 * NB)); CK(hipMalloc(&dpre, n * 8 * NB)); CK(hipMalloc(&dlr, n * 8 * NB));
  CK(hipMalloc(&slot, n * 4));
  CK(hipMemcpy(slot, hs.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dts, ht.data(), n * 8 * NB, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpre, hp.data(), n * 8 * NB, hipMemcpyHostToDevice));
  CK(hipMemcpy(dlr, hl.data(), n * 8 * NB, hipMemcpyHostToDevice));
  std::vector<Rec> hr(n * NB);
  for (int b = 0; b < NB; b++)
    for (u64 i = 0; i < n; i++) hr[b * n + i] = Rec{ht[b * n + i], hp[b * n + i], hl[b * n + i], hs[i]};
  CK(hipMemcpy(drec, hr.data(), n * 32 * NB, hipMemcpyHostToDevice));
  static u64 *s_ts, *s_h0; static Rec* s_rec; static u64 s_n;
  s_ts = ts; s_rec = rec; s_n = n;
  static u64* s_dev0; CK(hipMalloc(&s_dev0, n * 8)); CK(hipMemcpy(s_dev0, h0.data(), n * 8, hipMemcpyHostToDevice));
  static Rec* s_rec0; CK(hipMalloc(&s_rec0, n * 32));
  { std::vector<Rec> r0(n, Rec{1ull << 40, 0, 0, 0}); CK(hipMemcpy(s_rec0, r0.data(), n * 32, hipMemcpyHostToDevice)); }
  (void)s_h0;
  g_reset = []() {
    CK(hipMemcpy(s_ts, s_dev0, s_n * 8, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(s_rec, s_rec0, s_n * 32, hipMemcpyDeviceToDevice));
    CK(hipDeviceSynchronize());
  };
  auto reset = []() { g_reset(); };
  const int reps = 20;
  const double algo = 48.0 * n;  // 48 B per key
  auto rep = [&](const char* name, float ms) {
    printf("%-34s %8.1f us  %6.2f TB/s (48 B/key)\n", name, ms * 1e3, algo / (ms * 1e-3) / 1e12);
  };
  const u64 np = n / 2;
  const unsigned gA = (unsigned)((np + 511) / 512), g4 = (unsigned)((n + 1023) / 1024);
  printf("n=%llu wf=%.3f perm=%d\n", n, wf, perm);
  reset();
  rep("A SoA pairs (round 1)", timeit([&](int r) { int b = r % NB;
    kA<true><<<gA, 256>>>(ts, pre, lr, slot, dts + b * n, dpre + b * n, dlr + b * n, np); }, reps));
  reset();
  rep("A SoA pairs, no writes", timeit([&](int r) { int b = r % NB;
    kA<false><<<gA, 256>>>(ts, pre, lr, slot, dts + b * n, dpre + b * n, dlr + b * n, np); }, reps));
  reset();
  rep("C AoS 32-B state", timeit([&](int r) { int b = r % NB;
    kC<<<g4, 256>>>(rec, slot, dts + b * n, dpre + b * n, dlr + b * n, n); }, reps));
  reset();
  rep("D ts + 16-B rec, lazy delta", timeit([&](int r) { int b = r % NB;
    kD<<<g4, 256>>>(ts, pl, slot, dts + b * n, dpre + b * n, dlr + b * n, n); }, reps));
  reset();
  rep("D2 ts + 16-B rec, eager delta", timeit([&](int r) { int b = r % NB;
    kD2<<<g4, 256>>>(ts, pl, slot, dts + b * n, dpre + b * n, dlr + b * n, n); }, reps));
  reset();
  rep("D3 ts whole-line + 16-B rec", timeit([&](int r) { int b = r % NB;
    kD3<<<g4, 256>>>(ts, pl, slot, dts + b * n, dpre + b * n, dlr + b * n, n); }, reps));
  reset();
  rep("D4 ts + 16-B rec, whole lines", timeit([&](int r) { int b = r % NB;
    kD4<<<g4, 256>>>(ts, pl, slot, dts + b * n, dpre + b * n, dlr + b * n, n); }, reps));
  reset();
  rep("D5 D2 + nontemporal stores", timeit([&](int r) { int b = r % NB;
    kD5<<<g4, 256>>>(ts, pl, slot, dts + b * n, dpre + b * n, dlr + b * n, n); }, reps));
  reset();
  rep("D6<2>", timeit([&](int r) { int b = r % NB;
    kD6<2><<<(unsigned)((n + 511) / 512), 256>>>(ts, pl, slot, dts + b * n, dpre + b * n, dlr + b * n, n); }, reps));
  reset();
  rep("D6<8>", timeit([&](int r) { int b = r % NB;
    kD6<8><<<(unsigned)((n + 2047) / 2048), 256>>>(ts, pl, slot, dts + b * n, dpre + b * n, dlr + b * n, n); }, reps));
  reset();
  rep("C2 ts mirror + 32-B rec", timeit([&](int r) { int b = r % NB;
    kC2<<<g4, 256>>>(ts, rec, slot, dts + b * n, dpre + b * n, dlr + b * n, n); }, reps));
  reset();
  rep("E SoA full rewrite", timeit([&](int r) { int b = r % NB;
    kE<<<g4, 256>>>(ts, pre, lr, slot, dts + b * n, dpre + b * n, dlr + b * n, n); }, reps));
  reset();
  rep("F ts + 16-B rec, AoS delta", timeit([&](int r) { int b = r % NB;
    kF<<<g4, 256>>>(ts, pl, drec + b * n, n); }, reps));
  return 0;
}
