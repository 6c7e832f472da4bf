// mb_stream.hip -- microbenchmark of streaming max-merge variants on gfx950.
// Not part of the product: used to pick the k_block_max shape.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef unsigned long long u64;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

template <int U, bool NTLD_S, bool NTST>
__global__ __launch_bounds__(256) void k_max(u64* __restrict__ s, const u64* __restrict__ d, u64 n) {
  const u64 tile = 256 * 2 * U;
  for (u64 t = blockIdx.x; t * tile < n; t += gridDim.x) {
    u64 base = t * tile + threadIdx.x * 2;
    u64x2 dv[U], sv[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      u64 i = base + u * 512;
      if (i < n) {
        dv[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(d + i));
        if (NTLD_S) sv[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(s + i));
        else sv[u] = *reinterpret_cast<const u64x2*>(s + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      u64 i = base + u * 512;
      if (i < n) {
        u64x2 r;
        r.x = dv[u].x > sv[u].x ? dv[u].x : sv[u].x;
        r.y = dv[u].y > sv[u].y ? dv[u].y : sv[u].y;
        if (NTST) __builtin_nontemporal_store(r, reinterpret_cast<u64x2*>(s + i));
        else *reinterpret_cast<u64x2*>(s + i) = r;
      }
    }
  }
}

// copy reference: 1 read + 1 write
__global__ __launch_bounds__(256) void k_copy(u64* __restrict__ s, const u64* __restrict__ d, u64 n) {
  for (u64 i = ((u64)blockIdx.x * 256 + threadIdx.x) * 2; i < n; i += (u64)gridDim.x * 512)
    *reinterpret_cast<u64x2*>(s + i) = *reinterpret_cast<const u64x2*>(d + i);
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  u64 n = (argc > 1 ? strtoull(argv[1], 0, 10) : (1ull << 31));  // cells
  u64 *s, *d;
  CK(hipMalloc(&s, n * 8)); CK(hipMalloc(&d, n * 8));
  CK(hipMemset(s, 1, n * 8)); CK(hipMemset(d, 2, n * 8));
  const double gb = 24.0 * n / 1e9;
  int grids[] = {1024, 2048, 4096, 8192, 16384, 65536, 0};
  for (int g : grids) {
    u64 G = g ? g : (n + 2047) / 2048;
    float ms = timeit([&] { hipLaunchKernelGGL((k_max<4, false, false>), dim3(G), dim3(256), 0, 0, s, d, n); }, 5);
    printf("max U4 plain      grid %8llu: %.3f ms  %.0f GB/s\n", G, ms, gb / ms * 1e3);
  }
  for (int g : {2048, 8192, 0}) {
    u64 G1 = g ? g : (n + 1023) / 1024, G2 = g ? g : (n + 4095) / 4096;
    float ms = timeit([&] { hipLaunchKernelGGL((k_max<2, false, false>), dim3(G1), dim3(256), 0, 0, s, d, n); }, 5);
    printf("max U2            grid %8llu: %.3f ms  %.0f GB/s\n", G1, ms, gb / ms * 1e3);
    ms = timeit([&] { hipLaunchKernelGGL((k_max<8, false, false>), dim3(G2), dim3(256), 0, 0, s, d, n); }, 5);
    printf("max U8            grid %8llu: %.3f ms  %.0f GB/s\n", G2, ms, gb / ms * 1e3);
    u64 G = g ? g : (n + 2047) / 2048;
    ms = timeit([&] { hipLaunchKernelGGL((k_max<4, true, false>), dim3(G), dim3(256), 0, 0, s, d, n); }, 5);
    printf("max U4 ntld-state grid %8llu: %.3f ms  %.0f GB/s\n", G, ms, gb / ms * 1e3);
    ms = timeit([&] { hipLaunchKernelGGL((k_max<4, false, true>), dim3(G), dim3(256), 0, 0, s, d, n); }, 5);
    printf("max U4 ntst       grid %8llu: %.3f ms  %.0f GB/s\n", G, ms, gb / ms * 1e3);
    ms = timeit([&] { hipLaunchKernelGGL((k_max<4, true, true>), dim3(G), dim3(256), 0, 0, s, d, n); }, 5);
    printf("max U4 nt both    grid %8llu: %.3f ms  %.0f GB/s\n", G, ms, gb / ms * 1e3);
  }
  float ms = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, s, d, n); }, 5);
  printf("copy (16 B/cell)  grid 8192: %.3f ms  %.0f GB/s\n", ms, 16.0 * n / 1e9 / ms * 1e3);
  return 0;
}
