// mb_fetch.hip -- calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950
// for the load and store widths the engine's kernels use (4, 8 and 16 B per
// lane, coalesced).  Not part of the product: MI355X_MICROARCH.md establishes
// FETCH_SIZE = 1/2 of the bytes only for 16-B-per-lane streams; this tells
// which factor applies to the narrower loads of k_treg_lww / k_tlog_* / k_uj_*.
// Each kernel reads (or writes) exactly `bytes` once; the PMC run divides the
// counters by these byte counts (printed).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
typedef unsigned int u32;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("%s: %s\n", #x, hipGetErrorString(e));                    \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

template <typename T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ a, u64 n, u64* __restrict__ out) {
  u64 acc = 0;
  for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) {
    const T v = a[i];
    acc += reinterpret_cast<const u64*>(&v)[0] + (sizeof(T) > 8 ? reinterpret_cast<const u64*>(&v)[1] : 0);
  }
  if (acc == 0x12345) out[blockIdx.x] = acc;  // never true for the zero-filled input: no stores
}

template <typename T>
__global__ __launch_bounds__(256) void k_write(T* __restrict__ a, u64 n) {
  for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) a[i] = T{};
}

int main() {
  const u64 bytes = 1ull << 30;  // well past the 256 MiB Infinity Cache
  void* buf;
  u64* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(buf, 0, bytes));
  const dim3 grid(4096), blk(256);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_read<u32>, grid, blk, 0, 0, (const u32*)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_read<u64>, grid, blk, 0, 0, (const u64*)buf, bytes / 8, out);
    hipLaunchKernelGGL(k_read<u64x2>, grid, blk, 0, 0, (const u64x2*)buf, bytes / 16, out);
    hipLaunchKernelGGL(k_write<u32>, grid, blk, 0, 0, (u32*)buf, bytes / 4);
    hipLaunchKernelGGL(k_write<u64>, grid, blk, 0, 0, (u64*)buf, bytes / 8);
    hipLaunchKernelGGL(k_write<u64x2>, grid, blk, 0, 0, (u64x2*)buf, bytes / 16);
  }
  CK(hipDeviceSynchronize());
  printf("{\"bytes_per_launch\": %llu}\n", bytes);
  return 0;
}
