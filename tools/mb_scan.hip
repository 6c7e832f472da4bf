// mb_scan.hip -- microbenchmark of the single-pass look-back scan
// (jy_scan.hpp): tickets + look-back over T tiles of 1024 items, against
// tickets alone, to see what a look-back scan costs per launch on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../jylis_amd/csrc/jy_scan.hpp"
using namespace jyscan;
constexpr int kT = 256;

template <int kMode>  // 0 tickets only, 1 tickets + look-back
__global__ __launch_bounds__(kT) void k_scan(const u32* in, u32* out, u64 n, u32* tick, u64* status, u32 epoch) {
  __shared__ u64 red[kT / 64];
  __shared__ u64 pre;
  __shared__ u32 tk;
  const u64 tiles = (n + 1023) / 1024;
  for (;;) {
    const u32 t = ticket(tick, &tk);
    if (t >= tiles) return;
    u64 v[4], s = 0;
    for (int u = 0; u < 4; u++) {
      const u64 i = (u64)t * 1024 + threadIdx.x * 4 + u;
      v[u] = s;
      s += i < n ? in[i] : 0;
    }
    u64 tot;
    const u64 off = block_excl<kT, u64>(s, red, tot);
    u64 p = 0;
    if (kMode == 1) p = lookback(status, t, epoch, tot, &pre);
    for (int u = 0; u < 4; u++) {
      const u64 i = (u64)t * 1024 + threadIdx.x * 4 + u;
      if (i < n) out[i] = (u32)(p + off + v[u]);
    }
  }
}

int main() {
  for (u64 n : {700ull * 1024, 3000ull * 1024, 100000ull * 1024}) {
    u32 *in, *out, *tick;
    u64* st;
    hipMalloc(&in, n * 4);
    hipMalloc(&out, n * 4);
    hipMalloc(&tick, 64);
    const u64 tiles = (n + 1023) / 1024;
    hipMalloc(&st, tiles * 8);
    hipMemset(st, 0, tiles * 8);
    std::vector<u32> h(n, 1);
    hipMemcpy(in, h.data(), n * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 2; mode++)
      for (u32 grid : {1024u, (u32)tiles}) {
        float best = 1e9;
        for (int rep = 0; rep < 5; rep++) {
          hipMemset(tick, 0, 64);
          hipEventRecord(a);
          if (mode == 0) hipLaunchKernelGGL(k_scan<0>, dim3(grid), dim3(kT), 0, 0, in, out, n, tick, st, 100 + rep);
          else hipLaunchKernelGGL(k_scan<1>, dim3(grid), dim3(kT), 0, 0, in, out, n, tick, st, 100 + rep);
          hipEventRecord(b);
          hipEventSynchronize(b);
          float ms;
          hipEventElapsedTime(&ms, a, b);
          best = ms < best ? ms : best;
        }
        u32 last;
        hipMemcpy(&last, out + n - 1, 4, hipMemcpyDeviceToHost);
        printf("n=%llu tiles=%llu grid=%u mode=%d: %.1f us  last=%u (want %llu)\n", (unsigned long long)n,
               (unsigned long long)tiles, grid, mode, best * 1e3, last, (unsigned long long)(n - 1));
      }
    hipFree(in);
    hipFree(out);
    hipFree(tick);
    hipFree(st);
  }
}
