// mb_ticket.hip -- microbenchmark: the cost of one same-address ticket
// atomic per workgroup (jy_scan.hpp ticket) against the same empty launch
// without it, and against one atomic per workgroup on a per-XCD-spread
// counter.  Prints us per launch for several grid sizes.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_empty(unsigned* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0xFFFFFFFFu) out[0] = 1;
}
__global__ __launch_bounds__(256) void k_ticket(unsigned* ctr, unsigned* out) {
  __shared__ unsigned t;
  if (threadIdx.x == 0) t = atomicAdd(ctr, 1u);
  __syncthreads();
  if (threadIdx.x == 0 && t == 0xFFFFFFFFu) out[0] = t;
}
__global__ __launch_bounds__(256) void k_spread(unsigned* ctr, unsigned* out) {
  __shared__ unsigned t;
  if (threadIdx.x == 0) t = atomicAdd(ctr + (blockIdx.x & 63) * 64, 1u);
  __syncthreads();
  if (threadIdx.x == 0 && t == 0xFFFFFFFFu) out[0] = t;
}

int main() {
  unsigned *ctr, *out;
  hipMalloc(&ctr, 64 * 64 * 4);
  hipMalloc(&out, 64);
  hipMemset(ctr, 0, 64 * 64 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (unsigned g : {1024u, 4096u, 8192u, 32768u, 131072u}) {
    float ms[3];
    for (int k = 0; k < 3; k++) {
      for (int w = 0; w < 3; w++) {
        if (k == 0) k_empty<<<g, 256>>>(out);
        if (k == 1) k_ticket<<<g, 256>>>(ctr, out);
        if (k == 2) k_spread<<<g, 256>>>(ctr, out);
      }
      hipEventRecord(a);
      for (int r = 0; r < 10; r++) {
        if (k == 0) k_empty<<<g, 256>>>(out);
        if (k == 1) k_ticket<<<g, 256>>>(ctr, out);
        if (k == 2) k_spread<<<g, 256>>>(ctr, out);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms[k], a, b);
    }
    printf("grid %6u: empty %7.1f us  ticket %7.1f us  spread %7.1f us\n", g, ms[0] * 100, ms[1] * 100, ms[2] * 100);
  }
  return 0;
}
