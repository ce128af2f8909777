// Micro-benchmark (measurement tool, not product): how fast can MI355X stream a CSC
// index array and gather fp32 values through it?  Variants:
//   mode 0: stream indices only (sum of ids)
//   mode 1: gather x[idx[e]], 8 independent gathers per thread per round
//   mode 2: as 1 with non-temporal index loads
//   mode 3: as 2, ids < H served from an LDS copy of x[0:H) (persistent blocks)
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC scripts/ubench_gather.hip -o scripts/libubench.so
#include <hip/hip_runtime.h>
#include <cstdint>

template <int MODE>
__global__ __launch_bounds__(256) void k_gather(const int* __restrict__ idx, long n, const float* __restrict__ x,
                                                int H, float* out)
{
  extern __shared__ float hub[];
  if (MODE == 3) {
    for (int i = threadIdx.x; i < H; i += 256) hub[i] = x[i];
    __syncthreads();
  }
  float acc = 0;
  long stride = (long)gridDim.x * 256 * 8;
  for (long b = (long)blockIdx.x * 256 * 8; b < n; b += stride) {
    int u[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      long e = b + j * 256 + threadIdx.x;
      if (MODE >= 2) u[j] = e < n ? __builtin_nontemporal_load(idx + e) : 0;
      else u[j] = e < n ? idx[e] : 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (MODE == 0) acc += (float)u[j];
      else if (MODE == 3) acc += u[j] < H ? hub[u[j]] : x[u[j]];
      else acc += x[u[j]];
    }
  }
  if (acc == 12345.678f) out[0] = acc;  // keep live
}

extern "C" float ubench_gather(const int* idx, long n, const float* x, int mode, int H, int blocks, int reps)
{
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float* out;
  hipMalloc(&out, 4);
  size_t lds = mode == 3 ? (size_t)H * 4 : 0;
  auto launch = [&]() {
    switch (mode) {
      case 0: hipLaunchKernelGGL(k_gather<0>, dim3(blocks), dim3(256), 0, 0, idx, n, x, H, out); break;
      case 1: hipLaunchKernelGGL(k_gather<1>, dim3(blocks), dim3(256), 0, 0, idx, n, x, H, out); break;
      case 2: hipLaunchKernelGGL(k_gather<2>, dim3(blocks), dim3(256), 0, 0, idx, n, x, H, out); break;
      default: hipLaunchKernelGGL(k_gather<3>, dim3(blocks), dim3(256), lds, 0, idx, n, x, H, out); break;
    }
  };
  launch();
  hipDeviceSynchronize();
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipFree(out);
  return ms / reps;
}
