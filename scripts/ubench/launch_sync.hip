// Micro-benchmark: the fixed costs a level-synchronous BFS pays per level.
//  (1) back-to-back no-op kernels by grid size and static LDS
//  (2) tiny kernel + D2H copy + hipStreamSynchronize (the host-driven read-back)
//  (3) tiny kernel writing a flag to host-pinned memory + host spin (no sync call)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_noop(int const* st) { if (st[0]) return; }
__global__ void k_noop_lds(int const* st)
{
  __shared__ int buf[6144];  // 24 KB
  if (st[0]) return;
  buf[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (buf[(threadIdx.x + 1) & 255] == -1) printf("x");
}
__global__ void k_count(unsigned long long* c) { if (threadIdx.x == 0) atomicAdd(c, 1ull); }
__global__ void k_publish(unsigned long long const* c, unsigned long long volatile* host, unsigned long long seq)
{
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    __hip_atomic_store((unsigned long long*)host + 1, *c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store((unsigned long long*)host, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

int main()
{
  hipStream_t s;
  CK(hipStreamCreate(&s));
  int* st;
  CK(hipMalloc(&st, 4));
  CK(hipMemset(st, 1, 4));  // nonzero: the kernels return at once
  unsigned long long* dc;
  CK(hipMalloc(&dc, 64));
  CK(hipMemset(dc, 0, 64));
  unsigned long long* host;
  CK(hipHostMalloc(&host, 64, hipHostMallocDefault));
  host[0] = 0;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto now = [] { return std::chrono::steady_clock::now(); };
  // (1)
  for (int lds = 0; lds < 2; ++lds)
    for (int grid : {1, 64, 256, 1024, 4096}) {
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(lds ? k_noop_lds : k_noop, dim3(grid), dim3(256), 0, s, st);
      CK(hipStreamSynchronize(s));
      int const n = 200;
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < n; ++i) hipLaunchKernelGGL(lds ? k_noop_lds : k_noop, dim3(grid), dim3(256), 0, s, st);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("noop%s grid %5d: %.2f us per kernel (back to back)\n", lds ? "+24KB LDS" : "", grid, 1e3 * ms / n);
    }
  // (2) kernel + D2H + sync round trip
  {
    unsigned long long* hp = host + 4;
    double best = 1e9, tot = 0;
    int const n = 200;
    for (int i = 0; i < n; ++i) {
      auto t0 = now();
      hipLaunchKernelGGL(k_count, dim3(1024), dim3(256), 0, s, dc);
      CK(hipMemcpyAsync(hp, dc, 8, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      double us = std::chrono::duration<double, std::micro>(now() - t0).count();
      tot += us;
      best = us < best ? us : best;
    }
    printf("kernel(1024 blocks) + D2H 8 B + hipStreamSynchronize: mean %.1f us, best %.1f us\n", tot / n, best);
  }
  // (3) kernel + publish to pinned + host spin
  {
    double best = 1e9, tot = 0;
    int const n = 200;
    for (int i = 1; i <= n; ++i) {
      auto t0 = now();
      hipLaunchKernelGGL(k_count, dim3(1024), dim3(256), 0, s, dc);
      hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, s, dc, host, (unsigned long long)i);
      while (__atomic_load_n(&host[0], __ATOMIC_ACQUIRE) != (unsigned long long)i) {
      }
      double us = std::chrono::duration<double, std::micro>(now() - t0).count();
      tot += us;
      best = us < best ? us : best;
    }
    CK(hipStreamSynchronize(s));
    printf("kernel(1024 blocks) + publish kernel + host spin: mean %.1f us, best %.1f us\n", tot / n, best);
  }
  // (4) empty-queue round trip: sync on an idle stream
  {
    double tot = 0;
    int const n = 200;
    for (int i = 0; i < n; ++i) {
      auto t0 = now();
      hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, s, st);
      CK(hipStreamSynchronize(s));
      tot += std::chrono::duration<double, std::micro>(now() - t0).count();
    }
    printf("tiny kernel + hipStreamSynchronize: mean %.1f us\n", tot / n);
  }
  return 0;
}
