// Measurement tool (not product): the PageRank schedule build's keys-only sort of the
// window bits (build_push_packed_sym_cm, csrc/pagerank.hip) with rocprim's onesweep at
// 8 radix bits per pass (the gfx950 default: two passes for RMAT-24's 10 window bits)
// against 10 and 11 bits per pass (one pass), plus a plain 8-B copy of the same keys as
// the floor.  Keys: window (vbits) << 38 | a source-ordered low part, ne of them.
// usage: radix_bits <ne_millions> <vbits>; prints ms per sort (median of 5) per config.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/ubench/radix_bits scripts/ubench/radix_bits.hip
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

__global__ void k_gen(uint64_t* k, int64_t n, int vbits)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    z ^= z >> 29;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 32;
    uint64_t const w = z & ((1ull << vbits) - 1);
    k[i]             = (w << 38) | (uint64_t)i;
  }
}
__global__ void k_copy(uint64_t const* a, uint64_t* b, int64_t n)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) b[i] = a[i];
}

template <unsigned Bits, unsigned BS, unsigned IPT>
using cfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>, rocprim::kernel_config<BS, IPT>, Bits,
                                        rocprim::block_radix_rank_algorithm::match>>;

template <typename C>
float run(char const* name, uint64_t* a, uint64_t* b, uint64_t* src, int64_t n, int vbits)
{
  std::vector<float> t;
  size_t tmp = 0;
  rocprim::double_buffer<uint64_t> db0(a, b);
  CK(rocprim::radix_sort_keys<C>(nullptr, tmp, db0, (size_t)n, 38, 38 + vbits, 0));
  void* tb;
  CK(hipMalloc(&tb, tmp));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < 6; ++r) {
    k_copy<<<8192, 256>>>(src, a, n);
    rocprim::double_buffer<uint64_t> db(a, b);
    CK(hipEventRecord(e0, 0));
    CK(rocprim::radix_sort_keys<C>(tb, tmp, db, (size_t)n, 38, 38 + vbits, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r) t.push_back(ms);
    // check: windows nondecreasing, stable (low parts increasing within a window)
    if (r == 5) {
      std::vector<uint64_t> h(n);
      CK(hipMemcpy(h.data(), db.current(), n * 8, hipMemcpyDeviceToHost));
      for (int64_t i = 1; i < n; ++i)
        if (h[i] < h[i - 1]) {
          std::printf("%s: NOT SORTED at %lld\n", name, (long long)i);
          break;
        }
    }
  }
  CK(hipFree(tb));
  std::sort(t.begin(), t.end());
  std::printf("%-24s ne=%lld vbits=%d ms=%.3f\n", name, (long long)n, vbits, t[t.size() / 2]);
  return t[t.size() / 2];
}

int main(int argc, char** argv)
{
  int64_t const n = (int64_t)(argc > 1 ? std::atof(argv[1]) : 500.0) * 1000000;
  int const vbits = argc > 2 ? std::atoi(argv[2]) : 10;
  uint64_t *a, *b, *src;
  CK(hipMalloc(&a, n * 8));
  CK(hipMalloc(&b, n * 8));
  CK(hipMalloc(&src, n * 8));
  k_gen<<<8192, 256>>>(src, n, vbits);
  CK(hipDeviceSynchronize());
  {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < 6; ++r) {
      CK(hipEventRecord(e0, 0));
      k_copy<<<8192, 256>>>(src, a, n);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    std::printf("%-24s ne=%lld ms=%.3f\n", "copy", (long long)n, t[3]);
  }
  run<rocprim::default_config>("default", a, b, src, n, vbits);
  run<cfg<8, 256, 12>>("bits8 256x12", a, b, src, n, vbits);
  run<cfg<10, 256, 12>>("bits10 256x12", a, b, src, n, vbits);
  run<cfg<10, 512, 12>>("bits10 512x12", a, b, src, n, vbits);
  run<cfg<10, 1024, 8>>("bits10 1024x8", a, b, src, n, vbits);
  return 0;
}
