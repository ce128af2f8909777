// Measured HBM ceiling for the roofline lines of bench.py ("also
// report a measured stream-copy ceiling").  A 16-byte-per-lane copy, the access
// shape MI355X_MICROARCH.md quotes its 6.29 TB/s float4 copy for, nontemporal on
// both sides so the copy does not fill the caches it is measuring past.  Timed with HIP events on
// the handle's stream; bytes = read + write.
#include "capi.hpp"

#include <cugraph_amd/ext.h>

namespace cgx {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // 16 B per lane, a native vector type

constexpr int kCopyBlock  = 256;
constexpr int kCopyUnroll = 4;

__global__ __launch_bounds__(kCopyBlock) void k_copy16(u32x4 const* __restrict__ src, u32x4* __restrict__ dst,
                                                       int64_t n)
{
  int64_t const stride = (int64_t)gridDim.x * kCopyBlock;
  int64_t i            = blockIdx.x * (int64_t)kCopyBlock + threadIdx.x;
  for (; i + (kCopyUnroll - 1) * stride < n; i += kCopyUnroll * stride) {
    u32x4 v[kCopyUnroll];
#pragma unroll
    for (int j = 0; j < kCopyUnroll; ++j) v[j] = __builtin_nontemporal_load(src + i + j * stride);
#pragma unroll
    for (int j = 0; j < kCopyUnroll; ++j) __builtin_nontemporal_store(v[j], dst + i + j * stride);
  }
  for (; i < n; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

}  // namespace
}  // namespace cgx

extern "C" double cugraph_amd_measure_copy_bandwidth(const cugraph_resource_handle_t* handle, size_t bytes,
                                                     int reps)
{
  using namespace cgx;
  try {
    auto* h          = reinterpret_cast<handle_t*>(const_cast<cugraph_resource_handle_t*>(handle));
    hipStream_t s    = h->stream;
    int64_t const n  = (int64_t)(bytes / sizeof(u32x4));
    if (n <= 0 || reps <= 0) return 0.0;
    buffer a(n * sizeof(u32x4), s), b(n * sizeof(u32x4), s);
    HIP_CHECK(hipMemsetAsync(a.data(), 0, n * sizeof(u32x4), s));
    // one-shot grid (about one 16-B vector per lane, the tail of the unrolled loop
    // takes it): scripts/ubench/mem_calib.hip measured 6.27 TB/s this way against
    // 5.3-5.4 TB/s for persistent 2048-8192-block grids
    int const grid = (int)std::min<int64_t>((n + kCopyBlock - 1) / kCopyBlock, 1 << 20);
    hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(kCopyBlock), 0, s, a.data<u32x4>(), b.data<u32x4>(), n);
    CGX_LAUNCH_CHECK();
    hipEvent_t e0 = h->event(0), e1 = h->event(1);
    HIP_CHECK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(kCopyBlock), 0, s, (r & 1) ? b.data<u32x4>() : a.data<u32x4>(),
                         (r & 1) ? a.data<u32x4>() : b.data<u32x4>(), n);
    CGX_LAUNCH_CHECK();
    HIP_CHECK(hipEventRecord(e1, s));
    HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms > 0 ? 2.0 * (double)n * sizeof(u32x4) * reps / (ms * 1e-3) / 1e9 : 0.0;
  } catch (...) {
    return -1.0;
  }
}
