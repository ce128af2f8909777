// Small device primitives (fill, iota, gather/scatter, reductions, radix sort and
// scan wrappers over rocPRIM).  Header-only templates: every .hip that needs them
// instantiates its own.
#pragma once

#include "common.hpp"

#include <cstring>
#include <climits>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include <vector>

namespace cgx {

constexpr int kBlock = 256;

// ---------------------------------------------------------------- elementwise
template <typename T>
__global__ void k_fill(T* p, size_t n, T v)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}
template <typename T>
void fill(T* p, size_t n, T v, hipStream_t s)
{
  if (!n) return;
  hipLaunchKernelGGL(k_fill<T>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, p, n, v);
  CGX_LAUNCH_CHECK();
}

template <typename T>
__global__ void k_iota(T* p, size_t n, T first)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = first + static_cast<T>(i);
}
template <typename T>
void iota(T* p, size_t n, T first, hipStream_t s)
{
  if (!n) return;
  hipLaunchKernelGGL(k_iota<T>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, p, n, first);
  CGX_LAUNCH_CHECK();
}

template <typename TO, typename TI>
__global__ void k_convert(TO* o, TI const* in, size_t n)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    o[i] = static_cast<TO>(in[i]);
}
template <typename TO, typename TI>
void convert(TO* o, TI const* in, size_t n, hipStream_t s)
{
  if (!n) return;
  hipLaunchKernelGGL((k_convert<TO, TI>), dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, o, in, n);
  CGX_LAUNCH_CHECK();
}

// out[i] = table[idx[i]]
template <typename T, typename I>
__global__ void k_gather(T* out, T const* table, I const* idx, size_t n)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = table[idx[i]];
}
template <typename T, typename I>
void gather(T* out, T const* table, I const* idx, size_t n, hipStream_t s)
{
  if (!n) return;
  hipLaunchKernelGGL((k_gather<T, I>), dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, out, table, idx, n);
  CGX_LAUNCH_CHECK();
}

// out[idx[i]] = val[i]
template <typename T, typename I>
__global__ void k_scatter(T* out, T const* val, I const* idx, size_t n)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[idx[i]] = val[i];
}
template <typename T, typename I>
void scatter(T* out, T const* val, I const* idx, size_t n, hipStream_t s)
{
  if (!n) return;
  hipLaunchKernelGGL((k_scatter<T, I>), dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, out, val, idx, n);
  CGX_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- wave/block reductions
__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ long long wave_sum_ll(long long v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over a 256-thread block; result valid in thread 0.  Uses `sm` (>= 4 doubles).
__device__ __forceinline__ double block_sum_256(double v, double* sm)
{
  v = wave_sum(v);
  int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sm[wid] = v;
  __syncthreads();
  double r = 0;
  if (threadIdx.x == 0) r = sm[0] + sm[1] + sm[2] + sm[3];
  return r;
}

// Deterministic two-stage sum of f(i) over [0, n) in double: per-block partials in
// a fixed order, then a single-block pass.  Result left in *out (device).
template <typename F>
__global__ void k_sum_partials(F f, size_t n, double* partials)
{
  __shared__ double sm[4];
  double acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += f(i);
  double r = block_sum_256(acc, sm);
  if (threadIdx.x == 0) partials[blockIdx.x] = r;
}
static __global__ void k_sum_final(double const* partials, int np, double* out)
{
  __shared__ double sm[4];
  double acc = 0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) acc += partials[i];
  double r = block_sum_256(acc, sm);
  if (threadIdx.x == 0) *out = r;
}
template <typename F>
void device_sum(F f, size_t n, double* out_dev, double* scratch /* >= 1024 doubles */, hipStream_t s)
{
  unsigned g = grid_for(n, kBlock, 1024);
  hipLaunchKernelGGL((k_sum_partials<F>), dim3(g), dim3(kBlock), 0, s, f, n, scratch);
  CGX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sum_final, dim3(1), dim3(kBlock), 0, s, scratch, (int)g, out_dev);
  CGX_LAUNCH_CHECK();
}

// host-side synchronous helpers
template <typename T>
T to_host_scalar(T const* dev, hipStream_t s)
{
  T h{};
  HIP_CHECK(hipMemcpyAsync(&h, dev, sizeof(T), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return h;
}
template <typename T>
std::vector<T> to_host(T const* dev, size_t n, hipStream_t s)
{
  std::vector<T> h(n);
  if (n) {
    HIP_CHECK(hipMemcpyAsync(h.data(), dev, n * sizeof(T), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }
  return h;
}
template <typename T>
void to_device(T* dev, T const* host, size_t n, hipStream_t s)
{
  if (n) HIP_CHECK(hipMemcpyAsync(dev, host, n * sizeof(T), hipMemcpyHostToDevice, s));
}

template <typename T>
__global__ void k_minmax(T const* a, size_t n, long long* mn, long long* mx)
{
  __shared__ long long smn[4], smx[4];
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    long long v = (long long)a[i];
    lo = v < lo ? v : lo;
    hi = v > hi ? v : hi;
  }
  for (int o = 32; o > 0; o >>= 1) {
    long long l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
    lo = l2 < lo ? l2 : lo;
    hi = h2 > hi ? h2 : hi;
  }
  int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { smn[wid] = lo; smx[wid] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      lo = smn[w] < lo ? smn[w] : lo;
      hi = smx[w] > hi ? smx[w] : hi;
    }
    lo = smn[0] < lo ? smn[0] : lo;
    hi = smx[0] > hi ? smx[0] : hi;
    atomicMin(mn, lo);
    atomicMax(mx, hi);
  }
}
// min and max of an integer array (n may be 0 -> (LLONG_MAX, LLONG_MIN))
template <typename T>
std::pair<long long, long long> minmax(T const* a, size_t n, hipStream_t s)
{
  dbuf<long long> r(2, s);
  long long init[2] = {LLONG_MAX, LLONG_MIN};
  to_device(r.data(), init, 2, s);
  if (n) {
    hipLaunchKernelGGL(k_minmax<T>, dim3(grid_for(n, kBlock, 2048)), dim3(kBlock), 0, s, a, n, r.data(),
                       r.data() + 1);
    CGX_LAUNCH_CHECK();
  }
  auto h = to_host(r.data(), 2, s);
  return {h[0], h[1]};
}

// ---------------------------------------------------------------- rocPRIM wrappers
template <typename K, typename Vv>
void radix_sort_pairs(K const* kin, K* kout, Vv const* vin, Vv* vout, size_t n, int begin_bit, int end_bit,
                      hipStream_t s, bool descending = false)
{
  if (!n) return;
  size_t tmp = 0;
  if (descending) {
    HIP_CHECK(rocprim::radix_sort_pairs_desc(nullptr, tmp, kin, kout, vin, vout, n, begin_bit, end_bit, s));
  } else {
    HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tmp, kin, kout, vin, vout, n, begin_bit, end_bit, s));
  }
  buffer t(tmp, s);
  if (descending) {
    HIP_CHECK(rocprim::radix_sort_pairs_desc(t.data(), tmp, kin, kout, vin, vout, n, begin_bit, end_bit, s));
  } else {
    HIP_CHECK(rocprim::radix_sort_pairs(t.data(), tmp, kin, kout, vin, vout, n, begin_bit, end_bit, s));
  }
}

// The same sort over two caller buffers per array (rocprim::double_buffer): no
// temporary copy of the keys and values, which the form above allocates inside
// rocPRIM (16 B per u64 key + fp64 value: 33.6 GB for RMAT-26's level-0 pairs).
// Both buffers of each array are overwritten; returns true when the sorted data
// ended in k1 / v1, false when in k0 / v0.
template <typename K, typename Vv>
bool radix_sort_pairs_db(K* k0, K* k1, Vv* v0, Vv* v1, size_t n, int begin_bit, int end_bit, hipStream_t s)
{
  if (!n) return false;
  rocprim::double_buffer<K> kb(k0, k1);
  rocprim::double_buffer<Vv> vb(v0, v1);
  size_t tmp = 0;
  HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tmp, kb, vb, n, begin_bit, end_bit, s));
  buffer t(tmp, s);
  HIP_CHECK(rocprim::radix_sort_pairs(t.data(), tmp, kb, vb, n, begin_bit, end_bit, s));
  return kb.current() == k1;
}

template <typename K>
void radix_sort_keys(K const* kin, K* kout, size_t n, int begin_bit, int end_bit, hipStream_t s)
{
  if (!n) return;
  size_t tmp = 0;
  HIP_CHECK(rocprim::radix_sort_keys(nullptr, tmp, kin, kout, n, begin_bit, end_bit, s));
  buffer t(tmp, s);
  HIP_CHECK(rocprim::radix_sort_keys(t.data(), tmp, kin, kout, n, begin_bit, end_bit, s));
}

// exclusive prefix sum of n elements (pass n+1 with a trailing 0 to get the total)
template <typename TI, typename TO>
void exclusive_scan(TI const* in, TO* out, size_t n, hipStream_t s)
{
  if (!n) return;
  size_t tmp = 0;
  HIP_CHECK(rocprim::exclusive_scan(nullptr, tmp, in, out, TO(0), n, rocprim::plus<TO>(), s));
  buffer t(tmp, s);
  HIP_CHECK(rocprim::exclusive_scan(t.data(), tmp, in, out, TO(0), n, rocprim::plus<TO>(), s));
}

// number of bits needed to represent values in [0, x]
inline int bits_for(unsigned long long x)
{
  int b = 0;
  while (b < 64 && (x >> b) != 0) ++b;
  return b == 0 ? 1 : b;
}

}  // namespace cgx
