// Benchmark-input generation and cugraph.Graph edge-list preprocessing on the GPU.
//
// * R-MAT: counter-based Graph500 generator, bit-identical twin of oracle/rmat.py
//   (role of the reference cpp/src/generators/generate_rmat_edgelist.cu:36-103 +
//   scramble.cuh, whose RAFT RNG is not available to us).  One thread per edge,
//   `scale` splitmix64 draws, no state.
// * symmetrize + dedup keeping the minimum weight
//   (python/cugraph/cugraph/structure/symmetrize.py:78-93, done with cudf groupby in
//   the reference): one 64-bit (src << b | dst) radix sort, run-head flags, scan, scatter.
#include "capi.hpp"
#include "prims.hpp"

#include <cugraph_amd/ext.h>

namespace cgx {
namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z          = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z          = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t scramble(uint64_t v, int scale, uint64_t seed)
{
  if (scale == 0) return v;
  uint64_t mask = (scale >= 64) ? ~0ull : ((1ull << scale) - 1);
  int h         = (scale + 1) / 2;
  v             = (v * 0x9E3779B1ull + seed) & mask;
  v ^= v >> h;
  v = (v * 0x85EBCA77ull) & mask;
  v ^= v >> h;
  return v;
}

template <typename V>
__global__ void k_rmat(V* src, V* dst, size_t n, int scale, double a, double ab, double abc, uint64_t seed,
                       bool clip_and_flip, bool scramble_ids, uint64_t first)
{
  uint64_t const sg = seed * 0x9E3779B97F4A7C15ull;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t e = first + i;
    uint64_t s = 0, d = 0;
    for (int l = 0; l < scale; ++l) {
      uint64_t z = splitmix64(sg ^ (e * 64ull + (uint64_t)l));
      double r   = (double)(z >> 11) * (1.0 / 9007199254740992.0);
      uint64_t sb = r >= ab ? 1ull : 0ull;
      uint64_t db = ((r >= a && r < ab) || r >= abc) ? 1ull : 0ull;
      s |= sb << (scale - 1 - l);
      d |= db << (scale - 1 - l);
    }
    if (clip_and_flip && s < d) {
      uint64_t t = s;
      s          = d;
      d          = t;
    }
    if (scramble_ids) {
      s = scramble(s, scale, seed);
      d = scramble(d, scale, seed);
    }
    src[i] = (V)s;
    dst[i] = (V)d;
  }
}

template <typename W>
__global__ void k_weights(W* w, size_t n, uint64_t seed, uint64_t first)
{
  uint64_t const sg = seed * 0x9E3779B97F4A7C15ull;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = splitmix64(sg ^ (first + i));
    w[i]       = (W)(float)((double)(z >> 40) * (1.0 / 16777216.0));
  }
}

template <typename V>
__global__ void k_keys(V const* s, V const* d, size_t n, int b, bool sym, uint64_t* key)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    key[i] = ((uint64_t)s[i] << b) | (uint64_t)d[i];
    if (sym) key[n + i] = ((uint64_t)d[i] << b) | (uint64_t)s[i];
  }
}

__global__ void k_run_heads(uint64_t const* key, size_t n, int* flag)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    flag[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}

template <typename V, typename W>
__global__ void k_emit(uint64_t const* key, W const* w, int const* flag, int64_t const* pos, size_t n, int b,
                       V* so, V* dout, W* wo)
{
  uint64_t mask = (1ull << b) - 1;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (!flag[i]) continue;
    int64_t p = pos[i];
    so[p]     = (V)(key[i] >> b);
    dout[p]   = (V)(key[i] & mask);
    if (w) {
      W m = w[i];
      for (size_t j = i + 1; j < n && key[j] == key[i]; ++j) m = w[j] < m ? w[j] : m;
      wo[p] = m;
    }
  }
}

template <typename V, typename W>
void sym_dedup(handle_t& h, array_view_t const& src, array_view_t const& dst, array_view_t const* wv, bool sym,
               std::unique_ptr<device_array_t>& so, std::unique_ptr<device_array_t>& dout,
               std::unique_ptr<device_array_t>& wo)
{
  hipStream_t s = h.stream;
  size_t n      = src.size;
  size_t m      = sym ? 2 * n : n;
  auto [mn1, mx1] = minmax<V>(src.as<V>(), n, s);
  auto [mn2, mx2] = minmax<V>(dst.as<V>(), n, s);
  CGX_INPUT(n == 0 || std::min(mn1, mn2) >= 0, "Invalid input arguments: negative vertex id.");
  long long mx = std::max<long long>(std::max(mx1, mx2), 0);
  int b        = bits_for((unsigned long long)mx);
  CGX_EXPECTS(2 * b <= 64, CUGRAPH_NOT_IMPLEMENTED, "vertex ids >= 2^32 are not supported by symmetrize_dedup");
  dbuf<uint64_t> key(m, s), key_sorted(m, s);
  if (n) {
    hipLaunchKernelGGL(k_keys<V>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, src.as<V>(), dst.as<V>(), n, b,
                       sym, key.data());
    CGX_LAUNCH_CHECK();
  }
  dbuf<W> w_in, w_sorted;
  if (wv) {
    w_in.resize(m, s);
    w_sorted.resize(m, s);
    if (n) {
      HIP_CHECK(hipMemcpyAsync(w_in.data(), wv->data, n * sizeof(W), hipMemcpyDefault, s));
      if (sym) HIP_CHECK(hipMemcpyAsync(w_in.data() + n, wv->data, n * sizeof(W), hipMemcpyDefault, s));
    }
    radix_sort_pairs<uint64_t, W>(key.data(), key_sorted.data(), w_in.data(), w_sorted.data(), m, 0, 2 * b, s);
  } else {
    radix_sort_keys<uint64_t>(key.data(), key_sorted.data(), m, 0, 2 * b, s);
  }
  key.b.release();
  w_in.b.release();
  dbuf<int> flag(m + 1, s);
  dbuf<int64_t> pos(m + 1, s);
  fill<int>(flag.data() + m, 1, 0, s);
  if (m) {
    hipLaunchKernelGGL(k_run_heads, dim3(grid_for(m, kBlock, 8192)), dim3(kBlock), 0, s, key_sorted.data(), m,
                       flag.data());
    CGX_LAUNCH_CHECK();
  }
  exclusive_scan<int, int64_t>(flag.data(), pos.data(), m + 1, s);
  int64_t nu = to_host_scalar(pos.data() + m, s);
  so         = std::make_unique<device_array_t>((size_t)nu, dtype_of<V>(), s);
  dout       = std::make_unique<device_array_t>((size_t)nu, dtype_of<V>(), s);
  if (wv) wo = std::make_unique<device_array_t>((size_t)nu, dtype_of<W>(), s);
  if (m) {
    hipLaunchKernelGGL((k_emit<V, W>), dim3(grid_for(m, kBlock, 8192)), dim3(kBlock), 0, s, key_sorted.data(),
                       wv ? w_sorted.data() : nullptr, flag.data(), pos.data(), m, b, so->buf.data<V>(),
                       dout->buf.data<V>(), wv ? wo->buf.data<W>() : nullptr);
    CGX_LAUNCH_CHECK();
  }
  HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace
}  // namespace cgx

using namespace cgx;

extern "C" cugraph_error_code_t cugraph_amd_generate_rmat_edgelist(const cugraph_resource_handle_t* handle,
                                                                  size_t scale,
                                                                  size_t num_edges,
                                                                  double a,
                                                                  double b,
                                                                  double c,
                                                                  uint64_t seed,
                                                                  bool_t clip_and_flip,
                                                                  bool_t scramble_vertex_ids,
                                                                  size_t first_edge,
                                                                  data_type_id_t vertex_dtype,
                                                                  cugraph_type_erased_device_array_t** src,
                                                                  cugraph_type_erased_device_array_t** dst,
                                                                  cugraph_error_t** error)
{
  *src   = nullptr;
  *dst   = nullptr;
  *error = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    CGX_INPUT(scale < 63, "Invalid input argument: scale too large");
    CGX_INPUT(vertex_dtype == INT32 || vertex_dtype == INT64, "vertex dtype must be INT32 or INT64");
    CGX_INPUT(vertex_dtype == INT64 || scale <= 31, "scale > 31 needs INT64 vertices");
    CGX_INPUT(a >= 0 && b >= 0 && c >= 0 && a + b + c <= 1.0, "Invalid input argument: a, b, c");
    hipStream_t s = H(handle)->stream;
    auto* ps      = new device_array_t(num_edges, vertex_dtype, s);
    auto* pd      = new device_array_t(num_edges, vertex_dtype, s);
    double ab = a + b, abc = a + b + c;
    if (num_edges) {
      if (vertex_dtype == INT32)
        hipLaunchKernelGGL(k_rmat<int32_t>, dim3(grid_for(num_edges, kBlock, 16384)), dim3(kBlock), 0, s,
                           ps->buf.data<int32_t>(), pd->buf.data<int32_t>(), num_edges, (int)scale, a, ab, abc, seed,
                           clip_and_flip == TRUE, scramble_vertex_ids == TRUE, (uint64_t)first_edge);
      else
        hipLaunchKernelGGL(k_rmat<int64_t>, dim3(grid_for(num_edges, kBlock, 16384)), dim3(kBlock), 0, s,
                           ps->buf.data<int64_t>(), pd->buf.data<int64_t>(), num_edges, (int)scale, a, ab, abc, seed,
                           clip_and_flip == TRUE, scramble_vertex_ids == TRUE, (uint64_t)first_edge);
      CGX_LAUNCH_CHECK();
    }
    HIP_CHECK(hipStreamSynchronize(s));
    *src = reinterpret_cast<cugraph_type_erased_device_array_t*>(ps);
    *dst = reinterpret_cast<cugraph_type_erased_device_array_t*>(pd);
  });
}

extern "C" cugraph_error_code_t cugraph_amd_generate_edge_weights(const cugraph_resource_handle_t* handle,
                                                                 size_t num_edges,
                                                                 uint64_t seed,
                                                                 size_t first_edge,
                                                                 data_type_id_t weight_dtype,
                                                                 cugraph_type_erased_device_array_t** weights,
                                                                 cugraph_error_t** error)
{
  *weights = nullptr;
  *error   = nullptr;
  return guarded(error, [&] {
    CGX_INPUT(weight_dtype == FLOAT32 || weight_dtype == FLOAT64, "weight dtype must be FLOAT32 or FLOAT64");
    hipStream_t s = H(handle)->stream;
    auto* pw      = new device_array_t(num_edges, weight_dtype, s);
    if (num_edges) {
      if (weight_dtype == FLOAT32)
        hipLaunchKernelGGL(k_weights<float>, dim3(grid_for(num_edges, kBlock, 16384)), dim3(kBlock), 0, s,
                           pw->buf.data<float>(), num_edges, seed, (uint64_t)first_edge);
      else
        hipLaunchKernelGGL(k_weights<double>, dim3(grid_for(num_edges, kBlock, 16384)), dim3(kBlock), 0, s,
                           pw->buf.data<double>(), num_edges, seed, (uint64_t)first_edge);
      CGX_LAUNCH_CHECK();
    }
    HIP_CHECK(hipStreamSynchronize(s));
    *weights = reinterpret_cast<cugraph_type_erased_device_array_t*>(pw);
  });
}

extern "C" cugraph_error_code_t cugraph_amd_symmetrize_dedup(const cugraph_resource_handle_t* handle,
                                                            const cugraph_type_erased_device_array_view_t* src,
                                                            const cugraph_type_erased_device_array_view_t* dst,
                                                            const cugraph_type_erased_device_array_view_t* weights,
                                                            bool_t symmetrize,
                                                            cugraph_type_erased_device_array_t** src_out,
                                                            cugraph_type_erased_device_array_t** dst_out,
                                                            cugraph_type_erased_device_array_t** weights_out,
                                                            cugraph_error_t** error)
{
  *src_out = nullptr;
  *dst_out = nullptr;
  if (weights_out) *weights_out = nullptr;
  *error = nullptr;
  return guarded(error, [&] {
    auto const* ps = AV(src);
    auto const* pd = AV(dst);
    auto const* pw = weights ? AV(weights) : nullptr;
    CGX_INPUT(ps->size == pd->size && ps->type == pd->type, "src/dst size or type mismatch");
    CGX_INPUT(!pw || pw->size == ps->size, "weights size mismatch");
    std::unique_ptr<device_array_t> so, dout, wo;
    auto run = [&](auto vtag, auto wtag) {
      using V = decltype(vtag);
      using W = decltype(wtag);
      sym_dedup<V, W>(*H(handle), *ps, *pd, pw, symmetrize == TRUE, so, dout, wo);
    };
    bool w64 = pw && pw->type == FLOAT64;
    if (ps->type == INT32) {
      if (w64) run(int32_t{}, double{});
      else run(int32_t{}, float{});
    } else {
      if (w64) run(int64_t{}, double{});
      else run(int64_t{}, float{});
    }
    *src_out = reinterpret_cast<cugraph_type_erased_device_array_t*>(so.release());
    *dst_out = reinterpret_cast<cugraph_type_erased_device_array_t*>(dout.release());
    if (weights_out) *weights_out = reinterpret_cast<cugraph_type_erased_device_array_t*>(wo.release());
  });
}
