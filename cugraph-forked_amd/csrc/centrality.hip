// Katz, eigenvector centrality and HITS -- power iterations on the pull SpMV
// (they reuse PageRank's per_v_transform_reduce_incoming_e).
//
// Reference: centrality/katz_centrality_impl.cuh:41-150 (+ c_api/katz.cpp:95-130),
// centrality/eigenvector_centrality_impl.cuh:40-125 (+ c_api/eigenvector_centrality.cpp),
// link_analysis/hits_impl.cuh:40-160 (+ c_api/hits.cpp).  Same iteration, stop rules,
// error messages and normalisations; values are stored in weight_t every iteration
// as the reference does, sums are fp64.  One degree-binned pull kernel (schedule.hpp)
// serves all three; reductions are block-ordered (deterministic).
#include "capi.hpp"
#include "prims.hpp"
#include "schedule.hpp"

#include <cfloat>
#include <cmath>

namespace cgx {

namespace {

inline unsigned blocks(int64_t n) { return grid_for(n > 0 ? n : 1, kBlock, 8192); }

// y[v] = sum over the row of v of x[u] (* w)   -- rows in the schedule's processing order
template <typename V, typename E, typename R, bool WEIGHTED>
__global__ __launch_bounds__(256) void k_spmv(E const* off, V const* idx, R const* wgt, V const* order,
                                              work_item const* items, R const* x, double* y)
{
  __shared__ double sm[4];
  work_item const it = items[blockIdx.x];
  int const tid      = threadIdx.x;
  auto term          = [&](E e) -> double {
    double t = (double)x[idx[e]];
    if constexpr (WEIGHTED) t *= (double)wgt[e];
    return t;
  };
  if (it.width == 256) {
    for (int64_t p = it.begin; p < it.end; ++p) {
      V v      = order ? order[p] : (V)p;
      double s = 0;
      for (E e = off[v] + tid; e < off[v + 1]; e += 256) s += term(e);
      s = block_sum_256(s, sm);
      if (tid == 0) y[v] = s;
    }
  } else {
    int const w = it.width, lane = tid & (w - 1), group = tid / w, groups = 256 / w;
    for (int64_t p0 = it.begin; p0 < it.end; p0 += groups) {
      int64_t p  = p0 + group;
      bool valid = p < it.end;
      double s   = 0;
      V v        = 0;
      if (valid) {
        v = order ? order[p] : (V)p;
        for (E e = off[v] + lane; e < off[v + 1]; e += w) s += term(e);
      }
      for (int o = w >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (valid && lane == 0) y[v] = s;
    }
  }
}

template <typename V, typename E, typename R>
void spmv(handle_t& h, graph_t& g, adjacency_t& adj, bool use_weights, R const* x, double* y)
{
  if (adj.num_items == 0) return;
  bool w    = use_weights && g.weighted;
  auto kern = w ? k_spmv<V, E, R, true> : k_spmv<V, E, R, false>;
  hipLaunchKernelGGL(kern, dim3(adj.num_items), dim3(kBlock), 0, h.stream, adj.offsets.data<E>(), adj.indices.data<V>(),
                     w ? adj.weights.data<R>() : nullptr, adj.degree_sorted ? nullptr : adj.order.data<V>(),
                     adj.items.data<work_item>(), x, y);
  CGX_LAUNCH_CHECK();
}

struct absdiff_f {
  void const* a;
  void const* b;
  int fp64;
  __device__ double operator()(size_t i) const
  {
    return fp64 ? fabs(((double const*)a)[i] - ((double const*)b)[i])
                : fabs((double)((float const*)a)[i] - (double)((float const*)b)[i]);
  }
};
struct sq_f {
  void const* a;
  int fp64;
  __device__ double operator()(size_t i) const
  {
    double v = fp64 ? ((double const*)a)[i] : (double)((float const*)a)[i];
    return v * v;
  }
};
struct val_f {
  void const* a;
  int fp64;
  __device__ double operator()(size_t i) const { return fp64 ? ((double const*)a)[i] : (double)((float const*)a)[i]; }
};

template <typename R>
struct reducer {
  hipStream_t s;
  dbuf<double> scratch, out;
  explicit reducer(hipStream_t st) : s(st), scratch(1024, st), out(1, st) {}
  double absdiff(R const* a, R const* b, int64_t n)
  {
    device_sum(absdiff_f{a, b, sizeof(R) == 8}, (size_t)n, out.data(), scratch.data(), s);
    return to_host_scalar(out.data(), s);
  }
  double sumsq(R const* a, int64_t n)
  {
    device_sum(sq_f{a, sizeof(R) == 8}, (size_t)n, out.data(), scratch.data(), s);
    return to_host_scalar(out.data(), s);
  }
  double sum(R const* a, int64_t n)
  {
    device_sum(val_f{a, sizeof(R) == 8}, (size_t)n, out.data(), scratch.data(), s);
    return to_host_scalar(out.data(), s);
  }
};

// max of non-negative doubles via their bit patterns (ordered like unsigned integers)
__global__ void k_max_nonneg(double const* y, int64_t n, unsigned long long* out)
{
  unsigned long long m = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double v = y[i] > 0.0 ? y[i] : 0.0;
    unsigned long long b = __double_as_longlong(v);
    m = b > m ? b : m;
  }
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long t = __shfl_xor(m, o, 64);
    m = t > m ? t : m;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

double max_nonneg(double const* y, int64_t n, hipStream_t s)
{
  dbuf<unsigned long long> m(1, s);
  fill<unsigned long long>(m.data(), 1, 0ull, s);
  hipLaunchKernelGGL(k_max_nonneg, dim3(blocks(n)), dim3(kBlock), 0, s, y, n, m.data());
  CGX_LAUNCH_CHECK();
  unsigned long long b = to_host_scalar(m.data(), s);
  double v;
  std::memcpy(&v, &b, sizeof(v));
  return v;
}

template <typename R>
__global__ void k_katz_update(double const* y, R const* betas, double beta, double alpha, int64_t n, R* out)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
    out[v] = (R)((double)(R)(alpha * y[v]) + (betas ? (double)betas[v] : beta));
}

template <typename R>
__global__ void k_scale(double const* y, double inv, int64_t n, R* out)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
    out[v] = (R)(y[v] * inv);
}

template <typename R>
__global__ void k_scale_inplace(R* x, double inv, int64_t n)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
    x[v] = (R)((double)x[v] * inv);
}

// betas / initial values given by external vertex id i (c_api/katz.cpp:103-118:
// collect_local_vertex_values_from_ext_vertex_value_pairs, missing -> 0)
template <typename V, typename R>
__global__ void k_values_by_ext(V const* nmap, int64_t n, R const* vals, size_t nvals, R* out)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    int64_t ext = (int64_t)nmap[v];
    out[v]      = (ext >= 0 && (size_t)ext < nvals) ? vals[ext] : R(0);
  }
}

template <typename V, typename R>
__global__ void k_scatter(V const* ids, R const* vals, size_t n, R* out)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[ids[i]] = vals[i];
}

template <typename R>
__global__ void k_count_neg(R const* x, int64_t n, int* bad, bool nonpositive)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (nonpositive ? !(x[i] > R(0)) : x[i] < R(0)) atomicAdd(bad, 1);
}

template <typename R>
int count_bad(R const* x, int64_t n, bool nonpositive, hipStream_t s)
{
  if (n <= 0) return 0;
  dbuf<int> bad(1, s);
  fill<int>(bad.data(), 1, 0, s);
  hipLaunchKernelGGL(k_count_neg<R>, dim3(blocks(n)), dim3(kBlock), 0, s, x, n, bad.data(), nonpositive);
  CGX_LAUNCH_CHECK();
  return to_host_scalar(bad.data(), s);
}

// ---------------------------------------------------------------- Katz
template <typename V, typename E, typename R>
void katz_impl(handle_t& h, graph_t& g, array_view_t const* betas, double alpha, double beta, double eps,
               size_t max_iter, bool expensive, centrality_result_t& res)
{
  hipStream_t s = h.stream;
  int64_t nv    = g.num_vertices;
  res.vertices  = number_map_copy(h, g);
  res.values    = std::make_unique<device_array_t>((size_t)nv, dtype_of<R>(), s);
  if (nv == 0) return;
  CGX_INPUT(alpha >= 0.0 && alpha <= 1.0, "Invalid input argument: alpha should be in [0.0, 1.0].");
  CGX_INPUT(eps >= 0.0, "Invalid input argument: epsilon should be non-negative.");
  adjacency_t& adj = ensure_adjacency(h, g, true);
  ensure_schedule(h, g, adj);
  dbuf<R> b;
  if (betas) {
    CGX_INPUT(betas->type == dtype_of<R>(), "Invalid input argument: betas type must match the weight type");
    b.resize(nv, s);
    hipLaunchKernelGGL((k_values_by_ext<V, R>), dim3(blocks(nv)), dim3(kBlock), 0, s, g.number_map.data<V>(), nv,
                       betas->as<R>(), betas->size, b.data());
    CGX_LAUNCH_CHECK();
  }
  (void)expensive;
  R* x = res.values->buf.data<R>();
  dbuf<R> x2(nv, s);
  dbuf<double> y(nv, s);
  fill<R>(x, nv, R(0), s);
  reducer<R> red(s);
  R* cur = x;
  R* nxt = x2.data();
  size_t it = 0;
  while (true) {
    spmv<V, E, R>(h, g, adj, true, cur, y.data());
    hipLaunchKernelGGL(k_katz_update<R>, dim3(blocks(nv)), dim3(kBlock), 0, s, y.data(), betas ? b.data() : nullptr,
                       beta, alpha, nv, nxt);
    CGX_LAUNCH_CHECK();
    double diff = red.absdiff(nxt, cur, nv);
    std::swap(cur, nxt);
    ++it;
    if (diff < eps) break;
    if (it >= max_iter) fail(CUGRAPH_UNKNOWN_ERROR, "Katz Centrality failed to converge.");
  }
  if (cur != x) HIP_CHECK(hipMemcpyAsync(x, cur, nv * sizeof(R), hipMemcpyDeviceToDevice, s));
  double l2 = std::sqrt(red.sumsq(x, nv));
  CGX_EXPECTS(l2 > 0.0, CUGRAPH_UNKNOWN_ERROR, "L2 norm of the computed Katz Centrality values should be positive.");
  hipLaunchKernelGGL(k_scale_inplace<R>, dim3(blocks(nv)), dim3(kBlock), 0, s, x, 1.0 / l2, nv);
  CGX_LAUNCH_CHECK();
  h.last_iterations = it;
}

// ---------------------------------------------------------------- eigenvector
template <typename V, typename E, typename R>
void eigenvector_impl(handle_t& h, graph_t& g, double eps, size_t max_iter, bool expensive, centrality_result_t& res)
{
  hipStream_t s = h.stream;
  int64_t nv    = g.num_vertices;
  res.vertices  = number_map_copy(h, g);
  res.values    = std::make_unique<device_array_t>((size_t)nv, dtype_of<R>(), s);
  if (nv == 0) return;
  CGX_INPUT(eps >= 0.0, "Invalid input argument: epsilon should be non-negative.");
  adjacency_t& adj = ensure_adjacency(h, g, true);
  ensure_schedule(h, g, adj);
  if (expensive && g.weighted)
    CGX_INPUT(count_bad<R>(adj.weights.data<R>(), g.num_edges, true, s) == 0,
              "Invalid input argument: input graph should have postive edge weights.");
  R* x = res.values->buf.data<R>();
  dbuf<R> old(nv, s);
  dbuf<double> y(nv, s);
  fill<R>(x, nv, (R)(R(1.0) / (R)nv), s);
  reducer<R> red(s);
  size_t it = 0;
  while (true) {
    HIP_CHECK(hipMemcpyAsync(old.data(), x, nv * sizeof(R), hipMemcpyDeviceToDevice, s));
    spmv<V, E, R>(h, g, adj, true, x, y.data());
    dbuf<double> sc(1024, s), o(1, s);
    device_sum(sq_f{y.data(), 1}, (size_t)nv, o.data(), sc.data(), s);
    double hyp = std::sqrt(to_host_scalar(o.data(), s));
    hipLaunchKernelGGL(k_scale<R>, dim3(blocks(nv)), dim3(kBlock), 0, s, y.data(), 1.0 / hyp, nv, x);
    CGX_LAUNCH_CHECK();
    double diff = red.absdiff(x, old.data(), nv);
    ++it;
    if (diff < (double)nv * eps) break;
    if (it >= max_iter) fail(CUGRAPH_UNKNOWN_ERROR, "Eigenvector Centrality failed to converge.");
  }
  h.last_iterations = it;
}

// ---------------------------------------------------------------- HITS
template <typename V, typename E, typename R>
void hits_impl(handle_t& h, graph_t& g, double eps, size_t max_iter, array_view_t const* guess_v,
               array_view_t const* guess_s, bool normalize, bool expensive, hits_result_t& res)
{
  hipStream_t s = h.stream;
  int64_t nv    = g.num_vertices;
  res.vertices    = number_map_copy(h, g);
  res.hubs        = std::make_unique<device_array_t>((size_t)nv, dtype_of<R>(), s);
  res.authorities = std::make_unique<device_array_t>((size_t)nv, dtype_of<R>(), s);
  res.hub_score_differences = DBL_MAX;
  res.number_of_iterations  = max_iter;
  if (nv == 0) return;
  CGX_INPUT(eps >= 0.0, "Invalid input argument: epsilon should be non-negative.");
  adjacency_t& in = ensure_adjacency(h, g, true);
  ensure_schedule(h, g, in);
  adjacency_t& out = ensure_adjacency(h, g, false);
  ensure_schedule(h, g, out);
  R* hubs = res.hubs->buf.data<R>();
  R* auth = res.authorities->buf.data<R>();
  dbuf<R> hubs2(nv, s);
  dbuf<double> y(nv, s), z(nv, s);
  reducer<R> red(s);
  if (guess_v) {
    CGX_INPUT(guess_v->size == guess_s->size, "Invalid input argument: initial hubs vertices and values differ in size");
    CGX_INPUT(guess_v->type == g.vertex_type && guess_s->type == dtype_of<R>(),
              "Invalid input argument: initial hubs guess types do not match the graph");
    fill<R>(hubs, nv, R(0), s);
    dbuf<V> ids(std::max<size_t>(guess_v->size, 1), s);
    if (guess_v->size)
      HIP_CHECK(hipMemcpyAsync(ids.data(), guess_v->data, guess_v->size * sizeof(V), hipMemcpyDeviceToDevice, s));
    renumber_ext_to_int(h, g, ids.data(), guess_v->size, true);
    if (guess_v->size)
      hipLaunchKernelGGL((k_scatter<V, R>), dim3(blocks(guess_v->size)), dim3(kBlock), 0, s, ids.data(),
                         guess_s->as<R>(), guess_v->size, hubs);
    CGX_LAUNCH_CHECK();
    if (expensive)
      CGX_INPUT(count_bad<R>(hubs, nv, false, s) == 0,
                "Invalid input argument: initial guess values should be non-negative.");
    double sum = red.sum(hubs, nv);
    CGX_EXPECTS(sum > 0, CUGRAPH_UNKNOWN_ERROR, "Norm is required to be a positive value.");
    hipLaunchKernelGGL(k_scale_inplace<R>, dim3(blocks(nv)), dim3(kBlock), 0, s, hubs, 1.0 / sum, nv);
    CGX_LAUNCH_CHECK();
  } else {
    fill<R>(hubs, nv, (R)(R(1.0) / (R)nv), s);
  }
  R* prev = hubs;
  R* curr = hubs2.data();
  for (size_t it = 0; it < max_iter; ++it) {
    spmv<V, E, R>(h, g, in, false, prev, y.data());  // authorities = A^T hubs
    double ma = max_nonneg(y.data(), nv, s);
    // hubs' = A authorities, from the authorities stored in weight_t
    hipLaunchKernelGGL(k_scale<R>, dim3(blocks(nv)), dim3(kBlock), 0, s, y.data(), 1.0, nv, auth);
    CGX_LAUNCH_CHECK();
    spmv<V, E, R>(h, g, out, false, auth, z.data());
    double mh = max_nonneg(z.data(), nv, s);
    CGX_EXPECTS(mh > 0 && ma > 0, CUGRAPH_UNKNOWN_ERROR, "Norm is required to be a positive value.");
    hipLaunchKernelGGL(k_scale<R>, dim3(blocks(nv)), dim3(kBlock), 0, s, z.data(), 1.0 / mh, nv, curr);
    hipLaunchKernelGGL(k_scale_inplace<R>, dim3(blocks(nv)), dim3(kBlock), 0, s, auth, 1.0 / ma, nv);
    CGX_LAUNCH_CHECK();
    double diff = red.absdiff(curr, prev, nv);
    res.hub_score_differences = diff;
    std::swap(prev, curr);
    if (diff < eps) {
      res.number_of_iterations = it;
      break;
    }
  }
  if (normalize) {
    double sh = red.sum(prev, nv), sa = red.sum(auth, nv);
    CGX_EXPECTS(sh > 0 && sa > 0, CUGRAPH_UNKNOWN_ERROR, "Norm is required to be a positive value.");
    hipLaunchKernelGGL(k_scale_inplace<R>, dim3(blocks(nv)), dim3(kBlock), 0, s, prev, 1.0 / sh, nv);
    hipLaunchKernelGGL(k_scale_inplace<R>, dim3(blocks(nv)), dim3(kBlock), 0, s, auth, 1.0 / sa, nv);
    CGX_LAUNCH_CHECK();
  }
  if (prev != hubs) HIP_CHECK(hipMemcpyAsync(hubs, prev, nv * sizeof(R), hipMemcpyDeviceToDevice, s));
  h.last_iterations = res.number_of_iterations;
}

}  // namespace

void run_katz(handle_t& h, graph_t& g, array_view_t const* betas, double alpha, double beta, double eps,
              size_t max_iter, bool expensive, centrality_result_t& res)
{
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    katz_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g, betas, alpha, beta, eps, max_iter,
                                                                              expensive, res);
  });
}

void run_eigenvector(handle_t& h, graph_t& g, double eps, size_t max_iter, bool expensive, centrality_result_t& res)
{
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    eigenvector_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g, eps, max_iter, expensive,
                                                                                     res);
  });
}

void run_hits(handle_t& h, graph_t& g, double eps, size_t max_iter, array_view_t const* guess_v,
              array_view_t const* guess_s, bool normalize, bool expensive, hits_result_t& res)
{
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    hits_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g, eps, max_iter, guess_v, guess_s,
                                                                              normalize, expensive, res);
  });
}

}  // namespace cgx
