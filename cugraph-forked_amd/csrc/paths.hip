// extract_bfs_paths: paths from BFS/SSSP predecessors back to the source.
//
// Reference: cpp/src/traversal/extract_bfs_paths_impl.cuh:140-250 and
// c_api/extract_paths.cpp.  max_path_length = 1 + max over destinations of
// (predecessor invalid ? 0 : distance); paths is a row-major
// [destinations x max_path_length] matrix of external ids, -1 padded, the
// destination at column distance[d] and its predecessors to the left.  The
// reference indexes column distance[d] also for unreachable destinations (an
// out-of-range write); here their rows stay -1.  One thread walks one path (the
// depth is the BFS depth).
#include "capi.hpp"
#include "prims.hpp"

#include <limits>

namespace cgx {

namespace {

template <typename V>
__device__ inline V to_internal(V ext, V const* sorted_ext, V const* internal, int64_t nv)
{
  if (!sorted_ext) return ext;
  int64_t lo = 0, hi = nv;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (sorted_ext[mid] < ext) lo = mid + 1;
    else hi = mid;
  }
  return (lo < nv && sorted_ext[lo] == ext) ? internal[lo] : (V)-1;
}

template <typename V>
__global__ void k_path_length(V const* dest, size_t n, V const* dist, V const* pred, unsigned long long* maxlen)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    V d = dest[i];
    unsigned long long len = pred[d] == (V)-1 ? 0ull : (unsigned long long)dist[d];
    atomicMax(maxlen, len);
  }
}

template <typename V>
__global__ void k_extract(V const* dest, size_t n, V const* dist, V const* pred, V const* nmap, V const* sorted_ext,
                          V const* internal, int64_t nv, int64_t L, V* paths)
{
  V const INF = std::numeric_limits<V>::max();
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    V v = dest[i];
    if (dist[v] == INF) continue;
    int64_t pos = (int64_t)dist[v];
    V* row      = paths + i * L;
    row[pos]    = nmap ? nmap[v] : v;
    while (--pos >= 0) {
      V p = pred[v];  // external id
      if (p == (V)-1) break;
      row[pos] = p;
      v        = to_internal<V>(p, sorted_ext, internal, nv);
      if (v == (V)-1) break;
    }
  }
}

template <typename V>
void extract_impl(handle_t& h, graph_t& g, paths_result_t const& pr, array_view_t const* dests,
                  extract_paths_result_t& res)
{
  hipStream_t s = h.stream;
  CGX_INPUT(pr.distances != nullptr, "Invalid input argument: distances cannot be null");
  CGX_INPUT(pr.predecessors != nullptr && pr.predecessors->size == (size_t)g.num_vertices,
            "Invalid input argument: predecessors cannot be null");
  CGX_INPUT(dests->type == g.vertex_type, "Invalid input argument: destinations must have the graph's vertex type");
  size_t n = dests->size;
  dbuf<V> d(std::max<size_t>(n, 1), s);
  if (n) HIP_CHECK(hipMemcpyAsync(d.data(), dests->data, n * sizeof(V), hipMemcpyDeviceToDevice, s));
  renumber_ext_to_int(h, g, d.data(), n, true);
  V const* dist = pr.distances->buf.data<V>();
  V const* pred = pr.predecessors->buf.data<V>();
  dbuf<unsigned long long> ml(1, s);
  fill<unsigned long long>(ml.data(), 1, 0ull, s);
  if (n)
    hipLaunchKernelGGL(k_path_length<V>, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, d.data(), n, dist, pred,
                       ml.data());
  CGX_LAUNCH_CHECK();
  int64_t L = (int64_t)to_host_scalar(ml.data(), s) + 1;
  res.max_path_length = (size_t)L;
  res.paths           = std::make_unique<device_array_t>(n * (size_t)L, g.vertex_type, s);
  if (!n) return;
  fill<V>(res.paths->buf.data<V>(), n * (size_t)L, (V)-1, s);
  V const* sorted_ext = nullptr;
  V const* internal   = nullptr;
  if (g.renumbered) {
    ensure_ext_lookup(h, g);
    sorted_ext = g.ext_sorted.data<V>();
    internal   = g.ext_internal.data<V>();
  }
  hipLaunchKernelGGL(k_extract<V>, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, d.data(), n, dist, pred,
                     g.renumbered ? g.number_map.data<V>() : nullptr, sorted_ext, internal, g.num_vertices, L,
                     res.paths->buf.data<V>());
  CGX_LAUNCH_CHECK();
  HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace

void run_extract_paths(handle_t& h, graph_t& g, paths_result_t const& pr, array_view_t const* dests,
                       extract_paths_result_t& res)
{
  if (g.vertex_type == INT32) extract_impl<int32_t>(h, g, pr, dests, res);
  else extract_impl<int64_t>(h, g, pr, dests, res);
}

}  // namespace cgx
