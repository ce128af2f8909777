// Louvain modularity clustering (single GPU).
//
// Reference: cpp/src/community/louvain_impl.cuh:46-301 (level loop, dendrogram,
// flatten), community/detail/common_methods.cuh:49-382 (delta-modularity local
// move, cluster weights, modularity, contraction) and
// structure/coarsen_graph_impl.cuh:527-632.  Same control flow as the reference
// (and oracle/louvain.py): per level, vertex weights k = out-weight sums,
// singleton clusters, `while Q' > Q + 1e-4` synchronous sweeps with the up/down
// restriction alternating, keep the level's clustering only when Q improved,
// stop when the level brings no gain, else contract.
//
// Arithmetic is fp64 throughout (weights are widened once), with FMA contraction
// off so that every gain is the same IEEE expression as the oracle's; sums whose
// order differs from numpy's are exact for integer weights, so the clustering is
// bit-identical there and modularity agrees to rounding otherwise.
//
// Each level is a COO sorted by (source, destination) with 32-bit ids.  A sweep:
//   1. key = source << 32 | cluster(destination) per edge, stable radix sort;
//   2. reduce_by_key -> (u, c, sum of w) for every (vertex, neighbour cluster);
//   3. gain per pair, reduce_by_key over u with (max gain, smaller cluster) -> move.
// Cluster weights are a reduce_by_key over vertices sorted by cluster.  All
// reductions are rocPRIM's fixed-partition scans or block-ordered sums: the run is
// deterministic.
#include "capi.hpp"
#include "prims.hpp"

#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <cfloat>
#include <limits>

namespace cgx {

namespace {

using u64 = unsigned long long;

struct level_graph {
  int64_t nv = 0, ne = 0;
  dbuf<uint32_t> src, dst;  // sorted by (src, dst)
  dbuf<double> w;
};

struct gain_t {
  double dq;
  uint32_t c;
};

struct best_gain_op {
  __host__ __device__ gain_t operator()(gain_t const& a, gain_t const& b) const
  {
    if (a.dq > b.dq) return a;
    if (b.dq > a.dq) return b;
    return a.c < b.c ? a : b;
  }
};

struct key_hi {
  __host__ __device__ uint32_t operator()(u64 k) const { return (uint32_t)(k >> 32); }
};

template <typename KI, typename VI, typename KO, typename VO, typename Op, typename Eq>
int64_t reduce_by_key(KI keys, VI vals, size_t n, KO ukeys, VO aggs, Op op, Eq eq, hipStream_t s)
{
  if (n == 0) return 0;
  dbuf<u64> cnt(1, s);
  size_t tmp = 0;
  HIP_CHECK(rocprim::reduce_by_key(nullptr, tmp, keys, vals, n, ukeys, aggs, cnt.data(), op, eq, s));
  buffer t(tmp, s);
  HIP_CHECK(rocprim::reduce_by_key(t.data(), tmp, keys, vals, n, ukeys, aggs, cnt.data(), op, eq, s));
  return (int64_t)to_host_scalar(cnt.data(), s);
}

// ---------------------------------------------------------------- kernels
template <typename V, typename E, typename R>
__global__ void k_expand(E const* off, V const* idx, R const* w, int64_t nv, int64_t ne, uint32_t* src, uint32_t* dst,
                         double* ww)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nv - 1;  // last row with off[row] <= e
    while (lo < hi) {
      int64_t mid = (lo + hi + 1) >> 1;
      if ((int64_t)off[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    src[e] = (uint32_t)lo;
    dst[e] = (uint32_t)idx[e];
    ww[e]  = (double)w[e];
  }
}

// off[v] = first edge with src >= v, v in [0, nv]
__global__ void k_row_offsets(uint32_t const* src, int64_t ne, int64_t nv, int64_t* off)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v <= nv; v += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = ne;
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if ((int64_t)src[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    off[v] = lo;
  }
}

// vertex weights k[v] (row sums, in edge order) and self-loop weights
__global__ void k_vertex_weights(int64_t const* off, uint32_t const* src, uint32_t const* dst, double const* w,
                                 int64_t nv, double* k, double* self, uint8_t* has_edges)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x) {
    double s = 0, sl = 0;
    for (int64_t e = off[v]; e < off[v + 1]; ++e) {
      s += w[e];
      if (dst[e] == (uint32_t)v) sl += w[e];
    }
    k[v]         = s;
    self[v]      = sl;
    has_edges[v] = off[v + 1] > off[v] ? 1 : 0;
  }
}

__global__ void k_sweep_keys(uint32_t const* src, uint32_t const* dst, uint32_t const* c, int64_t ne, u64* keys)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x)
    keys[e] = ((u64)src[e] << 32) | (u64)c[dst[e]];
}

// old_sum[u] = weight from u into its own cluster, self loops excluded
__global__ void k_old_sum(u64 const* uk, double const* psum, int64_t np, uint32_t const* c, double const* self,
                          double* old_sum)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t u = (uint32_t)(uk[i] >> 32), cc = (uint32_t)uk[i];
    if (cc == c[u]) old_sum[u] = psum[i] - self[u];
  }
}

// delta modularity of moving u into cluster cc (common_methods.cuh:49-74)
__global__ void k_gain(u64 const* uk, double const* psum, int64_t np, uint32_t const* c, double const* self,
                       double const* old_sum, double const* a, uint8_t const* present, double const* k, double m,
                       double gamma, gain_t* out)
{
#pragma clang fp contract(off)
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t u = (uint32_t)(uk[i] >> 32), cc = (uint32_t)uk[i];
    double s   = psum[i];
    if (cc == c[u]) s = s - self[u];
    double a_new = present[cc] ? a[cc] : (double)FLT_MAX;
    double a_old = a[c[u]];
    double kk    = k[u];
    double dq    = 2.0 * (((s - old_sum[u]) / m) - gamma * (a_new * kk - a_old * kk + kk * kk) / (m * m));
    out[i]       = gain_t{dq, cc};
  }
}

__global__ void k_move(uint32_t const* uu, gain_t const* best, int64_t n, uint32_t const* c, uint32_t* next,
                       bool up_down)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t u = uu[i];
    gain_t b   = best[i];
    if (b.dq > 0.0 && ((b.c > c[u]) == up_down)) next[u] = b.c;
  }
}

__global__ void k_scatter_cluster_weights(uint32_t const* ck, double const* cw, int64_t n, double* a)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    a[ck[i]] = cw[i];
}

__global__ void k_mark_present(uint32_t const* c, uint8_t const* has_edges, int64_t nv, uint8_t* present)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x)
    if (has_edges[v]) present[c[v]] = 1;
}

struct internal_f {
  uint32_t const* s;
  uint32_t const* d;
  double const* w;
  uint32_t const* c;
  __device__ double operator()(size_t i) const { return c[s[i]] == c[d[i]] ? w[i] : 0.0; }
};
struct sumsq_f {
  double const* a;
  uint8_t const* p;
  __device__ double operator()(size_t i) const { return p[i] ? a[i] * a[i] : 0.0; }
};
struct plain_f {
  double const* w;
  __device__ double operator()(size_t i) const { return w[i]; }
};

// contraction
__global__ void k_pair_keys(uint32_t const* src, uint32_t const* dst, uint32_t const* lab, int64_t ne, u64* keys)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x)
    keys[e] = ((u64)lab[src[e]] << 32) | (u64)lab[dst[e]];
}

__global__ void k_mark_used(uint32_t const* lab, int64_t nv, uint32_t* used)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x)
    used[lab[v]] = 1u;
}

__global__ void k_count_src(u64 const* keys, int64_t n, uint32_t* deg)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(deg + (uint32_t)(keys[i] >> 32), 1u);
}

// uniq[pos[l]] = l for used labels; udeg likewise
__global__ void k_compact_labels(uint32_t const* used, uint32_t const* pos, uint32_t const* deg, int64_t nv,
                                 uint32_t* uniq, uint32_t* udeg)
{
  for (int64_t l = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; l < nv; l += (int64_t)gridDim.x * blockDim.x)
    if (used[l]) {
      uniq[pos[l]] = (uint32_t)l;
      udeg[pos[l]] = deg[l];
    }
}

__global__ void k_new_ids(uint32_t const* nmap, int64_t n, uint32_t* new_of_label)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    new_of_label[nmap[i]] = (uint32_t)i;
}

__global__ void k_relabel_pairs(u64 const* keys, int64_t n, uint32_t const* nl, u64* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = ((u64)nl[(uint32_t)(keys[i] >> 32)] << 32) | (u64)nl[(uint32_t)keys[i]];
}

__global__ void k_split_pairs(u64 const* keys, int64_t n, uint32_t* s, uint32_t* d)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    s[i] = (uint32_t)(keys[i] >> 32);
    d[i] = (uint32_t)keys[i];
  }
}

__global__ void k_gather_u32(uint32_t const* table, uint32_t* x, int64_t n)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = table[x[i]];
}

template <typename V>
__global__ void k_to_vertex(uint32_t const* x, int64_t n, V* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (V)x[i];
}

inline unsigned blocks(int64_t n) { return grid_for(n > 0 ? n : 1, kBlock, 16384); }

// ---------------------------------------------------------------- driver
struct louvain_state {
  hipStream_t s;
  double m;
  double gamma;
  dbuf<double> scratch;  // device_sum partials
  dbuf<double> scal;     // 2 scalars
  explicit louvain_state(hipStream_t st) : s(st), scratch(1024, st), scal(2, st) {}
};

double modularity(louvain_state& S, level_graph const& g, uint32_t const* c, double const* a, uint8_t const* present)
{
  device_sum(internal_f{g.src.data(), g.dst.data(), g.w.data(), c}, (size_t)g.ne, S.scal.data(), S.scratch.data(), S.s);
  device_sum(sumsq_f{a, present}, (size_t)g.nv, S.scal.data() + 1, S.scratch.data(), S.s);
  auto hv = to_host(S.scal.data(), 2, S.s);
  return hv[0] / S.m - (S.gamma * hv[1]) / (S.m * S.m);
}

// cluster weights a[c] = sum of k[v] over v in c; present[c] = some v in c has edges
void cluster_weights(louvain_state& S, level_graph const& g, uint32_t const* c, double const* k,
                     uint8_t const* has_edges, double* a, uint8_t* present)
{
  hipStream_t s = S.s;
  int64_t nv    = g.nv;
  dbuf<uint32_t> ck(nv, s), ck2(nv, s);
  dbuf<double> kv2(nv, s);
  HIP_CHECK(hipMemcpyAsync(ck.data(), c, nv * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  radix_sort_pairs<uint32_t, double>(ck.data(), ck2.data(), k, kv2.data(), (size_t)nv, 0, bits_for(nv - 1), s);
  dbuf<uint32_t> uk(nv, s);
  dbuf<double> uw(nv, s);
  int64_t nu = reduce_by_key(ck2.data(), kv2.data(), (size_t)nv, uk.data(), uw.data(), rocprim::plus<double>(),
                             rocprim::equal_to<uint32_t>(), s);
  fill<double>(a, nv, 0.0, s);
  fill<uint8_t>(present, nv, 0, s);
  hipLaunchKernelGGL(k_scatter_cluster_weights, dim3(blocks(nu)), dim3(kBlock), 0, s, uk.data(), uw.data(), nu, a);
  CGX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_mark_present, dim3(blocks(nv)), dim3(kBlock), 0, s, c, has_edges, nv, present);
  CGX_LAUNCH_CHECK();
}

// one synchronous local-move sweep (update_clustering_by_delta_modularity)
void sweep(louvain_state& S, level_graph const& g, uint32_t const* c, uint32_t* next, double const* k,
           double const* self, double const* a, uint8_t const* present, bool up_down)
{
  hipStream_t s = S.s;
  int64_t nv = g.nv, ne = g.ne;
  HIP_CHECK(hipMemcpyAsync(next, c, nv * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  if (ne == 0) return;
  dbuf<u64> keys(ne, s), keys2(ne, s);
  dbuf<double> w2(ne, s), psum(ne, s);
  hipLaunchKernelGGL(k_sweep_keys, dim3(blocks(ne)), dim3(kBlock), 0, s, g.src.data(), g.dst.data(), c, ne,
                     keys.data());
  CGX_LAUNCH_CHECK();
  radix_sort_pairs<u64, double>(keys.data(), keys2.data(), g.w.data(), w2.data(), (size_t)ne, 0,
                                32 + bits_for(nv - 1), s);
  // (vertex, neighbour cluster) -> sum of weights; `keys` reused for the pair keys
  int64_t np = reduce_by_key(keys2.data(), w2.data(), (size_t)ne, keys.data(), psum.data(), rocprim::plus<double>(),
                             rocprim::equal_to<u64>(), s);
  dbuf<double> old_sum(nv, s);
  fill<double>(old_sum.data(), nv, 0.0, s);
  hipLaunchKernelGGL(k_old_sum, dim3(blocks(np)), dim3(kBlock), 0, s, keys.data(), psum.data(), np, c, self,
                     old_sum.data());
  CGX_LAUNCH_CHECK();
  dbuf<gain_t> gains(np, s), best(nv, s);
  hipLaunchKernelGGL(k_gain, dim3(blocks(np)), dim3(kBlock), 0, s, keys.data(), psum.data(), np, c, self,
                     old_sum.data(), a, present, k, S.m, S.gamma, gains.data());
  CGX_LAUNCH_CHECK();
  dbuf<uint32_t> uu(nv, s);
  auto ukeys = rocprim::make_transform_iterator(keys.data(), key_hi());
  int64_t nu = reduce_by_key(ukeys, gains.data(), (size_t)np, uu.data(), best.data(), best_gain_op(),
                             rocprim::equal_to<uint32_t>(), s);
  hipLaunchKernelGGL(k_move, dim3(blocks(nu)), dim3(kBlock), 0, s, uu.data(), best.data(), nu, c, next, up_down);
  CGX_LAUNCH_CHECK();
}

// contract the level graph by `labels` (graph_contraction / coarsen_graph): sum
// parallel edges, renumber the used labels by descending coarse out-degree
// (stable: ties by ascending label), relabel the dendrogram level in place
level_graph contract(louvain_state& S, level_graph const& g, uint32_t* labels)
{
  hipStream_t s = S.s;
  int64_t nv = g.nv, ne = g.ne;
  dbuf<u64> keys(std::max<int64_t>(ne, 1), s), keys2(std::max<int64_t>(ne, 1), s);
  dbuf<double> w2(std::max<int64_t>(ne, 1), s), cw(std::max<int64_t>(ne, 1), s);
  int64_t nce = 0;
  if (ne) {
    hipLaunchKernelGGL(k_pair_keys, dim3(blocks(ne)), dim3(kBlock), 0, s, g.src.data(), g.dst.data(), labels, ne,
                       keys.data());
    CGX_LAUNCH_CHECK();
    radix_sort_pairs<u64, double>(keys.data(), keys2.data(), g.w.data(), w2.data(), (size_t)ne, 0,
                                  32 + bits_for(nv - 1), s);
    nce = reduce_by_key(keys2.data(), w2.data(), (size_t)ne, keys.data(), cw.data(), rocprim::plus<double>(),
                        rocprim::equal_to<u64>(), s);
  }
  // used labels (ascending) and their coarse out-degrees
  dbuf<uint32_t> used(nv + 1, s), pos(nv + 1, s), deg(nv, s);
  fill<uint32_t>(used.data(), nv + 1, 0u, s);
  fill<uint32_t>(deg.data(), nv, 0u, s);
  hipLaunchKernelGGL(k_mark_used, dim3(blocks(nv)), dim3(kBlock), 0, s, labels, nv, used.data());
  CGX_LAUNCH_CHECK();
  if (nce)
    hipLaunchKernelGGL(k_count_src, dim3(blocks(nce)), dim3(kBlock), 0, s, keys.data(), nce, deg.data());
  CGX_LAUNCH_CHECK();
  exclusive_scan<uint32_t, uint32_t>(used.data(), pos.data(), nv + 1, s);
  int64_t nu = (int64_t)to_host_scalar(pos.data() + nv, s);
  dbuf<uint32_t> uniq(nu, s), udeg(nu, s), udeg2(nu, s), nmap(nu, s), nl(nv, s);
  hipLaunchKernelGGL(k_compact_labels, dim3(blocks(nv)), dim3(kBlock), 0, s, used.data(), pos.data(), deg.data(), nv,
                     uniq.data(), udeg.data());
  CGX_LAUNCH_CHECK();
  radix_sort_pairs<uint32_t, uint32_t>(udeg.data(), udeg2.data(), uniq.data(), nmap.data(), (size_t)nu, 0,
                                       bits_for((unsigned long long)std::max<int64_t>(nce, 1)), s, /*descending=*/true);
  hipLaunchKernelGGL(k_new_ids, dim3(blocks(nu)), dim3(kBlock), 0, s, nmap.data(), nu, nl.data());
  CGX_LAUNCH_CHECK();
  level_graph out;
  out.nv = nu;
  out.ne = nce;
  out.src.resize(std::max<int64_t>(nce, 1), s);
  out.dst.resize(std::max<int64_t>(nce, 1), s);
  out.w.resize(std::max<int64_t>(nce, 1), s);
  if (nce) {
    hipLaunchKernelGGL(k_relabel_pairs, dim3(blocks(nce)), dim3(kBlock), 0, s, keys.data(), nce, nl.data(),
                       keys2.data());
    CGX_LAUNCH_CHECK();
    radix_sort_pairs<u64, double>(keys2.data(), keys.data(), cw.data(), out.w.data(), (size_t)nce, 0,
                                  32 + bits_for(nu - 1), s);
    hipLaunchKernelGGL(k_split_pairs, dim3(blocks(nce)), dim3(kBlock), 0, s, keys.data(), nce, out.src.data(),
                       out.dst.data());
    CGX_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_gather_u32, dim3(blocks(nv)), dim3(kBlock), 0, s, nl.data(), labels, nv);
  CGX_LAUNCH_CHECK();
  return out;
}

template <typename V, typename E, typename R>
void louvain_impl(handle_t& h, graph_t& g, size_t max_level, double resolution, clustering_result_t& res)
{
  hipStream_t s = h.stream;
  CGX_EXPECTS(g.weighted, CUGRAPH_UNKNOWN_ERROR, "Graph must be weighted");  // louvain_impl.cuh:290
  int64_t const nv0 = g.num_vertices;
  CGX_EXPECTS((uint64_t)nv0 < (1ull << 32), CUGRAPH_NOT_IMPLEMENTED, "Louvain: more than 2^32 vertices");
  res.vertices = number_map_copy(h, g);
  res.clusters = std::make_unique<device_array_t>((size_t)nv0, g.vertex_type, s);
  h.last_louvain_levels = 0;
  res.modularity        = 0;
  if (nv0 == 0) return;

  adjacency_t& adj = ensure_adjacency(h, g, /*transposed=*/false);
  louvain_state S(s);
  S.gamma = resolution;
  level_graph cur;
  cur.nv = nv0;
  cur.ne = g.num_edges;
  cur.src.resize(std::max<int64_t>(cur.ne, 1), s);
  cur.dst.resize(std::max<int64_t>(cur.ne, 1), s);
  cur.w.resize(std::max<int64_t>(cur.ne, 1), s);
  if (cur.ne)
    hipLaunchKernelGGL((k_expand<V, E, R>), dim3(blocks(cur.ne)), dim3(kBlock), 0, s, adj.offsets.data<E>(),
                       adj.indices.data<V>(), adj.weights.data<R>(), nv0, cur.ne, cur.src.data(), cur.dst.data(),
                       cur.w.data());
  CGX_LAUNCH_CHECK();
  device_sum(plain_f{cur.w.data()}, (size_t)cur.ne, S.scal.data(), S.scratch.data(), s);
  S.m = to_host_scalar(S.scal.data(), s);  // total edge weight (constant over levels)

  std::vector<dbuf<uint32_t>> dendrogram;
  double best_q = -1.0;
  while (dendrogram.size() < max_level) {
    int64_t nv = cur.nv;
    dendrogram.emplace_back(std::max<int64_t>(nv, 1), s);
    uint32_t* level = dendrogram.back().data();
    iota<uint32_t>(level, nv, 0u, s);
    // vertex weights, cluster keys = every vertex (louvain_impl.cuh:91-103)
    dbuf<int64_t> off(nv + 1, s);
    hipLaunchKernelGGL(k_row_offsets, dim3(blocks(nv + 1)), dim3(kBlock), 0, s, cur.src.data(), cur.ne, nv, off.data());
    CGX_LAUNCH_CHECK();
    dbuf<double> k(nv, s), self(nv, s), a(nv, s);
    dbuf<uint8_t> has_edges(nv, s), present(nv, s);
    hipLaunchKernelGGL(k_vertex_weights, dim3(blocks(nv)), dim3(kBlock), 0, s, off.data(), cur.src.data(),
                       cur.dst.data(), cur.w.data(), nv, k.data(), self.data(), has_edges.data());
    CGX_LAUNCH_CHECK();
    HIP_CHECK(hipMemcpyAsync(a.data(), k.data(), nv * sizeof(double), hipMemcpyDeviceToDevice, s));
    fill<uint8_t>(present.data(), nv, 1, s);
    dbuf<uint32_t> clusters(nv, s), next(nv, s);
    iota<uint32_t>(clusters.data(), nv, 0u, s);
    double new_q = modularity(S, cur, clusters.data(), a.data(), present.data());
    double cur_q = new_q - 1.0;
    bool up_down = true;
    while (new_q > cur_q + 0.0001) {
      cur_q = new_q;
      sweep(S, cur, clusters.data(), next.data(), k.data(), self.data(), a.data(), present.data(), up_down);
      std::swap(clusters, next);
      cluster_weights(S, cur, clusters.data(), k.data(), has_edges.data(), a.data(), present.data());
      up_down = !up_down;
      new_q   = modularity(S, cur, clusters.data(), a.data(), present.data());
      if (new_q > cur_q)
        HIP_CHECK(hipMemcpyAsync(level, clusters.data(), nv * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    }
    if (cur_q <= best_q) break;
    best_q = cur_q;
    cur    = contract(S, cur, level);
  }
  // flatten_dendrogram (louvain_impl.cuh:239-255)
  dbuf<uint32_t> flat(nv0, s);
  iota<uint32_t>(flat.data(), nv0, 0u, s);
  for (auto& lvl : dendrogram)
    hipLaunchKernelGGL(k_gather_u32, dim3(blocks(nv0)), dim3(kBlock), 0, s, lvl.data(), flat.data(), nv0);
  CGX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_to_vertex<V>, dim3(blocks(nv0)), dim3(kBlock), 0, s, flat.data(), nv0,
                     res.clusters->buf.data<V>());
  CGX_LAUNCH_CHECK();
  HIP_CHECK(hipStreamSynchronize(s));
  res.modularity        = best_q;
  h.last_louvain_levels = dendrogram.size();
}

}  // namespace

void run_louvain(handle_t& h, graph_t& g, size_t max_level, double resolution, bool /*expensive*/,
                 clustering_result_t& res)
{
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    louvain_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g, max_level, resolution, res);
  });
}

}  // namespace cgx
