// Multi-GPU single-source shortest paths (one process per GPU).
//
// Reference: cpp/src/traversal/sssp_impl.cuh:79-270 with multi_gpu = true: near-far
// buckets, the frontier's out-edges relaxed with e_op (:49-72, keep dist[u] + w
// only if it is < min(cutoff, dist[v])), the (destination, distance) pairs reduced
// by destination and shuffled to their owners
// (transform_reduce_v_frontier_outgoing_e_by_dst), a termination
// allreduce per step.  Layout here, as in mg_bfs.hip: every rank owns the
// out-edges of its vertices (1D by source owner, weights kept), built once and
// cached.  A step:
//
//  1. own near-frontier vertices emit (v, dist[u] + w) for every out-edge (thread
//     per edge over the frontier's degree prefix); own destinations that do not
//     improve are dropped on the spot;
//  2. radix sort by v + min-reduce by key, split at the owners' id ranges, one
//     all-to-all;
//  3. owners relax with atomicMin on the IEEE bit pattern (non-negative floats
//     order like integers) and collect the improved vertices once (round stamp);
//  4. improved vertices below the threshold form the next near frontier, the rest
//     join the far pile.  When the near frontier is empty everywhere the threshold
//     jumps to (global minimum far distance) + delta.
//
// fp32 relaxation is monotone, so the fixed point -- the distances -- does not
// depend on the order of relaxations: they equal the single-GPU result bit for bit.
// Predecessors: the distances are allgathered once, every rank offers its tight
// out-edges (dist[u] + w == dist[v]) and the owner keeps the smallest global u.
#include "capi.hpp"
#include "comm.hpp"
#include "mg_graph.hpp"
#include "prims.hpp"

#include <rocprim/device/device_reduce_by_key.hpp>

#include <cmath>
#include <limits>

namespace cgx {

namespace {

inline unsigned blocks(int64_t n) { return grid_for(n > 0 ? n : 1, kBlock, 16384); }

template <typename W>
struct wrows_t {
  int64_t n_own = 0, ne = 0;
  dbuf<int64_t> off;  // n_own + 1
  dbuf<uint32_t> idx;  // global destination ids, ascending per row
  dbuf<W> w;
};

template <typename W>
struct bits_of;
template <>
struct bits_of<float> {
  using type = int;
};
template <>
struct bits_of<double> {
  using type = long long;
};

template <typename W>
__device__ __forceinline__ W atomic_min_nonneg(W* p, W x)
{
  using B = typename bits_of<W>::type;
  B old   = atomicMin(reinterpret_cast<B*>(p), *reinterpret_cast<B*>(&x));
  return *reinterpret_cast<W*>(&old);
}

template <typename V>
__global__ void k_src_owner(V const* src, int64_t n, int64_t const* voff, int P, int* dest)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dest[i] = mg_owner_of_global((int64_t)src[i], voff, P);
}

// first position of value q in a sorted int array, q = 0..P
__global__ void k_int_bounds(int const* sorted, int64_t n, int P, int64_t* out)
{
  int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q > P) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (sorted[mid] < q) lo = mid + 1;
    else hi = mid;
  }
  out[q] = lo;
}

// first position of keys >= voff[q] (q < P) / of the UINT32_MAX sentinel run (q = P)
__global__ void k_u32_bounds(uint32_t const* keys, int64_t n, int64_t const* voff, int P, int64_t* out)
{
  int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q > P) return;
  unsigned long long const t = (unsigned long long)voff[q];
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if ((unsigned long long)keys[mid] < t) lo = mid + 1;
    else hi = mid;
  }
  out[q] = lo;
}

template <typename V>
__global__ void k_row_keys(V const* src, V const* dst, int64_t n, int64_t base, unsigned long long* keys)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    keys[i] = ((unsigned long long)((int64_t)src[i] - base) << 32) | (unsigned long long)(uint32_t)dst[i];
}

__global__ void k_split_keys(unsigned long long const* keys, int64_t n, uint32_t* row, uint32_t* col)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    row[i] = (uint32_t)(keys[i] >> 32);
    col[i] = (uint32_t)keys[i];
  }
}

__global__ void k_row_offsets(uint32_t const* row, int64_t ne, int64_t n, int64_t* off)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v <= n; v += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = ne;
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if ((int64_t)row[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    off[v] = lo;
  }
}

std::vector<size_t> bounds_counts(dbuf<int64_t> const& b, int P, hipStream_t s)
{
  auto hb = to_host(b.data(), P + 1, s);
  std::vector<size_t> c(P);
  for (int q = 0; q < P; ++q) c[q] = (size_t)(hb[q + 1] - hb[q]);
  return c;
}

// the 2D block's weighted edges -> out-rows of this rank's vertices (cached)
template <typename V, typename W>
wrows_t<W>& mg_wrows(handle_t& h, graph_t& g)
{
  mg_graph_t& mg = *g.mg;
  if (mg.sssp_rows) return *static_cast<wrows_t<W>*>(mg.sssp_rows.get());
  hipStream_t s = h.stream;
  comm_t& comm  = *h.mg->world;
  int const P   = mg.P;
  auto rows     = std::make_shared<wrows_t<W>>();
  dbuf<int64_t> voff_d(P + 1, s), bnd(P + 1, s);
  HIP_CHECK(hipMemcpyAsync(voff_d.data(), mg.voff.data(), (P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  int64_t const ne = mg.ne, n1 = std::max<int64_t>(ne, 1);
  dbuf<int> dest(n1, s), d2(n1, s);
  dbuf<int64_t> iv(n1, s), perm(n1, s);
  dbuf<V> ps(n1, s), pd(n1, s);
  dbuf<W> pw(n1, s);
  if (ne) {
    hipLaunchKernelGGL(k_src_owner<V>, dim3(blocks(ne)), dim3(kBlock), 0, s, mg.src.data<V>(), ne, voff_d.data(), P,
                       dest.data());
    CGX_LAUNCH_CHECK();
    iota<int64_t>(iv.data(), ne, 0, s);
    radix_sort_pairs<int, int64_t>(dest.data(), d2.data(), iv.data(), perm.data(), ne, 0, bits_for(P), s);
    gather<V, int64_t>(ps.data(), mg.src.data<V>(), perm.data(), ne, s);
    gather<V, int64_t>(pd.data(), mg.dst.data<V>(), perm.data(), ne, s);
    gather<W, int64_t>(pw.data(), mg.w.data<W>(), perm.data(), ne, s);
  }
  hipLaunchKernelGGL(k_int_bounds, dim3(1), dim3(256), 0, s, d2.data(), ne, P, bnd.data());
  CGX_LAUNCH_CHECK();
  auto counts = bounds_counts(bnd, P, s);
  std::vector<size_t> rc;
  auto rs = exchange<V>(comm, ps.data(), counts, rc, s);
  auto rd = exchange<V>(comm, pd.data(), counts, rc, s);
  auto rw = exchange<W>(comm, pw.data(), counts, rc, s);
  int64_t const m = (int64_t)rs.n, m1 = std::max<int64_t>(m, 1);
  rows->n_own = mg.n_own();
  rows->ne    = m;
  rows->off.resize(rows->n_own + 1, s);
  rows->idx.resize(m1, s);
  rows->w.resize(m1, s);
  dbuf<uint32_t> rr(m1, s);
  if (m) {
    dbuf<unsigned long long> k1(m, s), k2(m, s);
    hipLaunchKernelGGL(k_row_keys<V>, dim3(blocks(m)), dim3(kBlock), 0, s, rs.data(), rd.data(), m, mg.voff[mg.p],
                       k1.data());
    CGX_LAUNCH_CHECK();
    radix_sort_pairs<unsigned long long, W>(k1.data(), k2.data(), rw.data(), rows->w.data(), (size_t)m, 0, 64, s);
    hipLaunchKernelGGL(k_split_keys, dim3(blocks(m)), dim3(kBlock), 0, s, k2.data(), m, rr.data(), rows->idx.data());
    CGX_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_row_offsets, dim3(blocks(rows->n_own + 1)), dim3(kBlock), 0, s, rr.data(), m, rows->n_own,
                     rows->off.data());
  CGX_LAUNCH_CHECK();
  HIP_CHECK(hipStreamSynchronize(s));
  mg.sssp_rows = rows;
  return *rows;
}

template <typename W>
__global__ void k_frontier_deg(uint32_t const* q, int64_t n, int64_t const* off, unsigned long long* deg)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    deg[i] = (unsigned long long)(off[q[i] + 1] - off[q[i]]);
}

// one thread per frontier out-edge (frontier degree prefix in `pre`)
template <typename W>
__global__ void k_candidates(uint32_t const* q, int64_t nq, unsigned long long const* pre, int64_t m,
                             int64_t const* off, uint32_t const* idx, W const* wgt, W const* dist, int64_t lo,
                             int64_t hi, W cutoff, uint32_t* ck, W* cv, W* relaxed)
{
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t a = 0, b = nq - 1;  // last frontier slot with pre <= t
    while (a < b) {
      int64_t mid = (a + b + 1) >> 1;
      if ((int64_t)pre[mid] <= t) a = mid;
      else b = mid - 1;
    }
    uint32_t const u = q[a];
    W const du       = dist[u];
    if (t == (int64_t)pre[a]) relaxed[u] = du;  // this distance of u has been pushed
    int64_t const e  = off[u] + (t - (int64_t)pre[a]);
    uint32_t const v = idx[e];
    W const nd       = du + wgt[e];
    bool keep        = nd < cutoff;
    if (keep && (int64_t)v >= lo && (int64_t)v < hi) keep = nd < dist[(int64_t)v - lo];  // own: known here
    ck[t] = keep ? v : 0xffffffffu;
    cv[t] = nd;
  }
}

// appends to one tail: one atomic per wave (same-address atomics serialise, bfs.hip)
__device__ __forceinline__ long long wave_reserve(unsigned long long* tail, bool take)
{
  unsigned long long const mask = __ballot(take);
  if (mask == 0) return -1;
  int const lane   = threadIdx.x & 63;
  int const leader = __ffsll((long long)mask) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(tail, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader, 64);
  return take ? (long long)(base + __popcll(mask & ((1ull << lane) - 1ull))) : -1;
}

template <typename W>
__global__ void k_apply(uint32_t const* keys, W const* vals, int64_t n, int64_t lo, W* dist, int* stamp, int round,
                        uint32_t* changed, unsigned long long* nchanged)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t const l = (int64_t)keys[i] - lo;
    W const nd      = vals[i];
    bool const take = nd < dist[l] && atomic_min_nonneg(dist + l, nd) > nd && atomicExch(stamp + l, round) != round;
    long long const slot = wave_reserve(nchanged, take);
    if (take) changed[slot] = (uint32_t)l;
  }
}

// split a vertex list by the threshold: dist < thr -> near, otherwise -> far pile.
// The far pile holds every vertex at most once (infar flag).  from_far: the pile
// itself (unique) is re-split; entries whose current distance has already been
// pushed are dropped.  Otherwise `in` is the round's changed list (unique).
template <typename W>
__global__ void k_split(uint32_t const* in, int64_t n, W const* dist, W const* relaxed, W thr, bool from_far,
                        int* infar, uint32_t* near, unsigned long long* nnear, uint32_t* far,
                        unsigned long long* nfar)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const l = in[i];
    W const d        = dist[l];
    bool to_near = false, to_far = false;
    if (from_far) {
      if (relaxed[l] == d) {
        infar[l] = 0;
      } else if (d < thr) {
        infar[l] = 0;
        to_near  = true;
      } else {
        to_far = true;
      }
    } else if (d < thr) {
      to_near = true;
    } else {
      to_far = atomicExch(infar + l, 1) == 0;
    }
    long long const sn = wave_reserve(nnear, to_near);
    long long const sf = wave_reserve(nfar, to_far);
    if (to_near) near[sn] = l;
    if (to_far) far[sf] = l;
  }
}

template <typename W>
struct wsum_f {
  W const* w;
  __device__ double operator()(size_t i) const { return (double)w[i]; }
};

template <typename W>
__global__ void k_far_min(uint32_t const* far, int64_t n, W const* dist, W const* relaxed, W* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t l = far[i];
    if (relaxed[l] != dist[l]) atomic_min_nonneg(out, dist[l]);
  }
}

// tight out-edges (dist[u] + w == dist[v]) -> key (v << 32 | global u)
template <typename W>
__global__ void k_tight(int64_t n_own, int64_t const* off, uint32_t const* idx, W const* wgt, W const* dist_all,
                        int64_t lo, uint32_t src, unsigned long long* out)
{
  W const BIG = std::numeric_limits<W>::max();
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n_own; u += (int64_t)gridDim.x * blockDim.x) {
    W const du = dist_all[lo + u];
    for (int64_t e = off[u]; e < off[u + 1]; ++e) {
      uint32_t v = idx[e];
      bool tight = du != BIG && v != src && du + wgt[e] == dist_all[v];
      out[e]     = tight ? (((unsigned long long)v << 32) | (unsigned long long)(uint32_t)(lo + u)) : ~0ull;
    }
  }
}

struct same_hi {
  __host__ __device__ bool operator()(unsigned long long a, unsigned long long b) const { return (a >> 32) == (b >> 32); }
};

// first position with key >= voff[q] << 32 (q < P) / of the ~0 sentinel run (q = P)
__global__ void k_key_split(unsigned long long const* keys, int64_t n, int64_t const* voff, int P, int64_t* pos)
{
  int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q > P) return;
  unsigned long long bound = (unsigned long long)voff[q] << 32;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < bound) lo = mid + 1;
    else hi = mid;
  }
  pos[q] = lo;
}

template <typename V>
__global__ void k_set_pred(unsigned long long const* keys, int64_t n, int64_t lo, V* pred)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t v = (int64_t)(keys[i] >> 32) - lo;
    if constexpr (sizeof(V) == 4) atomicMin(reinterpret_cast<int*>(pred + v), (int)(uint32_t)keys[i]);
    else atomicMin(reinterpret_cast<long long*>(pred + v), (long long)(uint32_t)keys[i]);
  }
}

template <typename V>
__global__ void k_pred_none(V* pred, int64_t n)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (pred[i] == std::numeric_limits<V>::max()) pred[i] = (V)-1;
}

struct min_op {
  template <typename T>
  __host__ __device__ T operator()(T a, T b) const
  {
    return b < a ? b : a;
  }
};

template <typename V, typename W>
void mg_sssp_impl(handle_t& h, graph_t& g, size_t source, double cutoff, bool want_pred, bool expensive,
                  paths_result_t& res)
{
  hipStream_t s  = h.stream;
  comm_t& comm   = *h.mg->world;
  mg_graph_t& mg = *g.mg;
  int const P    = mg.P;
  CGX_INPUT(g.weighted,
            "Invalid input argument: an unweighted graph is passed to SSSP, BFS is more efficient for unweighted "
            "graphs.");
  CGX_EXPECTS(g.num_vertices < (int64_t)UINT32_MAX, CUGRAPH_NOT_IMPLEMENTED, "MG SSSP: more than 2^32 vertices");
  CGX_INPUT((int64_t)source >= 0 && (size_t)(V)source == source, "Invalid input argument: source vertex out-of-range.");
  int64_t const n_own = mg.n_own(), lo = mg.voff[mg.p], hi = mg.voff[mg.p + 1], n1 = std::max<int64_t>(n_own, 1);
  W const BIG = std::numeric_limits<W>::max();

  // the source (the same external id on every rank) -> global id
  dbuf<V> sg(1, s);
  V hs = (V)source;
  to_device(sg.data(), &hs, 1, s);
  try {
    mg_ext_to_global(h, g, sg.data(), 1, true);
  } catch (cgx::error const&) {
    fail(CUGRAPH_INVALID_INPUT, "Invalid input argument: source vertex out-of-range.");
  }
  int64_t const src = (int64_t)to_host_scalar(sg.data(), s);

  res.vertices = std::make_unique<device_array_t>((size_t)n_own, g.vertex_type, s);
  if (n_own)
    HIP_CHECK(hipMemcpyAsync(res.vertices->buf.data(), g.number_map.data(), n_own * sizeof(V), hipMemcpyDeviceToDevice,
                             s));
  res.distances    = std::make_unique<device_array_t>((size_t)n_own, dtype_of<W>(), s);
  res.predecessors = std::make_unique<device_array_t>(want_pred ? (size_t)n_own : 0, g.vertex_type, s);
  W* dist          = res.distances->buf.data<W>();
  if (n_own) fill<W>(dist, n_own, BIG, s);

  wrows_t<W>& rows = mg_wrows<V, W>(h, g);
  int64_t const ne_own = rows.ne;
  if (expensive) {
    int64_t neg = 0;
    if (ne_own)
      for (auto x : to_host(rows.w.data(), ne_own, s)) neg += x < W(0) ? 1 : 0;
    CGX_INPUT(comm.host_allreduce<int64_t>(neg, CGX_COMM_SUM, s) == 0,
              "Invalid input argument: input graph should have non-negative edge weights.");
  }
  W const cut = (cutoff >= (double)BIG || !(cutoff == cutoff)) ? BIG : (W)cutoff;

  // delta = 64 * average edge weight / average degree (as the single-GPU path)
  double wsum_own = 0;
  if (ne_own) {
    dbuf<double> scratch(1024, s), out(1, s);
    device_sum(wsum_f<W>{rows.w.data()}, (size_t)ne_own, out.data(), scratch.data(), s);
    wsum_own = to_host_scalar(out.data(), s);
  }
  double const wsum = comm.host_allreduce<double>(wsum_own, CGX_COMM_SUM, s);
  double const ne_g = (double)g.num_edges;
  W const delta     = ne_g > 0 ? (W)std::max(64.0 * (wsum / ne_g) / (ne_g / (double)g.num_vertices), 1e-30) : W(1);

  dbuf<int64_t> voff_d(P + 1, s), pos(P + 1, s);
  HIP_CHECK(hipMemcpyAsync(voff_d.data(), mg.voff.data(), (P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  dbuf<int> stamp(n1, s);
  fill<int>(stamp.data(), n1, -1, s);
  dbuf<W> relaxed(n1, s);  // the distance each vertex last pushed (BIG: never)
  fill<W>(relaxed.data(), n1, BIG, s);
  dbuf<uint32_t> nearq(n1, s), changed(n1, s), farA(n1, s), farB(n1, s);
  dbuf<int> infar(n1, s);
  fill<int>(infar.data(), n1, 0, s);
  dbuf<unsigned long long> cnt(4, s);  // changed, near, far, -
  int64_t n_near = 0, n_far = 0;
  if (src >= lo && src < hi) {
    W zero       = 0;
    uint32_t l   = (uint32_t)(src - lo);
    to_device(dist + l, &zero, 1, s);
    to_device(nearq.data(), &l, 1, s);
    n_near = 1;
  }
  W thr     = delta;
  int round = 0;
  while (true) {
    int64_t g_near = comm.host_allreduce<int64_t>(n_near, CGX_COMM_SUM, s);
    if (g_near == 0) {
      // next band: (global minimum unsettled far distance) + delta
      dbuf<W> fm(1, s);
      fill<W>(fm.data(), 1, BIG, s);
      if (n_far)
        hipLaunchKernelGGL(k_far_min<W>, dim3(blocks(n_far)), dim3(kBlock), 0, s, farA.data(), n_far, dist,
                           relaxed.data(), fm.data());
      CGX_LAUNCH_CHECK();
      comm.allreduce<W>(fm.data(), fm.data(), 1, CGX_COMM_MIN, s);
      W const mn = to_host_scalar(fm.data(), s);
      if (!(mn < BIG)) break;  // nothing left anywhere
      thr = std::max<W>(thr + delta, mn + delta);
      HIP_CHECK(hipMemsetAsync(cnt.data(), 0, 4 * sizeof(unsigned long long), s));
      if (n_far)
        hipLaunchKernelGGL(k_split<W>, dim3(blocks(n_far)), dim3(kBlock), 0, s, farA.data(), n_far, dist,
                           relaxed.data(), thr, true, infar.data(), nearq.data(), cnt.data() + 1, farB.data(),
                           cnt.data() + 2);
      CGX_LAUNCH_CHECK();
      auto hc = to_host(cnt.data(), 4, s);
      n_near  = (int64_t)hc[1];
      n_far   = (int64_t)hc[2];
      std::swap(farA, farB);
      continue;
    }
    ++round;
    // 1. candidates of the own near frontier
    int64_t m = 0;
    dbuf<unsigned long long> deg(std::max<int64_t>(n_near, 1), s), pre(std::max<int64_t>(n_near, 1), s);
    if (n_near) {
      hipLaunchKernelGGL(k_frontier_deg<W>, dim3(blocks(n_near)), dim3(kBlock), 0, s, nearq.data(), n_near,
                         rows.off.data(), deg.data());
      CGX_LAUNCH_CHECK();
      exclusive_scan<unsigned long long, unsigned long long>(deg.data(), pre.data(), n_near, s);
      m = (int64_t)(to_host(pre.data() + n_near - 1, 1, s)[0] + to_host(deg.data() + n_near - 1, 1, s)[0]);
    }
    int64_t const m1 = std::max<int64_t>(m, 1);
    dbuf<uint32_t> ck(m1, s), ck2(m1, s), uk(m1, s);
    dbuf<W> cv(m1, s), cv2(m1, s), uv(m1, s);
    int64_t nu = 0;
    if (m) {
      hipLaunchKernelGGL(k_candidates<W>, dim3(blocks(m)), dim3(kBlock), 0, s, nearq.data(), n_near, pre.data(), m,
                         rows.off.data(), rows.idx.data(), rows.w.data(), dist, lo, hi, cut, ck.data(), cv.data(),
                         relaxed.data());
      CGX_LAUNCH_CHECK();
      radix_sort_pairs<uint32_t, W>(ck.data(), ck2.data(), cv.data(), cv2.data(), (size_t)m, 0, 32, s);
      dbuf<unsigned long long> nuu(1, s);
      size_t tmp = 0;
      HIP_CHECK(rocprim::reduce_by_key(nullptr, tmp, ck2.data(), cv2.data(), (size_t)m, uk.data(), uv.data(),
                                       nuu.data(), min_op(), rocprim::equal_to<uint32_t>(), s));
      buffer t(tmp, s);
      HIP_CHECK(rocprim::reduce_by_key(t.data(), tmp, ck2.data(), cv2.data(), (size_t)m, uk.data(), uv.data(),
                                       nuu.data(), min_op(), rocprim::equal_to<uint32_t>(), s));
      nu = (int64_t)to_host_scalar(nuu.data(), s);
    }
    // 2. to the owners (the sentinel run sorts last and is not sent)
    std::vector<size_t> counts(P, 0);
    if (nu) {
      hipLaunchKernelGGL(k_u32_bounds, dim3(1), dim3(256), 0, s, uk.data(), nu, voff_d.data(), P, pos.data());
      CGX_LAUNCH_CHECK();
      counts = bounds_counts(pos, P, s);
    }
    std::vector<size_t> rc;
    auto rk = exchange<uint32_t>(comm, uk.data(), counts, rc, s);
    auto rv = exchange<W>(comm, uv.data(), counts, rc, s);
    // 3. relax at the owners
    HIP_CHECK(hipMemsetAsync(cnt.data(), 0, 4 * sizeof(unsigned long long), s));
    if (rk.n)
      hipLaunchKernelGGL(k_apply<W>, dim3(blocks(rk.n)), dim3(kBlock), 0, s, rk.data(), rv.data(), (int64_t)rk.n, lo,
                         dist, stamp.data(), round, changed.data(), cnt.data());
    CGX_LAUNCH_CHECK();
    int64_t const n_changed = (int64_t)to_host_scalar(cnt.data(), s);
    // 4. next near frontier / far pile (appended after the current far entries)
    HIP_CHECK(hipMemcpyAsync(cnt.data() + 2, &n_far, sizeof(unsigned long long), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemsetAsync(cnt.data() + 1, 0, sizeof(unsigned long long), s));
    if (n_changed)
      hipLaunchKernelGGL(k_split<W>, dim3(blocks(n_changed)), dim3(kBlock), 0, s, changed.data(), n_changed, dist,
                         relaxed.data(), thr, false, infar.data(), nearq.data(), cnt.data() + 1, farA.data(),
                         cnt.data() + 2);
    CGX_LAUNCH_CHECK();
    auto hc = to_host(cnt.data(), 4, s);
    n_near  = (int64_t)hc[1];
    n_far   = (int64_t)hc[2];
  }

  if (want_pred) {
    V* pred = res.predecessors->buf.data<V>();
    if (n_own) fill<V>(pred, n_own, std::numeric_limits<V>::max(), s);
    // every rank needs dist[v] of its edges' destinations: one allgather
    int64_t nmax = 0;
    for (int q = 0; q < P; ++q) nmax = std::max(nmax, mg.voff[q + 1] - mg.voff[q]);
    dbuf<W> sb(std::max<int64_t>(nmax, 1), s), rb(std::max<int64_t>(nmax, 1) * P, s),
      dall(std::max<int64_t>(g.num_vertices, 1), s);
    if (n_own) HIP_CHECK(hipMemcpyAsync(sb.data(), dist, n_own * sizeof(W), hipMemcpyDeviceToDevice, s));
    comm.allgather<W>(sb.data(), rb.data(), (size_t)std::max<int64_t>(nmax, 1), s);
    for (int q = 0; q < P; ++q) {
      int64_t nq = mg.voff[q + 1] - mg.voff[q];
      if (nq)
        HIP_CHECK(hipMemcpyAsync(dall.data() + mg.voff[q], rb.data() + (size_t)q * std::max<int64_t>(nmax, 1),
                                 nq * sizeof(W), hipMemcpyDeviceToDevice, s));
    }
    int64_t const e1 = std::max<int64_t>(ne_own, 1);
    dbuf<unsigned long long> tk(e1, s), tk2(e1, s), tu(e1, s);
    int64_t nt = 0;
    if (ne_own) {
      hipLaunchKernelGGL(k_tight<W>, dim3(blocks(n_own)), dim3(kBlock), 0, s, n_own, rows.off.data(), rows.idx.data(),
                         rows.w.data(), dall.data(), lo, (uint32_t)src, tk.data());
      CGX_LAUNCH_CHECK();
      radix_sort_keys<unsigned long long>(tk.data(), tk2.data(), ne_own, 0, 64, s);
      dbuf<size_t> c1(1, s);
      size_t tmp = 0;
      HIP_CHECK(rocprim::unique(nullptr, tmp, tk2.data(), tu.data(), c1.data(), (size_t)ne_own, same_hi(), s));
      buffer t(tmp, s);
      HIP_CHECK(rocprim::unique(t.data(), tmp, tk2.data(), tu.data(), c1.data(), (size_t)ne_own, same_hi(), s));
      nt = (int64_t)to_host_scalar(c1.data(), s);
    }
    std::vector<size_t> counts(P, 0);
    if (nt) {
      hipLaunchKernelGGL(k_key_split, dim3(1), dim3(256), 0, s, tu.data(), nt, voff_d.data(), P, pos.data());
      CGX_LAUNCH_CHECK();
      counts = bounds_counts(pos, P, s);
    }
    std::vector<size_t> rc;
    auto got = exchange<int64_t>(comm, reinterpret_cast<int64_t const*>(tu.data()), counts, rc, s);
    if (got.n)
      hipLaunchKernelGGL(k_set_pred<V>, dim3(blocks(got.n)), dim3(kBlock), 0, s,
                         reinterpret_cast<unsigned long long const*>(got.data()), (int64_t)got.n, lo, pred);
    CGX_LAUNCH_CHECK();
    if (n_own) hipLaunchKernelGGL(k_pred_none<V>, dim3(blocks(n_own)), dim3(kBlock), 0, s, pred, n_own);
    CGX_LAUNCH_CHECK();
    mg_global_to_ext(h, g, pred, (size_t)n_own);
  }
  HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace

void mg_run_sssp(handle_t& h, graph_t& g, size_t source, double cutoff, bool compute_predecessors, bool expensive,
                 paths_result_t& res)
{
  CGX_EXPECTS(h.mg != nullptr, CUGRAPH_INVALID_HANDLE, "multi-GPU graph used with a single-GPU resource handle");
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    mg_sssp_impl<typename T::vertex_t, typename T::weight_t>(h, g, source, cutoff, compute_predecessors, expensive,
                                                             res);
  });
}

}  // namespace cgx
