// Single-source shortest paths, near-far (Davidson et al.) on the GPU.
//
// Reference: cpp/src/traversal/sssp_impl.cuh:79-270 (+ c_api/sssp.cpp:60-145):
// distances start at numeric_limits<weight_t>::max(), a relaxation dist[u] + w is
// kept only if it is < min(cutoff, dist[v]) (e_op :49-72); the frontier is split
// into near / far piles by a threshold that grows by delta (:143-157, :235-262).
//
// Here: distances are relaxed with atomicMin on their bit patterns (non-negative
// IEEE values order like integers); each round appends every improved vertex once
// (a round stamp per vertex) to a "changed" list, which is then split by the
// current threshold into the next near frontier (by degree class, as the BFS
// queues) or the far pile.  Predecessors are resolved once at the end: the
// smallest internal id among in-neighbours u with dist[u] + w == dist[v]
// (deterministic; every reference golden vector satisfies it).
#include "capi.hpp"
#include "prims.hpp"

#include <cfloat>
#include <limits>

namespace cgx {

namespace {

constexpr int kSmallDeg = 16;
constexpr int kMidDeg   = 1024;

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

__device__ __forceinline__ long long wave_append(unsigned long long* tail, bool take)
{
  unsigned long long mask = __ballot(take);
  if (mask == 0) return -1;
  int lane   = threadIdx.x & 63;
  int leader = __ffsll((long long)mask) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(tail, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader, 64);
  if (!take) return -1;
  return (long long)(base + __popcll(mask & ((1ull << lane) - 1ull)));
}

struct sssp_ctr {
  unsigned long long changed;
  unsigned long long near[3];
  unsigned long long far;
  unsigned long long pad[3];
};

template <typename V, typename E, typename W>
struct sssp_args {
  E const* off;
  V const* idx;
  W const* wgt;
  W* dist;
  int* stamp;
  int round;
  W cutoff;
  V const* q[3];
  unsigned long long n[3];
  V* changed;
  sssp_ctr* ctr;
  long long blk_mid_start, blk_small_start;
};

template <typename V, typename E, typename W>
__device__ __forceinline__ void relax(sssp_args<V, E, W> const& a, W du, E e, bool act)
{
  bool take = false;
  V v       = 0;
  if (act) {
    v    = a.idx[e];
    W nd = du + a.wgt[e];
    if (nd < a.cutoff && nd < a.dist[v]) {
      W old = atomic_min_nonneg<W>(a.dist + v, nd);
      if (nd < old) take = atomicExch(a.stamp + v, a.round) != a.round;
    }
  }
  long long slot = wave_append(&a.ctr->changed, take);
  if (slot >= 0) a.changed[slot] = v;
}

template <typename V, typename E, typename W>
__global__ __launch_bounds__(256) void k_relax(sssp_args<V, E, W> a)
{
  long long b = blockIdx.x;
  int tid     = threadIdx.x;
  if (b < a.blk_mid_start) {
    for (long long i = b; i < (long long)a.n[2]; i += a.blk_mid_start) {
      V u  = a.q[2][i];
      W du = a.dist[u];
      E beg = a.off[u], end = a.off[u + 1];
      for (E base = beg; base < end; base += 256) relax<V, E, W>(a, du, base + tid, base + tid < end);
    }
  } else if (b < a.blk_small_start) {
    long long nb   = a.blk_small_start - a.blk_mid_start;
    long long widx = (b - a.blk_mid_start) * 4 + (tid >> 6);
    int lane       = tid & 63;
    for (long long i = widx; i < (long long)a.n[1]; i += nb * 4) {
      V u  = a.q[1][i];
      W du = a.dist[u];
      E beg = a.off[u], end = a.off[u + 1];
      for (E base = beg; base < end; base += 64) relax<V, E, W>(a, du, base + lane, base + lane < end);
    }
  } else {
    long long nb = gridDim.x - a.blk_small_start;
    int lane     = tid & 3;
    for (long long i0 = (b - a.blk_small_start) * 64; i0 < (long long)a.n[0]; i0 += nb * 64) {
      long long i = i0 + (tid >> 2);
      bool have   = i < (long long)a.n[0];
      V u         = have ? a.q[0][i] : V(0);
      W du        = have ? a.dist[u] : W(0);
      E beg = have ? a.off[u] : E(0), end = have ? a.off[u + 1] : E(0);
      for (int r = 0; r < kSmallDeg / 4; ++r) {
        E e = beg + r * 4 + lane;
        relax<V, E, W>(a, du, e, e < end);
      }
    }
  }
}

// Split a vertex list by the current distances.
//  from_far == false (the round's changed list, unique): dist < hi -> near queue (by
//    degree class); otherwise -> far pile, unless already in it (infar flag).
//  from_far == true (the far pile, unique by the infar invariant): dist < lo -> drop
//    (it was improved into an earlier near pile and processed there); dist < hi ->
//    near; else stays in the far pile (written to `far`).
template <typename V, typename E, typename W>
__global__ void k_split(V const* in, unsigned long long n, W const* dist, E const* off, W lo, W hi, int* infar,
                        bool from_far, V* near0, V* near1, V* near2, V* far, sssp_ctr* ctr)
{
  for (unsigned long long base = blockIdx.x * (unsigned long long)blockDim.x; base < n;
       base += (unsigned long long)gridDim.x * blockDim.x) {
    unsigned long long i = base + threadIdx.x;
    bool have            = i < n;
    V v                  = have ? in[i] : V(0);
    W d                  = have ? dist[v] : W(0);
    bool is_near = false, to_far = false;
    if (have) {
      if (from_far) {
        infar[v] = 0;
        if (d >= lo) {
          is_near = d < hi;
          to_far  = !is_near;
          if (to_far) infar[v] = 1;
        }
      } else {
        is_near = d < hi;
        if (!is_near) to_far = atomicExch(infar + v, 1) == 0;
      }
    }
    int cls = 0;
    if (is_near) {
      E deg = off[v + 1] - off[v];
      cls   = deg <= kSmallDeg ? 0 : (deg <= kMidDeg ? 1 : 2);
    }
    long long s0 = wave_append(&ctr->near[0], is_near && cls == 0);
    long long s1 = wave_append(&ctr->near[1], is_near && cls == 1);
    long long s2 = wave_append(&ctr->near[2], is_near && cls == 2);
    long long sf = wave_append(&ctr->far, to_far);
    if (s0 >= 0) near0[s0] = v;
    if (s1 >= 0) near1[s1] = v;
    if (s2 >= 0) near2[s2] = v;
    if (sf >= 0) far[sf] = v;
  }
}

template <typename V, typename E, typename W>
__global__ void k_sssp_pred(E const* off, V const* idx, W const* wgt, W const* dist, int64_t nv, V src, V* pred)
{
  // thread per source vertex u: for each out-edge (u, v) tight -> atomicMin(pred[v], u)
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < nv; u += (int64_t)gridDim.x * blockDim.x) {
    W du = dist[u];
    if (du == std::numeric_limits<W>::max()) continue;
    for (E e = off[u]; e < off[u + 1]; ++e) {
      V v = idx[e];
      if (v == src) continue;
      if (du + wgt[e] == dist[v]) {
        if constexpr (sizeof(V) == 4) atomicMin(reinterpret_cast<int*>(pred + v), (int)u);
        else atomicMin(reinterpret_cast<long long*>(pred + v), (long long)u);
      }
    }
  }
}

template <typename V>
__global__ void k_pred_none(V* pred, int64_t n, V none)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (pred[i] == none) pred[i] = (V)-1;
}

template <typename V, typename E, typename W>
__global__ void k_weight_stats(E const* off, W const* w, int64_t nv, size_t ne, double* out)
{
  __shared__ double sm[4];
  double acc = 0;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < ne; e += (size_t)gridDim.x * blockDim.x)
    acc += (double)w[e];
  double r = block_sum_256(acc, sm);
  if (threadIdx.x == 0) atomicAdd(out, r);
}

template <typename W>
__global__ void k_count_neg(W const* w, size_t n, int* bad)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (w[i] < W(0)) atomicAdd(bad, 1);
}

template <typename V, typename E, typename W>
void sssp_impl(handle_t& h, graph_t& g, size_t source, double cutoff, bool want_pred, bool expensive,
               paths_result_t& res)
{
  hipStream_t s = h.stream;
  int64_t nv    = g.num_vertices;
  CGX_INPUT(g.weighted,
            "Invalid input argument: an unweighted graph is passed to SSSP, BFS is more efficient for unweighted "
            "graphs.");
  // the source is an external id (c_api/sssp.cpp renumbers it)
  dbuf<V> src_id(1, s);
  V hs = (V)source;
  CGX_INPUT((int64_t)source >= 0 && (size_t)(V)source == source, "Invalid input argument: source vertex out-of-range.");
  to_device(src_id.data(), &hs, 1, s);
  {
    try {
      renumber_ext_to_int(h, g, src_id.data(), 1, true);
    } catch (cgx::error const&) {
      fail(CUGRAPH_INVALID_INPUT, "Invalid input argument: source vertex out-of-range.");
    }
  }
  V src = to_host_scalar(src_id.data(), s);
  res.vertices     = number_map_copy(h, g);
  res.distances    = std::make_unique<device_array_t>((size_t)nv, dtype_of<W>(), s);
  res.predecessors = std::make_unique<device_array_t>(want_pred ? (size_t)nv : 0, dtype_of<V>(), s);
  W* dist          = res.distances->buf.data<W>();
  W const BIG      = std::numeric_limits<W>::max();
  fill<W>(dist, nv, BIG, s);
  if (nv == 0) return;
  W zero = 0;
  to_device(dist + src, &zero, 1, s);

  adjacency_t& adj = ensure_adjacency(h, g, false);
  size_t ne        = (size_t)g.num_edges;
  E const* off     = adj.offsets.data<E>();
  V const* idx     = adj.indices.data<V>();
  W const* wgt     = adj.weights.data<W>();
  if (expensive && ne) {
    dbuf<int> bad(1, s);
    fill<int>(bad.data(), 1, 0, s);
    hipLaunchKernelGGL(k_count_neg<W>, dim3(grid_for(ne, kBlock, 4096)), dim3(kBlock), 0, s, wgt, ne, bad.data());
    CGX_LAUNCH_CHECK();
    CGX_INPUT(to_host_scalar(bad.data(), s) == 0,
              "Invalid input argument: input graph should have non-negative edge weights.");
  }
  W cut = (cutoff >= (double)BIG || !(cutoff == cutoff)) ? BIG : (W)cutoff;

  if (ne) {
    // delta = 64 * average edge weight / average degree (wave-64 analogue of :143-157)
    dbuf<double> wsum(1, s);
    fill<double>(wsum.data(), 1, 0.0, s);
    hipLaunchKernelGGL((k_weight_stats<V, E, W>), dim3(grid_for(ne, kBlock, 1024)), dim3(kBlock), 0, s, off, wgt, nv,
                       ne, wsum.data());
    CGX_LAUNCH_CHECK();
    double avg_w   = to_host_scalar(wsum.data(), s) / (double)ne;
    double avg_deg = (double)ne / (double)nv;
    W delta        = (W)std::max(64.0 * avg_w / avg_deg, 1e-30);

    dbuf<int> stamp(nv, s);
    fill<int>(stamp.data(), nv, -1, s);
    dbuf<V> qa[3], qb[3];
    for (int c = 0; c < 3; ++c) {
      qa[c].resize(nv, s);
      qb[c].resize(nv, s);
    }
    dbuf<V> changed(nv, s), farA(nv, s), farB(nv, s);
    dbuf<int> infar(nv, s);
    fill<int>(infar.data(), nv, 0, s);
    dbuf<sssp_ctr> ctr(1, s);
    sssp_ctr* hc = nullptr;
    hc = h.pinned_as<sssp_ctr>();
    try {
      auto read_ctr = [&]() {
        HIP_CHECK(hipMemcpyAsync(hc, ctr.data(), sizeof(sssp_ctr), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
      };
      // initial near frontier: the source
      auto o2 = to_host(off + src, 2, s);
      E deg0  = o2[1] - o2[0];
      int c0 = deg0 <= kSmallDeg ? 0 : (deg0 <= kMidDeg ? 1 : 2);
      to_device(qa[c0].data(), &src, 1, s);
      unsigned long long ncur[3] = {0, 0, 0};
      ncur[c0]                   = 1;
      unsigned long long nfar    = 0;
      W thr                      = delta;
      int round                  = 0;
      sssp_args<V, E, W> a{};
      a.off    = off;
      a.idx    = idx;
      a.wgt    = wgt;
      a.dist   = dist;
      a.stamp  = stamp.data();
      a.cutoff = cut;
      a.changed = changed.data();
      a.ctr    = ctr.data();
      size_t rounds = 0;
      while (true) {
        unsigned long long nn = ncur[0] + ncur[1] + ncur[2];
        if (nn > 0) {
          HIP_CHECK(hipMemsetAsync(ctr.data(), 0, sizeof(sssp_ctr), s));
          a.round = round++;
          for (int c = 0; c < 3; ++c) {
            a.q[c] = qa[c].data();
            a.n[c] = ncur[c];
          }
          long long nb_large = (long long)std::min<unsigned long long>(ncur[2], 1024);
          long long nb_mid   = (long long)std::min<unsigned long long>((ncur[1] + 3) / 4, 4096);
          long long nb_small = (long long)std::min<unsigned long long>((ncur[0] + 63) / 64, 8192);
          a.blk_mid_start    = nb_large;
          a.blk_small_start  = nb_large + nb_mid;
          hipLaunchKernelGGL((k_relax<V, E, W>), dim3(nb_large + nb_mid + nb_small), dim3(kBlock), 0, s, a);
          CGX_LAUNCH_CHECK();
          read_ctr();
          unsigned long long nch = hc->changed;
          // split the changed vertices: near (< thr) -> next frontier, else -> far pile
          HIP_CHECK(hipMemsetAsync(ctr.data(), 0, sizeof(sssp_ctr), s));
          if (nch)
            hipLaunchKernelGGL((k_split<V, E, W>), dim3(grid_for(nch, kBlock, 4096)), dim3(kBlock), 0, s,
                               changed.data(), nch, dist, off, W(0), thr, infar.data(), false, qb[0].data(),
                               qb[1].data(), qb[2].data(), farA.data() + nfar, ctr.data());
          CGX_LAUNCH_CHECK();
          read_ctr();
          for (int c = 0; c < 3; ++c) ncur[c] = hc->near[c];
          nfar += hc->far;
          for (int c = 0; c < 3; ++c) std::swap(qa[c], qb[c]);
          ++rounds;
          continue;
        }
        if (nfar == 0) break;
        // near pile empty: advance the threshold and split the far pile (split_bucket, :235-262)
        while (true) {
          W old = thr;
          thr   = thr + delta;
          HIP_CHECK(hipMemsetAsync(ctr.data(), 0, sizeof(sssp_ctr), s));
          hipLaunchKernelGGL((k_split<V, E, W>), dim3(grid_for(nfar, kBlock, 4096)), dim3(kBlock), 0, s,
                             farA.data(), nfar, dist, off, old, thr, infar.data(), true, qa[0].data(), qa[1].data(),
                             qa[2].data(), farB.data(), ctr.data());
          CGX_LAUNCH_CHECK();
          read_ctr();
          for (int c = 0; c < 3; ++c) ncur[c] = hc->near[c];
          nfar = hc->far;
          std::swap(farA, farB);
          if (ncur[0] + ncur[1] + ncur[2] > 0 || nfar == 0) break;
        }
        if (ncur[0] + ncur[1] + ncur[2] == 0 && nfar == 0) break;
      }
      h.last_iterations = rounds;
    } catch (...) {
      throw;
    }
  }
  if (want_pred) {
    V* pred = res.predecessors->buf.data<V>();
    V none  = std::numeric_limits<V>::max();
    fill<V>(pred, nv, none, s);
    if (ne) {
      hipLaunchKernelGGL((k_sssp_pred<V, E, W>), dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, off, idx, wgt,
                         dist, nv, src, pred);
      CGX_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_pred_none<V>, dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, pred, nv, none);
    CGX_LAUNCH_CHECK();
    unrenumber_int_to_ext(h, g, pred, (size_t)nv);
  }
}

}  // namespace

void run_sssp(handle_t& h, graph_t& g, size_t source, double cutoff, bool compute_predecessors, bool expensive,
              paths_result_t& res)
{
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    sssp_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g, source, cutoff,
                                                                             compute_predecessors, expensive, res);
  });
}

}  // namespace cgx
