// Graph construction on the GPU: edge list -> (renumbered) compressed adjacency.
//
// Behaviour follows the reference SG path
//   cpp/src/c_api/graph_sg.cpp:231-330 -> create_graph_from_edgelist_impl.cuh:557-776
//   renumber_edgelist_impl.cuh:95-452 (vertex set = sorted unique endpoints, ordered by
//   DESCENDING major degree, stable so ties keep ascending external id)
//   structure/detail/structure_utils.cuh:162-232 (compress + sorted adjacency lists)
// but is implemented as two rocPRIM radix sorts over 64-bit (major << b | minor)
// keys instead of Thrust sort/reduce_by_key chains.
#include "capi.hpp"
#include "prims.hpp"
#include "schedule.hpp"

#include <algorithm>
#include <cstring>

namespace cgx {

namespace {

// ---------------------------------------------------------------- kernels
template <typename V>
__global__ void k_dense_by_table(V* ids, size_t n, int64_t const* table, int64_t lo)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    ids[i] = static_cast<V>(table[(int64_t)ids[i] - lo]);
}

template <typename V>
__global__ void k_table_fill(int64_t* table, V const* verts, size_t nv, int64_t lo)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x)
    table[(int64_t)verts[i] - lo] = (int64_t)i;
}

// lower_bound of each id in a sorted array; writes the position (or -1 when absent)
template <typename V>
__global__ void k_dense_by_search(V* ids, size_t n, V const* sorted, size_t nv, int* missing)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    V x       = ids[i];
    size_t lo = 0, hi = nv;
    while (lo < hi) {
      size_t mid = (lo + hi) >> 1;
      if (sorted[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    if (lo < nv && sorted[lo] == x) ids[i] = static_cast<V>(lo);
    else {
      ids[i] = static_cast<V>(-1);
      if (missing) atomicAdd(missing, 1);
    }
  }
}

// offsets[v] = first i with sorted[i] >= v (v in [0, nv]): the CSR offsets of a
// sorted major array, i.e. degrees as run lengths -- no per-edge atomics (hub ids
// made same-address atomicAdd counting the graph build's hot spot)
template <typename V, typename E>
__global__ void k_lower_bounds(V const* sorted, size_t n, int64_t nv, E* out)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v <= nv; v += (int64_t)gridDim.x * blockDim.x) {
    size_t lo = 0, hi = n;
    while (lo < hi) {
      size_t mid = (lo + hi) >> 1;
      if ((int64_t)sorted[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    out[v] = static_cast<E>(lo);
  }
}

template <typename V>
__global__ void k_make_key(V const* major, V const* minor, size_t n, int b, uint64_t* key)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    key[i] = ((uint64_t)major[i] << b) | (uint64_t)minor[i];
}

template <typename V>
__global__ void k_split_key(uint64_t const* key, size_t n, int b, V* major, V* minor)
{
  uint64_t mask = (b >= 64) ? ~0ull : ((1ull << b) - 1);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t k = key[i];
    if (major) major[i] = static_cast<V>(k >> b);
    minor[i] = static_cast<V>(k & mask);
  }
}

template <typename V>
__global__ void k_relabel(V* ids, size_t n, V const* new_of)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    ids[i] = new_of[ids[i]];
}

template <typename V>
__global__ void k_inverse_perm(V const* order, size_t n, V* inv)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    inv[order[i]] = static_cast<V>(i);
}

// the major id of every edge: last row with offsets[row] <= e (one thread per
// edge, so a hub row is not one thread's loop)
template <typename V, typename E>
__global__ void k_expand_majors(E const* offsets, int64_t nv, int64_t ne, V* majors)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nv - 1;
    while (lo < hi) {
      int64_t mid = (lo + hi + 1) >> 1;
      if ((int64_t)offsets[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    majors[e] = static_cast<V>(lo);
  }
}

template <typename E, typename D>
__global__ void k_degrees(E const* offsets, int64_t nv, D* deg)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x)
    deg[v] = static_cast<D>(offsets[v + 1] - offsets[v]);
}

// is deg non-increasing?  flag set to 1 on any violation
template <typename E>
__global__ void k_check_sorted_desc(E const* offsets, int64_t nv, int* bad)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v + 1 < nv; v += (int64_t)gridDim.x * blockDim.x) {
    E d0 = offsets[v + 1] - offsets[v];
    E d1 = offsets[v + 2] - offsets[v + 1];
    if (d1 > d0) *bad = 1;
  }
}

// bin starts: for each threshold t, first position whose degree < t (degrees non-increasing in order)
template <typename V, typename E>
__global__ void k_bin_starts(E const* offsets, V const* order, int64_t nv, int64_t* out)
{
  int b = threadIdx.x;
  if (b >= kSchedBins) return;
  int64_t t  = kBinLo[b];
  int64_t lo = 0, hi = nv;
  while (lo < hi) {  // first position with degree < t
    int64_t mid = (lo + hi) >> 1;
    int64_t v   = order ? (int64_t)order[mid] : mid;
    int64_t d   = (int64_t)(offsets[v + 1] - offsets[v]);
    if (d >= t) lo = mid + 1;
    else hi = mid;
  }
  out[b] = lo;  // end of bin b (exclusive) == start of bin b+1
}

// ---- per-row weight sums over a CSR (compute_out_weight_sums, pagerank_impl.cuh:158-164)
// Edge tiles, not rows, are the unit of work, so a hub row (RMAT-24: 406K edges)
// is spread over ~200 blocks instead of one thread's loop (68.8 ms per call as a
// thread-per-row kernel).  Tile b = edges [bT, bT + T), T = 4096:
//  * the rows whose first edge lies in the tile (rows [lbs[b], lbs[b + 1]), found by
//    one binary search per tile beforehand) are summed from the tile's weights in
//    LDS, one thread per row, in edge order;
//  * the row that runs past the tile end leaves its in-tile partial in tail[b], and
//    the part of a row that started in an earlier tile its partial in head[b];
//  * k_row_sums_spill then adds, for each such row, tail[first tile] + head[...]
//    in tile order.
// fp64 sums in a fixed order: deterministic, rounded once to weight_t.
constexpr int kRsTile    = 4096;  // edges per tile (16 per thread)
constexpr int kRsThreads = 256;

template <typename E>
__global__ void k_row_sum_tile_rows(E const* off, int64_t nv, int64_t ntiles, int64_t* lbs)
{
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b <= ntiles; b += (int64_t)gridDim.x * blockDim.x) {
    if (b == ntiles) {
      lbs[b] = nv;
      continue;
    }
    int64_t const x = b * kRsTile;
    int64_t lo = 0, hi = nv;  // first row with off[row] >= x
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if ((int64_t)off[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    lbs[b] = lo;
  }
}

// The tile's weights (as loaded, weight_t) and, when the tile owns at most kRsTile rows,
// their offsets are staged in LDS together -- every global load of the block is issued
// before the first barrier, so a block makes one round trip to memory
template <typename E, typename W>
__global__ __launch_bounds__(kRsThreads) void k_row_sums_tiles(E const* off, W const* w, int64_t ne,
                                                               int64_t const* lbs, W* out, double* head, double* tail)
{
  __shared__ W t_w[kRsTile];
  __shared__ int32_t t_off[kRsTile + 1];  // row starts relative to t0, clamped to n + 1 (a spill)
  __shared__ double sm[4];
  __shared__ int32_t t_long[kRsTile / 48 + 1];  // rows longer than kRsShort (below): at most n / 49
  __shared__ int n_long;
  if (threadIdx.x == 0) n_long = 0;
  int64_t const b  = blockIdx.x;
  int64_t const t0 = b * kRsTile;
  int64_t const t1 = min(ne, t0 + kRsTile);
  int const n      = (int)(t1 - t0);
  int64_t const r0 = lbs[b], r1 = lbs[b + 1];
  int64_t const nr = r1 - r0;
  bool const staged = nr + 1 <= kRsTile;
  W wv[kRsTile / kRsThreads];
#pragma unroll
  for (int j = 0; j < kRsTile / kRsThreads; ++j) {
    int const i = j * kRsThreads + threadIdx.x;
    wv[j]       = i < n ? w[t0 + i] : W(0);
  }
  if (staged)
    for (int64_t i = threadIdx.x; i <= nr; i += kRsThreads) t_off[i] = (int32_t)min((int64_t)off[r0 + i] - t0, (int64_t)n + 1);
#pragma unroll
  for (int j = 0; j < kRsTile / kRsThreads; ++j) t_w[j * kRsThreads + threadIdx.x] = wv[j];
  __syncthreads();
  auto row_start = [&](int64_t r) { return staged ? t0 + (int64_t)t_off[r - r0] : min((int64_t)off[r], t1 + 1); };
  // head: the edges [t0, first owned row's start) belong to a row that began earlier
  int64_t const h_end = nr > 0 ? min(row_start(r0), t1) : t1;
  double hs = 0.0;
  for (int i = threadIdx.x; i < (int)(h_end - t0); i += kRsThreads) hs += (double)t_w[i];
  hs = block_sum_256(hs, sm);
  if (threadIdx.x == 0) head[b] = hs;
  // rows owned by the tile: complete ones summed here, the last may spill past t1.
  // Rows of up to kRsShort edges: one thread each, in edge order; longer rows: one
  // wave each (lane-strided fp64 partials, then a fixed shuffle tree) -- a thread
  // walking a 1000-edge row through LDS held its whole block back.  Both orders are
  // fixed, so the sums are deterministic.
  constexpr int kRsShort = 48;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kRsThreads) {
    int64_t const a = row_start(r), e = row_start(r + 1);
    if (e > t1) continue;  // the spill row: block partial below
    if (e - a > kRsShort) {
      t_long[atomicAdd(&n_long, 1)] = (int32_t)(r - r0);
      continue;
    }
    double s0 = 0.0, s1 = 0.0;
    int64_t k = a;
    for (; k + 1 < e; k += 2) {
      s0 += (double)t_w[k - t0];
      s1 += (double)t_w[k + 1 - t0];
    }
    if (k < e) s0 += (double)t_w[k - t0];
    out[r] = static_cast<W>(s0 + s1);
  }
  __syncthreads();
  int const lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int j = wave; j < n_long; j += kRsThreads / 64) {
    int64_t const r = r0 + t_long[j];
    int64_t const a = row_start(r), e = row_start(r + 1);
    double x = 0.0;
    for (int64_t k = a + lane; k < e; k += 64) x += (double)t_w[k - t0];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane == 0) out[r] = static_cast<W>(x);
  }
  double ts = 0.0;
  bool const spill = nr > 0 && row_start(r1) > t1;
  if (spill) {
    int64_t const a = row_start(r1 - 1);
    for (int i = (int)(a - t0) + threadIdx.x; i < n; i += kRsThreads) ts += (double)t_w[i];
  }
  ts = block_sum_256(ts, sm);
  if (threadIdx.x == 0) tail[b] = spill ? ts : 0.0;
}

// rows that span tiles: tail of their first tile + head of every later tile they reach
template <typename E, typename W>
__global__ void k_row_sums_spill(E const* off, int64_t ntiles, int64_t const* lbs, double const* head,
                                 double const* tail, W* out)
{
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < ntiles; b += (int64_t)gridDim.x * blockDim.x) {
    int64_t const r0 = lbs[b], r1 = lbs[b + 1];
    int64_t const t1 = (b + 1) * kRsTile;
    if (r0 >= r1 || (int64_t)off[r1] <= t1) continue;
    int64_t const r  = r1 - 1;
    int64_t const be = ((int64_t)off[r + 1] - 1) / kRsTile;
    double s         = tail[b];
    for (int64_t t = b + 1; t <= be; ++t) s += head[t];
    out[r] = static_cast<W>(s);
  }
}

template <typename V, typename W>
__global__ void k_atomic_weight_sums(V const* idx, W const* w, size_t ne, double* acc)
{
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < ne; e += (size_t)gridDim.x * blockDim.x)
    atomicAdd(acc + idx[e], (double)w[e]);
}

template <typename V>
__global__ void k_ext_to_int(V* ids, size_t n, V const* sorted_ext, V const* internal, size_t nv, int* bad)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    V x       = ids[i];
    size_t lo = 0, hi = nv;
    while (lo < hi) {
      size_t mid = (lo + hi) >> 1;
      if (sorted_ext[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    if (lo < nv && sorted_ext[lo] == x) ids[i] = internal[lo];
    else {
      ids[i] = static_cast<V>(-1);
      if (bad) atomicAdd(bad, 1);
    }
  }
}
// The same lookup with one wave per id, for a few ids (BFS / SSSP sources): a 64-way
// search, each step one load per lane, so a lookup over V = 8.9M ids is 4 dependent
// loads instead of the binary search's 24 (RMAT-24: 11.4 us for one source).
template <typename V>
__global__ void k_ext_to_int_wave(V* ids, size_t n, V const* sorted_ext, V const* internal, size_t nv, int* bad)
{
  int const lane = threadIdx.x & 63;
  for (size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6; i < n; i += ((size_t)gridDim.x * blockDim.x) >> 6) {
    V const x = ids[i];
    size_t lo = 0, hi = nv;  // the first position with sorted_ext >= x lies in [lo, hi]
    while (hi - lo > 64) {
      size_t const step = (hi - lo + 63) / 64;
      size_t const p    = lo + (size_t)lane * step;
      bool const below  = p < hi && sorted_ext[p] < x;
      int const k       = __popcll(__ballot(below));  // pivots below x: lanes 0..k-1
      if (k == 0) {
        hi = lo;
        break;
      }
      size_t const nlo = lo + (size_t)(k - 1) * step + 1;
      hi               = std::min(lo + (size_t)k * step, hi);
      lo               = nlo;
    }
    size_t const p   = lo + lane;
    bool const below = p < hi && sorted_ext[p] < x;
    size_t const pos = lo + __popcll(__ballot(below));
    if (lane == 0) {
      if (pos < nv && sorted_ext[pos] == x) ids[i] = internal[pos];
      else {
        ids[i] = static_cast<V>(-1);
        if (bad) atomicAdd(bad, 1);
      }
    }
  }
}

template <typename V>
__global__ void k_check_range(V const* ids, size_t n, int64_t nv, int* bad)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (ids[i] < 0 || (int64_t)ids[i] >= nv) atomicAdd(bad, 1);
}
template <typename V>
__global__ void k_int_to_ext(V* ids, size_t n, V const* nmap, int64_t nv)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    V x = ids[i];
    if (x >= 0 && (int64_t)x < nv) ids[i] = nmap[x];
  }
}

// ---------------------------------------------------------------- helpers
// CSR offsets [nv + 1] of a SORTED major array
template <typename V, typename E>
void offsets_of_sorted(V const* sorted, size_t n, int64_t nv, E* off, hipStream_t s)
{
  hipLaunchKernelGGL((k_lower_bounds<V, E>), dim3(grid_for(nv + 1, kBlock, 8192)), dim3(kBlock), 0, s, sorted, n, nv,
                     off);
  CGX_LAUNCH_CHECK();
}

// degree of every id in [0, nv) among n unsorted majors: radix sort of the ids
// over the bits in use, then run lengths (a sort streams ~4 passes of 8 B per
// edge; counting with atomics serialised on the hub ids at 20-55 ms on RMAT-24)
template <typename V, typename E, typename D>
void degrees_of(V const* majors, size_t n, int64_t nv, D* deg, hipStream_t s)
{
  dbuf<E> off(nv + 1, s);
  if (n) {
    dbuf<V> sorted(n, s);
    radix_sort_keys<V>(majors, sorted.data(), n, 0, bits_for((unsigned long long)std::max<int64_t>(nv - 1, 0)), s);
    offsets_of_sorted<V, E>(sorted.data(), n, nv, off.data(), s);
  } else {
    fill<E>(off.data(), nv + 1, E(0), s);
  }
  hipLaunchKernelGGL((k_degrees<E, D>), dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, off.data(), nv, deg);
  CGX_LAUNCH_CHECK();
}

// sort (major, minor[, w]) by (major, minor) and compress into adj
template <typename V, typename E, typename W>
void compress(hipStream_t s, int64_t nv, V const* majors, V const* minors, W const* w, size_t n, adjacency_t& adj)
{
  CGX_EXPECTS(nv <= (int64_t(1) << 32), CUGRAPH_NOT_IMPLEMENTED, "graphs with more than 2^32 vertices are not supported");
  int b = bits_for(nv > 0 ? (unsigned long long)(nv - 1) : 0ull);
  dbuf<uint64_t> key(n, s), key_sorted(n, s);
  if (n) {
    hipLaunchKernelGGL(k_make_key<V>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, majors, minors, n, b,
                       key.data());
    CGX_LAUNCH_CHECK();
  }
  adj.weights.set_stream(s);
  if (w) {
    adj.weights.resize(n * sizeof(W));
    radix_sort_pairs<uint64_t, W>(key.data(), key_sorted.data(), w, adj.weights.data<W>(), n, 0, 2 * b, s);
  } else {
    adj.weights.release();
    radix_sort_keys<uint64_t>(key.data(), key_sorted.data(), n, 0, 2 * b, s);
  }
  key.b.release();
  dbuf<V> smaj(n, s);
  adj.indices.set_stream(s);
  adj.indices.resize((n + kIdxPad) * sizeof(V));  // padded: vector loads may read past the last list
  adj.idx_padded = true;
  if (n) {
    hipLaunchKernelGGL(k_split_key<V>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, key_sorted.data(), n, b,
                       smaj.data(), adj.indices.data<V>());
    CGX_LAUNCH_CHECK();
  }
  key_sorted.b.release();
  adj.offsets.set_stream(s);
  adj.offsets.resize((nv + 1) * sizeof(E));
  offsets_of_sorted<V, E>(smaj.data(), n, nv, adj.offsets.data<E>(), s);
  adj.sched_valid = false;
}

template <typename V, typename E, typename W>
void build_impl(handle_t& h, graph_t& g, array_view_t const& src, array_view_t const& dst, array_view_t const* wv,
                bool renumber)
{
  hipStream_t s = h.stream;
  size_t n      = src.size;
  dbuf<V> es(n, s), ed(n, s);
  if (n) {
    HIP_CHECK(hipMemcpyAsync(es.data(), src.data, n * sizeof(V), hipMemcpyDefault, s));
    HIP_CHECK(hipMemcpyAsync(ed.data(), dst.data, n * sizeof(V), hipMemcpyDefault, s));
  }
  dbuf<W> ew;
  if (wv) {
    ew.resize(n, s);
    if (n) HIP_CHECK(hipMemcpyAsync(ew.data(), wv->data, n * sizeof(W), hipMemcpyDefault, s));
  }
  auto [mn, mx] = minmax<V>(es.data(), n, s);
  auto [mn2, mx2] = minmax<V>(ed.data(), n, s);
  mn = std::min(mn, mn2);
  mx = std::max(mx, mx2);
  CGX_INPUT(n == 0 || mn >= 0, "Invalid input arguments: negative vertex id.");

  V* majors = g.store_transposed ? ed.data() : es.data();
  V* minors = g.store_transposed ? es.data() : ed.data();
  int64_t nv = 0;
  g.number_map.set_stream(s);
  if (renumber) {
    // 1. sorted unique vertex set
    dbuf<V> all(2 * n, s), all_sorted(2 * n, s);
    if (n) {
      HIP_CHECK(hipMemcpyAsync(all.data(), es.data(), n * sizeof(V), hipMemcpyDeviceToDevice, s));
      HIP_CHECK(hipMemcpyAsync(all.data() + n, ed.data(), n * sizeof(V), hipMemcpyDeviceToDevice, s));
    }
    int vb = bits_for((unsigned long long)std::max<long long>(mx, 0));
    radix_sort_keys<V>(all.data(), all_sorted.data(), 2 * n, 0, vb, s);
    dbuf<V> verts(2 * n, s);
    dbuf<size_t> cnt(1, s);
    if (n) {
      size_t tmp = 0;
      HIP_CHECK(rocprim::unique(nullptr, tmp, all_sorted.data(), verts.data(), cnt.data(), 2 * n,
                                rocprim::equal_to<V>(), s));
      buffer t(tmp, s);
      HIP_CHECK(rocprim::unique(t.data(), tmp, all_sorted.data(), verts.data(), cnt.data(), 2 * n,
                                rocprim::equal_to<V>(), s));
      nv = (int64_t)to_host_scalar(cnt.data(), s);
    }
    all.b.release();
    all_sorted.b.release();
    // 2. dense ids (position in the sorted vertex set)
    int64_t range = n ? (mx - mn + 1) : 0;
    if (n && range <= std::max<int64_t>(4 * nv, 1 << 22) && range < (int64_t(1) << 31)) {
      dbuf<int64_t> table(range, s);
      hipLaunchKernelGGL(k_table_fill<V>, dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, table.data(),
                         verts.data(), (size_t)nv, (int64_t)mn);
      CGX_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_dense_by_table<V>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, es.data(), n,
                         table.data(), (int64_t)mn);
      hipLaunchKernelGGL(k_dense_by_table<V>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, ed.data(), n,
                         table.data(), (int64_t)mn);
      CGX_LAUNCH_CHECK();
    } else if (n) {
      hipLaunchKernelGGL(k_dense_by_search<V>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, es.data(), n,
                         verts.data(), (size_t)nv, nullptr);
      hipLaunchKernelGGL(k_dense_by_search<V>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, ed.data(), n,
                         verts.data(), (size_t)nv, nullptr);
      CGX_LAUNCH_CHECK();
    }
    // 3. major degrees, 4. stable descending sort by degree
    dbuf<E> deg(nv, s), deg_sorted(nv, s);
    degrees_of<V, E, E>(majors, n, nv, deg.data(), s);
    dbuf<V> ids(nv, s), order(nv, s);
    iota<V>(ids.data(), nv, V(0), s);
    radix_sort_pairs<E, V>(deg.data(), deg_sorted.data(), ids.data(), order.data(), nv, 0,
                           bits_for((unsigned long long)std::max<int64_t>((int64_t)n, 1)), s, /*descending=*/true);
    // 5. number map and relabel
    g.number_map.resize(nv * sizeof(V));
    gather<V, V>(g.number_map.data<V>(), verts.data(), order.data(), nv, s);
    hipLaunchKernelGGL(k_inverse_perm<V>, dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, order.data(),
                       (size_t)nv, ids.data());
    CGX_LAUNCH_CHECK();
    if (n) {
      hipLaunchKernelGGL(k_relabel<V>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, es.data(), n,
                         ids.data());
      hipLaunchKernelGGL(k_relabel<V>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, ed.data(), n,
                         ids.data());
      CGX_LAUNCH_CHECK();
    }
  } else {
    nv = n ? (int64_t)mx + 1 : 0;
    g.number_map.resize(nv * sizeof(V));
    iota<V>(g.number_map.data<V>(), nv, V(0), s);
  }
  g.num_vertices = nv;
  g.num_edges    = (int64_t)n;
  g.renumbered   = renumber;
  auto adj       = std::make_shared<adjacency_t>();
  compress<V, E, W>(s, nv, majors, minors, wv ? ew.data() : nullptr, n, *adj);
  adj->degree_sorted = renumber;
  if (g.store_transposed) g.in = adj;
  else g.out = adj;
  if (g.symmetric) {
    g.in  = adj;
    g.out = adj;
  }
  HIP_CHECK(hipStreamSynchronize(s));
}

template <typename V, typename E, typename W>
void transpose_impl(handle_t& h, graph_t& g, bool to_transposed)
{
  hipStream_t s          = h.stream;
  adjacency_t& from      = to_transposed ? *g.out : *g.in;
  int64_t nv             = g.num_vertices;
  size_t n               = (size_t)g.num_edges;
  dbuf<V> majors(n, s);
  if (nv && n) {
    hipLaunchKernelGGL((k_expand_majors<V, E>), dim3(grid_for(n, kBlock, 16384)), dim3(kBlock), 0, s,
                       from.offsets.data<E>(), nv, (int64_t)n, majors.data());
    CGX_LAUNCH_CHECK();
  }
  auto adj = std::make_shared<adjacency_t>();
  // new majors = old minors
  compress<V, E, W>(s, nv, from.indices.data<V>(), majors.data(), g.weighted ? from.weights.data<W>() : nullptr, n,
                    *adj);
  adj->degree_sorted = false;
  if (to_transposed) g.in = adj;
  else g.out = adj;
  HIP_CHECK(hipStreamSynchronize(s));
}

template <typename V, typename E, typename W>
void schedule_impl(handle_t& h, graph_t& g, adjacency_t& adj)
{
  hipStream_t s = h.stream;
  int64_t nv    = g.num_vertices;
  E const* off  = adj.offsets.data<E>();
  bool sorted   = adj.degree_sorted;
  if (!sorted && nv > 1) {
    dbuf<int> bad(1, s);
    fill<int>(bad.data(), 1, 0, s);
    hipLaunchKernelGGL(k_check_sorted_desc<E>, dim3(grid_for(nv, kBlock, 4096)), dim3(kBlock), 0, s, off, nv,
                       bad.data());
    CGX_LAUNCH_CHECK();
    sorted = to_host_scalar(bad.data(), s) == 0;
  } else if (nv <= 1) {
    sorted = true;
  }
  adj.degree_sorted = sorted;
  adj.order.set_stream(s);
  if (!sorted) {
    dbuf<E> deg(nv, s), deg_sorted(nv, s);
    hipLaunchKernelGGL((k_degrees<E, E>), dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, off, nv, deg.data());
    CGX_LAUNCH_CHECK();
    dbuf<V> ids(nv, s);
    iota<V>(ids.data(), nv, V(0), s);
    adj.order.resize(nv * sizeof(V));
    radix_sort_pairs<E, V>(deg.data(), deg_sorted.data(), ids.data(), adj.order.data<V>(), nv, 0,
                           bits_for((unsigned long long)std::max<int64_t>(g.num_edges, 1)), s, true);
  } else {
    adj.order.release();
  }
  dbuf<int64_t> ends(kSchedBins, s);
  hipLaunchKernelGGL((k_bin_starts<V, E>), dim3(1), dim3(64), 0, s, off, sorted ? nullptr : adj.order.data<V>(), nv,
                     ends.data());
  CGX_LAUNCH_CHECK();
  auto hend = to_host(ends.data(), kSchedBins, s);
  hend[kSchedBins - 1] = nv;  // degree >= 0: everything
  adj.bin_begin.assign(kSchedBins + 1, 0);
  for (int b = 0; b < kSchedBins; ++b) adj.bin_begin[b + 1] = hend[b];
  // host-built work items, ~8K edges each
  std::vector<work_item> items;
  constexpr int64_t kTargetEdges = 8192;
  for (int b = 0; b < kSchedBins; ++b) {
    int64_t p0 = adj.bin_begin[b], p1 = adj.bin_begin[b + 1];
    if (p1 <= p0) continue;
    int w = kBinWidth[b];
    if (w == 256) {
      for (int64_t p = p0; p < p1; ++p) items.push_back(work_item{256, b, p, p + 1});
      continue;
    }
    int64_t groups = 256 / w;
    int64_t d_est  = std::max<int64_t>(1, kBinLo[b] + kBinLo[b] / 2);
    int64_t rounds = std::clamp<int64_t>(kTargetEdges / (groups * d_est), 1, 64);
    if (b == kSchedBins - 1) rounds = 16;  // zero-degree tail: pure vector epilogue
    int64_t per = groups * rounds;
    for (int64_t p = p0; p < p1; p += per) items.push_back(work_item{w, b, p, std::min(p1, p + per)});
  }
  adj.num_items = (int64_t)items.size();
  adj.items.set_stream(s);
  adj.items.resize(std::max<size_t>(items.size(), 1) * sizeof(work_item));
  to_device(adj.items.data<work_item>(), items.data(), items.size(), s);
  HIP_CHECK(hipStreamSynchronize(s));
  adj.sched_valid = true;
}

template <typename V>
void ext_lookup_impl(handle_t& h, graph_t& g)
{
  hipStream_t s = h.stream;
  int64_t nv    = g.num_vertices;
  g.ext_sorted.set_stream(s);
  g.ext_internal.set_stream(s);
  g.ext_sorted.resize(nv * sizeof(V));
  g.ext_internal.resize(nv * sizeof(V));
  dbuf<V> ids(nv, s);
  iota<V>(ids.data(), nv, V(0), s);
  auto [mn, mx] = minmax<V>(g.number_map.data<V>(), nv, s);
  (void)mn;
  radix_sort_pairs<V, V>(g.number_map.data<V>(), g.ext_sorted.data<V>(), ids.data(), g.ext_internal.data<V>(), nv,
                         0, bits_for((unsigned long long)std::max<long long>(mx, 0)), s);
  HIP_CHECK(hipStreamSynchronize(s));
  g.ext_lookup_valid = true;
}

template <typename V, typename E, typename W>
void outw_impl(handle_t& h, graph_t& g)
{
  hipStream_t s = h.stream;
  int64_t nv    = g.num_vertices;
  g.outw.set_stream(s);
  g.outw.resize(std::max<int64_t>(nv, 1) * sizeof(W));
  W* out = g.outw.data<W>();
  if (nv == 0) return;
  if (g.out) {
    E const* off = g.out->offsets.data<E>();
    if (g.weighted) {
      int64_t const ne     = g.num_edges;
      int64_t const ntiles = (ne + kRsTile - 1) / kRsTile;
      if (ntiles == 0) {
        fill<W>(out, nv, W(0), s);
      } else {
        dbuf<int64_t> lbs(ntiles + 1, s);
        dbuf<double> head(ntiles, s), tail(ntiles, s);
        hipLaunchKernelGGL((k_row_sum_tile_rows<E>), dim3(grid_for(ntiles + 1, kBlock, 8192)), dim3(kBlock), 0, s, off,
                           nv, ntiles, lbs.data());
        CGX_LAUNCH_CHECK();
        // rows of degree 0 past the last edge belong to no tile's edges: the last tile owns them
        hipLaunchKernelGGL((k_row_sums_tiles<E, W>), dim3((unsigned)ntiles), dim3(kRsThreads), 0, s, off,
                           g.out->weights.data<W>(), ne, lbs.data(), out, head.data(), tail.data());
        CGX_LAUNCH_CHECK();
        hipLaunchKernelGGL((k_row_sums_spill<E, W>), dim3(grid_for(ntiles, kBlock, 8192)), dim3(kBlock), 0, s, off,
                           ntiles, lbs.data(), head.data(), tail.data(), out);
      }
    } else {
      hipLaunchKernelGGL((k_degrees<E, W>), dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, off, nv, out);
    }
    CGX_LAUNCH_CHECK();
  } else {
    // only in-edges stored: accumulate by source (integer counts are exact; fp64 sums
    // round once to weight_t)
    size_t ne    = (size_t)g.num_edges;
    V const* idx = g.in->indices.data<V>();
    if (g.weighted) {
      dbuf<double> acc(nv, s);
      fill<double>(acc.data(), nv, 0.0, s);
      if (ne) {
        hipLaunchKernelGGL((k_atomic_weight_sums<V, W>), dim3(grid_for(ne, kBlock, 8192)), dim3(kBlock), 0, s, idx,
                           g.in->weights.data<W>(), ne, acc.data());
        CGX_LAUNCH_CHECK();
      }
      convert<W, double>(out, acc.data(), nv, s);
    } else {
      degrees_of<V, int64_t, W>(idx, ne, nv, out, s);
    }
  }
  HIP_CHECK(hipStreamSynchronize(s));
  g.outw_valid = true;
}

}  // namespace

// ---------------------------------------------------------------- public (internal API)
void build_sg_graph(handle_t& h, graph_t& g, array_view_t const& src, array_view_t const& dst,
                    array_view_t const* weights, bool renumber)
{
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    build_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g, src, dst, weights, renumber);
  });
}

adjacency_t& ensure_adjacency(handle_t& h, graph_t& g, bool transposed)
{
  auto& slot = transposed ? g.in : g.out;
  if (slot) return *slot;
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    transpose_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g, transposed);
  });
  return *slot;
}

void ensure_schedule(handle_t& h, graph_t& g, adjacency_t& adj)
{
  if (adj.sched_valid) return;
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    schedule_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g, adj);
  });
}

template <typename V>
void ext_to_int_launch(V* ids, size_t n, V const* sorted_ext, V const* internal, size_t nv, int* bad, hipStream_t s)
{
  if (n <= 1024)  // a wave per id
    hipLaunchKernelGGL(k_ext_to_int_wave<V>, dim3(grid_for(n * 64, kBlock, 4096)), dim3(kBlock), 0, s, ids, n,
                       sorted_ext, internal, nv, bad);
  else
    hipLaunchKernelGGL(k_ext_to_int<V>, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, ids, n, sorted_ext,
                       internal, nv, bad);
}

void renumber_ext_to_int(handle_t& h, graph_t& g, void* ids, size_t n, bool /*check*/)
{
  if (!n) return;
  hipStream_t s = h.stream;
  dbuf<int> bad(1, s);
  fill<int>(bad.data(), 1, 0, s);
  auto run = [&](auto vtag) {
    using V = decltype(vtag);
    V* p    = static_cast<V*>(ids);
    if (g.renumbered) {
      if (!g.ext_lookup_valid) ext_lookup_impl<V>(h, g);
      ext_to_int_launch<V>(p, n, g.ext_sorted.data<V>(), g.ext_internal.data<V>(), (size_t)g.num_vertices, bad.data(),
                           s);
    } else {
      hipLaunchKernelGGL(k_check_range<V>, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, p, n,
                         g.num_vertices, bad.data());
    }
    CGX_LAUNCH_CHECK();
  };
  if (g.vertex_type == INT32) run(int32_t{});
  else run(int64_t{});
  CGX_INPUT(to_host_scalar(bad.data(), s) == 0, "Invalid input argument: vertex id not in the graph.");
}

void renumber_ext_to_int_unchecked(handle_t& h, graph_t& g, void* ids, size_t n)
{
  if (!n || !g.renumbered) return;
  hipStream_t s = h.stream;
  auto run      = [&](auto vtag) {
    using V = decltype(vtag);
    if (!g.ext_lookup_valid) ext_lookup_impl<V>(h, g);
    ext_to_int_launch<V>(static_cast<V*>(ids), n, g.ext_sorted.data<V>(), g.ext_internal.data<V>(),
                         (size_t)g.num_vertices, nullptr, s);
    CGX_LAUNCH_CHECK();
  };
  if (g.vertex_type == INT32) run(int32_t{});
  else run(int64_t{});
}

void ensure_ext_lookup(handle_t& h, graph_t& g)
{
  if (!g.renumbered || g.ext_lookup_valid) return;
  if (g.vertex_type == INT32) ext_lookup_impl<int32_t>(h, g);
  else ext_lookup_impl<int64_t>(h, g);
}

void unrenumber_int_to_ext(handle_t& h, graph_t& g, void* ids, size_t n)
{
  if (!n || !g.renumbered) return;
  hipStream_t s = h.stream;
  auto run      = [&](auto vtag) {
    using V = decltype(vtag);
    hipLaunchKernelGGL(k_int_to_ext<V>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, static_cast<V*>(ids), n,
                       g.number_map.data<V>(), g.num_vertices);
    CGX_LAUNCH_CHECK();
  };
  if (g.vertex_type == INT32) run(int32_t{});
  else run(int64_t{});
}

std::unique_ptr<device_array_t> number_map_copy(handle_t& h, graph_t& g)
{
  auto a = std::make_unique<device_array_t>((size_t)g.num_vertices, g.vertex_type, h.stream);
  if (g.num_vertices)
    HIP_CHECK(hipMemcpyAsync(a->buf.data(), g.number_map.data(), g.num_vertices * dtype_size(g.vertex_type),
                             hipMemcpyDeviceToDevice, h.stream));
  return a;
}

void const* out_weight_sums(handle_t& h, graph_t& g)
{
  if (!g.outw_valid) {
    dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
      using T = decltype(t);
      outw_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g);
    });
  }
  return g.outw.data();
}

}  // namespace cgx
