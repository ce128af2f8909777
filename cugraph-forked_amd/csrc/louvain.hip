// Louvain modularity clustering (single GPU; the multi-GPU driver is at the end).
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
// Each level is a COO sorted by (source, destination) with 32-bit ids.  A sweep
// (the local move) aggregates every row's (neighbour cluster, weight) pairs in LDS
// hash tables with 64-bit fixed-point sums, no per-sweep sort (plan_sweeps /
// sweep below):
//   * rows of <= 1024 edges: k_sweep_hash, one block per chunk of whole rows;
//   * heavier rows: k_big_partials (2048-edge segments -> per-bucket partials),
//     k_big_buckets (merge a bucket's partials, gains), k_big_move (best bucket);
//   * a row the tables cannot hold (or a level with negative weights): the sort
//     path sweep_sorted -- key = row << cb | cluster(destination), radix sort,
//     reduce_by_key to (row, cluster, sum), gains, reduce_by_key over the row
//     (also the A/B option louvain_hash = 0).
// Ties go to the smaller cluster id in every path.  Cluster weights are 64-bit
// fixed-point totals updated by each sweep's moves (as the multi-GPU owners keep
// them); the modularity's internal weight
// comes from the sweep's own-cluster sums.  The run is deterministic.
#include "capi.hpp"
#include "comm.hpp"
#include "mg_graph.hpp"
#include "prims.hpp"

#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <limits>

namespace cgx {

namespace {

using u64 = unsigned long long;

// One level's edges.  Single GPU: every vertex is a row (base 0, nrows = nv).
// Multi-GPU: the rows are this rank's vertices [base, base + nrows) of the nv
// global ids; `src` holds row indices (global id - base), `dst` global ids.
struct level_graph {
  int64_t nv = 0, ne = 0;
  int64_t base = 0, nrows = 0;
  dbuf<uint32_t> src, dst;  // sorted by (src, dst)
  dbuf<double> w;
  float const* wf = nullptr;  // level 0 of fp32 input: the same weights as fp32 (the graph's own array,
                              // or wfbuf on the multi-GPU level 0)
  dbuf<float> wfbuf;
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
// level 0 from the adjacency: each row with edges marks its first edge with its id
// (an empty row shares its start with the next row, so only rows with edges write),
// and an inclusive max-scan carries the id over the row -- where a binary search
// over the offsets per edge (25 dependent loads at RMAT-26) took 43 ms
template <typename E>
__global__ void k_row_starts(E const* off, int64_t nv, uint32_t* src)
{
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nv; r += (int64_t)gridDim.x * blockDim.x)
    if (off[r + 1] > off[r]) src[off[r]] = (uint32_t)r;
}
template <typename V, typename R>
__global__ void k_expand_cols(V const* idx, R const* w, int64_t ne, uint32_t* dst, double* ww)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
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


// compact sweep key: row << cb | cluster(destination), cb = bits of the cluster ids,
// so the radix sort runs over the bits in use only (RMAT-23 level 1: 38 instead of
// 51 bits, 5 instead of 7 onesweep passes)
__global__ void k_sweep_keys(uint32_t const* src, uint32_t const* dst, uint32_t const* c, int64_t ne, int cb, u64* keys)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x)
    keys[e] = ((u64)src[e] << cb) | (u64)c[dst[e]];
}

// compact (row << cb | cluster) -> the row << 32 | cluster form the gain kernels read
__global__ void k_expand_keys(u64* keys, int64_t n, int cb)
{
  u64 const mask = (1ull << cb) - 1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    u64 const k = keys[i];
    keys[i]     = ((k >> cb) << 32) | (k & mask);
  }
}

// old_sum[u] = weight from u into its own cluster, self loops excluded
// (u is a row index; its cluster is c[u + base]); own[u] = the same with self loops
// (the row's share of the clustering's internal weight)
__global__ void k_old_sum(u64 const* uk, double const* psum, int64_t np, uint32_t const* c, uint32_t base,
                          double const* self, double* old_sum, double* own)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t u = (uint32_t)(uk[i] >> 32), cc = (uint32_t)uk[i];
    if (cc == c[u + base]) {
      old_sum[u] = psum[i] - self[u];
      own[u]     = psum[i];
    }
  }
}

// delta modularity of moving u into cluster cc (common_methods.cuh:49-74)
__global__ void k_gain(u64 const* uk, double const* psum, int64_t np, uint32_t const* c, uint32_t base,
                       double const* self, double const* old_sum, double const* a, uint8_t const* present,
                       double const* k, double m, double gamma, gain_t* out)
{
#pragma clang fp contract(off)
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t u = (uint32_t)(uk[i] >> 32), cc = (uint32_t)uk[i];
    uint32_t const cu = c[u + base];
    double s   = psum[i];
    if (cc == cu) s = s - self[u];
    double a_new = present[cc] ? a[cc] : (double)FLT_MAX;
    double a_old = a[cu];
    double kk    = k[u];
    double dq    = 2.0 * (((s - old_sum[u]) / m) - gamma * (a_new * kk - a_old * kk + kk * kk) / (m * m));
    out[i]       = gain_t{dq, cc};
  }
}

// next[u] for row u (next is indexed by row)
__global__ void k_move(uint32_t const* uu, gain_t const* best, int64_t n, uint32_t const* c, uint32_t base,
                       uint32_t* next, bool up_down)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t u = uu[i];
    gain_t b   = best[i];
    if (b.dq > 0.0 && ((b.c > c[u + base]) == up_down)) next[u] = b.c;
  }
}

struct sumsq_f {
  double const* a;
  uint8_t const* p;
  __device__ double operator()(size_t i) const { return p[i] ? a[i] * a[i] : 0.0; }
};
struct plain_f {
  double const* w;
  __device__ double operator()(size_t i) const { return w[i]; }
};

// self-loop weight of edge e (its row is src[e] + base)
__global__ void k_has_edges(int64_t const* off, int64_t n, uint8_t* has)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
    has[v] = off[v + 1] > off[v] ? 1 : 0;
}

// contraction
// compact pair key label(u) << cb | label(v) (cb = label bits; see k_sweep_keys)
__global__ void k_pair_keys(uint32_t const* src, uint32_t const* dst, uint32_t const* lab, int64_t ne, int cb,
                            u64* keys)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x)
    keys[e] = ((u64)lab[src[e]] << cb) | (u64)lab[dst[e]];
}

__global__ void k_mark_used(uint32_t const* lab, int64_t nv, uint32_t* used)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x)
    used[lab[v]] = 1u;
}

// deg[l - lo] = number of (sorted, unique) pair keys whose high word is l, for l in
// [lo, lo + n): two binary searches per label.  (A per-pair atomicAdd serialised on
// the hub clusters' counters: the first RMAT-23 contraction took 0.77 s instead of
// 0.04 s on some runs.)
__global__ void k_count_src(u64 const* keys, int64_t nk, int64_t lo, int64_t n, uint32_t* deg)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    u64 const k0 = (u64)(lo + i) << 32, k1 = (u64)(lo + i + 1) << 32;
    int64_t a = 0, b = nk;
    while (a < b) {
      int64_t m = (a + b) >> 1;
      if (keys[m] < k0) a = m + 1;
      else b = m;
    }
    int64_t c = a, d = nk;
    while (c < d) {
      int64_t m = (c + d) >> 1;
      if (keys[m] < k1) c = m + 1;
      else d = m;
    }
    deg[i] = (uint32_t)(c - a);
  }
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

// (l(u) << 32 | l(v)) -> compact (new(l(u)) << cb | new(l(v)))
__global__ void k_relabel_pairs(u64 const* keys, int64_t n, uint32_t const* nl, int cb, u64* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = ((u64)nl[(uint32_t)(keys[i] >> 32)] << cb) | (u64)nl[(uint32_t)keys[i]];
}

// key = s << cb | d (cb = 32 for the plain form)
__global__ void k_split_pairs(u64 const* keys, int64_t n, uint32_t* s, uint32_t* d, int cb)
{
  u64 const mask = cb >= 64 ? ~0ull : (1ull << cb) - 1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    s[i] = (uint32_t)(keys[i] >> cb);
    d[i] = (uint32_t)(keys[i] & mask);
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

// ------------------------------------------------ hash local move
// One block per chunk of whole rows (<= kHashRows rows, <= kHashEdges edges, so a
// chunk's distinct (row, neighbour cluster) pairs fit an LDS table at load <= 1/2).
// The pair sums are 64-bit fixed point (scale 2^(61 - e), every row weight < 2^e):
// order-independent, and exact for integer weights, so the gains are the same IEEE
// values as the sort path's and the oracle's.  Replaces key build + radix sort +
// two reduce_by_key passes (~20 B of HBM traffic per edge per pass) by one pass
// over the edges.  Small blocks (256 threads, 30 KB of LDS with 32-bit pair keys: 5
// per CU) so that one block's gathers overlap another's LDS phases; the grid is
// persistent, each block loading its next chunk's edges while it works on the current
// one (RMAT-23 level 0: a chunk holds ~36 rows, so 128 rows per chunk rarely binds).
constexpr int kHashEdges   = 1024;
constexpr int kHashRows    = 128;  // row arrays 5 KB: 5 blocks per CU
constexpr int kHashResident = 5;    // resident blocks per CU (the persistent grid)
constexpr int kHashSlots   = 2048;
constexpr int kHashThreads = 256;

struct hash_sweep_args {
  uint32_t const* dst;
  double const* w;
  float const* wf;  // when set, the weights as read (fp32 input at level 0: 4 bytes an edge fewer)
  int64_t const* off;
  int64_t const* chunks;  // 4 per chunk: first row, end row, first edge, end edge
  int64_t nchunks;
  uint32_t const* c;
  uint32_t base;
  double const* self;
  double const* a;
  double const* ag;  // gain weights: a[c] for a present cluster, FLT_MAX otherwise (one gather)
  double const* k;
  double m, gamma, scale, inv_scale;
  uint32_t* next;
  bool up_down;
  double* own;  // [row] weight into the row's own cluster, self loops included
};

// (row in chunk, neighbour cluster) keys: 8 + 24 bits when the level has < 2^24 - 1
// ids (never the all-ones empty key), else 32 + 32
template <typename K>
struct pair_key;
template <>
struct pair_key<uint32_t> {
  static constexpr uint32_t empty = ~0u;
  __device__ static uint32_t make(int i, uint32_t c) { return ((uint32_t)i << 24) | c; }
  __device__ static int row(uint32_t k) { return (int)(k >> 24); }
  __device__ static uint32_t cluster(uint32_t k) { return k & 0xffffffu; }
  __device__ static unsigned slot(uint32_t k, int bits) { return (k * 0x9E3779B1u) >> (32 - bits); }
};
template <>
struct pair_key<u64> {
  static constexpr u64 empty = ~0ull;
  __device__ static u64 make(int i, uint32_t c) { return ((u64)i << 32) | c; }
  __device__ static int row(u64 k) { return (int)(k >> 32); }
  __device__ static uint32_t cluster(u64 k) { return (uint32_t)k; }
  __device__ static unsigned slot(u64 k, int bits) { return (unsigned)((k * 0x9E3779B97F4A7C15ull) >> (64 - bits)); }
};

// monotone map double -> u64 (larger gain -> larger key)
__device__ inline u64 order_bits(double d)
{
  u64 const b = (u64)__double_as_longlong(d);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ inline double unorder_bits(u64 o)
{
  return __longlong_as_double((long long)((o >> 63) ? (o & 0x7fffffffffffffffull) : ~o));
}

// WT: the weight type read (float: hash_sweep_args::wf, double: w)
template <typename WT>
__device__ __forceinline__ WT const* sweep_weights(hash_sweep_args const& p);
template <>
__device__ __forceinline__ float const* sweep_weights<float>(hash_sweep_args const& p)
{
  return p.wf;
}
template <>
__device__ __forceinline__ double const* sweep_weights<double>(hash_sweep_args const& p)
{
  return p.w;
}

// (5 waves per SIMD: 5 blocks per CU at 30 KB; the fp64-weight form spills at 5)
template <typename K, typename WT>
__global__ __launch_bounds__(kHashThreads) __attribute__((amdgpu_waves_per_eu(sizeof(WT) == 4 ? 5 : 4, 5))) void
k_sweep_hash(
  hash_sweep_args p)
{
#pragma clang fp contract(off)
  using PK = pair_key<K>;
  constexpr int kEPT = kHashEdges / kHashThreads;
  __shared__ K key[kHashSlots];
  __shared__ u64 val[kHashSlots];
  __shared__ uint32_t r_cu[kHashRows], r_bc[kHashRows];
  __shared__ double r_k[kHashRows], r_aold[kHashRows], r_old[kHashRows];
  __shared__ u64 r_best[kHashRows];
  __shared__ uint32_t r_off[kHashRows + 1];  // the rows' first edges, from the chunk's first
  int const tid = threadIdx.x;
  // Persistent blocks: chunk ch is processed while the edges of the block's next chunk
  // (and the record of the one after) are in flight, so a chunk waits on its cluster
  // and gain gathers only, not on its edge loads.
  int64_t ch = blockIdx.x;
  if (ch >= p.nchunks) return;
  int64_t const* rc = p.chunks + 4 * ch;
  int64_t r0 = rc[0], r1 = rc[1], e0 = rc[2], e1 = rc[3];
  WT const* const wp = sweep_weights<WT>(p);
  uint32_t dv[kEPT];
  WT wv[kEPT];
  // thread t <= rows holds row t's first edge (an edge's row is found in r_off: no
  // per-edge row array is read)
  int64_t ro = tid <= (int)(r1 - r0) ? p.off[r0 + tid] : 0;
#pragma unroll
  for (int q = 0; q < kEPT; ++q) {
    int64_t const e = e0 + tid + q * kHashThreads;
    if (e < e1) {
      dv[q] = p.dst[e];
      wv[q] = wp[e];
    }
  }
  int64_t nch = ch + gridDim.x;
  int64_t n0 = 0, n1 = 0, ne0 = 0, ne1 = 0;  // the next chunk's record
  if (nch < p.nchunks) {
    rc  = p.chunks + 4 * nch;
    n0  = rc[0];
    n1  = rc[1];
    ne0 = rc[2];
    ne1 = rc[3];
  }
  while (true) {
    int const nrow = (int)(r1 - r0);
    int bits       = 6;  // table of 2^bits >= 2 * edges slots
    while ((1 << bits) < 2 * (int)(e1 - e0)) ++bits;
    int const nslot     = 1 << bits;
    unsigned const mask = (unsigned)nslot - 1;
    // this chunk's clusters, then the next chunk's edges and the record after it
#pragma unroll
    for (int q = 0; q < kEPT; ++q)
      if (e0 + tid + q * kHashThreads < e1) dv[q] = p.c[dv[q]];
    uint32_t ndv[kEPT];
    WT nwv[kEPT];
    int64_t nro = 0;
    if (nch < p.nchunks) {
      if (tid <= (int)(n1 - n0)) nro = p.off[n0 + tid];
#pragma unroll
      for (int q = 0; q < kEPT; ++q) {
        int64_t const e = ne0 + tid + q * kHashThreads;
        if (e < ne1) {
          ndv[q] = p.dst[e];
          nwv[q] = wp[e];
        }
      }
    }
    int64_t const nnch = nch + gridDim.x;
    int64_t m0 = 0, m1 = 0, me0 = 0, me1 = 0;
    if (nnch < p.nchunks) {
      rc  = p.chunks + 4 * nnch;
      m0  = rc[0];
      m1  = rc[1];
      me0 = rc[2];
      me1 = rc[3];
    }
    for (int i = tid; i < nslot; i += kHashThreads) {
      key[i] = PK::empty;
      val[i] = 0;
    }
    // thread t owns row t of the chunk
    bool const has_row = tid < nrow;
    int64_t const u    = r0 + tid;
    uint32_t cu        = 0;
    double self        = 0.0;
    if (has_row) {
      cu          = p.c[u + p.base];
      self        = p.self[u];
      r_cu[tid]   = cu;
      r_k[tid]    = p.k[u];
      r_aold[tid] = p.a[cu];
      r_old[tid]  = 0.0;
      r_best[tid] = 0;
      r_bc[tid]   = 0xffffffffu;
    }
    if (tid <= nrow) r_off[tid] = (uint32_t)(ro - e0);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kEPT; ++q) {
      int const j = tid + q * kHashThreads;
      if (e0 + j >= e1) break;
      int lo = 0, hi = nrow - 1;  // the edge's row: the last with r_off <= j (empty rows share starts)
      while (lo < hi) {
        int const mid = (lo + hi + 1) >> 1;
        if ((int)r_off[mid] <= j) lo = mid;
        else hi = mid - 1;
      }
      K const kk  = PK::make(lo, dv[q]);
      u64 const v = (u64)__double2ll_rn((double)wv[q] * p.scale);
      unsigned h  = PK::slot(kk, bits);
      while (true) {
        K const prev = atomicCAS(&key[h], PK::empty, kk);
        if (prev == PK::empty || prev == kk) {
          atomicAdd(&val[h], v);
          break;
        }
        h = (h + 1) & mask;
      }
    }
    __syncthreads();
    // weight into the own cluster, self loop excluded (k_old_sum)
    if (has_row) {
      K const kk = PK::make(tid, cu);
      unsigned h = PK::slot(kk, bits);
      double own = 0.0;
      while (key[h] != PK::empty) {
        if (key[h] == kk) {
          own        = (double)(long long)val[h] * p.inv_scale;
          r_old[tid] = own - self;
          break;
        }
        h = (h + 1) & mask;
      }
      p.own[u] = own;
    }
    __syncthreads();
    // gains (k_gain), per-row maximum.  For the own cluster s = sum - self = old_s,
    // the same IEEE value as k_gain's.
    {
      constexpr int kSPT = kHashSlots / kHashThreads;
      double an[kSPT];
#pragma unroll
      for (int q = 0; q < kSPT; ++q) {  // the neighbour clusters' gain weights, all in flight
        int const h = tid + q * kHashThreads;
        K const kk  = h < nslot ? key[h] : PK::empty;
        if (kk != PK::empty) {
          uint32_t const cc = PK::cluster(kk);
          an[q]             = p.ag[cc];
        }
      }
#pragma unroll
      for (int q = 0; q < kSPT; ++q) {
        int const h = tid + q * kHashThreads;
        if (h >= nslot) break;
        K const kk = key[h];
        if (kk == PK::empty) continue;
        int const i       = PK::row(kk);
        uint32_t const cc = PK::cluster(kk);
        double s          = cc == r_cu[i] ? r_old[i] : (double)(long long)val[h] * p.inv_scale;
        double a_new      = an[q];
        double a_old      = r_aold[i];
        double kv         = r_k[i];
        double dq = 2.0 * (((s - r_old[i]) / p.m) - p.gamma * (a_new * kv - a_old * kv + kv * kv) / (p.m * p.m));
        u64 const o = order_bits(dq);
        val[h]      = o;
        atomicMax(&r_best[i], o);
      }
    }
    __syncthreads();
    // ties: the smaller cluster (best_gain_op)
    for (int h = tid; h < nslot; h += kHashThreads) {
      K const kk = key[h];
      if (kk == PK::empty) continue;
      int const i = PK::row(kk);
      if (val[h] == r_best[i]) atomicMin(&r_bc[i], PK::cluster(kk));
    }
    __syncthreads();
    if (has_row && r_best[tid] != 0) {
      double const dq  = unorder_bits(r_best[tid]);
      uint32_t const b = r_bc[tid];
      if (dq > 0.0 && ((b > cu) == p.up_down)) p.next[u] = b;
    }
    if (nch >= p.nchunks) break;
    __syncthreads();  // the table and the row arrays are cleared for the next chunk
    ch = nch;
    r0 = n0;
    r1 = n1;
    e0 = ne0;
    e1 = ne1;
    ro = nro;
#pragma unroll
    for (int q = 0; q < kEPT; ++q) {
      dv[q] = ndv[q];
      wv[q] = nwv[q];
    }
    nch = nnch;
    n0  = m0;
    n1  = m1;
    ne0 = me0;
    ne1 = me1;
  }
}

// out[0] != 0: some weight is negative (or NaN); out[1] = largest row weight's bits
__global__ void k_level_stats(double const* w, int64_t ne, double const* k, int64_t nr, u64* out)
{
  __shared__ u64 sn[kBlock], sk[kBlock];
  u64 neg = 0, kmax = 0;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x)
    if (!(w[e] >= 0.0)) neg = 1;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nr; r += (int64_t)gridDim.x * blockDim.x) {
    u64 const b = (u64)__double_as_longlong(k[r]);
    kmax        = b > kmax ? b : kmax;
  }
  sn[threadIdx.x] = neg;
  sk[threadIdx.x] = kmax;
  __syncthreads();
  for (int st = kBlock / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) {
      sn[threadIdx.x] |= sn[threadIdx.x + st];
      sk[threadIdx.x] = sk[threadIdx.x] > sk[threadIdx.x + st] ? sk[threadIdx.x] : sk[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (sn[0]) atomicOr(&out[0], 1ull);
    atomicMax(&out[1], sk[0]);
  }
}

// big-row edges gathered into their own COO: rows[j]'s edges start at first[j] and
// land at pos[j] (pos has nb + 1 entries)
__global__ void k_gather_rows(int64_t const* first, int64_t const* pos, int64_t nb, uint32_t const* src,
                              uint32_t const* dst, double const* w, int64_t n, uint32_t* os, uint32_t* od, double* ow)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nb - 1;  // last j with pos[j] <= i
    while (lo < hi) {
      int64_t mid = (lo + hi + 1) >> 1;
      if (pos[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    int64_t const e = first[lo] + (i - pos[lo]);
    os[i]           = src[e];
    od[i]           = dst[e];
    ow[i]           = w[e];
  }
}

// ------------------------------------------------ hash local move, heavy rows
// Rows of degree > kHashEdges (RMAT hubs: ~15 % of the edges at level 0, more after
// the first contraction) in two LDS passes instead of a radix sort:
//  A. one block per segment of <= kBigSeg edges of one row: LDS table keyed by the
//     neighbour cluster -> the segment's distinct (cluster, partial sum) pairs,
//     written grouped by bucket (hash of the cluster, 2^logb buckets per row sized
//     for ~kBigPerBucket distinct clusters each); the own-cluster partial is added
//     to the row's own-sum (integer fixed point: order-free);
//  B. one block per (row, bucket): merges that bucket's partials of every segment
//     of the row in an LDS table, evaluates the gains, keeps the bucket's best;
//  C. one thread per row: best over the buckets -> move.
// A bucket whose distinct clusters exceed the table's cap raises a flag and the
// level falls back to the sort path for its heavy rows (never seen on RMAT).
constexpr int kBigSeg        = 2048;
constexpr int kBigSlots      = 4096;
constexpr int kBigThreads    = 512;
constexpr int kBigMaxBuckets = 1024;  // LDS of pass A: 52 KB -> 3 blocks per CU
constexpr int kBigPerBucket  = 2048;
constexpr int kBigMaxSegs    = 2048;  // rows of <= 4M edges (heavier: sort path)
constexpr int kBktSegGroup   = 512;   // pass B stages a row's segment runs 512 at a time (LDS: 3 blocks per CU)
constexpr int kBktSlots      = 4096;
constexpr int kBktThreads    = 512;
constexpr int kBktCap        = 3072;  // < kBktSlots - kBktThreads: probing always ends
constexpr uint32_t kEmpty32  = 0xffffffffu;

struct big_seg {
  int64_t e0, e1;  // edges in the level COO
  int64_t pbase;   // first partial slot
  int64_t boff;    // this segment's 2^logb + 1 bucket offsets
  uint32_t j, pad;
};
struct big_row {
  int64_t first;        // first edge
  uint32_t row, logb;   // row index, log2 of the bucket count
  uint32_t sbeg, send;  // segments
  uint32_t bbeg;        // first (row, bucket) block
  uint32_t single;      // one segment: pass A moves the row itself
};

// one pass-B block: bucket b of heavy row j (row id u), the row's first bucket-offset
// slot ob and first partial slot pb (segment q's offsets are ob + q (2^logb + 1), its
// partials start at pb + q kBigSeg), so the block reads its runs without the row and
// segment records in between
struct big_bblk {
  int64_t ob, pb;
  uint32_t j, u, b, ns, logb, pad;
};

struct big_args {
  uint32_t const* dst;
  double const* w;
  float const* wf;  // hash_sweep_args::wf
  uint32_t const* c;
  uint32_t base;
  big_seg const* segs;
  big_row const* rows;
  int64_t nrows;
  uint32_t* pkey;
  u64* pval;
  int32_t* boffs;
  u64* own;
  big_bblk const* bblk;
  double const* self;
  double const* a;
  double const* ag;  // gain weights (hash_sweep_args::ag)
  double const* k;
  double m, gamma, scale, inv_scale;
  u64* best_q;
  uint32_t* best_c;
  int* overflow;
  int cap;
  uint32_t* next;
  bool up_down;
  double* own_d;  // [row] weight into the row's own cluster (k_sweep_hash's own)
};

__device__ inline unsigned slot32(uint32_t x, int bits) { return (x * 0x9E3779B1u) >> (32 - bits); }
__device__ inline unsigned bucket_of(uint32_t x, unsigned logb)
{
  return logb ? ((x ^ 0x5bd1e995u) * 0x85EBCA6Bu) >> (32 - logb) : 0u;
}

// exclusive scan of a[0, n) in LDS, n <= T * PER; returns the total
template <int T, int PER>
__device__ uint32_t block_excl_scan(uint32_t* a, int n, uint32_t* wsum)
{
  int const t = threadIdx.x;
  uint32_t v[PER], s = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    int const i = PER * t + q;
    v[q]        = i < n ? a[i] : 0u;
    s += v[q];
  }
  uint32_t x = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t const y = __shfl_up(x, d, 64);
    if ((t & 63) >= d) x += y;
  }
  if ((t & 63) == 63) wsum[t >> 6] = x;
  __syncthreads();
  if (t == 0) {
    uint32_t r = 0;
    for (int i = 0; i < T / 64; ++i) {
      uint32_t const q = wsum[i];
      wsum[i]          = r;
      r += q;
    }
    wsum[T / 64] = r;
  }
  __syncthreads();
  uint32_t run = x - s + wsum[t >> 6];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    int const i = PER * t + q;
    if (i < n) a[i] = run;
    run += v[q];
  }
  uint32_t const total = wsum[T / 64];
  __syncthreads();
  return total;
}

// gains of one row's neighbour clusters key[0, nslot) (sums in val, replaced by the
// ordered gains), the maximum into bq.  The clusters' weights are gathered for all
// of a thread's slots before any of them is used.
template <int T, int S>
__device__ void gains_one_row(big_args const& p, uint32_t const* key, u64* val, int nslot, uint32_t cu, double old_s,
                              double kv, double a_old, u64& bq)
{
#pragma clang fp contract(off)
  constexpr int kSPT = S / T;
  int const tid      = threadIdx.x;
  double an[kSPT];
  u64 tmax = 0;
#pragma unroll
  for (int q = 0; q < kSPT; ++q) {
    int const h       = tid + q * T;
    uint32_t const cc = h < nslot ? key[h] : kEmpty32;
    if (cc != kEmpty32) an[q] = p.ag[cc];
  }
#pragma unroll
  for (int q = 0; q < kSPT; ++q) {
    int const h = tid + q * T;
    if (h >= nslot) break;
    uint32_t const cc = key[h];
    if (cc == kEmpty32) continue;
    double s     = cc == cu ? old_s : (double)(long long)val[h] * p.inv_scale;
    double a_new = an[q];
    double dq    = 2.0 * (((s - old_s) / p.m) - p.gamma * (a_new * kv - a_old * kv + kv * kv) / (p.m * p.m));
    u64 const o  = order_bits(dq);
    val[h]       = o;
    tmax         = o > tmax ? o : tmax;
  }
  // the wave's maximum first: one LDS atomic per wave instead of one per slot (a row's
  // thousands of slots all hit the one word)
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    u64 const y = __shfl_xor(tmax, d, 64);
    tmax        = y > tmax ? y : tmax;
  }
  if ((tid & 63) == 0 && tmax != 0) atomicMax(&bq, tmax);
}

// the block's LDS table holds every neighbour cluster of row rw.row: gains, best,
// move (k_gain + best_gain_op + k_move for one row); bq / bc: LDS scratch
__device__ void move_whole_row(big_args const& p, big_row const& rw, uint32_t const* key, u64* val, int nslot,
                               unsigned bits, u64& bq, uint32_t& bc, double& old_sh, uint32_t cu, double self,
                               double kv, double a_old)
{
#pragma clang fp contract(off)
  int const tid      = threadIdx.x;
  uint32_t const u   = rw.row;
  if (tid == 0) {
    double own     = 0.0;
    unsigned h     = slot32(cu, (int)bits);
    while (key[h] != kEmpty32) {
      if (key[h] == cu) {
        own = (double)(long long)val[h] * p.inv_scale;
        break;
      }
      h = (h + 1) & (unsigned)(nslot - 1);
    }
    p.own_d[u] = own;
    old_sh     = own == 0.0 ? 0.0 : own - self;
    bq     = 0;
    bc     = kEmpty32;
  }
  __syncthreads();
  double const old_s = old_sh;
  gains_one_row<kBigThreads, kBigSlots>(p, key, val, nslot, cu, old_s, kv, a_old, bq);
  __syncthreads();
  for (int h = tid; h < nslot; h += blockDim.x)
    if (key[h] != kEmpty32 && val[h] == bq) atomicMin(&bc, key[h]);
  __syncthreads();
  if (tid == 0 && bq != 0) {
    double const dq = unorder_bits(bq);
    if (dq > 0.0 && ((bc > cu) == p.up_down)) p.next[u] = bc;
  }
}

__global__ __launch_bounds__(kBigThreads) void k_big_partials(big_args p)
{
  __shared__ uint32_t key[kBigSlots];
  __shared__ u64 val[kBigSlots];
  __shared__ uint32_t hist[kBigMaxBuckets];
  __shared__ uint32_t wsum[kBigThreads / 64 + 1];
  __shared__ u64 bq;
  __shared__ uint32_t bc;
  __shared__ double old_sh;
  int const tid     = threadIdx.x;
  big_seg const sg  = p.segs[blockIdx.x];
  big_row const rw  = p.rows[sg.j];
  // the row's values are loaded here, in flight under the edge loads and gathers
  uint32_t const cu = p.c[rw.row + p.base];
  double kv = 0.0, self = 0.0, a_old = 0.0;
  if (rw.single) {
    kv    = p.k[rw.row];
    self  = p.self[rw.row];
    a_old = p.a[cu];
  }
  int const nbk     = 1 << rw.logb;
  int bits          = 6;  // 2^bits >= 2 * edges slots
  while ((1 << bits) < 2 * (int)(sg.e1 - sg.e0)) ++bits;
  int const nslot     = 1 << bits;
  unsigned const mask = (unsigned)nslot - 1;
  for (int i = tid; i < nslot; i += kBigThreads) {
    key[i] = kEmpty32;
    val[i] = 0;
  }
  for (int i = tid; i < nbk; i += kBigThreads) hist[i] = 0;
  __syncthreads();
  {
    constexpr int kEPT = kBigSeg / kBigThreads;
    uint32_t dv[kEPT];
    double wv[kEPT];
#pragma unroll
    for (int q = 0; q < kEPT; ++q) {
      int64_t const e = sg.e0 + tid + q * kBigThreads;
      if (e < sg.e1) {
        dv[q] = p.dst[e];
        wv[q] = p.wf ? (double)p.wf[e] : p.w[e];
      }
    }
#pragma unroll
    for (int q = 0; q < kEPT; ++q)
      if (sg.e0 + tid + q * kBigThreads < sg.e1) dv[q] = p.c[dv[q]];
#pragma unroll
    for (int q = 0; q < kEPT; ++q) {
      if (sg.e0 + tid + q * kBigThreads >= sg.e1) break;
      uint32_t const cc = dv[q];
      u64 const v       = (u64)__double2ll_rn(wv[q] * p.scale);
      unsigned h        = slot32(cc, bits);
      while (true) {
        uint32_t const prev = atomicCAS(&key[h], kEmpty32, cc);
        if (prev == kEmpty32 || prev == cc) {
          atomicAdd(&val[h], v);
          break;
        }
        h = (h + 1) & mask;
      }
    }
  }
  __syncthreads();
  if (rw.single) {
    move_whole_row(p, rw, key, val, nslot, (unsigned)bits, bq, bc, old_sh, cu, self, kv, a_old);
    return;
  }
  // The segment's distinct (cluster, partial) pairs, grouped by bucket: each thread
  // keeps its slots in registers, the pairs are placed in bucket order in the LDS table
  // itself (positions < distinct <= edges <= nslot / 2) and written out as one
  // contiguous run -- coalesced, where a store per pair at its bucket's position wrote
  // one partial line per 4- and 8-byte value
  constexpr int kSPT = kBigSlots / kBigThreads;
  uint32_t ck[kSPT], cpos[kSPT];
  u64 cv[kSPT];
#pragma unroll
  for (int q = 0; q < kSPT; ++q) {
    int const i = tid + q * kBigThreads;
    ck[q]       = i < nslot ? key[i] : kEmpty32;
    cv[q]       = i < nslot ? val[i] : 0ull;
    if (ck[q] != kEmpty32) {
      if (ck[q] == cu) atomicAdd(&p.own[sg.j], cv[q]);
      atomicAdd(&hist[bucket_of(ck[q], rw.logb)], 1u);
    }
  }
  __syncthreads();
  uint32_t const total = block_excl_scan<kBigThreads, kBigMaxBuckets / kBigThreads>(hist, nbk, wsum);
  for (int b = tid; b < nbk; b += kBigThreads) p.boffs[sg.boff + b] = (int32_t)hist[b];
  if (tid == 0) p.boffs[sg.boff + nbk] = (int32_t)total;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kSPT; ++q)
    if (ck[q] != kEmpty32) cpos[q] = atomicAdd(&hist[bucket_of(ck[q], rw.logb)], 1u);
  __syncthreads();  // every slot is in registers before the table is overwritten
#pragma unroll
  for (int q = 0; q < kSPT; ++q)
    if (ck[q] != kEmpty32) {
      key[cpos[q]] = ck[q];
      val[cpos[q]] = cv[q];
    }
  __syncthreads();
  for (uint32_t i = tid; i < total; i += kBigThreads) {
    p.pkey[sg.pbase + i] = key[i];
    p.pval[sg.pbase + i] = val[i];
  }
}

__global__ __launch_bounds__(kBktThreads) void k_big_buckets(big_args p)
{
#pragma clang fp contract(off)
  __shared__ uint32_t key[kBktSlots];
  __shared__ u64 val[kBktSlots];
  __shared__ uint32_t pre[kBktSegGroup];
  __shared__ uint32_t start[kBktSegGroup];  // from the row's first partial slot (< 4M)
  __shared__ uint32_t wsum[kBktThreads / 64 + 1];
  __shared__ uint32_t distinct, bc;
  __shared__ int over;
  __shared__ u64 bq;
  int const tid      = threadIdx.x;
  big_bblk const bk  = p.bblk[blockIdx.x];
  int const nbk      = 1 << bk.logb;
  int const ns       = (int)bk.ns;
  uint32_t const b   = bk.b;
  // row data first: independent of the partials, in flight meanwhile
  uint32_t const u   = bk.u;
  uint32_t const cu  = p.c[u + p.base];
  double const kv    = p.k[u], self = p.self[u];
  u64 const ownj     = p.own[bk.j];
  double const a_old = p.a[cu];
  if (tid == 0) {
    distinct = 0;
    over     = 0;
    bq       = 0;
    bc       = kEmpty32;
  }
  // the segments' runs of bucket b, kBktSegGroup segments at a time (one group below
  // 1M-edge rows, so the table is sized by its partials)
  int bits            = 6;  // 2^bits >= 2 * partials slots, at most kBktSlots (then the cap guards)
  int nslot           = 0;
  unsigned mask       = 0;
  int const cap       = p.cap;  // below kBktSlots slots total <= nslot / 2: never full
  bool stop           = false;
  for (int g0 = 0; g0 < ns; g0 += kBktSegGroup) {
    int const gn = ns - g0 < kBktSegGroup ? ns - g0 : kBktSegGroup;
    for (int i = tid; i < gn; i += kBktThreads) {
      int64_t const o  = bk.ob + (int64_t)(g0 + i) * (nbk + 1) + b;
      int32_t const lo = p.boffs[o], hi = p.boffs[o + 1];
      pre[i]           = (uint32_t)(hi - lo);
      start[i]         = (uint32_t)((g0 + i) * kBigSeg + lo);
    }
    __syncthreads();
    uint32_t const total = block_excl_scan<kBktThreads, kBktSegGroup / kBktThreads>(pre, gn, wsum);
    if (g0 == 0) {
      if (ns > kBktSegGroup) bits = 12;
      while ((1 << bits) < kBktSlots && (1u << bits) < 2 * total) ++bits;
      nslot = 1 << bits;
      mask  = (unsigned)nslot - 1;
      for (int i = tid; i < nslot; i += kBktThreads) {
        key[i] = kEmpty32;
        val[i] = 0;
      }
      __syncthreads();
    }
    constexpr int kPPT = 4;  // partials per thread per batch, loaded before their inserts
    for (uint32_t f0 = 0; f0 < total && !stop; f0 += kPPT * kBktThreads) {
      uint32_t kq[kPPT];
      u64 vq[kPPT];
#pragma unroll
      for (int q = 0; q < kPPT; ++q) {
        uint32_t const f = f0 + tid + q * kBktThreads;
        if (f >= total) break;
        int lo = 0, hi = gn - 1;  // last segment with pre <= f
        while (lo < hi) {
          int const mid = (lo + hi + 1) >> 1;
          if (pre[mid] <= f) lo = mid;
          else hi = mid - 1;
        }
        int64_t const x = bk.pb + start[lo] + (f - pre[lo]);
        kq[q]           = p.pkey[x];
        vq[q]           = p.pval[x];
      }
#pragma unroll
      for (int q = 0; q < kPPT; ++q) {
        if (stop || f0 + tid + q * kBktThreads >= total) break;
        uint32_t const cc = kq[q];
        unsigned h        = slot32(cc, bits);
        while (true) {
          uint32_t const prev = atomicCAS(&key[h], kEmpty32, cc);
          if (prev == kEmpty32 || prev == cc) {
            atomicAdd(&val[h], vq[q]);
            if (prev == kEmpty32 && (int)atomicAdd(&distinct, 1u) >= cap) {
              over = 1;
              stop = true;
            }
            break;
          }
          h = (h + 1) & mask;
        }
      }
    }
    __syncthreads();  // pre / start are rewritten by the next group
    if (over) break;
  }
  if (over) {
    if (tid == 0) atomicOr(p.overflow, 1);
    return;
  }
  double const old_s = (double)(long long)ownj * p.inv_scale - self;
  gains_one_row<kBktThreads, kBktSlots>(p, key, val, nslot, cu, old_s, kv, a_old, bq);
  __syncthreads();
  for (int h = tid; h < nslot; h += kBktThreads)
    if (key[h] != kEmpty32 && val[h] == bq) atomicMin(&bc, key[h]);
  __syncthreads();
  if (tid == 0) {
    p.best_q[blockIdx.x] = bq;
    p.best_c[blockIdx.x] = bc;
  }
}

__global__ void k_big_move(big_args p)
{
  if (*p.overflow) return;  // pass B gave up: the sweep is redone on the sort path
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < p.nrows; j += (int64_t)gridDim.x * blockDim.x) {
    big_row const rw = p.rows[j];
    if (rw.single) continue;
    p.own_d[rw.row] = (double)(long long)p.own[j] * p.inv_scale;
    u64 best         = 0;
    uint32_t bc      = kEmpty32;
    for (uint32_t i = rw.bbeg; i < rw.bbeg + (1u << rw.logb); ++i) {
      u64 const o = p.best_q[i];
      if (o == 0) continue;
      uint32_t const c = p.best_c[i];
      if (o > best || (o == best && c < bc)) {
        best = o;
        bc   = c;
      }
    }
    if (best == 0) continue;
    double const dq = unorder_bits(best);
    if (dq > 0.0 && ((bc > p.c[rw.row + p.base]) == p.up_down)) p.next[rw.row] = bc;
  }
}

// Chunk schedule of a level (the host loop took 28 ms at RMAT-23 level 0): thread t
// walks rows [256 t, 256 t + 256) greedily -- a chunk closes before the row that
// would take it past kHashEdges edges; rows above kHashEdges are heavy rows.
// Pass 0 counts chunks and heavy rows per thread, pass 1 writes them at the
// scanned positions.  Chunks never cross a 256-row block (= kHashRows).
__global__ void k_chunk_walk(int64_t const* off, int64_t nr, int pass, uint32_t* ccount, uint32_t* bcount,
                             int64_t const* cpos, int64_t const* bpos, int64_t* chunks, int64_t* bigrows)
{
  int64_t const nblk = (nr + kHashRows - 1) / kHashRows;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nblk; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t const rb = t * kHashRows, re = rb + kHashRows < nr ? rb + kHashRows : nr;
    int64_t nc = 0, nb = 0, r0 = rb, ce = 0;
    int64_t* co = pass ? chunks + 4 * cpos[t] : nullptr;
    int64_t* bo = pass ? bigrows + bpos[t] : nullptr;
    int64_t lo  = off[rb];
    auto emit   = [&](int64_t a, int64_t b, int64_t eb) {  // rows [a, b), edges [eb - ce, eb)
      if (pass) {
        co[4 * nc]     = a;
        co[4 * nc + 1] = b;
        co[4 * nc + 2] = eb - ce;
        co[4 * nc + 3] = eb;
      }
      ++nc;
    };
    for (int64_t r = rb; r < re; ++r) {
      int64_t const hi = off[r + 1], d = hi - lo;
      if (d > kHashEdges) {
        if (ce > 0) emit(r0, r, lo);
        if (pass) bo[nb] = r;
        ++nb;
        ce = 0;
        r0 = r + 1;
        lo = hi;
        continue;
      }
      if (ce + d > kHashEdges) {
        emit(r0, r, lo);
        ce = 0;
        r0 = r;
      }
      ce += d;
      lo = hi;
    }
    if (ce > 0) emit(r0, re, lo);
    if (!pass) {
      ccount[t] = (uint32_t)nc;
      bcount[t] = (uint32_t)nb;
    }
  }
}

__global__ void k_big_info(int64_t const* rows, int64_t const* off, int64_t n, int64_t* first, int64_t* deg)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    first[i] = off[rows[i]];
    deg[i]   = off[rows[i] + 1] - first[i];
  }
}

// Heavy-row schedule on the device (plan_big_rows' host loop and its uploads were a
// 2.2 ms gap per level at RMAT-23).  Per heavy row j (rows[j], ascending): segments of
// kBigSeg edges, 2^logb buckets, partial slots = degree, bucket-offset slots.  Pass 0
// counts (cnt[4][n + 1], a zero after each list so the exclusive scans end with the
// totals) and flags rows the LDS passes cannot take (the host plan then runs as
// before); pass 1 writes big_row / big_seg / the (row, bucket) blocks at the scanned
// positions.  Segment order, buckets and offsets are plan_big_rows' exactly.
__device__ __forceinline__ int ceil_log2_dev(int64_t x)
{
  int l = 0;
  while ((int64_t(1) << l) < x) ++l;
  return l;
}

__global__ void k_big_plan(int64_t const* rows, int64_t const* off, int64_t n, int64_t maxdeg, int pass,
                           u64* cnt, u64 const* pos, big_row* brows, big_seg* bsegs, big_bblk* bblk, int* rest)
{
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    int64_t const r = rows[j], first = off[r], d = off[r + 1] - first;
    int64_t const nseg = (d + kBigSeg - 1) / kBigSeg;
    bool const single  = nseg == 1;
    int const logb     = single ? 0 : min(ceil_log2_dev((d + kBigPerBucket - 1) / kBigPerBucket),
                                          ceil_log2_dev(kBigMaxBuckets));
    int64_t const nbk  = single ? 0 : (int64_t(1) << logb);
    if (pass == 0) {
      if (nseg > kBigMaxSegs || d > maxdeg) atomicOr(rest, 1);
      cnt[0 * (n + 1) + j] = (u64)nseg;
      cnt[1 * (n + 1) + j] = (u64)nbk;
      cnt[2 * (n + 1) + j] = single ? 0ull : (u64)(nseg * (nbk + 1));
      cnt[3 * (n + 1) + j] = (u64)d;
      if (j == 0)
        for (int q = 0; q < 4; ++q) cnt[q * (n + 1) + n] = 0ull;
      continue;
    }
    int64_t const sb = (int64_t)pos[0 * (n + 1) + j], bb = (int64_t)pos[1 * (n + 1) + j];
    int64_t const ob = (int64_t)pos[2 * (n + 1) + j], pb = (int64_t)pos[3 * (n + 1) + j];
    big_row rw;
    rw.first  = first;
    rw.row    = (uint32_t)r;
    rw.logb   = (uint32_t)logb;
    rw.sbeg   = (uint32_t)sb;
    rw.send   = (uint32_t)(sb + nseg);
    rw.bbeg   = (uint32_t)bb;
    rw.single = single ? 1u : 0u;
    brows[j]  = rw;
    for (int64_t q = 0; q < nseg; ++q) {
      big_seg sg;
      sg.e0    = first + q * kBigSeg;
      sg.e1    = min(first + d, sg.e0 + kBigSeg);
      sg.pbase = pb + q * kBigSeg;
      sg.boff  = single ? ob : ob + q * (nbk + 1);
      sg.j     = (uint32_t)j;
      sg.pad   = 0;
      bsegs[sb + q] = sg;
    }
    for (int64_t b = 0; b < nbk; ++b) {
      big_bblk k;
      k.ob         = ob;
      k.pb         = pb;
      k.j          = (uint32_t)j;
      k.u          = (uint32_t)r;
      k.b          = (uint32_t)b;
      k.ns         = (uint32_t)nseg;
      k.logb       = (uint32_t)logb;
      k.pad        = 0;
      bblk[bb + b] = k;
    }
  }
}

__global__ void k_plan_totals(u64 const* pos, int64_t n, int const* rest, u64* tot)
{
  if (threadIdx.x < 4) tot[threadIdx.x] = pos[threadIdx.x * (n + 1) + n];
  if (threadIdx.x == 4) tot[4] = (u64)*rest;
}

// the two chunk-walk totals (chunks, heavy rows) in one read
__global__ void k_walk_totals(int64_t const* cp, uint32_t const* cc, int64_t const* bp, uint32_t const* bc, int64_t n,
                              int64_t* tot)
{
  if (threadIdx.x == 0) tot[0] = cp[n - 1] + (int64_t)cc[n - 1];
  if (threadIdx.x == 1) tot[1] = bp[n - 1] + (int64_t)bc[n - 1];
}

inline unsigned blocks(int64_t n) { return grid_for(n > 0 ? n : 1, kBlock, 16384); }

// ---------------------------------------------------------------- driver
struct louvain_state {
  hipStream_t s;
  double m;
  double gamma;
  comm_t* comm = nullptr;  // multi-GPU: the world communicator; nullptr on one GPU
  dbuf<double> scratch;    // device_sum partials
  dbuf<double> scal;       // 2 scalars
  size_t bytes = 0;        // multi-GPU: bytes this rank sent in the exchanges being counted
  tuning_t tune;           // the handle's A/B switches (louvain_*)
  bool trace = false;      // CGX_LOUVAIN_TRACE: per-level plan statistics on stderr (measurement only)
  louvain_state(hipStream_t st, tuning_t const& t) : s(st), scratch(1024, st), scal(2, st), tune(t) {}
};

// k[v] = weight of row v, self[v] = its self-loop weight, has_edges[v], in one pass
// over the level COO (the two rocPRIM segmented reductions this replaces read the 2 GB
// of RMAT-23 level-0 weights twice at ~0.6 TB/s: 3.4 + 3.6 ms).  A wave takes 64
// consecutive rows: a row of <= kVwLane edges is summed by its own lane in edge
// order; a row of <= kVwWave edges by the whole wave, lane l summing edges l, l + 64,
// ... in order and the 64 partials combined by a fixed xor tree (lane 0's value); the
// longer rows (the hubs: a wave that met the top 64 of RMAT-23 spent 14 ms on them)
// are listed for k_vertex_weights_big, one 1024-thread block per row, thread t summing
// edges t, t + 1024, ... and the 16 wave values added in wave order.  Every order
// depends only on the row's edges and degree, so every rank layout that holds the row
// gives the same bits.  The same passes flag negative (or NaN) weights and take the
// largest row weight (the fixed-point scale of the hash sweeps), so plan_sweeps needs
// no pass of its own over the weights.
constexpr int kVwLane   = 16;
constexpr int kVwWave   = 4096;
constexpr int kVwBigThr = 1024;

__device__ __forceinline__ void vw_stats_flush(u64 neg, u64 kmax, u64* stats)
{
  __shared__ u64 sn[16], sk[16];
  int const lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    neg |= __shfl_xor(neg, o, 64);
    u64 const y = __shfl_xor(kmax, o, 64);
    kmax        = y > kmax ? y : kmax;
  }
  if (lane == 0) {
    sn[threadIdx.x >> 6] = neg;
    sk[threadIdx.x >> 6] = kmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 n = 0, m = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      n |= sn[i];
      m = sk[i] > m ? sk[i] : m;
    }
    if (n) atomicOr(&stats[0], 1ull);
    atomicMax(&stats[1], m);
  }
}

// big: [0] rows listed, [1] rows taken by k_vertex_weights_big; list: the rows
__global__ __launch_bounds__(256) void k_vertex_weights(int64_t const* off, uint32_t const* dst, double const* w,
                                                         int64_t nr, uint32_t base, double* k, double* self,
                                                         uint8_t* has, u64* stats, unsigned* big, uint32_t* list)
{
  int const lane    = threadIdx.x & 63;
  int64_t const nw  = (int64_t)gridDim.x * (blockDim.x >> 6);
  u64 neg = 0, kmax = 0;
  for (int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t * 64 < nr; t += nw) {
    int64_t const r = t * 64 + lane;
    bool const ok   = r < nr;
    int64_t const b = ok ? off[r] : 0, e = ok ? off[r + 1] : 0;
    double kv = 0.0, sv = 0.0;
    if (e - b <= kVwLane) {
      for (int64_t i = b; i < e; ++i) {
        double const x = w[i];
        neg |= !(x >= 0.0);
        kv += x;
        sv += dst[i] == (uint32_t)r + base ? x : 0.0;
      }
    }
    u64 const bigm = __ballot(ok && e - b > kVwWave);
    if (bigm) {  // one atomic per wave: the hubs go to the block kernel
      unsigned at = 0;
      if (lane == 0) at = atomicAdd(&big[0], (unsigned)__popcll(bigm));
      at = __shfl(at, 0, 64);
      if ((bigm >> lane) & 1ull) list[at + __popcll(bigm & ((1ull << lane) - 1ull))] = (uint32_t)r;
    }
    u64 longm = __ballot(ok && e - b > kVwLane && e - b <= kVwWave);
    while (longm) {
      int const j       = __builtin_ctzll(longm);
      longm &= longm - 1;
      int64_t const rj  = t * 64 + j;
      int64_t const bj  = __shfl(b, j, 64), ej = __shfl(e, j, 64);
      double pk = 0.0, ps = 0.0;
      for (int64_t i = bj + lane; i < ej; i += 64) {
        double const x = w[i];
        neg |= !(x >= 0.0);
        pk += x;
        ps += dst[i] == (uint32_t)rj + base ? x : 0.0;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        pk += __shfl_xor(pk, o, 64);
        ps += __shfl_xor(ps, o, 64);
      }
      double const pk0 = __shfl(pk, 0, 64);  // lane 0's sums (the xor tree associates per lane)
      double const ps0 = __shfl(ps, 0, 64);
      if (lane == j) {
        kv = pk0;
        sv = ps0;
      }
    }
    if (ok) {
      has[r] = e > b ? 1 : 0;
      if (e - b <= kVwWave) {
        k[r]           = kv;
        self[r]        = sv;
        u64 const bits = (u64)__double_as_longlong(kv);
        kmax           = bits > kmax ? bits : kmax;
      }
    }
  }
  vw_stats_flush(neg, kmax, stats);
}

// the listed rows, one at a time per block (taken by an atomic counter: which block
// sums a row does not change its bits)
__global__ __launch_bounds__(kVwBigThr) void k_vertex_weights_big(int64_t const* off, uint32_t const* dst,
                                                                   double const* w, uint32_t base, double* k,
                                                                   double* self, u64* stats, unsigned* big,
                                                                   uint32_t const* list)
{
  __shared__ double wk[kVwBigThr / 64], wsf[kVwBigThr / 64];
  __shared__ unsigned s_i;
  int const lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u64 neg = 0, kmax = 0;
  unsigned const n = big[0];
  while (true) {
    if (threadIdx.x == 0) s_i = atomicAdd(&big[1], 1u);
    __syncthreads();
    unsigned const i = s_i;
    __syncthreads();
    if (i >= n) break;
    uint32_t const r = list[i];
    int64_t const b = off[r], e = off[r + 1];
    double pk = 0.0, ps = 0.0;
    for (int64_t q = b + threadIdx.x; q < e; q += kVwBigThr) {
      double const x = w[q];
      neg |= !(x >= 0.0);
      pk += x;
      ps += dst[q] == r + base ? x : 0.0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      pk += __shfl_xor(pk, o, 64);
      ps += __shfl_xor(ps, o, 64);
    }
    if (lane == 0) {
      wk[wv]  = pk;
      wsf[wv] = ps;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double kv = 0.0, sv = 0.0;
      for (int j = 0; j < kVwBigThr / 64; ++j) {
        kv += wk[j];
        sv += wsf[j];
      }
      k[r]           = kv;
      self[r]        = sv;
      u64 const bits = (u64)__double_as_longlong(kv);
      kmax           = bits > kmax ? bits : kmax;
    }
  }
  vw_stats_flush(neg, kmax, stats);
}

// stats (u64[2], device): [0] nonzero if a weight is negative or NaN, [1] the bits of
// the largest row weight -- plan_sweeps' inputs
void vertex_weights(louvain_state& S, level_graph const& g, int64_t const* off, double* k, double* self,
                    uint8_t* has_edges, u64* stats)
{
  hipStream_t s    = S.s;
  int64_t const nr = g.nrows;
  fill<u64>(stats, 2, 0ull, s);
  if (nr == 0) return;
  int64_t const nbig = std::min<int64_t>(nr, g.ne / kVwWave + 1);
  dbuf<unsigned> big(2, s);
  dbuf<uint32_t> list(std::max<int64_t>(nbig, 1), s);
  fill<unsigned>(big.data(), 2, 0u, s);
  unsigned const grid = grid_for((size_t)((nr + 63) / 64), 4, 16384);
  hipLaunchKernelGGL(k_vertex_weights, dim3(grid), dim3(256), 0, s, off, g.dst.data(), g.w.data(), nr,
                     (uint32_t)g.base, k, self, has_edges, stats, big.data(), list.data());
  CGX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_vertex_weights_big, dim3((unsigned)std::min<int64_t>(nbig, 512)), dim3(kVwBigThr), 0, s, off,
                     g.dst.data(), g.w.data(), (uint32_t)g.base, k, self, stats, big.data(), list.data());
  CGX_LAUNCH_CHECK();
}

// Q = internal / m - gamma * sum_c a_c^2 / m^2 (compute_modularity,
// common_methods.cuh:121-170).  Each rank sums its own edges and the a_c of the
// cluster ids in its own range; the two partials are allreduced.
// The same Q with the internal weight taken from a sweep's by-product: own[row] =
// the row's weight into its own cluster under the clustering the sweep started from
// (self loops included), so sum_rows own = sum of w over edges inside clusters.  The
// level loop runs the next sweep before deciding (one extra, discarded sweep per
// level) instead of an edge pass per sweep (1.7 ms at RMAT-23 level 0).
double modularity_own(louvain_state& S, level_graph const& g, double const* own, double const* a, uint8_t const* present)
{
  device_sum(plain_f{own}, (size_t)g.nrows, S.scal.data(), S.scratch.data(), S.s);
  device_sum(sumsq_f{a + g.base, present + g.base}, (size_t)g.nrows, S.scal.data() + 1, S.scratch.data(), S.s);
  if (S.comm) S.comm->allreduce<double>(S.scal.data(), S.scal.data(), 2, CGX_COMM_SUM, S.s);
  auto hv = to_host(S.scal.data(), 2, S.s);
  return hv[0] / S.m - (S.gamma * hv[1]) / (S.m * S.m);
}

// the sort-based local move over the edges (src, dst, w)[0, ne) of some of the
// rows (whole rows only): next[row] is written for the rows that move
void sweep_sorted(louvain_state& S, level_graph const& g, uint32_t const* src, uint32_t const* dst, double const* w,
                  int64_t ne, uint32_t const* c, uint32_t* next, double const* k, double const* self, double const* a,
                  uint8_t const* present, bool up_down, double* own)
{
  hipStream_t s = S.s;
  int64_t nv = g.nv, nr = g.nrows;
  uint32_t const base = (uint32_t)g.base;
  if (ne == 0) return;
  dbuf<u64> keys(ne, s), keys2(ne, s);
  dbuf<double> w2(ne, s), psum(ne, s);
  int const cb = bits_for((unsigned long long)std::max<int64_t>(nv - 1, 0));
  hipLaunchKernelGGL(k_sweep_keys, dim3(blocks(ne)), dim3(kBlock), 0, s, src, dst, c, ne, cb, keys.data());
  CGX_LAUNCH_CHECK();
  radix_sort_pairs<u64, double>(keys.data(), keys2.data(), w, w2.data(), (size_t)ne, 0,
                                cb + bits_for(std::max<int64_t>(nr - 1, 0)), s);
  // (row, neighbour cluster) -> sum of weights; `keys` reused for the pair keys
  int64_t np = reduce_by_key(keys2.data(), w2.data(), (size_t)ne, keys.data(), psum.data(), rocprim::plus<double>(),
                             rocprim::equal_to<u64>(), s);
  hipLaunchKernelGGL(k_expand_keys, dim3(blocks(np)), dim3(kBlock), 0, s, keys.data(), np, cb);
  CGX_LAUNCH_CHECK();
  dbuf<double> old_sum(nr, s);
  fill<double>(old_sum.data(), nr, 0.0, s);
  hipLaunchKernelGGL(k_old_sum, dim3(blocks(np)), dim3(kBlock), 0, s, keys.data(), psum.data(), np, c, base, self,
                     old_sum.data(), own);
  CGX_LAUNCH_CHECK();
  dbuf<gain_t> gains(np, s), best(nr, s);
  hipLaunchKernelGGL(k_gain, dim3(blocks(np)), dim3(kBlock), 0, s, keys.data(), psum.data(), np, c, base, self,
                     old_sum.data(), a, present, k, S.m, S.gamma, gains.data());
  CGX_LAUNCH_CHECK();
  dbuf<uint32_t> uu(nr, s);
  auto ukeys = rocprim::make_transform_iterator(keys.data(), key_hi());
  int64_t nu = reduce_by_key(ukeys, gains.data(), (size_t)np, uu.data(), best.data(), best_gain_op(),
                             rocprim::equal_to<uint32_t>(), s);
  hipLaunchKernelGGL(k_move, dim3(blocks(nu)), dim3(kBlock), 0, s, uu.data(), best.data(), nu, c, base, next, up_down);
  CGX_LAUNCH_CHECK();
  (void)nv;
}

// Per-level schedule of the local move (the level graph is fixed across its
// sweeps): rows of degree <= kHashEdges go to the LDS-hash kernel in chunks of
// whole rows; heavier rows (the RMAT hubs, a prefix when rows are in descending
// degree order as contraction numbers them) keep the sort path over their own edges.
struct sweep_plan {
  bool hash       = false;
  int64_t e_big   = 0;  // edges of the rows on the sort path
  uint32_t const* bsrc = nullptr;
  uint32_t const* bdst = nullptr;
  double const* bw     = nullptr;
  dbuf<uint32_t> gsrc, gdst;  // big rows gathered, when they are not a prefix
  dbuf<double> gw;
  dbuf<int64_t> chunks;
  int64_t nchunks = 0;
  double scale = 0, inv_scale = 0;
  int64_t const* off = nullptr;  // the level's row offsets
  // heavy rows on the LDS two-pass path (k_big_*); big_hash false: sort path
  bool big_hash = false;
  int64_t nbig = 0, nsegs = 0, nbblocks = 0;
  dbuf<big_row> brows;
  dbuf<big_seg> bsegs;
  dbuf<big_bblk> bblocks;
  dbuf<u64> own, best_q;
  dbuf<uint32_t> best_c, pkey;
  dbuf<u64> pval;
  dbuf<int32_t> boffs;
  dbuf<int> overflow;
  std::vector<int64_t> big, big_first, big_deg;  // every heavy row (host; filled when a host plan needs them)
  dbuf<int64_t> bigd;                            // the heavy rows, ascending (device)
  dbuf<double> ag;                               // the sweep's gain weights (k_gain_weights)
  int64_t tb = 0;
};

// the heavy rows' (row, first edge, degree) on the host, for the host plan and the
// sort-path fallback
inline void big_rows_to_host(hipStream_t s, sweep_plan& P)
{
  if (P.tb == 0 || !P.big.empty()) return;
  dbuf<int64_t> fd(P.tb, s), dd(P.tb, s);
  hipLaunchKernelGGL(k_big_info, dim3(grid_for(P.tb, kBlock, 16384)), dim3(kBlock), 0, s, P.bigd.data(), P.off, P.tb,
                     fd.data(), dd.data());
  CGX_LAUNCH_CHECK();
  P.big       = to_host(P.bigd.data(), (size_t)P.tb, s);
  P.big_first = to_host(fd.data(), (size_t)P.tb, s);
  P.big_deg   = to_host(dd.data(), (size_t)P.tb, s);
}

// tuning_t::louvain_big_cap: lower the (row, bucket) table cap (tests of the fallback)
inline int big_bucket_cap(tuning_t const& tu)
{
  int const v = tu.louvain_big_cap;
  return v > 0 && v < kBktCap ? v : kBktCap;
}

inline int ceil_log2(int64_t x)
{
  int l = 0;
  while ((1ll << l) < x) ++l;
  return l;
}

// the heavy rows the LDS passes take; returns the others (sort path)
std::vector<int64_t> plan_big_rows(hipStream_t s, sweep_plan& P, tuning_t const& tu)
{
  std::vector<int64_t> const& big = P.big;
  std::vector<int64_t> rest;
  std::vector<big_row> rows;
  std::vector<big_seg> segs;
  std::vector<big_bblk> bb;
  int64_t pstart = 0, boff = 0;
  int64_t const md     = tu.louvain_big_maxdeg;  // tests: a lower limit
  int64_t const maxdeg = std::min<int64_t>(md > 0 ? md : INT64_MAX, (int64_t)kBigMaxBuckets * kBktCap * 4 / 5);
  for (size_t q = 0; q < big.size(); ++q) {
    int64_t const r = big[q], first = P.big_first[q], d = P.big_deg[q];
    int64_t const nseg  = (d + kBigSeg - 1) / kBigSeg;
    if (nseg > kBigMaxSegs || d > maxdeg) {
      rest.push_back(r);  // a bucket could outgrow its table
      continue;
    }
    int64_t const j = (int64_t)rows.size();
    rows.emplace_back();
    bool const single = nseg == 1;
    int const logb    = single ? 0 : std::min(ceil_log2((d + kBigPerBucket - 1) / kBigPerBucket), ceil_log2(kBigMaxBuckets));
    big_row& rw = rows[j];
    rw.first    = first;
    rw.row      = (uint32_t)r;
    rw.logb     = (uint32_t)logb;
    rw.sbeg     = (uint32_t)segs.size();
    rw.bbeg     = (uint32_t)bb.size();
    for (int64_t q = 0; q < nseg; ++q) {
      big_seg sg;
      sg.e0    = first + q * kBigSeg;
      sg.e1    = std::min(first + d, sg.e0 + kBigSeg);
      sg.pbase = pstart + q * kBigSeg;
      sg.boff  = boff;
      sg.j     = (uint32_t)j;
      sg.pad   = 0;
      if (!single) boff += (1 << logb) + 1;
      segs.push_back(sg);
    }
    rw.send   = (uint32_t)segs.size();
    rw.single = single ? 1u : 0u;
    if (!single)
      for (int b = 0; b < (1 << logb); ++b)
        bb.push_back(big_bblk{segs[rw.sbeg].boff, segs[rw.sbeg].pbase, (uint32_t)j, (uint32_t)r, (uint32_t)b,
                              (uint32_t)nseg, (uint32_t)logb, 0u});
    pstart += d;
  }
  int64_t const nb = (int64_t)rows.size();
  if (nb == 0) return rest;
  P.nbig     = nb;
  P.nsegs    = (int64_t)segs.size();
  P.nbblocks = (int64_t)bb.size();
  P.brows.resize(nb, s);
  P.bsegs.resize(P.nsegs, s);
  P.bblocks.resize(P.nbblocks, s);
  to_device(P.brows.data(), rows.data(), nb, s);
  to_device(P.bsegs.data(), segs.data(), P.nsegs, s);
  to_device(P.bblocks.data(), bb.data(), P.nbblocks, s);
  P.own.resize(nb, s);
  P.best_q.resize(P.nbblocks, s);
  P.best_c.resize(P.nbblocks, s);
  P.pkey.resize(pstart, s);
  P.pval.resize(pstart, s);
  P.boffs.resize(boff, s);
  P.overflow.resize(1, s);
  HIP_CHECK(hipStreamSynchronize(s));  // host vectors go out of scope
  P.big_hash = true;
  return rest;
}

// plan_big_rows on the device (k_big_plan); false: some heavy row needs the sort path,
// and nothing was planned (the caller runs the host plan)
bool plan_big_rows_device(hipStream_t s, sweep_plan& P, tuning_t const& tu)
{
  int64_t const n = P.tb;
  if (n == 0) return true;
  int64_t const md     = tu.louvain_big_maxdeg;
  int64_t const maxdeg = std::min<int64_t>(md > 0 ? md : INT64_MAX, (int64_t)kBigMaxBuckets * kBktCap * 4 / 5);
  dbuf<u64> cnt(4 * (n + 1), s), pos(4 * (n + 1), s);
  dbuf<int> rest(1, s);
  fill<int>(rest.data(), 1, 0, s);
  unsigned const g = grid_for(n, kBlock, 16384);
  hipLaunchKernelGGL(k_big_plan, dim3(g), dim3(kBlock), 0, s, P.bigd.data(), P.off, n, maxdeg, 0, cnt.data(),
                     (u64 const*)nullptr, (big_row*)nullptr, (big_seg*)nullptr, (big_bblk*)nullptr, rest.data());
  CGX_LAUNCH_CHECK();
  for (int q = 0; q < 4; ++q)
    exclusive_scan<u64, u64>(cnt.data() + q * (n + 1), pos.data() + q * (n + 1), (size_t)(n + 1), s);
  // one read: the four totals and the rest flag
  dbuf<u64> tot(5, s);
  hipLaunchKernelGGL(k_plan_totals, dim3(1), dim3(64), 0, s, pos.data(), n, rest.data(), tot.data());
  CGX_LAUNCH_CHECK();
  auto const t = to_host(tot.data(), 5, s);
  if (t[4]) return false;
  P.nbig     = n;
  P.nsegs    = (int64_t)t[0];
  P.nbblocks = (int64_t)t[1];
  P.brows.resize(n, s);
  P.bsegs.resize(P.nsegs, s);
  P.bblocks.resize(std::max<int64_t>(P.nbblocks, 1), s);
  hipLaunchKernelGGL(k_big_plan, dim3(g), dim3(kBlock), 0, s, P.bigd.data(), P.off, n, maxdeg, 1, (u64*)nullptr,
                     pos.data(), P.brows.data(), P.bsegs.data(), P.bblocks.data(), rest.data());
  CGX_LAUNCH_CHECK();
  P.own.resize(n, s);
  P.best_q.resize(std::max<int64_t>(P.nbblocks, 1), s);
  P.best_c.resize(std::max<int64_t>(P.nbblocks, 1), s);
  P.pkey.resize(std::max<u64>(t[3], 1), s);
  P.pval.resize(std::max<u64>(t[3], 1), s);
  P.boffs.resize(std::max<u64>(t[2], 1), s);
  P.overflow.resize(1, s);
  HIP_CHECK(hipStreamSynchronize(s));  // cnt / pos / rest / tot go out of scope
  P.big_hash = true;
  return true;
}

// the edges of `rows` for the sort path: the level COO itself when they are a
// prefix of the rows, else gathered
void build_sort_coo(hipStream_t s, level_graph const& g, sweep_plan& P, std::vector<int64_t> const& rows)
{
  int64_t const nb = (int64_t)rows.size();
  P.e_big          = 0;
  if (nb == 0) return;
  std::vector<int64_t> first(nb), pos(nb + 1, 0);
  bool prefix = true;
  for (int64_t j = 0; j < nb; ++j) {
    size_t const q = (size_t)(std::lower_bound(P.big.begin(), P.big.end(), rows[j]) - P.big.begin());
    first[j]       = P.big_first[q];
    pos[j + 1]     = pos[j] + P.big_deg[q];
    prefix         = prefix && rows[j] == j;
  }
  P.e_big = pos[nb];
  if (prefix) {
    P.bsrc = g.src.data();
    P.bdst = g.dst.data();
    P.bw   = g.w.data();
    return;
  }
  dbuf<int64_t> fd(nb, s), pd(nb + 1, s);
  to_device(fd.data(), first.data(), nb, s);
  to_device(pd.data(), pos.data(), nb + 1, s);
  P.gsrc.resize(P.e_big, s);
  P.gdst.resize(P.e_big, s);
  P.gw.resize(P.e_big, s);
  hipLaunchKernelGGL(k_gather_rows, dim3(blocks(P.e_big)), dim3(kBlock), 0, s, fd.data(), pd.data(), nb, g.src.data(),
                     g.dst.data(), g.w.data(), P.e_big, P.gsrc.data(), P.gdst.data(), P.gw.data());
  CGX_LAUNCH_CHECK();
  HIP_CHECK(hipStreamSynchronize(s));  // fd / pd go out of scope
  P.bsrc = P.gsrc.data();
  P.bdst = P.gdst.data();
  P.bw   = P.gw.data();
}

// stats: vertex_weights' (negative-weight flag, largest row weight) of this level
void plan_sweeps(louvain_state& S, level_graph const& g, int64_t const* off, u64 const* stats, sweep_plan& P)
{
  hipStream_t s    = S.s;
  int64_t const nr = g.nrows, ne = g.ne;
  if (ne == 0 || nr == 0 || !S.tune.louvain_hash) return;  // (louvain_hash = 0: sort path only, A/B)
  auto sh = to_host(stats, 2, s);
  if (sh[0]) return;  // negative weights: the fixed-point sums assume w >= 0
  double kmax;
  std::memcpy(&kmax, &sh[1], sizeof(double));
  if (!(kmax < 1e300)) return;
  int const e = kmax > 0 ? std::ilogb(kmax) + 1 : 0;  // every row weight < 2^e
  P.scale     = std::ldexp(1.0, 61 - e);
  P.inv_scale = std::ldexp(1.0, e - 61);

  int64_t const nblk = (nr + kHashRows - 1) / kHashRows;
  dbuf<uint32_t> cc(nblk, s), bc(nblk, s);
  dbuf<int64_t> cp(nblk + 1, s), bp(nblk + 1, s);
  unsigned const wg = grid_for(nblk, kBlock, 16384);
  hipLaunchKernelGGL(k_chunk_walk, dim3(wg), dim3(kBlock), 0, s, off, nr, 0, cc.data(), bc.data(), nullptr, nullptr,
                     nullptr, nullptr);
  CGX_LAUNCH_CHECK();
  exclusive_scan<uint32_t, int64_t>(cc.data(), cp.data(), (size_t)nblk, s);
  exclusive_scan<uint32_t, int64_t>(bc.data(), bp.data(), (size_t)nblk, s);
  dbuf<int64_t> tot(2, s);
  hipLaunchKernelGGL(k_walk_totals, dim3(1), dim3(64), 0, s, cp.data(), cc.data(), bp.data(), bc.data(), nblk,
                     tot.data());
  CGX_LAUNCH_CHECK();
  auto const th    = to_host(tot.data(), 2, s);
  int64_t const tc = th[0], tb = th[1];
  P.nchunks        = tc;
  P.chunks.resize(std::max<int64_t>(4 * tc, 1), s);
  P.bigd.resize(std::max<int64_t>(tb, 1), s);
  P.tb = tb;
  hipLaunchKernelGGL(k_chunk_walk, dim3(wg), dim3(kBlock), 0, s, off, nr, 1, cc.data(), bc.data(), cp.data(), bp.data(),
                     P.chunks.data(), P.bigd.data());
  CGX_LAUNCH_CHECK();
  P.off = off;
  // (louvain_big_hash = 0: heavy rows on the sort path, A/B)
  if (!S.tune.louvain_big_hash || !plan_big_rows_device(s, P, S.tune)) {
    big_rows_to_host(s, P);
    build_sort_coo(s, g, P, S.tune.louvain_big_hash ? plan_big_rows(s, P, S.tune) : P.big);
  }
  HIP_CHECK(hipStreamSynchronize(s));  // the walk's scratch goes out of scope
  P.hash = true;
  if (S.trace && tb > 0) {  // heavy rows by degree (measurement only)
    dbuf<int64_t> first(tb, s), deg(tb, s);
    hipLaunchKernelGGL(k_big_info, dim3(grid_for(tb, kBlock, 16384)), dim3(kBlock), 0, s, P.bigd.data(), P.off, tb,
                       first.data(), deg.data());
    CGX_LAUNCH_CHECK();
    auto const hd = to_host(deg.data(), (size_t)tb, s);
    int64_t const lim[6] = {2048, 4096, 8192, 32768, 262144, INT64_MAX};
    int64_t rows[6] = {}, edges[6] = {};
    for (int64_t d : hd) {
      int b = 0;
      while (d > lim[b]) ++b;
      ++rows[b];
      edges[b] += d;
    }
    std::fprintf(stderr, "[louvain] plan: %lld hash chunks, %lld heavy rows (%lld segments, %lld bucket blocks); "
                         "heavy rows / edges by degree <=2K %lld/%lld <=4K %lld/%lld <=8K %lld/%lld <=32K %lld/%lld "
                         "<=256K %lld/%lld more %lld/%lld\n",
                 (long long)P.nchunks, (long long)tb, (long long)P.nsegs, (long long)P.nbblocks, (long long)rows[0],
                 (long long)edges[0], (long long)rows[1], (long long)edges[1], (long long)rows[2], (long long)edges[2],
                 (long long)rows[3], (long long)edges[3], (long long)rows[4], (long long)edges[4], (long long)rows[5],
                 (long long)edges[5]);
  }
}

__global__ void k_gain_weights(double const* a, uint8_t const* present, int64_t n, double* ag)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    ag[i] = present[i] ? a[i] : (double)FLT_MAX;
}

// one synchronous local-move sweep (update_clustering_by_delta_modularity) over
// this rank's rows; next[row] = the row's cluster after the sweep
void sweep(louvain_state& S, level_graph const& g, sweep_plan& P, uint32_t const* c, uint32_t* next,
           double const* k, double const* self, double const* a, uint8_t const* present, int64_t na, bool up_down,
           double* own)
{
  hipStream_t s = S.s;
  if (g.nrows) {
    HIP_CHECK(hipMemcpyAsync(next, c + g.base, g.nrows * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    fill<double>(own, g.nrows, 0.0, s);
  }
  if (g.ne == 0) return;
  if (!P.hash) {
    sweep_sorted(S, g, g.src.data(), g.dst.data(), g.w.data(), g.ne, c, next, k, self, a, present, up_down, own);
    return;
  }
  // the gain weights of this sweep's clusters: one 8-byte gather per (row, cluster)
  // pair where a and present took two
  if (P.ag.n < (size_t)std::max<int64_t>(na, 1)) P.ag.resize(std::max<int64_t>(na, 1), s);
  if (na) hipLaunchKernelGGL(k_gain_weights, dim3(blocks(na)), dim3(kBlock), 0, s, a, present, na, P.ag.data());
  CGX_LAUNCH_CHECK();
  if (P.big_hash) {
    big_args ba{g.dst.data(), g.w.data(), g.wf, c, (uint32_t)g.base, P.bsegs.data(), P.brows.data(), P.nbig, P.pkey.data(),
                P.pval.data(), P.boffs.data(), P.own.data(), P.bblocks.data(), self, a, P.ag.data(), k, S.m, S.gamma,
                P.scale, P.inv_scale, P.best_q.data(), P.best_c.data(), P.overflow.data(), big_bucket_cap(S.tune), next,
                up_down, own};
    fill<u64>(P.own.data(), P.nbig, 0ull, s);
    fill<int>(P.overflow.data(), 1, 0, s);
    hipLaunchKernelGGL(k_big_partials, dim3((unsigned)P.nsegs), dim3(kBigThreads), 0, s, ba);
    CGX_LAUNCH_CHECK();
    if (P.nbblocks) hipLaunchKernelGGL(k_big_buckets, dim3((unsigned)P.nbblocks), dim3(kBktThreads), 0, s, ba);
    CGX_LAUNCH_CHECK();
    // moves nothing when a bucket outgrew its table (the flag is read after the sweep:
    // no host round trip between the heavy and the light rows)
    hipLaunchKernelGGL(k_big_move, dim3(blocks(P.nbig)), dim3(kBlock), 0, s, ba);
    CGX_LAUNCH_CHECK();
  }
  if (P.e_big)
    sweep_sorted(S, g, P.bsrc, P.bdst, P.bw, P.e_big, c, next, k, self, a, present, up_down, own);
  if (P.nchunks) {
    hash_sweep_args ha{g.dst.data(), g.w.data(), g.wf, P.off, P.chunks.data(), P.nchunks, c, (uint32_t)g.base,
                       self, a, P.ag.data(), k, S.m, S.gamma, P.scale, P.inv_scale, next, up_down, own};
    // persistent blocks: the resident count (5 per CU at 30 KB of LDS with fp32 weights,
    // 4 with fp64 weights (registers) or 64-bit keys (38 KB of LDS))
    int64_t const cus  = device_cu_count();
    unsigned const hg  = (unsigned)std::min<int64_t>(P.nchunks, (int64_t)(g.wf ? kHashResident : kHashResident - 1) * cus);
    unsigned const hgw = (unsigned)std::min<int64_t>(P.nchunks, (int64_t)(kHashResident - 1) * cus);  // 38 KB
    bool const wide = S.tune.louvain_wide_keys;  // tests of the 64-bit keys
    if (g.nv < (1 << 24) - 1 && !wide) {
      if (g.wf) hipLaunchKernelGGL((k_sweep_hash<uint32_t, float>), dim3(hg), dim3(kHashThreads), 0, s, ha);
      else hipLaunchKernelGGL((k_sweep_hash<uint32_t, double>), dim3(hg), dim3(kHashThreads), 0, s, ha);
    } else {
      if (g.wf) hipLaunchKernelGGL((k_sweep_hash<u64, float>), dim3(hgw), dim3(kHashThreads), 0, s, ha);
      else hipLaunchKernelGGL((k_sweep_hash<u64, double>), dim3(hgw), dim3(kHashThreads), 0, s, ha);
    }
    CGX_LAUNCH_CHECK();
  }
  if (P.big_hash && to_host_scalar(P.overflow.data(), s) != 0) {
    // a bucket outgrew its table: this level's heavy rows take the sort path, and the
    // sweep runs again from the start (never seen on R-MAT)
    P.big_hash = false;
    big_rows_to_host(s, P);
    build_sort_coo(s, g, P, P.big);
    sweep(S, g, P, c, next, k, self, a, present, na, up_down, own);
  }
}

// fixed-point vertex weights of the rows: K = rint(k * scale)
__global__ void k_to_fixed(double const* k, int64_t n, double scale, long long* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = __double2ll_rn(k[i] * scale);
}

// the sweep's cluster weights and present flags from the owners' answers
__global__ void k_cluster_vals(long long const* afix, int const* pcnt, int64_t n, double inv, int all_present,
                               double* a, uint8_t* present)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    a[i]       = (double)afix[i] * inv;
    present[i] = (all_present || pcnt[i] > 0) ? 1 : 0;
  }
}

// single GPU: the moves' fixed-point weight deltas (every moved vertex takes its K
// and its has-edges count from the old cluster to the new one; integer adds, so the
// totals do not depend on the order of the atomics)
__global__ void k_apply_moves(uint32_t const* old_c, uint32_t const* new_c, int64_t n, long long const* kfix,
                              uint8_t const* has_edges, long long* afix, int* pcnt)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const o = old_c[v], c = new_c[v];
    if (o == c) continue;
    unsigned long long const kv = (unsigned long long)kfix[v];
    atomicAdd(reinterpret_cast<unsigned long long*>(afix + o), 0ull - kv);
    atomicAdd(reinterpret_cast<unsigned long long*>(afix + c), kv);
    if (has_edges[v]) {
      atomicSub(pcnt + o, 1);
      atomicAdd(pcnt + c, 1);
    }
  }
}

// contract the level graph by `labels` (graph_contraction / coarsen_graph): sum
// parallel edges, renumber the used labels by descending coarse out-degree
// (stable: ties by ascending label), relabel the dendrogram level in place
level_graph contract(louvain_state& S, level_graph const& g, uint32_t* labels)
{
  hipStream_t s = S.s;
  int64_t nv = g.nv, ne = g.ne;
  // the used labels' dense ranks first (order-preserving, so every sort order and tie
  // below is the labels' own): the pair keys need bits for the used labels only
  // (RMAT-26 level 0: 22 instead of 25, one radix pass fewer in each sort)
  dbuf<uint32_t> used(nv + 1, s), pos(nv + 1, s);
  fill<uint32_t>(used.data(), nv + 1, 0u, s);
  hipLaunchKernelGGL(k_mark_used, dim3(blocks(nv)), dim3(kBlock), 0, s, labels, nv, used.data());
  CGX_LAUNCH_CHECK();
  exclusive_scan<uint32_t, uint32_t>(used.data(), pos.data(), nv + 1, s);
  int64_t const nu = (int64_t)to_host_scalar(pos.data() + nv, s);
  hipLaunchKernelGGL(k_gather_u32, dim3(blocks(nv)), dim3(kBlock), 0, s, pos.data(), labels, nv);  // label -> rank
  CGX_LAUNCH_CHECK();
  used.free();
  pos.free();
  dbuf<u64> keys(std::max<int64_t>(ne, 1), s), keys2(std::max<int64_t>(ne, 1), s);
  dbuf<double> cw(std::max<int64_t>(ne, 1), s);
  int64_t nce = 0;
  if (ne) {
    int const cb = bits_for((unsigned long long)std::max<int64_t>(nu - 1, 0));
    hipLaunchKernelGGL(k_pair_keys, dim3(blocks(ne)), dim3(kBlock), 0, s, g.src.data(), g.dst.data(), labels, ne, cb,
                       keys.data());
    CGX_LAUNCH_CHECK();
    if (g.wf) {  // fp32 level-0 weights ride the sort as fp32 (12 B a pair); sums in fp64 as before
      dbuf<float> w2(ne, s);
      radix_sort_pairs<u64, float>(keys.data(), keys2.data(), g.wf, w2.data(), (size_t)ne, 0, 2 * cb, s);
      nce = reduce_by_key(keys2.data(), w2.data(), (size_t)ne, keys.data(), cw.data(), rocprim::plus<double>(),
                          rocprim::equal_to<u64>(), s);
    } else {
      dbuf<double> w2(ne, s);
      radix_sort_pairs<u64, double>(keys.data(), keys2.data(), g.w.data(), w2.data(), (size_t)ne, 0, 2 * cb, s);
      nce = reduce_by_key(keys2.data(), w2.data(), (size_t)ne, keys.data(), cw.data(), rocprim::plus<double>(),
                          rocprim::equal_to<u64>(), s);
    }
    hipLaunchKernelGGL(k_expand_keys, dim3(blocks(nce)), dim3(kBlock), 0, s, keys.data(), nce, cb);
    CGX_LAUNCH_CHECK();
  }
  // the ranks' coarse out-degrees; new ids by descending degree, ties by ascending rank
  dbuf<uint32_t> deg(std::max<int64_t>(nu, 1), s), udeg2(std::max<int64_t>(nu, 1), s), uniq(std::max<int64_t>(nu, 1), s),
    nmap(std::max<int64_t>(nu, 1), s), nl(std::max<int64_t>(nu, 1), s);
  fill<uint32_t>(deg.data(), nu, 0u, s);
  if (nce)
    hipLaunchKernelGGL(k_count_src, dim3(blocks(nu)), dim3(kBlock), 0, s, keys.data(), nce, (int64_t)0, nu,
                       deg.data());
  CGX_LAUNCH_CHECK();
  iota<uint32_t>(uniq.data(), nu, 0u, s);
  radix_sort_pairs<uint32_t, uint32_t>(deg.data(), udeg2.data(), uniq.data(), nmap.data(), (size_t)nu, 0,
                                       bits_for((unsigned long long)std::max<int64_t>(nce, 1)), s, /*descending=*/true);
  hipLaunchKernelGGL(k_new_ids, dim3(blocks(nu)), dim3(kBlock), 0, s, nmap.data(), nu, nl.data());
  CGX_LAUNCH_CHECK();
  level_graph out;
  out.nv    = nu;
  out.nrows = nu;
  out.ne    = nce;
  out.src.resize(std::max<int64_t>(nce, 1), s);
  out.dst.resize(std::max<int64_t>(nce, 1), s);
  out.w.resize(std::max<int64_t>(nce, 1), s);
  if (nce) {
    int const cb2 = bits_for((unsigned long long)std::max<int64_t>(nu - 1, 0));
    hipLaunchKernelGGL(k_relabel_pairs, dim3(blocks(nce)), dim3(kBlock), 0, s, keys.data(), nce, nl.data(), cb2,
                       keys2.data());
    CGX_LAUNCH_CHECK();
    radix_sort_pairs<u64, double>(keys2.data(), keys.data(), cw.data(), out.w.data(), (size_t)nce, 0, 2 * cb2, s);
    hipLaunchKernelGGL(k_split_pairs, dim3(blocks(nce)), dim3(kBlock), 0, s, keys.data(), nce, out.src.data(),
                       out.dst.data(), cb2);
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
  louvain_state S(s, h.tune);
  S.gamma = resolution;
  level_graph cur;
  cur.nv    = nv0;
  cur.nrows = nv0;
  cur.ne    = g.num_edges;
  cur.src.resize(std::max<int64_t>(cur.ne, 1), s);
  cur.dst.resize(std::max<int64_t>(cur.ne, 1), s);
  cur.w.resize(std::max<int64_t>(cur.ne, 1), s);
  if (cur.ne) {
    dbuf<uint32_t> marks(cur.ne, s);
    fill<uint32_t>(marks.data(), cur.ne, 0u, s);
    hipLaunchKernelGGL((k_row_starts<E>), dim3(blocks(nv0)), dim3(kBlock), 0, s, adj.offsets.data<E>(), nv0,
                       marks.data());
    CGX_LAUNCH_CHECK();
    size_t tmp = 0;
    HIP_CHECK(rocprim::inclusive_scan(nullptr, tmp, marks.data(), cur.src.data(), (size_t)cur.ne,
                                      rocprim::maximum<uint32_t>(), s));
    buffer t(tmp, s);
    HIP_CHECK(rocprim::inclusive_scan(t.data(), tmp, marks.data(), cur.src.data(), (size_t)cur.ne,
                                      rocprim::maximum<uint32_t>(), s));
    hipLaunchKernelGGL((k_expand_cols<V, R>), dim3(blocks(cur.ne)), dim3(kBlock), 0, s, adj.indices.data<V>(),
                       adj.weights.data<R>(), cur.ne, cur.dst.data(), cur.w.data());
    CGX_LAUNCH_CHECK();
  }
  // fp32 input: level 0's hash sweeps read the adjacency's own fp32 weights (edge order
  // is the adjacency's; the fp64 values are the same numbers)
  if constexpr (std::is_same_v<R, float>) cur.wf = cur.ne ? adj.weights.data<float>() : nullptr;
  device_sum(plain_f{cur.w.data()}, (size_t)cur.ne, S.scal.data(), S.scratch.data(), s);
  S.m = to_host_scalar(S.scal.data(), s);  // total edge weight (constant over levels)

  std::vector<dbuf<uint32_t>> dendrogram;
  double best_q = -1.0;
  bool const trace = std::getenv("CGX_LOUVAIN_TRACE") != nullptr;  // measurement only
  S.trace          = trace;
  auto t_last      = std::chrono::steady_clock::now();
  auto lap         = [&](char const* what, int64_t nv, int64_t ne, double q) {
    if (!trace) return;
    auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[louvain] %-9s nv=%lld ne=%lld q=%.6f %.2f ms\n", what, (long long)nv, (long long)ne, q,
                 std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };
  lap("start", cur.nv, cur.ne, 0.0);
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
    dbuf<u64> vstats(2, s);
    vertex_weights(S, cur, off.data(), k.data(), self.data(), has_edges.data(), vstats.data());
    // Cluster weights in 64-bit fixed point, as the multi-GPU owners keep them (scale
    // 2^(60 - e), the total weight < 2^e): every move adds its vertex's K to the new
    // cluster and takes it from the old one (k_apply_moves), integer adds that give
    // the same totals in any order -- one pass over the vertices per sweep where the
    // re-summation sorted every vertex by cluster (~0.3 ms a sweep at RMAT-23).  a and
    // present are read off them; the first sweep sees every vertex present.
    int const ea        = S.m > 0 ? std::ilogb(S.m) + 1 : 0;
    double const ascale = std::ldexp(1.0, 60 - ea), ainv = std::ldexp(1.0, ea - 60);
    dbuf<long long> kfix(nv, s), afix(nv, s);
    dbuf<int> pcnt(nv, s);
    hipLaunchKernelGGL(k_to_fixed, dim3(blocks(nv)), dim3(kBlock), 0, s, k.data(), nv, ascale, kfix.data());
    CGX_LAUNCH_CHECK();
    HIP_CHECK(hipMemcpyAsync(afix.data(), kfix.data(), nv * sizeof(long long), hipMemcpyDeviceToDevice, s));
    convert<int, uint8_t>(pcnt.data(), has_edges.data(), nv, s);
    hipLaunchKernelGGL(k_cluster_vals, dim3(blocks(nv)), dim3(kBlock), 0, s, afix.data(), pcnt.data(), nv, ainv, 1,
                       a.data(), present.data());
    CGX_LAUNCH_CHECK();
    dbuf<uint32_t> clusters(nv, s), next(nv, s);
    iota<uint32_t>(clusters.data(), nv, 0u, s);
    sweep_plan plan;
    plan_sweeps(S, cur, off.data(), vstats.data(), plan);
    dbuf<double> own(nv, s);
    // every sweep also returns the internal weight of the clustering it started from
    // (modularity_own): sweep k + 1 runs before the loop decides on clustering k
    bool up_down = true;
    sweep(S, cur, plan, clusters.data(), next.data(), k.data(), self.data(), a.data(), present.data(), nv, up_down,
          own.data());
    double new_q = modularity_own(S, cur, own.data(), a.data(), present.data());
    lap("setup", nv, cur.ne, new_q);
    double cur_q = new_q - 1.0;
    while (new_q > cur_q + 0.0001) {
      cur_q = new_q;
      hipLaunchKernelGGL(k_apply_moves, dim3(blocks(nv)), dim3(kBlock), 0, s, clusters.data(), next.data(), nv,
                         kfix.data(), has_edges.data(), afix.data(), pcnt.data());
      CGX_LAUNCH_CHECK();
      std::swap(clusters, next);
      hipLaunchKernelGGL(k_cluster_vals, dim3(blocks(nv)), dim3(kBlock), 0, s, afix.data(), pcnt.data(), nv, ainv, 0,
                         a.data(), present.data());
      CGX_LAUNCH_CHECK();
      up_down = !up_down;
      sweep(S, cur, plan, clusters.data(), next.data(), k.data(), self.data(), a.data(), present.data(), nv, up_down,
            own.data());
      new_q = modularity_own(S, cur, own.data(), a.data(), present.data());
      if (new_q > cur_q)
        HIP_CHECK(hipMemcpyAsync(level, clusters.data(), nv * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
      lap("sweep", nv, cur.ne, new_q);
    }
    if (cur_q <= best_q) break;
    best_q = cur_q;
    // the level's sweep state goes before the contraction's sort buffers are allocated
    plan = sweep_plan{};
    for (auto* b : {&own, &k, &self, &a}) b->free();
    kfix.free();
    afix.free();
    pcnt.free();
    for (auto* b : {&clusters, &next}) b->free();
    has_edges.free();
    present.free();
    off.free();
    cur = contract(S, cur, level);
    lap("contract", cur.nv, cur.ne, best_q);
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
  for (auto& lvl : dendrogram) {
    res.levels.push_back(std::make_unique<device_array_t>(lvl.n, g.vertex_type, s));
    hipLaunchKernelGGL(k_to_vertex<V>, dim3(blocks(lvl.n)), dim3(kBlock), 0, s, lvl.data(), (int64_t)lvl.n,
                       res.levels.back()->buf.data<V>());
    CGX_LAUNCH_CHECK();
  }
  HIP_CHECK(hipStreamSynchronize(s));
  res.modularity        = best_q;
  h.last_louvain_levels = dendrogram.size();
}

// ================================================================ multi-GPU
//
// Reference: louvain_impl.cuh:46-237 with multi_gpu = true, the MG branches of
// common_methods.cuh:200-382 (cluster weights kept at the key owner,
// louvain_impl.cuh:91-103; the neighbour clusters' weights collected from their
// owners, per_v_transform_reduce_dst_key_aggregated_outgoing_e.cuh:506-611,736-753)
// and coarsen_graph_impl.cuh:243-516 (coarse edges shuffled to the owner of their
// source, renumbered per owner).  The MI355X layout (owner-sharded, no O(V) state
// or collective per rank):
//
//  * rows: every rank holds the out-edges of the vertices it owns ([voff[p],
//    voff[p+1]) of the level's global ids, a 1D partition by source owner),
//    sorted by (row, destination) with fp64 weights.  Per level the destinations
//    become local ids: own rows [0, nr), then the ghosts (distinct remote
//    destinations, sorted), so the single-GPU sweep kernels run unchanged;
//  * clusters: every rank keeps the clusters of its rows and of its ghosts; the
//    owners know which of their rows each rank mirrors (one exchange per level);
//  * cluster weights: at the owner of the cluster id, in 64-bit fixed point (scale
//    2^(60 - e), total weight < 2^e: integer adds, order-free and exact for
//    integer weights), with a count of members that have edges (present flag);
//  * a sweep: the referenced clusters (own rows' and ghosts') are collected from
//    their owners (keys out, values back), the single-GPU local move runs on local
//    cluster ids (order-preserving, so the tie rule on cluster ids is unchanged);
//    then the moved rows send (old, -k) / (new, +k) to the cluster owners and the
//    owners send the moved rows' new clusters to the ranks that mirror them.
//    Per-sweep traffic per rank: O(referenced clusters + moved rows + their
//    mirrors), reported per sweep (CGX_LOUVAIN_TRACE) and as the handle statistic
//    last_louvain_sweep_bytes;
//  * modularity: per-rank partials (own internal weight, own cluster ids' a_c^2)
//    and a 2-double allreduce, so every rank takes the same branch of the level
//    loop;
//  * contraction: coarse pairs (label(u), label(v)) are reduced locally, sent to
//    the owner of label(u) and merged there; each owner numbers its used labels by
//    descending coarse degree (ties: ascending label), the owners' ranges stay
//    contiguous, and the new ids of label(v) and of the rows' labels are collected
//    from their owners (no dense label table);
//  * flatten: each level's owners answer for the ids the owned level-0 vertices
//    have reached.
//
// With one rank this is the single-GPU algorithm (same ids, same exact sums for
// integer weights).  With several, every decision is the single-GPU decision on the
// same (MG-numbered) level graph whenever the sums are exact (integer weights),
// which is what the reference's MG test checks level by level
// (mg_louvain_test.cpp:82-151).

template <typename V>
__global__ void k_owner_of_src(V const* src, int64_t n, int64_t const* voff, int P, int* dest)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dest[i] = mg_owner_of_global((int64_t)src[i], voff, P);
}

// first position of rank q's run in a sorted owner array, q = 0..P
__global__ void k_rank_bounds(int const* sorted, int64_t n, int P, int64_t* out)
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

// first position of keys with (key >> 32) >= voff[q], q = 0..P (keys sorted)
__global__ void k_key_bounds(u64 const* keys, int64_t n, int64_t const* voff, int P, int64_t* out)
{
  int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q > P) return;
  u64 const t = (u64)voff[q] << 32;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < t) lo = mid + 1;
    else hi = mid;
  }
  out[q] = lo;
}

template <typename V>
__global__ void k_mg_row_keys(V const* src, V const* dst, int64_t n, int64_t base, u64* keys)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    keys[i] = ((u64)((int64_t)src[i] - base) << 32) | (u64)(uint32_t)dst[i];
}


__global__ void k_new_ids_off(uint32_t const* nmap, int64_t n, uint32_t first, uint32_t* new_of_label)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    new_of_label[nmap[i]] = first + (uint32_t)i;
}

std::vector<int64_t> bounds_to_counts(dbuf<int64_t> const& b, int P, hipStream_t s)
{
  auto hb = to_host(b.data(), P + 1, s);
  std::vector<int64_t> c(P);
  for (int q = 0; q < P; ++q) c[q] = hb[q + 1] - hb[q];
  return c;
}

// level 0: the 2D block's edges -> rows of this rank's sources
template <typename V, typename R>
level_graph mg_level0(handle_t& h, graph_t& g)
{
  hipStream_t s = h.stream;
  mg_graph_t& mg = *g.mg;
  comm_t& comm   = *h.mg->world;
  int const P    = mg.P;
  dbuf<int64_t> voff_d(P + 1, s);
  HIP_CHECK(hipMemcpyAsync(voff_d.data(), mg.voff.data(), (P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  int64_t const ne = mg.ne, n1 = std::max<int64_t>(ne, 1);
  // Every temporary is released as soon as its last reader is enqueued (RMAT-26 on one
  // rank: 2.1G edges, 8-16 B each per array)
  dbuf<int64_t> bnd(P + 1, s), perm(n1, s);
  {
    dbuf<int> dest(n1, s), d2(n1, s);
    dbuf<int64_t> iv(n1, s);
    if (ne) {
      hipLaunchKernelGGL(k_owner_of_src<V>, dim3(blocks(ne)), dim3(kBlock), 0, s, mg.src.data<V>(), ne,
                         voff_d.data(), P, dest.data());
      CGX_LAUNCH_CHECK();
      iota<int64_t>(iv.data(), ne, 0, s);
      if (!radix_sort_pairs_db<int, int64_t>(dest.data(), d2.data(), iv.data(), perm.data(), ne, 0, bits_for(P), s)) {
        std::swap(dest, d2);  // sorted owners in d2, the permutation in perm
        std::swap(iv, perm);
      }
    }
    hipLaunchKernelGGL(k_rank_bounds, dim3(1), dim3(256), 0, s, d2.data(), ne, P, bnd.data());
    CGX_LAUNCH_CHECK();
  }
  auto c64 = bounds_to_counts(bnd, P, s);
  std::vector<size_t> counts(c64.begin(), c64.end()), rc;
  auto moved = [&](auto const* col, auto tag) {  // one column in owner order, exchanged
    using T = decltype(tag);
    dbuf<T> t(n1, s);
    if (ne) gather<T, int64_t>(t.data(), col, perm.data(), ne, s);
    return exchange<T>(comm, t.data(), counts, rc, s);
  };
  auto rs = moved(mg.src.data<V>(), V{});
  auto rd = moved(mg.dst.data<V>(), V{});
  auto rw = moved(mg.w.data<R>(), R{});
  perm.free();
  level_graph out;
  out.nv    = g.num_vertices;
  out.base  = mg.voff[mg.p];
  out.nrows = mg.n_own();
  out.ne    = (int64_t)rs.n;
  int64_t const m = out.ne, m1 = std::max<int64_t>(m, 1);
  out.src.resize(m1, s);
  out.dst.resize(m1, s);
  out.w.resize(m1, s);
  if (m) {
    dbuf<u64> k1(m, s), k2(m, s);
    hipLaunchKernelGGL(k_mg_row_keys<V>, dim3(blocks(m)), dim3(kBlock), 0, s, rs.data(), rd.data(), m, out.base,
                       k1.data());
    CGX_LAUNCH_CHECK();
    rs.free();
    rd.free();
    int const kb = 32 + bits_for(std::max<int64_t>(out.nrows - 1, 0));
    bool in1     = false;
    if constexpr (std::is_same_v<R, float>) {
      // fp32 input: the weights are sorted as fp32 and kept beside the fp64 copy, for
      // the level-0 hash sweeps (as the single-GPU level 0 reads the adjacency's)
      dbuf<float> f2(m, s);
      in1 = radix_sort_pairs_db<u64, float>(k1.data(), k2.data(), rw.data(), f2.data(), (size_t)m, 0, kb, s);
      out.wfbuf = std::move(in1 ? f2 : rw);
      out.wf    = out.wfbuf.data();
      convert<double, float>(out.w.data(), out.wf, m, s);
    } else {
      dbuf<double> w1(m, s);
      convert<double, R>(w1.data(), rw.data(), m, s);
      rw.free();
      in1 = radix_sort_pairs_db<u64, double>(k1.data(), k2.data(), w1.data(), out.w.data(), (size_t)m, 0, kb, s);
      if (!in1) std::swap(out.w, w1);
    }
    hipLaunchKernelGGL(k_split_pairs, dim3(blocks(m)), dim3(kBlock), 0, s, in1 ? k2.data() : k1.data(), m,
                       out.src.data(), out.dst.data(), /*cb=*/32);
    CGX_LAUNCH_CHECK();
  }
  return out;
}

// ---------------------------------------------------------------- owner-sharded state
// Every exchange of the sweep loop goes through these helpers, which also count the
// bytes this rank sends (S.sweep_bytes; per-sweep figure in DESIGN.md, trace
// CGX_LOUVAIN_TRACE=1, handle statistic last_louvain_sweep_bytes).
template <typename T>
dbuf<T> xchg(louvain_state& S, T const* send, std::vector<size_t> const& counts, std::vector<size_t>& rcounts)
{
  size_t n = 0;
  for (size_t q = 0; q < counts.size(); ++q)
    if ((int)q != S.comm->rank) n += counts[q];
  S.bytes += n * sizeof(T);
  return exchange<T>(*S.comm, send, counts, rcounts, S.s);
}

template <typename T>
dbuf<T> xchg_known(louvain_state& S, T const* send, std::vector<size_t> const& counts,
                   std::vector<size_t> const& rcounts)
{
  size_t n = 0;
  for (size_t q = 0; q < counts.size(); ++q)
    if ((int)q != S.comm->rank) n += counts[q];
  S.bytes += n * sizeof(T);
  return exchange_known<T>(*S.comm, send, counts, rcounts, S.s);
}

// first position of ids >= voff[q] in a sorted u32 array, q = 0..P
__global__ void k_id_bounds(uint32_t const* ids, int64_t n, int64_t const* voff, int P, int64_t* out)
{
  int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q > P) return;
  int64_t const t = voff[q];
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if ((int64_t)ids[mid] < t) lo = mid + 1;
    else hi = mid;
  }
  out[q] = lo;
}

// destinations outside this rank's rows [lo, lo + nr) -> their ids, others -> ~0u
__global__ void k_remote_ids(uint32_t const* dst, int64_t ne, uint32_t lo, uint32_t nr, uint32_t* out)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const d = dst[e];
    out[e]           = (d - lo < nr) ? ~0u : d;
  }
}

__device__ inline int64_t lower_bound_u32(uint32_t const* a, int64_t n, uint32_t x)
{
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// global destination -> local index: own rows [0, nr), ghosts nr + their position
// in the sorted ghost list
__global__ void k_localize(uint32_t* dst, int64_t ne, uint32_t lo, uint32_t nr, uint32_t const* ghost, int64_t ng)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const d = dst[e];
    dst[e]           = (d - lo < nr) ? d - lo : nr + (uint32_t)lower_bound_u32(ghost, ng, d);
  }
}

// owner side of a lookup: out[i] = table[key[i] - lo]
template <typename T>
__global__ void k_owner_gather(uint32_t const* key, int64_t n, uint32_t lo, T const* table, T* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = table[key[i] - lo];
}

__global__ void k_sub_u32(uint32_t* x, int64_t n, uint32_t lo)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] -= lo;
}

// sum over the owned cluster ids of a_c^2 (present clusters only)
struct sumsq_fixed_f {
  long long const* afix;
  int const* pcnt;
  double inv;
  int all_present;
  __device__ double operator()(int64_t i) const
  {
    double const a = (double)afix[i] * inv;
    return (all_present || pcnt[i] > 0) ? a * a : 0.0;
  }
};

// local clusters after the sweep -> global ids; moved rows flagged, the owners'
// weight deltas listed: (old cluster, -K, -has) and (new cluster, +K, +has) per move
__global__ void k_advance(uint32_t const* next_loc, uint32_t const* ref, int64_t nr, uint32_t* c_own,
                          uint8_t* moved)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nr; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const nc = ref[next_loc[i]];
    moved[i]          = nc != c_own[i];
    c_own[i]          = nc;
  }
}

__global__ void k_move_deltas(uint32_t const* old_c, uint32_t const* new_c, uint8_t const* moved,
                              uint32_t const* pos, int64_t nr, long long const* kfix, uint8_t const* has_edges,
                              uint32_t* key, long long* dk, int* dh)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nr; i += (int64_t)gridDim.x * blockDim.x) {
    if (!moved[i]) continue;
    int64_t const j = 2 * (int64_t)pos[i];
    key[j]          = old_c[i];
    dk[j]           = -kfix[i];
    dh[j]           = -(int)has_edges[i];
    key[j + 1]      = new_c[i];
    dk[j + 1]       = kfix[i];
    dh[j + 1]       = (int)has_edges[i];
  }
}

// owner side: apply the received weight deltas (integer adds: order-free)
__global__ void k_apply_deltas(uint32_t const* key, long long const* dk, int const* dh, int64_t n, uint32_t lo,
                               long long* afix, int* pcnt)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    atomicAdd(reinterpret_cast<unsigned long long*>(afix + (key[i] - lo)), (unsigned long long)dk[i]);
    atomicAdd(pcnt + (key[i] - lo), dh[i]);
  }
}

// mirror entries whose row moved -> flag (for the compaction of ghost updates)
__global__ void k_mirror_flags(uint32_t const* mir, int64_t n, uint8_t const* moved, uint32_t* flag)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = moved[mir[i]];
}

__global__ void k_mirror_pack(uint32_t const* mir, uint32_t const* mir_pos, uint32_t const* flag,
                              uint32_t const* pos, int64_t n, uint32_t const* c_own, uint32_t* out_pos,
                              uint32_t* out_c)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (flag[i]) {
      out_pos[pos[i]] = mir_pos[i];
      out_c[pos[i]]   = c_own[mir[i]];
    }
}

__global__ void k_scatter_u32(uint32_t const* pos, uint32_t const* val, int64_t n, uint32_t* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[pos[i]] = val[i];
}

// coarse pair key (label(u), label(v)) of every local edge; labels of the local
// ids: own rows from lab_own, ghosts from lab_gh
__global__ void k_mg_pair_keys_loc(uint32_t const* src, uint32_t const* dst, uint32_t const* lab_own,
                                   uint32_t const* lab_gh, uint32_t nr, int64_t ne, u64* keys)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const d  = dst[e];
    uint32_t const lv = d < nr ? lab_own[d] : lab_gh[d - nr];
    keys[e]           = ((u64)lab_own[src[e]] << 32) | (u64)lv;
  }
}

__global__ void k_mark_used_list(uint32_t const* lab, int64_t n, uint32_t lo, uint32_t* used)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    used[lab[i] - lo] = 1u;
}

// (l(u), l(v)) -> (new(l(u)) - new_lo, new(l(v))): l(u) is owned (nl_own), l(v)
// through the looked-up table (keys sorted, values new ids)
// dense: the new id of every wanted label, indexed by label (k_scatter_table; a
// binary search over the wanted labels per pair was 7 ms a level at RMAT-24)
__global__ void k_relabel_pairs_mg(u64 const* keys, int64_t n, uint32_t const* nl_own, uint32_t lo,
                                   uint32_t const* dense, uint32_t new_lo, u64* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const lu = (uint32_t)(keys[i] >> 32), lv = (uint32_t)keys[i];
    uint32_t const nv = dense[lv];
    out[i]            = ((u64)(nl_own[lu - lo] - new_lo) << 32) | (u64)nv;
  }
}

__global__ void k_key_lo(u64 const* keys, int64_t n, uint32_t* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)keys[i];
}

__global__ void k_scatter_table(uint32_t const* tk, uint32_t const* tv, int64_t nt, uint32_t* dense)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nt; i += (int64_t)gridDim.x * blockDim.x)
    dense[tk[i]] = tv[i];
}

__global__ void k_lookup_dense(uint32_t* x, int64_t n, uint32_t const* dense)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = dense[x[i]];
}

// x[i] -> the value of x[i] in the table (keys sorted, every x present)
__global__ void k_lookup_u32(uint32_t* x, int64_t n, uint32_t const* tk, uint32_t const* tv, int64_t nt)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = tv[lower_bound_u32(tk, nt, x[i])];
}

// sorted unique of n u32 keys (values < 2^bits) into out; returns the count
int64_t sort_unique_u32(uint32_t const* in, int64_t n, dbuf<uint32_t>& out, int bits, hipStream_t s)
{
  out.resize(std::max<int64_t>(n, 1), s);
  if (n == 0) return 0;
  dbuf<uint32_t> tmp(n, s);
  radix_sort_keys<uint32_t>(in, tmp.data(), (size_t)n, 0, bits, s);
  dbuf<size_t> cnt(1, s);
  size_t tb = 0;
  HIP_CHECK(rocprim::unique(nullptr, tb, tmp.data(), out.data(), cnt.data(), (size_t)n,
                            rocprim::equal_to<uint32_t>(), s));
  buffer t(std::max<size_t>(tb, 1), s);
  HIP_CHECK(rocprim::unique(t.data(), tb, tmp.data(), out.data(), cnt.data(), (size_t)n,
                            rocprim::equal_to<uint32_t>(), s));
  return (int64_t)to_host_scalar(cnt.data(), s);
}

// distinct ids through a bitmap of the id range (ids < nv): nv / 8 bytes, where a sort
// of n keys reads and writes them once per radix pass.  The ids repeat (cluster ids of
// many vertices), so they are marked as bytes with plain stores (idempotent, no
// read-modify-write) and packed into the bitmap by a pass over the nv flag bytes: an
// atomicOr per id serialised on the shared words (0.72 ms a call at RMAT-24; 0.47
// with a load before each atomic)
__global__ void k_set_flags(uint32_t const* in, int64_t n, uint8_t* fl)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    fl[in[i]] = 1;
}
// word i of the bitmap from flag bytes [32 i, 32 i + 32) (the flag array is padded to
// whole words), and its popcount (wc[nw] = 0)
__global__ void k_flags_to_bits(uint8_t const* fl, int64_t nw, uint32_t* bm, uint32_t* wc)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= nw; i += (int64_t)gridDim.x * blockDim.x) {
    if (i == nw) {
      wc[i] = 0u;
      continue;
    }
    uint4 const* p = reinterpret_cast<uint4 const*>(fl + i * 32);
    uint4 const a = p[0], b = p[1];
    uint32_t const w8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t bits        = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) bits |= ((w8[k] >> (8 * j)) & 1u) << (4 * k + j);
    bm[i] = bits;
    wc[i] = (uint32_t)__popc(bits);
  }
}
__global__ void k_emit_bits(uint32_t const* bm, uint32_t const* wp, int64_t nw, uint32_t* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nw; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t b = bm[i], o = wp[i];
    while (b) {
      int const t = __ffs(b) - 1;
      out[o++]    = (uint32_t)(i * 32 + t);
      b &= b - 1;
    }
  }
}
__global__ void k_rank_bits(uint32_t const* in, int64_t n, uint32_t const* bm, uint32_t const* wp, uint32_t* rank)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const x = in[i], w = x >> 5;
    rank[i]          = wp[w] + (uint32_t)__popc(bm[w] & ((1u << (x & 31u)) - 1u));
  }
}

// the sorted distinct ids of in[0, n) (ids < nv) into out, and each input's position
// among them into rank (sort_unique_u32 and a lower bound per id, through a bitmap)
int64_t unique_ranks_bitmap(uint32_t const* in, int64_t n, int64_t nv, dbuf<uint32_t>& out, uint32_t* rank,
                            hipStream_t s)
{
  int64_t const nw = (nv + 31) / 32;
  dbuf<uint32_t> bm(std::max<int64_t>(nw, 1), s), wc(nw + 1, s), wp(nw + 1, s);
  dbuf<uint8_t> fl(std::max<int64_t>(nw, 1) * 32, s);
  HIP_CHECK(hipMemsetAsync(fl.data(), 0, (size_t)std::max<int64_t>(nw, 1) * 32, s));
  if (n) hipLaunchKernelGGL(k_set_flags, dim3(blocks(n)), dim3(kBlock), 0, s, in, n, fl.data());
  CGX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_flags_to_bits, dim3(blocks(nw + 1)), dim3(kBlock), 0, s, fl.data(), nw, bm.data(), wc.data());
  CGX_LAUNCH_CHECK();
  exclusive_scan<uint32_t, uint32_t>(wc.data(), wp.data(), (size_t)(nw + 1), s);
  int64_t const ncl = (int64_t)to_host_scalar(wp.data() + nw, s);
  out.resize(std::max<int64_t>(ncl, 1), s);
  if (nw) hipLaunchKernelGGL(k_emit_bits, dim3(blocks(nw)), dim3(kBlock), 0, s, bm.data(), wp.data(), nw, out.data());
  CGX_LAUNCH_CHECK();
  if (n) hipLaunchKernelGGL(k_rank_bits, dim3(blocks(n)), dim3(kBlock), 0, s, in, n, bm.data(), wp.data(), rank);
  CGX_LAUNCH_CHECK();
  return ncl;
}

// per-owner counts of a sorted id list (owner ranges voff, device copy voff_d)
std::vector<size_t> owner_counts(uint32_t const* ids, int64_t n, dbuf<int64_t> const& voff_d, int P, hipStream_t s)
{
  dbuf<int64_t> bnd(P + 1, s);
  hipLaunchKernelGGL(k_id_bounds, dim3(1), dim3(256), 0, s, ids, n, voff_d.data(), P, bnd.data());
  CGX_LAUNCH_CHECK();
  auto c = bounds_to_counts(bnd, P, s);
  return std::vector<size_t>(c.begin(), c.end());
}

// collect_values_for_keys: keys (sorted unique ids of this level, n) -> the values
// their owners hold in own_vals[id - voff[owner]] (out[i] for keys[i])
template <typename T>
dbuf<T> collect_by_key(louvain_state& S, uint32_t const* keys, int64_t n, dbuf<int64_t> const& voff_d, int64_t lo,
                       T const* own_vals)
{
  hipStream_t s = S.s;
  auto counts   = owner_counts(keys, n, voff_d, S.comm->size, s);
  std::vector<size_t> rc;
  auto rk = xchg<uint32_t>(S, keys, counts, rc);
  dbuf<T> ans(std::max<size_t>(rk.n, 1), s);
  if (rk.n)
    hipLaunchKernelGGL(k_owner_gather<T>, dim3(blocks((int64_t)rk.n)), dim3(kBlock), 0, s, rk.data(), (int64_t)rk.n,
                       (uint32_t)lo, own_vals, ans.data());
  CGX_LAUNCH_CHECK();
  return xchg_known<T>(S, ans.data(), rc, counts);
}

// One level of the owner-sharded local move.  The level graph's destinations are
// turned into local ids ([0, nr): own rows, then the ghosts), so the single-GPU
// sweep kernels run unchanged on (rows, local ids, local cluster ids).
struct mg_level {
  int64_t nv = 0, lo = 0, nr = 0, ng = 0;
  std::vector<int64_t> voff;
  dbuf<int64_t> voff_d;
  dbuf<uint32_t> ghost;     // ng: sorted global ids of remote destinations
  dbuf<uint32_t> mir;       // rows (id - lo) mirrored to other ranks, in requester order
  dbuf<uint32_t> mir_pos;   // their positions in the requester's ghost list
  std::vector<size_t> mir_cnt, mir_rcv;  // per requester; the update exchange's receive counts are unknown
  dbuf<uint32_t> c_own, c_gh;  // clusters (global ids) of the rows and of the ghosts
  dbuf<long long> kfix, afix;  // rows' fixed-point weights; owned clusters' fixed-point weights
  dbuf<int> pcnt;              // owned clusters: members with edges
  double scale = 0, inv = 0;
};

void mg_setup_level(louvain_state& S, level_graph& g, mg_level& L, uint8_t const* has_edges, double const* k)
{
  hipStream_t s = S.s;
  int const P   = S.comm->size;
  int64_t const ne = g.ne, nr = L.nr, r1 = std::max<int64_t>(nr, 1);
  // ghosts: distinct remote destinations
  dbuf<uint32_t> rem(std::max<int64_t>(ne, 1), s);
  if (ne)
    hipLaunchKernelGGL(k_remote_ids, dim3(blocks(ne)), dim3(kBlock), 0, s, g.dst.data(), ne, (uint32_t)L.lo,
                       (uint32_t)nr, rem.data());
  CGX_LAUNCH_CHECK();
  int64_t nu = sort_unique_u32(rem.data(), ne, L.ghost, 32, s);
  if (nu && to_host_scalar(L.ghost.data() + nu - 1, s) == ~0u) --nu;  // the own-destination marker
  L.ng = nu;
  // mirror lists: every ghost list goes to the owners of its ids
  auto gcount = owner_counts(L.ghost.data(), L.ng, L.voff_d, P, s);
  {
    dbuf<uint32_t> gpos(std::max<int64_t>(L.ng, 1), s);
    iota<uint32_t>(gpos.data(), L.ng, 0u, s);
    L.mir     = xchg<uint32_t>(S, L.ghost.data(), gcount, L.mir_cnt);
    L.mir_pos = xchg_known<uint32_t>(S, gpos.data(), gcount, L.mir_cnt);
  }
  if (L.mir.n)
    hipLaunchKernelGGL(k_sub_u32, dim3(blocks((int64_t)L.mir.n)), dim3(kBlock), 0, s, L.mir.data(), (int64_t)L.mir.n,
                       (uint32_t)L.lo);
  CGX_LAUNCH_CHECK();
  L.mir_rcv = gcount;  // ghost updates come back from the owners in these blocks at most
  // local destination ids
  if (ne)
    hipLaunchKernelGGL(k_localize, dim3(blocks(ne)), dim3(kBlock), 0, s, g.dst.data(), ne, (uint32_t)L.lo,
                       (uint32_t)nr, L.ghost.data(), L.ng);
  CGX_LAUNCH_CHECK();
  g.base = 0;
  g.nv   = nr + L.ng;
  // singleton clusters: rows lo + i, ghosts their own ids
  L.c_own.resize(r1, s);
  iota<uint32_t>(L.c_own.data(), nr, (uint32_t)L.lo, s);
  L.c_gh.resize(std::max<int64_t>(L.ng, 1), s);
  if (L.ng)
    HIP_CHECK(hipMemcpyAsync(L.c_gh.data(), L.ghost.data(), L.ng * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  // fixed-point cluster weights at the owners: scale 2^(60 - e), sum of all weights < 2^e
  int const e = S.m > 0 ? std::ilogb(S.m) + 1 : 0;
  L.scale     = std::ldexp(1.0, 60 - e);
  L.inv       = std::ldexp(1.0, e - 60);
  L.kfix.resize(r1, s);
  L.afix.resize(r1, s);
  L.pcnt.resize(r1, s);
  if (nr) {
    hipLaunchKernelGGL(k_to_fixed, dim3(blocks(nr)), dim3(kBlock), 0, s, k, nr, L.scale, L.kfix.data());
    CGX_LAUNCH_CHECK();
    HIP_CHECK(hipMemcpyAsync(L.afix.data(), L.kfix.data(), nr * sizeof(long long), hipMemcpyDeviceToDevice, s));
    convert<int, uint8_t>(L.pcnt.data(), has_edges, nr, s);
  }
}

// the local clustering of the sweep: referenced clusters (own rows' and ghosts'),
// their weights and present flags from the owners
struct mg_sweep_view {
  int64_t ncl = 0;
  dbuf<uint32_t> ref;       // sorted global cluster ids referenced here
  dbuf<uint32_t> c_loc;     // nr + ng local cluster ids
  dbuf<double> a;           // ncl
  dbuf<uint8_t> present;    // ncl
};

void mg_view(louvain_state& S, mg_level& L, bool all_present, mg_sweep_view& W)
{
  hipStream_t s   = S.s;
  int64_t const n = L.nr + L.ng;
  dbuf<uint32_t> all(std::max<int64_t>(n, 1), s);
  if (L.nr) HIP_CHECK(hipMemcpyAsync(all.data(), L.c_own.data(), L.nr * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  if (L.ng)
    HIP_CHECK(hipMemcpyAsync(all.data() + L.nr, L.c_gh.data(), L.ng * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  // the referenced clusters, sorted, and the local (order-preserving) ids: a bitmap of
  // the level's ids (nv / 8 bytes) where a radix sort of the nr + ng ids ran each sweep
  W.c_loc.resize(std::max<int64_t>(n, 1), s);
  W.ncl = unique_ranks_bitmap(all.data(), n, L.nv, W.ref, W.c_loc.data(), s);
  auto af = collect_by_key<long long>(S, W.ref.data(), W.ncl, L.voff_d, L.lo, L.afix.data());
  auto pc = collect_by_key<int>(S, W.ref.data(), W.ncl, L.voff_d, L.lo, L.pcnt.data());
  W.a.resize(std::max<int64_t>(W.ncl, 1), s);
  W.present.resize(std::max<int64_t>(W.ncl, 1), s);
  if (W.ncl)
    hipLaunchKernelGGL(k_cluster_vals, dim3(blocks(W.ncl)), dim3(kBlock), 0, s, af.data(), pc.data(), W.ncl, L.inv,
                       all_present ? 1 : 0, W.a.data(), W.present.data());
  CGX_LAUNCH_CHECK();
}

// Q of the clustering the sweep started from: sum of own(row) (the internal weight
// by-product of the sweep) and sum of a_c^2 over the owned cluster ids
double mg_modularity(louvain_state& S, mg_level& L, double const* own, bool all_present)
{
  device_sum(plain_f{own}, (size_t)L.nr, S.scal.data(), S.scratch.data(), S.s);
  device_sum(sumsq_fixed_f{L.afix.data(), L.pcnt.data(), L.inv, all_present ? 1 : 0}, (size_t)L.nr,
             S.scal.data() + 1, S.scratch.data(), S.s);
  S.comm->allreduce<double>(S.scal.data(), S.scal.data(), 2, CGX_COMM_SUM, S.s);
  auto hv = to_host(S.scal.data(), 2, S.s);
  return hv[0] / S.m - (S.gamma * hv[1]) / (S.m * S.m);
}

// clusters <- the sweep's result: rows' new global clusters, the owners' weights
// updated by the moves, the moved rows' new clusters sent to the ranks that
// mirror them.  Traffic: O(moved rows + their mirrors).
void mg_advance(louvain_state& S, mg_level& L, mg_sweep_view& W, uint32_t const* next_loc, uint8_t const* has_edges)
{
  hipStream_t s    = S.s;
  int const P      = S.comm->size;
  int64_t const nr = L.nr, r1 = std::max<int64_t>(nr, 1);
  dbuf<uint32_t> old_c(r1, s);
  dbuf<uint8_t> moved(r1, s);
  dbuf<uint32_t> mflag(r1, s), mpos(r1 + 1, s);
  int64_t nm = 0;
  if (nr) {
    HIP_CHECK(hipMemcpyAsync(old_c.data(), L.c_own.data(), nr * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_advance, dim3(blocks(nr)), dim3(kBlock), 0, s, next_loc, W.ref.data(), nr, L.c_own.data(),
                       moved.data());
    CGX_LAUNCH_CHECK();
    convert<uint32_t, uint8_t>(mflag.data(), moved.data(), nr, s);
    exclusive_scan<uint32_t, uint32_t>(mflag.data(), mpos.data(), (size_t)nr + 1, s);
    nm = (int64_t)to_host_scalar(mpos.data() + nr, s);
  }
  // 1. weight deltas to the owners of the old and the new clusters
  int64_t const nd = 2 * nm, d1 = std::max<int64_t>(nd, 1);
  dbuf<uint32_t> dkey(d1, s), dkey2(d1, s);
  dbuf<long long> dk(d1, s);
  dbuf<int> dh(d1, s);
  dbuf<int64_t> perm(d1, s), perm2(d1, s);
  if (nm) {
    hipLaunchKernelGGL(k_move_deltas, dim3(blocks(nr)), dim3(kBlock), 0, s, old_c.data(), L.c_own.data(),
                       moved.data(), mpos.data(), nr, L.kfix.data(), has_edges, dkey.data(), dk.data(), dh.data());
    CGX_LAUNCH_CHECK();
    iota<int64_t>(perm.data(), nd, 0, s);
    radix_sort_pairs<uint32_t, int64_t>(dkey.data(), dkey2.data(), perm.data(), perm2.data(), (size_t)nd, 0, 32, s);
  }
  dbuf<long long> dk2(d1, s);
  dbuf<int> dh2(d1, s);
  if (nm) {
    gather<long long, int64_t>(dk2.data(), dk.data(), perm2.data(), nd, s);
    gather<int, int64_t>(dh2.data(), dh.data(), perm2.data(), nd, s);
  }
  auto counts = owner_counts(dkey2.data(), nd, L.voff_d, P, s);
  std::vector<size_t> rc;
  auto rk  = xchg<uint32_t>(S, dkey2.data(), counts, rc);
  auto rdk = xchg_known<long long>(S, dk2.data(), counts, rc);
  auto rdh = xchg_known<int>(S, dh2.data(), counts, rc);
  if (rk.n)
    hipLaunchKernelGGL(k_apply_deltas, dim3(blocks((int64_t)rk.n)), dim3(kBlock), 0, s, rk.data(), rdk.data(),
                       rdh.data(), (int64_t)rk.n, (uint32_t)L.lo, L.afix.data(), L.pcnt.data());
  CGX_LAUNCH_CHECK();
  // 2. ghost updates: mirror entries of moved rows, per requester
  int64_t const nmir = (int64_t)L.mir.n, m1 = std::max<int64_t>(nmir, 1);
  dbuf<uint32_t> fl(m1, s), fpos(m1 + 1, s);
  std::vector<size_t> ucnt(P, 0);
  int64_t nup = 0;
  if (nmir) {
    hipLaunchKernelGGL(k_mirror_flags, dim3(blocks(nmir)), dim3(kBlock), 0, s, L.mir.data(), nmir, moved.data(),
                       fl.data());
    CGX_LAUNCH_CHECK();
    exclusive_scan<uint32_t, uint32_t>(fl.data(), fpos.data(), (size_t)nmir + 1, s);
    // per-requester counts from the scan at the block boundaries
    std::vector<int64_t> bo(P + 1, 0);
    for (int q = 0; q < P; ++q) bo[q + 1] = bo[q] + (int64_t)L.mir_cnt[q];
    dbuf<int64_t> bod(P + 1, s);
    dbuf<uint32_t> atd(P + 1, s);
    to_device(bod.data(), bo.data(), (size_t)P + 1, s);
    gather<uint32_t, int64_t>(atd.data(), fpos.data(), bod.data(), (size_t)P + 1, s);
    auto at = to_host(atd.data(), (size_t)P + 1, s);
    for (int q = 0; q < P; ++q) ucnt[q] = at[q + 1] - at[q];
    nup = at[P];
  }
  dbuf<uint32_t> upos(std::max<int64_t>(nup, 1), s), uc(std::max<int64_t>(nup, 1), s);
  if (nup)
    hipLaunchKernelGGL(k_mirror_pack, dim3(blocks(nmir)), dim3(kBlock), 0, s, L.mir.data(), L.mir_pos.data(),
                       fl.data(), fpos.data(), nmir, L.c_own.data(), upos.data(), uc.data());
  CGX_LAUNCH_CHECK();
  std::vector<size_t> urc;
  auto rpos = xchg<uint32_t>(S, upos.data(), ucnt, urc);
  auto rc2  = xchg_known<uint32_t>(S, uc.data(), ucnt, urc);
  if (rpos.n)
    hipLaunchKernelGGL(k_scatter_u32, dim3(blocks((int64_t)rpos.n)), dim3(kBlock), 0, s, rpos.data(), rc2.data(),
                       (int64_t)rpos.n, L.c_gh.data());
  CGX_LAUNCH_CHECK();
}

// contract by the level's clustering (lab_own: rows' clusters, lab_gh: ghosts'
// clusters, global ids): coarse pairs to the owner of label(u), used labels numbered
// there by descending coarse degree, the new ids of label(v) and of the rows'
// labels collected from their owners.  On return lab_own holds the rows' coarse ids
// and voff the coarse level's ranges.
level_graph mg_contract(louvain_state& S, level_graph const& g, mg_level& L, uint32_t* lab_own, uint32_t const* lab_gh,
                        std::vector<int64_t>& voff)
{
  hipStream_t s  = S.s;
  comm_t& comm   = *S.comm;
  int const P = comm.size, p = comm.rank;
  int64_t const ne = g.ne, nr = L.nr, lo = L.lo, nv = L.nv;
  int64_t const n1 = std::max<int64_t>(ne, 1);
  int const lb = bits_for((unsigned long long)std::max<int64_t>(nv - 1, 1));
  // 1. local coarse pairs, summed (double-buffered sort, the reduction into the free
  //    pair of buffers: 32 B per edge at the peak, RMAT-26 on one rank 67 GB)
  dbuf<u64> keys, ka(n1, s);
  dbuf<double> cw, wa(n1, s);
  int64_t nce = 0;
  {
    dbuf<u64> kb(n1, s);
    dbuf<double> wb(n1, s);
    if (ne) {
      hipLaunchKernelGGL(k_mg_pair_keys_loc, dim3(blocks(ne)), dim3(kBlock), 0, s, g.src.data(), g.dst.data(),
                         lab_own, lab_gh, (uint32_t)nr, ne, ka.data());
      CGX_LAUNCH_CHECK();
      HIP_CHECK(hipMemcpyAsync(wa.data(), g.w.data(), ne * sizeof(double), hipMemcpyDeviceToDevice, s));
      if (radix_sort_pairs_db<u64, double>(ka.data(), kb.data(), wa.data(), wb.data(), (size_t)ne, 0, 32 + lb, s)) {
        std::swap(ka, kb);
        std::swap(wa, wb);
      }
      // sorted pairs in ka / wa; sums into kb / wb
      nce = reduce_by_key(ka.data(), wa.data(), (size_t)ne, kb.data(), wb.data(), rocprim::plus<double>(),
                          rocprim::equal_to<u64>(), s);
    }
    keys = std::move(kb);
    cw   = std::move(wb);
  }
  ka.free();
  wa.free();
  // 2. to the owner of label(u) (keys sorted, owner ranges ascending); one rank owns
  //    every label: its pairs are already sorted and summed
  dbuf<u64> mk, mk2;
  dbuf<double> mw;
  int64_t nm = 0;
  if (P == 1) {
    nm = nce;
    mk = std::move(keys);
    mw = std::move(cw);
    mk2.resize(std::max<int64_t>(nm, 1), s);  // (scratch for the relabelled keys below)
  } else {
    dbuf<int64_t> bnd(P + 1, s);
    hipLaunchKernelGGL(k_key_bounds, dim3(1), dim3(256), 0, s, keys.data(), nce, L.voff_d.data(), P, bnd.data());
    CGX_LAUNCH_CHECK();
    auto c64 = bounds_to_counts(bnd, P, s);
    std::vector<size_t> counts(c64.begin(), c64.end()), rc;
    auto rk = exchange<u64>(comm, keys.data(), counts, rc, s);
    keys.free();
    auto rw = exchange<double>(comm, cw.data(), counts, rc, s);
    cw.free();
    int64_t const nrcv = (int64_t)rk.n, r1 = std::max<int64_t>(nrcv, 1);
    mk2.resize(r1, s);
    dbuf<double> mw2(r1, s);
    if (nrcv) {
      if (radix_sort_pairs_db<u64, double>(rk.data(), mk2.data(), rw.data(), mw2.data(), (size_t)nrcv, 0, 32 + lb,
                                           s)) {
        std::swap(rk, mk2);
        std::swap(rw, mw2);
      }
      // sorted in rk / rw; merged sums into mk2 / mw2
      nm = reduce_by_key(rk.data(), rw.data(), (size_t)nrcv, mk2.data(), mw2.data(), rocprim::plus<double>(),
                         rocprim::equal_to<u64>(), s);
    }
    mk  = std::move(mk2);
    mw  = std::move(mw2);
    mk2 = std::move(rk);  // (scratch for the relabelled keys below)
    rw.free();
  }
  // 3. used labels: every rank sends its rows' distinct labels to their owners
  dbuf<uint32_t> ul;
  int64_t const nul = sort_unique_u32(lab_own, nr, ul, lb, s);
  auto ucounts = owner_counts(ul.data(), nul, L.voff_d, P, s);
  std::vector<size_t> urc;
  auto rl = exchange<uint32_t>(comm, ul.data(), ucounts, urc, s);
  dbuf<uint32_t> used(nr + 1, s), pos(nr + 1, s), deg(std::max<int64_t>(nr, 1), s);
  fill<uint32_t>(used.data(), nr + 1, 0u, s);
  fill<uint32_t>(deg.data(), std::max<int64_t>(nr, 1), 0u, s);
  if (rl.n)
    hipLaunchKernelGGL(k_mark_used_list, dim3(blocks((int64_t)rl.n)), dim3(kBlock), 0, s, rl.data(), (int64_t)rl.n,
                       (uint32_t)lo, used.data());
  CGX_LAUNCH_CHECK();
  if (nm && nr)
    hipLaunchKernelGGL(k_count_src, dim3(blocks(nr)), dim3(kBlock), 0, s, mk.data(), nm, lo, nr, deg.data());
  CGX_LAUNCH_CHECK();
  exclusive_scan<uint32_t, uint32_t>(used.data(), pos.data(), nr + 1, s);
  int64_t const nu = (int64_t)to_host_scalar(pos.data() + nr, s), u1 = std::max<int64_t>(nu, 1);
  dbuf<uint32_t> uniq(u1, s), udeg(u1, s), udeg2(u1, s), nmap(u1, s), nl_own(std::max<int64_t>(nr, 1), s);
  if (nr)
    hipLaunchKernelGGL(k_compact_labels, dim3(blocks(nr)), dim3(kBlock), 0, s, used.data(), pos.data(), deg.data(), nr,
                       uniq.data(), udeg.data());
  CGX_LAUNCH_CHECK();
  if (nu)
    radix_sort_pairs<uint32_t, uint32_t>(udeg.data(), udeg2.data(), uniq.data(), nmap.data(), (size_t)nu, 0,
                                         bits_for((unsigned long long)std::max<int64_t>(nm, 1)), s,
                                         /*descending=*/true);
  auto all_nu = comm.host_allgather<int64_t>(nu, s);
  std::vector<int64_t> nvoff(P + 1, 0);
  for (int q = 0; q < P; ++q) nvoff[q + 1] = nvoff[q] + all_nu[q];
  uint32_t const new_lo = (uint32_t)nvoff[p];
  if (nu)
    hipLaunchKernelGGL(k_new_ids_off, dim3(blocks(nu)), dim3(kBlock), 0, s, nmap.data(), nu, new_lo, nl_own.data());
  CGX_LAUNCH_CHECK();
  // (nl_own: the new id of every used label, indexed by label - lo)
  // 4. new ids of the labels this rank still needs: label(v) of its merged pairs and
  //    its rows' labels
  int64_t const nq = nm + nr;
  dbuf<uint32_t> want(std::max<int64_t>(nq, 1), s), wk;
  if (nm)
    hipLaunchKernelGGL(k_key_lo, dim3(blocks(nm)), dim3(kBlock), 0, s, mk.data(), nm, want.data());
  CGX_LAUNCH_CHECK();
  if (nr) HIP_CHECK(hipMemcpyAsync(want.data() + nm, lab_own, nr * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  int64_t const nw = sort_unique_u32(want.data(), nq, wk, lb, s);
  auto wv = collect_by_key<uint32_t>(S, wk.data(), nw, L.voff_d, lo, nl_own.data());
  // the wanted labels' new ids as a dense table over the level's ids (only wanted
  // entries are written and read)
  dbuf<uint32_t> dense(std::max<int64_t>(L.nv, 1), s);
  if (nw) hipLaunchKernelGGL(k_scatter_table, dim3(blocks(nw)), dim3(kBlock), 0, s, wk.data(), wv.data(), nw, dense.data());
  CGX_LAUNCH_CHECK();
  level_graph out;
  out.nv    = nvoff[P];
  out.base  = nvoff[p];
  out.nrows = nu;
  out.ne    = nm;
  out.src.resize(std::max<int64_t>(nm, 1), s);
  out.dst.resize(std::max<int64_t>(nm, 1), s);
  out.w.resize(std::max<int64_t>(nm, 1), s);
  if (nm) {
    hipLaunchKernelGGL(k_relabel_pairs_mg, dim3(blocks(nm)), dim3(kBlock), 0, s, mk.data(), nm, nl_own.data(),
                       (uint32_t)lo, dense.data(), new_lo, mk2.data());
    CGX_LAUNCH_CHECK();
    if (!radix_sort_pairs_db<u64, double>(mk2.data(), mk.data(), mw.data(), out.w.data(), (size_t)nm, 0,
                                          32 + bits_for(std::max<int64_t>(nu - 1, 0)), s)) {
      std::swap(mk2, mk);  // sorted keys in mk, weights in out.w
      std::swap(mw, out.w);
    }
    hipLaunchKernelGGL(k_split_pairs, dim3(blocks(nm)), dim3(kBlock), 0, s, mk.data(), nm, out.src.data(),
                       out.dst.data(), /*cb=*/32);
    CGX_LAUNCH_CHECK();
  }
  if (nr) hipLaunchKernelGGL(k_lookup_dense, dim3(blocks(nr)), dim3(kBlock), 0, s, lab_own, nr, dense.data());
  CGX_LAUNCH_CHECK();
  voff = nvoff;
  return out;
}

template <typename V, typename E, typename R>
void mg_louvain_impl(handle_t& h, graph_t& g, size_t max_level, double resolution, clustering_result_t& res)
{
  hipStream_t s = h.stream;
  CGX_EXPECTS(g.weighted, CUGRAPH_UNKNOWN_ERROR, "Graph must be weighted");  // louvain_impl.cuh:290
  mg_graph_t& mg = *g.mg;
  comm_t& comm   = *h.mg->world;
  int const p    = mg.p, P = mg.P;
  int64_t const nv0 = g.num_vertices, n_own = mg.n_own();
  CGX_EXPECTS((uint64_t)nv0 < (1ull << 32) - 1, CUGRAPH_NOT_IMPLEMENTED, "Louvain: 2^32 - 1 or more vertices");
  res.vertices = std::make_unique<device_array_t>((size_t)n_own, g.vertex_type, s);
  if (n_own)
    HIP_CHECK(hipMemcpyAsync(res.vertices->buf.data(), g.number_map.data(), n_own * sizeof(V), hipMemcpyDeviceToDevice,
                             s));
  res.clusters = std::make_unique<device_array_t>((size_t)n_own, g.vertex_type, s);
  h.last_louvain_levels      = 0;
  h.last_louvain_sweep_bytes = 0;
  h.last_louvain_local_edges = 0;
  h.last_louvain_ghosts      = 0;
  res.modularity             = 0;
  if (nv0 == 0) return;

  louvain_state S(s, h.tune);
  S.gamma         = resolution;
  S.comm          = &comm;
  level_graph cur = mg_level0<V, R>(h, g);
  device_sum(plain_f{cur.w.data()}, (size_t)cur.ne, S.scal.data(), S.scratch.data(), s);
  comm.allreduce<double>(S.scal.data(), S.scal.data(), 1, CGX_COMM_SUM, s);
  S.m = to_host_scalar(S.scal.data(), s);
  {  // the owners' fixed-point cluster weights (scale 2^(60 - e), every |k| and cluster
     // weight below the total 2^e) assume w >= 0: negative (or NaN) weights are refused
    dbuf<u64> st(2, s);
    fill<u64>(st.data(), 2, 0ull, s);
    if (cur.ne)
      hipLaunchKernelGGL(k_level_stats, dim3(std::min<unsigned>(blocks(cur.ne), 2048)), dim3(kBlock), 0, s,
                         cur.w.data(), cur.ne, (double const*)nullptr, (int64_t)0, st.data());
    CGX_LAUNCH_CHECK();
    int64_t const bad = comm.host_allreduce<int64_t>(to_host(st.data(), 1, s)[0] ? 1 : 0, CGX_COMM_SUM, s);
    CGX_EXPECTS(bad == 0, CUGRAPH_NOT_IMPLEMENTED, "multi-GPU Louvain: negative edge weights are not supported");
  }

  bool const trace = std::getenv("CGX_LOUVAIN_TRACE") != nullptr;  // measurement only
  // CGX_LOUVAIN_TRACE=2 (debugging only): every rank syncs and names each phase as it
  // ends, so a rank that stops shows where
  bool const phases = trace && std::atoi(std::getenv("CGX_LOUVAIN_TRACE")) >= 2;
  auto phase        = [&](char const* what, size_t i) {
    if (!phases) return;
    HIP_CHECK(hipStreamSynchronize(s));
    std::fprintf(stderr, "[louvain-mg r%d] %s %zu\n", p, what, i);
  };
  std::vector<int64_t> voff = mg.voff;
  std::vector<dbuf<uint32_t>> dendrogram;  // per level: the owned ids' clusters (coarse ids after contraction)
  std::vector<std::vector<int64_t>> level_voff;
  double best_q = -1.0;
  size_t sweeps = 0, sweep_bytes = 0;
  while (dendrogram.size() < max_level) {
    mg_level L;
    L.nv   = cur.nv;
    L.lo   = cur.base;
    L.nr   = cur.nrows;
    L.voff = voff;
    L.voff_d.resize(P + 1, s);
    to_device(L.voff_d.data(), voff.data(), (size_t)P + 1, s);
    int64_t const nr = L.nr, r1 = std::max<int64_t>(nr, 1);
    level_voff.push_back(voff);
    dbuf<int64_t> off(nr + 1, s);
    hipLaunchKernelGGL(k_row_offsets, dim3(blocks(nr + 1)), dim3(kBlock), 0, s, cur.src.data(), cur.ne, nr,
                       off.data());
    CGX_LAUNCH_CHECK();
    dbuf<double> k(r1, s), self(r1, s);
    dbuf<uint8_t> has_edges(r1, s);
    // vertex weights on the global destinations (self loops: dst == row + base), then
    // the destinations become local ids
    dbuf<u64> vstats(2, s);
    vertex_weights(S, cur, off.data(), k.data(), self.data(), has_edges.data(), vstats.data());
    S.bytes = 0;
    mg_setup_level(S, cur, L, has_edges.data(), k.data());
    if (dendrogram.empty()) {  // the 1D partition's shape at level 0 (handle statistics)
      h.last_louvain_local_edges = cur.ne;
      h.last_louvain_ghosts      = L.ng;
    }
    phase("setup", dendrogram.size());
    size_t const setup_bytes = S.bytes;
    dendrogram.emplace_back(r1, s);
    uint32_t* level = dendrogram.back().data();
    dbuf<uint32_t> level_gh(std::max<int64_t>(L.ng, 1), s);
    HIP_CHECK(hipMemcpyAsync(level, L.c_own.data(), nr * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    if (L.ng)
      HIP_CHECK(hipMemcpyAsync(level_gh.data(), L.c_gh.data(), L.ng * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    sweep_plan plan;
    plan_sweeps(S, cur, off.data(), vstats.data(), plan);
    phase("plan", dendrogram.size());
    dbuf<double> own(r1, s);
    dbuf<uint32_t> next(r1, s);
    mg_sweep_view W;
    bool all_present = true;  // the first sweep: every cluster present (fill 1, as the single-GPU loop)
    bool up_down     = true;  // as the single-GPU loop: sweep k + 1 before the decision on clustering k
    S.bytes          = 0;
    mg_view(S, L, all_present, W);
    phase("view", sweeps);
    sweep(S, cur, plan, W.c_loc.data(), next.data(), k.data(), self.data(), W.a.data(), W.present.data(), W.ncl, up_down,
          own.data());
    phase("sweep", sweeps);
    double new_q = mg_modularity(S, L, own.data(), all_present);
    ++sweeps;
    sweep_bytes += S.bytes;
    if (trace && p == 0)
      std::fprintf(stderr, "[louvain-mg] level %zu nv=%lld setup %zu B/rank, sweep %zu B/rank q=%.6f\n",
                   dendrogram.size() - 1, (long long)L.nv, setup_bytes, S.bytes, new_q);
    double cur_q = new_q - 1.0;
    while (new_q > cur_q + 0.0001) {
      cur_q = new_q;
      S.bytes = 0;
      mg_advance(S, L, W, next.data(), has_edges.data());
      phase("advance", sweeps);
      all_present = false;
      up_down     = !up_down;
      mg_view(S, L, all_present, W);
      phase("view", sweeps);
      sweep(S, cur, plan, W.c_loc.data(), next.data(), k.data(), self.data(), W.a.data(), W.present.data(), W.ncl,
            up_down,
            own.data());
      phase("sweep", sweeps);
      new_q = mg_modularity(S, L, own.data(), all_present);
      ++sweeps;
      sweep_bytes += S.bytes;
      if (trace && p == 0)
        std::fprintf(stderr, "[louvain-mg]   sweep %zu B/rank (%lld referenced clusters) q=%.6f\n", S.bytes,
                     (long long)W.ncl, new_q);
      if (new_q > cur_q) {
        HIP_CHECK(hipMemcpyAsync(level, L.c_own.data(), nr * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
        if (L.ng)
          HIP_CHECK(
            hipMemcpyAsync(level_gh.data(), L.c_gh.data(), L.ng * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
      }
    }
    if (cur_q <= best_q) break;
    best_q = cur_q;
    // the level's sweep state goes before the contraction's sort buffers are allocated
    plan = sweep_plan{};
    W    = mg_sweep_view{};
    for (auto* b : {&own, &k, &self}) b->free();
    next.free();
    has_edges.free();
    off.free();
    cur = mg_contract(S, cur, L, level, level_gh.data(), voff);
    phase("contract", dendrogram.size());
  }
  // flatten_dendrogram for the owned level-0 vertices: level i's owners answer
  // for the ids the chain has reached
  dbuf<uint32_t> flat(std::max<int64_t>(n_own, 1), s);
  if (n_own)
    HIP_CHECK(hipMemcpyAsync(flat.data(), dendrogram[0].data(), n_own * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  for (size_t i = 1; i < dendrogram.size(); ++i) {
    dbuf<int64_t> vd(P + 1, s);
    to_device(vd.data(), level_voff[i].data(), (size_t)P + 1, s);
    dbuf<uint32_t> fk;
    int const lb = bits_for((unsigned long long)std::max<int64_t>(level_voff[i][P] - 1, 1));
    int64_t const nk = sort_unique_u32(flat.data(), n_own, fk, lb, s);
    auto fv          = collect_by_key<uint32_t>(S, fk.data(), nk, vd, level_voff[i][p], dendrogram[i].data());
    if (n_own)
      hipLaunchKernelGGL(k_lookup_u32, dim3(blocks(n_own)), dim3(kBlock), 0, s, flat.data(), n_own, fk.data(),
                         fv.data(), nk);
    CGX_LAUNCH_CHECK();
  }
  if (n_own) {
    hipLaunchKernelGGL(k_to_vertex<V>, dim3(blocks(n_own)), dim3(kBlock), 0, s, flat.data(), n_own,
                       res.clusters->buf.data<V>());
    CGX_LAUNCH_CHECK();
  }
  for (size_t i = 0; i < dendrogram.size(); ++i) {
    int64_t const n = level_voff[i][p + 1] - level_voff[i][p];
    res.levels.push_back(std::make_unique<device_array_t>((size_t)n, g.vertex_type, s));
    if (n)
      hipLaunchKernelGGL(k_to_vertex<V>, dim3(blocks(n)), dim3(kBlock), 0, s, dendrogram[i].data(), n,
                         res.levels.back()->buf.data<V>());
    CGX_LAUNCH_CHECK();
  }
  HIP_CHECK(hipStreamSynchronize(s));
  res.modularity             = best_q;
  h.last_louvain_levels      = dendrogram.size();
  h.last_louvain_sweep_bytes = sweeps ? (double)sweep_bytes / (double)sweeps : 0.0;
}

}  // namespace

void run_louvain(handle_t& h, graph_t& g, size_t max_level, double resolution, bool /*expensive*/,
                 clustering_result_t& res)
{
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    if (g.multi_gpu)
      mg_louvain_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g, max_level, resolution,
                                                                                      res);
    else
      louvain_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(h, g, max_level, resolution, res);
  });
}

}  // namespace cgx
