// Multi-GPU BFS (one process per GPU).
//
// Reference: cpp/src/traversal/bfs_impl.cuh:94-287 (MG path: the frontier is
// broadcast inside the communicator that shares the edge block's sources
// (extract_transform_v_frontier_e.cuh:858-876), the (destination, parent) pairs go
// to the destinations' owners with one all-to-all inside the other communicator
// (transform_reduce_v_frontier_outgoing_e_by_dst.cuh:396-451), then a termination
// allreduce).  A level is either
//
//  * top-down, on the 2D partition (mg_graph.hpp): rank (r, c) holds the edges
//    from row r's vertices (one contiguous global range) to column c's.  The own
//    frontiers of the C ranks of row r are allgathered inside the row
//    communicator; every rank expands them over its block into (v, u) candidates,
//    sorts them by (v, u), keeps the smallest parent per v, and sends them to v's
//    owner -- one of the R ranks of column c -- with one all-to-all inside the
//    column communicator; owners claim unvisited v with parent = smallest u.  On a
//    1 x P grid the column has one rank: no candidate exchange at all;
//  * bottom-up (symmetric graphs, direction_optimizing): every rank owns the
//    out-adjacency of its own vertices (a 1D partition by source owner, built once
//    from the 2D blocks and cached).  Neighbours are stored as positions in the
//    allgathered frontier bitmap -- rank q's vertices at q * W + (u - voff[q]), W =
//    the largest rank's vertex count rounded up to 32 -- so a neighbour's frontier
//    bit is one load, with no per-edge owner search (positions keep the global id
//    order).  The rank's frontier bitmap segment (V/P/8 bytes) is allgathered, and
//    the single-GPU two-pass scan runs over the owned vertices (bfs.hip k_bu_probe /
//    k_bu_residual): a lane per vertex loads its first 8 neighbours and their
//    frontier words back to back, the misses of longer lists go to 16 residual
//    sub-queues scanned by 16-lane groups, and each wave writes its vertices' next-
//    frontier bits as whole words.  Level counts go to 16 partial counters.
//
// Both pick the frontier neighbour with the smallest global id, so distances and
// predecessors do not depend on the direction schedule.  The direction switch on
// global counts is the handle's mg_bfs_alpha / mg_bfs_beta, 40 / 64 like the single
// GPU's: through a one-rank RCCL communicator (no exchange cost) RMAT-24 takes 2.92
// ms per traversal with them against 3.20 with Beamer's 14 / 24
// (scripts/mg_bfs_ab.py); with several ranks a bottom-up level adds a V/8-byte
// bitmap allgather (1.1 MB at RMAT-24) and a top-down level its candidates'
// all-to-all, so the measured kernel trade stands until a multi-rank run says
// otherwise.  Predecessors are returned as external ids.
#include "capi.hpp"
#include "comm.hpp"
#include "mg_graph.hpp"
#include "prims.hpp"

#include <rocprim/device/device_select.hpp>

#include <limits>
#include <tuple>

namespace cgx {

namespace {

inline unsigned blocks(int64_t n) { return grid_for(n > 0 ? n : 1, kBlock, 16384); }

constexpr int64_t kPosPad = 16;  // entries past the end of bfs_rows_t::pos

struct bfs_rows_t {
  int64_t n_own = 0, ne = 0;
  buffer off;  // int64[n_own + 1]
  buffer pos;  // uint32 bitmap positions of the neighbours (q * W + local id), ascending per row
               // (+ 16 entries of padding: the probe's vector loads)
  int64_t words = 0;  // 32-bit words of each rank's bitmap segment (max over ranks); W = 32 * words
  buffer head;        // bottom-up probe's head table (k_mg_head), built by the first direction-optimising call
};

typedef uint32_t v4u_t __attribute__((ext_vector_type(4)));
constexpr int kHeadN = 3;  // neighbours in the head table (bfs.hip's kHeadN)

// per own vertex 16 bytes: its first kHeadN neighbour positions (the first repeated
// past the list) and its degree clamped to 32 bits -- the probe reads 16 contiguous
// bytes per vertex instead of two offsets and a span of the adjacency (bfs.hip)
__global__ void k_mg_head(int64_t const* off, uint32_t const* pos, int64_t n, v4u_t* head)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    int64_t const beg = off[v], deg = off[v + 1] - beg;
    uint32_t w[kHeadN];
#pragma unroll
    for (int t = 0; t < kHeadN; ++t) w[t] = deg > 0 ? pos[beg + (t < deg ? t : 0)] : 0u;
    head[v] = v4u_t{w[0], w[1], w[2], (uint32_t)std::min<int64_t>(deg, 0xffffffffll)};
  }
}

// global id -> position in the allgathered frontier bitmap
__global__ void k_global_to_pos(uint32_t* ids, int64_t n, int64_t const* voff, int P, int64_t W)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t const u = ids[i];
    int const q     = mg_owner_of_global(u, voff, P);
    ids[i]          = (uint32_t)(q * W + (u - voff[q]));
  }
}

template <typename V>
__global__ void k_owner_src(V const* src, int64_t n, int64_t const* voff, int P, int* dest)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dest[i] = mg_owner_of_global((int64_t)src[i], voff, P);
}

template <typename V>
__global__ void k_row_keys(V const* src, V const* dst, int64_t n, int64_t base, unsigned long long* keys)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    keys[i] = ((unsigned long long)((int64_t)src[i] - base) << 32) | (unsigned long long)(uint32_t)dst[i];
}

__global__ void k_split_row_keys(unsigned long long const* keys, int64_t n, uint32_t* row, uint32_t* col)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    row[i] = (uint32_t)(keys[i] >> 32);
    col[i] = (uint32_t)keys[i];
  }
}

__global__ void k_offsets_u32(uint32_t const* row, int64_t ne, int64_t n, int64_t* off)
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

template <typename V>
bfs_rows_t& mg_rows(handle_t& h, graph_t& g)
{
  mg_graph_t& mg = *g.mg;
  if (mg.bfs_rows) return *static_cast<bfs_rows_t*>(mg.bfs_rows.get());
  hipStream_t s = h.stream;
  comm_t& comm  = *h.mg->world;
  CGX_EXPECTS(g.num_vertices < (int64_t)UINT32_MAX, CUGRAPH_NOT_IMPLEMENTED, "MG BFS: more than 2^32 vertices");
  auto rows   = std::make_shared<bfs_rows_t>();
  int const P = mg.P;
  dbuf<int64_t> voff_d(P + 1, s);
  HIP_CHECK(hipMemcpyAsync(voff_d.data(), mg.voff.data(), (P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  int64_t ne = mg.ne;
  // edges of the 2D block -> owner of the source (a 1D partition by rows)
  dbuf<int> dest(std::max<int64_t>(ne, 1), s);
  if (ne)
    hipLaunchKernelGGL(k_owner_src<V>, dim3(blocks(ne)), dim3(kBlock), 0, s, mg.src.data<V>(), ne, voff_d.data(), P,
                       dest.data());
  CGX_LAUNCH_CHECK();
  dbuf<int> d2(std::max<int64_t>(ne, 1), s);
  dbuf<int64_t> iv(std::max<int64_t>(ne, 1), s), perm(std::max<int64_t>(ne, 1), s);
  std::vector<size_t> counts(P, 0);
  if (ne) {
    iota<int64_t>(iv.data(), ne, 0, s);
    radix_sort_pairs<int, int64_t>(dest.data(), d2.data(), iv.data(), perm.data(), ne, 0, bits_for(P), s);
    auto hd = to_host(d2.data(), ne, s);
    for (auto q : hd) counts[q]++;
  }
  dbuf<V> ps(std::max<int64_t>(ne, 1), s), pd(std::max<int64_t>(ne, 1), s);
  if (ne) {
    gather<V, int64_t>(ps.data(), mg.src.data<V>(), perm.data(), ne, s);
    gather<V, int64_t>(pd.data(), mg.dst.data<V>(), perm.data(), ne, s);
  }
  std::vector<size_t> rc;
  auto rs = exchange<V>(comm, ps.data(), counts, rc, s);
  auto rd = exchange<V>(comm, pd.data(), counts, rc, s);
  int64_t m = (int64_t)rs.n;
  rows->n_own = mg.n_own();
  rows->ne    = m;
  dbuf<unsigned long long> k1(std::max<int64_t>(m, 1), s), k2(std::max<int64_t>(m, 1), s);
  dbuf<uint32_t> rr(std::max<int64_t>(m, 1), s);
  int64_t maxn = 0;
  for (int q = 0; q < P; ++q) maxn = std::max(maxn, mg.voff[q + 1] - mg.voff[q]);
  rows->words = std::max<int64_t>((maxn + 31) / 32, 1);
  CGX_EXPECTS((uint64_t)P * (uint64_t)rows->words * 32ull < (1ull << 32), CUGRAPH_NOT_IMPLEMENTED,
              "MG BFS: frontier bitmap positions exceed 32 bits");
  rows->pos.set_stream(s);
  rows->pos.resize((m + kPosPad) * sizeof(uint32_t));
  HIP_CHECK(hipMemsetAsync(rows->pos.data<uint32_t>() + m, 0, kPosPad * sizeof(uint32_t), s));
  rows->off.set_stream(s);
  rows->off.resize((rows->n_own + 1) * sizeof(int64_t));
  if (m) {
    hipLaunchKernelGGL(k_row_keys<V>, dim3(blocks(m)), dim3(kBlock), 0, s, rs.data(), rd.data(), m, mg.voff[mg.p],
                       k1.data());
    CGX_LAUNCH_CHECK();
    radix_sort_keys<unsigned long long>(k1.data(), k2.data(), m, 0, 64, s);
    hipLaunchKernelGGL(k_split_row_keys, dim3(blocks(m)), dim3(kBlock), 0, s, k2.data(), m, rr.data(),
                       rows->pos.data<uint32_t>());
    CGX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_global_to_pos, dim3(blocks(m)), dim3(kBlock), 0, s, rows->pos.data<uint32_t>(), m,
                       voff_d.data(), P, rows->words * 32);
    CGX_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_offsets_u32, dim3(blocks(rows->n_own + 1)), dim3(kBlock), 0, s, rr.data(), m, rows->n_own,
                     rows->off.data<int64_t>());
  CGX_LAUNCH_CHECK();
  HIP_CHECK(hipStreamSynchronize(s));
  mg.bfs_rows = rows;
  return *rows;
}

// this rank's 2D edge block as a CSR over row r's vertices (local index u - row_lo)
struct bfs_block_t {
  int64_t row_lo = 0, nrow = 0, ne = 0;
  buffer off;  // int64[nrow + 1]
  buffer idx;  // uint32 global destination ids, ascending per row
};

template <typename V>
__global__ void k_block_keys(V const* src, V const* dst, int64_t n, int64_t row_lo, unsigned long long* keys)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    keys[i] = ((unsigned long long)((int64_t)src[i] - row_lo) << 32) | (unsigned long long)(uint32_t)dst[i];
}

template <typename V>
bfs_block_t& mg_block_csr(handle_t& h, graph_t& g)
{
  mg_graph_t& mg = *g.mg;
  if (mg.bfs_block) return *static_cast<bfs_block_t*>(mg.bfs_block.get());
  hipStream_t s = h.stream;
  auto blk      = std::make_shared<bfs_block_t>();
  int const r   = mg.p / mg.C;
  blk->row_lo   = mg.voff[r * mg.C];
  blk->nrow     = mg.voff[r * mg.C + mg.C] - blk->row_lo;
  int64_t const m = mg.ne;
  blk->ne       = m;
  dbuf<unsigned long long> k1(std::max<int64_t>(m, 1), s), k2(std::max<int64_t>(m, 1), s);
  dbuf<uint32_t> rr(std::max<int64_t>(m, 1), s);
  blk->idx.set_stream(s);
  blk->idx.resize(std::max<int64_t>(m, 1) * sizeof(uint32_t));
  blk->off.set_stream(s);
  blk->off.resize((blk->nrow + 1) * sizeof(int64_t));
  if (m) {
    hipLaunchKernelGGL(k_block_keys<V>, dim3(blocks(m)), dim3(kBlock), 0, s, mg.src.data<V>(), mg.dst.data<V>(), m,
                       blk->row_lo, k1.data());
    CGX_LAUNCH_CHECK();
    radix_sort_keys<unsigned long long>(k1.data(), k2.data(), m, 0, 64, s);
    hipLaunchKernelGGL(k_split_row_keys, dim3(blocks(m)), dim3(kBlock), 0, s, k2.data(), m, rr.data(),
                       blk->idx.data<uint32_t>());
    CGX_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_offsets_u32, dim3(blocks(blk->nrow + 1)), dim3(kBlock), 0, s, rr.data(), m, blk->nrow,
                     blk->off.data<int64_t>());
  CGX_LAUNCH_CHECK();
  HIP_CHECK(hipStreamSynchronize(s));
  mg.bfs_block = blk;
  return *blk;
}

// ---------------------------------------------------------------- level kernels
constexpr int kParts = 16;  // partial counters 256 B apart (different L2 channels), as bfs.hip
struct level_ctr {
  unsigned long long next_n;  // own vertices discovered (top-down appends)
  unsigned long long next_m;  // sum of their degrees
  unsigned long long nconv;   // bitmap -> queue conversion appends
  unsigned long long bad;     // sources that are not vertices (k_init_sources)
  unsigned long long pad[28];
  unsigned long long part[kParts][32];  // bottom-up: [p][0] vertices, [p][1] edges, [p][2] residual sub-queue p
};

// (vertices, edges) of a level: the top-down fields plus the bottom-up partials (host)
inline std::pair<unsigned long long, unsigned long long> level_counts(level_ctr const& c)
{
  unsigned long long n = c.next_n, m = c.next_m;
  for (int p = 0; p < kParts; ++p) {
    n += c.part[p][0];
    m += c.part[p][1];
  }
  return {n, m};
}

// residual sub-queue capacity: sub-queue p holds at most the 64 vertices of each of its chunks
__host__ __device__ __forceinline__ int64_t mg_residual_cap(int64_t n) { return ((((n + 63) >> 6) + kParts - 1) / kParts) * 64; }

// Same-address atomics serialise at the memory side (≈8 ns each, bfs.hip): top-down
// appends are reserved once per wave and sums added once per block on capped grids;
// the bottom-up kernels add per block to one of the kParts partial counters.
inline unsigned capped(int64_t n) { return grid_for(n > 0 ? n : 1, kBlock, 1024); }

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

// block sum of v added to *dst (one atomic per block, none when zero); all threads call
__device__ __forceinline__ void block_add(unsigned long long* dst, unsigned long long v)
{
  __shared__ unsigned long long sm[kBlock / 64];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) tot += sm[w];
    if (tot) atomicAdd(dst, tot);
  }
}

// every source (all ranks' lists, gathered; pads -2, unknown ids -1): the owner
// claims it (frontier count and degree sum into the level counters), every rank
// counts the unknown ones (the same count on every rank: the same list)
template <typename V>
__global__ void k_init_sources(V const* src_global, size_t n, int64_t lo, int64_t hi, V* dist, uint32_t* queue,
                               level_ctr* ctr, int* flag, int64_t const* roff)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int64_t v = (int64_t)src_global[i];
    if (v == -1) atomicAdd(&ctr->bad, 1ull);
    if (v >= lo && v < hi) {
      int64_t l = v - lo;
      if (atomicCAS(flag + l, 0, 1) == 0) {
        dist[l]                                 = 0;
        queue[atomicAdd(&ctr->next_n, 1ull)]    = (uint32_t)l;
        atomicAdd(&ctr->next_m, (unsigned long long)(roff[l + 1] - roff[l]));
      }
    }
  }
}

// 2D top-down: frontier = row-local source ids gathered from the row (pads
// UINT32_MAX); candidate v << gb | parent for every block edge; v is filtered only
// when it is this rank's own vertex and already visited
//
// m: the candidate buffer's length, at least the real count *total (positions past
// it get the sentinel ~0, which sorts last)
template <typename V>
__global__ void k_block_candidates(uint32_t const* frontier, int64_t nf, unsigned long long const* pre, int64_t m,
                                   unsigned long long const* total, int64_t const* off, uint32_t const* idx,
                                   int64_t row_lo, int64_t lo, int64_t hi, V const* dist, int gb,
                                   unsigned long long* out)
{
  V const INF       = std::numeric_limits<V>::max();
  int64_t const mr  = (int64_t)*total;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
    if (t >= mr) {
      out[t] = ~0ull;
      continue;
    }
    int64_t a = 0, b = nf - 1;  // last frontier slot with pre <= t
    while (a < b) {
      int64_t mid = (a + b + 1) >> 1;
      if ((int64_t)pre[mid] <= t) a = mid;
      else b = mid - 1;
    }
    uint32_t u   = frontier[a];  // never a pad: pads have degree 0
    int64_t e    = off[u] + (t - (int64_t)pre[a]);
    uint32_t v   = idx[e];
    bool visited = (int64_t)v >= lo && (int64_t)v < hi && dist[(int64_t)v - lo] != INF;
    out[t]       = visited ? ~0ull : (((unsigned long long)v << gb) | (unsigned long long)(row_lo + u));
  }
}

__global__ void k_gathered_degrees(uint32_t const* frontier, int64_t nf, int64_t const* off, unsigned long long* deg)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nf; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const u = frontier[i];
    deg[i]           = u == 0xffffffffu ? 0ull : (unsigned long long)(off[u + 1] - off[u]);
  }
}

// own frontier (local ids) -> row-local ids, padded to `pad` entries with UINT32_MAX
__global__ void k_to_row_local(uint32_t const* q, int64_t n, int64_t shift, int64_t pad, uint32_t* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < pad; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = i < n ? (uint32_t)((int64_t)q[i] + shift) : 0xffffffffu;
}

template <typename V>
__global__ void k_frontier_degrees(uint32_t const* frontier, int64_t nf, int64_t const* off, unsigned long long* deg)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nf; i += (int64_t)gridDim.x * blockDim.x)
    deg[i] = (unsigned long long)(off[frontier[i] + 1] - off[frontier[i]]);
}

// first position with key >= voff[q] << 32, for q in [0, P]
__global__ void k_split_points(unsigned long long const* keys, size_t const* count, int64_t const* voff, int P,
                               int64_t* pos)
{
  int q = threadIdx.x;
  if (q > P) return;
  int64_t const n = (int64_t)*count;  // the unique run count, left on the device
  unsigned long long bound = q == P ? ~0ull : ((unsigned long long)voff[q] << 32);
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < bound) lo = mid + 1;
    else hi = mid;
  }
  pos[q] = lo;
}

struct same_v {
  int gb;  // candidate keys are v << gb | parent
  __host__ __device__ bool operator()(unsigned long long a, unsigned long long b) const { return (a >> gb) == (b >> gb); }
};

// compact candidate keys -> v << 32 | parent (the sentinel ~0 stays ~0)
__global__ void k_expand_cand(unsigned long long* k, size_t const* count, int gb)
{
  unsigned long long const mask = (1ull << gb) - 1;
  int64_t const n                = (int64_t)*count;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    unsigned long long const x = k[i];
    if (x != ~0ull) k[i] = ((x >> gb) << 32) | (x & mask);
  }
}

template <typename V>
__global__ void k_td_claim(unsigned long long const* cand, int64_t n, int64_t lo, V const* dist, long long* best,
                           int* flag, uint32_t* next, level_ctr* ctr)
{
  V const INF = std::numeric_limits<V>::max();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    unsigned long long const x = cand[i];  // ~0: a padded segment's filler
    int64_t v   = (int64_t)(x >> 32) - lo;
    long long u = (long long)(uint32_t)x;
    bool take   = false;
    if (x != ~0ull && dist[v] == INF) {
      atomicMin(best + v, u);
      take = atomicCAS(flag + v, 0, 1) == 0;
    }
    long long const slot = wave_reserve(&ctr->next_n, take);
    if (take) next[slot] = (uint32_t)v;
  }
}

template <typename V>
__global__ void k_td_finalize(uint32_t const* next, V depth1, V* dist, V* pred, long long* best, int64_t const* off,
                              level_ctr* ctr)
{
  int64_t const n      = (int64_t)ctr->next_n;  // the claims of k_td_claim (launched before, same stream)
  unsigned long long m = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t v = next[i];
    dist[v]    = depth1;
    if (pred) pred[v] = (V)best[v];
    best[v] = std::numeric_limits<long long>::max();
    m += (unsigned long long)(off[v + 1] - off[v]);
  }
  block_add(&ctr->next_m, m);
}

// total candidate count: the exclusive scan's last entry plus the last degree
__global__ void k_scan_total(unsigned long long const* pre, unsigned long long const* dg, int64_t n,
                             unsigned long long* out)
{
  if (threadIdx.x == 0) *out = pre[n - 1] + dg[n - 1];
}

// a level's (vertices, edges) of this rank folded on the device, with the unknown
// source count: allgathered over the ranks, one read-back per level gives every
// rank's counts (the totals, and the row's frontier sizes for a top-down level)
//
// The fold is the level's last reader of the counters: it clears them for the next
// level (one memset launch fewer per level)
__global__ void k_level_fold(level_ctr* c, double* red)
{
  if (threadIdx.x == 0) {
    unsigned long long n = c->next_n, m = c->next_m;
    for (int p = 0; p < kParts; ++p) {
      n += c->part[p][0];
      m += c->part[p][1];
    }
    red[0] = (double)n;
    red[1] = (double)m;
    red[2] = (double)c->bad;
  }
  __syncthreads();
  unsigned long long* w = reinterpret_cast<unsigned long long*>(c);
  for (size_t i = threadIdx.x; i < sizeof(level_ctr) / 8; i += blockDim.x) w[i] = 0ull;
}

// padded send: destination q's segment [q * m, (q + 1) * m) holds its split range of
// the expanded candidates, then the filler ~0
__global__ void k_pad_send(unsigned long long const* cu, int64_t const* pos, int R, int64_t m,
                           unsigned long long* out)
{
  int64_t const n = (int64_t)R * m;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t const q = t / m, i = t - q * m;
    out[t]          = i < pos[q + 1] - pos[q] ? cu[pos[q] + i] : ~0ull;
  }
}

// send counts per column owner from the split points (and zero when there are none)
__global__ void k_pos_counts(int64_t const* pos, int R, int have, int64_t* cnt)
{
  int const q = threadIdx.x;
  if (q < R) cnt[q] = have ? pos[q + 1] - pos[q] : 0;
}

__global__ void k_mark_bits(uint32_t const* q, int64_t n, uint32_t* bits)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    atomicOr(bits + (q[i] >> 5), 1u << (q[i] & 31u));
}

// per-block (vertices, edges) to partial counter blockIdx % kParts; all threads call
__device__ __forceinline__ void flush_parts(level_ctr* ctr, unsigned long long n, unsigned long long m)
{
  __shared__ unsigned long long sn[kBlock / 64], sm[kBlock / 64];
  for (int o = 32; o > 0; o >>= 1) {
    n += __shfl_xor(n, o, 64);
    m += __shfl_xor(m, o, 64);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    sn[threadIdx.x >> 6] = n;
    sm[threadIdx.x >> 6] = m;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tn = 0, tm = 0;
    for (int w = 0; w < kBlock / 64; ++w) tn += sn[w], tm += sm[w];
    int const p = blockIdx.x % kParts;
    if (tn) atomicAdd(&ctr->part[p][0], tn);
    if (tm) atomicAdd(&ctr->part[p][1], tm);
  }
}

constexpr int kProbe = 8;  // first neighbours tested per vertex in the probe (bfs.hip: 8 measured best)
// bottom-up -> top-down only while more than V / kTdBack vertices are unvisited
constexpr double kTdBack = 64.0;
// top-down candidate counts up to this are not read back: the buffer takes the row
// frontier's degree sum (a bound) and is sorted at that length
constexpr int64_t kCandRead = int64_t(1) << 17;
// every column peer's candidate buffer at most this: the column exchange sends padded
// segments of the buffer's length, known to every rank from the level counts (no
// count read; at most R * kPadSend * 8 bytes a rank)
constexpr int64_t kPadSend = 8192;

// the global id of bitmap position x
__device__ __forceinline__ int64_t pos_to_global(uint32_t x, int64_t const* voff, int64_t W)
{
  int64_t const q = (int64_t)x / W;
  return voff[q] + ((int64_t)x - q * W);
}

// Bottom-up probe: one lane per owned vertex, 64 consecutive vertices per wave.  An
// unvisited vertex tests its first kHeadN neighbours from the head table (one
// 16-byte load), then, on a miss, the next kProbe from the adjacency (three aligned
// 16-byte loads of the padded position array), every frontier word loaded back to
// back, and takes the lowest hit (the smallest-global-id frontier neighbour:
// positions keep the id order).  The wave's next-frontier bits are two whole words
// of seg_next that no other wave writes (no atomics, no memset); misses of longer
// lists go to residual sub-queue (chunk % kParts).
//
// mode (pipelined bottom-up levels, bu_state::mode; null: run): not 1 -> this level
// was enqueued ahead and is not to run: the own frontier segment (own, the
// allgathered copy) is copied to seg_next unchanged, so the host's swap keeps it
template <typename V>
__global__ __launch_bounds__(256) void k_mg_bu_probe(int64_t n_own, int64_t const* off, uint32_t const* pos,
                                                      v4u_t const* head, V* dist, V* pred, uint32_t const* bitmap,
                                                      int64_t const* voff, int64_t W, V depth1, uint32_t* seg_next,
                                                      uint32_t* res, level_ctr* ctr, int const* mode,
                                                      uint32_t const* own, int64_t words)
{
  if (mode && *mode != 1) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x)
      seg_next[i] = own[i];
    return;
  }
  V const INF    = std::numeric_limits<V>::max();
  int const lane = threadIdx.x & 63;
  unsigned long long my_n = 0, my_m = 0;
  int64_t const nchunks = (n_own + 63) >> 6;
  int64_t const stride  = (int64_t)gridDim.x * (kBlock / 64);
  int64_t const rcap    = mg_residual_cap(n_own);
  for (int64_t c = blockIdx.x * (int64_t)(kBlock / 64) + (threadIdx.x >> 6); c < nchunks; c += stride) {
    int64_t const v = (c << 6) + lane;
    bool const un   = v < n_own && dist[v] == INF;
    v4u_t hv        = {0u, 0u, 0u, 0u};
    if (un) hv = head[v];
    int64_t const deg = (int64_t)hv.w;
    bool hit = false, more = false;
    uint32_t par = 0;
    if (deg > 0) {
      uint32_t const u[kHeadN] = {hv.x, hv.y, hv.z};
      uint32_t fw[kHeadN];
#pragma unroll
      for (int t = 0; t < kHeadN; ++t) fw[t] = bitmap[u[t] >> 5];
      uint32_t hm = 0;
#pragma unroll
      for (int t = 0; t < kHeadN; ++t) hm |= (t < deg ? (fw[t] >> (u[t] & 31u)) & 1u : 0u) << t;
#pragma unroll
      for (int t = kHeadN - 1; t >= 0; --t)
        if ((hm >> t) & 1u) par = u[t];
      hit  = hm != 0;
      more = !hit && deg > kHeadN;
      if (more) {
        // the next kProbe positions: the aligned 12-entry span around them (the
        // position array has kPosPad entries of padding past its end)
        int64_t const b2  = off[v] + kHeadN;
        int64_t const a0  = b2 & ~int64_t(3);
        int const sh      = (int)(b2 - a0);
        int64_t const rem = deg - kHeadN;
        v4u_t const* p    = reinterpret_cast<v4u_t const*>(pos + a0);
        v4u_t const c0 = p[0], c1 = p[1], c2 = p[2];
        uint32_t const wv[12] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w};
        uint32_t w2[kProbe];
#pragma unroll
        for (int t = 0; t < kProbe; ++t) w2[t] = sh == 0 ? wv[t] : sh == 1 ? wv[t + 1] : sh == 2 ? wv[t + 2] : wv[t + 3];
#pragma unroll
        for (int t = 1; t < kProbe; ++t) w2[t] = t < rem ? w2[t] : w2[0];
        uint32_t f2[kProbe];
#pragma unroll
        for (int t = 0; t < kProbe; ++t) f2[t] = bitmap[w2[t] >> 5];
        uint32_t h2 = 0;
#pragma unroll
        for (int t = 0; t < kProbe; ++t) h2 |= (t < rem ? (f2[t] >> (w2[t] & 31u)) & 1u : 0u) << t;
#pragma unroll
        for (int t = kProbe - 1; t >= 0; --t)
          if ((h2 >> t) & 1u) par = w2[t];
        hit  = h2 != 0;
        more = !hit && rem > kProbe;
      }
    }
    if (hit) {
      dist[v] = depth1;
      if (pred) pred[v] = (V)pos_to_global(par, voff, W);
      my_n += 1;
      my_m += (unsigned long long)deg;
    }
    unsigned long long const hb = __ballot(hit);
    if ((lane & 31) == 0 && (c << 6) + lane < n_own) seg_next[((c << 6) + lane) >> 5] = (uint32_t)(hb >> lane);
    unsigned long long const mm = __ballot(more);
    if (mm) {
      unsigned long long base = 0;
      int const leader = __ffsll((long long)mm) - 1;
      int const sq     = (int)(c % kParts);
      if (lane == leader) base = atomicAdd(&ctr->part[sq][2], (unsigned long long)__popcll(mm));
      base = __shfl(base, leader, 64);
      if (more) res[sq * rcap + (int64_t)base + __popcll(mm & ((1ull << lane) - 1ull))] = (uint32_t)v;
    }
  }
  flush_parts(ctr, my_n, my_m);
}

// Bottom-up residual: 16-lane groups scan the probe's misses from neighbour kHeadN + kProbe on
template <typename V>
__global__ __launch_bounds__(256) void k_mg_bu_residual(int64_t n_own, int64_t const* off, uint32_t const* pos,
                                                         V* dist, V* pred, uint32_t const* bitmap, int64_t const* voff,
                                                         int64_t W, V depth1, uint32_t* seg_next, uint32_t const* res,
                                                         level_ctr* ctr, int const* mode)
{
  if (mode && *mode != 1) return;
  constexpr int w = 16;
  int const tid   = threadIdx.x;
  int const lane  = tid & (w - 1);
  int const gbase = (tid & 63) & ~(w - 1);
  __shared__ unsigned long long s_pre[kParts + 1];
  if (tid == 0) {
    s_pre[0] = 0ull;
    for (int p = 0; p < kParts; ++p) s_pre[p + 1] = s_pre[p] + ctr->part[p][2];
  }
  __syncthreads();
  int64_t const n    = (int64_t)s_pre[kParts];
  int64_t const rcap = mg_residual_cap(n_own);
  int64_t const ng   = (int64_t)gridDim.x * (kBlock / w);
  unsigned long long my_n = 0, my_m = 0;
  for (int64_t i = blockIdx.x * (int64_t)(kBlock / w) + tid / w; i < n; i += ng) {
    int p = 0;
    while ((unsigned long long)i >= s_pre[p + 1]) ++p;
    int64_t const v   = res[p * rcap + (i - (int64_t)s_pre[p])];
    int64_t const beg = off[v], end = off[v + 1];
    for (int64_t base = beg + kHeadN + kProbe; base < end; base += w) {
      int64_t const e = base + lane;
      bool hit        = false;
      uint32_t u      = 0;
      if (e < end) {
        u   = pos[e];
        hit = (bitmap[u >> 5] >> (u & 31u)) & 1u;
      }
      unsigned long long const gm = (__ballot(hit) >> gbase) & 0xffffull;
      if (gm) {
        if (lane == __ffsll((long long)gm) - 1) {
          dist[v] = depth1;
          if (pred) pred[v] = (V)pos_to_global(u, voff, W);
          atomicOr(seg_next + (v >> 5), 1u << (uint32_t(v) & 31u));
          my_n += 1;
          my_m += (unsigned long long)(end - beg);
        }
        break;
      }
    }
  }
  flush_parts(ctr, my_n, my_m);
}

// the own frontier bitmap segment -> a list of local ids (bottom-up -> top-down):
// a lane per word, the block's bit counts scanned in LDS, one tail atomic per block
// (a wave-serial append per set bit made it 73 us at RMAT-24's largest frontier)
__global__ __launch_bounds__(256) void k_seg_to_queue(uint32_t const* seg, int64_t nwords, uint32_t* q,
                                                      unsigned long long* tail)
{
  __shared__ unsigned s_w[kBlock / 64];
  __shared__ unsigned long long s_base;
  int const lane = threadIdx.x & 63;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < nwords; base += (int64_t)gridDim.x * blockDim.x) {
    int64_t const wi = base + threadIdx.x;
    uint32_t word    = wi < nwords ? seg[wi] : 0u;
    unsigned const c = (unsigned)__popc(word);
    unsigned x       = c;  // inclusive scan over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      unsigned const y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) s_w[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned t = 0;
      for (int w = 0; w < kBlock / 64; ++w) {
        unsigned const v = s_w[w];
        s_w[w]           = t;
        t += v;
      }
      s_base = t ? atomicAdd(tail, (unsigned long long)t) : 0ull;
    }
    __syncthreads();
    unsigned long long o = s_base + s_w[threadIdx.x >> 6] + (x - c);
    while (word) {
      q[o++] = (uint32_t)(wi * 32 + (__ffs(word) - 1));
      word &= word - 1;
    }
    __syncthreads();
  }
}

// ---------------------------------------------- pipelined bottom-up levels
// Every bottom-up level has the same fixed-size exchange (the frontier bitmap
// segments), so once a traversal is bottom-up the host enqueues the next level before
// it has read the last one's counts: the direction rule runs on the device
// (k_bu_ctl) and a level enqueued past a switch or the end runs as a no-op (mode !=
// 1).  The host reads every level's counts one level late.
struct bu_state {
  double m_u;      // degree sum of the unvisited vertices (global)
  double reached;  // vertices with a distance (global)
  int mode;        // the next level: 1 bottom-up, 0 top-down (the host takes over), 2 done
  int pad;
};

constexpr int kPipeMaxP = 64;  // ranks whose counts fit the report (the host path beyond)

struct bu_report {
  double nf, mf, mu, reached;
  int mode, skipped, pad[2];
  double red[3 * kPipeMaxP];  // every rank's (vertices, edges, unknown sources) of the level
};
struct bu_reports {
  bu_report r[2];
};

__global__ void k_bu_init(bu_state* st, double m_u, double reached)
{
  st->m_u     = m_u;
  st->reached = reached;
  st->mode    = 1;
}

// a pipelined level's counts (every rank's, allgathered) -> the next level's mode by the
// host loop's rule (mg_bfs_impl: back to top-down only below V / beta frontier vertices
// with more than V / tdback unvisited), reported with the counts; a no-op level
// reports itself skipped and changes nothing
__global__ void k_bu_ctl(double const* red_all, int P, bu_state* st, bu_report* rep, double nv, double beta,
                         double tdback)
{
  int const t = threadIdx.x;
  if (st->mode != 1) {
    if (t == 0) {
      rep->skipped = 1;
      rep->mode    = st->mode;
    }
    return;
  }
  for (int i = t; i < 3 * P; i += blockDim.x) rep->red[i] = red_all[i];
  if (t) return;
  double nf = 0, mf = 0;
  for (int q = 0; q < P; ++q) {
    nf += red_all[3 * q];
    mf += red_all[3 * q + 1];
  }
  double const reached = st->reached + nf;
  double const mu      = st->m_u > mf ? st->m_u - mf : 0.0;
  int md               = 1;
  if (nf == 0) md = 2;
  else if (nf < nv / beta && nv - reached > nv / tdback) md = 0;
  st->reached  = reached;
  st->m_u      = mu;
  st->mode     = md;
  rep->nf      = nf;
  rep->mf      = mf;
  rep->mu      = mu;
  rep->reached = reached;
  rep->mode    = md;
  rep->skipped = 0;
}

template <typename V>
__global__ void k_pred_to_ext(V* pred, int64_t n, V const* nmap, int64_t nv)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t const p = (int64_t)pred[i];
    pred[i]         = p >= 0 && p < nv ? nmap[p] : (V)-1;
  }
}

struct deg_sum_f {
  int64_t const* off;
  __device__ double operator()(size_t i) const { return (double)(off[i + 1] - off[i]); }
};

template <typename V>
void mg_bfs_impl(handle_t& h, graph_t& g, array_view_t* sources, bool dir_opt, size_t depth_limit, bool want_pred,
                 paths_result_t& res)
{
  hipStream_t s   = h.stream;
  mg_context& ctx = *h.mg;
  comm_t& comm    = *ctx.world;
  mg_graph_t& mg  = *g.mg;
  int const P     = mg.P;
  CGX_INPUT(!dir_opt || g.symmetric,
            "Invalid input argument: input graph should be symmetric for direction optimizing BFS.");
  // every rank's source count (one host read), then every rank sees every source
  auto const src_counts = comm.host_allgather<int64_t>((int64_t)sources->size, s);
  int64_t nsrc_total = 0, src_mx = 0;
  for (auto c : src_counts) nsrc_total += c, src_mx = std::max(src_mx, c);
  CGX_INPUT(nsrc_total > 0, "Invalid input argument: input should have at least one source");
  bfs_rows_t& rows = mg_rows<V>(h, g);
  if (dir_opt && rows.n_own && rows.head.empty()) {
    rows.head.set_stream(s);
    rows.head.resize(rows.n_own * sizeof(v4u_t));
    hipLaunchKernelGGL(k_mg_head, dim3(blocks(rows.n_own)), dim3(kBlock), 0, s, rows.off.data<int64_t>(),
                       rows.pos.data<uint32_t>(), rows.n_own, rows.head.data<v4u_t>());
    CGX_LAUNCH_CHECK();
  }
  int64_t const n_own = mg.n_own(), lo = mg.voff[mg.p], hi = mg.voff[mg.p + 1];
  V const INF = std::numeric_limits<V>::max();

  res.vertices = std::make_unique<device_array_t>((size_t)n_own, g.vertex_type, s);
  if (n_own)
    HIP_CHECK(hipMemcpyAsync(res.vertices->buf.data(), g.number_map.data(), n_own * sizeof(V), hipMemcpyDeviceToDevice,
                             s));
  res.distances    = std::make_unique<device_array_t>((size_t)n_own, g.vertex_type, s);
  res.predecessors = std::make_unique<device_array_t>(want_pred ? (size_t)n_own : 0, g.vertex_type, s);
  V* dist = res.distances->buf.data<V>();
  V* pred = want_pred ? res.predecessors->buf.data<V>() : nullptr;
  fill<V>(dist, std::max<int64_t>(n_own, 0), INF, s);
  if (pred) fill<V>(pred, std::max<int64_t>(n_own, 0), INF, s);
  h.last_bfs_levels    = 0;
  h.last_bfs_bottom_up = 0;

  // sources: external -> global ids through the replicated id maps (no exchange;
  // unknown ids become -1, counted by k_init_sources), gathered to every rank (pads
  // -2), claimed by their owners
  dbuf<V> all_src;
  {
    int64_t const mx = std::max<int64_t>(src_mx, 1);
    dbuf<V> pad(mx, s), gath(mx * P, s);
    fill<V>(pad.data(), mx, (V)-2, s);
    if (sources->size) {
      HIP_CHECK(hipMemcpyAsync(pad.data(), sources->data, sources->size * sizeof(V), hipMemcpyDeviceToDevice, s));
      mg_ext_to_global_local(h, g, pad.data(), sources->size);
    } else {
      mg_ensure_replicated_ids(h, g);
    }
    comm.allgather<V>(pad.data(), gath.data(), (size_t)mx, s);
    all_src   = std::move(gath);
    all_src.n = (size_t)mx * P;
  }
  dbuf<uint32_t> qa(std::max<int64_t>(n_own, 1), s), qb(std::max<int64_t>(n_own, 1), s);
  dbuf<int> flag(std::max<int64_t>(n_own, 1), s);
  fill<int>(flag.data(), std::max<int64_t>(n_own, 1), 0, s);
  dbuf<long long> best(std::max<int64_t>(n_own, 1), s);
  fill<long long>(best.data(), std::max<int64_t>(n_own, 1), std::numeric_limits<long long>::max(), s);
  dbuf<level_ctr> ctr(1, s);
  HIP_CHECK(hipMemsetAsync(ctr.data(), 0, sizeof(level_ctr), s));
  hipLaunchKernelGGL(k_init_sources<V>, dim3(blocks(all_src.n)), dim3(kBlock), 0, s, all_src.data(), all_src.n, lo, hi,
                     dist, qa.data(), ctr.data(), flag.data(), rows.off.data<int64_t>());
  CGX_LAUNCH_CHECK();

  dbuf<int64_t> voff_d(P + 1, s);
  HIP_CHECK(hipMemcpyAsync(voff_d.data(), mg.voff.data(), (P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  // own frontier bitmap segments (current / next: the probe writes every word of the
  // next, so neither needs a memset per level once cleared here) and the allgathered bitmap
  dbuf<uint32_t> seg(rows.words, s), seg_next(rows.words, s), bitmap(rows.words * P, s);
  HIP_CHECK(hipMemsetAsync(seg_next.data(), 0, rows.words * 4, s));
  dbuf<uint32_t> resq(dir_opt ? std::max<int64_t>(kParts * mg_residual_cap(n_own), 1) : 1, s);
  int64_t const W  = rows.words * 32;
  bool have_queue  = true;   // the own frontier is in qa (else in seg)
  // a level's counts: every rank's (vertices, edges, unknown sources) allgathered,
  // one read: the totals, this rank's and its row's frontier sizes
  dbuf<double> red(3, s), red_all(3 * (size_t)P, s);
  std::vector<int64_t> n_of(P, 0), m_of(P, 0);
  auto fold = [&]() {
    hipLaunchKernelGGL(k_level_fold, dim3(1), dim3(64), 0, s, ctr.data(), red.data());
    CGX_LAUNCH_CHECK();
    comm.allgather<double>(red.data(), red_all.data(), 3, s);
    auto const gr = to_host(red_all.data(), 3 * (size_t)P, s);
    int64_t nf_ = 0;
    double mf_  = 0;
    for (int q = 0; q < P; ++q) {
      n_of[q] = (int64_t)gr[3 * q];
      m_of[q] = (int64_t)gr[3 * q + 1];
      nf_ += n_of[q];
      mf_ += gr[3 * q + 1];
    }
    return std::make_tuple(nf_, mf_, (int64_t)gr[2]);
  };
  auto [nf, m_f, bad_src] = fold();
  CGX_INPUT(bad_src == 0, "Invalid input argument: vertex id not in the graph");
  int64_t nf_own  = n_of[mg.p];
  int64_t reached = nf;  // vertices with a distance (global)
  // m_u: degrees of the unvisited vertices (every stored edge once, less the sources')
  double m_u = (double)g.num_edges - m_f;
  V limit    = (V)std::min<unsigned long long>((unsigned long long)depth_limit,
                                               (unsigned long long)std::numeric_limits<V>::max());
  V depth    = 0;
  bool bottom_up = false;
  size_t levels = 0, bu_steps = 0;
  int const gb = bits_for((unsigned long long)std::max<int64_t>(g.num_vertices - 1, 0));  // candidate key bits
  // 2D top-down: the block CSR, the row / column communicators, the column owners' id ranges
  bfs_block_t& blk = mg_block_csr<V>(h, g);
  comm_t& rowc     = *ctx.row;
  comm_t& colc     = *ctx.col;
  CGX_EXPECTS(rowc.size == mg.C && colc.size == mg.R, CUGRAPH_INVALID_HANDLE,
              "MG BFS: the handle's grid does not match the graph's");
  std::vector<int64_t> colvoff(mg.R + 1);
  for (int q = 0; q < mg.R; ++q) colvoff[q] = mg.voff[q * mg.C + mg.p % mg.C];
  colvoff[mg.R] = g.num_vertices;
  dbuf<int64_t> colvoff_d(mg.R + 1, s);
  to_device(colvoff_d.data(), colvoff.data(), colvoff.size(), s);
  bool const pipe_bu = dir_opt && h.tune.mg_bfs_pipelined && P <= kPipeMaxP;
  dbuf<bu_state> bst(1, s);
  dbuf<bu_report> brep(2, s);
  hipEvent_t bev[2] = {nullptr, nullptr};
  bool decided = false;  // the direction of the next level was set by a pipelined segment's end
  while (nf > 0 && depth < limit) {
    if (dir_opt && !decided) {
      if (!bottom_up && m_f > m_u / h.tune.mg_bfs_alpha) bottom_up = true;
      // back to top-down (Beamer's beta) only while many vertices are unvisited: a
      // multi-GPU top-down level costs ~0.1-0.3 ms of small launches and exchanges,
      // a bottom-up level over the few vertices left of a small-diameter graph
      // ~20 us (RMAT-24 one rank: 1.45 -> 1.30 ms per traversal); a long-diameter
      // graph's tail (many levels, most vertices unvisited) still goes top-down
      else if (bottom_up && (double)nf < (double)g.num_vertices / h.tune.mg_bfs_beta &&
               (double)(g.num_vertices - reached) > (double)g.num_vertices / kTdBack)
        bottom_up = false;
    }
    decided        = false;
    V const depth1 = depth + 1;  // (the counters were cleared by the last fold)
    if (bottom_up && pipe_bu) {
      // the rest of the bottom-up run, enqueued a level ahead (see bu_state)
      if (!bev[0])
        for (auto& e : bev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      bu_reports* hrep = h.pinned_as<bu_reports>();
      hipLaunchKernelGGL(k_bu_init, dim3(1), dim3(1), 0, s, bst.data(), m_u, (double)reached);
      CGX_LAUNCH_CHECK();
      int const* mode = &bst.data()->mode;
      auto enqueue = [&](V d1, int slot) {
        if (have_queue) {  // queue -> own bitmap segment (the segment's first level: nf_own is known)
          HIP_CHECK(hipMemsetAsync(seg.data(), 0, rows.words * 4, s));
          if (nf_own)
            hipLaunchKernelGGL(k_mark_bits, dim3(blocks(nf_own)), dim3(kBlock), 0, s, qa.data(), nf_own, seg.data());
          CGX_LAUNCH_CHECK();
          have_queue = false;
        }
        comm.allgather<uint32_t>(seg.data(), bitmap.data(), (size_t)rows.words, s);
        if (n_own) {
          hipLaunchKernelGGL(k_mg_bu_probe<V>, dim3(grid_for((n_own + 63) / 64, kBlock / 64, 4096)), dim3(kBlock), 0,
                             s, n_own, rows.off.data<int64_t>(), rows.pos.data<uint32_t>(), rows.head.data<v4u_t>(),
                             dist, pred, bitmap.data(), voff_d.data(), W, d1, seg_next.data(), resq.data(), ctr.data(),
                             mode, bitmap.data() + (size_t)mg.p * rows.words, rows.words);
          CGX_LAUNCH_CHECK();
          hipLaunchKernelGGL(k_mg_bu_residual<V>, dim3(1024), dim3(kBlock), 0, s, n_own, rows.off.data<int64_t>(),
                             rows.pos.data<uint32_t>(), dist, pred, bitmap.data(), voff_d.data(), W, d1,
                             seg_next.data(), resq.data(), ctr.data(), mode);
          CGX_LAUNCH_CHECK();
        }
        std::swap(seg, seg_next);
        hipLaunchKernelGGL(k_level_fold, dim3(1), dim3(64), 0, s, ctr.data(), red.data());
        CGX_LAUNCH_CHECK();
        comm.allgather<double>(red.data(), red_all.data(), 3, s);
        hipLaunchKernelGGL(k_bu_ctl, dim3(1), dim3(64), 0, s, red_all.data(), P, bst.data(), brep.data() + slot,
                           (double)g.num_vertices, h.tune.mg_bfs_beta, kTdBack);
        CGX_LAUNCH_CHECK();
        HIP_CHECK(hipMemcpyAsync(&hrep->r[slot], brep.data() + slot, sizeof(bu_report), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipEventRecord(bev[slot], s));
      };
      int slot = 0;
      enqueue(depth1, slot);
      while (true) {
        bool const more = (V)(depth + 1) < limit;  // the level after this one may run
        if (more) enqueue((V)(depth + 2), slot ^ 1);
        HIP_CHECK(hipEventSynchronize(bev[slot]));
        bu_report const& r = hrep->r[slot];  // the level at depth: it ran bottom-up
        ++levels;
        ++bu_steps;
        ++depth;
        nf      = (int64_t)r.nf;
        m_f     = r.mf;
        m_u     = r.mu;
        reached = (int64_t)r.reached;
        for (int q = 0; q < P; ++q) {
          n_of[q] = (int64_t)r.red[3 * q];
          m_of[q] = (int64_t)r.red[3 * q + 1];
        }
        nf_own = n_of[mg.p];
        if (r.mode != 1 || !more) {
          if (more) HIP_CHECK(hipEventSynchronize(bev[slot ^ 1]));  // the level enqueued ahead: a no-op
          bottom_up = r.mode == 1;
          decided   = true;
          break;
        }
        slot ^= 1;
      }
      continue;
    }
    if (bottom_up) {
      if (have_queue) {  // queue -> own bitmap segment
        HIP_CHECK(hipMemsetAsync(seg.data(), 0, rows.words * 4, s));
        if (nf_own)
          hipLaunchKernelGGL(k_mark_bits, dim3(blocks(nf_own)), dim3(kBlock), 0, s, qa.data(), nf_own, seg.data());
        CGX_LAUNCH_CHECK();
      }
      comm.allgather<uint32_t>(seg.data(), bitmap.data(), (size_t)rows.words, s);
      if (n_own) {
        hipLaunchKernelGGL(k_mg_bu_probe<V>, dim3(grid_for((n_own + 63) / 64, kBlock / 64, 4096)), dim3(kBlock), 0, s,
                           n_own, rows.off.data<int64_t>(), rows.pos.data<uint32_t>(), rows.head.data<v4u_t>(), dist,
                           pred, bitmap.data(), voff_d.data(), W, depth1, seg_next.data(), resq.data(), ctr.data(),
                           nullptr, nullptr, 0);
        CGX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_mg_bu_residual<V>, dim3(1024), dim3(kBlock), 0, s, n_own, rows.off.data<int64_t>(),
                           rows.pos.data<uint32_t>(), dist, pred, bitmap.data(), voff_d.data(), W, depth1,
                           seg_next.data(), resq.data(), ctr.data(), nullptr);
        CGX_LAUNCH_CHECK();
      }
      std::swap(seg, seg_next);
      have_queue = false;
      ++bu_steps;
    } else {
      if (!have_queue) {  // own bitmap segment -> queue (nf_own vertices)
        if (nf_own)
          hipLaunchKernelGGL(k_seg_to_queue, dim3(grid_for(rows.words, kBlock, 4096)), dim3(kBlock), 0, s, seg.data(),
                             rows.words, qa.data(), &ctr.data()->nconv);
        CGX_LAUNCH_CHECK();
        have_queue = true;
      }
      // 2D: the row's own frontiers to every rank of the row (row-local source ids);
      // the row's frontier sizes and degree sums are the last level's counts
      int const row0 = (mg.p / mg.C) * mg.C;
      int64_t mx = 0, cap = 0;
      for (int q = row0; q < row0 + mg.C; ++q) {
        mx = std::max(mx, n_of[q]);
        cap += m_of[q];  // every candidate edge of the block leaves a row frontier vertex
      }
      int64_t const nfg = mx * (int64_t)rowc.size;
      dbuf<unsigned long long> tot(1, s);
      HIP_CHECK(hipMemsetAsync(tot.data(), 0, sizeof(unsigned long long), s));
      dbuf<uint32_t> fsend(std::max<int64_t>(mx, 1), s), fgath(std::max<int64_t>(nfg, 1), s);
      dbuf<unsigned long long> dg(std::max<int64_t>(nfg, 1), s), pre(std::max<int64_t>(nfg, 1), s);
      if (mx) {
        hipLaunchKernelGGL(k_to_row_local, dim3(blocks(mx)), dim3(kBlock), 0, s, qa.data(), nf_own,
                           lo - blk.row_lo, mx, fsend.data());
        CGX_LAUNCH_CHECK();
        rowc.allgather<uint32_t>(fsend.data(), fgath.data(), (size_t)mx, s);
        hipLaunchKernelGGL(k_gathered_degrees, dim3(blocks(nfg)), dim3(kBlock), 0, s, fgath.data(), nfg,
                           blk.off.data<int64_t>(), dg.data());
        CGX_LAUNCH_CHECK();
        exclusive_scan<unsigned long long, unsigned long long>(dg.data(), pre.data(), nfg, s);
        hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(64), 0, s, pre.data(), dg.data(), nfg, tot.data());
        CGX_LAUNCH_CHECK();
      }
      // the candidate count: below kCandRead the row's degree sum bounds it and the
      // buffer is sorted at that length (sentinels past the real count) with no host
      // read; above, the exact count is read (the sort's length then matters more)
      int64_t mcand = cap;
      if (mx && cap > kCandRead) mcand = (int64_t)to_host_scalar(tot.data(), s);
      if (!mx) mcand = 0;
      // candidates over the block, smallest parent per destination
      dbuf<unsigned long long> cand(std::max<int64_t>(mcand, 1), s), cs(std::max<int64_t>(mcand, 1), s),
        cu(std::max<int64_t>(mcand, 1), s);
      dbuf<size_t> cnt(1, s);
      if (mcand) {
        hipLaunchKernelGGL(k_block_candidates<V>, dim3(blocks(mcand)), dim3(kBlock), 0, s, fgath.data(), nfg,
                           pre.data(), mcand, tot.data(), blk.off.data<int64_t>(), blk.idx.data<uint32_t>(), blk.row_lo,
                           lo, hi, dist, gb, cand.data());
        CGX_LAUNCH_CHECK();
        radix_sort_keys<unsigned long long>(cand.data(), cs.data(), mcand, 0, 2 * gb, s);
        size_t tmp = 0;
        HIP_CHECK(rocprim::unique(nullptr, tmp, cs.data(), cu.data(), cnt.data(), (size_t)mcand, same_v{gb}, s));
        buffer t(tmp, s);
        HIP_CHECK(rocprim::unique(t.data(), tmp, cs.data(), cu.data(), cnt.data(), (size_t)mcand, same_v{gb}, s));
        // the run count stays on the device: unique leaves at least one run of mcand >= 1 keys
        hipLaunchKernelGGL(k_expand_cand, dim3(capped(mcand)), dim3(kBlock), 0, s, cu.data(), cnt.data(), gb);
        CGX_LAUNCH_CHECK();
      }
      // to the destinations' owners: the R ranks of column c (the sentinel run, if
      // any, sorts last and is dropped).
      int const Rn = colc.size;
      dbuf<int64_t> pos(Rn + 1, s);
      if (mcand)
        hipLaunchKernelGGL(k_split_points, dim3(1), dim3(64), 0, s, cu.data(), cnt.data(), colvoff_d.data(), Rn,
                           pos.data());
      // every column peer's buffer length (peer q of the column is in grid row q):
      // all small -> padded segments, no count read
      std::vector<int64_t> peer_m(Rn, 0);
      bool padded = true;
      for (int q = 0; q < Rn && padded; ++q) {
        int64_t pmx = 0, pcap = 0;
        for (int j = 0; j < mg.C; ++j) {
          pmx = std::max(pmx, n_of[q * mg.C + j]);
          pcap += m_of[q * mg.C + j];
        }
        peer_m[q] = pmx ? pcap : 0;
        padded    = peer_m[q] <= kPadSend;
      }
      std::vector<size_t> counts(Rn), rcnt(Rn);
      dbuf<unsigned long long> sendp(padded ? std::max<int64_t>((int64_t)Rn * mcand, 1) : 1, s);
      unsigned long long const* sendv = cu.data();
      if (padded) {
        if (mcand) {
          hipLaunchKernelGGL(k_pad_send, dim3(blocks((int64_t)Rn * mcand)), dim3(kBlock), 0, s, cu.data(), pos.data(),
                             Rn, mcand, sendp.data());
          CGX_LAUNCH_CHECK();
        }
        sendv = sendp.data();
        for (int q = 0; q < Rn; ++q) {
          counts[q] = (size_t)mcand;
          rcnt[q]   = (size_t)peer_m[q];
        }
      } else {
        // send counts from the split points, their allgather inside the column, one
        // read for both directions' counts
        dbuf<int64_t> cnts((size_t)Rn * (Rn + 1), s);
        hipLaunchKernelGGL(k_pos_counts, dim3(1), dim3(64), 0, s, pos.data(), Rn, mcand ? 1 : 0, cnts.data());
        CGX_LAUNCH_CHECK();
        colc.allgather<int64_t>(cnts.data(), cnts.data() + Rn, (size_t)Rn, s);
        auto const hc = to_host(cnts.data(), (size_t)Rn * (Rn + 1), s);
        for (int q = 0; q < Rn; ++q) {
          counts[q] = (size_t)hc[q];
          rcnt[q]   = (size_t)hc[Rn + (size_t)q * Rn + colc.rank];
        }
      }
      auto got = exchange_known<int64_t>(colc, reinterpret_cast<int64_t const*>(sendv), counts, rcnt, s);
      if (got.n)
        hipLaunchKernelGGL(k_td_claim<V>, dim3(capped(got.n)), dim3(kBlock), 0, s,
                           reinterpret_cast<unsigned long long const*>(got.data()), (int64_t)got.n, lo, dist,
                           best.data(), flag.data(), qb.data(), ctr.data());
      CGX_LAUNCH_CHECK();
      // the claim count stays on the device (at most got.n)
      if (got.n)
        hipLaunchKernelGGL(k_td_finalize<V>, dim3(capped(got.n)), dim3(kBlock), 0, s, qb.data(), depth1, dist, pred,
                           best.data(), rows.off.data<int64_t>(), ctr.data());
      CGX_LAUNCH_CHECK();
      std::swap(qa, qb);
    }
    std::tie(nf, m_f, std::ignore) = fold();
    reached += nf;
    nf_own = n_of[mg.p];
    m_u    = m_u > m_f ? m_u - m_f : 0;
    ++depth;
    ++levels;
  }
  for (auto& e : bev)
    if (e) HIP_CHECK(hipEventDestroy(e));
  h.last_bfs_levels    = levels;
  h.last_bfs_bottom_up = bu_steps;
  if (pred) {
    // global parent ids -> external ids through the replicated number map (built for the
    // sources at the start), unreached -> -1, in one pass
    if (n_own)
      hipLaunchKernelGGL(k_pred_to_ext<V>, dim3(blocks(n_own)), dim3(kBlock), 0, s, pred, n_own,
                         mg.rep_nmap.data<V>(), g.num_vertices);
    CGX_LAUNCH_CHECK();
  }
  HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace

void mg_run_bfs(handle_t& h, graph_t& g, array_view_t* sources, bool direction_optimizing, size_t depth_limit,
                bool compute_predecessors, bool /*expensive*/, paths_result_t& res)
{
  CGX_EXPECTS(h.mg != nullptr, CUGRAPH_INVALID_HANDLE, "multi-GPU graph used with a single-GPU resource handle");
  if (g.vertex_type == INT32)
    mg_bfs_impl<int32_t>(h, g, sources, direction_optimizing, depth_limit, compute_predecessors, res);
  else
    mg_bfs_impl<int64_t>(h, g, sources, direction_optimizing, depth_limit, compute_predecessors, res);
}

}  // namespace cgx
