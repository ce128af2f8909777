// PageRank power iteration on the pull (CSC) adjacency -- the hot path.
//
// Algorithm: cpp/src/link_analysis/pagerank_impl.cuh:48-293 (init :168-183, loop
// :209-292, stop rule :287-290).  The reference runs, per iteration, a copy, a
// dangling transform_reduce (host sync), a divide pass, the 4 segment SpMV
// kernels of prims/per_v_transform_reduce_incoming_outgoing_e.cuh and an L1
// transform_reduce (host sync).  Here ONE kernel per iteration does all of it:
//
//   for every vertex v (degree-binned lane groups, schedule.hpp):
//     s      = sum_{u in in(v)} x~[u] * w(u,v)        fp64 accumulation of fp32 gathers
//     pr'[v] = base + alpha*s (+ pers[v]*(alpha*dangling + 1 - alpha))
//     x~'[v] = pr'[v] / outw[v]   (0 for dangling)     -> the next iteration's gather source
//     diff  += |pr'[v] - pr[v]|,  dangling' += pr'[v] if outw[v] == 0
//   per-block (diff, dangling) partials; the last block to arrive (agent-scope
//   release/acquire ticket) reduces them in block order -- deterministic -- and
//   writes the next iteration's base, the convergence flag and the iteration count.
//
// The host enqueues iterations in chunks and reads the flag once per chunk; a
// kernel launched after convergence returns immediately, so no per-iteration
// host round trip remains (the reference has two).
//
// Roofline: HBM.  Algorithmic bytes per iteration = 4E (indices) + 4V (offsets,
// int32) + 4V (x~ read, compulsory) + 4V (pr' write) + 4V (outw) [+4E weights]
// = 4E + 16V.
#include "capi.hpp"
#include "prims.hpp"
#include "schedule.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace cgx {

struct pr_state {
  double base;         // unvarying part of the current iteration
  double pers_factor;  // alpha*dangling + 1 - alpha (personalised runs)
  double diff;         // L1 difference of the last iteration
  double dangling;     // dangling mass after the last iteration
  unsigned int ticket;
  int iter;
  int done;  // 0 running, 1 converged, 2 max_iterations reached
  int pad;
};

template <typename V, typename E, typename R>
struct pr_args {
  E const* off;
  V const* idx;
  R const* wgt;
  V const* order;  // processing order (nullptr: identity)
  work_item const* items;
  R const* x_in;
  R* x_out;
  R* pr;
  R const* outw;
  R const* pers;  // personalisation coefficients value/sum (nullptr: none)
  double alpha;
  double eps;
  int max_iter;
  int64_t nv;
  double* partials;
  pr_state* st;
};

namespace {

// the last-arriving block reduces the per-block (diff, dangling) partials and
// updates the iteration state (cdna_hip_programming.md §6 Guideline 16 ticket form)
template <typename V, typename E, typename R>
__device__ void finish_iteration(pr_args<V, E, R> const& a, double my_diff, double my_dang, bool count_iter)
{
  __shared__ double sm[4];
  __shared__ int s_last;
  double bd = block_sum_256(my_diff, sm);
  double bg = block_sum_256(my_dang, sm);
  if (threadIdx.x == 0) {
    a.partials[2 * blockIdx.x]     = bd;
    a.partials[2 * blockIdx.x + 1] = bg;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(&a.st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last     = (t == gridDim.x - 1);
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  double d = 0, g = 0;
  for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
    d += a.partials[2 * b];
    g += a.partials[2 * b + 1];
  }
  d = block_sum_256(d, sm);
  g = block_sum_256(g, sm);
  if (threadIdx.x == 0) {
    pr_state* st    = a.st;
    int it          = st->iter + (count_iter ? 1 : 0);
    st->iter        = it;
    st->diff        = d;
    st->dangling    = g;
    double pf       = g * a.alpha + (1.0 - a.alpha);
    st->pers_factor = pf;
    st->base        = a.pers ? 0.0 : pf / (double)a.nv;
    int done        = 0;
    if (count_iter) {
      if (d < a.eps) done = 1;
      else if (it >= a.max_iter) done = 2;
    }
    st->ticket = 0;
    st->done   = done;
  }
}

// init: x~ = pr / outw, dangling mass of the initial vector
template <typename V, typename E, typename R>
__global__ __launch_bounds__(256) void k_pr_init(pr_args<V, E, R> a)
{
  double dang = 0;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < a.nv; v += (int64_t)gridDim.x * blockDim.x) {
    R p  = a.pr[v];
    R ow = a.outw[v];
    if (ow == R(0)) {
      dang += (double)p;
      a.x_out[v] = R(0);
    } else {
      a.x_out[v] = (R)((double)p / (double)ow);
    }
  }
  finish_iteration<V, E, R>(a, 0.0, dang, false);
}

template <typename V, typename E, typename R, bool WEIGHTED>
__device__ __forceinline__ double row_partial(pr_args<V, E, R> const& a, E beg, E end, int lane, int w)
{
  double s0 = 0, s1 = 0;
  E e = beg + lane;
  for (; e + w < end; e += 2 * w) {
    V u0 = a.idx[e];
    V u1 = a.idx[e + w];
    R x0 = a.x_in[u0];
    R x1 = a.x_in[u1];
    if constexpr (WEIGHTED) {
      s0 += (double)x0 * (double)a.wgt[e];
      s1 += (double)x1 * (double)a.wgt[e + w];
    } else {
      s0 += (double)x0;
      s1 += (double)x1;
    }
  }
  if (e < end) {
    R x0 = a.x_in[a.idx[e]];
    if constexpr (WEIGHTED) s0 += (double)x0 * (double)a.wgt[e];
    else s0 += (double)x0;
  }
  return s0 + s1;
}

template <typename V, typename E, typename R, bool WEIGHTED>
__device__ __forceinline__ double row_partial_block(pr_args<V, E, R> const& a, E beg, E end, int tid)
{
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  E e = beg + tid;
  for (; e + 3 * 256 < end; e += 4 * 256) {
    V u0 = a.idx[e], u1 = a.idx[e + 256], u2 = a.idx[e + 512], u3 = a.idx[e + 768];
    R x0 = a.x_in[u0], x1 = a.x_in[u1], x2 = a.x_in[u2], x3 = a.x_in[u3];
    if constexpr (WEIGHTED) {
      s0 += (double)x0 * (double)a.wgt[e];
      s1 += (double)x1 * (double)a.wgt[e + 256];
      s2 += (double)x2 * (double)a.wgt[e + 512];
      s3 += (double)x3 * (double)a.wgt[e + 768];
    } else {
      s0 += (double)x0;
      s1 += (double)x1;
      s2 += (double)x2;
      s3 += (double)x3;
    }
  }
  for (; e < end; e += 256) {
    R x0 = a.x_in[a.idx[e]];
    if constexpr (WEIGHTED) s0 += (double)x0 * (double)a.wgt[e];
    else s0 += (double)x0;
  }
  return (s0 + s1) + (s2 + s3);
}

template <typename V, typename E, typename R>
__device__ __forceinline__ void vertex_update(pr_args<V, E, R> const& a, V v, double s, double base, double pf,
                                              double& my_diff, double& my_dang)
{
  R old    = a.pr[v];
  double n = base + a.alpha * s;
  if (a.pers) n += pf * (double)a.pers[v];
  R nr     = (R)n;
  a.pr[v]  = nr;
  my_diff += fabs((double)nr - (double)old);
  R ow = a.outw[v];
  if (ow == R(0)) {
    my_dang += (double)nr;
    a.x_out[v] = R(0);
  } else {
    a.x_out[v] = (R)((double)nr / (double)ow);
  }
}

template <typename V, typename E, typename R, bool WEIGHTED>
__global__ __launch_bounds__(256) void k_pr_iter(pr_args<V, E, R> a)
{
  __shared__ double sm[4];
  if (a.st->done) return;  // converged in an earlier launch of this chunk
  work_item const it = a.items[blockIdx.x];
  double const base  = a.st->base;
  double const pf    = a.st->pers_factor;
  double my_diff = 0, my_dang = 0;
  int const tid = threadIdx.x;
  if (it.width == 256) {
    for (int64_t p = it.begin; p < it.end; ++p) {
      V v      = a.order ? a.order[p] : (V)p;
      double s = row_partial_block<V, E, R, WEIGHTED>(a, a.off[v], a.off[v + 1], tid);
      s        = block_sum_256(s, sm);
      if (tid == 0) vertex_update<V, E, R>(a, v, s, base, pf, my_diff, my_dang);
    }
  } else {
    int const w      = it.width;
    int const lane   = tid & (w - 1);
    int const group  = tid / w;
    int const groups = 256 / w;
    for (int64_t p0 = it.begin; p0 < it.end; p0 += groups) {
      int64_t p  = p0 + group;
      bool valid = p < it.end;
      double s   = 0;
      V v        = 0;
      if (valid) {
        v = a.order ? a.order[p] : (V)p;
        s = row_partial<V, E, R, WEIGHTED>(a, a.off[v], a.off[v + 1], lane, w);
      }
      for (int o = w >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (valid && lane == 0) vertex_update<V, E, R>(a, v, s, base, pf, my_diff, my_dang);
    }
  }
  finish_iteration<V, E, R>(a, my_diff, my_dang, true);
}

// ---------------------------------------------------------------- edge-tiled iteration
// Identity processing order (renumbered: rows sorted by descending degree).
//
// Two kernels per iteration:
//  * k_pr_push: the nhub highest-degree rows ("hubs", ids [0, nhub)) are not pulled:
//    their in-neighbours are spread over the whole vertex range, so pulled gathers
//    would be uniformly random (Infinity-Cache/HBM misses).  Instead every vertex u
//    pushes x~[u] (x w) to its hub out-neighbours, read from a compact "hub CSR"
//    (the id < nhub prefix of each sorted out-adjacency row, 16-bit ids) that is
//    streamed once, into per-block LDS accumulators.  Accumulation is in 64-bit
//    fixed point (scale 2^62; every hub sum is <= the total rank mass 1), so the
//    result is exact integer arithmetic: order-independent and bitwise
//    deterministic.  Blocks flush into a global fixed-point vector with integer
//    atomics.
//  * k_pr_stream (persistent): hub rows (fixed point -> fp64), rows of degree >=
//    kTileHalf one block per row, edge tiles of whole low-degree rows (< kTile edges:
//    coalesced non-temporal index loads + 8 independent gathers per thread; row data
//    prefetched into LDS so a tile costs two dependent memory latencies), then the
//    zero-degree rows; one ticket per block for the iteration state.
constexpr int kTileHalf   = 1024;           // rows below this degree are tiled
constexpr int kTile       = 2 * kTileHalf;  // max edges (and rows) per tile = 8 per thread
constexpr int kZeroRows   = 2048;           // rows per zero-degree unit
constexpr int kHubMax     = 8192;           // LDS accumulators per push block (64 KB)
constexpr int kPushThreads = 512;
constexpr double kFixScale    = 4611686018427387904.0;  // 2^62
constexpr double kFixScaleInv = 1.0 / 4611686018427387904.0;

struct tile_desc {
  int64_t rb, re;  // rows [rb, re)
  int64_t eb, ee;  // edges [eb, ee) = [off[rb], off[re])
};

struct push_unit {
  int64_t k0, k1;  // entries
  int64_t base;    // source id of (entry >> kHubBits) == 0
};

template <typename V, typename E, typename R>
struct pr_stream_args {
  pr_args<V, E, R> a;
  tile_desc const* tiles;
  // push side (hub rows)
  uint32_t const* push_ent;      // (source offset << kHubBits) | hub id, grouped by source
  struct push_unit const* push_units;
  int64_t npush_units;
  R const* hub_w;                // their weights (weighted graphs)
  unsigned long long* hub_acc;   // [nhub] fixed-point sums (zeroed; reset by k_pr_stream)
  int64_t nhub;
  int64_t nmid;                  // rows [nhub, nmid): degree >= kTileHalf, one block each
  int64_t ntiles, nzero_units, zero_row;
  int ablate;  // measurement only (CGX_PR_ABLATE): 1 no gathers, 2 no row phase, 4 no push, 8 no tiles
};

template <typename T>
__device__ __forceinline__ T nt_load(T const* p)
{
  return __builtin_nontemporal_load(p);
}

__device__ __forceinline__ unsigned long long to_fixed(double v)
{
  return (unsigned long long)__double2ull_rn(v * kFixScale);
}

// push entries: (source - unit base) << kHubBits | hub id, grouped by source; a unit
// covers <= kPushUnit entries of sources within 2^(32-kHubBits) of its base
constexpr int kHubBits  = 13;  // kHubMax = 2^13
constexpr int kPushUnit = 8 * kPushThreads;

template <typename V, typename E, typename R, bool WEIGHTED>
__global__ __launch_bounds__(kPushThreads) void k_pr_push(pr_stream_args<V, E, R> sa)
{
  __shared__ unsigned long long acc[kHubMax];
  auto const& a = sa.a;
  if (a.st->done || (sa.ablate & 4)) return;
  int const tid  = threadIdx.x;
  int const nhub = (int)sa.nhub;
  for (int i = tid; i < nhub; i += kPushThreads) acc[i] = 0ull;
  __syncthreads();
  for (int64_t un = blockIdx.x; un < sa.npush_units; un += gridDim.x) {
    push_unit const pu = sa.push_units[un];
    uint32_t ent[8];
    R w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int64_t k = pu.k0 + j * kPushThreads + tid;
      ent[j]    = k < pu.k1 ? nt_load(sa.push_ent + k) : 0xffffffffu;
      if constexpr (WEIGHTED) w[j] = k < pu.k1 ? nt_load(sa.hub_w + k) : R(0);
    }
    R x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      x[j] = ent[j] != 0xffffffffu ? a.x_in[pu.base + (int64_t)(ent[j] >> kHubBits)] : R(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (ent[j] != 0xffffffffu && x[j] != R(0)) {
        double v = (double)x[j];
        if constexpr (WEIGHTED) v *= (double)w[j];
        atomicAdd(&acc[ent[j] & (kHubMax - 1)], to_fixed(v));
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < nhub; i += kPushThreads)
    if (acc[i]) atomicAdd(sa.hub_acc + i, acc[i]);
}

// LDS image of one tile (rows <= kTile, edges < kTile).  Small (16-24 KB) so that 6-8
// blocks fit a CU: the gathers are latency-bound and need the occupancy.
template <typename R, bool WEIGHTED>
struct tile_lds {
  using val_t = std::conditional_t<WEIGHTED, double, R>;
  val_t vals[kTile];   // gathered (weighted) values in edge order
  int off[kTile + 1];  // row offsets relative to eb
};

template <typename V, typename E, typename R>
__device__ __forceinline__ void vertex_update_lds(pr_args<V, E, R> const& a, V v, R old, R ow, double s, double base,
                                                  double pf, double& my_diff, double& my_dang)
{
  double n = base + a.alpha * s;
  if (a.pers) n += pf * (double)a.pers[v];
  R nr    = (R)n;
  a.pr[v] = nr;
  my_diff += fabs((double)nr - (double)old);
  if (ow == R(0)) {
    my_dang += (double)nr;
    a.x_out[v] = R(0);
  } else {
    a.x_out[v] = (R)((double)nr / (double)ow);
  }
}

// One tile: every global load is issued up front (indices, weights, row offsets into
// LDS, old pagerank and out-weights into registers), then the gathers, so a tile
// costs two dependent memory latencies; per-row sums run out of LDS.
template <typename V, typename E, typename R, bool WEIGHTED>
__device__ void pr_tile(pr_stream_args<V, E, R> const& sa, tile_desc const& t, double base, double pf,
                        double& my_diff, double& my_dang, tile_lds<R, WEIGHTED>& L)
{
  auto const& a   = sa.a;
  int const tid   = threadIdx.x;
  int const lane  = tid & 63, wid = tid >> 6;
  int const nrows = (int)(t.re - t.rb);
  E const eb = (E)t.eb, ee = (E)t.ee;
  bool const wave_rows = (int64_t)(ee - eb) >= 32 * (int64_t)nrows;  // <= 64 rows: one wave per row
  V u[8];
  R w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    E e  = eb + j * 256 + tid;
    u[j] = e < ee ? nt_load(a.idx + e) : V(0);
    if constexpr (WEIGHTED) w[j] = e < ee ? nt_load(a.wgt + e) : R(0);
  }
  for (int i = tid; i <= nrows; i += 256) L.off[i] = (int)(a.off[t.rb + i] - eb);
  R rpr[8], row_[8];
  if (wave_rows) {  // lane l holds row wid + 4 l
    int i = wid + 4 * lane;
    rpr[0] = i < nrows ? a.pr[t.rb + i] : R(0);
    row_[0] = i < nrows ? a.outw[t.rb + i] : R(0);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int i   = tid + k * 256;
      rpr[k]  = i < nrows ? a.pr[t.rb + i] : R(0);
      row_[k] = i < nrows ? a.outw[t.rb + i] : R(0);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    E e = eb + j * 256 + tid;
    if (e < ee) {
      R x = (sa.ablate & 1) ? (R)u[j] : a.x_in[u[j]];
      if constexpr (WEIGHTED) L.vals[j * 256 + tid] = (double)x * (double)w[j];
      else L.vals[j * 256 + tid] = x;
    }
  }
  __syncthreads();
  if (!(sa.ablate & 2)) {
    if (wave_rows) {
      for (int i = wid, k = 0; i < nrows; i += 4, ++k) {
        int lo = L.off[i], hi = L.off[i + 1];
        double s = 0;
        for (int q = lo + lane; q < hi; q += 64) s += (double)L.vals[q];
        s        = wave_sum(s);
        R old    = __shfl(rpr[0], k, 64);
        R ow     = __shfl(row_[0], k, 64);
        if (lane == 0) vertex_update_lds<V, E, R>(a, (V)(t.rb + i), old, ow, s, base, pf, my_diff, my_dang);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        int i = tid + k * 256;
        if (i < nrows) {
          int lo = L.off[i], hi = L.off[i + 1];
          double s = 0;
          for (int q = lo; q < hi; ++q) s += (double)L.vals[q];
          vertex_update_lds<V, E, R>(a, (V)(t.rb + i), rpr[k], row_[k], s, base, pf, my_diff, my_dang);
        }
      }
    }
  }
  __syncthreads();
}

// one block per row of degree >= kTileHalf (rows [nhub, nmid)), 8 edges per thread per round
template <typename V, typename E, typename R, bool WEIGHTED>
__device__ void pr_block_row(pr_args<V, E, R> const& a, int64_t r, double base, double pf, double& my_diff,
                             double& my_dang, double* sm)
{
  int const tid = threadIdx.x;
  E const e0 = a.off[r], e1 = a.off[r + 1];
  double s0 = 0, s1 = 0;
  for (E b = e0; b < e1; b += 8 * 256) {
    V u[8];
    R w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      E e  = b + j * 256 + tid;
      u[j] = e < e1 ? nt_load(a.idx + e) : V(0);
      if constexpr (WEIGHTED) w[j] = e < e1 ? nt_load(a.wgt + e) : R(0);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      E e = b + j * 256 + tid;
      if (e < e1) {
        double t = (double)a.x_in[u[j]];
        if constexpr (WEIGHTED) t *= (double)w[j];
        if (j & 1) s1 += t;
        else s0 += t;
      }
    }
  }
  double s = block_sum_256(s0 + s1, sm);
  if (tid == 0) vertex_update<V, E, R>(a, (V)r, s, base, pf, my_diff, my_dang);
}

template <typename V, typename E, typename R, bool WEIGHTED>
__global__ __launch_bounds__(256) void k_pr_stream(pr_stream_args<V, E, R> sa)
{
  __shared__ tile_lds<R, WEIGHTED> L;
  __shared__ double sm[4];
  auto const& a = sa.a;
  if (a.st->done) return;
  double const base = a.st->base;
  double const pf   = a.st->pers_factor;
  double my_diff = 0, my_dang = 0;
  int64_t const nhubu = (sa.nhub + 255) / 256;
  int64_t const nmid  = sa.nmid - sa.nhub;
  int64_t const total = nhubu + nmid + sa.ntiles + sa.nzero_units;
  for (int64_t u = blockIdx.x; u < total; u += gridDim.x) {
    if (u < nhubu) {  // hub rows: fixed-point push sums -> fp64
      int64_t r = u * 256 + threadIdx.x;
      if (r < sa.nhub) {
        unsigned long long f = sa.hub_acc[r];
        sa.hub_acc[r]        = 0ull;  // ready for the next iteration's push
        vertex_update<V, E, R>(a, (V)r, (double)f * kFixScaleInv, base, pf, my_diff, my_dang);
      }
    } else if (u < nhubu + nmid) {
      pr_block_row<V, E, R, WEIGHTED>(a, sa.nhub + (u - nhubu), base, pf, my_diff, my_dang, sm);
    } else if (u < nhubu + nmid + sa.ntiles) {
      if (sa.ablate & 8) continue;
      tile_desc t = sa.tiles[u - nhubu - nmid];
      pr_tile<V, E, R, WEIGHTED>(sa, t, base, pf, my_diff, my_dang, L);
    } else {
      int64_t r0 = sa.zero_row + (u - nhubu - nmid - sa.ntiles) * kZeroRows;
      int64_t r1 = r0 + kZeroRows < a.nv ? r0 + kZeroRows : a.nv;
      for (int64_t r = r0 + threadIdx.x; r < r1; r += 256)
        vertex_update<V, E, R>(a, (V)r, 0.0, base, pf, my_diff, my_dang);
    }
  }
  finish_iteration<V, E, R>(a, my_diff, my_dang, true);
}

// hub_cnt[u] = number of out-neighbours of u with id < nhub (prefix of the sorted row)
template <typename V, typename E>
__global__ void k_hub_count(E const* off, V const* idx, int64_t nv, int64_t nhub, int64_t* cnt)
{
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < nv; u += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = (int64_t)off[u], hi = (int64_t)off[u + 1], b = lo;
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if ((int64_t)idx[mid] < nhub) lo = mid + 1;
      else hi = mid;
    }
    cnt[u] = lo - b;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[nv] = 0;
}

// unit_base[i] = source row of entry i * kPushUnit (last row whose offset <= it)
__global__ void k_push_unit_base(int64_t const* hoff, int64_t nv, int64_t nunits, int64_t* unit_base)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nunits; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t k  = i * kPushUnit;
    int64_t lo = 0, hi = nv;  // last u with hoff[u] <= k
    while (lo < hi) {
      int64_t mid = (lo + hi + 1) >> 1;
      if (hoff[mid] <= k) lo = mid;
      else hi = mid - 1;
    }
    unit_base[i] = lo;
  }
}

template <typename V, typename E, typename R>
__global__ void k_hub_fill(E const* off, V const* idx, R const* w, int64_t nv, int64_t const* hoff,
                           int64_t const* unit_base, uint32_t* ent, R* hw, int* bad)
{
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < nv; u += (int64_t)gridDim.x * blockDim.x) {
    int64_t k0 = hoff[u], k1 = hoff[u + 1];
    E e = off[u];
    for (int64_t k = k0; k < k1; ++k, ++e) {
      int64_t rel = u - unit_base[k / kPushUnit];
      if (rel >= (int64_t(1) << (32 - kHubBits))) atomicAdd(bad, 1);
      ent[k] = ((uint32_t)rel << kHubBits) | (uint32_t)idx[e];
      if (hw) hw[k] = w[e];
    }
  }
}

__global__ void k_push_units(int64_t const* unit_base, int64_t nunits, int64_t nent, push_unit* units)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nunits; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t k0 = i * kPushUnit;
    int64_t k1 = k0 + kPushUnit < nent ? k0 + kPushUnit : nent;
    units[i]   = push_unit{k0, k1, unit_base[i]};
  }
}

template <typename E>
__global__ void k_tile_desc(E const* off, int64_t const* rows, int64_t ntiles, tile_desc* out)
{
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < ntiles; k += (int64_t)gridDim.x * blockDim.x)
    out[k] = tile_desc{rows[k], rows[k + 1], (int64_t)off[rows[k]], (int64_t)off[rows[k + 1]]};
}

template <typename E>
__global__ void k_tile_rows(E const* off, int64_t r0, int64_t r1, int64_t ntiles, int64_t* out)
{
  E base = off[r0];
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k <= ntiles; k += (int64_t)gridDim.x * blockDim.x) {
    if (k == ntiles) {
      out[k] = r1;
      continue;
    }
    E t = base + (E)(k * kTileHalf);
    int64_t lo = r0, hi = r1;  // first row in [r0, r1) with off[row] >= t
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if (off[mid] < t) lo = mid + 1;
      else hi = mid;
    }
    out[k] = lo;
  }
}

template <typename E>
__global__ void k_first_below(E const* off, int64_t nv, int64_t t0, int64_t t1, int64_t* out)
{
  // first row with degree < t (degrees non-increasing), for t0 and t1
  if (threadIdx.x >= 2) return;
  int64_t t  = threadIdx.x == 0 ? t0 : t1;
  int64_t lo = 0, hi = nv;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if ((int64_t)(off[mid + 1] - off[mid]) >= t) lo = mid + 1;
    else hi = mid;
  }
  out[threadIdx.x] = lo;
}

// Schedule (cached on the pull adjacency): hub count, the hub CSR built from the
// out-adjacency (same object for symmetric graphs), block rows, tiles.
template <typename V, typename E, typename R>
void build_pr_stream_schedule(handle_t& h, graph_t& g, adjacency_t& adj)
{
  hipStream_t s  = h.stream;
  int64_t nv     = g.num_vertices;
  E const* off   = adj.offsets.data<E>();
  dbuf<int64_t> fb(2, s);
  hipLaunchKernelGGL(k_first_below<E>, dim3(1), dim3(64), 0, s, off, nv, (int64_t)kTileHalf, (int64_t)1, fb.data());
  CGX_LAUNCH_CHECK();
  auto hb = to_host(fb.data(), 2, s);
  int64_t nmid = hb[0], nzero = hb[1];
  int64_t nhub = std::min<int64_t>(nmid, kHubMax);
  adj.pr_nhub = nhub;
  adj.pr_nmid = nmid;
  // hub CSR from the out-adjacency (rows sorted ascending: hubs are each row's prefix)
  adjacency_t& out = ensure_adjacency(h, g, false);
  E const* ooff    = out.offsets.data<E>();
  V const* oidx    = out.indices.data<V>();
  dbuf<int64_t> cnt(nv + 1, s);
  hipLaunchKernelGGL((k_hub_count<V, E>), dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, ooff, oidx, nv, nhub,
                     cnt.data());
  CGX_LAUNCH_CHECK();
  adj.pr_hub_off.set_stream(s);
  adj.pr_hub_off.resize((nv + 1) * sizeof(int64_t));
  exclusive_scan<int64_t, int64_t>(cnt.data(), adj.pr_hub_off.data<int64_t>(), nv + 1, s);
  int64_t nent = to_host(adj.pr_hub_off.data<int64_t>() + nv, 1, s)[0];
  int64_t nunits = (nent + kPushUnit - 1) / kPushUnit;
  dbuf<int64_t> ubase(std::max<int64_t>(nunits, 1), s);
  if (nunits)
    hipLaunchKernelGGL(k_push_unit_base, dim3(grid_for(nunits, kBlock, 4096)), dim3(kBlock), 0, s,
                       adj.pr_hub_off.data<int64_t>(), nv, nunits, ubase.data());
  CGX_LAUNCH_CHECK();
  adj.pr_hub_idx.set_stream(s);
  adj.pr_hub_idx.resize(std::max<int64_t>(nent, 1) * sizeof(uint32_t));
  adj.pr_hub_w.set_stream(s);
  if (g.weighted) adj.pr_hub_w.resize(std::max<int64_t>(nent, 1) * sizeof(R));
  else adj.pr_hub_w.release();
  dbuf<int> bad(1, s);
  fill<int>(bad.data(), 1, 0, s);
  hipLaunchKernelGGL((k_hub_fill<V, E, R>), dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, ooff, oidx,
                     g.weighted ? out.weights.data<R>() : nullptr, nv, adj.pr_hub_off.data<int64_t>(), ubase.data(),
                     adj.pr_hub_idx.data<uint32_t>(), g.weighted ? adj.pr_hub_w.data<R>() : nullptr, bad.data());
  CGX_LAUNCH_CHECK();
  adj.pr_push_units.set_stream(s);
  adj.pr_push_units.resize(std::max<int64_t>(nunits, 1) * sizeof(push_unit));
  if (nunits)
    hipLaunchKernelGGL(k_push_units, dim3(grid_for(nunits, kBlock, 4096)), dim3(kBlock), 0, s, ubase.data(), nunits,
                       nent, adj.pr_push_units.data<push_unit>());
  CGX_LAUNCH_CHECK();
  adj.pr_npush_units = nunits;
  adj.pr_push_ok     = to_host_scalar(bad.data(), s) == 0;
  adj.pr_hub_off.release();  // only needed to build the entries
  adj.pr_hub_acc.set_stream(s);
  adj.pr_hub_acc.resize(std::max<int64_t>(nhub, 1) * sizeof(unsigned long long));
  HIP_CHECK(hipMemsetAsync(adj.pr_hub_acc.data(), 0, std::max<int64_t>(nhub, 1) * sizeof(unsigned long long), s));
  // edge tiles over the remaining non-empty rows [nmid, nzero)
  E o_mid  = to_host(off + nmid, 1, s)[0];
  E o_zero = to_host(off + nzero, 1, s)[0];
  int64_t ntiles = ((int64_t)(o_zero - o_mid) + kTileHalf - 1) / kTileHalf;
  adj.pr_ntiles      = ntiles;
  adj.pr_nzero_row   = nzero;
  adj.pr_nzero_tiles = (nv - nzero + kZeroRows - 1) / kZeroRows;
  adj.pr_tile_rows.set_stream(s);
  {
    dbuf<int64_t> rows(ntiles + 1, s);
    hipLaunchKernelGGL(k_tile_rows<E>, dim3(grid_for(ntiles + 1, kBlock, 4096)), dim3(kBlock), 0, s, off, nmid, nzero,
                       ntiles, rows.data());
    CGX_LAUNCH_CHECK();
    adj.pr_tile_rows.resize(std::max<int64_t>(ntiles, 1) * sizeof(tile_desc));
    if (ntiles)
      hipLaunchKernelGGL(k_tile_desc<E>, dim3(grid_for(ntiles, kBlock, 4096)), dim3(kBlock), 0, s, off, rows.data(),
                         ntiles, adj.pr_tile_rows.data<tile_desc>());
    CGX_LAUNCH_CHECK();
  }
  HIP_CHECK(hipStreamSynchronize(s));
  adj.pr_valid = true;
}

template <typename V, typename R>
__global__ void k_scatter_values(R* dst, V const* ids, R const* vals, size_t n, double scale)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[ids[i]] = (R)((double)vals[i] * scale);
}

template <typename R>
__global__ void k_count_negative(R const* p, size_t n, int* bad)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (p[i] < R(0)) atomicAdd(bad, 1);
}

template <typename R>
int count_negative(R const* p, size_t n, hipStream_t s)
{
  if (!n) return 0;
  dbuf<int> bad(1, s);
  fill<int>(bad.data(), 1, 0, s);
  hipLaunchKernelGGL(k_count_negative<R>, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, p, n, bad.data());
  CGX_LAUNCH_CHECK();
  return to_host_scalar(bad.data(), s);
}

template <typename V, typename R>
dbuf<V> internal_ids(handle_t& h, graph_t& g, array_view_t const* ext)
{
  dbuf<V> ids(ext->size, h.stream);
  if (ext->size)
    HIP_CHECK(hipMemcpyAsync(ids.data(), ext->data, ext->size * sizeof(V), hipMemcpyDefault, h.stream));
  renumber_ext_to_int(h, g, ids.data(), ext->size, true);
  return ids;
}

template <typename V, typename E, typename R>
void pagerank_impl(handle_t& h, graph_t& g, array_view_t const* pow_v, array_view_t const* pow_s,
                   array_view_t const* guess_v, array_view_t const* guess_s, array_view_t const* pers_v,
                   array_view_t const* pers_s, double alpha, double eps, size_t max_iter, bool expensive,
                   centrality_result_t& res)
{
  hipStream_t s = h.stream;
  CGX_INPUT(alpha >= 0.0 && alpha <= 1.0, "Invalid input argument: alpha should be in [0.0, 1.0].");
  CGX_INPUT(eps >= 0.0, "Invalid input argument: epsilon should be non-negative.");
  CGX_INPUT((pers_v == nullptr) == (pers_s == nullptr) && (!pers_v || pers_v->size == pers_s->size),
            "Invalid input argument: personalization vertices and values must be given together.");
  CGX_INPUT((guess_v == nullptr) == (guess_s == nullptr), "Invalid input argument: initial guess vertices and values must be given together.");
  CGX_INPUT((pow_v == nullptr) == (pow_s == nullptr), "Invalid input argument: precomputed out weight vertices and sums must be given together.");
  int64_t nv = g.num_vertices;
  res.vertices = number_map_copy(h, g);
  res.values   = std::make_unique<device_array_t>((size_t)nv, dtype_of<R>(), s);
  h.last_iterations = 0;
  h.last_hot_ms     = 0;
  h.last_hot_launches = 0;
  if (nv == 0) return;

  adjacency_t& adj = ensure_adjacency(h, g, /*transposed=*/true);
  ensure_schedule(h, g, adj);
  if (expensive && g.weighted) {
    CGX_INPUT(count_negative<R>(adj.weights.data<R>(), (size_t)g.num_edges, s) == 0,
              "Invalid input argument: input graph should have non-negative edge weights.");
  }

  // out-weight sums
  dbuf<R> outw_own;
  R const* outw = nullptr;
  if (pow_v) {
    outw_own.resize(nv, s);
    fill<R>(outw_own.data(), nv, R(0), s);
    auto ids = internal_ids<V, R>(h, g, pow_v);
    if (pow_v->size)
      hipLaunchKernelGGL((k_scatter_values<V, R>), dim3(grid_for(pow_v->size, kBlock, 4096)), dim3(kBlock), 0, s,
                         outw_own.data(), ids.data(), pow_s->as<R>(), pow_v->size, 1.0);
    CGX_LAUNCH_CHECK();
    if (expensive)
      CGX_INPUT(count_negative<R>(outw_own.data(), nv, s) == 0,
                "Invalid input argument: outgoing edge weight sum values should be non-negative.");
    outw = outw_own.data();
  } else {
    outw = static_cast<R const*>(out_weight_sums(h, g));
  }

  // initial values
  R* pr = res.values->buf.data<R>();
  if (guess_v) {
    fill<R>(pr, nv, R(0), s);
    auto ids = internal_ids<V, R>(h, g, guess_v);
    auto hv  = to_host(guess_s->as<R>(), guess_s->size, s);
    double sum = 0;
    for (auto x : hv) sum += (double)x;
    if (expensive) {
      for (auto x : hv) CGX_INPUT(x >= R(0), "Invalid input argument: initial guess values should be non-negative.");
    }
    CGX_INPUT(sum > 0.0, "Invalid input argument: sum of the PageRank initial guess values should be positive.");
    if (guess_v->size)
      hipLaunchKernelGGL((k_scatter_values<V, R>), dim3(grid_for(guess_v->size, kBlock, 4096)), dim3(kBlock), 0, s,
                         pr, ids.data(), guess_s->as<R>(), guess_v->size, 1.0 / sum);
    CGX_LAUNCH_CHECK();
  } else {
    fill<R>(pr, nv, (R)(R(1.0) / (R)nv), s);
  }

  // personalisation coefficients value / sum(values)
  dbuf<R> pers;
  if (pers_v && pers_v->size > 0) {
    auto hv    = to_host(pers_s->as<R>(), pers_s->size, s);
    double sum = 0;
    for (auto x : hv) {
      if (expensive) CGX_INPUT(x >= R(0), "Invalid input argument: peresonalization values should be non-negative.");
      sum += (double)x;
    }
    CGX_INPUT(sum > 0.0, "Invalid input argument: sum of personalization valuese should be positive.");
    pers.resize(nv, s);
    fill<R>(pers.data(), nv, R(0), s);
    auto ids = internal_ids<V, R>(h, g, pers_v);
    hipLaunchKernelGGL((k_scatter_values<V, R>), dim3(grid_for(pers_v->size, kBlock, 4096)), dim3(kBlock), 0, s,
                       pers.data(), ids.data(), pers_s->as<R>(), pers_v->size, 1.0 / sum);
    CGX_LAUNCH_CHECK();
  }

  // iteration state
  int const nblk_iter = (int)adj.num_items;
  int const nblk_init = (int)grid_for(nv, kBlock, 1024);
  dbuf<double> partials(2 * std::max({nblk_iter, nblk_init, 2048}), s);
  dbuf<pr_state> st(1, s);
  HIP_CHECK(hipMemsetAsync(st.data(), 0, sizeof(pr_state), s));
  dbuf<R> xa(nv, s), xb(nv, s);

  pr_args<V, E, R> a{};
  a.off      = adj.offsets.data<E>();
  a.idx      = adj.indices.data<V>();
  a.wgt      = g.weighted ? adj.weights.data<R>() : nullptr;
  a.order    = adj.degree_sorted ? nullptr : adj.order.data<V>();
  a.items    = adj.items.data<work_item>();
  a.pr       = pr;
  a.outw     = outw;
  a.pers     = pers.data();
  a.alpha    = alpha;
  a.eps      = eps;
  a.max_iter = (int)std::min<size_t>(max_iter, (size_t)INT32_MAX);
  a.nv       = nv;
  a.partials = partials.data();
  a.st       = st.data();
  a.x_in     = nullptr;
  a.x_out    = xa.data();
  hipLaunchKernelGGL((k_pr_init<V, E, R>), dim3(nblk_init), dim3(kBlock), 0, s, a);
  CGX_LAUNCH_CHECK();

  if (max_iter == 0) fail(CUGRAPH_UNKNOWN_ERROR, "PageRank failed to converge.");

  // identity order (degree-sorted majors) with our own out-weight sums: hub push + edge tiles
  // (user-precomputed out-weights could break the fixed-point bound: generic kernel then)
  bool stream = adj.degree_sorted && pow_v == nullptr;
  pr_stream_args<V, E, R> sa{};
  int nblk_stream = 0, nblk_push = 0;
  auto pkernel = g.weighted ? k_pr_push<V, E, R, true> : k_pr_push<V, E, R, false>;
  auto skernel = g.weighted ? k_pr_stream<V, E, R, true> : k_pr_stream<V, E, R, false>;
  if (stream) {
    if (!adj.pr_valid) build_pr_stream_schedule<V, E, R>(h, g, adj);
  }
  if (stream && !adj.pr_push_ok) stream = false;  // source span too wide for the packed entries
  if (stream) {
    sa.tiles       = adj.pr_tile_rows.data<tile_desc>();
    sa.push_ent    = adj.pr_hub_idx.data<uint32_t>();
    sa.push_units  = adj.pr_push_units.data<push_unit>();
    sa.npush_units = adj.pr_npush_units;
    sa.hub_w       = g.weighted ? adj.pr_hub_w.data<R>() : nullptr;
    sa.hub_acc     = adj.pr_hub_acc.data<unsigned long long>();
    sa.nhub        = adj.pr_nhub;
    sa.nmid        = adj.pr_nmid;
    sa.ntiles      = adj.pr_ntiles;
    sa.nzero_units = adj.pr_nzero_tiles;
    sa.zero_row    = adj.pr_nzero_row;
    if (char const* ab = std::getenv("CGX_PR_ABLATE")) sa.ablate = std::atoi(ab);
    int64_t units = (sa.nhub + 255) / 256 + (sa.nmid - sa.nhub) + sa.ntiles + sa.nzero_units;
    // persistent grids: as many blocks as the LDS footprint lets every CU hold
    size_t lds  = g.weighted ? sizeof(tile_lds<R, true>) : sizeof(tile_lds<R, false>);
    int per_cu  = (int)std::clamp<size_t>((160 * 1024) / (lds + 512), 1, 8);
    nblk_stream = (int)std::max<int64_t>(1, std::min<int64_t>(units, 256 * per_cu));
    nblk_push   = sa.nhub > 0 ? 512 : 0;
  }
  // chunked enqueue; profiling records HIP events around every iteration launch
  int const chunk = 8;
  std::vector<hipEvent_t> ev;
  pr_state hst{};
  R* bufs[2]    = {xa.data(), xb.data()};
  size_t launched = 0;
  auto kernel  = g.weighted ? k_pr_iter<V, E, R, true> : k_pr_iter<V, E, R, false>;
  pr_state* hpin = nullptr;
  HIP_CHECK(hipHostMalloc((void**)&hpin, sizeof(pr_state), hipHostMallocDefault));
  try {
    while (true) {
      for (int i = 0; i < chunk; ++i) {
        a.x_in  = bufs[launched & 1];
        a.x_out = bufs[(launched + 1) & 1];
        if (h.profiling) {
          hipEvent_t e0, e1;
          HIP_CHECK(hipEventCreate(&e0));
          HIP_CHECK(hipEventCreate(&e1));
          ev.push_back(e0);
          ev.push_back(e1);
          HIP_CHECK(hipEventRecord(e0, s));
        }
        if (stream) {
          sa.a = a;
          if (nblk_push) hipLaunchKernelGGL(pkernel, dim3(nblk_push), dim3(kPushThreads), 0, s, sa);
          hipLaunchKernelGGL(skernel, dim3(nblk_stream), dim3(kBlock), 0, s, sa);
        } else {
          hipLaunchKernelGGL(kernel, dim3(nblk_iter), dim3(kBlock), 0, s, a);
        }
        CGX_LAUNCH_CHECK();
        if (h.profiling) HIP_CHECK(hipEventRecord(ev.back(), s));
        ++launched;
      }
      HIP_CHECK(hipMemcpyAsync(hpin, st.data(), sizeof(pr_state), hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
      hst = *hpin;
      if (hst.done) break;
    }
  } catch (...) {
    (void)hipHostFree(hpin);
    for (auto e : ev) (void)hipEventDestroy(e);
    throw;
  }
  HIP_CHECK(hipHostFree(hpin));
  h.last_iterations = (size_t)hst.iter;
  if (h.profiling) {
    double tot = 0;
    size_t k   = std::min<size_t>((size_t)hst.iter, ev.size() / 2);
    for (size_t i = 0; i < k; ++i) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
      tot += ms;
    }
    for (auto e : ev) HIP_CHECK(hipEventDestroy(e));
    h.last_hot_ms       = tot;
    h.last_hot_launches = k;
  }
  if (hst.done == 2) fail(CUGRAPH_UNKNOWN_ERROR, "PageRank failed to converge.");
}

}  // namespace

void run_pagerank(handle_t& h, graph_t& g, array_view_t const* pow_v, array_view_t const* pow_s,
                  array_view_t const* guess_v, array_view_t const* guess_s, array_view_t const* pers_v,
                  array_view_t const* pers_s, double alpha, double eps, size_t max_iter, bool expensive,
                  centrality_result_t& res)
{
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    pagerank_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(
      h, g, pow_v, pow_s, guess_v, guess_s, pers_v, pers_s, alpha, eps, max_iter, expensive, res);
  });
}

}  // namespace cgx
