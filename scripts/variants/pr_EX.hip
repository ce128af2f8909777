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
    // write-through (sc1) partials: no agent release (an L2 write-back per block) needed
    __hip_atomic_store(&a.partials[2 * blockIdx.x], bd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.partials[2 * blockIdx.x + 1], bg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(&a.st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last     = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last) return;
  double d = 0, g = 0;
  for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) {  // sc1 loads: L1 bypassed
    d += __hip_atomic_load(&a.partials[2 * b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g += __hip_atomic_load(&a.partials[2 * b + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// ---------------------------------------------------------------- windowed push iteration
// A pulled gather x~[u] costs one L2 lookup per edge wherever u lands (random 4 B
// reads: ~300 G lookups/s for the whole chip, the bound of a CSC pull).  The push
// form below reads x~ in SOURCE order instead, so consecutive entries share cache
// lines, and scatters into LDS, which is per-CU and scales with the CUs:
//
//  * destinations are cut into windows of kWin ids (kWin u64 accumulators = 64 KB
//    of LDS per block);
//  * push entries are the CSC edges re-sorted by (window, source) and packed in
//    32 bits: (source - segment base) << kWinBits | (destination - window base),
//    a segment being the sources of one window inside one 2^kSrcBits-aligned block;
//  * units of <= kPushUnit entries never cross a segment, and blocks take
//    contiguous runs of units, so a block flushes its LDS window to the global
//    accumulator (integer atomics) only when the window changes -- once or twice;
//  * sums are 64-bit fixed point (scale 2^62; every destination's sum is at most
//    the total rank mass 1 since x~[u] w(u, v) summed over v is pr[u]).  Integer
//    addition is associative: the result is bitwise deterministic whatever the
//    order of the atomics.
//
// k_pr_apply then turns the sums into pr'/x~' per vertex (streaming) and resets the
// accumulators.  Per iteration HBM traffic: 4E (entries) [+4E weights] + x~ lines
// + 8V acc read + 8V acc reset + 16V vertex state.
constexpr int kWinBits     = 13;
constexpr int kWin         = 1 << kWinBits;
constexpr int kSrcBits     = 32 - kWinBits;  // 19
constexpr int kPushThreads = 1024;
constexpr int kPushUnit    = 8 * kPushThreads;
constexpr double kFixScale    = 4611686018427387904.0;  // 2^62
constexpr double kFixScaleInv = 1.0 / 4611686018427387904.0;

struct push_unit {
  int64_t k0, k1;  // entries [k0, k1)
  int64_t base;    // source id of offset 0
  int64_t win;     // destination window
};

template <typename V, typename E, typename R>
struct push_args {
  pr_args<V, E, R> a;
  uint32_t const* ent;
  R const* ew;  // entry weights (weighted graphs)
  push_unit const* units;
  int64_t nunits;
  unsigned long long* acc;  // [nwin * kWin] fixed-point sums, zero between iterations
  int ablate;  // measurement only (CGX_PR_ABLATE): 1 no gathers, 2 no LDS atomics, 4 no push
};

template <typename T>
__device__ __forceinline__ T nt_load(T const* p)
{
  return __builtin_nontemporal_load(p);
}

__device__ __forceinline__ unsigned long long to_fixed(double v)
{
  return (unsigned long long)__double2ll_rn(v * kFixScale);
}

template <typename V, typename E, typename R>
__device__ __forceinline__ void flush_window(push_args<V, E, R> const& sa, unsigned long long* acc, int64_t win)
{
  __syncthreads();
  unsigned long long* g = sa.acc + win * kWin;
  for (int i = threadIdx.x; i < kWin; i += kPushThreads) {
    unsigned long long v = acc[i];
    if (v) {
      atomicAdd(g + i, v);
      acc[i] = 0ull;
    }
  }
  __syncthreads();
}

// 16-byte vectors for the streamed arrays (4 B-per-lane loads cap near 3.8 TB/s)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <typename R>
__device__ __forceinline__ void load4(R const* p, R* out, bool nt)
{
  if constexpr (sizeof(R) == 4) {
    f32x4 v = nt ? __builtin_nontemporal_load(reinterpret_cast<f32x4 const*>(p)) : *reinterpret_cast<f32x4 const*>(p);
    out[0] = v.x, out[1] = v.y, out[2] = v.z, out[3] = v.w;
  } else {
    f64x2 a = nt ? __builtin_nontemporal_load(reinterpret_cast<f64x2 const*>(p)) : *reinterpret_cast<f64x2 const*>(p);
    f64x2 b = nt ? __builtin_nontemporal_load(reinterpret_cast<f64x2 const*>(p) + 1)
                 : *(reinterpret_cast<f64x2 const*>(p) + 1);
    out[0] = a.x, out[1] = a.y, out[2] = b.x, out[3] = b.y;
  }
}

template <typename R>
__device__ __forceinline__ void store4(R* p, R const* v)
{
  if constexpr (sizeof(R) == 4) {
    *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
  } else {
    reinterpret_cast<f64x2*>(p)[0] = f64x2{v[0], v[1]};
    reinterpret_cast<f64x2*>(p)[1] = f64x2{v[2], v[3]};
  }
}

// A unit lies inside one kPushUnit-aligned block of entries.  Inside a block the
// entries are stored permuted (k_push_pack: phys = (j / 4) * kPushUnit/2 + 4t + j % 4
// for logical entry j * kPushThreads + t) so that thread t loads its 8 entries as two
// 16-byte quads while every gather instruction still covers kPushThreads consecutive
// logical entries (same-source entries coalesce into few cache lines).
template <typename V, typename E, typename R, bool WEIGHTED>
__global__ __launch_bounds__(kPushThreads) void k_pr_push(push_args<V, E, R> sa)
{
  __shared__ unsigned long long acc[kWin];
  auto const& a = sa.a;
  if (a.st->done || (sa.ablate & 4)) return;
  int const tid = threadIdx.x;
  for (int i = tid; i < kWin; i += kPushThreads) acc[i] = 0ull;
  int64_t const nb = gridDim.x;
  int64_t const lb = nb % 8 == 0 ? (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8 : blockIdx.x;
  int64_t const u0 = lb * sa.nunits / nb;
  int64_t const u1 = (lb + 1) * sa.nunits / nb;
  int64_t cur      = u0 < u1 ? sa.units[u0].win : -1;
  __syncthreads();
  uint32_t ent[8];
  R w[8];
  push_unit pu{};
  auto load_unit = [&](int64_t un, push_unit& p, uint32_t* e, R* ww) {
    p = sa.units[un];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int64_t k = p.k0 + j * kPushThreads + tid;
      e[j]      = k < p.k1 ? nt_load(sa.ent + k) : 0u;
      if constexpr (WEIGHTED) ww[j] = k < p.k1 ? nt_load(sa.ew + k) : R(0);
    }
  };
  if (u0 < u1) load_unit(u0, pu, ent, w);
  for (int64_t un = u0; un < u1; ++un) {
    uint32_t ent_n[8];
    R w_n[8];
    push_unit pu_n{};
    if (un + 1 < u1) load_unit(un + 1, pu_n, ent_n, w_n);
    if (pu.win != cur) {
      flush_window<V, E, R>(sa, acc, cur);
      cur = pu.win;
    }
    R x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bool const ok = pu.k0 + j * kPushThreads + tid < pu.k1;
      if (sa.ablate & 1) x[j] = ok ? R(1e-9) : R(0);
      else x[j] = ok ? a.x_in[pu.base + (int64_t)(ent[j] >> kWinBits)] : R(0);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (x[j] != R(0) && !(sa.ablate & 2)) {
        double v = (double)x[j];
        if constexpr (WEIGHTED) v *= (double)w[j];
        atomicAdd(&acc[ent[j] & (kWin - 1)], to_fixed(v));
      }
    }
    pu = pu_n;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ent[j] = ent_n[j];
      if constexpr (WEIGHTED) w[j] = w_n[j];
    }
  }
  if (cur >= 0) flush_window<V, E, R>(sa, acc, cur);
}

template <typename V, typename E, typename R>
__global__ __launch_bounds__(256) void k_pr_apply(push_args<V, E, R> sa)
{
  auto const& a = sa.a;
  if (a.st->done) return;
  double const base = a.st->base;
  double const pf   = a.st->pers_factor;
  double my_diff = 0, my_dang = 0;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < a.nv; v += (int64_t)gridDim.x * blockDim.x) {
    unsigned long long f = sa.acc[v];
    if (f) sa.acc[v] = 0ull;
    vertex_update<V, E, R>(a, (V)v, (double)(long long)f * kFixScaleInv, base, pf, my_diff, my_dang);
  }
  finish_iteration<V, E, R>(a, my_diff, my_dang, true);
}

// ---- push schedule construction (once per graph, cached on the pull adjacency)
template <typename E>
__global__ void k_edge_rows(E const* off, int64_t nv, int64_t ne, uint32_t* rows)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nv - 1;  // last row with off[row] <= e
    while (lo < hi) {
      int64_t mid = (lo + hi + 1) >> 1;
      if ((int64_t)off[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    rows[e] = (uint32_t)lo;
  }
}

template <typename V>
__global__ void k_push_keys(V const* idx, uint32_t const* rows, int64_t ne, uint64_t* keys, uint32_t* vals)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    keys[e] = ((uint64_t)(rows[e] >> kWinBits) << 32) | (uint64_t)(uint32_t)idx[e];
    vals[e] = (uint32_t)e;
  }
}

// unit starts: a new segment (window, source block) or every kPushUnit-th entry
__global__ void k_unit_flags(uint64_t const* keys, int64_t ne, uint32_t* flag)
{
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < ne; k += (int64_t)gridDim.x * blockDim.x) {
    bool head = k == 0 || (k % kPushUnit) == 0 || (keys[k] >> kSrcBits) != (keys[k - 1] >> kSrcBits);
    flag[k]   = head ? 1u : 0u;
  }
}

template <typename R>
__global__ void k_push_pack(uint64_t const* keys, uint32_t const* vals, uint32_t const* rows, R const* w,
                            uint32_t const* flag, uint32_t const* uid, int64_t ne, uint32_t* ent, R* ew,
                            push_unit* units)
{
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < ne; k += (int64_t)gridDim.x * blockDim.x) {
    uint64_t key = keys[k];
    uint32_t e   = vals[k];
    uint32_t src = (uint32_t)key;
    int64_t ph   = k;
    ent[ph]      = ((src & ((1u << kSrcBits) - 1)) << kWinBits) | (rows[e] & (kWin - 1));
    if (w) ew[ph] = w[e];
    if (flag[k]) units[uid[k]] = push_unit{k, 0, (int64_t)(src >> kSrcBits) << kSrcBits, (int64_t)(key >> 32)};
  }
}

__global__ void k_unit_ends(push_unit* units, int64_t nunits, int64_t ne)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nunits; i += (int64_t)gridDim.x * blockDim.x)
    units[i].k1 = i + 1 < nunits ? units[i + 1].k0 : ne;
}

template <typename V, typename E, typename R>
void build_pr_push_schedule(handle_t& h, graph_t& g, adjacency_t& adj)
{
  hipStream_t s = h.stream;
  int64_t nv    = g.num_vertices;
  int64_t ne    = g.num_edges;
  adj.pr_valid  = true;
  adj.pr_push_ok = (uint64_t)nv < (1ull << 32) && (uint64_t)ne < (1ull << 32);
  if (!adj.pr_push_ok) return;
  int64_t nwin = (nv + kWin - 1) / kWin;
  adj.pr_acc.set_stream(s);
  adj.pr_acc.resize(std::max<int64_t>(nwin * kWin, 1) * sizeof(unsigned long long));
  HIP_CHECK(hipMemsetAsync(adj.pr_acc.data(), 0, std::max<int64_t>(nwin * kWin, 1) * sizeof(unsigned long long), s));
  adj.pr_nunits = 0;
  if (ne == 0) return;
  E const* off = adj.offsets.data<E>();
  V const* idx = adj.indices.data<V>();
  dbuf<uint32_t> rows(ne, s);
  hipLaunchKernelGGL(k_edge_rows<E>, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, off, nv, ne, rows.data());
  CGX_LAUNCH_CHECK();
  dbuf<uint64_t> keys_out(ne, s);
  dbuf<uint32_t> vals_out(ne, s);
  {
    dbuf<uint64_t> keys(ne, s);
    dbuf<uint32_t> vals(ne, s);
    hipLaunchKernelGGL(k_push_keys<V>, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, idx, rows.data(), ne,
                       keys.data(), vals.data());
    CGX_LAUNCH_CHECK();
    radix_sort_pairs<uint64_t, uint32_t>(keys.data(), keys_out.data(), vals.data(), vals_out.data(), (size_t)ne, 0,
                                         32 + bits_for((unsigned long long)(nwin - 1)), s);
  }
  dbuf<uint32_t> flag(ne + 1, s), uid(ne + 1, s);
  hipLaunchKernelGGL(k_unit_flags, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, keys_out.data(), ne,
                     flag.data());
  CGX_LAUNCH_CHECK();
  fill<uint32_t>(flag.data() + ne, 1, 0u, s);
  exclusive_scan<uint32_t, uint32_t>(flag.data(), uid.data(), ne + 1, s);
  int64_t nunits = (int64_t)to_host(uid.data() + ne, 1, s)[0];
  adj.pr_ent.set_stream(s);
  int64_t const ne_pad = (ne + kPushUnit - 1) / kPushUnit * kPushUnit;  // whole aligned quads
  adj.pr_ent.resize(ne_pad * sizeof(uint32_t));
  adj.pr_ew.set_stream(s);
  if (g.weighted) adj.pr_ew.resize(ne_pad * sizeof(R));
  else adj.pr_ew.release();
  adj.pr_units.set_stream(s);
  adj.pr_units.resize(std::max<int64_t>(nunits, 1) * sizeof(push_unit));
  hipLaunchKernelGGL(k_push_pack<R>, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, keys_out.data(),
                     vals_out.data(), rows.data(), g.weighted ? adj.weights.data<R>() : nullptr, flag.data(),
                     uid.data(), ne, adj.pr_ent.data<uint32_t>(), g.weighted ? adj.pr_ew.data<R>() : nullptr,
                     adj.pr_units.data<push_unit>());
  CGX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_unit_ends, dim3(grid_for(nunits, kBlock, 4096)), dim3(kBlock), 0, s,
                     adj.pr_units.data<push_unit>(), nunits, ne);
  CGX_LAUNCH_CHECK();
  adj.pr_nunits = nunits;
  HIP_CHECK(hipStreamSynchronize(s));
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

  // windowed push (our own out-weight sums keep every fixed-point sum <= 1; user
  // precomputed out-weights may not: generic pull kernel then)
  bool push = pow_v == nullptr;
  if (push && !adj.pr_valid) build_pr_push_schedule<V, E, R>(h, g, adj);
  push = push && adj.pr_push_ok;
  push_args<V, E, R> sa{};
  int nblk_push = 0, nblk_apply = 0;
  auto pkernel = g.weighted ? k_pr_push<V, E, R, true> : k_pr_push<V, E, R, false>;
  if (push) {
    sa.ent    = adj.pr_ent.data<uint32_t>();
    sa.ew     = g.weighted ? adj.pr_ew.data<R>() : nullptr;
    sa.units  = adj.pr_units.data<push_unit>();
    sa.nunits = adj.pr_nunits;
    sa.acc    = adj.pr_acc.data<unsigned long long>();
    if (char const* ab = std::getenv("CGX_PR_ABLATE")) sa.ablate = std::atoi(ab);
    nblk_push  = (int)std::min<int64_t>(sa.nunits, 256 * 2);  // 64 KB LDS: two blocks per CU
    nblk_apply = (int)grid_for(nv, kBlock, 2048);
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
        if (push) {
          sa.a = a;
          if (nblk_push) hipLaunchKernelGGL(pkernel, dim3(nblk_push), dim3(kPushThreads), 0, s, sa);
          hipLaunchKernelGGL((k_pr_apply<V, E, R>), dim3(nblk_apply), dim3(kBlock), 0, s, sa);
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
