// PageRank power iteration -- the hot path.
//
// Algorithm: cpp/src/link_analysis/pagerank_impl.cuh:48-293 (init :168-183, loop
// :209-292, stop rule :287-290).  The reference runs, per iteration, a copy, a
// dangling transform_reduce (host sync), a divide pass, the 4 segment SpMV
// kernels of prims/per_v_transform_reduce_incoming_outgoing_e.cuh and an L1
// transform_reduce (host sync).  Per iteration here:
//
//   s[v]   = sum_{u in in(v)} x~[u] * w(u,v)
//   pr'[v] = base + alpha*s (+ pers[v]*(alpha*dangling + 1 - alpha))
//   x~'[v] = pr'[v] / outw[v]   (0 for dangling)     -> the next iteration's source
//   diff  += |pr'[v] - pr[v]|,  dangling' += pr'[v] if outw[v] == 0
//
// Main path (windowed push, below): k_pr_push computes s in 64-bit fixed point from
// a source-ordered copy of the edges, k_pr_apply does the per-vertex update.  The
// generic path (k_pr_iter: user-supplied out-weight sums, or ids beyond 32 bits)
// pulls over the degree-binned CSC schedule in one kernel with fp64 sums.
// Both end an iteration with per-block (diff, dangling) partials that the last
// block to arrive (ticket) reduces in block order -- deterministic -- writing the
// next iteration's base, the convergence flag and the iteration count.
//
// The host enqueues iterations in chunks and reads the flag once per chunk; a
// kernel launched after convergence returns immediately, so no per-iteration
// host round trip remains (the reference has two).
//
// Roofline: HBM.  Algorithmic bytes per iteration (the reference's pull
// formulation) = 4E (indices) + 4V (offsets, int32) + 4V (x~ read)
// + 4V (pr' write) + 4V (outw) [+4E weights] = 4E + 16V.
#include "capi.hpp"
#include "comm.hpp"
#include "mg_graph.hpp"
#include "prims.hpp"
#include "schedule.hpp"

#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>

// Stores and atomics are ordered before hand-offs (the iteration state's host words,
// the fused finish's counters) by s_waitcnt vmcnt(0) alone: vmcnt counts stores only on
// the gfx9 family (gfx10+ counts them in vscnt), so the build is gfx9-only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "s_waitcnt vmcnt(0) orders stores on gfx9-family (gfx950) targets only"
#endif

namespace cgx {

struct pr_state {
  double base;         // unvarying part of the current iteration
  double pers_factor;  // alpha*dangling + 1 - alpha (personalised runs)
  double diff;         // L1 difference of the last iteration
  double prev_diff;    // ... and of the one before (host chunk sizing)
  double dangling;     // dangling mass after the last iteration
  unsigned int ticket;
  int iter;
  int done;  // 0 running, 1 converged, 2 max_iterations reached
  unsigned int wticket;       // fused push + apply: windows applied this iteration
  unsigned long long fdiff;   // ... and their (diff, dangling) sums, fixed point (kSumScale)
  unsigned long long fdang;
};

// The L1 difference and the dangling mass of an iteration are summed in 64-bit fixed
// point (scale 2^61; both are at most 2 when the out-weights are the graph's own, so
// the rank mass stays 1): integer adds, so the totals -- and the next iteration's
// base, which depends on the dangling mass -- are the same bits however the vertices
// are split over blocks (the fused push + apply and the separate apply agree).  The
// pull path (user-supplied out-weights, which may understate the graph's and let the
// mass grow past any fixed range) sums in fp64 instead, per block in a fixed tree and
// over the blocks in block order: deterministic too.
constexpr double kSumScale    = 2305843009213693952.0;  // 2^61
constexpr double kSumScaleInv = 1.0 / 2305843009213693952.0;

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
  int64_t nv;         // vertices this process updates
  int64_t nv_global;  // |V| of the graph (teleport base)
  double* partials;  // per-block (diff, dangling) partials (fixed-point words, see kSumScale)
  pr_state* st;
  unsigned long long* mg_sums;  // multi-GPU: this rank's (diff, dangling) fixed-point sums, allreduced (u64,
                                // exact: the totals are SG's bit for bit) before k_mg_finish
  int enc;          // x~ stored as fixed-point words (enc_fixed; single-GPU fp32 packed push only)
  int fp64;         // (diff, dangling) summed in fp64 (the pull path: user out-weights bound no sum)
};

// x~ as the push consumes it: the 64-bit fixed-point value RNE(x * 2^52) of an fp32
// x in [0, 1] written as one 32-bit word, significand M (24 bits) | shift s << 24,
// value = M << s.  x = M * 2^(eb - 150) for the biased exponent eb, so s = eb - 98
// for x >= 2^-29 (exact); smaller x are rounded to nearest-even here, once per
// vertex, and stored with s = 0.  The push then converts with an and, a shift and
// a 64-bit shift instead of the 7-op fp32 sequence per entry (to_fixed_f32), with
// the same bits.
__device__ __forceinline__ uint32_t enc_fixed(float x)
{
  uint32_t const b  = __float_as_uint(x);
  uint32_t const eb = b >> 23;  // x >= 0
  uint32_t const m  = (b & 0x7fffffu) | 0x800000u;
  if (eb >= 98u) return ((eb - 98u) << 24) | m;
  if (eb == 0u) return 0u;  // denormal or zero: below 2^-126, rounds to 0
  uint32_t const k = 98u - eb;
  if (k > 24u) return 0u;  // m / 2^k < 1/2
  uint32_t const q    = m >> k;
  uint32_t const r    = m & ((1u << k) - 1u);
  uint32_t const half = 1u << (k - 1u);
  return q + ((r > half || (r == half && (q & 1u))) ? 1u : 0u);
}

__device__ __forceinline__ unsigned long long dec_fixed(uint32_t w)
{
  return (unsigned long long)(w & 0xffffffu) << (w >> 24);
}

template <typename R>
__device__ __forceinline__ void store_x(R* x, int64_t v, R val, int enc)
{
  if constexpr (std::is_same<R, float>::value) {
    if (enc) {
      reinterpret_cast<uint32_t*>(x)[v] = enc_fixed(val);
      return;
    }
  }
  x[v] = val;
}

// Iterations to enqueue before the host next reads the state.  The L1 difference
// of the power iteration falls geometrically (ratio ~ alpha times the second
// eigenvalue), so the count still needed is predicted from the last two
// differences, plus one for rounding; the first check comes after 8.  Launches
// after convergence return at once, so an overshoot costs an empty launch and an
// undershoot one more host round trip.  Not tied to any one graph.
inline int next_chunk(pr_state const& st, double eps, int max_iter)
{
  int const left = std::max(1, max_iter - st.iter);
  if (st.iter < 2 || !(st.diff > 0.0) || !(st.prev_diff > 0.0) || !(eps > 0.0)) return std::min(8, left);
  double const r = std::min(0.995, std::max(1e-3, st.diff / st.prev_diff));
  double const n = std::ceil(std::log(eps / st.diff) / std::log(r)) + 1.0;
  int const k    = n < 1.0 ? 1 : n > 64.0 ? 64 : (int)n;
  return std::min(k, left);
}

namespace {

__device__ __forceinline__ unsigned long long sum_fix(double x) { return (unsigned long long)__double2ll_rn(x * kSumScale); }
__device__ __forceinline__ void acc_add(unsigned long long& s, double x) { s += sum_fix(x); }
__device__ __forceinline__ void acc_add(double& s, double x) { s += x; }

// sum over an NT-thread block (NT a multiple of 64); result valid in thread 0; sm >= NT / 64 words
template <int NT>
__device__ __forceinline__ unsigned long long block_sum_u64(unsigned long long v, unsigned long long* sm)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  __syncthreads();
  unsigned long long r = 0;
  if (threadIdx.x == 0)
    for (int w = 0; w < NT / 64; ++w) r += sm[w];
  return r;
}

// next iteration's base, convergence flag and iteration count from the global
// L1 difference d and dangling mass g (pagerank_impl.cuh:209-292)
template <typename V, typename E, typename R>
__device__ void update_state(pr_args<V, E, R> const& a, double d, double g, bool count_iter)
{
  pr_state* st    = a.st;
  int it          = st->iter + (count_iter ? 1 : 0);
  st->iter        = it;
  if (count_iter) st->prev_diff = st->diff;
  st->diff        = d;
  st->dangling    = g;
  double pf       = g * a.alpha + (1.0 - a.alpha);
  st->pers_factor = pf;
  st->base        = a.pers ? 0.0 : pf / (double)a.nv_global;
  int done        = 0;
  if (count_iter) {
    if (d < a.eps) done = 1;
    else if (it >= a.max_iter) done = 2;
  }
  st->ticket = 0;
  st->done   = done;
}

// the last-arriving block reduces the per-block (diff, dangling) partials and
// updates the iteration state (cdna_hip_programming.md §6 Guideline 16 ticket form)
template <typename V, typename E, typename R>
__device__ void finish_iteration(pr_args<V, E, R> const& a, unsigned long long my_diff, unsigned long long my_dang,
                                 bool count_iter)
{
  __shared__ unsigned long long sm[8];
  __shared__ int s_last;
  unsigned long long bd = block_sum_u64<256>(my_diff, sm);
  unsigned long long bg = block_sum_u64<256>(my_dang, sm);
  auto* part = reinterpret_cast<unsigned long long*>(a.partials);
  if (threadIdx.x == 0) {
    // write-through (sc1) partials: no agent release (an L2 write-back per block) needed
    __hip_atomic_store(&part[2 * blockIdx.x], bd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&part[2 * blockIdx.x + 1], bg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(&a.st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last     = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last) return;
  unsigned long long d = 0, g = 0;
  for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) {  // sc1 loads: L1 bypassed
    d += __hip_atomic_load(&part[2 * b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g += __hip_atomic_load(&part[2 * b + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  d = block_sum_u64<256>(d, sm);
  g = block_sum_u64<256>(g, sm);
  if (threadIdx.x == 0) {
    if (a.mg_sums) {
      a.mg_sums[0] = d;
      a.mg_sums[1] = g;
      a.st->ticket = 0;
    } else {
      update_state<V, E, R>(a, (double)d * kSumScaleInv, (double)g * kSumScaleInv, count_iter);
    }
  }
}

// the same in fp64 (pull path, pr_args::fp64): 256-thread blocks
template <typename V, typename E, typename R>
__device__ void finish_iteration(pr_args<V, E, R> const& a, double my_diff, double my_dang, bool count_iter)
{
  __shared__ double sm[4];
  __shared__ int s_last;
  double const bd = block_sum_256(my_diff, sm);
  double const bg = block_sum_256(my_dang, sm);
  auto* part = reinterpret_cast<unsigned long long*>(a.partials);
  if (threadIdx.x == 0) {
    __hip_atomic_store(&part[2 * blockIdx.x], (unsigned long long)__double_as_longlong(bd), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&part[2 * blockIdx.x + 1], (unsigned long long)__double_as_longlong(bg), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(&a.st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last     = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last) return;
  double d = 0, g = 0;
  for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
    d += __longlong_as_double((long long)__hip_atomic_load(&part[2 * b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    g += __longlong_as_double(
      (long long)__hip_atomic_load(&part[2 * b + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  d = block_sum_256(d, sm);
  g = block_sum_256(g, sm);
  if (threadIdx.x == 0) update_state<V, E, R>(a, d, g, count_iter);  // (single GPU only)
}

// multi-GPU: the state update from the allreduced (diff, dangling)
template <typename V, typename E, typename R>
__global__ void k_mg_finish(pr_args<V, E, R> a, bool count_iter)
{
  if (threadIdx.x == 0 && blockIdx.x == 0)
    update_state<V, E, R>(a, (double)a.mg_sums[0] * kSumScaleInv, (double)a.mg_sums[1] * kSumScaleInv, count_iter);
}

// init: x~ = pr / outw, dangling mass of the initial vector
template <typename V, typename E, typename R, typename Acc>
__device__ __forceinline__ void init_body(pr_args<V, E, R> const& a)
{
  Acc dang = 0;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < a.nv; v += (int64_t)gridDim.x * blockDim.x) {
    R p  = a.pr[v];
    R ow = a.outw[v];
    if (ow == R(0)) {
      acc_add(dang, (double)p);
      store_x<R>(a.x_out, v, R(0), a.enc);
    } else {
      store_x<R>(a.x_out, v, (R)((double)p / (double)ow), a.enc);
    }
  }
  finish_iteration<V, E, R>(a, Acc(0), dang, false);
}

template <typename V, typename E, typename R>
__global__ __launch_bounds__(256) void k_pr_init(pr_args<V, E, R> a)
{
  if (a.fp64) init_body<V, E, R, double>(a);
  else init_body<V, E, R, unsigned long long>(a);
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

template <typename V, typename E, typename R, typename Acc = unsigned long long>
__device__ __forceinline__ void vertex_update_from(pr_args<V, E, R> const& a, V v, double s, R old, R ow, double base,
                                                   double pf, Acc& my_diff, Acc& my_dang)
{
  double n = base + a.alpha * s;
  if (a.pers) n += pf * (double)a.pers[v];
  R nr     = (R)n;
  a.pr[v]  = nr;
  acc_add(my_diff, fabs((double)nr - (double)old));
  R xv = R(0);
  if (ow == R(0)) acc_add(my_dang, (double)nr);
  else xv = (R)((double)nr / (double)ow);
  store_x<R>(a.x_out, v, xv, a.enc);
}

template <typename V, typename E, typename R, typename Acc = unsigned long long>
__device__ __forceinline__ void vertex_update(pr_args<V, E, R> const& a, V v, double s, double base, double pf,
                                              Acc& my_diff, Acc& my_dang)
{
  vertex_update_from<V, E, R, Acc>(a, v, s, a.pr[v], a.outw[v], base, pf, my_diff, my_dang);
}

template <typename V, typename E, typename R, bool WEIGHTED>
__global__ __launch_bounds__(256) void k_pr_iter(pr_args<V, E, R> a)
{
  __shared__ double sm[4];
  if (a.st->done) return;  // converged in an earlier launch of this chunk
  work_item const it = a.items[blockIdx.x];
  double const base  = a.st->base;
  double const pf    = a.st->pers_factor;
  double my_diff = 0, my_dang = 0;  // fp64 (pr_args::fp64)
  int const tid = threadIdx.x;
  if (it.width == 256) {
    for (int64_t p = it.begin; p < it.end; ++p) {
      V v      = a.order ? a.order[p] : (V)p;
      double s = row_partial_block<V, E, R, WEIGHTED>(a, a.off[v], a.off[v + 1], tid);
      s        = block_sum_256(s, sm);
      if (tid == 0) vertex_update<V, E, R, double>(a, v, s, base, pf, my_diff, my_dang);
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
      if (valid && lane == 0) vertex_update<V, E, R, double>(a, v, s, base, pf, my_diff, my_dang);
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
//  * destinations are cut into windows of 2^WB consecutive ids (2^WB u64
//    accumulators = 32 KB (WB 12) or 64 KB (WB 13) of LDS per block; two blocks per CU);
//  * push entries are the CSC edges sorted by (window, source) and packed in 32
//    bits: (source - unit's first source) << WB | (destination - window base);
//  * a unit is <= kPushUnit entries of one window whose sources span less than
//    2^(32 - WB); an item is a run of units of one window (a whole window, or an
//    equal share of a window larger than ~E / 2048 entries);
//  * (from 2^22 rows; below, items are tiles of <= 8 units in one queue) items
//    are grouped 128 at a time in window order and the groups dealt to 8
//    queues (balanced by entries); block b takes items from queue b % 8 -- blocks
//    b and b + 8 share an XCD -- and then steals from the others.  A block sums
//    an item into the LDS window in source order and flushes it to the global
//    accumulators (integer atomics) once.  The 64 blocks of an XCD so work on
//    neighbouring windows that sweep the sources at about the same pace, and the
//    x~ lines one gathers are in that XCD's L2 for the others: an offline LRU
//    model of the 8 L2s (RMAT-24) gives 12.9M x~ misses per iteration against
//    22.4M for one queue of 8-unit tiles;
//  * sums are 64-bit fixed point (scale fix_scale<R>: 2^52 for fp32, 2^62 for fp64;
//    every destination's sum is at most the total rank mass 1 since x~[u] w(u, v)
//    summed over v is pr[u]).  Integer addition is associative: the result is bitwise
//    deterministic whatever the order of the atomics.  fp32's 2^52 keeps a typical contribution
//    (x~ ~ 2^-27 at RMAT-24) well below 2^32, so the 32K-destination windows can sum
//    in 32-bit LDS words with rare carries (push_body16, WB = 15); the resolution
//    2^-52 is about half an fp32 ulp of the smallest rank, (1 - alpha) / V, at RMAT-26.
//
// Ids descend by degree, so a window of low-degree destinations draws its sources
// mostly from the hubs (few x~ lines); measured alternative: windows dealt runs of
// 64 ids round robin (every window a sample of all degrees, equal sizes, blocks
// sweeping the sources in lockstep) gathered 2.3x the L1->L2 requests and ran
// 1.45x slower on RMAT-24.  The gathers that miss L2 are what this kernel waits
// on: RMAT-24, 4K windows, ~0.09 distinct x~ lines of 128 B per entry.
//
// k_pr_apply then turns the sums into pr'/x~' per vertex (streaming) and resets the
// accumulators.  Per iteration HBM traffic: 4E (entries) [+4E weights] + x~ lines
// + 8V acc read + 8V acc reset + 16V vertex state.
constexpr int kPushThreads = 1024;
constexpr int kPerThread   = 8;  // entries per thread per unit
constexpr int kPushUnit    = kPerThread * kPushThreads;
constexpr int kQueues      = 8;    // XCDs
constexpr int kTileUnits   = 8;    // units per tile below 2^22 rows (RMAT-22: 8: 0.221, 16: 0.222, 32: 0.229 ms/iteration)
constexpr int kGroupItems  = 128;  // items per group dealt to a queue
constexpr int kCtrStride   = 32;   // queue heads 128 B apart
constexpr int kPushBlocks  = 512;  // persistent grid: two 1024-thread blocks per CU, 256 CUs
constexpr int kCommCUs     = 16;   // multi-GPU, overlapped reduce-scatters: CUs the push leaves to RCCL (modelled)
// LDS left beside a 16K-window push block's 128 KB of sums (163,840 B per workgroup on
// gfx950, less the block's other shared words) for the hub x~ (push_body16 HUB)
constexpr int kHubBytes = 32768 - 512;
#ifndef CGX_APPLY_BATCH
#define CGX_APPLY_BATCH 4
#endif
// Fixed-point scale of the push's per-destination sums, by result type.  fp32: 2^52
// on every schedule, so the 32K-window push's 32-bit LDS words (a typical term ~2^-27
// stays far below 2^32) and every other schedule -- MG blocks included -- give the same
// bits; the resolution is half an fp32 ulp of the smallest rank at RMAT-26.  fp64: 2^62
// (every destination's sum <= sum(pr) = 1, below 2 with accepted precomputed
// out-weights), and fp64 never takes 32K windows (build_pr_push_schedule).
template <typename R>
__host__ __device__ constexpr double fix_scale()
{
  return sizeof(R) == 8 ? 4611686018427387904.0 /* 2^62 */ : 4503599627370496.0 /* 2^52 */;
}
template <typename R>
__host__ __device__ constexpr double fix_scale_inv()
{
  return 1.0 / fix_scale<R>();
}

// Window bits: about 500-600 windows measured best -- fewer x~ line visits per
// entry as windows grow, against the load balance of few windows.  14 (16K
// destinations, 128 KB of LDS, one 1024-thread block per CU) from 2^23 destinations
// up (RMAT-24, 542 windows: 0.709 ms/iteration against 0.786 with 13, same box),
// 13 (8K, 64 KB, two blocks per CU) from 2^22, 12 below (RMAT-22, 586 windows:
// 0.181 ms against 0.199 with 13 and 0.219 with 14).  tuning_t::pr_win_bits
// overrides (12, 13 or 14).
// wide: the caller's schedule can take 32K windows (15: single GPU, packed entries --
// the symmetric unweighted build), else 15 falls back to 14.  32K windows from 2^24
// rows: RMAT-26 2.84 vs 2.98 ms/iteration, but RMAT-24 0.70 vs 0.58 (same box,
// gpurun_out/r05q): 21 % fewer L1->L2 requests, yet as many L2 misses (fewer windows
// in flight per XCD share fewer lines) and the carry check's returning LDS adds cost
// 0.085 ms (0.619 without them, wrong sums).
inline int push_win_bits(int64_t n_rows, tuning_t const& tu, bool wide = false)
{
  if (tu.pr_win_bits == 12 || tu.pr_win_bits == 13 || tu.pr_win_bits == 14) return tu.pr_win_bits;
  if (tu.pr_win_bits == 15) return wide ? 15 : 14;
  if (n_rows >= (int64_t(1) << 24)) return wide ? 15 : 14;
  return n_rows >= (int64_t(1) << 23) ? 14 : n_rows >= (int64_t(1) << 22) ? 13 : 12;
}

// Source-band cut of the single-GPU 16K-window push (build_push_from_coo): tuning_t::
// pr_band_cut > 0 sets it, 0 turns bands off, -1 picks by size (off until measured)
inline int64_t push_band_cut(int64_t n, tuning_t const& tu)
{
  if (tu.pr_band_cut >= 0) return tu.pr_band_cut;
  (void)n;
  return 0;
}

// persistent push blocks: two per CU, one per CU for 16K-destination windows
inline int push_blocks(int win_bits) { return win_bits >= 14 ? kPushBlocks / 2 : kPushBlocks; }

// items per push block on average: a window larger than 1.5 x E / (blocks x this) is
// cut into shares.  RMAT-24 ms/iteration with 2 / 4 / 8 / 16: 0.593 / 0.589-0.599 /
// 0.620-0.630 / 0.687 (RMAT-26 4: 2.98, 8: 3.06, 16: 3.23; same box): more shares
// mean more added (not stored) windows, and the balance gained does not pay for them
constexpr int64_t kShareDiv = 4;

struct push_unit {
  int64_t k0, k1;  // entries [k0, k1)
  int64_t base;    // source id of offset 0 (the unit's first source)
  int64_t win;     // window
};

template <typename V, typename E, typename R>
struct push_args {
  pr_args<V, E, R> a;
  uint32_t const* ent;
  R const* ew;  // entry weights (weighted graphs)
  uint16_t const* ent16;     // packed 16-bit entries (unweighted graphs, see push_body16)
  uint32_t const* seg_base;  // packed: running source before every 512-entry wave segment
  push_unit const* units;
  int64_t nunits;
  unsigned long long* acc;  // [n_rows] fixed-point sums, zero between iterations
  uint32_t* carry;          // 32K windows (WB = 15): per destination, 2^32 units of its sum that the
                            // 32-bit LDS words carried out (and high words of large terms); zero
                            // between iterations, read and cleared with the sums; else nullptr
  int64_t const* items;     // first unit of every item, nitems + 1 entries
  int64_t const* queue;     // item ids, queue by queue
  int64_t qoff[kQueues + 1];
  int64_t nitems;
  unsigned int* tile_ctr;   // queue heads, kCtrStride apart, two sets (iteration parity)
  uint8_t const* win_multi; // per window: 1 = summed by several items (k_pr_apply clears
                            // its sums), 0 = stored whole; nullptr: clear every sum
  int keep_acc;             // k_pr_apply leaves the sums (MG: a reduce-scatter overwrites them)
  int win_bits;
  int64_t nwin;
  // fused apply (single GPU): the block that completes a window applies it
  int fuse;
  int parity;                  // queue-head set of this launch (launch index & 1)
  uint32_t* win_left;          // items of each window still to finish this iteration
  uint32_t const* win_items;   // items of each window (win_left's value between iterations)
  int64_t const* empty_wins;   // windows without items: applied by the last window's block
  int64_t nempty;
  int64_t nwin_items;          // windows with items
  // source bands (pr_push_t::bands): item windows are virtual, vw = band * nwin_real + w
  int bands;
  int64_t nwin_real;
  uint32_t* win_pub;           // per real window: items that published their sums this iteration
  int64_t nhub;                // sources whose x~ the 16K-window push stages in LDS (0: none)
  // CGX_PR_TIMELINE (measurement only): per item {launch << 32 | block, item, start, end}
  // in s_memrealtime ticks (100 MHz), tl[0] = records written
  unsigned long long* tl;
  int64_t tl_cap;
  int launch;
  uint32_t* item_ticks;  // calibration launch: every item's duration (s_memrealtime ticks), else nullptr
};

template <typename T>
__device__ __forceinline__ T nt_load(T const* p)
{
  return __builtin_nontemporal_load(p);
}

template <typename R>
__device__ __forceinline__ unsigned long long to_fixed(double v)
{
  return (unsigned long long)__double2ll_rn(v * fix_scale<R>());
}

// The same value, round-to-nearest-even(x * 2^52), for an fp32 x in [0, 1) in fp32
// arithmetic only: the fp64 sequence (cvt, 2 ldexp, rndne, floor, fma, 2 cvt) was
// most of the push's VALU issue time (SQ_ACTIVE_INST_ANY at ~75 % of the waves'
// cycles, RMAT-24).  y = x * 2^20 and its fraction are exact in fp32; the fraction
// times 2^32 is the fixed-point value's low word before rounding, so rint(frac * 2^32)
// rounds exactly where __double2ll_rn does and never reaches 2^32 (24-bit significands).
__device__ __forceinline__ unsigned long long to_fixed_f32(float x)
{
  float const y     = x * 1048576.0f;  // 2^20
  uint32_t const hi = (uint32_t)y;
  float const fr    = y - (float)hi;
  uint32_t const lo = (uint32_t)__builtin_rintf(fr * 4294967296.0f);  // 2^32
  return ((unsigned long long)hi << 32) | lo;
}

template <typename R>
__device__ __forceinline__ unsigned long long fixed_of(R x)
{
  if constexpr (std::is_same<R, float>::value) return to_fixed_f32(x);
  else return to_fixed<R>((double)x);
}

// push_unit::win of an item's first unit carries kWholeItem when the item is all of
// its window's units: that window's sums are then stored, not added, and k_pr_apply
// need not clear them (win_multi)
constexpr int64_t kWholeItem = int64_t(1) << 40;
constexpr int64_t kWinMask   = kWholeItem - 1;

// add the LDS window to the global accumulators (or store it: the item is the
// whole window) and clear it
template <int WB, typename V, typename E, typename R, typename A>
__device__ __forceinline__ void flush_window(push_args<V, E, R> const& sa, A* acc, int64_t win_w)
{
  __syncthreads();
  unsigned long long* g = sa.acc + ((win_w & kWinMask) << WB);
  if (win_w & kWholeItem) {
    for (int i = threadIdx.x; i < (1 << WB); i += kPushThreads) {
      g[i]   = (unsigned long long)acc[i];
      acc[i] = 0;
    }
  } else {
    for (int i = threadIdx.x; i < (1 << WB); i += kPushThreads) {
      unsigned long long v = (unsigned long long)acc[i];
      if (v) {
        atomicAdd(g + i, v);
        acc[i] = 0;
      }
    }
  }
  __syncthreads();
}

// ---- fused apply (single GPU, pagerank_impl): an item's block adds its LDS window to
// the global sums and counts the item off its window; the block that finishes a
// window's last item applies the window (k_pr_apply's per-vertex update) -- from
// LDS when the item is the whole window, so such a window's sums never leave the
// CU.  The diff / dangling sums go to the state in fixed point (order-free), and the
// block of the last window applied (ticket) applies the windows without items,
// updates the iteration state and clears the other parity's queue heads (unused
// since the previous launch ended).  No separate apply launch, and the apply
// overlaps the other blocks' pushes.
//
// No agent-scope fence anywhere: a fence's acquire half (buffer_inv sc1) drops the
// XCD's cached lines -- the x~ lines every other block on the XCD is gathering -- and
// with one per item the iteration took 1.31 instead of 0.71 ms (RMAT-24).  Every
// hand-off here goes through device-scope atomics instead, which are performed at the
// coherence point: a window's partial sums are u64 atomic adds, each thread waits for
// its own (s_waitcnt vmcnt(0)) before the block counts the item off, and the
// finishing block reads and clears the sums with atomic exchanges; the (diff,
// dangling) sums are atomic adds waited for before the ticket, and read back by the
// last block with exchanges.  Nothing else written in the launch is read in it
// (pr / x~' / the queue heads of the other parity are read by the next launch).
__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int WB, typename V, typename E, typename R, typename A>
__device__ __forceinline__ void apply_window(push_args<V, E, R> const& sa, int64_t w, A* lds,
                                             unsigned long long& my_diff, unsigned long long& my_dang)
{
  auto const& a     = sa.a;
  double const base = a.st->base;
  double const pf   = a.st->pers_factor;
  int64_t const v0  = w << WB;
  int const n       = (int)min((int64_t)1 << WB, a.nv - v0);
  // vertices per thread and pass, loads first: 4 for 16K windows (8: the same time, and
  // the kernel spilled); 1 in the 64-VGPR kernels of 4K / 8K windows
  constexpr int kB = WB >= 14 ? 4 : 1;
  for (int i0 = threadIdx.x; i0 < n; i0 += kB * kPushThreads) {
    unsigned long long f[kB];
    R old[kB], ow[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      int const i = i0 + j * kPushThreads;
      if (i < n) {
        if (lds) {
          f[j]   = (unsigned long long)lds[i];
          lds[i] = 0;
        } else {  // read and zero for the next iteration, at the coherence point
          f[j] = __hip_atomic_exchange(sa.acc + v0 + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if constexpr (WB == 15)  // the 32-bit LDS words' carries (push_body16)
          f[j] += (unsigned long long)__hip_atomic_exchange(sa.carry + v0 + i, 0u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT) << 32;
        old[j] = a.pr[v0 + i];
        ow[j]  = a.outw[v0 + i];
      }
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      int const i = i0 + j * kPushThreads;
      if (i < n)
        vertex_update_from<V, E, R>(a, (V)(v0 + i), (double)(long long)f[j] * fix_scale_inv<R>(), old[j], ow[j], base, pf,
                                    my_diff, my_dang);
    }
  }
}

// Source bands: the sums of real window rw are its two virtual windows' -- the own
// item's LDS when it is the whole of its virtual window (lds), else the plane in acc
// at vw << WB: read and cleared (atomic exchange) when several items add into it
// (win_multi), read (device-scope load) when one item stores it every iteration
template <int WB, typename V, typename E, typename R>
__device__ __forceinline__ void apply_window_banded(push_args<V, E, R> const& sa, int64_t rw, unsigned long long* lds,
                                                    int64_t own_vw, unsigned long long& my_diff,
                                                    unsigned long long& my_dang)
{
  auto const& a     = sa.a;
  double const base = a.st->base;
  double const pf   = a.st->pers_factor;
  int64_t const v0  = rw << WB;
  int const n       = (int)min((int64_t)1 << WB, a.nv - v0);
  int64_t const vw0 = rw, vw1 = rw + sa.nwin_real;
  bool const multi0 = sa.win_multi[vw0] != 0, multi1 = sa.win_multi[vw1] != 0;
  unsigned long long* const p0 = sa.acc + (vw0 << WB);
  unsigned long long* const p1 = sa.acc + (vw1 << WB);
  auto plane = [&](unsigned long long* p, bool multi, int i) -> unsigned long long {
    return multi ? __hip_atomic_exchange(p + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                 : __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  constexpr int kB = 2;
  for (int i0 = threadIdx.x; i0 < n; i0 += kB * kPushThreads) {
    unsigned long long f[kB];
    R old[kB], ow[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      int const i = i0 + j * kPushThreads;
      if (i < n) {
        unsigned long long x0, x1;
        if (lds && own_vw == vw0) {
          x0     = lds[i];
          lds[i] = 0ull;
        } else {
          x0 = plane(p0, multi0, i);
        }
        if (lds && own_vw == vw1) {
          x1     = lds[i];
          lds[i] = 0ull;
        } else {
          x1 = plane(p1, multi1, i);
        }
        f[j]   = x0 + x1;
        old[j] = a.pr[v0 + i];
        ow[j]  = a.outw[v0 + i];
      }
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      int const i = i0 + j * kPushThreads;
      if (i < n)
        vertex_update_from<V, E, R>(a, (V)(v0 + i), (double)(long long)f[j] * fix_scale_inv<R>(), old[j], ow[j], base, pf,
                                    my_diff, my_dang);
    }
  }
}

// fused finish of a banded item: count the item off its real window first; an item
// that is not the window's last publishes its sums (stores them when it is the whole
// of its virtual window, else adds them) and then counts itself published; the last
// waits for the others' publications -- blocks already past their counting, so the
// wait always ends -- and applies the window from its LDS and the planes.  The last
// item of a whole virtual window never writes its sums out: with two bands per window
// one 128 KB plane is written and read per window instead of none.
template <int WB, typename V, typename E, typename R>
__device__ __forceinline__ bool banded_finish(push_args<V, E, R> const& sa, unsigned long long* acc, int64_t win_w,
                                              unsigned long long& my_diff, unsigned long long& my_dang)
{
  __shared__ int s_last;
  int const tid     = threadIdx.x;
  int64_t const vw  = win_w & kWinMask;
  bool const whole  = (win_w & kWholeItem) != 0;
  int64_t const rw  = vw >= sa.nwin_real ? vw - sa.nwin_real : vw;
  __syncthreads();  // the item's LDS sums are complete
  if (tid == 0)
    s_last = __hip_atomic_fetch_sub(sa.win_left + rw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u;
  __syncthreads();
  bool const last = s_last != 0;
  if (!last || !whole) {
    unsigned long long* g = sa.acc + (vw << WB);
    if (whole) {
      for (int i = tid; i < (1 << WB); i += kPushThreads) {
        __hip_atomic_store(g + i, acc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc[i] = 0ull;
      }
    } else {
      for (int i = tid; i < (1 << WB); i += kPushThreads) {
        unsigned long long const v = acc[i];
        if (v) {
          __hip_atomic_fetch_add(g + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          acc[i] = 0ull;
        }
      }
    }
    wait_vmem();  // this thread's stores / adds are performed before the item counts as published
    __syncthreads();
    if (!last) {
      if (tid == 0) __hip_atomic_fetch_add(sa.win_pub + rw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  if (tid == 0) {
    uint32_t const need = sa.win_items[rw] - 1u;
    while (__hip_atomic_load(sa.win_pub + rw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need)
      __builtin_amdgcn_s_sleep(2);
    __hip_atomic_store(sa.win_pub + rw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sa.win_left + rw, sa.win_items[rw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  apply_window_banded<WB, V, E, R>(sa, rw, whole ? acc : nullptr, vw, my_diff, my_dang);
  return true;
}

template <int WB, typename V, typename E, typename R, bool BANDS = false, typename A>
__device__ __forceinline__ void fused_finish(push_args<V, E, R> const& sa, A* acc, int64_t win_w)
{
  __shared__ unsigned long long s_red[kPushThreads / 64];
  __shared__ int s_flag;
  int const tid       = threadIdx.x;
  int64_t const w     = win_w & kWinMask;
  bool const whole    = (win_w & kWholeItem) != 0;
  unsigned long long my_diff = 0, my_dang = 0;
  if constexpr (BANDS) {
    if (!banded_finish<WB, V, E, R>(sa, acc, win_w, my_diff, my_dang)) return;
  } else {
  __syncthreads();  // the item's LDS sums are complete
  if (!whole) {
    unsigned long long* g = sa.acc + (w << WB);
    for (int i = tid; i < (1 << WB); i += kPushThreads) {
      unsigned long long const v = (unsigned long long)acc[i];
      if (v) {
        __hip_atomic_fetch_add(g + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc[i] = 0;
      }
    }
    wait_vmem();  // this thread's adds are performed before the item is counted off
    __syncthreads();
    if (tid == 0)
      s_flag = __hip_atomic_fetch_sub(sa.win_left + w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u;
    __syncthreads();
    if (!s_flag) return;
    if (tid == 0)
      __hip_atomic_store(sa.win_left + w, sa.win_items[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  apply_window<WB, V, E, R>(sa, w, whole ? acc : nullptr, my_diff, my_dang);
  }
  unsigned long long const bd = block_sum_u64<kPushThreads>(my_diff, s_red);
  unsigned long long const bg = block_sum_u64<kPushThreads>(my_dang, s_red);
  if (tid == 0) {
    __hip_atomic_fetch_add(&sa.a.st->fdiff, bd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&sa.a.st->fdang, bg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    wait_vmem();
    s_flag = __hip_atomic_fetch_add(&sa.a.st->wticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (unsigned)(sa.nwin_items - 1);
  }
  __syncthreads();
  if (!s_flag) return;  // (a whole window's LDS was cleared by apply_window)
  my_diff = my_dang = 0;
  for (int64_t k = 0; k < sa.nempty; ++k) {
    if constexpr (BANDS) apply_window_banded<WB, V, E, R>(sa, sa.empty_wins[k], nullptr, -1, my_diff, my_dang);
    else apply_window<WB, V, E, R>(sa, sa.empty_wins[k], (A*)nullptr, my_diff, my_dang);
  }
  unsigned long long const ed = block_sum_u64<kPushThreads>(my_diff, s_red);
  unsigned long long const eg = block_sum_u64<kPushThreads>(my_dang, s_red);
  if (tid == 0) {
    unsigned long long const d =
        __hip_atomic_exchange(&sa.a.st->fdiff, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + ed;
    unsigned long long const g =
        __hip_atomic_exchange(&sa.a.st->fdang, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + eg;
    __hip_atomic_store(&sa.a.st->wticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sa.a.mg_sums) {  // multi-GPU (one grid row): the rank's sums, allreduced before k_mg_finish
      sa.a.mg_sums[0] = d;
      sa.a.mg_sums[1] = g;
    } else {
      update_state<V, E, R>(sa.a, (double)d * kSumScaleInv, (double)g * kSumScaleInv, true);
    }
  }
  if (tid < kQueues) sa.tile_ctr[((sa.parity ^ 1) * kQueues + tid) * kCtrStride] = 0u;
  __syncthreads();
}

// the end of an item: fused finish, or the global sums for k_pr_apply.  FUSE: the
// kernel has the fused finish (16K windows only, decided at run time by sa.fuse).  In
// the 64-VGPR kernels of 4K / 8K windows its code costs 140-156 B of scratch per lane:
// measured on RMAT-22, 0.274 against 0.176 ms/iteration unfused (same box)
template <int WB, typename V, typename E, typename R, bool FUSE, bool BANDS = false, typename A>
__device__ __forceinline__ void end_item(push_args<V, E, R> const& sa, A* acc, int64_t win_w)
{
  if constexpr (BANDS) {  // (a banded schedule is always fused)
    fused_finish<WB, V, E, R, true>(sa, acc, win_w);
    return;
  }
  if constexpr (FUSE) {
    if (sa.fuse) {
      fused_finish<WB, V, E, R>(sa, acc, win_w);
      return;
    }
  }
  flush_window<WB, V, E, R>(sa, acc, win_w);
}

// The push: persistent blocks take items from their queue, then from the others.
// The unit body is branch-free (masked lanes load x~[base] and add 0; the next
// unit of the item is always prefetched, the last re-reading itself -- ent and ew
// are padded by a unit), so the only waits are "gathers done" and "prefetch done".
template <int WB, typename V, typename E, typename R, bool WEIGHTED>
__device__ __forceinline__ void push_body(push_args<V, E, R> const& sa)
{
  constexpr int kWin = 1 << WB;
  __shared__ unsigned long long acc[kWin];
  __shared__ int64_t s_item;
  __shared__ unsigned long long s_t0;
  if (sa.a.st->done) return;
  int const tid = threadIdx.x;
  for (int i = tid; i < kWin; i += kPushThreads) acc[i] = 0ull;
  using cunit_t        = __attribute__((address_space(4))) push_unit const;
  cunit_t* const units = (cunit_t*)sa.units;  // read-only here: scalar loads
  R const* const x     = sa.a.x_in;
  int q                = (int)(blockIdx.x % kQueues);
  for (int tries = 0; tries < kQueues;) {
    if (tid == 0) {
      if (sa.item_ticks) s_t0 = __builtin_amdgcn_s_memrealtime();  // (in LDS: no register across the item)
      int64_t const i = (int64_t)atomicAdd(sa.tile_ctr + (sa.parity * kQueues + q) * kCtrStride, 1u);
      s_item          = i < sa.qoff[q + 1] - sa.qoff[q] ? sa.queue[sa.qoff[q] + i] : -1;
    }
    __syncthreads();
    int64_t const it = s_item;
    __syncthreads();  // every thread has read s_item before thread 0 takes the next
    if (it < 0) {  // uniform: this queue is drained, steal from the next
      q = (q + 1) % kQueues;
      ++tries;
      continue;
    }
    int64_t const ua = sa.items[it], ub = sa.items[it + 1];
    int64_t const win = units[ua].win;
    int64_t k0   = units[ua].k0;
    int n        = (int)(units[ua].k1 - k0);
    int64_t base = units[ua].base;
    uint32_t ent[kPerThread];
    R w[kPerThread];
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) {
      ent[j] = nt_load(sa.ent + k0 + j * kPushThreads + tid);
      if constexpr (WEIGHTED) w[j] = nt_load(sa.ew + k0 + j * kPushThreads + tid);
    }
    for (int64_t un = ua; un < ub; ++un) {
      R const* const xb = x + base;
      R xv[kPerThread];
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) {
        bool const ok = j * kPushThreads + tid < n;
        xv[j]         = xb[ok ? (ent[j] >> WB) : 0u];
        xv[j]         = ok ? xv[j] : R(0);
      }
      int64_t const nx  = un + 1 < ub ? un + 1 : un;
      int64_t const k0n = units[nx].k0;
      int const nn      = (int)(units[nx].k1 - k0n);
      int64_t const bsn = units[nx].base;
      uint32_t ent_n[kPerThread];
      R w_n[kPerThread];
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) {
        ent_n[j] = nt_load(sa.ent + k0n + j * kPushThreads + tid);
        if constexpr (WEIGHTED) w_n[j] = nt_load(sa.ew + k0n + j * kPushThreads + tid);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the first use of a gather
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) {
        if constexpr (WEIGHTED) {
          atomicAdd(&acc[ent[j] & (kWin - 1)], to_fixed<R>((double)xv[j] * (double)w[j]));
        } else {
          atomicAdd(&acc[ent[j] & (kWin - 1)], fixed_of(xv[j]));
        }
      }
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) {
        ent[j] = ent_n[j];
        if constexpr (WEIGHTED) w[j] = w_n[j];
      }
      n    = nn;
      base = bsn;
    }
    end_item<WB, V, E, R, (WB >= 14)>(sa, acc, win);
    // (the item id from LDS too: s_item holds it until thread 0 takes the next)
    if (sa.item_ticks && tid == 0) sa.item_ticks[s_item] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - s_t0);
  }
}

// Two 1024-thread blocks per CU need <= 64 VGPRs (8 waves per SIMD): the bound
// takes the unweighted kernels from 62-65 to 47-54 VGPRs with no spill (at 65 only
// one block fits a CU).  fp64 entry weights would spill 42 VGPRs under it, so that
// instantiation keeps one block per CU.
template <int WB, typename V, typename E, typename R, bool WEIGHTED>
__global__ __launch_bounds__(kPushThreads, 8) void k_pr_push_q(push_args<V, E, R> sa)
{
  push_body<WB, V, E, R, WEIGHTED>(sa);
}

template <int WB, typename V, typename E, typename R, bool WEIGHTED>
__global__ __launch_bounds__(kPushThreads) void k_pr_push_q_wide(push_args<V, E, R> sa)
{
  push_body<WB, V, E, R, WEIGHTED>(sa);
}

// ---- packed 16-bit entries (unweighted graphs)
// In (window, source) order most entries repeat or nearly repeat the previous
// entry's source: RMAT-22 / 4K windows, source delta 0 for 74 % and <= 14 for 96 %
// of the entries (RMAT-24 / 8K windows: <= 6 for 92 %).  An entry is 16 bits:
//   delta << WB | slot                  for delta < 2^(16-WB) - 1, or
//   (2^(16-WB) - 1) << WB | payload      a "jump": source += payload, no edge,
// so a larger gap costs one or more jump entries before an entry of delta 0.  A
// wave's 512 consecutive entries (8 rows of 64) start from seg_base[unit * 16 +
// wave]; a row's sources are an inclusive prefix sum of the deltas (DPP) plus the
// carry, the same dependent-load depth as the 32-bit format (no escape loads).
// Entry bytes per edge ~2.1 instead of 4: the 4E entry stream is the push's floor.
constexpr int kSegEntries = 512;  // entries per wave segment (8 rows of 64 lanes)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// storage index of packed position p: within its 512-entry segment, entry j * 64 + l
// (row j, lane l) sits at l * 8 + j, so lane l reads its 8 rows as one 16-byte word
__host__ __device__ __forceinline__ int64_t seg_store_index(int64_t p)
{
  int64_t const e = p & (kSegEntries - 1);
  return (p & ~(int64_t)(kSegEntries - 1)) | ((e & 63) << 3) | (e >> 6);
}
constexpr int kSegsPerUnit = kPushUnit / kSegEntries;

// inclusive prefix sum over the 64 lanes of a wave (DPP row shifts + row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

// the same scan over N independent rows, step by step across the rows: each DPP
// op's input was written N instructions earlier, so no s_nop hazard padding (the
// row-at-a-time form spent 31 s_nop on 47 DPP adds per unit)
template <int N>
__device__ __forceinline__ void wave_incl_scan_rows(uint32_t (&v)[N])
{
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[j], 0x111, 0xf, 0xf, false);
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[j], 0x112, 0xf, 0xf, false);
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[j], 0x114, 0xf, 0xf, false);
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[j], 0x118, 0xf, 0xf, false);
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[j], 0x142, 0xa, 0xf, false);
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[j], 0x143, 0xc, 0xf, false);
}

// Rows are 64 consecutive entries, so one gather instruction spans a short source
// range.  (Measured: lane-major segments -- a lane's 8 consecutive entries from one
// 16-byte load, sources as a running sum plus one wave scan, 6 DPP adds per 8
// entries instead of 48 -- were 20 % slower: each gather then spans the whole
// 512-entry segment, and the gathers' cost follows the distinct lines each touches.)
//
// HUB (16K windows): the x~ of the first sa.nhub sources (the hubs: ids descend by
// degree) are staged in the LDS left beside the window, once per launch, and a wave
// segment whose sources are all hubs reads them there instead of gathering through
// the texture path -- the push's busiest unit (TA 71 %, TD 80 % busy).  Sources are
// sorted within a window, so almost every segment is all-hub or hub-free; a segment
// that straddles the boundary gathers from global memory.
template <int WB, typename V, typename E, typename R, bool ENC, bool HUB = false, bool FUSE = false, bool BANDS = false>
__device__ __forceinline__ void push_body16(push_args<V, E, R> const& sa)
{
  // ENC: x~ holds enc_fixed words (fp32 single-GPU), decoded with dec_fixed.
  using xw_t = typename std::conditional<ENC, uint32_t, R>::type;
  constexpr int kWin        = 1 << WB;
  constexpr uint32_t kJump  = (1u << (16 - WB)) - 1;  // delta code of a jump entry
  constexpr uint32_t kLow   = (1u << WB) - 1;
  constexpr int kRows       = kSegEntries / 64;
  static_assert(kRows == kPerThread, "a wave segment is one unit row per thread");
  // 32K-destination windows (WB = 15) sum in 32-bit LDS words: 128 KB like the 16K
  // windows' 64-bit words, so the 16K-source hub table still fits beside them
  constexpr bool kAcc32 = WB == 15;
  using acc_t           = typename std::conditional<kAcc32, uint32_t, unsigned long long>::type;
  __shared__ acc_t acc[kWin];
  constexpr int kHub = HUB ? kHubBytes / (int)sizeof(xw_t) : 1;
  __shared__ xw_t hub[kHub];
  __shared__ int64_t s_item;
  __shared__ unsigned long long s_t0;
  if (sa.a.st->done) return;
  int const tid  = threadIdx.x;
  int const lane = tid & 63;
  int const wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < kWin; i += kPushThreads) acc[i] = 0;
  using cunit_t        = __attribute__((address_space(4))) push_unit const;
  cunit_t* const units = (cunit_t*)sa.units;
  xw_t const* const x  = reinterpret_cast<xw_t const*>(sa.a.x_in);
  uint32_t const nh    = HUB ? (uint32_t)min((int64_t)kHub, sa.nhub) : 0u;
  if constexpr (HUB)
    for (uint32_t i = tid; i < nh; i += kPushThreads) hub[i] = x[i];  // (the first item's barrier publishes it)
  int q                = (int)(blockIdx.x % kQueues);
  for (int tries = 0; tries < kQueues;) {
    if (tid == 0) {
      // item start time in LDS: a 64-bit register live across the item made the
      // 16K-window kernel spill (127 VGPRs + 12 B scratch)
      if (sa.tl || sa.item_ticks) s_t0 = __builtin_amdgcn_s_memrealtime();
      int64_t const i = (int64_t)atomicAdd(sa.tile_ctr + (sa.parity * kQueues + q) * kCtrStride, 1u);
      s_item          = i < sa.qoff[q + 1] - sa.qoff[q] ? sa.queue[sa.qoff[q] + i] : -1;
    }
    __syncthreads();
    int64_t const it = s_item;
    __syncthreads();
    if (it < 0) {
      q = (q + 1) % kQueues;
      ++tries;
      continue;
    }
    int64_t const ua = sa.items[it], ub = sa.items[it + 1];
    int64_t const win = units[ua].win;
    // A wave's 512-entry segment is stored lane-interleaved (seg_store_index): lane l
    // holds its 8 rows' entries (row j = entry j * 64 + l) in one 16-byte word, so
    // a segment is one dwordx4 load per lane and two more units' segments can be in
    // flight while this one is summed (3 x 4 VGPRs; the row-major layout needed 8
    // VGPRs per unit).  Measured: the entry stream was the push's largest stall
    // (RMAT-24: 0.794 -> 0.464 ms/iteration with the entries served from L2).
    auto seg_ptr = [&](int64_t u) {
      return reinterpret_cast<u32x4_t const*>(sa.ent16 + units[u].k0 + wave * kSegEntries) + lane;
    };
    // entries of this wave's segment: a multiple of kSegEntries (windows are padded
    // to whole segments), <= 0 for the waves past the end of a window's last unit
    auto seg_n = [&](int64_t u) { return (int)(units[u].k1 - units[u].k0) - wave * kSegEntries; };
    auto entry = [&](u32x4_t const& w, int j) { return (w[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu; };
    // decode a segment's sources (DPP scan of the deltas + the running base) and
    // issue its 8 gathers; jumps and padding read a valid source and add nothing to LDS
    // (an exec-masked add instead of adding 0: RMAT-24 0.577-0.595 vs 0.596-0.599
    // ms/iteration, same box).  Masking their gathers too was slower (RMAT-24 0.640,
    // RMAT-26 3.09 vs 3.00 ms): the mask costs registers and exec switches in the loop
    auto gather = [&](u32x4_t const& w, uint32_t base, xw_t (&xv)[kRows]) {
      uint32_t sc[kRows];
#pragma unroll
      for (int j = 0; j < kRows; ++j) {
        uint32_t const e = entry(w, j);
        sc[j]            = (e >> WB) == kJump ? (e & kLow) : (e >> WB);
      }
      wave_incl_scan_rows<kRows>(sc);
      uint32_t run = base;
      if constexpr (HUB) {
        uint32_t src[kRows];
#pragma unroll
        for (int j = 0; j < kRows; ++j) {
          src[j] = run + sc[j];
          run += (uint32_t)__builtin_amdgcn_readlane((int)sc[j], 63);
        }
        if (run < nh) {  // wave-uniform: the segment's last source (lane 63 of row 7) is a hub
#pragma unroll
          for (int j = 0; j < kRows; ++j) xv[j] = hub[src[j]];
        } else {
#pragma unroll
          for (int j = 0; j < kRows; ++j) xv[j] = x[src[j]];
        }
        return;
      }
#pragma unroll
      for (int j = 0; j < kRows; ++j) {
        uint32_t const src = run + sc[j];
        run += (uint32_t)__builtin_amdgcn_readlane((int)sc[j], 63);
        xv[j] = x[src];
      }
    };
    auto sum = [&](u32x4_t const& w, xw_t const (&xv)[kRows]) {
      if constexpr (kAcc32) {
        // A term's low word goes into the 32-bit LDS sum; the old value the add returns
        // says whether it carried out, and a carry (or a term of 2^32 or more: x~ above
        // 2^-20) is counted in the destination's global carry word -- rare (about
        // sum / 2^32 per destination and iteration), and integer like the rest, so the
        // sums stay exact and order-free.  All 8 adds are issued before the first
        // return is waited for.
        uint32_t lo[kRows], old[kRows];
        uint32_t* const cw = sa.carry + ((win & kWinMask) << WB);
#pragma unroll
        for (int j = 0; j < kRows; ++j) {
          uint32_t const e = entry(w, j);
          unsigned long long fix;
          if constexpr (ENC) fix = dec_fixed(xv[j]);
          else fix = fixed_of(xv[j]);
          lo[j] = (e >> WB) != kJump ? (uint32_t)fix : 0u;
          if ((e >> WB) != kJump) {
            old[j] = atomicAdd(&acc[e & kLow], lo[j]);
            if (fix >> 32) atomicAdd(cw + (e & kLow), (uint32_t)(fix >> 32));
          }
        }
#pragma unroll
        for (int j = 0; j < kRows; ++j) {
          uint32_t const e = entry(w, j);
          if ((e >> WB) != kJump && old[j] > ~lo[j]) atomicAdd(cw + (e & kLow), 1u);
        }
      } else {
#pragma unroll
        for (int j = 0; j < kRows; ++j) {
          uint32_t const e = entry(w, j);
          xw_t const v     = xv[j];
          unsigned long long fix;
          if constexpr (ENC) fix = dec_fixed(v);
          else fix = fixed_of(v);
          if ((e >> WB) != kJump) atomicAdd(&acc[e & kLow], fix);
        }
      }
    };
    // Software pipeline: the next unit's gathers are issued before this unit is
    // summed into LDS, so two units' gathers are in flight per wave (the push waits
    // on its gathers: SQ_WAIT_ANY 52 % of the wave cycles, issue 9 %), and the entries
    // of the unit after that are prefetched.
    int64_t const u1 = ua + 1 < ub ? ua + 1 : ua;
    int nA      = seg_n(ua);
    int nB      = seg_n(u1);
    uint32_t bB = __builtin_amdgcn_readfirstlane(sa.seg_base[u1 * kSegsPerUnit + wave]);
    u32x4_t wA  = nt_load(seg_ptr(ua));  // padded: the stream has a unit past its end
    u32x4_t wB  = nt_load(seg_ptr(u1));
    xw_t xA[kRows];
    if (nA > 0) gather(wA, __builtin_amdgcn_readfirstlane(sa.seg_base[ua * kSegsPerUnit + wave]), xA);
    for (int64_t un = ua; un < ub; ++un) {
      bool const actB = un + 1 < ub && nB > 0;  // wave-uniform
      xw_t xB[kRows];
      if (actB) gather(wB, bB, xB);
      int64_t const u2  = un + 2 < ub ? un + 2 : un;
      int const n2      = seg_n(u2);
      uint32_t const b2 = sa.seg_base[u2 * kSegsPerUnit + wave];
      u32x4_t const e2  = nt_load(seg_ptr(u2));
      __builtin_amdgcn_sched_barrier(0);  // keep the next gathers and the prefetch ahead of the sums
      if (nA > 0) sum(wA, xA);
      wA = wB;
#pragma unroll
      for (int j = 0; j < kRows; ++j) xA[j] = xB[j];
      nA = actB ? nB : 0;
      wB = e2;
      nB = n2;
      bB = __builtin_amdgcn_readfirstlane(b2);
    }
    end_item<WB, V, E, R, FUSE, BANDS>(sa, acc, win);
    // (the item id from LDS too: s_item holds it until thread 0 takes the next)
    if (sa.item_ticks && tid == 0) sa.item_ticks[s_item] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - s_t0);
    if (sa.tl && tid == 0) {
      unsigned long long const t_end = __builtin_amdgcn_s_memrealtime();
      unsigned long long const k     = atomicAdd(sa.tl, 1ull);
      if ((int64_t)k < sa.tl_cap) {
        unsigned long long* r = sa.tl + 1 + 4 * k;
        r[0] = ((unsigned long long)sa.launch << 32) | blockIdx.x;
        int64_t const iu = s_item;
        r[1] = ((unsigned long long)(units[sa.items[iu + 1] - 1].k1 - units[sa.items[iu]].k0) << 32) | (unsigned long long)iu;
        r[2] = s_t0;
        r[3] = t_end;
      }
    }
  }
}

template <int WB, typename V, typename E, typename R, bool ENC>
__global__ __launch_bounds__(kPushThreads, 8) void k_pr_push16(push_args<V, E, R> sa)
{
  // (hub x~ in LDS at 4K windows -- 2 x (32 + 32) KB per CU -- measured no faster on RMAT-22,
  // 0.163-0.167 vs 0.163 ms, and spills 12 B under the 64-VGPR bound)
  push_body16<WB, V, E, R, ENC>(sa);
}

// 16K-destination windows: 128 KB of LDS, one block (16 waves) per CU, no 8-waves bound
// (BANDS: source-banded schedules, a kernel of its own: the banded finish in the same
// kernel took it from 115 VGPRs to 127 and 12 B of scratch)
template <typename V, typename E, typename R, bool ENC, bool BANDS = false>
__global__ __launch_bounds__(kPushThreads) void k_pr_push16_w14(push_args<V, E, R> sa)
{
  push_body16<14, V, E, R, ENC, true, true, BANDS>(sa);
}

// 32K-destination windows in 32-bit LDS words (fewer (window, x~ line) pairs than 16K
// windows: RMAT-22 0.41 -> 0.26 GB of line fills for 1.053E -> 1.115E entries,
// scripts/l2model pairs model); single GPU, packed entries, fused apply
template <typename V, typename E, typename R, bool ENC>
__global__ __launch_bounds__(kPushThreads) void k_pr_push16_w15(push_args<V, E, R> sa)
{
  push_body16<15, V, E, R, ENC, true, true, false>(sa);
}

template <typename V, typename E, typename R, bool WEIGHTED>
__global__ __launch_bounds__(kPushThreads) void k_pr_push_q_w14(push_args<V, E, R> sa)
{
  push_body<14, V, E, R, WEIGHTED>(sa);
}

template <typename V, typename E, typename R>
__global__ __launch_bounds__(256) void k_pr_apply(push_args<V, E, R> sa)
{
  auto const& a = sa.a;
  if (sa.tile_ctr && blockIdx.x == 0 && threadIdx.x < kQueues)
    sa.tile_ctr[(sa.parity * kQueues + threadIdx.x) * kCtrStride] = 0u;  // push done
  if (a.st->done) return;
  double const base = a.st->base;
  double const pf   = a.st->pers_factor;
  unsigned long long my_diff = 0, my_dang = 0;
  int64_t const stride = (int64_t)gridDim.x * blockDim.x;
  int64_t v            = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  // a 32K-window schedule's carries (sa.carry): the sums' high parts, read and cleared here
  auto take_carry = [&](int64_t vv) -> unsigned long long {
    if (!sa.carry) return 0ull;
    uint32_t const c = sa.carry[vv];
    if (c) sa.carry[vv] = 0u;
    return (unsigned long long)c << 32;
  };
  if constexpr (std::is_same<R, float>::value) {
    // fp32: four consecutive vertices per lane through 16-byte loads and stores (pr,
    // outw, x~) and two 16-byte loads of the sums -- a quarter of the memory
    // instructions of the scalar loop; the scalar loop below takes the tail
    typedef float f4_t __attribute__((ext_vector_type(4)));
    typedef unsigned u4_t __attribute__((ext_vector_type(4)));
    typedef unsigned long long u2_t __attribute__((ext_vector_type(2)));
    bool const aligned = ((reinterpret_cast<uintptr_t>(a.pr) | reinterpret_cast<uintptr_t>(a.outw) |
                           reinterpret_cast<uintptr_t>(a.x_out) | reinterpret_cast<uintptr_t>(sa.acc)) & 15) == 0 &&
                         !sa.carry;
    if (aligned) {
      int64_t const nq = a.nv / 4;
      for (int64_t q = v; q < nq; q += stride) {
        u2_t const f01 = reinterpret_cast<u2_t const*>(sa.acc)[2 * q];
        u2_t const f23 = reinterpret_cast<u2_t const*>(sa.acc)[2 * q + 1];
        f4_t const old = reinterpret_cast<f4_t const*>(a.pr)[q];
        f4_t const ow  = reinterpret_cast<f4_t const*>(a.outw)[q];
        unsigned long long const f[4] = {f01.x, f01.y, f23.x, f23.y};
        float const o[4] = {old.x, old.y, old.z, old.w}, w[4] = {ow.x, ow.y, ow.z, ow.w};
        float nr[4], xv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          int64_t const vj = 4 * q + j;
          double n = base + a.alpha * ((double)(long long)f[j] * fix_scale_inv<R>());
          if (a.pers) n += pf * (double)a.pers[vj];
          nr[j] = (float)n;
          acc_add(my_diff, fabs((double)nr[j] - (double)o[j]));
          xv[j] = 0.0f;
          if (w[j] == 0.0f) acc_add(my_dang, (double)nr[j]);
          else xv[j] = (float)((double)nr[j] / (double)w[j]);
          if (!sa.keep_acc && f[j] && (!sa.win_multi || sa.win_multi[vj >> sa.win_bits])) sa.acc[vj] = 0ull;
        }
        reinterpret_cast<f4_t*>(a.pr)[q] = f4_t{nr[0], nr[1], nr[2], nr[3]};
        if (a.enc)
          reinterpret_cast<u4_t*>(a.x_out)[q] = u4_t{enc_fixed(xv[0]), enc_fixed(xv[1]), enc_fixed(xv[2]), enc_fixed(xv[3])};
        else
          reinterpret_cast<f4_t*>(a.x_out)[q] = f4_t{xv[0], xv[1], xv[2], xv[3]};
      }
      v = 4 * nq + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;  // (at most 3 left: the scalar loop)
    }
  }
  // kApplyBatch vertices per thread with all loads issued before the first store
  // (pr and outw may alias as far as the compiler knows, which serialises the plain loop)
  constexpr int kApplyBatch = CGX_APPLY_BATCH;
  for (; v + (kApplyBatch - 1) * stride < a.nv; v += kApplyBatch * stride) {
    unsigned long long f[kApplyBatch];
    R old[kApplyBatch], ow[kApplyBatch];
#pragma unroll
    for (int j = 0; j < kApplyBatch; ++j) {
      f[j]   = sa.acc[v + j * stride];
      old[j] = a.pr[v + j * stride];
      ow[j]  = a.outw[v + j * stride];
    }
#pragma unroll
    for (int j = 0; j < kApplyBatch; ++j) {
      int64_t const vj = v + j * stride;
      if (!sa.keep_acc && f[j] && (!sa.win_multi || sa.win_multi[vj >> sa.win_bits])) sa.acc[vj] = 0ull;
      f[j] += take_carry(vj);
      vertex_update_from<V, E, R>(a, (V)vj, (double)(long long)f[j] * fix_scale_inv<R>(), old[j], ow[j], base, pf, my_diff,
                                  my_dang);
    }
  }
  for (; v < a.nv; v += stride) {
    unsigned long long f = sa.acc[v];
    if (!sa.keep_acc && f && (!sa.win_multi || sa.win_multi[v >> sa.win_bits])) sa.acc[v] = 0ull;
    f += take_carry(v);
    vertex_update<V, E, R>(a, (V)v, (double)(long long)f * fix_scale_inv<R>(), base, pf, my_diff, my_dang);
  }
  finish_iteration<V, E, R>(a, my_diff, my_dang, true);
}

// ---- push schedule construction (once per graph, cached on the pull adjacency)
// the row of every edge.  A block takes 4096 consecutive edges: thread 0 finds the
// rows of the first and the last (binary search over all offsets), the offsets of the
// rows between go to LDS when there are at most 4096 of them, and each edge searches
// only those (one thread per edge searching all V offsets was 5.7 ms of a first
// PageRank call at RMAT-24)
constexpr int kRowsTile = 4096;
template <typename E>
__device__ __forceinline__ int64_t row_of_edge(E const* off, int64_t lo, int64_t hi, int64_t e)
{
  while (lo < hi) {  // last row in [lo, hi] with off[row] <= e
    int64_t const mid = (lo + hi + 1) >> 1;
    if ((int64_t)off[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

template <typename E>
__global__ __launch_bounds__(256) void k_edge_rows(E const* off, int64_t nv, int64_t ne, uint32_t* rows)
{
  __shared__ int64_t s_r[2];
  __shared__ E s_off[kRowsTile + 1];
  for (int64_t e0 = (int64_t)blockIdx.x * kRowsTile; e0 < ne; e0 += (int64_t)gridDim.x * kRowsTile) {
    int64_t const e1 = min(e0 + kRowsTile, ne);
    if (threadIdx.x == 0) {
      s_r[0] = row_of_edge(off, 0, nv - 1, e0);
      s_r[1] = row_of_edge(off, s_r[0], nv - 1, e1 - 1);
    }
    __syncthreads();
    int64_t const r0 = s_r[0], r1 = s_r[1];
    bool const staged = r1 - r0 < kRowsTile;
    if (staged)
      for (int64_t i = threadIdx.x; i <= r1 - r0; i += blockDim.x) s_off[i] = off[r0 + i];
    __syncthreads();
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
      int64_t r;
      if (staged) {
        int64_t lo = 0, hi = r1 - r0;
        while (lo < hi) {
          int64_t const mid = (lo + hi + 1) >> 1;
          if ((int64_t)s_off[mid] <= e) lo = mid;
          else hi = mid - 1;
        }
        r = r0 + lo;
      } else {
        r = row_of_edge(off, r0, r1, e);
      }
      rows[e] = (uint32_t)r;
    }
    __syncthreads();
  }
}

// key = window << 32 | source, value = edge position; with source bands (cut > 0) the
// window is the virtual one, band * nwin_real + window, band = source >= cut
template <typename C>
__global__ void k_push_keys(C const* cols, uint32_t const* rows, int64_t ne, int wb, uint32_t cut, int64_t nwin_real,
                            uint64_t* keys, uint32_t* vals)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const c = (uint32_t)cols[e];
    uint64_t const w = (uint64_t)(rows[e] >> wb) + (cut && c >= cut ? (uint64_t)nwin_real : 0ull);
    keys[e]          = (w << 32) | c;
    vals[e]          = (uint32_t)e;
  }
}

// Key codecs of the schedule sort.  key_w32: window << 32 | source, the edge position
// in a value array beside it (weighted graphs, any input order).  key_p: one word per
// entry, window << shv | source << wb | slot -- the symmetric unweighted build, whose
// keys come out of the out-edge adjacency already in source order (k_push_keys_p): a
// keys-only sort of the window bits moves 8 B per entry and pass instead of 12, and the
// packing reads the slot from the key instead of gathering the destination.
struct key_w32 {
  __device__ __forceinline__ int64_t win(uint64_t k) const { return (int64_t)(k >> 32); }
  __device__ __forceinline__ uint32_t src(uint64_t k) const { return (uint32_t)k; }
};
struct key_p {
  int shv, wb;
  uint64_t smask;
  __device__ __forceinline__ int64_t win(uint64_t k) const { return (int64_t)(k >> shv); }
  __device__ __forceinline__ uint32_t src(uint64_t k) const { return (uint32_t)((k >> wb) & smask); }
  __device__ __forceinline__ uint32_t slot(uint64_t k) const { return (uint32_t)k & ((1u << wb) - 1u); }
};

// first position of every window w in [0, nwin] among the sorted keys
template <typename KC = key_w32>
__global__ void k_win_starts(uint64_t const* keys, int64_t ne, int64_t nwin, int64_t* ws, KC kc = {})
{
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w <= nwin; w += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = ne;
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if (kc.win(keys[mid]) < w) lo = mid + 1;
      else hi = mid;
    }
    ws[w] = lo;
  }
}

// key_p keys of a symmetric graph's out-edges (row = source, index = destination), in
// the adjacency's source order; rows found per 4096-edge tile as k_edge_rows does
template <typename E>
__global__ __launch_bounds__(256) void k_push_keys_p(E const* off, uint32_t const* idx, int64_t nv, int64_t ne,
                                                     int wb, int shv, uint32_t cut, int64_t nwin_real, uint64_t* keys)
{
  __shared__ int64_t s_r[2];
  __shared__ E s_off[kRowsTile + 1];
  uint32_t const low = (1u << wb) - 1u;
  for (int64_t e0 = (int64_t)blockIdx.x * kRowsTile; e0 < ne; e0 += (int64_t)gridDim.x * kRowsTile) {
    int64_t const e1 = min(e0 + kRowsTile, ne);
    if (threadIdx.x == 0) {
      s_r[0] = row_of_edge(off, 0, nv - 1, e0);
      s_r[1] = row_of_edge(off, s_r[0], nv - 1, e1 - 1);
    }
    __syncthreads();
    int64_t const r0 = s_r[0], r1 = s_r[1];
    bool const staged = r1 - r0 < kRowsTile;
    if (staged)
      for (int64_t i = threadIdx.x; i <= r1 - r0; i += blockDim.x) s_off[i] = off[r0 + i];
    __syncthreads();
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
      int64_t r;
      if (staged) {
        int64_t lo = 0, hi = r1 - r0;
        while (lo < hi) {
          int64_t const mid = (lo + hi + 1) >> 1;
          if ((int64_t)s_off[mid] <= e) lo = mid;
          else hi = mid - 1;
        }
        r = r0 + lo;
      } else {
        r = row_of_edge(off, r0, r1, e);
      }
      uint32_t const d = idx[e], src = (uint32_t)r;
      uint64_t const w = (uint64_t)(d >> wb) + (cut && src >= cut ? (uint64_t)nwin_real : 0ull);
      keys[e]          = (w << shv) | ((uint64_t)src << wb) | (d & low);
    }
    __syncthreads();
  }
}

// unit heads: a window's first entry, every entry at a multiple of kPushUnit (so
// whole units start 32 KB-aligned in ent: measured 5 % faster than window-relative
// units on RMAT-22), and -- only inside such a chunk whose sources span 2^sb or
// more -- every change of the aligned 2^sb source block, so an offset from the
// unit's first source fits sb bits
__global__ void k_unit_flags(uint64_t const* keys, int64_t ne, int64_t const* ws, int sb, uint32_t* flag)
{
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < ne; k += (int64_t)gridDim.x * blockDim.x) {
    int64_t const w  = (int64_t)(keys[k] >> 32);
    int64_t const w0 = ws[w], w1 = ws[w + 1];
    bool head        = k == w0 || k % kPushUnit == 0;
    if (!head) {
      int64_t const a   = k / kPushUnit * kPushUnit;
      int64_t const c0  = a > w0 ? a : w0;
      int64_t const c1  = a + kPushUnit < w1 ? a + kPushUnit : w1;
      uint32_t const s0 = (uint32_t)keys[c0], s1 = (uint32_t)keys[c1 - 1];
      head = ((s1 - s0) >> sb) != 0 && ((uint32_t)keys[k] >> sb) != ((uint32_t)keys[k - 1] >> sb);
    }
    flag[k] = head ? 1u : 0u;
  }
}

__global__ void k_unit_heads(uint64_t const* keys, uint32_t const* flag, uint32_t const* uid, int64_t ne,
                             push_unit* units)
{
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < ne; k += (int64_t)gridDim.x * blockDim.x)
    if (flag[k]) units[uid[k]] = push_unit{k, 0, (int64_t)(uint32_t)keys[k], (int64_t)(keys[k] >> 32)};
}

__global__ void k_unit_ends(push_unit* units, int64_t nunits, int64_t ne)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nunits; i += (int64_t)gridDim.x * blockDim.x)
    units[i].k1 = i + 1 < nunits ? units[i + 1].k0 : ne;
}

template <typename R>
__global__ void k_push_pack(uint64_t const* keys, uint32_t const* vals, uint32_t const* rows, R const* w,
                            uint32_t const* flag, uint32_t const* uid, push_unit const* units, int64_t ne, int wb,
                            uint32_t* ent, R* ew)
{
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < ne; k += (int64_t)gridDim.x * blockDim.x) {
    uint32_t const e   = vals[k];
    int64_t const u    = (int64_t)uid[k] + flag[k] - 1;
    uint32_t const off = (uint32_t)((uint32_t)keys[k] - units[u].base);
    ent[k]             = (off << wb) | (rows[e] & ((1u << wb) - 1));
    if (w) ew[k] = w[e];
  }
}

// ---- packed 16-bit schedule construction (push_body16)
// jumps in front of real entry k: its source gap D to the previous entry of the
// window (0 before the window's first) is coded in the entry when D <= dmax,
// else by ceil(D / pmax) jumps and an entry of delta 0
template <typename KC = key_w32>
__global__ void k_jump_counts(uint64_t const* keys, int64_t ne, int64_t const* ws, uint32_t dmax, uint32_t pmax,
                              uint32_t* mj, KC kc = {})
{
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < ne; k += (int64_t)gridDim.x * blockDim.x) {
    int64_t const w     = kc.win(keys[k]);
    uint32_t const prev = k == ws[w] ? 0u : kc.src(keys[k - 1]);
    uint32_t const D    = kc.src(keys[k]) - prev;
    mj[k]               = D > dmax ? (D + pmax - 1) / pmax : 0u;
  }
}

// the same count as a scan input (k_jump_counts without the array: the scan reads the
// keys and writes the prefix in one pass; position ne counts 0)
struct jump_count_p {
  uint64_t const* keys;
  int64_t const* ws;
  int64_t ne;
  key_p kc;
  uint32_t dmax, pmax;
  __device__ __forceinline__ uint32_t operator()(int64_t k) const
  {
    if (k >= ne) return 0u;
    uint64_t const key  = keys[k];
    int64_t const w     = kc.win(key);
    uint32_t const prev = k == ws[w] ? 0u : kc.src(keys[k - 1]);
    uint32_t const D    = kc.src(key) - prev;
    return D > dmax ? (D + pmax - 1) / pmax : 0u;
  }
};

// real entry k at k + cm[k] (cm = inclusive prefix of the jump counts), its jumps
// right before it
__global__ void k_pack16(uint64_t const* keys, uint32_t const* vals, uint32_t const* rows, int64_t ne,
                         int64_t const* ws, uint32_t const* mj, unsigned long long const* cm,
                         unsigned long long const* pb, int wb, uint32_t pmax,
                         uint16_t* ent16)
{
  uint32_t const jump = (1u << (16 - wb)) - 1, low = (1u << wb) - 1;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < ne; k += (int64_t)gridDim.x * blockDim.x) {
    int64_t const w     = (int64_t)(keys[k] >> 32);
    uint32_t const prev = k == ws[w] ? 0u : (uint32_t)keys[k - 1];
    uint32_t const D    = (uint32_t)keys[k] - prev;
    uint32_t const m    = mj[k];
    int64_t const pos   = k + (int64_t)cm[k] + (int64_t)pb[w];
    uint32_t const slot = rows[vals[k]] & low;
    if (m == 0) {
      ent16[seg_store_index(pos)] = (uint16_t)((D << wb) | slot);
    } else {
      for (uint32_t j = 0; j < m; ++j) {
        uint32_t const pay                  = j + 1 < m ? pmax : D - pmax * (m - 1);
        ent16[seg_store_index(pos - m + j)] = (uint16_t)((jump << wb) | pay);
      }
      ent16[seg_store_index(pos)] = (uint16_t)slot;  // delta 0
    }
  }
}

// the same from key_p keys (the slot in the key); cm a 32-bit prefix when the edges
// are below 2^31 (no jump total can wrap it), else 64-bit
template <typename CM>
__global__ void k_pack16_p(uint64_t const* keys, int64_t ne, int64_t const* ws, CM const* cm,
                           unsigned long long const* pb, key_p kc, uint32_t pmax, uint16_t* ent16)
{
  int const wb        = kc.wb;
  uint32_t const jump = (1u << (16 - wb)) - 1;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < ne; k += (int64_t)gridDim.x * blockDim.x) {
    uint64_t const key  = keys[k];
    int64_t const w     = kc.win(key);
    uint32_t const prev = k == ws[w] ? 0u : kc.src(keys[k - 1]);
    uint32_t const D    = kc.src(key) - prev;
    uint32_t const m    = (uint32_t)(cm[k] - cm[k - 1]);  // cm[-1] is the exclusive scan's 0
    int64_t const pos   = k + (int64_t)cm[k] + (int64_t)pb[w];
    uint32_t const slot = kc.slot(key);
    if (m == 0) {
      ent16[seg_store_index(pos)] = (uint16_t)((D << wb) | slot);
    } else {
      for (uint32_t j = 0; j < m; ++j) {
        uint32_t const pay                  = j + 1 < m ? pmax : D - pmax * (m - 1);
        ent16[seg_store_index(pos - m + j)] = (uint16_t)((jump << wb) | pay);
      }
      ent16[seg_store_index(pos)] = (uint16_t)slot;  // delta 0
    }
  }
}

// Every window's packed stream starts at a multiple of kSegEntries and is padded
// with jumps of 0 (no edge) to a multiple of it, so every wave segment of a unit
// is whole and the push needs no per-entry bound check.
// unpadded packed start of window w (w == nwin: total)
template <typename CM>
__device__ __forceinline__ int64_t packed_start(int64_t const* ws, CM const* cm, int64_t w, int64_t nwin, int64_t total)
{
  return w == nwin ? total : ws[w] + (ws[w] > 0 ? (int64_t)cm[ws[w] - 1] : 0);
}
// padding after every window (pad[nwin] = 0)
template <typename CM>
__global__ void k_packed_pads(int64_t const* ws, CM const* cm, int64_t nwin, int64_t total, unsigned long long* pad)
{
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w <= nwin; w += (int64_t)gridDim.x * blockDim.x) {
    int64_t const len = w == nwin ? 0 : packed_start(ws, cm, w + 1, nwin, total) - packed_start(ws, cm, w, nwin, total);
    pad[w]            = (unsigned long long)((kSegEntries - len % kSegEntries) % kSegEntries);
  }
}
// padded window starts (pb = exclusive prefix of the pads; nws[nwin] = padded total)
template <typename CM>
__global__ void k_packed_win_starts(int64_t const* ws, CM const* cm, unsigned long long const* pb, int64_t nwin,
                                    int64_t total, int64_t* nws)
{
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w <= nwin; w += (int64_t)gridDim.x * blockDim.x)
    nws[w] = packed_start(ws, cm, w, nwin, total) + (int64_t)pb[w];
}

// units straight from the padded window starts: window w's units start at nws[w] + j *
// kPushUnit (what the flag marks + scan + heads below give, without a pass over every
// packed position)
__global__ void k_unit_counts(int64_t const* nws, int64_t nwin, uint32_t* cnt)
{
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w <= nwin; w += (int64_t)gridDim.x * blockDim.x)
    cnt[w] = w == nwin ? 0u : (uint32_t)((nws[w + 1] - nws[w] + kPushUnit - 1) / kPushUnit);
}
__global__ void k_units_direct(int64_t const* nws, int64_t nwin, uint32_t const* upos, int64_t nunits,
                               push_unit* units)
{
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < nunits; u += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nwin - 1;  // the last window whose units start at or before u
    while (lo < hi) {
      int64_t const mid = (lo + hi + 1) >> 1;
      if ((int64_t)upos[mid] <= u) lo = mid;
      else hi = mid - 1;
    }
    units[u] = push_unit{nws[lo] + (u - (int64_t)upos[lo]) * kPushUnit, 0, 0, lo};
  }
}

// unit heads: every window start and every kPushUnit entries into a window
__global__ void k_packed_unit_marks(int64_t const* nws, int64_t nwin, uint32_t* flag)
{
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nwin; w += (int64_t)gridDim.x * blockDim.x)
    for (int64_t p = nws[w]; p < nws[w + 1]; p += kPushUnit) flag[p] = 1u;
}
__global__ void k_packed_unit_heads(uint32_t const* flag, uint32_t const* uid, int64_t total, int64_t const* nws,
                                    int64_t nwin, push_unit* units)
{
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    if (!flag[p]) continue;
    int64_t lo = 0, hi = nwin - 1;  // last window with nws[w] <= p
    while (lo < hi) {
      int64_t mid = (lo + hi + 1) >> 1;
      if (nws[mid] <= p) lo = mid;
      else hi = mid - 1;
    }
    units[uid[p]] = push_unit{p, 0, 0, lo};
  }
}

// running source before the first entry of every (unit, wave segment)
template <typename KC, typename CM>
__global__ void k_seg_bases(push_unit const* units, int64_t nunits, uint64_t const* keys, int64_t ne,
                            int64_t const* ws, uint32_t const* mj, CM const* cm, unsigned long long const* pb,
                            uint32_t dmax, uint32_t pmax, uint32_t* seg_base, KC kc)
{
  int64_t const n = nunits * kSegsPerUnit;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    push_unit const u = units[i / kSegsPerUnit];
    int64_t const p   = u.k0 + (i % kSegsPerUnit) * kSegEntries;
    uint32_t base     = 0;
    if (p < u.k1) {  // a segment never starts in a window's padding
      int64_t lo = 0, hi = ne - 1;  // first real entry at a packed position >= p
      while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (mid + (int64_t)cm[mid] + (int64_t)pb[kc.win(keys[mid])] < p) lo = mid + 1;
        else hi = mid;
      }
      int64_t const k     = lo;
      uint32_t const m    = mj ? mj[k] : (uint32_t)(cm[k] - cm[k - 1]);  // no mj: cm[-1] is the scan's 0
      int64_t const w     = kc.win(keys[k]);
      int64_t const j     = p - (k + (int64_t)cm[k] + (int64_t)pb[w] - m);
      uint32_t const prev = k == ws[w] ? 0u : kc.src(keys[k - 1]);
      uint32_t const src  = kc.src(keys[k]);
      uint32_t const D    = src - prev;
      base = j < (int64_t)m ? prev + pmax * (uint32_t)j : src - (m ? 0u : (D <= dmax ? D : 0u));
    }
    seg_base[i] = base;
  }
}

// Whole items (all of a window's units): kWholeItem on the item's first unit (the
// push stores that window's sums), 0 in win_multi (k_pr_apply leaves them)
inline void mark_whole_items(hipStream_t s, pr_push_t& pp, push_unit* units, std::vector<push_unit>& hu,
                             std::vector<int64_t> const& item_u, int64_t nitems, tuning_t const& tu)
{
  int64_t const nunits = (int64_t)hu.size();
  bool const no_whole  = !tu.pr_whole;  // A/B: every flush adds, the apply clears every sum
  std::vector<uint8_t> multi((size_t)std::max<int64_t>(pp.nwin, 1), 0);
  for (int64_t i = 0; i < nitems; ++i) {
    int64_t const u = item_u[i], last = item_u[i + 1] - 1;
    // the flag may already sit on an earlier item's first unit: compare and index
    // by the window bits only
    int64_t const wu = hu[u].win & kWinMask;
    bool const whole = !no_whole && (u == 0 || (hu[u - 1].win & kWinMask) != wu) &&
                       (last + 1 >= nunits || (hu[last + 1].win & kWinMask) != wu);
    CGX_EXPECTS(!(hu[u].win & kWholeItem), CUGRAPH_UNKNOWN_ERROR, "mark_whole_items: unit already flagged");
    if (whole) hu[u].win |= kWholeItem;
    else multi[wu] = 1;
  }
  to_device(units, hu.data(), (size_t)nunits, s);
  // items per window (fused apply)
  {
    // (source bands: the items of a real window over both of its virtual windows)
    int64_t const nreal = pp.bands ? pp.nwin_real : pp.nwin;
    std::vector<uint32_t> cnt((size_t)std::max<int64_t>(nreal, 1), 0u);
    for (int64_t i = 0; i < nitems; ++i) {
      int64_t const wu = hu[item_u[i]].win & kWinMask;
      if (wu < pp.nwin) ++cnt[pp.bands ? wu % nreal : wu];
    }
    std::vector<int64_t> empty;
    pp.nwin_items = 0;
    for (int64_t w = 0; w < nreal; ++w) {
      if (cnt[w]) ++pp.nwin_items;
      else empty.push_back(w);
    }
    if (pp.bands) {
      pp.win_pub.set_stream(s);
      pp.win_pub.resize(cnt.size() * sizeof(uint32_t));
      HIP_CHECK(hipMemsetAsync(pp.win_pub.data(), 0, cnt.size() * sizeof(uint32_t), s));
    }
    pp.nempty = (int64_t)empty.size();
    pp.win_items.set_stream(s);
    pp.win_items.resize(cnt.size() * sizeof(uint32_t));
    to_device(pp.win_items.data<uint32_t>(), cnt.data(), cnt.size(), s);
    pp.win_left.set_stream(s);
    pp.win_left.resize(cnt.size() * sizeof(uint32_t));
    pp.empty_wins.set_stream(s);
    pp.empty_wins.resize(std::max<size_t>(empty.size(), 1) * sizeof(int64_t));
    if (!empty.empty()) to_device(pp.empty_wins.data<int64_t>(), empty.data(), empty.size(), s);
    HIP_CHECK(hipStreamSynchronize(s));
  }
  pp.win_multi.set_stream(s);
  pp.win_multi.resize(multi.size());
  to_device(pp.win_multi.data<uint8_t>(), multi.data(), multi.size(), s);
  HIP_CHECK(hipStreamSynchronize(s));  // the host vectors go out of scope
}

inline void upload_items(hipStream_t s, pr_push_t& pp, std::vector<int64_t> const& item_u,
                         std::vector<int64_t> const& queue, int64_t nitems)
{
  pp.items.set_stream(s);
  pp.items.resize(item_u.size() * sizeof(int64_t));
  to_device(pp.items.data<int64_t>(), item_u.data(), item_u.size(), s);
  pp.queue.set_stream(s);
  pp.queue.resize(std::max<size_t>(queue.size(), 1) * sizeof(int64_t));
  to_device(pp.queue.data<int64_t>(), queue.data(), queue.size(), s);
  pp.nitems = nitems;
}

// Items and queues over the units (host logic, once per graph)
inline void build_items(hipStream_t s, pr_push_t& pp, push_unit* units, int64_t nunits, bool xcd_queues,
                        tuning_t const& tu)
{
  int64_t const ne = nunits ? to_host(&units[nunits - 1].k1, 1, s)[0] : 0;
  // Items and queues.  From 2^22 rows (8K windows): an item is a window's units,
  // or an equal share of a window of more than 1.5 tg entries; groups of
  // kGroupItems consecutive items are dealt to the 8 queues by longest-processing-
  // time on their entries (RMAT-24: 0.986 -> 0.950 ms/iteration, same-box A/B).
  // Below: one queue of tiles of <= 8 units of a window (RMAT-22: the XCD queues
  // measured 0.199 -> 0.216, the last groups' imbalance outweighing the L2 hits).
  auto hu = to_host(units, nunits, s);
  int64_t const div = tu.pr_share_div > 0 ? tu.pr_share_div : kShareDiv;
  int64_t const tg  = std::max<int64_t>(kPushUnit, ne / (push_blocks(pp.win_bits) * div));
  std::vector<int64_t> item_u, item_e;
  for (int64_t u0 = 0; u0 < nunits;) {
    int64_t u1 = u0;
    while (u1 < nunits && hu[u1].win == hu[u0].win) ++u1;
    int64_t const size = hu[u1 - 1].k1 - hu[u0].k0;
    int64_t const n    = std::max<int64_t>(1, (size + tg / 2) / tg);
    int64_t k          = 0;
    for (int64_t u = u0; u < u1; ++u) {
      int64_t const done = hu[u].k0 - hu[u0].k0;
      bool const head    = u == u0 || (xcd_queues ? (k < n && done * n >= k * size) : (u - u0) % kTileUnits == 0);
      if (head) {
        item_u.push_back(u);
        item_e.push_back(0);
        ++k;
      }
      item_e.back() += hu[u].k1 - hu[u].k0;
    }
    u0 = u1;
  }
  int64_t const nitems = (int64_t)item_u.size();
  item_u.push_back(nunits);
  std::vector<int64_t> queue;
  queue.reserve(nitems);
  if (xcd_queues) {
    int64_t const ngroups = (nitems + kGroupItems - 1) / kGroupItems;
    std::vector<int64_t> gsize(ngroups, 0), gorder(ngroups);
    for (int64_t i = 0; i < nitems; ++i) gsize[i / kGroupItems] += item_e[i];
    for (int64_t g = 0; g < ngroups; ++g) gorder[g] = g;
    std::stable_sort(gorder.begin(), gorder.end(), [&](int64_t a, int64_t b) { return gsize[a] > gsize[b]; });
    std::vector<int> gq(ngroups, 0);
    int64_t load[kQueues] = {};
    for (int64_t g : gorder) {
      int best = 0;
      for (int q = 1; q < kQueues; ++q)
        if (load[q] < load[best]) best = q;
      gq[g] = best;
      load[best] += gsize[g];
    }
    for (int q = 0; q < kQueues; ++q) {
      pp.qoff[q] = (int64_t)queue.size();
      for (int64_t i = 0; i < nitems; ++i)
        if (gq[i / kGroupItems] == q) queue.push_back(i);
    }
  } else {  // everything in queue 0; the other labels' blocks steal from it at once
    for (int64_t i = 0; i < nitems; ++i) queue.push_back(i);
    pp.qoff[0] = 0;
    for (int q = 1; q < kQueues; ++q) pp.qoff[q] = nitems;
  }
  pp.qoff[kQueues] = (int64_t)queue.size();
  mark_whole_items(s, pp, units, hu, item_u, nitems, tu);
  upload_items(s, pp, item_u, queue, nitems);
}

// Measured-cost queues.  An item's entries do not predict its time well: on RMAT-24
// the items of the middle windows (low-degree destinations drawing sources from the
// whole id range) take up to 2.3x the median for the same entries, and with the
// groups dealt by entries the last items ended up to 140 us after most blocks had
// run out of work (per-item timeline, CGX_PR_TIMELINE: blocks busy 83.5 % of a
// launch).  So the first launch on a schedule records every item's duration
// (item_ticks) and the host re-deals the items by those costs: groups of kCalGroup
// consecutive items (neighbouring windows keep sharing x~ lines in their XCD's L2)
// dealt longest-first to the least-loaded queue, each queue taking its groups
// costliest-first, so what is left for the last blocks is short.  Queue order does
// not change any sum (fixed-point adds), only who takes an item when.
// tuning_t::pr_calib = 0 keeps the entry-dealt queues; pr_deal_global puts every item
// in one queue, longest-first (A/B).
constexpr int kCalGroup = 16;

inline bool calibration_wanted(pr_push_t const& pp, tuning_t const& tu)
{
  return pp.calib == 0 && pp.nitems > 0 && tu.pr_calib;
}

inline void calibrate_queues(hipStream_t s, pr_push_t& pp, tuning_t const& tu)
{
  int64_t const n = pp.nitems;
  auto t          = to_host(pp.item_ticks.data<uint32_t>(), n, s);
  std::vector<int64_t> queue;
  queue.reserve(n);
  // below 2^22 rows the items are tiles of <= 8 units in one queue (build_items): that
  // queue, longest-first
  if (tu.pr_deal_global || pp.win_bits < 13) {
    for (int64_t i = 0; i < n; ++i) queue.push_back(i);
    std::stable_sort(queue.begin(), queue.end(), [&](int64_t a, int64_t b) { return t[a] > t[b]; });
    pp.qoff.assign(kQueues + 1, n);
    pp.qoff[0] = 0;
  } else {
    int64_t const G  = kCalGroup;
    int64_t const ng = (n + G - 1) / G;
    std::vector<uint64_t> gc(ng, 0);
    for (int64_t i = 0; i < n; ++i) gc[i / G] += t[i];
    std::vector<int64_t> go(ng);
    for (int64_t g = 0; g < ng; ++g) go[g] = g;
    std::stable_sort(go.begin(), go.end(), [&](int64_t a, int64_t b) { return gc[a] > gc[b]; });
    std::vector<std::vector<int64_t>> qg(kQueues);
    uint64_t load[kQueues] = {};
    for (int64_t g : go) {  // costliest group first, to the least-loaded queue: each queue's list is costliest-first
      int best = 0;
      for (int q = 1; q < kQueues; ++q)
        if (load[q] < load[best]) best = q;
      qg[best].push_back(g);
      load[best] += gc[g];
    }
    if (pp.bands) {  // source bands: each queue takes its band-0 groups first (items are band-major)
      std::vector<int> gband(ng, 0);
      {
        auto hu = to_host(pp.units.data<push_unit>(), (size_t)pp.nunits, s);
        auto iu = to_host(pp.items.data<int64_t>(), (size_t)n, s);
        for (int64_t g = 0; g < ng; ++g) gband[g] = (hu[iu[g * G]].win & kWinMask) >= pp.nwin_real ? 1 : 0;
      }
      for (auto& l : qg) std::stable_sort(l.begin(), l.end(), [&](int64_t a, int64_t b) { return gband[a] < gband[b]; });
    }
    pp.qoff.assign(kQueues + 1, 0);
    for (int q = 0; q < kQueues; ++q) {
      pp.qoff[q] = (int64_t)queue.size();
      for (int64_t g : qg[q])
        for (int64_t i = g * G; i < std::min(n, (g + 1) * G); ++i) queue.push_back(i);
    }
    pp.qoff[kQueues] = n;
  }
  to_device(pp.queue.data<int64_t>(), queue.data(), queue.size(), s);  // same size: in place, stream-ordered
  HIP_CHECK(hipStreamSynchronize(s));
  pp.calib = 2;
}

// Push schedule of an edge list given as (row = destination, col = source) with
// destinations in [0, n_rows) and sources in [0, n_cols) -- the SG pull adjacency
// or one MG 2D block.  col_sorted: the list is in (source, destination) order (the
// out-edge adjacency of a symmetric graph), so a stable sort on the window bits alone
// gives the (window, source, destination) order the full key sort gives -- 2 radix
// passes over the edges instead of 6 (RMAT-24: the first call's largest step)
//
// band_cut > 0 (16K-window packed pushes only): source bands -- each window's entries
// split at the source cut into two virtual windows, vw = band * nwin_real + window, so
// the stream, the items and the queues run every window's low-source entries first
// and the whole grid gathers one band of x~ at a time (push_body16 BANDS)
//
// wide: 32K windows from 2^24 rows as the symmetric builder takes them (packed
// entries only; their carries are folded by the fused apply or k_pr_apply, so a
// caller whose sums leave through a collective -- MG with several grid rows -- passes
// false)
template <typename C, typename R>
void build_push_from_coo(hipStream_t s, uint32_t const* rows, C const* cols, R const* w, int64_t ne, int64_t n_rows,
                         int64_t n_cols, pr_push_t& pp, tuning_t const& tu, bool col_sorted = false,
                         int64_t band_cut = 0, bool wide = false)
{
  pp.built = true;
  pp.ok    = (uint64_t)n_rows < (1ull << 32) && (uint64_t)n_cols < (1ull << 32) && (uint64_t)ne < (1ull << 32);
  if (!pp.ok) return;
  int const wb = push_win_bits(n_rows, tu, wide && !w && tu.pr_packed);
  int const sb = 32 - wb;
  if (wb != 14 || w || !tu.pr_packed || band_cut >= n_cols) band_cut = 0;
  pp.carry.release();
  int64_t const nwin_real = std::max<int64_t>(1, (n_rows + (int64_t(1) << wb) - 1) >> wb);
  int64_t const nwin      = band_cut > 0 ? 2 * nwin_real : nwin_real;
  pp.win_bits        = wb;
  pp.nwin            = nwin;
  pp.bands           = band_cut > 0;
  pp.nwin_real       = nwin_real;
  pp.nacc            = nwin << wb;
  pp.acc.set_stream(s);
  pp.acc.resize(pp.nacc * sizeof(unsigned long long));
  HIP_CHECK(hipMemsetAsync(pp.acc.data(), 0, pp.nacc * sizeof(unsigned long long), s));
  pp.tile_ctr.set_stream(s);
  pp.tile_ctr.resize(2 * kQueues * kCtrStride * sizeof(unsigned int));  // two sets: iteration parity
  HIP_CHECK(hipMemsetAsync(pp.tile_ctr.data(), 0, 2 * kQueues * kCtrStride * sizeof(unsigned int), s));
  pp.nunits = 0;
  pp.nitems = 0;
  pp.qoff.assign(kQueues + 1, 0);
  if (ne == 0) return;
  dbuf<uint64_t> keys_out(ne, s);
  dbuf<uint32_t> vals_out(ne, s);
  {
    dbuf<uint64_t> keys(ne, s);
    dbuf<uint32_t> vals(ne, s);
    hipLaunchKernelGGL(k_push_keys<C>, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, cols, rows, ne, wb,
                       (uint32_t)band_cut, nwin_real, keys.data(), vals.data());
    CGX_LAUNCH_CHECK();
    radix_sort_pairs<uint64_t, uint32_t>(keys.data(), keys_out.data(), vals.data(), vals_out.data(), (size_t)ne,
                                         col_sorted ? 32 : 0,
                                         32 + bits_for((unsigned long long)std::max<int64_t>(nwin - 1, 1)), s);
  }
  dbuf<int64_t> ws(nwin + 1, s);
  hipLaunchKernelGGL(k_win_starts<key_w32>, dim3(grid_for(nwin + 1, kBlock, 4096)), dim3(kBlock), 0, s,
                     keys_out.data(), ne, nwin, ws.data(), key_w32{});
  CGX_LAUNCH_CHECK();
  pp.packed = false;
  if (!w && tu.pr_packed) {  // 16-bit entries unless the jumps would grow the entries by more than half
    uint32_t const dmax = (1u << (16 - wb)) - 2;  // coded deltas 0 .. dmax; dmax + 1 marks a jump
    uint32_t const pmax = (1u << wb) - 1;         // jump payloads 1 .. pmax
    dbuf<uint32_t> mj(ne + 1, s);
    dbuf<unsigned long long> ex(ne + 1, s);
    hipLaunchKernelGGL(k_jump_counts<key_w32>, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s,
                       keys_out.data(), ne, ws.data(), dmax, pmax, mj.data(), key_w32{});
    CGX_LAUNCH_CHECK();
    fill<uint32_t>(mj.data() + ne, 1, 0u, s);
    exclusive_scan<uint32_t, unsigned long long>(mj.data(), ex.data(), ne + 1, s);
    int64_t const total0 = ne + (int64_t)to_host(ex.data() + ne, 1, s)[0];
    unsigned long long const* cm = ex.data() + 1;  // inclusive prefix
    // windows padded to whole wave segments (k_packed_pads)
    dbuf<unsigned long long> pad(nwin + 1, s), pb(nwin + 1, s);
    hipLaunchKernelGGL(k_packed_pads<unsigned long long>, dim3(grid_for(nwin + 1, kBlock, 4096)), dim3(kBlock), 0, s, ws.data(), cm, nwin,
                       total0, pad.data());
    CGX_LAUNCH_CHECK();
    exclusive_scan<unsigned long long, unsigned long long>(pad.data(), pb.data(), nwin + 1, s);
    int64_t const total = total0 + (int64_t)to_host(pb.data() + nwin, 1, s)[0];
    if (std::getenv("CGX_PR_DEBUG"))  // measurement only
      std::fprintf(stderr, "[pr] schedule: %lld rows, %lld sources, %lld edges, %d-bit windows, %lld packed entries\n",
                   (long long)n_rows, (long long)n_cols, (long long)ne, wb, (long long)total);
    if (total <= ne + ne / 2 && (uint64_t)total < (1ull << 32)) {
      uint16_t const pad_code = (uint16_t)(((1u << (16 - wb)) - 1) << wb);  // a jump of 0: no edge
      pp.packed = true;
      if (wb == 15) {  // the 32K push's per-destination carry words
        pp.carry.set_stream(s);
        pp.carry.resize(pp.nacc * sizeof(uint32_t));
        HIP_CHECK(hipMemsetAsync(pp.carry.data(), 0, pp.nacc * sizeof(uint32_t), s));
      }
      pp.ent16.set_stream(s);
      pp.ent16.resize((total + kPushUnit) * sizeof(uint16_t));  // + a unit: the kernel prefetches whole units
      fill<uint16_t>(pp.ent16.data<uint16_t>(), (size_t)(total + kPushUnit), pad_code, s);
      hipLaunchKernelGGL(k_pack16, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, keys_out.data(),
                         vals_out.data(), rows, ne, ws.data(), mj.data(), cm, pb.data(), wb, pmax,
                         pp.ent16.data<uint16_t>());
      CGX_LAUNCH_CHECK();
      dbuf<int64_t> nws(nwin + 1, s);
      hipLaunchKernelGGL(k_packed_win_starts<unsigned long long>, dim3(grid_for(nwin + 1, kBlock, 4096)), dim3(kBlock), 0, s, ws.data(),
                         cm, pb.data(), nwin, total0, nws.data());
      dbuf<uint32_t> pflag(total + 1, s), puid(total + 1, s);
      fill<uint32_t>(pflag.data(), (size_t)(total + 1), 0u, s);
      hipLaunchKernelGGL(k_packed_unit_marks, dim3(grid_for(nwin, 64, 4096)), dim3(64), 0, s, nws.data(), nwin,
                         pflag.data());
      CGX_LAUNCH_CHECK();
      exclusive_scan<uint32_t, uint32_t>(pflag.data(), puid.data(), total + 1, s);
      int64_t const nunits = (int64_t)to_host(puid.data() + total, 1, s)[0];
      pp.units.set_stream(s);
      pp.units.resize(std::max<int64_t>(nunits, 1) * sizeof(push_unit));
      push_unit* units = pp.units.data<push_unit>();
      hipLaunchKernelGGL(k_packed_unit_heads, dim3(grid_for(total, kBlock, 16384)), dim3(kBlock), 0, s, pflag.data(),
                         puid.data(), total, nws.data(), nwin, units);
      CGX_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_unit_ends, dim3(grid_for(nunits, kBlock, 4096)), dim3(kBlock), 0, s, units, nunits, total);
      CGX_LAUNCH_CHECK();
      pp.seg_base.set_stream(s);
      pp.seg_base.resize(std::max<int64_t>(nunits * kSegsPerUnit, 1) * sizeof(uint32_t));
      hipLaunchKernelGGL((k_seg_bases<key_w32, unsigned long long>), dim3(grid_for(nunits * kSegsPerUnit, kBlock, 16384)), dim3(kBlock), 0, s, units,
                         nunits, keys_out.data(), ne, ws.data(), mj.data(), cm, pb.data(), dmax, pmax,
                         pp.seg_base.data<uint32_t>(), key_w32{});
      CGX_LAUNCH_CHECK();
      pp.ent.release();
      pp.ew.release();
      build_items(s, pp, units, nunits, wb >= 13, tu);
      pp.nunits = nunits;
      HIP_CHECK(hipStreamSynchronize(s));
      return;
    }
  }
  if (band_cut > 0 || wb == 15) {  // bands and 32K windows need the packed format: the schedule without them
    keys_out.free();
    vals_out.free();
    ws.free();
    build_push_from_coo<C, R>(s, rows, cols, w, ne, n_rows, n_cols, pp, tu, col_sorted, 0, false);
    return;
  }
  dbuf<uint32_t> flag(ne + 1, s), uid(ne + 1, s);
  hipLaunchKernelGGL(k_unit_flags, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, keys_out.data(), ne,
                     ws.data(), sb, flag.data());
  CGX_LAUNCH_CHECK();
  fill<uint32_t>(flag.data() + ne, 1, 0u, s);
  exclusive_scan<uint32_t, uint32_t>(flag.data(), uid.data(), ne + 1, s);
  int64_t const nunits = (int64_t)to_host(uid.data() + ne, 1, s)[0];
  pp.units.set_stream(s);
  pp.units.resize(std::max<int64_t>(nunits, 1) * sizeof(push_unit));
  push_unit* units = pp.units.data<push_unit>();
  hipLaunchKernelGGL(k_unit_heads, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, keys_out.data(),
                     flag.data(), uid.data(), ne, units);
  CGX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_unit_ends, dim3(grid_for(nunits, kBlock, 4096)), dim3(kBlock), 0, s, units, nunits, ne);
  CGX_LAUNCH_CHECK();
  pp.ent.set_stream(s);
  pp.ent.resize((ne + kPushUnit) * sizeof(uint32_t));  // padded: the kernel loads whole units
  HIP_CHECK(hipMemsetAsync(pp.ent.data<uint32_t>() + ne, 0, kPushUnit * sizeof(uint32_t), s));
  pp.ew.set_stream(s);
  if (w) {
    pp.ew.resize((ne + kPushUnit) * sizeof(R));  // padded like ent
    HIP_CHECK(hipMemsetAsync(pp.ew.data<R>() + ne, 0, kPushUnit * sizeof(R), s));
  } else {
    pp.ew.release();
  }
  hipLaunchKernelGGL(k_push_pack<R>, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, keys_out.data(),
                     vals_out.data(), rows, w, flag.data(), uid.data(), units, ne, wb, pp.ent.data<uint32_t>(),
                     w ? pp.ew.data<R>() : nullptr);
  CGX_LAUNCH_CHECK();
  build_items(s, pp, units, nunits, wb >= 13, tu);
  pp.nunits = nunits;
  HIP_CHECK(hipStreamSynchronize(s));
}

// weights all exactly 1 (what cugraph.Graph attaches to an unweighted edge list,
// simpleGraph.py:840-843): then outw = degree and x~ * w = x~ bit for bit, so the
// push takes the unweighted 16-bit entries and skips the 4 B/edge weight stream
template <typename R>
__global__ void k_count_non_unit(R const* w, size_t n, int* bad)
{
  int mine = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    mine |= w[i] != R(1);
  if (__any(mine) && (threadIdx.x & 63) == 0) atomicOr(bad, 1);
}

template <typename R>
bool unit_weights(handle_t& h, graph_t& g, adjacency_t& adj)
{
  if (!g.weighted) return false;
  if (adj.unit_weights < 0) {
    hipStream_t s = h.stream;
    dbuf<int> bad(1, s);
    fill<int>(bad.data(), 1, 0, s);
    if (g.num_edges)
      hipLaunchKernelGGL(k_count_non_unit<R>, dim3(grid_for((size_t)g.num_edges, kBlock, 4096)), dim3(kBlock), 0, s,
                         adj.weights.data<R>(), (size_t)g.num_edges, bad.data());
    CGX_LAUNCH_CHECK();
    adj.unit_weights = (to_host_scalar(bad.data(), s) == 0 && h.tune.pr_unit_w) ? 1 : 0;  // A/B
  }
  return adj.unit_weights == 1;
}

// The window sort of the one-word keys: up to 10 window bits (RMAT-24 and below at
// 16K windows) in ONE onesweep pass of 10 radix bits (1024-thread blocks, match
// ranking, 8 keys a thread) -- 5.75 ms for 500M keys against 7.03 for the gfx950
// default's two 8-bit passes (scripts/ubench/radix_bits.hip, profiles/r05/radix_bits.txt);
// wider window fields keep the default (a 10-bit pass is slower there: 9.8 vs 7.1 ms
// at 12 bits).
using window_sort_10 = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, 10,
                                        rocprim::block_radix_rank_algorithm::match>>;
template <typename C>
void sort_window_keys(rocprim::double_buffer<uint64_t>& db, int64_t ne, int shv, int vbits, hipStream_t s)
{
  size_t tmp = 0;
  HIP_CHECK(rocprim::radix_sort_keys<C>(nullptr, tmp, db, (size_t)ne, shv, shv + vbits, s));
  buffer t(tmp, s);
  HIP_CHECK(rocprim::radix_sort_keys<C>(t.data(), tmp, db, (size_t)ne, shv, shv + vbits, s));
}

// The packed schedule of a symmetric unweighted graph straight from its adjacency
// (build_push_from_coo's packed path with key_p keys; same stream, units, bases and
// items bit for bit): one word per entry through a keys-only sort of the window bits,
// no destination gather while packing, units from the window starts.  RMAT-24's first
// call spent 29 ms in the general build.  false: the keys do not fit a word or the
// stream would not pack -- nothing built, the caller takes the general path.
template <typename E, typename CM>
bool build_push_packed_sym_cm(hipStream_t s, E const* off, uint32_t const* idx, int64_t ne, int64_t nv, pr_push_t& pp,
                              tuning_t const& tu, int64_t band_cut, bool wide)
{
  int const wb = push_win_bits(nv, tu, wide);
  if (wb != 14 || band_cut >= nv) band_cut = 0;
  int64_t const nwin_real = std::max<int64_t>(1, (nv + (int64_t(1) << wb) - 1) >> wb);
  int64_t const nwin      = band_cut > 0 ? 2 * nwin_real : nwin_real;
  int const sbits = std::max(1, bits_for((unsigned long long)std::max<int64_t>(nv - 1, 1)));
  int const vbits = std::max(1, bits_for((unsigned long long)std::max<int64_t>(nwin - 1, 1)));
  int const shv   = wb + sbits;
  if (shv + vbits > 64 || (uint64_t)ne >= (1ull << 32) || (uint64_t)nv >= (1ull << 32)) return false;
  key_p const kc{shv, wb, (sbits >= 32 ? ~0ull : ((1ull << sbits) - 1ull))};
  uint32_t const dmax = (1u << (16 - wb)) - 2, pmax = (1u << wb) - 1;
  dbuf<uint64_t> kbuf(std::max<int64_t>(ne, 1), s);
  {
    dbuf<uint64_t> k2(std::max<int64_t>(ne, 1), s);
    if (ne) {
      hipLaunchKernelGGL(k_push_keys_p<E>, dim3((unsigned)std::min<int64_t>((ne + kRowsTile - 1) / kRowsTile, 65536)),
                         dim3(256), 0, s, off, idx, nv, ne, wb, shv, (uint32_t)band_cut, nwin_real, kbuf.data());
      CGX_LAUNCH_CHECK();
      rocprim::double_buffer<uint64_t> db(kbuf.data(), k2.data());
      if (vbits <= 10) sort_window_keys<window_sort_10>(db, ne, shv, vbits, s);
      else sort_window_keys<rocprim::default_config>(db, ne, shv, vbits, s);
      if (db.current() != kbuf.data()) std::swap(kbuf, k2);
    }
  }
  uint64_t const* keys = kbuf.data();
  dbuf<int64_t> ws(nwin + 1, s);
  hipLaunchKernelGGL(k_win_starts<key_p>, dim3(grid_for(nwin + 1, kBlock, 4096)), dim3(kBlock), 0, s, keys, ne, nwin,
                     ws.data(), kc);
  CGX_LAUNCH_CHECK();
  dbuf<CM> ex(ne + 1, s);
  {
    auto jumps = rocprim::make_transform_iterator(rocprim::make_counting_iterator<int64_t>(0),
                                                  jump_count_p{keys, ws.data(), ne, kc, dmax, pmax});
    size_t tmp = 0;
    HIP_CHECK(rocprim::exclusive_scan(nullptr, tmp, jumps, ex.data(), CM(0), (size_t)(ne + 1), rocprim::plus<CM>(), s));
    buffer t(tmp, s);
    HIP_CHECK(rocprim::exclusive_scan(t.data(), tmp, jumps, ex.data(), CM(0), (size_t)(ne + 1), rocprim::plus<CM>(), s));
  }
  int64_t const total0 = ne + (int64_t)to_host(ex.data() + ne, 1, s)[0];
  CM const* cm         = ex.data() + 1;  // inclusive prefix
  dbuf<unsigned long long> pad(nwin + 1, s), pb(nwin + 1, s);
  hipLaunchKernelGGL(k_packed_pads<CM>, dim3(grid_for(nwin + 1, kBlock, 4096)), dim3(kBlock), 0, s, ws.data(), cm, nwin,
                     total0, pad.data());
  CGX_LAUNCH_CHECK();
  exclusive_scan<unsigned long long, unsigned long long>(pad.data(), pb.data(), nwin + 1, s);
  int64_t const total = total0 + (int64_t)to_host(pb.data() + nwin, 1, s)[0];
  if (!(total <= ne + ne / 2 && (uint64_t)total < (1ull << 32))) return false;
  pp.built     = true;
  pp.ok        = true;
  pp.win_bits  = wb;
  pp.nwin      = nwin;
  pp.bands     = band_cut > 0;
  pp.nwin_real = nwin_real;
  pp.nacc      = nwin << wb;
  pp.acc.set_stream(s);
  pp.acc.resize(pp.nacc * sizeof(unsigned long long));
  HIP_CHECK(hipMemsetAsync(pp.acc.data(), 0, pp.nacc * sizeof(unsigned long long), s));
  pp.tile_ctr.set_stream(s);
  pp.tile_ctr.resize(2 * kQueues * kCtrStride * sizeof(unsigned int));
  HIP_CHECK(hipMemsetAsync(pp.tile_ctr.data(), 0, 2 * kQueues * kCtrStride * sizeof(unsigned int), s));
  pp.carry.release();
  if (wb == 15) {
    pp.carry.set_stream(s);
    pp.carry.resize(pp.nacc * sizeof(uint32_t));
    HIP_CHECK(hipMemsetAsync(pp.carry.data(), 0, pp.nacc * sizeof(uint32_t), s));
  }
  pp.qoff.assign(kQueues + 1, 0);
  pp.nitems = 0;
  pp.packed = true;
  uint16_t const pad_code = (uint16_t)(((1u << (16 - wb)) - 1) << wb);  // a jump of 0: no edge
  pp.ent16.set_stream(s);
  pp.ent16.resize((total + kPushUnit) * sizeof(uint16_t));  // + a unit: the kernel prefetches whole units
  fill<uint16_t>(pp.ent16.data<uint16_t>(), (size_t)(total + kPushUnit), pad_code, s);
  if (ne)
    hipLaunchKernelGGL(k_pack16_p<CM>, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, keys, ne, ws.data(),
                       cm, pb.data(), kc, pmax, pp.ent16.data<uint16_t>());
  CGX_LAUNCH_CHECK();
  dbuf<int64_t> nws(nwin + 1, s);
  hipLaunchKernelGGL(k_packed_win_starts<CM>, dim3(grid_for(nwin + 1, kBlock, 4096)), dim3(kBlock), 0, s, ws.data(),
                     cm, pb.data(), nwin, total0, nws.data());
  CGX_LAUNCH_CHECK();
  dbuf<uint32_t> ucnt(nwin + 1, s), upos(nwin + 1, s);
  hipLaunchKernelGGL(k_unit_counts, dim3(grid_for(nwin + 1, kBlock, 4096)), dim3(kBlock), 0, s, nws.data(), nwin,
                     ucnt.data());
  CGX_LAUNCH_CHECK();
  exclusive_scan<uint32_t, uint32_t>(ucnt.data(), upos.data(), nwin + 1, s);
  int64_t const nunits = (int64_t)to_host(upos.data() + nwin, 1, s)[0];
  pp.units.set_stream(s);
  pp.units.resize(std::max<int64_t>(nunits, 1) * sizeof(push_unit));
  push_unit* units = pp.units.data<push_unit>();
  if (nunits)
    hipLaunchKernelGGL(k_units_direct, dim3(grid_for(nunits, kBlock, 4096)), dim3(kBlock), 0, s, nws.data(), nwin,
                       upos.data(), nunits, units);
  CGX_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_unit_ends, dim3(grid_for(nunits, kBlock, 4096)), dim3(kBlock), 0, s, units, nunits, total);
  CGX_LAUNCH_CHECK();
  pp.seg_base.set_stream(s);
  pp.seg_base.resize(std::max<int64_t>(nunits * kSegsPerUnit, 1) * sizeof(uint32_t));
  if (nunits)
    hipLaunchKernelGGL((k_seg_bases<key_p, CM>), dim3(grid_for(nunits * kSegsPerUnit, kBlock, 16384)), dim3(kBlock), 0,
                       s, units, nunits, keys, ne, ws.data(), (uint32_t const*)nullptr, cm, pb.data(), dmax, pmax,
                       pp.seg_base.data<uint32_t>(), kc);
  CGX_LAUNCH_CHECK();
  pp.ent.release();
  pp.ew.release();
  build_items(s, pp, units, nunits, wb >= 13, tu);
  pp.nunits = nunits;
  HIP_CHECK(hipStreamSynchronize(s));
  return true;
}

template <typename E>
bool build_push_packed_sym(hipStream_t s, E const* off, uint32_t const* idx, int64_t ne, int64_t nv, pr_push_t& pp,
                           tuning_t const& tu, int64_t band_cut, bool wide)
{
  if (ne < (int64_t(1) << 31)) return build_push_packed_sym_cm<E, uint32_t>(s, off, idx, ne, nv, pp, tu, band_cut, wide);
  return build_push_packed_sym_cm<E, unsigned long long>(s, off, idx, ne, nv, pp, tu, band_cut, wide);
}

template <typename V, typename E, typename R>
void build_pr_push_schedule(handle_t& h, graph_t& g, adjacency_t& adj, bool use_weights)
{
  hipStream_t s = h.stream;
  int64_t nv    = g.num_vertices;
  int64_t ne    = g.num_edges;
  if ((uint64_t)ne >= (1ull << 32) || (uint64_t)nv >= (1ull << 32)) {
    adj.pr.built = true;
    adj.pr.ok    = false;
    return;
  }
  if constexpr (sizeof(V) == 4) {
    if (g.symmetric && !use_weights && h.tune.pr_packed && h.tune.pr_fast_build &&
        build_push_packed_sym<E>(s, adj.offsets.data<E>(), reinterpret_cast<uint32_t const*>(adj.indices.data<V>()), ne,
                                 nv, adj.pr, h.tune, push_band_cut(nv, h.tune), /*wide=*/sizeof(R) == 4))
      return;
  }
  dbuf<uint32_t> rows(std::max<int64_t>(ne, 1), s);
  if (ne)
    hipLaunchKernelGGL(k_edge_rows<E>, dim3((unsigned)std::min<int64_t>((ne + kRowsTile - 1) / kRowsTile, 65536)),
                       dim3(256), 0, s, adj.offsets.data<E>(), nv, ne, rows.data());
  CGX_LAUNCH_CHECK();
  if constexpr (sizeof(V) == 4) {
    if (g.symmetric) {  // the same edges read as out-edges: (source = row, destination = index), source-sorted
      build_push_from_coo<uint32_t, R>(s, reinterpret_cast<uint32_t const*>(adj.indices.data<V>()), rows.data(),
                                       use_weights ? adj.weights.data<R>() : nullptr, ne, nv, nv, adj.pr, h.tune,
                                       /*col_sorted=*/true, push_band_cut(nv, h.tune), /*wide=*/sizeof(R) == 4);
      return;
    }
  }
  build_push_from_coo<V, R>(s, rows.data(), adj.indices.data<V>(), use_weights ? adj.weights.data<R>() : nullptr, ne,
                            nv, nv, adj.pr, h.tune, false, push_band_cut(nv, h.tune), /*wide=*/sizeof(R) == 4);
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
void set_queue_args(push_args<V, E, R>& sa, pr_push_t& pp, hipStream_t s)
{
  sa.ent      = pp.ent.data<uint32_t>();
  sa.ew       = pp.ew.empty() ? nullptr : pp.ew.data<R>();
  sa.ent16    = pp.ent16.data<uint16_t>();
  sa.seg_base = pp.seg_base.data<uint32_t>();
  sa.units    = pp.units.data<push_unit>();
  sa.nunits   = pp.nunits;
  sa.acc      = pp.acc.data<unsigned long long>();
  sa.carry    = pp.win_bits == 15 ? pp.carry.data<uint32_t>() : nullptr;
  sa.items    = pp.items.data<int64_t>();
  sa.queue    = pp.queue.data<int64_t>();
  sa.nitems   = pp.nitems;
  for (int q = 0; q <= kQueues; ++q) sa.qoff[q] = q < (int)pp.qoff.size() ? pp.qoff[q] : 0;
  sa.tile_ctr = pp.tile_ctr.data<unsigned int>();
  sa.nwin     = pp.nwin;
  HIP_CHECK(hipMemsetAsync(sa.tile_ctr, 0, 2 * kQueues * kCtrStride * sizeof(unsigned int), s));
  sa.fuse      = 0;  // the caller opts in (fuse_apply)
  sa.parity    = 0;
  sa.bands     = pp.bands ? 1 : 0;
  sa.nwin_real = pp.nwin_real;
  sa.win_pub   = pp.bands ? pp.win_pub.data<uint32_t>() : nullptr;
  if (!pp.win_items.empty()) {
    sa.win_items  = pp.win_items.data<uint32_t>();
    sa.win_left   = pp.win_left.data<uint32_t>();
    sa.empty_wins = pp.empty_wins.data<int64_t>();
    sa.nempty     = pp.nempty;
    sa.nwin_items = pp.nwin_items;
    int64_t const nreal = pp.bands ? pp.nwin_real : pp.nwin;
    HIP_CHECK(hipMemcpyAsync(sa.win_left, sa.win_items, nreal * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    if (pp.bands) HIP_CHECK(hipMemsetAsync(sa.win_pub, 0, nreal * sizeof(uint32_t), s));
  }

}

// fused apply (fused_finish): 16K windows, items, few windows without items (the last
// block applies those alone); tuning_t::pr_fuse = 0 keeps the separate k_pr_apply (A/B)
inline bool fuse_apply(pr_push_t const& pp, tuning_t const& tu)
{
  if (pp.bands) return pp.nitems > 0;  // (a banded schedule has no separate apply)
  return pp.win_bits >= 14 && pp.nitems > 0 && pp.nwin_items > 0 && pp.nempty <= 64 && !pp.win_items.empty() &&
         tu.pr_fuse;
}

// the push kernel for the schedule's window bits and entry format
template <typename V, typename E, typename R>
auto push_kernel(pr_push_t const& pp, bool weighted, bool enc = false)
{
  if (pp.win_bits == 15) return enc ? k_pr_push16_w15<V, E, R, true> : k_pr_push16_w15<V, E, R, false>;
  if (pp.win_bits == 14) {
    if (pp.packed && pp.bands) return enc ? k_pr_push16_w14<V, E, R, true, true> : k_pr_push16_w14<V, E, R, false, true>;
    if (pp.packed) return enc ? k_pr_push16_w14<V, E, R, true> : k_pr_push16_w14<V, E, R, false>;
    return weighted ? k_pr_push_q_w14<V, E, R, true> : k_pr_push_q_w14<V, E, R, false>;
  }
  if (pp.packed) {
    if (enc) return pp.win_bits == 13 ? k_pr_push16<13, V, E, R, true> : k_pr_push16<12, V, E, R, true>;
    return pp.win_bits == 13 ? k_pr_push16<13, V, E, R, false> : k_pr_push16<12, V, E, R, false>;
  }
  constexpr bool wide = sizeof(R) == 8;  // fp64 weights: no 8-waves bound (see k_pr_push_q_wide)
  if (pp.win_bits == 13)
    return weighted ? (wide ? k_pr_push_q_wide<13, V, E, R, true> : k_pr_push_q<13, V, E, R, true>)
                    : k_pr_push_q<13, V, E, R, false>;
  return weighted ? (wide ? k_pr_push_q_wide<12, V, E, R, true> : k_pr_push_q<12, V, E, R, true>)
                  : k_pr_push_q<12, V, E, R, false>;
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

  // windowed push (our own out-weight sums keep every fixed-point sum <= 1; user
  // precomputed out-weights may not: generic pull kernel then)
  bool push = pow_v == nullptr && max_iter > 0;
  bool const push_w = g.weighted && !(push && unit_weights<R>(h, g, adj));  // entry weights in the push
  if (push && !adj.pr.built) build_pr_push_schedule<V, E, R>(h, g, adj, push_w);
  push = push && adj.pr.ok;
  // the degree-binned pull schedule only for the pull path (its host-built items were
  // 7.4 ms of a first call at RMAT-24 that never used them)
  if (!push) ensure_schedule(h, g, adj);

  // iteration state
  int const nblk_iter = push ? 0 : (int)adj.num_items;
  int const nblk_init = (int)grid_for(nv, kBlock, 1024);
  dbuf<double> partials(2 * std::max<int64_t>({nblk_iter, nblk_init, 2048, (nv + 4095) / 4096}), s);
  dbuf<pr_state> st(1, s);
  HIP_CHECK(hipMemsetAsync(st.data(), 0, sizeof(pr_state), s));
  dbuf<R> xa(nv, s), xb(nv, s);

  pr_args<V, E, R> a{};
  a.off      = adj.offsets.data<E>();
  a.idx      = adj.indices.data<V>();
  a.wgt      = g.weighted ? adj.weights.data<R>() : nullptr;
  a.order    = push || adj.degree_sorted ? nullptr : adj.order.data<V>();
  a.items    = push ? nullptr : adj.items.data<work_item>();
  a.pr       = pr;
  a.outw     = outw;
  a.pers     = pers.data();
  a.alpha    = alpha;
  a.eps      = eps;
  a.max_iter = (int)std::min<size_t>(max_iter, (size_t)INT32_MAX);
  a.nv       = nv;
  a.nv_global = nv;
  a.partials = partials.data();
  a.st       = st.data();
  a.x_in     = nullptr;
  a.x_out    = xa.data();

  // fp32 packed push: x~ as enc_fixed words (tuning_t::pr_enc = 0: plain floats, A/B)
  a.enc  = push && adj.pr.packed && std::is_same<R, float>::value && h.tune.pr_enc;
  a.fp64 = push ? 0 : 1;
  hipLaunchKernelGGL((k_pr_init<V, E, R>), dim3(nblk_init), dim3(kBlock), 0, s, a);
  CGX_LAUNCH_CHECK();

  if (max_iter == 0) fail(CUGRAPH_UNKNOWN_ERROR, "PageRank failed to converge.");

  push_args<V, E, R> sa{};
  int nblk_push = 0, nblk_apply = 0;
  bool const fuse = push && fuse_apply(adj.pr, h.tune);
  auto pkernel    = push_kernel<V, E, R>(adj.pr, push_w, a.enc != 0);
  if (push) {
    set_queue_args(sa, adj.pr, s);
    sa.win_multi = adj.pr.win_multi.data<uint8_t>();  // single GPU: stored windows are not cleared
    sa.win_bits  = adj.pr.win_bits;
    nblk_push  = sa.nitems ? push_blocks(sa.win_bits) : 0;
    nblk_apply = (int)grid_for(nv, kBlock, 512);  // fewer tickets: 512 measured best
    sa.fuse    = fuse ? 1 : 0;
    sa.nhub    = h.tune.pr_hub ? nv : 0;  // hub x~ staged in LDS (16K windows; A/B switch)
  }
  // measured-cost queues: the first launch on this schedule records item durations
  bool calibrating = push && calibration_wanted(adj.pr, h.tune);
  if (calibrating) {
    adj.pr.item_ticks.set_stream(s);
    adj.pr.item_ticks.resize(adj.pr.nitems * sizeof(uint32_t));
    HIP_CHECK(hipMemsetAsync(adj.pr.item_ticks.data(), 0, adj.pr.nitems * sizeof(uint32_t), s));
    adj.pr.calib = 1;
  } else if (push && adj.pr.calib == 0) {
    adj.pr.calib = 2;
  }
  // CGX_PR_TIMELINE=<file>: per-item timeline of the packed push (measurement only)
  char const* tl_path = push ? std::getenv("CGX_PR_TIMELINE") : nullptr;
  dbuf<unsigned long long> tl;
  if (tl_path) {
    sa.tl_cap = 1 << 20;
    tl.resize(1 + 4 * sa.tl_cap, s);
    HIP_CHECK(hipMemsetAsync(tl.data(), 0, sizeof(unsigned long long), s));
    sa.tl = tl.data();
  }
  // Chunked enqueue (next_chunk): a host check after 8 iterations, then after the
  // predicted remainder.  Profiling records one pair of pooled HIP events around each chunk -- an event
  // between every two iterations cost a ~10 us queue gap per iteration -- and
  // reports chunk time / iterations run, so the no-op launches after convergence
  // in the last chunk count against the kernels.
  std::vector<hipEvent_t> ev;
  pr_state hst{};
  R* bufs[2]    = {xa.data(), xb.data()};
  size_t launched = 0;
  // A repeated plain call on this graph (same alpha and epsilon, no initial guess or
  // personalization: the same iterations) enqueues the last call's count at once: one
  // host round trip instead of two (launches past convergence return at once)
  bool const plain = push && !guess_v && !pers.data() && !calibrating;
  int const hint   = plain && adj.pr.last_alpha == alpha && adj.pr.last_eps == eps ? adj.pr.last_iters : 0;
  auto kernel  = g.weighted ? k_pr_iter<V, E, R, true> : k_pr_iter<V, E, R, false>;
  pr_state* hpin = h.pinned_as<pr_state>();
  while (true) {
    if (h.profiling) {
      ev.push_back(h.event(ev.size()));  // pooled on the handle
      ev.push_back(h.event(ev.size()));
      HIP_CHECK(hipEventRecord(ev[ev.size() - 2], s));
    }
    int const chunk = launched == 0 && hint > 0 ? std::min(std::min(hint, 64), std::max(1, a.max_iter))
                                                : next_chunk(hst, eps, a.max_iter);
    for (int i = 0; i < chunk; ++i) {
      a.x_in  = bufs[launched & 1];
      a.x_out = bufs[(launched + 1) & 1];
      if (push) {
        sa.a          = a;
        sa.parity     = (int)(launched & 1);
        sa.launch     = (int)launched;
        sa.item_ticks = calibrating && launched == 0 ? adj.pr.item_ticks.data<uint32_t>() : nullptr;
        if (nblk_push) hipLaunchKernelGGL(pkernel, dim3(nblk_push), dim3(kPushThreads), 0, s, sa);
        if (!sa.fuse) hipLaunchKernelGGL((k_pr_apply<V, E, R>), dim3(nblk_apply), dim3(kBlock), 0, s, sa);
      } else {
        hipLaunchKernelGGL(kernel, dim3(nblk_iter), dim3(kBlock), 0, s, a);
      }
      CGX_LAUNCH_CHECK();
      ++launched;
    }
    if (h.profiling) HIP_CHECK(hipEventRecord(ev.back(), s));
    HIP_CHECK(hipMemcpyAsync(hpin, st.data(), sizeof(pr_state), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    hst = *hpin;
    if (calibrating) {  // re-deal the queues by the recorded costs (the stream is idle here)
      calibrate_queues(s, adj.pr, h.tune);
      for (int q = 0; q <= kQueues; ++q) sa.qoff[q] = adj.pr.qoff[q];
      calibrating = false;
    }
    if (hst.done) break;
  }
  h.last_iterations = (size_t)hst.iter;
  if (push && !guess_v && !pers.data()) {
    adj.pr.last_iters = hst.iter;
    adj.pr.last_alpha = alpha;
    adj.pr.last_eps   = eps;
  }
  if (tl_path) {
    unsigned long long n = 0;
    HIP_CHECK(hipMemcpyAsync(&n, tl.data(), sizeof(n), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    n = std::min<unsigned long long>(n, (unsigned long long)sa.tl_cap);
    std::vector<unsigned long long> rec(4 * n);
    if (n) HIP_CHECK(hipMemcpyAsync(rec.data(), tl.data() + 1, rec.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (FILE* f = std::fopen(tl_path, "w")) {
      std::fprintf(f, "launch,block,item,entries,window,start,end\n");
      auto hu = to_host(adj.pr.units.data<push_unit>(), adj.pr.nunits, s);
      auto hi = to_host(adj.pr.items.data<int64_t>(), adj.pr.nitems + 1, s);
      for (unsigned long long i = 0; i < n; ++i) {
        unsigned long long const it = rec[4 * i + 1] & 0xffffffffull;
        std::fprintf(f, "%llu,%llu,%llu,%llu,%lld,%llu,%llu\n", rec[4 * i] >> 32, rec[4 * i] & 0xffffffffull, it,
                     rec[4 * i + 1] >> 32, (long long)(hu[hi[it]].win & kWinMask), rec[4 * i + 2], rec[4 * i + 3]);
      }
      std::fclose(f);
    }
  }
  if (h.profiling) {
    double tot = 0;
    for (size_t i = 0; i + 1 < ev.size(); i += 2) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
      tot += ms;
    }
    h.last_hot_ms       = tot;
    h.last_hot_launches = std::max<size_t>((size_t)hst.iter, 1);
  }
  if (hst.done == 2) fail(CUGRAPH_UNKNOWN_ERROR, "PageRank failed to converge.");
}

// ---------------------------------------------------------------- multi-GPU (2D partition)
// Rank (r, c) holds the edges whose source is owned by row r and destination by
// column c (mg_graph.hpp).  Per iteration (pagerank_impl.cuh:241-257 MG path):
//   row allgather of x~ (each rank's owned slice, padded to the row's largest) ->
//   windowed push over the local block into fixed-point sums for the column's
//   destinations -> column reduce-scatter (u64 sums: exact) -> apply on the owned
//   vertices -> world allreduce of (diff, dangling) -> state update.
// Everything is stream-ordered; the host reads the convergence flag once per chunk.
//
// Row chunks (R > 1): the block's destination rows are cut into K chunks of cs
// owner-local rows, chunk k holding rows [k cs, (k + 1) cs) of every owner in the
// column, laid out [owner][row] -- so chunk k's sums are one contiguous R x cs array
// and its reduce-scatter hands each owner its cs rows of the chunk.  Each chunk has
// its own push schedule; the iteration pushes the chunks one after another and
// reduce-scatters chunk k on a second stream while the push works on chunk k + 1.
struct mg_chunk {
  pr_push_t pp;              // rows: owner * cs + (owner-local row - k cs)
  dbuf<int64_t> multi_wins;  // windows summed by several items (their sums are added: cleared per iteration)
  int64_t nmulti = 0;
};

struct mg_pr_block {
  int64_t nmax_row = 0, nmax_col = 0;
  int K = 1;                       // row chunks (1 when R = 1: no reduce-scatter to overlap)
  int64_t cs = 0;                  // owner-local rows per chunk
  std::vector<mg_chunk> ch;
  buffer outw;  // weight_t[n_own]
  hipStream_t comm_stream = nullptr;  // the chunks' reduce-scatters (R > 1)
  std::vector<hipEvent_t> ev;         // K push-done events + 1 reduce-scatters-done
  ~mg_pr_block()
  {
    for (auto e : ev) (void)hipEventDestroy(e);
    if (comm_stream) (void)hipStreamDestroy(comm_stream);
  }
};

// first position of each key 0..K in a sorted array (K + 1 binary searches)
__global__ void k_sorted_starts(uint32_t const* sorted, int64_t n, int K, int64_t* st)
{
  for (int k = threadIdx.x; k <= K; k += blockDim.x) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      int64_t const mid = (lo + hi) >> 1;
      if ((int)sorted[mid] < k) lo = mid + 1;
      else hi = mid;
    }
    st[k] = lo;
  }
}

// chunk of each edge's destination row, and the row within the chunk's [owner][row] array
__global__ void k_mg_row_chunks(uint32_t* rows, int64_t ne, int64_t nmax_col, int64_t cs, uint32_t* chunk)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t const q = rows[e] / nmax_col, l = rows[e] % nmax_col, k = l / cs;
    chunk[e] = (uint32_t)k;
    rows[e]  = (uint32_t)(q * cs + (l - k * cs));
  }
}

// zero the sums of the listed windows (each 2^wb u64 words)
__global__ void k_clear_windows(unsigned long long* acc, int64_t const* wins, int64_t n, int wb)
{
  int64_t const per = int64_t(1) << wb;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * per; i += (int64_t)gridDim.x * blockDim.x)
    acc[(wins[i >> wb] << wb) + (i & (per - 1))] = 0ull;
}

template <typename V>
__global__ void k_mg_block_coo(V const* src, V const* dst, int64_t ne, int64_t const* voff, int P, int C,
                               int64_t nmax_row, int64_t nmax_col, uint32_t* rows, uint32_t* cols)
{
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    int ou  = mg_owner_of_global((int64_t)src[e], voff, P);
    int ov  = mg_owner_of_global((int64_t)dst[e], voff, P);
    cols[e] = (uint32_t)((ou % C) * nmax_row + ((int64_t)src[e] - voff[ou]));
    rows[e] = (uint32_t)((ov / C) * nmax_col + ((int64_t)dst[e] - voff[ov]));
  }
}

template <typename R>
__global__ void k_weight_or_one(R const* w, int64_t n, double* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = w ? (double)w[i] : 1.0;
}

__global__ void k_scatter_sums(uint32_t const* keys, double const* vals, int64_t n, double* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[keys[i]] = vals[i];
}

template <typename R>
__global__ void k_to_weight(double const* in, int64_t n, R* out)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (R)in[i];
}

template <typename V, typename E, typename R>
__global__ void k_mg_finish_guarded(pr_args<V, E, R> a, bool count_iter)
{
  // after convergence the (stale) sums are allreduced again: never touch a finished state
  if (threadIdx.x == 0 && blockIdx.x == 0 && !a.st->done)
    update_state<V, E, R>(a, (double)a.mg_sums[0] * kSumScaleInv, (double)a.mg_sums[1] * kSumScaleInv, count_iter);
}

template <typename V, typename E, typename R>
mg_pr_block& mg_block(handle_t& h, graph_t& g)
{
  mg_graph_t& mg = *g.mg;
  if (mg.pr_block) return *static_cast<mg_pr_block*>(mg.pr_block.get());
  hipStream_t s = h.stream;
  mg_context& ctx = *h.mg;
  auto blk      = std::make_shared<mg_pr_block>();
  int const P = mg.P, C = mg.C, R_ = mg.R, r = mg.p / C, c = mg.p % C;
  for (int q = 0; q < C; ++q) blk->nmax_row = std::max(blk->nmax_row, mg.voff[r * C + q + 1] - mg.voff[r * C + q]);
  for (int q = 0; q < R_; ++q) blk->nmax_col = std::max(blk->nmax_col, mg.voff[q * C + c + 1] - mg.voff[q * C + c]);
  int64_t const ne = mg.ne, n_cols = C * blk->nmax_row, n_rows = R_ * blk->nmax_col;
  dbuf<int64_t> voff_d(P + 1, s);
  HIP_CHECK(hipMemcpyAsync(voff_d.data(), mg.voff.data(), (P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  dbuf<uint32_t> rows(std::max<int64_t>(ne, 1), s), cols(std::max<int64_t>(ne, 1), s);
  if (ne)
    hipLaunchKernelGGL(k_mg_block_coo<V>, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, mg.src.data<V>(),
                       mg.dst.data<V>(), ne, voff_d.data(), P, C, blk->nmax_row, blk->nmax_col, rows.data(),
                       cols.data());
  CGX_LAUNCH_CHECK();
  // row chunks (overlapped column reduce-scatters, several grid rows only): K =
  // tuning_t::mg_chunks; the default is one chunk = the whole block.  The overlap's
  // device-side concurrency with RCCL has never run on more than one GPU (the
  // rehearsals go through gloo, which host-synchronises every collective), so it
  // stays opt-in; bench.py --gpus N > 1 times K = 4 beside the default and checks
  // the ranks bitwise equal
  int K = 1;
  if (R_ > 1) {
    K = h.tune.mg_chunks > 0 ? h.tune.mg_chunks : 1;
    K = (int)std::min<int64_t>(K, std::max<int64_t>(blk->nmax_col, 1));
  }
  blk->K  = K;
  blk->cs = std::max<int64_t>((blk->nmax_col + K - 1) / K, 1);
  blk->ch.resize(K);
  int64_t const n_rows_k = R_ * blk->cs;
  R const* const w_in    = g.weighted ? mg.w.data<R>() : nullptr;
  (void)n_rows;
  if (K == 1) {  // (cs = nmax_col: the rows are already owner * cs + owner-local row)
    // one grid row: the sums stay on this rank, so 32K windows as on one GPU
    build_push_from_coo<uint32_t, R>(s, rows.data(), cols.data(), w_in, ne, n_rows_k, n_cols, blk->ch[0].pp, h.tune,
                                     false, 0, R_ == 1 && sizeof(R) == 4);
  } else {
    dbuf<uint32_t> chunk(ne, s), chunk_s(ne, s), iv(ne, s), perm(ne, s), rows_s(ne, s), cols_s(ne, s);
    dbuf<R> w_s(w_in ? ne : 1, s);
    hipLaunchKernelGGL(k_mg_row_chunks, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s, rows.data(), ne,
                       blk->nmax_col, blk->cs, chunk.data());
    CGX_LAUNCH_CHECK();
    iota<uint32_t>(iv.data(), ne, 0u, s);
    radix_sort_pairs<uint32_t, uint32_t>(chunk.data(), chunk_s.data(), iv.data(), perm.data(), ne, 0,
                                         bits_for((unsigned long long)K), s);
    gather<uint32_t, uint32_t>(rows_s.data(), rows.data(), perm.data(), ne, s);
    gather<uint32_t, uint32_t>(cols_s.data(), cols.data(), perm.data(), ne, s);
    if (w_in) gather<R, uint32_t>(w_s.data(), w_in, perm.data(), ne, s);
    dbuf<int64_t> st_d(K + 1, s);
    hipLaunchKernelGGL(k_sorted_starts, dim3(1), dim3(64), 0, s, chunk_s.data(), ne, K, st_d.data());
    CGX_LAUNCH_CHECK();
    auto const st = to_host(st_d.data(), K + 1, s);
    for (int k = 0; k < K; ++k)
      build_push_from_coo<uint32_t, R>(s, rows_s.data() + st[k], cols_s.data() + st[k],
                                       w_in ? w_s.data() + st[k] : nullptr, st[k + 1] - st[k], n_rows_k, n_cols,
                                       blk->ch[k].pp, h.tune);
  }
  bool ok = true;
  for (auto const& c_ : blk->ch) ok = ok && c_.pp.ok;
  int64_t bad = ctx.world->host_allreduce<int64_t>(ok ? 0 : 1, CGX_COMM_SUM, s);
  CGX_EXPECTS(bad == 0, CUGRAPH_NOT_IMPLEMENTED, "MG PageRank: a 2D block exceeds the 32-bit push packing");
  // out-weight sums: per-block partials (sorted, deterministic) -> row reduce-scatter
  dbuf<double> part(std::max<int64_t>(n_cols, 1), s), own(std::max<int64_t>(blk->nmax_row, 1), s);
  fill<double>(part.data(), std::max<int64_t>(n_cols, 1), 0.0, s);
  if (ne) {
    dbuf<double> wv(ne, s), wv2(ne, s), sums(ne, s);
    dbuf<uint32_t> k2(ne, s), uk(ne, s);
    hipLaunchKernelGGL(k_weight_or_one<R>, dim3(grid_for(ne, kBlock, 16384)), dim3(kBlock), 0, s,
                       g.weighted ? mg.w.data<R>() : nullptr, ne, wv.data());
    CGX_LAUNCH_CHECK();
    radix_sort_pairs<uint32_t, double>(cols.data(), k2.data(), wv.data(), wv2.data(), ne, 0,
                                       bits_for((unsigned long long)std::max<int64_t>(n_cols - 1, 1)), s);
    dbuf<unsigned long long> nu(1, s);
    size_t tmp = 0;
    HIP_CHECK(rocprim::reduce_by_key(nullptr, tmp, k2.data(), wv2.data(), (size_t)ne, uk.data(), sums.data(),
                                     nu.data(), rocprim::plus<double>(), rocprim::equal_to<uint32_t>(), s));
    buffer t(tmp, s);
    HIP_CHECK(rocprim::reduce_by_key(t.data(), tmp, k2.data(), wv2.data(), (size_t)ne, uk.data(), sums.data(),
                                     nu.data(), rocprim::plus<double>(), rocprim::equal_to<uint32_t>(), s));
    int64_t n_u = (int64_t)to_host_scalar(nu.data(), s);
    hipLaunchKernelGGL(k_scatter_sums, dim3(grid_for(n_u, kBlock, 16384)), dim3(kBlock), 0, s, uk.data(), sums.data(),
                       n_u, part.data());
    CGX_LAUNCH_CHECK();
  }
  ctx.row->reduce_scatter<double>(part.data(), own.data(), (size_t)blk->nmax_row, CGX_COMM_SUM, s);
  int64_t n_own = mg.n_own();
  blk->outw.set_stream(s);
  blk->outw.resize(std::max<int64_t>(n_own, 1) * sizeof(R));
  if (n_own)
    hipLaunchKernelGGL(k_to_weight<R>, dim3(grid_for(n_own, kBlock, 4096)), dim3(kBlock), 0, s, own.data(), n_own,
                       blk->outw.data<R>());
  CGX_LAUNCH_CHECK();
  for (auto& c_ : blk->ch) {  // the windows whose sums are added (several items), cleared after each reduce-scatter
    auto hm = c_.pp.win_multi.empty() ? std::vector<uint8_t>{}
                                      : to_host(c_.pp.win_multi.data<uint8_t>(), (size_t)c_.pp.nwin, s);
    std::vector<int64_t> wl;
    for (int64_t w = 0; w < (int64_t)hm.size(); ++w)
      if (hm[w]) wl.push_back(w);
    c_.nmulti = (int64_t)wl.size();
    c_.multi_wins.resize(std::max<size_t>(wl.size(), 1), s);
    to_device(c_.multi_wins.data(), wl.data(), wl.size(), s);
  }
  if (R_ > 1) {
    HIP_CHECK(hipStreamCreateWithFlags(&blk->comm_stream, hipStreamNonBlocking));
    blk->ev.resize(K + 1);
    for (auto& e : blk->ev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  HIP_CHECK(hipStreamSynchronize(s));
  mg.pr_block = blk;
  return *blk;
}

template <typename V>
__global__ void k_pr_owner(V const* gid, int64_t n, int64_t const* voff, int P, int* dest)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dest[i] = mg_owner_of_global((int64_t)gid[i], voff, P);
}

template <typename V, typename R>
__global__ void k_scatter_owned(V const* gid, R const* val, int64_t n, int64_t lo, double scale, R* owned)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    owned[(int64_t)gid[i] - lo] = (R)((double)val[i] * scale);
}

// user out-weights that are far below the graph's own would let a fixed-point sum
// pass 2 (the push kernel's range); count them
template <typename R>
__global__ void k_count_small_outw(R const* given, R const* actual, int64_t n, int* bad)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (given[i] > R(0) && (double)actual[i] > 1.5 * (double)given[i]) atomicAdd(bad, 1);
}

struct mg_pairs_info {
  double sum        = 0;  // over every rank's values
  int64_t count     = 0;
  int64_t negatives = 0;
};

// (external id, value) pairs given on any rank -> a dense array over this rank's
// owned vertices, value * scale(sum) where given and 0 elsewhere (the reference
// shuffles such pairs to their owners, c_api/pagerank.cpp:115-170 MG branch).
// Collective; errors are raised on every rank alike.
template <typename V, typename R, typename Scale>
mg_pairs_info mg_pairs_to_owned(handle_t& h, graph_t& g, array_view_t const* vv, array_view_t const* vs, R* owned,
                                Scale scale_of)
{
  hipStream_t s  = h.stream;
  mg_graph_t& mg = *g.mg;
  comm_t& comm   = *h.mg->world;
  int const P    = mg.P;
  size_t const n = vv ? vv->size : 0;
  int64_t const n_own = mg.n_own(), lo = mg.voff[mg.p];
  if (n_own) fill<R>(owned, n_own, R(0), s);
  dbuf<V> ids(std::max<size_t>(n, 1), s);
  dbuf<R> vals(std::max<size_t>(n, 1), s);
  if (n) {
    HIP_CHECK(hipMemcpyAsync(ids.data(), vv->data, n * sizeof(V), hipMemcpyDeviceToDevice, s));
    HIP_CHECK(hipMemcpyAsync(vals.data(), vs->data, n * sizeof(R), hipMemcpyDeviceToDevice, s));
  }
  mg_ext_to_global(h, g, ids.data(), n, /*check=*/true);
  mg_pairs_info info;
  double lsum  = 0;
  int64_t lneg = 0;
  for (auto x : to_host(vals.data(), n, s)) {
    lsum += (double)x;
    lneg += x < R(0) ? 1 : 0;
  }
  info.sum       = comm.host_allreduce<double>(lsum, CGX_COMM_SUM, s);
  info.count     = comm.host_allreduce<int64_t>((int64_t)n, CGX_COMM_SUM, s);
  info.negatives = comm.host_allreduce<int64_t>(lneg, CGX_COMM_SUM, s);
  double const scale = scale_of(info);
  // to the owners: sort by owner, exchange, scatter
  dbuf<int64_t> voff_d(P + 1, s);
  HIP_CHECK(hipMemcpyAsync(voff_d.data(), mg.voff.data(), (P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  dbuf<int> dest(std::max<size_t>(n, 1), s), d2(std::max<size_t>(n, 1), s);
  dbuf<int64_t> iv(std::max<size_t>(n, 1), s), perm(std::max<size_t>(n, 1), s);
  dbuf<V> sid(std::max<size_t>(n, 1), s);
  dbuf<R> sval(std::max<size_t>(n, 1), s);
  std::vector<size_t> counts(P, 0), rc;
  if (n) {
    hipLaunchKernelGGL(k_pr_owner<V>, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, ids.data(), (int64_t)n,
                       voff_d.data(), P, dest.data());
    CGX_LAUNCH_CHECK();
    iota<int64_t>(iv.data(), n, 0, s);
    radix_sort_pairs<int, int64_t>(dest.data(), d2.data(), iv.data(), perm.data(), n, 0, bits_for(P), s);
    gather<V, int64_t>(sid.data(), ids.data(), perm.data(), n, s);
    gather<R, int64_t>(sval.data(), vals.data(), perm.data(), n, s);
    for (int q : to_host(d2.data(), n, s)) counts[q]++;
  }
  auto rid  = exchange<V>(comm, sid.data(), counts, rc, s);
  auto rval = exchange<R>(comm, sval.data(), counts, rc, s);
  if (rid.n)
    hipLaunchKernelGGL((k_scatter_owned<V, R>), dim3(grid_for(rid.n, kBlock, 4096)), dim3(kBlock), 0, s, rid.data(),
                       rval.data(), (int64_t)rid.n, lo, scale, owned);
  CGX_LAUNCH_CHECK();
  return info;
}

template <typename V, typename E, typename R>
void mg_pagerank_impl(handle_t& h, graph_t& g, array_view_t const* pow_v, array_view_t const* pow_s,
                      array_view_t const* guess_v, array_view_t const* guess_s, array_view_t const* pers_v,
                      array_view_t const* pers_s, double alpha, double eps, size_t max_iter, bool expensive,
                      centrality_result_t& res)
{
  hipStream_t s   = h.stream;
  mg_context& ctx = *h.mg;
  mg_graph_t& mg  = *g.mg;
  CGX_INPUT(alpha >= 0.0 && alpha <= 1.0, "Invalid input argument: alpha should be in [0.0, 1.0].");
  CGX_INPUT(eps >= 0.0, "Invalid input argument: epsilon should be non-negative.");
  int64_t const n_own = mg.n_own();
  res.vertices        = std::make_unique<device_array_t>((size_t)n_own, g.vertex_type, s);
  if (n_own)
    HIP_CHECK(hipMemcpyAsync(res.vertices->buf.data(), g.number_map.data(), n_own * sizeof(V), hipMemcpyDeviceToDevice,
                             s));
  res.values = std::make_unique<device_array_t>((size_t)n_own, dtype_of<R>(), s);
  h.last_iterations   = 0;
  h.last_hot_ms       = 0;
  h.last_hot_launches = 0;
  if (g.num_vertices == 0) return;
  mg_pr_block& blk = mg_block<V, E, R>(h, g);
  int const C = mg.C, R_ = mg.R;
  int64_t const n1 = std::max<int64_t>(n_own, 1);
  auto unit  = [](mg_pairs_info const&) { return 1.0; };
  auto prob  = [](mg_pairs_info const& i) { return i.sum > 0.0 ? 1.0 / i.sum : 0.0; };

  // precomputed out-weight sums (pagerank_impl.cuh:64-87)
  dbuf<R> outw_user;
  R const* outw = blk.outw.data<R>();
  if (pow_v) {
    outw_user.resize(n1, s);
    auto info = mg_pairs_to_owned<V, R>(h, g, pow_v, pow_s, outw_user.data(), unit);
    CGX_INPUT(!expensive || info.negatives == 0,
              "Invalid input argument: outgoing edge weight sum values should be non-negative.");
    dbuf<int> bad(1, s);
    fill<int>(bad.data(), 1, 0, s);
    if (n_own)
      hipLaunchKernelGGL(k_count_small_outw<R>, dim3(grid_for(n_own, kBlock, 4096)), dim3(kBlock), 0, s,
                         outw_user.data(), blk.outw.data<R>(), n_own, bad.data());
    CGX_LAUNCH_CHECK();
    int64_t nbad = ctx.world->host_allreduce<int64_t>((int64_t)to_host_scalar(bad.data(), s), CGX_COMM_SUM, s);
    CGX_EXPECTS(nbad == 0, CUGRAPH_NOT_IMPLEMENTED,
                "multi-GPU PageRank: precomputed out-weight sums below 2/3 of the graph's own are not supported");
    outw = outw_user.data();
  }
  // personalisation coefficients value / sum(values)
  dbuf<R> pers;
  bool personalized = false;
  if (pers_v || pers_s) {
    CGX_INPUT(pers_v && pers_s && pers_v->size == pers_s->size,
              "Invalid input argument: personalization vertices and values must be given together.");
    pers.resize(n1, s);
    auto info = mg_pairs_to_owned<V, R>(h, g, pers_v, pers_s, pers.data(), prob);
    CGX_INPUT(!expensive || info.negatives == 0,
              "Invalid input argument: peresonalization values should be non-negative.");
    if (info.count > 0) {
      CGX_INPUT(info.sum > 0.0, "Invalid input argument: sum of personalization valuese should be positive.");
      personalized = true;
    }
  }

  R* pr = res.values->buf.data<R>();
  if (guess_v || guess_s) {  // initial guess, normalised to sum 1
    CGX_INPUT(guess_v && guess_s, "Invalid input argument: initial guess vertices and values must be given together.");
    auto info = mg_pairs_to_owned<V, R>(h, g, guess_v, guess_s, pr, prob);
    CGX_INPUT(!expensive || info.negatives == 0,
              "Invalid input argument: initial guess values should be non-negative.");
    CGX_INPUT(info.sum > 0.0, "Invalid input argument: sum of the PageRank initial guess values should be positive.");
  } else {
    fill<R>(pr, std::max<int64_t>(n_own, 0), (R)(R(1.0) / (R)g.num_vertices), s);
  }
  dbuf<R> x_send(std::max<int64_t>(blk.nmax_row, 1), s), x_row(std::max<int64_t>(C * blk.nmax_row, 1), s);
  fill<R>(x_send.data(), std::max<int64_t>(blk.nmax_row, 1), R(0), s);
  int const K         = blk.K;
  int64_t const n_accown = std::max<int64_t>(K * blk.cs, 1);  // chunk k's reduce-scatter lands at k cs
  dbuf<unsigned long long> acc_own(n_accown, s);
  fill<unsigned long long>(acc_own.data(), n_accown, 0ull, s);
  dbuf<double> partials(2 * 4096, s);
  dbuf<unsigned long long> sums(2, s);
  dbuf<pr_state> st(1, s);
  HIP_CHECK(hipMemsetAsync(st.data(), 0, sizeof(pr_state), s));

  pr_args<V, E, R> a{};
  a.pr        = pr;
  a.outw      = outw;
  a.pers      = personalized ? pers.data() : nullptr;
  a.alpha     = alpha;
  a.eps       = eps;
  a.max_iter  = (int)std::min<size_t>(max_iter, (size_t)INT32_MAX);
  a.nv        = n_own;
  a.nv_global = g.num_vertices;
  a.partials  = partials.data();
  a.st        = st.data();
  a.mg_sums   = sums.data();
  a.x_in      = x_row.data();
  a.x_out     = x_send.data();
  // fp32 packed push: x~ travels (allgather) and is read as enc_fixed words, as on one
  // GPU -- when every chunk with edges has the packed format (the words are shared)
  bool all_packed = true;
  for (auto const& c_ : blk.ch) all_packed = all_packed && (c_.pp.packed || c_.pp.nunits == 0);
  a.enc = all_packed && std::is_same<R, float>::value && h.tune.pr_enc;
  int const nblk_init = (int)grid_for(std::max<int64_t>(n_own, 1), kBlock, 1024);
  hipLaunchKernelGGL((k_pr_init<V, E, R>), dim3(nblk_init), dim3(kBlock), 0, s, a);
  CGX_LAUNCH_CHECK();
  ctx.world->allreduce<unsigned long long>(sums.data(), sums.data(), 2, CGX_COMM_SUM, s);
  hipLaunchKernelGGL((k_mg_finish<V, E, R>), dim3(1), dim3(64), 0, s, a, false);
  CGX_LAUNCH_CHECK();
  if (max_iter == 0) fail(CUGRAPH_UNKNOWN_ERROR, "PageRank failed to converge.");

  // R > 1: the block's sums go through the column reduce-scatter into acc_own, which
  // the apply reads and leaves (the next reduce-scatter overwrites it); afterwards only
  // the windows summed by several items are cleared (stored windows are overwritten).
  // With K > 1 row chunks the chunks are pushed one after another and chunk k's
  // reduce-scatter (with its clears and queue-head reset) runs on the block's comm
  // stream, after an event, while the push works on chunk k + 1; the apply waits for
  // the last one.
  // R = 1 (one grid row): the block's sums are already the owner's; as on one GPU the
  // apply reads them in place and clears the added windows -- or, with 16K windows, the
  // push applies each window itself (fused_finish) and leaves its (diff, dangling) in
  // mg_sums
  bool const col_reduce = R_ > 1;
  hipStream_t const cst = K > 1 ? blk.comm_stream : s;
  std::vector<push_args<V, E, R>> spk(K);
  std::vector<int> nblk_push(K);
  std::vector<decltype(push_kernel<V, E, R>(blk.ch[0].pp, false, false))> pker(K);
  std::vector<char> calibrating(K, 0);
  for (int k = 0; k < K; ++k) {
    pr_push_t& pp = blk.ch[k].pp;
    spk[k].a      = a;
    set_queue_args(spk[k], pp, s);
    spk[k].win_bits      = pp.win_bits;
    nblk_push[k]    = spk[k].nitems && pp.nunits ? push_blocks(pp.win_bits) : 0;
    // the push's persistent blocks fill every CU (LDS or registers), so an RCCL
    // kernel launched beside it would wait for the push to end: with overlapped
    // reduce-scatters the push leaves kCommCUs CUs free for them
    if (col_reduce && K > 1 && nblk_push[k])
      nblk_push[k] -= kCommCUs * (pp.win_bits >= 14 ? 1 : 2);  // (blocks per CU)
    pker[k]         = push_kernel<V, E, R>(pp, g.weighted, a.enc != 0);
    // measured-cost queues (calibrate_queues), per rank and chunk: no collective
    calibrating[k] = nblk_push[k] && calibration_wanted(pp, h.tune);
    if (calibrating[k]) {
      pp.item_ticks.set_stream(s);
      pp.item_ticks.resize(pp.nitems * sizeof(uint32_t));
      HIP_CHECK(hipMemsetAsync(pp.item_ticks.data(), 0, pp.nitems * sizeof(uint32_t), s));
      pp.calib = 1;
    } else if (pp.calib == 0) {
      pp.calib = 2;
    }
  }
  push_args<V, E, R> sap = spk[0];
  sap.acc       = col_reduce ? acc_own.data() : spk[0].acc;
  sap.keep_acc  = col_reduce ? 1 : 0;
  sap.win_multi = col_reduce ? nullptr : blk.ch[0].pp.win_multi.data<uint8_t>();
  if (K > 1) sap.tile_ctr = nullptr;  // (every chunk's heads are reset on the comm stream)
  int const nblk_apply = (int)grid_for(std::max<int64_t>(n_own, 1), kBlock, 512);
  bool const fused     = !col_reduce && K == 1 && nblk_push[0] && fuse_apply(blk.ch[0].pp, h.tune);
  if (fused) {
    spk[0].fuse = 1;
    spk[0].nhub = h.tune.pr_hub ? C * blk.nmax_row : 0;  // hub x~ in LDS (row-local source ids)
  }

  size_t launched = 0;
  std::vector<hipEvent_t> ev;
  pr_state hst{};
  pr_state* hpin = h.pinned_as<pr_state>();
  {
    // (collectives run even in the no-op iterations after convergence: next_chunk;
    // one pair of pooled events per chunk, as on one GPU)
    while (true) {
      if (h.profiling) {
        ev.push_back(h.event(ev.size()));
        ev.push_back(h.event(ev.size()));
        HIP_CHECK(hipEventRecord(ev[ev.size() - 2], s));
      }
      int const chunk = next_chunk(hst, eps, a.max_iter);
      for (int i = 0; i < chunk; ++i) {
        ctx.row->allgather<R>(x_send.data(), x_row.data(), (size_t)blk.nmax_row, s);
        int const parity = (int)(launched & 1);
        for (int k = 0; k < K; ++k) {
          mg_chunk& ck     = blk.ch[k];
          auto& sp         = spk[k];
          sp.item_ticks    = calibrating[k] && launched == 0 ? ck.pp.item_ticks.data<uint32_t>() : nullptr;
          sp.parity        = parity;
          if (nblk_push[k]) hipLaunchKernelGGL(pker[k], dim3(nblk_push[k]), dim3(kPushThreads), 0, s, sp);
          CGX_LAUNCH_CHECK();
          if (!col_reduce) continue;
          if (K > 1) {
            HIP_CHECK(hipEventRecord(blk.ev[k], s));
            HIP_CHECK(hipStreamWaitEvent(cst, blk.ev[k], 0));
          }
          ctx.col->reduce_scatter<unsigned long long>(sp.acc, acc_own.data() + k * blk.cs, (size_t)blk.cs,
                                                      CGX_COMM_SUM, cst);
          if (ck.nmulti)
            hipLaunchKernelGGL(k_clear_windows, dim3(grid_for(ck.nmulti << ck.pp.win_bits, kBlock, 8192)),
                               dim3(kBlock), 0, cst, sp.acc, ck.multi_wins.data(), ck.nmulti, ck.pp.win_bits);
          CGX_LAUNCH_CHECK();
          if (K > 1 && sp.tile_ctr)  // this parity's heads, for the iteration after next
            HIP_CHECK(hipMemsetAsync(sp.tile_ctr + parity * kQueues * kCtrStride, 0,
                                     kQueues * kCtrStride * sizeof(unsigned int), cst));
        }
        if (col_reduce && K > 1) {
          HIP_CHECK(hipEventRecord(blk.ev[K], cst));
          HIP_CHECK(hipStreamWaitEvent(s, blk.ev[K], 0));
        }
        ++launched;
        sap.parity = parity;
        if (!fused) hipLaunchKernelGGL((k_pr_apply<V, E, R>), dim3(nblk_apply), dim3(kBlock), 0, s, sap);
        CGX_LAUNCH_CHECK();
        ctx.world->allreduce<unsigned long long>(sums.data(), sums.data(), 2, CGX_COMM_SUM, s);
        hipLaunchKernelGGL((k_mg_finish_guarded<V, E, R>), dim3(1), dim3(64), 0, s, a, true);
        CGX_LAUNCH_CHECK();
      }
      if (h.profiling) HIP_CHECK(hipEventRecord(ev.back(), s));
      HIP_CHECK(hipMemcpyAsync(hpin, st.data(), sizeof(pr_state), hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
      hst = *hpin;
      for (int k = 0; k < K; ++k) {
        if (!calibrating[k]) continue;
        calibrate_queues(s, blk.ch[k].pp, h.tune);
        for (int q = 0; q <= kQueues; ++q) spk[k].qoff[q] = blk.ch[k].pp.qoff[q];
        calibrating[k] = 0;
      }
      if (hst.done) break;
    }
  }
  h.last_iterations = (size_t)hst.iter;
  if (h.profiling) {
    double tot = 0;
    for (size_t i = 0; i + 1 < ev.size(); i += 2) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
      tot += ms;
    }
    h.last_hot_ms       = tot;
    h.last_hot_launches = std::max<size_t>((size_t)hst.iter, 1);
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

namespace cgx {
void mg_run_pagerank(handle_t& h, graph_t& g, array_view_t const* pow_v, array_view_t const* pow_s,
                     array_view_t const* guess_v, array_view_t const* guess_s, array_view_t const* pers_v,
                     array_view_t const* pers_s, double alpha, double eps, size_t max_iter, bool expensive,
                     centrality_result_t& res)
{
  CGX_EXPECTS(h.mg != nullptr, CUGRAPH_INVALID_HANDLE, "multi-GPU graph used with a single-GPU resource handle");
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    mg_pagerank_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(
      h, g, pow_v, pow_s, guess_v, guess_s, pers_v, pers_s, alpha, eps, max_iter, expensive, res);
  });
}
}  // namespace cgx
