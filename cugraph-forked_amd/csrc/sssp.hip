// Single-source shortest paths on the GPU: near-far buckets (Davidson et al., the
// reference's scheme) with light / heavy edges (Meyer and Sanders' delta-stepping).
//
// Reference: cpp/src/traversal/sssp_impl.cuh:79-270 (+ c_api/sssp.cpp:60-145):
// distances start at numeric_limits<weight_t>::max(), a relaxation dist[u] + w is
// kept only if it is < min(cutoff, dist[v]) (e_op :49-72); the frontier is split
// into near / far piles by a threshold that grows by delta (:143-157, :235-262).
// Every vertex there relaxes all its edges each time it is processed; on RMAT-24
// with the bench's weights that is 3-6 E of relaxations per traversal (the compiled
// restatement counts 3.0 E at RMAT-20).  Here a bucket [lo, thr) relaxes only its
// vertices' light edges (w < delta) while it fills, then each of its vertices' heavy
// edges once, when the bucket is done: a heavy edge lands at d + w >= lo + delta =
// thr (rounding is monotone and thr is computed as the same fp sum), outside the
// bucket, so nothing the bucket settles changes by it.  The distances are the same
// fixed point (the minimum over paths of the left-folded weight_t sums below the
// cutoff); the order of work differs.
//
// Every round runs on the device with no host read in between:
//  * a frontier list lives in an edge space: each appended vertex gets a slot and
//    the start of its edges from one 64-bit counter, (slots << eb) | edges, added
//    once per wave stage, and the slot holding the start of every 2048-edge chunk is
//    recorded;
//  * k_relax: persistent blocks take 2048-edge chunks of the near list's light edges
//    (light round) or the bucket list's heavy edges (heavy round) -- a hub's 400K
//    edges spread over the grid, a chunk of low-degree vertices holds up to 2048 of
//    them -- find each position's vertex by a max-scan of the chunk's slot starts in
//    LDS, load 8 edges a thread coalesced with every load issued before the first
//    compare, and relax with non-returning atomicMin on the distance's bit pattern
//    (non-negative IEEE values order like integers), marking every improved vertex
//    in a changed bitmap;
//  * k_split: the changed bitmap (V / 8 bytes, read and cleared whole): below thr ->
//    the next near list and (once per bucket) the bucket list; otherwise the vertex
//    is in the far set, whose smallest distance is kept;
//  * k_pull: a dense list (its edges above a quarter of its part's) is relaxed as a
//    pull over the part in order instead: rows above the round's floor take the
//    smallest candidate from frontier sources (the list's bitmap), one atomic per
//    row and chunk -- the part read coalesced, only the frontier's distances
//    gathered (symmetric graphs);
//  * k_sssp_ctl: the next round -- light while the near list
//    fills, one heavy round when it empties, then a far split (split_bucket,
//    :235-262) with the threshold raised past the smallest far distance (the
//    reference raises it by delta until the near bucket fills: the same buckets,
//    fewer empty passes);
//  * k_far_split: a dense pass over the distances -- [old, thr) to the near list, the
//    far set's minimum -- instead of a pile of ids (the reference's far bucket: each
//    split re-reads every far entry in arbitrary order, 0.3-0.5 ms a split at
//    RMAT-24).  Termination is k_sssp_ctl's (nothing left: the round after the last
//    far split), push or pull each relax kernel's own reading of the list's size
//    (a one-thread finishing kernel per round was 4-5 us of each ~100 rounds).
// The state lives in one device block; the host enqueues kChunkRounds rounds and
// reads the state once per chunk (rounds after termination return at once).  Every
// grid is fixed and grid-strides over device-side counts.  The light-first copy of
// the adjacency is built once per graph and delta (adjacency_t::sssp_*).
// Predecessors are resolved once at the end by a pull over the in-edges (sorted
// ascending): the first -- smallest-id -- in-neighbour u with dist[u] + w == dist[v]
// (deterministic; every reference golden vector satisfies it).
#include "capi.hpp"
#include "prims.hpp"

#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <limits>

namespace cgx {

namespace {

constexpr int kChunk       = 2048;  // edges per relax work item: 256 threads x 8
constexpr int kPerThread   = kChunk / 256;
constexpr int kRelaxGrid   = 1280;  // persistent relax blocks (32 KB of LDS: 5 per CU)
constexpr int kPullGrid    = 1024;  // persistent pull blocks (2048: 4.6 vs 4.2 ms of pulls per RMAT-24 traversal)
constexpr int kSplitGrid   = 1024;
constexpr int kStage       = 128;   // staged entries per wave and list
constexpr int kChunkRounds = 8;     // rounds enqueued per host read
// delta = kDeltaScale * average weight / average degree (tuning_t::sssp_delta)
constexpr double kDeltaScale = 8.0;
// a list whose edges exceed its part's / kPullDiv is relaxed by a pull (tuning_t::sssp_pull)
constexpr int kPullDiv = 4;

template <typename W>
struct bits_of;
template <>
struct bits_of<float> {
  using type  = int;
  using utype = unsigned int;
};
template <>
struct bits_of<double> {
  using type  = long long;
  using utype = unsigned long long;
};

enum : int { kLight = 0, kHeavy = 1 };

// device-side state of one SSSP call (counters 128 B apart: same-address atomics of
// different counters do not share a line)
template <typename W>
struct sssp_state {
  unsigned long long nq[2][16];   // near lists by parity: (slots << eb) | light edges
  unsigned long long nr[2][16];   // bucket lists (the bucket's vertices): (slots << eb) | heavy edges
  typename bits_of<W>::utype minfar;  // smallest distance at or past thr noted since the last far split
  W thr, old, delta;
  int fs;     // this round splits the far set
  int phase;  // the next relax: kLight (near list nq[P]) or kHeavy (bucket list nr[hl])
  int pad0;
  int rp;     // bucket list receiving this bucket's vertices
  int hl;     // bucket list a heavy round relaxes
  int epoch;  // a vertex joins bucket list rp once per epoch (stamp)
  int done;
  int bad;    // the source is not a vertex
  unsigned long long rounds;  // relax rounds with work
  unsigned long long work[16][16];  // CGX_SSSP_TRACE partials: [p][0] light edges, [p][1] vertices improved,
                                    // [p][2] distance atomics, [p][3] heavy edges
};

// one frontier list in an edge space: vertex, first edge in the list's edge space,
// and the slot holding edge c * kChunk
template <typename V>
struct flist {
  V* q;
  int64_t* ep;
  int64_t* cs;
};

// one part of the adjacency (the light or the heavy edges of every row) as a CSR,
// with the row holding edge c * kChunk of the part (the pull's chunk starts)
template <typename V, typename E, typename W>
struct part_t {
  E const* off;
  V const* idx;
  W const* w;
  int64_t const* crow;
  int64_t ne;
};

template <typename V, typename E, typename W>
struct sssp_args {
  E const* off;          // the graph's rows (degrees)
  part_t<V, E, W> pt[2]; // kLight: edges with w < delta, kHeavy: the rest
  uint32_t* fbits[4];    // frontier bitmaps of the lists: near by parity (0, 1), bucket by index (2, 3)
  int pull_div;          // a list whose edges exceed its part's / pull_div is relaxed by a pull (0: never)
  W* dist;
  int* stamp;         // bucket-list epoch of each vertex
  W cutoff;
  flist<V> near[2];    // by parity
  flist<V> bucket[2];  // by index (rp / hl)
  uint32_t* cbits;     // the round's changed vertices (a bit each), cleared by k_split
  sssp_state<W>* st;
  int64_t nv;
  int eb;     // edge field bits of the list counters
  int trace;  // CGX_SSSP_TRACE: count the work (debug output only)
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// A wave's appends to one frontier list (vertex, edges) staged in its own LDS slice
// and moved out with one 64-bit atomic per full slice: slots and edge starts come
// from the same add, so both are monotonic in slot order (every wave appending with
// its own atomic to one list counter serialised at the memory side: the first
// version's changed list took 148 ms per RMAT-24 traversal that way).  Every call
// is made by the whole wave (wave-uniform control flow).
template <typename V>
struct edge_stage {
  V* vb;
  uint32_t* db;
  int n;
  __device__ __forceinline__ void flush(flist<V> const& L, unsigned long long* ctr, int eb)
  {
    if (n == 0) return;
    __builtin_amdgcn_wave_barrier();
    int const lane     = lane_id();
    constexpr int kPer = kStage / 64;  // entries per lane, contiguous
    unsigned long long d[kPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      int const i = lane * kPer + k;
      d[k]        = i < n ? (unsigned long long)db[i] : 0ull;
      sum += d[k];
    }
    unsigned long long pre = sum;  // inclusive wave scan of the lane sums
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      unsigned long long const y = __shfl_up(pre, o, 64);
      if (lane >= o) pre += y;
    }
    unsigned long long const total = __shfl(pre, 63, 64);
    pre -= sum;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(ctr, ((unsigned long long)n << eb) | total);
    base                = __shfl(base, 0, 64);
    int64_t const slot0 = (int64_t)(base >> eb);
    int64_t e           = (int64_t)(base & ((1ull << eb) - 1ull)) + (int64_t)pre;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      int const i = lane * kPer + k;
      if (i < n) {
        int64_t const slot = slot0 + i;
        L.q[slot]          = vb[i];
        L.ep[slot]         = e;
        for (int64_t c = (e + kChunk - 1) / kChunk; c * kChunk < e + (int64_t)d[k]; ++c) L.cs[c] = slot;
        e += (int64_t)d[k];
      }
    }
    __builtin_amdgcn_wave_barrier();
    n = 0;
  }
  __device__ __forceinline__ void push(flist<V> const& L, unsigned long long* ctr, int eb, bool take, V v,
                                       uint32_t deg)
  {
    unsigned long long const m = __ballot(take);
    int const lane             = lane_id();
    if (take) {
      int const i = n + __popcll(m & ((1ull << lane) - 1ull));
      vb[i]       = v;
      db[i]       = deg;
    }
    n += __popcll(m);
    if (n > kStage - 64) flush(L, ctr, eb);
  }
};

// A wave's stages of the two lists a split fills (LDS slices of the block)
template <typename V>
struct split_stages {
  edge_stage<V> nst, bst;
};

#define CGX_SPLIT_LDS(V)                                \
  __shared__ V s_v[4][kStage], s_b[4][kStage];          \
  __shared__ uint32_t s_dn[4][kStage], s_db[4][kStage]; \
  int const wv_ = threadIdx.x >> 6;                     \
  split_stages<V> sg{{s_v[wv_], s_dn[wv_], 0}, {s_b[wv_], s_db[wv_], 0}}

// The smallest of every thread's v into st->minfar: one atomic per block (every
// thread of the block calls)
template <typename W>
__device__ __forceinline__ void block_min_far(sssp_state<W>* st, W v)
{
  using U = typename bits_of<W>::utype;
  __shared__ W s_m[4];
  for (int o = 32; o > 0; o >>= 1) {
    W const y = __shfl_xor(v, o, 64);
    v         = y < v ? y : v;
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) v = s_m[w] < v ? s_m[w] : v;
    if (v < std::numeric_limits<W>::max()) atomicMin(&st->minfar, *reinterpret_cast<U const*>(&v));
  }
}

// A vertex at distance d with `light` light and `heavy` heavy edges leaving a split:
// below thr -> the next near list (its light edges) and, once per bucket epoch, the
// bucket list (its heavy edges, relaxed when the bucket is done); otherwise it is
// in the far set (every reached vertex at or past thr), whose smallest distance is
// kept in fmin.  Vertices without edges go nowhere.
template <typename V, typename E, typename W>
__device__ __forceinline__ void route(sssp_args<V, E, W> const& a, split_stages<V>& sg, int Q, bool have, V v, W d,
                                      W thr, uint32_t light, uint32_t heavy, W& fmin)
{
  sssp_state<W>* st = a.st;
  bool const live   = have && light + heavy > 0;
  bool const near   = live && d < thr;
  bool to_bucket    = false;
  if (near && heavy > 0) to_bucket = atomicExch(a.stamp + v, st->epoch) != st->epoch;
  if (live && !near) fmin = d < fmin ? d : fmin;
  int const rp = st->rp;
  if (a.pull_div) {  // the lists' frontier bits (a pull reads them)
    if (near && light > 0) atomicOr(a.fbits[Q] + (v >> 5), 1u << (uint32_t(v) & 31u));
    if (to_bucket) atomicOr(a.fbits[2 + rp] + (v >> 5), 1u << (uint32_t(v) & 31u));
  }
  sg.nst.push(a.near[Q], &st->nq[Q][0], a.eb, near && light > 0, v, light);
  sg.bst.push(a.bucket[rp], &st->nr[rp][0], a.eb, to_bucket, v, heavy);
}

template <typename V, typename E, typename W>
__device__ __forceinline__ void route_flush(sssp_args<V, E, W> const& a, split_stages<V>& sg, int Q)
{
  sssp_state<W>* st = a.st;
  int const rp      = st->rp;
  sg.nst.flush(a.near[Q], &st->nq[Q][0], a.eb);
  sg.bst.flush(a.bucket[rp], &st->nr[rp][0], a.eb);
}

// Whether round P's list is relaxed by a pull: its edges above the part's / pull_div
// (a dense round: a pull reads the part in order and gathers only the frontier
// sources' distances; a push gathers every destination's).  k_relax and k_pull
// decide it alike from the same state words (neither changes them before reading).
template <typename V, typename E, typename W>
__device__ __forceinline__ bool round_pulls(sssp_args<V, E, W> const& a, sssp_state<W> const* st, int P)
{
  bool const hvy               = st->phase == kHeavy;
  unsigned long long const c0  = hvy ? st->nr[st->hl][0] : st->nq[P][0];
  unsigned long long const tot = c0 & ((1ull << a.eb) - 1ull);
  return a.pull_div > 0 && tot * (unsigned long long)a.pull_div > (unsigned long long)a.pt[hvy ? kHeavy : kLight].ne;
}

// One relax round over a list's edge space, chunk by chunk: the near list's light
// edges (kLight) or the bucket list's heavy edges (kHeavy).  Block 0 clears the
// next near counter.
template <typename V, typename E, typename W>
__global__ __launch_bounds__(256) void k_relax(sssp_args<V, E, W> a, int round)
{
  using B           = typename bits_of<W>::type;
  sssp_state<W>* st = a.st;
  if (st->done) return;
  int const P = round & 1, Q = P ^ 1;
  int const tid   = threadIdx.x;
  bool const hvy  = st->phase == kHeavy;
  int const hl    = st->hl;
  bool const pulls = round_pulls(a, st, P);
  if (blockIdx.x == 0 && tid == 0) st->nq[Q][0] = 0;
  if (pulls) return;  // (k_pull relaxes this round)
  part_t<V, E, W> const pt    = a.pt[hvy ? kHeavy : kLight];
  flist<V> const L            = hvy ? a.bucket[hl] : a.near[P];
  unsigned long long const c0 = hvy ? st->nr[hl][0] : st->nq[P][0];
  int64_t const n   = (int64_t)(c0 >> a.eb);
  int64_t const tot = (int64_t)(c0 & ((1ull << a.eb) - 1ull));
  int64_t const nch = (tot + kChunk - 1) / kChunk;
  __shared__ int64_t s_ob[kChunk + 1];  // per slot of the chunk: first edge of the row's part - its edge start
  __shared__ W s_du[kChunk + 1];        // per slot: dist[u]
  __shared__ int s_slot[kChunk];        // per position: the slot (a max-scan of the slot starts)
  __shared__ int s_wmax[4];
  unsigned long long my_e = 0, my_a = 0;
  for (int64_t c = blockIdx.x; c < nch; c += gridDim.x) {
    int64_t const t0 = c * kChunk;
    int64_t const t1 = t0 + kChunk < tot ? t0 + kChunk : tot;
    int64_t const s0 = L.cs[c];
    int64_t const s1 = c + 1 < nch ? L.cs[c + 1] : n - 1;
    int const ns     = (int)(s1 - s0 + 1);  // <= kChunk + 1: every slot holds at least one edge
    for (int p = tid; p < kChunk; p += 256) s_slot[p] = 0;
    __syncthreads();
    for (int i = tid; i < ns; i += 256) {
      V const u        = L.q[s0 + i];
      int64_t const e0 = L.ep[s0 + i];
      s_ob[i]          = (int64_t)pt.off[u] - e0;
      s_du[i]          = a.dist[u];
      int64_t const p  = e0 - t0;
      if (i > 0 && p < kChunk) s_slot[p] = i;  // (slot 0 starts at or before t0)
    }
    __syncthreads();
    {  // inclusive max-scan: thread tid owns positions [8 tid, 8 tid + 8)
      int m = 0, loc[kPerThread];
#pragma unroll
      for (int k = 0; k < kPerThread; ++k) {
        int const x = s_slot[tid * kPerThread + k];
        m           = x > m ? x : m;
        loc[k]      = m;
      }
      int pre = m;  // inclusive wave max-scan of the thread maxima
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        int const y = __shfl_up(pre, o, 64);
        if ((tid & 63) >= o) pre = y > pre ? y : pre;
      }
      if ((tid & 63) == 63) s_wmax[tid >> 6] = pre;
      int excl = __shfl_up(pre, 1, 64);
      if ((tid & 63) == 0) excl = 0;
      __syncthreads();
      for (int w = 0; w < (tid >> 6); ++w) excl = s_wmax[w] > excl ? s_wmax[w] : excl;
#pragma unroll
      for (int k = 0; k < kPerThread; ++k) s_slot[tid * kPerThread + k] = loc[k] > excl ? loc[k] : excl;
    }
    __syncthreads();
    // 8 edges a thread, position k * 256 + tid: coalesced loads of each row
    V v[kPerThread];
    W nd[kPerThread];
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) {
      int const p     = k * 256 + tid;
      int64_t const t = t0 + p;
      v[k]            = V(-1);
      nd[k]           = W(0);
      if (t < t1) {
        int const j     = s_slot[p];
        int64_t const e = s_ob[j] + t;
        v[k]            = pt.idx[e];
        nd[k]           = s_du[j] + pt.w[e];
      }
    }
    W dv[kPerThread];
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) dv[k] = v[k] >= 0 ? a.dist[v[k]] : W(0);
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) {
      if (v[k] >= 0 && nd[k] < a.cutoff && nd[k] < dv[k]) {
        atomicMin(reinterpret_cast<B*>(a.dist + v[k]), *reinterpret_cast<B const*>(&nd[k]));
        atomicOr(a.cbits + (v[k] >> 5), 1u << (uint32_t(v[k]) & 31u));
        ++my_a;
      }
    }
    if (tid == 0) my_e += (unsigned long long)(t1 - t0);
    __syncthreads();
  }
  if (a.trace) {
    for (int o = 32; o > 0; o >>= 1) {
      my_e += __shfl_xor(my_e, o, 64);
      my_a += __shfl_xor(my_a, o, 64);
    }
    int const p = (int)((blockIdx.x * 4 + (tid >> 6)) & 15);
    if ((tid & 63) == 0 && my_e) atomicAdd(&st->work[p][hvy ? 3 : 0], my_e);
    if ((tid & 63) == 0 && my_a) atomicAdd(&st->work[p][2], my_a);
  }
}

// The round's changed bitmap (cleared as it is read) through route().
template <typename V, typename E, typename W>
__global__ __launch_bounds__(256) void k_split(sssp_args<V, E, W> a, int round)
{
  sssp_state<W>* st = a.st;
  if (st->done) return;
  int const P = round & 1, Q = P ^ 1;
  W const thr = st->thr;
  uint32_t* const Fu = a.pull_div ? a.fbits[st->phase == kHeavy ? 2 + st->hl : P] : nullptr;
  CGX_SPLIT_LDS(V);
  int64_t const nwords        = (a.nv + 31) >> 5;
  unsigned long long improved = 0;
  W fmin                      = std::numeric_limits<W>::max();
  for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < nwords; base += (int64_t)gridDim.x * blockDim.x) {
    int64_t const wi = base + threadIdx.x;
    uint32_t word    = wi < nwords ? a.cbits[wi] : 0u;
    if (word) a.cbits[wi] = 0u;
    if (Fu && wi < nwords && Fu[wi]) Fu[wi] = 0u;  // the relaxed list's frontier bits
    improved += (unsigned long long)__popc(word);
    while (__any(word != 0)) {
      bool const have = word != 0;
      V v             = 0;
      if (have) {
        v = (V)(wi * 32 + (__ffs(word) - 1));
        word &= word - 1;
      }
      uint32_t light = 0, heavy = 0;
      W d = W(0);
      if (have) {
        light = (uint32_t)(a.pt[kLight].off[v + 1] - a.pt[kLight].off[v]);
        heavy = (uint32_t)(a.pt[kHeavy].off[v + 1] - a.pt[kHeavy].off[v]);
        d     = a.dist[v];
      }
      route(a, sg, Q, have, v, d, thr, light, heavy, fmin);
    }
  }
  route_flush(a, sg, Q);
  block_min_far(st, fmin);
  if (a.trace) {
    for (int o = 32; o > 0; o >>= 1) improved += __shfl_xor(improved, o, 64);
    if ((threadIdx.x & 63) == 0 && improved) atomicAdd(&st->work[(blockIdx.x * 4 + wv_) & 15][1], improved);
  }
}

// One thread, after the split: what the next round does.
//  * the next near list is not empty -> a light round;
//  * else, after light rounds, a bucket list with heavy edges -> a heavy round (the
//    list is swapped out: vertices that join later start the next epoch's list);
//  * else the bucket is done: with a far set (a distance noted at or past thr), a far
//    split over the distances with the threshold past the smallest far distance
//    (split_bucket, :235-262; the reference raises it by delta until the near bucket
//    fills).
template <typename W>
__global__ void k_sssp_ctl(sssp_state<W>* st, int round, int eb)
{
  if (st->done) return;
  using U     = typename bits_of<W>::utype;
  U const inf = ~U(0) >> 1;  // above every non-negative value's bits
  int const P = round & 1, Q = P ^ 1;
  unsigned long long const did = st->phase == kHeavy ? st->nr[st->hl][0] : st->nq[P][0];
  st->rounds += (did >> eb) > 0;
  st->fs = 0;
  if ((st->nq[Q][0] >> eb) > 0) {
    st->phase = kLight;
  } else if (st->phase == kLight && (st->nr[st->rp][0] >> eb) > 0) {
    st->phase = kHeavy;
    st->hl    = st->rp;
    st->rp ^= 1;
    st->nr[st->rp][0] = 0;
    st->epoch += 1;
  } else {
    st->phase = kLight;
    if (st->minfar != inf) {
      U const mb  = st->minfar;
      W const mf  = *reinterpret_cast<W const*>(&mb);
      W const old = st->thr;
      W thr       = old + st->delta;
      if (!(mf < thr)) thr = mf + st->delta;
      st->old    = old;
      st->thr    = thr;
      st->fs     = 1;
      st->minfar = inf;  // k_far_split notes the far set's exact minimum past the new thr
      st->epoch += 1;
    } else {
      // no near list, no bucket waiting for its heavy round, no far set: done (seen one
      // round after the far split that emptied the far set: that round's launches
      // found nothing to do)
      st->done = 1;
    }
  }
}

// The far split, dense: every vertex with old <= dist < thr (unprocessed: the
// buckets below old are done) through route(); the smallest distance at or past thr
// (the rest of the far set) noted exactly.  One pass over the distances in id order
// (coalesced) instead of a pile of ids in arbitrary order.
template <typename V, typename E, typename W>
__global__ __launch_bounds__(256) void k_far_split(sssp_args<V, E, W> a, int round)
{
  sssp_state<W>* st = a.st;
  if (st->done || !st->fs) return;
  int const Q = (round & 1) ^ 1;
  W const lo = st->old, thr = st->thr;
  W const BIG = std::numeric_limits<W>::max();
  CGX_SPLIT_LDS(V);
  W fmin = BIG;
  for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < a.nv; base += (int64_t)gridDim.x * blockDim.x) {
    int64_t const i = base + threadIdx.x;
    W const d       = i < a.nv ? a.dist[i] : BIG;
    bool const cand = d >= lo && d < thr;
    if (!cand && d >= thr && d < BIG) fmin = d < fmin ? d : fmin;  // (a vertex without edges only lowers fmin)
    if (!__any(cand)) continue;
    uint32_t light = 0, heavy = 0;
    if (cand) {
      light = (uint32_t)(a.pt[kLight].off[i + 1] - a.pt[kLight].off[i]);
      heavy = (uint32_t)(a.pt[kHeavy].off[i + 1] - a.pt[kHeavy].off[i]);
    }
    route(a, sg, Q, cand, (V)i, d, thr, light, heavy, fmin);
  }
  route_flush(a, sg, Q);
  block_min_far(st, fmin);
}

// A dense round as a pull over the part (the light edges of every row in a light
// round, the heavy edges in a heavy one), 2048 edges per chunk in order: a row
// whose distance is above the round's floor (bucket start, or thr for heavy edges:
// nothing below can improve) takes the smallest dist[u] + w over its edges from
// frontier sources u (the list's bitmap), and an improvement is one atomicMin per
// row and chunk (a per-row minimum in LDS first).  A row's edges here are its
// in-edges: symmetric graphs only.  Block 0 clears the next near counter (as
// k_relax does on push rounds).
template <typename V, typename E, typename W>
__global__ __launch_bounds__(256) void k_pull(sssp_args<V, E, W> a, int round)
{
  using B           = typename bits_of<W>::type;
  sssp_state<W>* st = a.st;
  int const P = round & 1;
  if (st->done || !round_pulls(a, st, P)) return;
  int const tid    = threadIdx.x;
  bool const hvy   = st->phase == kHeavy;
  part_t<V, E, W> const pt = a.pt[hvy ? kHeavy : kLight];
  uint32_t const* F        = a.fbits[hvy ? 2 + st->hl : P];
  W const floor_           = hvy ? st->thr : st->old;
  W const BIG              = std::numeric_limits<W>::max();
  int64_t const nch        = (pt.ne + kChunk - 1) / kChunk;
  __shared__ int s_row[kChunk];  // per position: its row (a max-scan of the row starts)
  __shared__ B s_best[kChunk];   // per row start position: the row's best candidate (bits)
  __shared__ int s_wmax[4];
  unsigned long long my_e = 0;
  for (int64_t c = blockIdx.x; c < nch; c += gridDim.x) {
    int64_t const t0 = c * kChunk;
    int64_t const t1 = t0 + kChunk < pt.ne ? t0 + kChunk : pt.ne;
    int64_t const r0 = pt.crow[c];
    int64_t const r1 = c + 1 < nch ? pt.crow[c + 1] : a.nv - 1;
    B const binf     = *reinterpret_cast<B const*>(&BIG);
    for (int p = tid; p < kChunk; p += 256) {
      s_row[p]  = p == 0 ? (int)(r0 - r0) : -1;
      s_best[p] = binf;
    }
    __syncthreads();
    for (int64_t r = r0 + 1 + tid; r <= r1; r += 256) {  // rows starting inside the chunk (the last of equal starts wins)
      int64_t const p = (int64_t)pt.off[r] - t0;
      if (p > 0 && p < kChunk) atomicMax(&s_row[p], (int)(r - r0));
    }
    __syncthreads();
    {  // inclusive max-scan: thread tid owns positions [8 tid, 8 tid + 8)
      int m = -1, loc[kPerThread];
#pragma unroll
      for (int k = 0; k < kPerThread; ++k) {
        int const x = s_row[tid * kPerThread + k];
        m           = x > m ? x : m;
        loc[k]      = m;
      }
      int pre = m;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        int const y = __shfl_up(pre, o, 64);
        if ((tid & 63) >= o) pre = y > pre ? y : pre;
      }
      if ((tid & 63) == 63) s_wmax[tid >> 6] = pre;
      int excl = __shfl_up(pre, 1, 64);
      if ((tid & 63) == 0) excl = -1;
      __syncthreads();
      for (int w = 0; w < (tid >> 6); ++w) excl = s_wmax[w] > excl ? s_wmax[w] : excl;
#pragma unroll
      for (int k = 0; k < kPerThread; ++k) s_row[tid * kPerThread + k] = loc[k] > excl ? loc[k] : excl;
    }
    __syncthreads();
    V u[kPerThread];
    W w[kPerThread], dv[kPerThread];
    int rl[kPerThread];
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) {
      int const p     = k * 256 + tid;
      int64_t const t = t0 + p;
      u[k]            = V(-1);
      rl[k]           = -1;
      if (t < t1) {
        rl[k] = s_row[p];
        dv[k] = a.dist[r0 + rl[k]];
        if (dv[k] > floor_) {
          u[k] = pt.idx[t];
          w[k] = pt.w[t];
        }
      }
    }
    bool fr[kPerThread];
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) fr[k] = u[k] >= 0 && ((F[u[k] >> 5] >> (uint32_t(u[k]) & 31u)) & 1u);
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) {
      if (!fr[k]) continue;
      W const nd = a.dist[u[k]] + w[k];
      if (nd < a.cutoff && nd < dv[k]) {
        int64_t const rs = (int64_t)pt.off[r0 + rl[k]] - t0;  // the row's start position in the chunk (0 if before)
        atomicMin(&s_best[rs > 0 ? rs : 0], *reinterpret_cast<B const*>(&nd));
      }
    }
    if (tid == 0) my_e += (unsigned long long)(t1 - t0);
    __syncthreads();
    for (int p = tid; p < kChunk; p += 256) {
      B const bb = s_best[p];
      if (bb != binf) {
        int64_t const v = r0 + s_row[p];
        W const nd      = *reinterpret_cast<W const*>(&bb);
        if (nd < a.dist[v]) {
          atomicMin(reinterpret_cast<B*>(a.dist + v), bb);
          atomicOr(a.cbits + (v >> 5), 1u << (uint32_t(v) & 31u));
        }
      }
    }
    __syncthreads();
  }
  if (a.trace) {
    for (int o = 32; o > 0; o >>= 1) my_e += __shfl_xor(my_e, o, 64);
    int const p = (int)((blockIdx.x * 4 + (tid >> 6)) & 15);
    if ((tid & 63) == 0 && my_e) atomicAdd(&st->work[p][hvy ? 5 : 4], my_e);
  }
}

// One wave: the source (an internal id, -1 when the external id is not a vertex)
// through route() as the only vertex of the first split (parity 0); distance 0.
template <typename V, typename E, typename W>
__global__ __launch_bounds__(64) void k_sssp_init(sssp_args<V, E, W> a, V const* src, W delta)
{
  sssp_state<W>* st = a.st;
  V const s_        = *src;
  if (threadIdx.x == 0) {
    st->delta  = delta;
    st->thr    = delta;
    st->minfar = ~typename bits_of<W>::utype(0) >> 1;
    st->epoch  = 1;
  }
  if (s_ < 0 || (int64_t)s_ >= a.nv) {
    if (threadIdx.x == 0) {
      st->bad  = 1;
      st->done = 1;
    }
    return;
  }
  if (threadIdx.x == 0) a.dist[s_] = W(0);
  __shared__ V s_v[1][kStage], s_b[1][kStage];
  __shared__ uint32_t s_dn[1][kStage], s_db[1][kStage];
  split_stages<V> sg{{s_v[0], s_dn[0], 0}, {s_b[0], s_db[0], 0}};
  uint32_t const light = (uint32_t)(a.pt[kLight].off[s_ + 1] - a.pt[kLight].off[s_]);
  uint32_t const heavy = (uint32_t)(a.pt[kHeavy].off[s_ + 1] - a.pt[kHeavy].off[s_]);
  W fmin               = std::numeric_limits<W>::max();
  route(a, sg, 0, threadIdx.x == 0, s_, W(0), delta, light, heavy, fmin);
  route_flush(a, sg, 0);
  __syncthreads();
  // a source with light edges starts with a light round; with heavy edges only, its
  // bucket list goes first; without edges there is nothing to do
  if (threadIdx.x == 0 && (st->nq[0][0] >> a.eb) == 0) {
    if ((st->nr[st->rp][0] >> a.eb) > 0) {
      st->phase = kHeavy;
      st->hl    = st->rp;
      st->rp ^= 1;
      st->epoch += 1;
    } else {
      st->done = 1;
    }
  }
}

// The light (w < delta) and heavy edges of every row as two CSRs: light counts
// (a wave per row), their scan (host), then the rows' edges scattered in order.
template <typename V, typename E, typename W>
__global__ __launch_bounds__(256) void k_count_light(E const* off, W const* wgt, int64_t nv, W delta, E* nl)
{
  int const lane = lane_id();
  for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; r < nv;
       r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    E const beg = off[r], end = off[r + 1];
    E cnt       = 0;
    for (E base = beg; base < end; base += 64) {
      E const e = base + lane;
      cnt += (E)__popcll(__ballot(e < end && wgt[e] < delta));
    }
    if (lane == 0) nl[r] = cnt;
  }
}

template <typename E>
__global__ void k_heavy_offsets(E const* off, E const* offL, int64_t n, E* offH)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    offH[i] = off[i] - offL[i];
}

template <typename V, typename E, typename W>
__global__ __launch_bounds__(256) void k_scatter_parts(E const* off, V const* idx, W const* wgt, int64_t nv, W delta,
                                                        E const* offL, E const* offH, V* idxL, W* wL, V* idxH,
                                                        W* wH)
{
  int const lane = lane_id();
  for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; r < nv;
       r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    E const beg = off[r], end = off[r + 1];
    E oL = offL[r], oH = offH[r];
    for (E base = beg; base < end; base += 64) {
      E const e     = base + lane;
      bool const in = e < end;
      V v           = 0;
      W w           = W(0);
      if (in) {
        v = idx[e];
        w = wgt[e];
      }
      bool const lt               = in && w < delta;
      unsigned long long const ml = __ballot(lt), mh = __ballot(in && !lt);
      unsigned long long const below = (1ull << lane) - 1ull;
      if (lt) {
        E const o = oL + (E)__popcll(ml & below);
        idxL[o]   = v;
        wL[o]     = w;
      } else if (in) {
        E const o = oH + (E)__popcll(mh & below);
        idxH[o]   = v;
        wH[o]     = w;
      }
      oL += (E)__popcll(ml);
      oH += (E)__popcll(mh);
    }
  }
}

// the row holding edge c * kChunk of a CSR, for every chunk c
template <typename E>
__global__ void k_chunk_rows(E const* off, int64_t nv, int64_t* crow)
{
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nv; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t const b = (int64_t)off[r], e = (int64_t)off[r + 1];
    for (int64_t c = (b + kChunk - 1) / kChunk; c * kChunk < e; ++c) crow[c] = r;
  }
}

// Predecessors by a pull over the in-edges (sorted ascending): the first -- the
// smallest-id -- in-neighbour u with dist[u] + w == dist[v]; -1 for the source and
// unreached vertices.  k_sssp_pred_probe: a lane per vertex tests its first 4
// in-edges with every load issued at once (ids descend by degree, so a vertex's
// first neighbours are its hubs, usually the tight ones) and marks the rest kMiss;
// k_sssp_pred_scan: a 16-lane group per marked vertex walks the list from the 5th
// edge on, 16 at a time.
constexpr int kPredProbe = 4;

template <typename V, typename E, typename W>
__global__ __launch_bounds__(256) void k_sssp_pred_probe(E const* off, V const* idx, W const* wgt, W const* dist,
                                                         int64_t nv, V const* src, V* pred)
{
  V const s_  = *src;
  W const BIG = std::numeric_limits<W>::max();
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x) {
    W const dv      = dist[v];
    bool const want = (V)v != s_ && dv != BIG;
    E beg = 0, end = 0;
    if (want) {
      beg = off[v];
      end = off[v + 1];
    }
    V u[kPredProbe];
    W w[kPredProbe];
#pragma unroll
    for (int k = 0; k < kPredProbe; ++k) {
      bool const in = want && beg + k < end;
      u[k]          = in ? idx[beg + k] : V(-1);
      w[k]          = in ? wgt[beg + k] : W(0);
    }
    W du[kPredProbe];
#pragma unroll
    for (int k = 0; k < kPredProbe; ++k) du[k] = u[k] >= 0 ? dist[u[k]] : BIG;
    V found = V(-1);
#pragma unroll
    for (int k = kPredProbe - 1; k >= 0; --k)
      if (u[k] >= 0 && (W)(du[k] + w[k]) == dv) found = u[k];
    pred[v] = want && found < 0 && end - beg > kPredProbe ? V(-2) : found;
  }
}

template <typename V, typename E, typename W>
__global__ __launch_bounds__(256) void k_sssp_pred_scan(E const* off, V const* idx, W const* wgt, W const* dist,
                                                        int64_t nv, V* pred)
{
  int const lane = threadIdx.x & 15;
  int const gsh  = threadIdx.x & 48;  // the group's first lane within the wave
  for (int64_t v0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 4; v0 < nv;
       v0 += ((int64_t)gridDim.x * blockDim.x) >> 4) {
    if (pred[v0] != V(-2)) continue;
    W const dv  = dist[v0];
    E const beg = off[v0] + kPredProbe, end = off[v0 + 1];
    V found     = V(-1);
    for (E base = beg; base < end; base += 16) {
      E const e  = base + lane;
      bool tight = false;
      V u        = 0;
      if (e < end) {
        u     = idx[e];
        tight = (W)(dist[u] + wgt[e]) == dv;
      }
      unsigned long long const m = (__ballot(tight) >> gsh) & 0xffffull;
      if (m) {
        found = __shfl(u, gsh + __ffsll((long long)m) - 1, 64);
        break;
      }
    }
    if (lane == 0) pred[v0] = found;
  }
}

template <typename W>
__global__ void k_weight_stats(W const* w, size_t ne, double* out)
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

template <typename V>
flist<V> make_list(dbuf<V>& q, dbuf<int64_t>& ep, dbuf<int64_t>& cs)
{
  return flist<V>{q.data(), ep.data(), cs.data()};
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
  // the source is an external id (c_api/sssp.cpp renumbers it): looked up on the
  // device, checked by k_sssp_init, reported with the first chunk's state read
  V hs = (V)source;
  CGX_INPUT((int64_t)source >= 0 && (size_t)(V)source == source, "Invalid input argument: source vertex out-of-range.");
  dbuf<V> src_id(1, s);
  to_device(src_id.data(), &hs, 1, s);
  renumber_ext_to_int_unchecked(h, g, src_id.data(), 1);
  res.vertices     = number_map_copy(h, g);
  res.distances    = std::make_unique<device_array_t>((size_t)nv, dtype_of<W>(), s);
  res.predecessors = std::make_unique<device_array_t>(want_pred ? (size_t)nv : 0, dtype_of<V>(), s);
  W* dist          = res.distances->buf.data<W>();
  W const BIG      = std::numeric_limits<W>::max();
  fill<W>(dist, nv, BIG, s);
  if (nv == 0) return;

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
  // list counters: (slots << eb) | edges in one 64-bit word
  int const eb = bits_for((unsigned long long)std::max<size_t>(ne, 1));
  CGX_EXPECTS(bits_for((unsigned long long)nv) + eb <= 64, CUGRAPH_NOT_IMPLEMENTED,
              "SSSP: vertex and edge counts exceed the 64-bit frontier counter");

  // delta = kDeltaScale * average edge weight / average degree (the reference:
  // warp_size = 32 times the same, :143-157); the weight sum is cached on the
  // adjacency (one read of the weights per graph, not per call)
  if (adj.wsum < 0 && ne) {
    dbuf<double> wsum(1, s);
    fill<double>(wsum.data(), 1, 0.0, s);
    hipLaunchKernelGGL(k_weight_stats<W>, dim3(grid_for(ne, kBlock, 1024)), dim3(kBlock), 0, s, wgt, ne, wsum.data());
    CGX_LAUNCH_CHECK();
    adj.wsum = to_host_scalar(wsum.data(), s);
  }
  double const avg_w   = ne ? std::max(adj.wsum, 0.0) / (double)ne : 0.0;
  double const avg_deg = (double)ne / (double)nv;
  double const dscale  = h.tune.sssp_delta > 0 ? h.tune.sssp_delta : kDeltaScale;
  W const delta        = (W)std::max(avg_deg > 0 ? dscale * avg_w / avg_deg : 1.0, 1e-30);
  // the light and heavy CSRs for this delta (cached on the adjacency)
  if (adj.sssp_delta != (double)delta) {
    for (buffer* b : {&adj.sssp_offL, &adj.sssp_offH, &adj.sssp_idxL, &adj.sssp_wL, &adj.sssp_idxH, &adj.sssp_wH,
                      &adj.sssp_crowL, &adj.sssp_crowH})
      b->set_stream(s);
    adj.sssp_offL.resize((size_t)(nv + 1) * sizeof(E));
    adj.sssp_offH.resize((size_t)(nv + 1) * sizeof(E));
    E* offL = adj.sssp_offL.data<E>();
    E* offH = adj.sssp_offH.data<E>();
    {
      dbuf<E> nl(nv + 1, s);
      HIP_CHECK(hipMemsetAsync(nl.data() + nv, 0, sizeof(E), s));
      hipLaunchKernelGGL((k_count_light<V, E, W>), dim3(grid_for((size_t)nv * 64, 256, 16384)), dim3(256), 0, s, off,
                         wgt, nv, delta, nl.data());
      CGX_LAUNCH_CHECK();
      exclusive_scan<E, E>(nl.data(), offL, (size_t)nv + 1, s);
    }
    hipLaunchKernelGGL(k_heavy_offsets<E>, dim3(grid_for((size_t)nv + 1, kBlock, 8192)), dim3(kBlock), 0, s, off, offL,
                       nv + 1, offH);
    CGX_LAUNCH_CHECK();
    E eL = 0;
    HIP_CHECK(hipMemcpyAsync(&eL, offL + nv, sizeof(E), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    adj.sssp_eL = (int64_t)eL;
    adj.sssp_eH = (int64_t)ne - (int64_t)eL;
    adj.sssp_idxL.resize(std::max<int64_t>(adj.sssp_eL, 1) * sizeof(V));
    adj.sssp_wL.resize(std::max<int64_t>(adj.sssp_eL, 1) * sizeof(W));
    adj.sssp_idxH.resize(std::max<int64_t>(adj.sssp_eH, 1) * sizeof(V));
    adj.sssp_wH.resize(std::max<int64_t>(adj.sssp_eH, 1) * sizeof(W));
    hipLaunchKernelGGL((k_scatter_parts<V, E, W>), dim3(grid_for((size_t)nv * 64, 256, 16384)), dim3(256), 0, s, off,
                       idx, wgt, nv, delta, offL, offH, adj.sssp_idxL.data<V>(), adj.sssp_wL.data<W>(),
                       adj.sssp_idxH.data<V>(), adj.sssp_wH.data<W>());
    CGX_LAUNCH_CHECK();
    adj.sssp_crowL.resize((size_t)(adj.sssp_eL / kChunk + 2) * sizeof(int64_t));
    adj.sssp_crowH.resize((size_t)(adj.sssp_eH / kChunk + 2) * sizeof(int64_t));
    hipLaunchKernelGGL(k_chunk_rows<E>, dim3(grid_for((size_t)nv, kBlock, 8192)), dim3(kBlock), 0, s, offL, nv,
                       adj.sssp_crowL.data<int64_t>());
    hipLaunchKernelGGL(k_chunk_rows<E>, dim3(grid_for((size_t)nv, kBlock, 8192)), dim3(kBlock), 0, s, offH, nv,
                       adj.sssp_crowH.data<int64_t>());
    CGX_LAUNCH_CHECK();
    adj.sssp_delta = (double)delta;
  }

  int64_t const nchunk_max = (int64_t)(ne + kChunk - 1) / kChunk + 1;
  dbuf<int> stamp(nv, s);
  fill<int>(stamp.data(), nv, 0, s);
  int64_t const nwords = (nv + 31) / 32;
  dbuf<uint32_t> cbits(nwords, s), fbits(4 * nwords, s);
  HIP_CHECK(hipMemsetAsync(cbits.data(), 0, nwords * sizeof(uint32_t), s));
  HIP_CHECK(hipMemsetAsync(fbits.data(), 0, 4 * nwords * sizeof(uint32_t), s));
  dbuf<V> q[4] = {dbuf<V>(nv, s), dbuf<V>(nv, s), dbuf<V>(nv, s), dbuf<V>(nv, s)};
  dbuf<int64_t> ep[4] = {dbuf<int64_t>(nv, s), dbuf<int64_t>(nv, s), dbuf<int64_t>(nv, s), dbuf<int64_t>(nv, s)};
  dbuf<int64_t> cs[4] = {dbuf<int64_t>(nchunk_max, s), dbuf<int64_t>(nchunk_max, s), dbuf<int64_t>(nchunk_max, s),
                         dbuf<int64_t>(nchunk_max, s)};
  dbuf<sssp_state<W>> st(1, s);
  HIP_CHECK(hipMemsetAsync(st.data(), 0, sizeof(sssp_state<W>), s));
  sssp_args<V, E, W> a{};
  a.off   = off;
  a.pt[kLight] = part_t<V, E, W>{adj.sssp_offL.data<E>(), adj.sssp_idxL.data<V>(), adj.sssp_wL.data<W>(),
                                 adj.sssp_crowL.data<int64_t>(), adj.sssp_eL};
  a.pt[kHeavy] = part_t<V, E, W>{adj.sssp_offH.data<E>(), adj.sssp_idxH.data<V>(), adj.sssp_wH.data<W>(),
                                 adj.sssp_crowH.data<int64_t>(), adj.sssp_eH};
  // a pull reads a row's edges as its in-edges: symmetric graphs only
  a.pull_div = g.symmetric && h.tune.sssp_pull >= 0 ? (h.tune.sssp_pull > 0 ? h.tune.sssp_pull : kPullDiv) : 0;
  for (int i = 0; i < 4; ++i) a.fbits[i] = fbits.data() + i * nwords;
  a.dist   = dist;
  a.stamp  = stamp.data();
  a.cutoff = cut;
  for (int i = 0; i < 2; ++i) {
    a.near[i]   = make_list(q[i], ep[i], cs[i]);
    a.bucket[i] = make_list(q[2 + i], ep[2 + i], cs[2 + i]);
  }
  a.cbits  = cbits.data();
  a.st     = st.data();
  a.nv     = nv;
  a.eb     = eb;
  static bool const trace = std::getenv("CGX_SSSP_TRACE") != nullptr;
  a.trace                 = trace ? 1 : 0;
  hipLaunchKernelGGL((k_sssp_init<V, E, W>), dim3(1), dim3(64), 0, s, a, src_id.data(), delta);
  CGX_LAUNCH_CHECK();
  auto* hs_st = h.pinned_as<sssp_state<W>>();
  int round   = 0;
  while (true) {
    for (int k = 0; k < kChunkRounds; ++k, ++round) {
      hipLaunchKernelGGL((k_relax<V, E, W>), dim3(kRelaxGrid), dim3(256), 0, s, a, round);
      hipLaunchKernelGGL((k_pull<V, E, W>), dim3(kPullGrid), dim3(256), 0, s, a, round);
      hipLaunchKernelGGL((k_split<V, E, W>), dim3(kSplitGrid), dim3(256), 0, s, a, round);
      hipLaunchKernelGGL(k_sssp_ctl<W>, dim3(1), dim3(1), 0, s, a.st, round, eb);
      hipLaunchKernelGGL((k_far_split<V, E, W>), dim3(kSplitGrid), dim3(256), 0, s, a, round);
      CGX_LAUNCH_CHECK();
    }
    HIP_CHECK(hipMemcpyAsync(hs_st, st.data(), sizeof(sssp_state<W>), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    CGX_INPUT(!hs_st->bad, "Invalid input argument: source vertex out-of-range.");
    if (hs_st->done) break;
  }
  h.last_iterations = (size_t)hs_st->rounds;
  if (trace) {
    unsigned long long light = 0, heavy = 0, impr = 0, atom = 0, pl = 0, ph = 0;
    for (int p = 0; p < 16; ++p) {
      light += hs_st->work[p][0];
      impr += hs_st->work[p][1];
      atom += hs_st->work[p][2];
      heavy += hs_st->work[p][3];
      pl += hs_st->work[p][4];
      ph += hs_st->work[p][5];
    }
    double const E1 = ne ? (double)ne : 1.0;
    std::fprintf(stderr, "[sssp] V %lld E %zu delta %.6g (light part %.3f E): %llu rounds (%d enqueued), pushed "
                 "light %.2f E heavy %.2f E, pulled light %.2f E heavy %.2f E, %llu push atomics, %llu improved "
                 "vertices (%.2f V)\n", (long long)nv, ne, (double)delta, (double)adj.sssp_eL / E1, hs_st->rounds,
                 round, (double)light / E1, (double)heavy / E1, (double)pl / E1, (double)ph / E1, atom, impr,
                 (double)impr / (double)nv);
  }
  if (want_pred) {
    V* pred = res.predecessors->buf.data<V>();
    // in-edges: a symmetric graph's own rows, else the cached CSC
    adjacency_t& in = g.symmetric ? adj : ensure_adjacency(h, g, true);
    hipLaunchKernelGGL((k_sssp_pred_probe<V, E, W>), dim3(grid_for((size_t)nv, 256, 8192)), dim3(256), 0, s,
                       in.offsets.data<E>(), in.indices.data<V>(), in.weights.data<W>(), dist, nv, src_id.data(), pred);
    hipLaunchKernelGGL((k_sssp_pred_scan<V, E, W>), dim3(grid_for((size_t)nv * 16, 256, 16384)), dim3(256), 0, s,
                       in.offsets.data<E>(), in.indices.data<V>(), in.weights.data<W>(), dist, nv, pred);
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
