// Breadth-first search, direction-optimising (single GPU).
//
// Reference semantics: cpp/src/traversal/bfs_impl.cuh:94-287 (+ c_api/bfs.cpp:60-145):
// distances INT_MAX / predecessors -1 for unreached vertices, every source at 0,
// level-synchronous, stop on an empty frontier or depth >= depth_limit.  The
// reference only implements top-down ("direction_optimizing ... unimplemented",
// bfs_impl.cuh:206-207) and lets atomicOr winners pick predecessors; this build:
//
//  * top-down step (frontier queues): frontier vertices are kept in three queues
//    by degree class (<=16: 4 lanes, <=1024: one wave, larger: one block), so the
//    expansion is load-balanced without a per-level scan; discovered vertices are
//    claimed with a CAS on the distance and appended to the next queues with a
//    64-lane __ballot/popcount compaction (one atomic per wave and class).
//  * bottom-up step (frontier bitmap, symmetric graphs): every unvisited vertex
//    scans its sorted adjacency in lane groups (degree-binned schedule, as the
//    PageRank kernel) and stops at the first neighbour in the frontier bitmap
//    (the bitmap is V/8 bytes: L2/Infinity-Cache resident).
//  * Beamer switching from per-level counters, alpha = 40 / beta = 64 (measured on
//    RMAT-24, see bfs_impl; mg_bfs.hip keeps Beamer's 14 / 24).
//  * predecessor = the frontier neighbour with the smallest internal id in both
//    directions (atomicMin top-down, first hit in the sorted list bottom-up), so
//    results are deterministic and independent of the direction schedule.
#include "capi.hpp"
#include "prims.hpp"
#include "schedule.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <stdexcept>

namespace cgx {

namespace {

constexpr int kSmallDeg = 16;    // 4-lane groups
constexpr int kMidDeg   = 1024;  // one wave; above: edge chunks over blocks
constexpr int kChunk    = 2048;  // edges per large-class chunk

// What the host reads of a level (64 B)
struct bfs_ctr_hdr {
  unsigned long long qlen[3];  // next queues: small / mid / large (first: bfs_args::ncur_dev points here)
  unsigned long long next_n;   // vertices discovered this level
  unsigned long long next_m;   // sum of their degrees
  unsigned long long pad[3];  // [0]: publish sequence, [1]: source check, [2]: sources' edge count
};
static_assert(sizeof(bfs_ctr_hdr) == 64, "k_publish_seq writes host words 0..7 and 8..12 by index");

// The device block.  Every kernel block adds its discovered-vertex and edge counts
// at the end (flush_counts); same-address atomics serialise at the memory side
// (~8 ns each), so the block counts go to kCtrParts partial counters 256 B apart
// (different L2 channels) and the publish kernel folds them into next_n / next_m.
// That lets the bottom-up probe run on larger grids.
constexpr int kCtrParts = 16;
struct bfs_ctr : bfs_ctr_hdr {
  unsigned long long part[kCtrParts][32];  // [p][0]: vertices, [p][1]: edges, [p][2]: residual sub-queue length
};

// The bottom-up probe's misses (rows longer than the probe, no frontier neighbour in
// it) go to kCtrParts sub-queues, chunk c's to sub-queue c % kCtrParts, each with its
// length in its own partial counter: one queue with one counter serialised every
// wave's append at the memory side -- RMAT-24 root 7's first bottom-up level (a
// frontier of a few vertices, nearly every vertex a miss: ~139K appends) took 579 us
// in the probe.  Sub-queue p holds at most the 64 vertices of each of its chunks.
__host__ __device__ __forceinline__ int64_t residual_cap(int64_t nv)
{
  return ((((nv + 63) >> 6) + kCtrParts - 1) / kCtrParts) * 64;
}

// (next_n, next_m) of a block with the partial counters folded in; lanes 0..15 of
// one wave read the parts, every lane gets the totals; zero: clear the parts
__device__ __forceinline__ void fold_parts(bfs_ctr* c, bool zero, unsigned long long& n, unsigned long long& m)
{
  int const lane = threadIdx.x & 63;
  unsigned long long pn = 0, pm = 0;
  if (lane < kCtrParts) {
    pn = c->part[lane][0];
    pm = c->part[lane][1];
    if (zero) {
      c->part[lane][0] = 0ull;
      c->part[lane][1] = 0ull;
      c->part[lane][2] = 0ull;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    pn += __shfl_xor(pn, o, 64);
    pm += __shfl_xor(pm, o, 64);
  }
  n = pn + c->next_n;
  m = pm + c->next_m;
}

// the level counters (then zeroed for the next level: no memset launch per level)
// and the source check flag (pad[1]), then seq (the host's poll word, pad[0]) behind
// a system fence.  ctr_b: a second level's counters (a speculative top-down level)
// -> host[1], also zeroed; src_m: the sources' edge count of a conversion the host
// did not read (bfs_ctr::next_m of that block) -> pad[2]
__global__ void k_publish_seq(bfs_ctr* ctr, bfs_ctr_hdr* host, unsigned long long seq, int const* bad, bfs_ctr* ctr_b,
                              bfs_ctr* src_m, bfs_ctr* ctr_c)
{
  unsigned long long n, m, nb = 0, mb = 0, ns = 0, ms = 0, nc = 0, mc = 0;
  fold_parts(ctr, true, n, m);
  if (ctr_b) fold_parts(ctr_b, true, nb, mb);
  if (src_m) fold_parts(src_m, false, ns, ms);
  if (ctr_c) fold_parts(ctr_c, true, nc, mc);
  // One host word per lane, all stores in flight at once (one thread storing the
  // words one after another made this kernel 4.6 us): lanes 0..4 this level (host
  // words 0..4), 5..9 ctr_b (host[1]), 10..11 pad[2] / pad[1], 12..16 ctr_c (host[2]).
  // No lane leaves early: every store is issued before the wave reconverges and
  // waits for them, and only then is the sequence word stored -- a lane group that
  // returned early could run its branch after the sequence store.
  int const i                = threadIdx.x;
  unsigned long long* const c  = reinterpret_cast<unsigned long long*>(ctr);
  unsigned long long* const cb = reinterpret_cast<unsigned long long*>(ctr_b);
  unsigned long long* const cc = reinterpret_cast<unsigned long long*>(ctr_c);
  unsigned long long* const hp = reinterpret_cast<unsigned long long*>(host);
  unsigned long long v  = 0;
  int slot              = -1;  // host word
  unsigned long long* z = nullptr;  // device counter word to clear
  if (i < 5) {
    v    = i < 3 ? c[i] : (i == 3 ? n : m);
    slot = i;
    z    = c + i;
  } else if (i < 10) {
    int const k = i - 5;
    if (ctr_b) {
      v    = k < 3 ? cb[k] : (k == 3 ? nb : mb);
      slot = 8 + k;
      z    = cb + k;
    }
  } else if (i == 10) {
    v    = ms;
    slot = 7;  // pad[2]
  } else if (i == 11) {
    v    = bad ? (unsigned long long)*bad : 0ull;
    slot = 6;  // pad[1]
  } else if (i < 17) {
    int const k = i - 12;
    if (ctr_c) {
      v    = k < 3 ? cc[k] : (k == 3 ? nc : mc);
      slot = 16 + k;
      z    = cc + k;
    }
  }
  if (slot >= 0) __hip_atomic_store(hp + slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (z) *z = 0ull;
  // The host block is fine-grained (coherent, uncached) memory: the words reach it
  // in order once the wave's stores are acknowledged, so waiting for them orders the
  // sequence word behind the data without writing the L2 back (nothing the host
  // reads is in it; the next kernels are stream-ordered behind this one anyway).  A
  // system-scope release there (its L2 write-back) measured 0.674-0.675 against
  // 0.667-0.669 ms per RMAT-24 traversal, same box.
  // (gfx9 family only: there vmcnt counts stores as well as loads; gfx10+ counts
  // stores in vscnt, and this wait would not order them -- the build rejects it below.
  // It also relies on handle_t::polled_as staying fine-grained coherent memory.)
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "k_publish_seq orders its stores with s_waitcnt vmcnt(0): gfx9-family (gfx950) targets only"
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (i != 0) return;
  __hip_atomic_store(&host->pad[0], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename V>
__device__ __forceinline__ bool cas_claim(V* dist, V v, V nd)
{
  if constexpr (sizeof(V) == 4) {
    return atomicCAS(reinterpret_cast<int*>(dist + v), (int)std::numeric_limits<int32_t>::max(), (int)nd) ==
           std::numeric_limits<int32_t>::max();
  } else {
    unsigned long long inf = (unsigned long long)std::numeric_limits<int64_t>::max();
    return atomicCAS(reinterpret_cast<unsigned long long*>(dist + v), inf, (unsigned long long)nd) == inf;
  }
}

// unsigned: predecessors start at -1 (all ones), the unreached value of the result.
// Returns whether this was the vertex's first parent (the old value was -1).
template <typename V>
__device__ __forceinline__ bool atomic_min_first(V* p, V x)
{
  if constexpr (sizeof(V) == 4) return atomicMin(reinterpret_cast<unsigned*>(p), (unsigned)x) == ~0u;
  else return atomicMin(reinterpret_cast<unsigned long long*>(p), (unsigned long long)x) == ~0ull;
}

// wave-aggregated append: every active lane with `take` gets a distinct slot
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

template <typename V, typename E>
struct bfs_args {
  E const* off;
  V const* idx;
  V* dist;
  V* pred;  // nullptr when predecessors are not requested; -1 until set
  V const* nmap;  // internal -> external ids (nullptr: not renumbered); predecessors are stored external
  uint32_t* vis;
  uint32_t* fr;   // bottom-up: current frontier bitmap
  uint32_t* nxt;  // bottom-up: next frontier bitmap
  V const* qcur[3];
  unsigned long long ncur[3];
  unsigned long long const* ncur_dev;  // if set: the current queue lengths, read on the device (ncur: bounds)
  V* qnext[3];
  bfs_ctr* ctr;
  V depth;  // distance of the current frontier
  int64_t nv;
  V const* order;
  work_item const* items;
  long long blk_mid_start, blk_small_start;  // top-down grid segmentation
  bool head2;       // with head: misses probe the next kProbe neighbours in the adjacency too
  int const* head;  // nullptr, or kHeadN + 1 words per vertex: its first kHeadN neighbours + degree (k_bfs_head)
};

// Next-queue appends are staged per wave in LDS (kStage entries per class) and
// written out in bulk: one global atomic per ~450 discovered vertices instead of one
// per wave and class per 64-edge batch -- at a hub level (hundreds of frontier hubs,
// ~1M discoveries) the per-batch atomics serialised on the three queue tails.
constexpr int kStage = 512;

template <typename V>
struct wave_stage {
  V* buf;     // this wave's 3 * kStage LDS entries
  int n[3];   // wave-uniform fill counts
};

template <typename V, typename E>
__device__ __forceinline__ void stage_flush(bfs_args<V, E> const& a, wave_stage<V>& st, int c)
{
  int const cnt = st.n[c];
  if (cnt == 0) return;
  // DS operations of one wave complete in order; the barrier only pins the compiler
  __builtin_amdgcn_wave_barrier();
  int const lane          = threadIdx.x & 63;
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd(&a.ctr->qlen[c], (unsigned long long)cnt);
  base = __shfl(base, 0, 64);
  for (int j = lane; j < cnt; j += 64) a.qnext[c][base + j] = st.buf[c * kStage + j];
  __builtin_amdgcn_wave_barrier();
  st.n[c] = 0;
}

template <typename V, typename E>
__device__ __forceinline__ void push_next(bfs_args<V, E> const& a, wave_stage<V>& st, V v, bool take,
                                          unsigned long long& my_m)
{
  int cls = 0;
  if (take) {
    E deg = a.off[v + 1] - a.off[v];
    cls   = deg <= kSmallDeg ? 0 : (deg <= kMidDeg ? 1 : 2);
    my_m += (unsigned long long)deg;
  }
  int const lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    bool const mine          = take && cls == c;
    unsigned long long const mask = __ballot(mine);
    if (mask == 0) continue;
    if (mine) st.buf[c * kStage + st.n[c] + __popcll(mask & ((1ull << lane) - 1ull))] = v;
    st.n[c] += __popcll(mask);
    if (st.n[c] > kStage - 64) stage_flush<V, E>(a, st, c);
  }
}

template <typename V, typename E>
__device__ __forceinline__ void stage_flush_all(bfs_args<V, E> const& a, wave_stage<V>& st)
{
  for (int c = 0; c < 3; ++c) stage_flush<V, E>(a, st, c);
}

#define CGX_WAVE_STAGE(V, st)                                   \
  __shared__ V s_stage_[4][3 * kStage];                         \
  wave_stage<V> st{s_stage_[threadIdx.x >> 6], {0, 0, 0}}

template <typename V, typename E>
__device__ __forceinline__ void visit_edge(bfs_args<V, E> const& a, wave_stage<V>& st, V u, V v, bool active,
                                           unsigned long long& my_m)
{
  bool take = false;
  if (active) {
    uint32_t bit = 1u << (uint32_t(v) & 31u);
    if (!(a.vis[v >> 5] & bit)) {  // not visited before this level
      if (a.pred) {
        // one atomic per edge: the smallest-parent atomicMin is also the claim (its
        // first caller sees -1), and the claimer stores the distance -- was atomicMin
        // + a CAS on the distance
        take = atomic_min_first<V>(a.pred + v, u);
        if (take) a.dist[v] = (V)(a.depth + 1);
      } else {
        take = cas_claim<V>(a.dist, v, (V)(a.depth + 1));
      }
    }
  }
  push_next<V, E>(a, st, v, take, my_m);
}

__device__ __forceinline__ void flush_counts(bfs_ctr* ctr, unsigned long long n, unsigned long long m)
{
  __shared__ unsigned long long sn[4], sm_[4];
  unsigned long long wn = 0, wm = 0;
  for (int o = 32; o > 0; o >>= 1) {
    n += __shfl_xor(n, o, 64);
    m += __shfl_xor(m, o, 64);
  }
  wn = n;
  wm = m;
  int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    sn[wid]  = wn;
    sm_[wid] = wm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tn = sn[0] + sn[1] + sn[2] + sn[3];
    unsigned long long tm = sm_[0] + sm_[1] + sm_[2] + sm_[3];
    int const pi = blockIdx.x % kCtrParts;
    if (tn) atomicAdd(&ctr->part[pi][0], tn);
    if (tm) atomicAdd(&ctr->part[pi][1], tm);
  }
}

// top-down: blocks [0, mid_start) -> large queue (block per vertex),
// [mid_start, small_start) -> mid queue (wave per vertex, 4 per block),
// [small_start, grid) -> small queue (4 lanes per vertex, 64 per block)
template <typename V, typename E>
__global__ __launch_bounds__(256) void k_topdown(bfs_args<V, E> a)
{
  CGX_WAVE_STAGE(V, st);
  unsigned long long my_m = 0, my_n = 0;
  long long b = blockIdx.x;
  int tid     = threadIdx.x;
  unsigned long long const n0 = a.ncur_dev ? a.ncur_dev[0] : a.ncur[0];
  unsigned long long const n1 = a.ncur_dev ? a.ncur_dev[1] : a.ncur[1];
  unsigned long long const n2 = a.ncur_dev ? a.ncur_dev[2] : a.ncur[2];
  if (b < a.blk_mid_start) {
    // large class, edge-parallel: every vertex's row is cut into kChunk-edge chunks
    // and the blocks stride over the global chunk index (a root of degree 4e5 would
    // otherwise serialise on one block)
    long long const nb = a.blk_mid_start;
    long long i = 0, chunk_base = 0;
    for (long long c = b;; c += nb) {
      V u = 0;
      E beg = 0, end = 0;
      while (i < (long long)n2) {
        u   = a.qcur[2][i];
        beg = a.off[u];
        end = a.off[u + 1];
        long long nch = ((long long)(end - beg) + kChunk - 1) / kChunk;
        if (c < chunk_base + nch) break;
        chunk_base += nch;
        ++i;
      }
      if (i >= (long long)n2) break;
      E cb = beg + (E)((c - chunk_base) * kChunk);
      E ce = cb + (E)kChunk < end ? cb + (E)kChunk : end;
      for (E base = cb; base < ce; base += 256) {
        E e      = base + tid;
        bool act = e < ce;
        V v      = act ? a.idx[e] : V(0);
        visit_edge<V, E>(a, st, u, v, act, my_m);
      }
    }
  } else if (b < a.blk_small_start) {
    long long nb   = a.blk_small_start - a.blk_mid_start;
    long long widx = (b - a.blk_mid_start) * 4 + (tid >> 6);
    int lane       = tid & 63;
    for (long long i = widx; i < (long long)n1; i += nb * 4) {
      V u   = a.qcur[1][i];
      E beg = a.off[u], end = a.off[u + 1];
      for (E base = beg; base < end; base += 64) {
        E e      = base + lane;
        bool act = e < end;
        V v      = act ? a.idx[e] : V(0);
        visit_edge<V, E>(a, st, u, v, act, my_m);
      }
    }
  } else {
    long long nb  = gridDim.x - a.blk_small_start;
    long long g   = (b - a.blk_small_start) * 64 + (tid >> 2);
    int lane      = tid & 3;
    // all 4 lanes of a group share u; lanes of a wave run the same trip count (<= 4 rounds)
    for (long long i0 = (b - a.blk_small_start) * 64; i0 < (long long)n0; i0 += nb * 64) {
      long long i = i0 + (tid >> 2);
      bool have   = i < (long long)n0;
      V u         = have ? a.qcur[0][i] : V(0);
      E beg = have ? a.off[u] : E(0), end = have ? a.off[u + 1] : E(0);
      for (int r = 0; r < kSmallDeg / 4; ++r) {
        E e      = beg + r * 4 + lane;
        bool act = e < end;
        V v      = act ? a.idx[e] : V(0);
        visit_edge<V, E>(a, st, u, v, act, my_m);
      }
    }
    (void)g;
  }
  (void)my_n;
  stage_flush_all<V, E>(a, st);
  flush_counts(a.ctr, 0, my_m);
}

// mark the next queues as visited (their distances were set by the claim);
// cdev: read the queue lengths on the device (a level the host has not read yet).
// pred + nmap: the queues are a finished top-down level's discoveries, whose
// predecessors (smallest internal id, atomicMin) become external ids here -- every
// such level's output passes through exactly one k_mark_queues (or the final one
// after the loop), so the traversal needs no finishing pass over all vertices
template <typename V>
__global__ void k_mark_queues(V const* q0, unsigned long long n0, V const* q1, unsigned long long n1, V const* q2,
                              unsigned long long n2, uint32_t* vis, uint32_t* fr, bfs_ctr const* cdev, V* pred,
                              V const* nmap)
{
  if (cdev) {
    n0 = cdev->qlen[0];
    n1 = cdev->qlen[1];
    n2 = cdev->qlen[2];
  }
  unsigned long long tot = n0 + n1 + n2;
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < tot;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    V v = i < n0 ? q0[i] : (i < n0 + n1 ? q1[i - n0] : q2[i - n0 - n1]);
    uint32_t bit = 1u << (uint32_t(v) & 31u);
    atomicOr(vis + (v >> 5), bit);
    if (fr) atomicOr(fr + (v >> 5), bit);
    if (nmap) {  // (sources keep -1)
      V const p = pred[v];
      if (p != (V)-1) pred[v] = nmap[p];
    }
  }
}

// The same conversion for a large frontier (queues -> bitmaps before a bottom-up
// level), from the distances instead of the queues: one lane per vertex, 64
// consecutive vertices per wave, visited = reached, frontier = at distance d, both
// written as whole words (no atomics); the frontier's predecessors become external
// ids as in k_mark_queues.  Reads 4 B per vertex where k_mark_queues made two
// scattered atomics per frontier vertex.
template <typename V>
__global__ __launch_bounds__(256) void k_frontier_from_dist(V const* dist, int64_t nv, V d, V inf, uint32_t* vis,
                                                            uint32_t* fr, V* pred, V const* nmap)
{
  int const lane = threadIdx.x & 63;
  int64_t const nchunks = (nv + 63) >> 6;
  for (int64_t c = blockIdx.x * (int64_t)(kBlock / 64) + (threadIdx.x >> 6); c < nchunks;
       c += (int64_t)gridDim.x * (kBlock / 64)) {
    int64_t const v = (c << 6) + lane;
    bool const in   = v < nv;
    V const x       = in ? dist[v] : inf;
    bool const f    = in && x == d;
    if (f && nmap) {
      V const p = pred[v];
      if (p != (V)-1) pred[v] = nmap[p];
    }
    unsigned long long const vb = __ballot(x != inf), fb = __ballot(f);
    if ((lane & 31) == 0 && in) {
      vis[v >> 5] = (uint32_t)(vb >> lane);
      fr[v >> 5]  = (uint32_t)(fb >> lane);
    }
  }
}

typedef int v4i_t __attribute__((ext_vector_type(4)));

// bitmap -> class queues (bottom-up to top-down switch).
// The bitmap is cleared as it is read: while the frontier lives in queues the
// bitmap stays all zero, so a later queues -> bitmap conversion needs no memset.
template <typename V, typename E>
__global__ __launch_bounds__(256) void k_bitmap_to_queues(bfs_args<V, E> a, uint32_t* bm, int64_t nwords)
{
  CGX_WAVE_STAGE(V, st);
  unsigned long long my_m = 0;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < nwords; base += (int64_t)gridDim.x * blockDim.x) {
    int64_t w     = base + threadIdx.x;
    uint32_t word = w < nwords ? bm[w] : 0u;
    if (word) bm[w] = 0u;
    // up to 32 rounds: every lane walks its word's set bits
    for (int r = 0; r < 32; ++r) {
      bool take = word != 0;
      V v       = 0;
      if (take) {
        int bit = __ffs(word) - 1;
        word &= word - 1;
        v = (V)(w * 32 + bit);
      }
      if (!__any(take)) break;
      push_next<V, E>(a, st, v, take, my_m);
    }
  }
  stage_flush_all<V, E>(a, st);
  flush_counts(a.ctr, 0, my_m);
}

// bottom-up step over all vertices (degree-binned schedule)
template <typename V, typename E>
__global__ __launch_bounds__(256) void k_bottomup(bfs_args<V, E> a)
{
  __shared__ int s_hit;
  work_item const it = a.items[blockIdx.x];
  unsigned long long my_n = 0, my_m = 0;
  int tid = threadIdx.x;
  V const nd = (V)(a.depth + 1);
  if (it.width == 256) {
    for (int64_t p = it.begin; p < it.end; ++p) {
      V v = a.order ? a.order[p] : (V)p;
      uint32_t bit = 1u << (uint32_t(v) & 31u);
      if (a.vis[v >> 5] & bit) continue;  // uniform across the block
      E beg = a.off[v], end = a.off[v + 1];
      bool done = false;
      for (E base = beg; base < end && !done; base += 256) {
        if (tid == 0) s_hit = 0x7fffffff;
        __syncthreads();
        E e = base + tid;
        if (e < end) {
          V u = a.idx[e];
          if ((a.fr[u >> 5] >> (uint32_t(u) & 31u)) & 1u) atomicMin(&s_hit, tid);
        }
        __syncthreads();
        int h = s_hit;
        if (h != 0x7fffffff) {
          done = true;
          if (tid == h) {
            V u     = a.idx[e];
            a.dist[v] = nd;
            if (a.pred) a.pred[v] = a.nmap ? a.nmap[u] : u;
            atomicOr(a.nxt + (v >> 5), bit);
            atomicOr(a.vis + (v >> 5), bit);
            my_n += 1;
            my_m += (unsigned long long)(end - beg);
          }
        }
        __syncthreads();
      }
    }
  } else {
    int const w      = it.width;
    int const lane   = tid & (w - 1);
    int const gbase  = (tid & 63) & ~(w - 1);  // first lane of my group within the wave
    int const groups = 256 / w;
    unsigned long long const gmask = (w == 64) ? ~0ull : ((1ull << w) - 1ull);
    // identity order (degree-sorted renumbering): a block step covers <= 256
    // consecutive vertices, so the next/visited bits are gathered in LDS and
    // published with one global atomicOr per 32-vertex word instead of per vertex
    __shared__ uint32_t s_bits[kBlock / 32 + 2];
    bool const agg = a.order == nullptr;
    for (int64_t p0 = it.begin; p0 < it.end; p0 += groups) {
      if (agg) {
        if (tid < kBlock / 32 + 2) s_bits[tid] = 0;
        __syncthreads();
      }
      int64_t p  = p0 + tid / w;
      bool valid = p < it.end;
      V v        = valid ? (a.order ? a.order[p] : (V)p) : V(0);
      uint32_t bit = 1u << (uint32_t(v) & 31u);
      if (valid && (a.vis[v >> 5] & bit)) valid = false;  // same for the whole group
      E beg = valid ? a.off[v] : E(0), end = valid ? a.off[v + 1] : E(0);
      for (E base = beg; base < end; base += w) {
        E e      = base + lane;
        bool hit = false;
        V u      = 0;
        if (e < end) {
          u   = a.idx[e];
          hit = (a.fr[u >> 5] >> (uint32_t(u) & 31u)) & 1u;
        }
        unsigned long long m  = __ballot(hit);
        unsigned long long gm = (m >> gbase) & gmask;
        if (gm) {
          int first = __ffsll((long long)gm) - 1;
          if (lane == first) {
            a.dist[v] = nd;
            if (a.pred) a.pred[v] = a.nmap ? a.nmap[u] : u;
            if (agg) {
              atomicOr(&s_bits[(int64_t(v) >> 5) - (p0 >> 5)], bit);
            } else {
              atomicOr(a.nxt + (v >> 5), bit);
              atomicOr(a.vis + (v >> 5), bit);
            }
            my_n += 1;
            my_m += (unsigned long long)(end - beg);
          }
          break;
        }
      }
      if (agg) {
        __syncthreads();
        if (tid < kBlock / 32 + 2) {
          uint32_t const b = s_bits[tid];
          if (b) {
            int64_t const wd = (p0 >> 5) + tid;
            atomicOr(a.nxt + wd, b);
            atomicOr(a.vis + wd, b);
          }
        }
      }
    }
  }
  flush_counts(a.ctr, my_n, my_m);
}

// Bottom-up in two passes (identity order only, i.e. degree-renumbered graphs).
//
// Adjacency lists are sorted by id and ids descend by degree, so a vertex's first
// neighbours are its hubs, and those are the likeliest to be in the frontier.
//  * probe: one lane per vertex, 64 consecutive vertices per wave.  An unvisited
//    vertex loads its first (up to) 4 neighbours at once and takes the first one in
//    the frontier.  The wave's 64 visited/next bits are two whole words that no
//    other wave touches, written without atomics.  Vertices of degree > 4 that miss
//    go to a residual list.
//  * residual: 16-lane groups scan the rest of those lists (from the 5th neighbour).
// Both take the first hit in sorted order, i.e. the smallest-id frontier
// neighbour, the same predecessor as the one-pass k_bottomup.  (The one-pass kernel
// gives a low-degree vertex a 4..64-lane group, so a wave advances 1..16 vertices
// per dependent load chain.)
#ifndef CGX_BFS_PROBE
#define CGX_BFS_PROBE 8  // RMAT-24 MTEPS: 1: 116K, 2: 129K, 4: 141K, 8: 146K, 16: 142K, 32: 136K
#endif
constexpr int kProbe = CGX_BFS_PROBE;

// The probe's head table (int32 ids): per vertex 16 bytes, its first kHeadN = 3
// neighbours (slots past the list repeat the first) and its degree (clamped to
// 32 bits), so the probe reads 16 contiguous bytes per vertex -- a wave 1 KB in
// one run -- instead of offsets + a 48-byte span at an unaligned place in the
// adjacency, and the chain of dependent loads loses its offsets step.  Fewer
// neighbours per vertex than the adjacency probe's 8 send more vertices to the
// residual scan, and still win: the probe pass reads every unvisited vertex, the
// residual only the misses.
#ifndef CGX_BFS_HEADN
#define CGX_BFS_HEADN 3
#endif
constexpr int kHeadN = CGX_BFS_HEADN;  // 3, 7 or 15 (RMAT-24 ms/traversal: 0.58 / 0.61-0.64 / 0.73)
constexpr int kHeadQ = (kHeadN + 1) / 4;  // 16-byte words per vertex
template <typename E>
__global__ void k_bfs_head(E const* off, int const* idx, int64_t nv, v4i_t* head)
{
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x) {
    E const beg = off[v];
    E const deg = off[v + 1] - beg;
    int w[kHeadN + 1];
#pragma unroll
    for (int t = 0; t < kHeadN; ++t) w[t] = deg > 0 ? idx[beg + (t < deg ? t : 0)] : 0;
    unsigned long long const d = (unsigned long long)deg;
    w[kHeadN] = (int)(uint32_t)(d > 0xffffffffull ? 0xffffffffull : d);
#pragma unroll
    for (int q = 0; q < kHeadQ; ++q) head[kHeadQ * v + q] = v4i_t{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
  }
}

// VEC: a lane's first 8 neighbours from three 16-byte loads of the aligned
// 12-entry span around them (adjacency arrays are padded by 16 entries) instead of
// 8 dword gathers: consecutive lanes' lists are adjacent, so each load instruction
// touches about as many cache lines as one dword gather did.
// HEAD: the first kHeadN neighbours and the degree from the head table (a.head).
template <typename V, typename E, bool VEC, bool HEAD, bool STAGE2>
__global__ __launch_bounds__(256) void k_bu_probe(bfs_args<V, E> a, V* res)
{
  constexpr int NP = HEAD ? kHeadN : kProbe;
  V const nd    = (V)(a.depth + 1);
  int const lane = threadIdx.x & 63;
  unsigned long long my_n = 0, my_m = 0;
  int64_t const nchunks = (a.nv + 63) >> 6;
  int64_t const stride  = (int64_t)gridDim.x * (kBlock / 64);
  int64_t const rcap    = residual_cap(a.nv);
  // A hit's predecessor is stored as an external id one chunk later: its number-map
  // gather is issued ahead of the next chunk's loads, so it adds no step to the
  // chain of dependent loads a chunk is (vis -> offsets -> neighbours -> frontier)
  int64_t pend_v = -1;
  V pend_par     = 0;
  for (int64_t c = blockIdx.x * (int64_t)(kBlock / 64) + (threadIdx.x >> 6); c < nchunks; c += stride) {
    V pend_ext = pend_par;
    if (a.nmap && pend_v >= 0) pend_ext = a.nmap[pend_par];
    int64_t const v  = (c << 6) + lane;
    bool const in    = v < a.nv;
    uint32_t const vw = in ? a.vis[v >> 5] : 0xffffffffu;
    bool const un    = in && !((vw >> (uint32_t(v) & 31u)) & 1u);
    E beg = 0, end = 0;
    int hv[kHeadN + 1] = {};
    if (un) {
      if constexpr (HEAD) {
        v4i_t const* hp = reinterpret_cast<v4i_t const*>(a.head) + kHeadQ * v;
#pragma unroll
        for (int q = 0; q < kHeadQ; ++q) {
          v4i_t const x = hp[q];
          hv[4 * q]     = x.x;
          hv[4 * q + 1] = x.y;
          hv[4 * q + 2] = x.z;
          hv[4 * q + 3] = x.w;
        }
      } else {
        beg = a.off[v];
        end = a.off[v + 1];
      }
    }
    int64_t const deg = HEAD ? (int64_t)(uint32_t)hv[kHeadN] : (int64_t)(end - beg);
    bool hit = false, more = false;
    V par    = 0;
    if (deg > 0) {
      V u[NP];
      if constexpr (HEAD) {
#pragma unroll
        for (int t = 0; t < NP; ++t) u[t] = (V)hv[t];
      } else if constexpr (VEC && sizeof(V) == 4 && kProbe == 8) {
        E const a0   = beg & ~E(3);
        int const sh = (int)(beg - a0);
        v4i_t const* p = reinterpret_cast<v4i_t const*>(a.idx + a0);
        v4i_t const c0 = p[0], c1 = p[1], c2 = p[2];
        int const wv[12] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w};
#pragma unroll
        for (int t = 0; t < kProbe; ++t) {
          int const x = sh == 0 ? wv[t] : sh == 1 ? wv[t + 1] : sh == 2 ? wv[t + 2] : wv[t + 3];
          u[t]        = (V)x;
        }
#pragma unroll
        for (int t = 1; t < kProbe; ++t) u[t] = t < deg ? u[t] : u[0];  // past the list: another list or padding
      } else {
#pragma unroll
        for (int t = 0; t < kProbe; ++t) u[t] = a.idx[beg + (t < deg ? t : 0)];
      }
      uint32_t fw[NP];  // all frontier words first: the loads issue back to back
#pragma unroll
      for (int t = 0; t < NP; ++t) fw[t] = a.fr[u[t] >> 5];
      uint32_t hm = 0;
#pragma unroll
      for (int t = 0; t < NP; ++t) hm |= (t < deg ? (fw[t] >> (uint32_t(u[t]) & 31u)) & 1u : 0u) << t;
#pragma unroll
      for (int t = NP - 1; t >= 0; --t)  // the lowest hit wins: the smallest-id frontier neighbour
        if ((hm >> t) & 1u) par = u[t];
      hit  = hm != 0;
      more = !hit && deg > NP;
      if constexpr (HEAD && STAGE2 && sizeof(V) == 4) {
        // the head missed: the next kProbe neighbours from the adjacency (three 16-byte
        // loads, as the VEC probe) before the vertex goes to the residual scan
        if (more) {
          E const b2    = a.off[v] + kHeadN;
          E const a0    = b2 & ~E(3);
          int const sh  = (int)(b2 - a0);
          int64_t const rem = deg - kHeadN;
          v4i_t const* p = reinterpret_cast<v4i_t const*>(a.idx + a0);
          v4i_t const c0 = p[0], c1 = p[1], c2 = p[2];
          int const wv[12] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w};
          V w2[kProbe];
#pragma unroll
          for (int t = 0; t < kProbe; ++t)
            w2[t] = (V)(sh == 0 ? wv[t] : sh == 1 ? wv[t + 1] : sh == 2 ? wv[t + 2] : wv[t + 3]);
#pragma unroll
          for (int t = 1; t < kProbe; ++t) w2[t] = t < rem ? w2[t] : w2[0];
          uint32_t f2[kProbe];
#pragma unroll
          for (int t = 0; t < kProbe; ++t) f2[t] = a.fr[w2[t] >> 5];
          uint32_t h2 = 0;
#pragma unroll
          for (int t = 0; t < kProbe; ++t) h2 |= (t < rem ? (f2[t] >> (uint32_t(w2[t]) & 31u)) & 1u : 0u) << t;
#pragma unroll
          for (int t = kProbe - 1; t >= 0; --t)
            if ((h2 >> t) & 1u) par = w2[t];
          hit  = h2 != 0;
          more = !hit && rem > kProbe;
        }
      }
    }
    if (a.pred && pend_v >= 0) a.pred[pend_v] = pend_ext;
    pend_v = -1;
    if (hit) {
      a.dist[v] = nd;
      pend_v   = v;
      pend_par = par;
      my_n += 1;
      my_m += (unsigned long long)deg;
    }
    unsigned long long const hm = __ballot(hit);
    if ((lane & 31) == 0 && in) {
      uint32_t const b = (uint32_t)(hm >> lane);  // this half-wave's word
      if (b) a.vis[v >> 5] = vw | b;
      a.nxt[v >> 5] = b;  // every word of nxt is written here: no memset before the probe
    }
    unsigned long long const mm = __ballot(more);
    if (mm) {
      unsigned long long base = 0;
      int const leader = __ffsll((long long)mm) - 1;
      int const sq = (int)(c % kCtrParts);
      if (lane == leader) base = atomicAdd(&a.ctr->part[sq][2], (unsigned long long)__popcll(mm));
      base = __shfl(base, leader, 64);
      if (more) res[sq * rcap + (int64_t)base + __popcll(mm & ((1ull << lane) - 1ull))] = (V)v;
    }
  }
  if (a.pred && pend_v >= 0) a.pred[pend_v] = a.nmap ? a.nmap[pend_par] : pend_par;
  flush_counts(a.ctr, my_n, my_m);
}

template <typename V, typename E>
__global__ __launch_bounds__(256) void k_bu_residual(bfs_args<V, E> a, V const* res)
{
#ifndef CGX_BFS_RES_W
#define CGX_BFS_RES_W 16
#endif
  constexpr int w = CGX_BFS_RES_W;
  static_assert(w >= 2 && w <= 32 && (w & (w - 1)) == 0, "residual group width: a power of two in [2, 32]");
  V const nd       = (V)(a.depth + 1);
  int const tid    = threadIdx.x;
  int const lane   = tid & (w - 1);
  int const gbase  = (tid & 63) & ~(w - 1);
  // the probe's sub-queues (written by an earlier launch), concatenated
  __shared__ unsigned long long s_pre[kCtrParts + 1];
  if (tid == 0) {
    s_pre[0] = 0ull;
    for (int p = 0; p < kCtrParts; ++p) s_pre[p + 1] = s_pre[p] + a.ctr->part[p][2];
  }
  __syncthreads();
  int64_t const n    = (int64_t)s_pre[kCtrParts];
  int64_t const rcap = residual_cap(a.nv);
  int64_t const ng   = (int64_t)gridDim.x * (kBlock / w);
  unsigned long long my_n = 0, my_m = 0;
  for (int64_t i = blockIdx.x * (int64_t)(kBlock / w) + tid / w; i < n; i += ng) {
    int p = 0;
    while ((unsigned long long)i >= s_pre[p + 1]) ++p;
    V const v     = res[p * rcap + (i - (int64_t)s_pre[p])];
    E const beg0  = a.off[v];
    E const end   = a.off[v + 1];
    for (E base = beg0 + (a.head ? (a.head2 ? kHeadN + kProbe : kHeadN) : kProbe); base < end; base += w) {
      E const e = base + lane;
      bool hit  = false;
      V u       = 0;
      if (e < end) {
        u   = a.idx[e];
        hit = (a.fr[u >> 5] >> (uint32_t(u) & 31u)) & 1u;
      }
      unsigned long long const gm = (__ballot(hit) >> gbase) & ((1ull << w) - 1ull);
      if (gm) {
        if (lane == __ffsll((long long)gm) - 1) {
          uint32_t const bit = 1u << (uint32_t(v) & 31u);
          a.dist[v] = nd;
          if (a.pred) a.pred[v] = a.nmap ? a.nmap[u] : u;
          atomicOr(a.nxt + (v >> 5), bit);
          atomicOr(a.vis + (v >> 5), bit);
          my_n += 1;
          my_m += (unsigned long long)(end - beg0);
        }
        break;
      }
    }
  }
  flush_counts(a.ctr, my_n, my_m);
}

// dist = INF, pred = -1, the result's vertex ids (the number map) and the three
// bitmaps cleared in one launch (was 2 fills + 3 memsets + a copy)
template <typename V>
__global__ void k_bfs_setup(V* dist, V* pred, int64_t nv, V inf, uint32_t* vis, uint32_t* fr, uint32_t* nxt,
                            int64_t nwords, int* bad, V const* nmap, V* vout)
{
  int64_t const stride = (int64_t)gridDim.x * blockDim.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) *bad = 0;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv; v += stride) {
    dist[v] = inf;
    if (pred) pred[v] = (V)-1;
    vout[v] = nmap[v];
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nwords; i += stride) {
    vis[i] = 0u;
    fr[i]  = 0u;
    nxt[i] = 0u;
  }
}

// distance 0, visited and frontier bits of every valid source
template <typename V>
__global__ void k_bfs_sources(V* dist, V const* src, size_t ns, int64_t nv, int* bad, uint32_t* vis, uint32_t* fr)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < ns; i += (size_t)gridDim.x * blockDim.x) {
    V s = src[i];
    if (s < 0 || (int64_t)s >= nv) {
      atomicAdd(bad, 1);
      continue;
    }
    dist[s] = 0;
    atomicOr(vis + (s >> 5), 1u << (uint32_t(s) & 31u));
    atomicOr(fr + (s >> 5), 1u << (uint32_t(s) & 31u));
  }
}

// Quick start (level 0 certainly top-down): the sources straight into the degree-class
// queues, their lengths and the sources' edge count in c (as k_bitmap_to_queues
// leaves them) -- one small launch instead of the bitmap pass over all V / 32 words
// (k_bfs_sources + k_bitmap_to_queues); the frontier bitmap is never set.  A
// repeated source is dropped by the visited bit it finds already set.
template <typename V, typename E>
__global__ void k_bfs_sources_q(V* dist, V const* src, size_t ns, int64_t nv, int* bad, uint32_t* vis, E const* off,
                                V* q0, V* q1, V* q2, bfs_ctr* c)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < ns; i += (size_t)gridDim.x * blockDim.x) {
    V const x = src[i];
    if (x < 0 || (int64_t)x >= nv) {
      atomicAdd(bad, 1);
      continue;
    }
    uint32_t const bit = 1u << (uint32_t(x) & 31u);
    if (atomicOr(vis + (x >> 5), bit) & bit) continue;
    dist[x]       = 0;
    E const deg   = off[x + 1] - off[x];
    int const cls = deg <= kSmallDeg ? 0 : (deg <= kMidDeg ? 1 : 2);
    unsigned long long const pos = atomicAdd(&c->qlen[cls], 1ull);
    (cls == 0 ? q0 : cls == 1 ? q1 : q2)[pos] = x;
    atomicAdd(&c->next_m, (unsigned long long)deg);
  }
}

template <typename V, typename E, typename W>
void bfs_impl(handle_t& h, graph_t& g, array_view_t* sources, bool dir_opt, size_t depth_limit, bool want_pred,
              bool expensive, paths_result_t& res)
{
  hipStream_t s = h.stream;
  int64_t nv    = g.num_vertices;
  CGX_INPUT(sources->size > 0, "Invalid input argument: input should have at least one source");
  CGX_INPUT(!dir_opt || g.symmetric,
            "Invalid input argument: input graph should be symmetric for direction optimizing BFS.");
  (void)expensive;
  // sources: external -> internal, in place (c_api/bfs.cpp:96-114)
  // ids not in the graph become -1 and are reported by k_bfs_sources' range check
  // (no host round trip here)
  if (g.renumbered) renumber_ext_to_int_unchecked(h, g, sources->data, sources->size);
  V const INF = std::numeric_limits<V>::max();
  // the result's vertex ids: the number map, copied by k_bfs_setup (one pass with the initialisation)
  res.vertices  = std::make_unique<device_array_t>((size_t)nv, g.vertex_type, s);
  res.distances = std::make_unique<device_array_t>((size_t)nv, dtype_of<V>(), s);
  res.predecessors = std::make_unique<device_array_t>(want_pred ? (size_t)nv : 0, dtype_of<V>(), s);
  V* dist = res.distances->buf.data<V>();
  V* pred = want_pred ? res.predecessors->buf.data<V>() : nullptr;
  h.last_bfs_levels    = 0;
  h.last_bfs_bottom_up = 0;
  if (nv == 0) return;

  adjacency_t& adj = ensure_adjacency(h, g, false);
  if (dir_opt) ensure_schedule(h, g, adj);

  int64_t nwords = (nv + 31) / 32;
  dbuf<uint32_t> vis(nwords, s), fr(nwords, s), nxt(nwords, s);
  dbuf<int> bad(1, s);
  hipLaunchKernelGGL(k_bfs_setup<V>, dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, dist, pred, nv, INF,
                     vis.data(), fr.data(), nxt.data(), nwords, bad.data(), g.number_map.data<V>(),
                     res.vertices->buf.data<V>());
  CGX_LAUNCH_CHECK();
  dbuf<V> qa[3], qb[3];
  for (int c = 0; c < 3; ++c) {
    qa[c].resize(nv, s);
    qb[c].resize(c == 0 ? std::max<int64_t>(nv, kCtrParts * residual_cap(nv)) : nv, s);  // qb[0]: residual sub-queues too
  }
  // ctr2: queue lengths of a bitmap -> queues conversion; ctr3: a speculative level's counters
  // one allocation and one memset for the three counter blocks; k_publish_seq
  // zeroes ctr and ctr3 after every read, so they stay clean without more memsets
  dbuf<bfs_ctr> ctrs(4, s);  // (+ ctr4: a second speculative bottom-up level's counters)
  HIP_CHECK(hipMemsetAsync(ctrs.data(), 0, 4 * sizeof(bfs_ctr), s));
  struct ctr_ref {
    bfs_ctr* p;
    bfs_ctr* data() const { return p; }
  };
  ctr_ref const ctr{ctrs.data()}, ctr2{ctrs.data() + 1}, ctr3{ctrs.data() + 2}, ctr4{ctrs.data() + 3};
  bfs_ctr_hdr* hctr = h.pinned_as<bfs_ctr_hdr>();

  bfs_args<V, E> a{};
  a.off   = adj.offsets.data<E>();
  a.idx   = adj.indices.data<V>();
  a.dist  = dist;
  a.pred  = pred;
  a.vis   = vis.data();
  a.fr    = fr.data();
  a.nxt   = nxt.data();
  a.ctr   = ctr.data();
  a.nv    = nv;
  a.order = (dir_opt && !adj.degree_sorted) ? adj.order.data<V>() : nullptr;
  a.items = dir_opt ? adj.items.data<work_item>() : nullptr;
  a.nmap  = (pred && g.renumbered) ? g.number_map.data<V>() : nullptr;
  // Level counters: k_publish_seq into the handle's coherent block and a host spin on
  // its sequence word -- no hipStreamSynchronize per level (measured against a D2H
  // copy + synchronize per level: that form was removed)
  bfs_ctr_hdr* pctr = h.polled_as<bfs_ctr_hdr>();  // [0]: a level, [1]: a speculative level
  // ctr_b / src_m: see k_publish_seq
  auto read_ctr = [&](int const* bad_flag = nullptr, bfs_ctr* ctr_b = nullptr, bfs_ctr* src_m = nullptr,
                      bfs_ctr* ctr_c = nullptr) {
    {
      unsigned long long const seq = __atomic_load_n(&pctr->pad[0], __ATOMIC_ACQUIRE) + 1;
      hipLaunchKernelGGL(k_publish_seq, dim3(1), dim3(64), 0, s, ctr.data(), pctr, seq, bad_flag, ctr_b, src_m, ctr_c);
      CGX_LAUNCH_CHECK();
      for (unsigned long long n = 1; __atomic_load_n(&pctr->pad[0], __ATOMIC_ACQUIRE) != seq; ++n) {
        __builtin_ia32_pause();
        if ((n & 0xfffff) == 0) {  // ~every few ms: the stream must still be running, or done
          hipError_t const q = hipStreamQuery(s);
          if (q != hipSuccess && q != hipErrorNotReady) HIP_CHECK(q);
          if (q == hipSuccess && __atomic_load_n(&pctr->pad[0], __ATOMIC_ACQUIRE) != seq)
            throw std::runtime_error("BFS: level counters not published");
        }
      }
      std::memcpy(hctr, pctr, sizeof(bfs_ctr_hdr));
    }
  };

  try {
    // the source check comes back with the first counters (one host round trip
    // fewer); invalid ids are skipped by the source kernels
    for (int c = 0; c < 3; ++c) a.qnext[c] = qa[c].data();
    // Level 0 is certainly top-down when even every source at the maximum degree
    // stays below the switch rule: then the source counts are not read here -- level
    // 0 takes its queue lengths on the device (as after a bitmap -> queues
    // conversion) and the source check and the sources' edge count come back with
    // level 0's counters (one host round trip fewer)
    tuning_t const& tu    = h.tune;
    double const alpha_do = tu.bfs_alpha;
    bool quick_start      = false;
    if (adj.degree_sorted) {
      if (adj.max_degree < 0) {
        E o[2];
        HIP_CHECK(hipMemcpyAsync(o, adj.offsets.data<E>(), sizeof(o), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        adj.max_degree = (int64_t)(o[1] - o[0]);  // vertex 0 has the largest degree
      }
      double const m_src = (double)sources->size * (double)adj.max_degree;
      quick_start        = !dir_opt || m_src <= ((double)g.num_edges - m_src) / alpha_do;
    }
    unsigned long long ncur[3];
    unsigned long long n_f, m_f, m_u;
    bool pending_src = false;  // level 0's read also returns the source check and the sources' edge count
    if (quick_start) {  // (ctr2 is still zero from the allocation memset)
      hipLaunchKernelGGL((k_bfs_sources_q<V, E>), dim3(grid_for(sources->size, kBlock, 1024)), dim3(kBlock), 0, s,
                         dist, sources->as<V>(), sources->size, nv, bad.data(), vis.data(), a.off, qa[0].data(),
                         qa[1].data(), qa[2].data(), ctr2.data());
      CGX_LAUNCH_CHECK();
      for (int c = 0; c < 3; ++c) ncur[c] = sources->size;  // bounds: the grid covers every class
      a.ncur_dev = reinterpret_cast<unsigned long long const*>(ctr2.data());
      n_f        = sources->size;
      m_f        = 0;  // counted into m_u when level 0's counters come back
      m_u        = (unsigned long long)g.num_edges;
      pending_src = true;
    } else {
      // sources -> distance 0, visited, frontier bitmap; then bitmap -> queues
      hipLaunchKernelGGL(k_bfs_sources<V>, dim3(grid_for(sources->size, kBlock, 1024)), dim3(kBlock), 0, s, dist,
                         sources->as<V>(), sources->size, nv, bad.data(), vis.data(), fr.data());
      CGX_LAUNCH_CHECK();
      hipLaunchKernelGGL((k_bitmap_to_queues<V, E>), dim3(grid_for(nwords, kBlock, 4096)), dim3(kBlock), 0, s, a,
                         fr.data(), nwords);
      CGX_LAUNCH_CHECK();
      read_ctr(bad.data());
      CGX_INPUT(pctr->pad[1] == 0, "Invalid input argument: sources have invalid vertex IDs.");
      for (int c = 0; c < 3; ++c) ncur[c] = hctr->qlen[c];
      n_f = ncur[0] + ncur[1] + ncur[2];
      m_f = hctr->next_m;
      m_u = (unsigned long long)g.num_edges - m_f;
    }
    bool bottom_up  = false;
    bool have_queue = true;  // frontier available as queues (qa); else as bitmap fr
    bool have_bitmap = false; // frontier bitmap fr valid (else fr is all zero: k_bitmap_to_queues clears it)
    V depth = 0;
    V limit = (V)std::min<unsigned long long>((unsigned long long)depth_limit,
                                              (unsigned long long)std::numeric_limits<V>::max());
    size_t levels = 0, bu_steps = 0;
    int bu_phase = 0;  // bottom-up levels since the last top-down one
    bool const dbg = std::getenv("CGX_BFS_DEBUG") != nullptr;  // measurement only
    // probe neighbours by 16-byte loads (needs the padded adjacency, int32 ids; RMAT-24
    // k_bu_probe 133.6 -> 129.5 us average; bfs_probe_vec = 0: dword gathers, A/B)
    bool const probe_vec = adj.idx_padded && tu.bfs_probe_vec;
    // the probe's head table (bfs_head = 0: the adjacency probe, A/B; RMAT-24 0.579 vs 0.666 ms)
    if constexpr (sizeof(V) == 4) {
      if (dir_opt && a.order == nullptr && tu.bfs_head) {
        if (adj.bfs_head.empty()) {
          adj.bfs_head = buffer((size_t)nv * 16 * kHeadQ, s);
          hipLaunchKernelGGL(k_bfs_head<E>, dim3(grid_for(nv, kBlock, 8192)), dim3(kBlock), 0, s, a.off,
                             reinterpret_cast<int const*>(a.idx), nv, adj.bfs_head.data<v4i_t>());
          CGX_LAUNCH_CHECK();
        }
        a.head = adj.bfs_head.data<int>();
        // head misses then probe neighbours 3..10 in the adjacency (RMAT-24 0.537-0.545 vs
        // 0.591-0.595 ms without: root 7's first bottom-up level, a frontier few vertices
        // find among their first 3 neighbours, 0.90 -> 0.66 ms)
        a.head2 = probe_vec;
      }
    }
    // Grid sizes: every block ends with same-address atomics on the level counters,
    // which serialise at the memory side (≈8 ns each): RMAT-24 MTEPS with the probe
    // on 512 / 1024 / 2048 / 8192 / 32768 blocks: 166K / 173K / 168K / 148K / 101K
    unsigned const residual_grid = (unsigned)std::max(1, tu.bfs_res_grid);
    // (top-down segments capped at 1024 blocks each: 176.5K vs 148K MTEPS uncapped; 256-2048 within noise)
    long long const td_cap = std::max<int64_t>(1, tu.bfs_td_cap);
    // probe grid: with the level counters spread over kCtrParts slots the block-end
    // atomics no longer serialise, and more waves hide the probe's dependent loads
    // (RMAT-24, 3 reps x 8 roots: 1024 / 2048 / 4096 blocks = 318K / 335K / 339K MTEPS)
    unsigned const probe_grid = (unsigned)std::max(1, tu.bfs_probe_grid);
    // Direction switch thresholds (Beamer's form).  Our bottom-up is cheap per edge
    // (hub-first adjacency, early exit), so it pays to stay top-down longer and
    // bottom-up longer than Beamer's alpha 14 / beta 24.  RMAT-24 harmonic-mean MTEPS
    // (alpha, beta): (4, 24) 135K; (14, 24) 211K; (14, 64) 218K; (40, 24) 224K;
    // (40, 64) 226K; (80, 64) 223K; (80, 128) 225K; (150, 64) 209K.
    // tuning_t overrides are measurement only.
    double const beta_do  = tu.bfs_beta;
    // The switch rule, in one place: the direction of the level whose frontier has n_f
    // vertices and m_f edges (m_u unexplored edges) after a level run bottom-up (cur_bu)
    // or top-down.  Also the "next level is bottom-up" test after a top-down level,
    // which decides which kernel turns that level's predecessors into external ids
    // (k_mark_queues now, or k_frontier_from_dist / k_mark_queues at the next level's
    // conversion) -- so both uses must agree, and they do by calling this.
    auto next_dir_bu = [&](bool cur_bu, unsigned long long nf, unsigned long long mf, unsigned long long mu) {
      if (!dir_opt) return false;
      if (!cur_bu) return (double)mf > (double)mu / alpha_do;
      return !((double)nf < (double)nv / beta_do);
    };
    while (n_f > 0 && depth < limit) {
      auto tl = std::chrono::steady_clock::now();
      bottom_up = next_dir_bu(bottom_up, n_f, m_f, m_u);
      a.depth = depth;  // (k_publish_seq zeroed the counters it read)
      if (bottom_up) {
        if (!have_bitmap) {  // queues -> frontier bitmap (fr is all zero here)
          // a frontier above V / 32 from the distances (RMAT-24: 0.516-0.517 vs 0.542 ms per
          // traversal from the queues; root 3's conversion 107 us of atomics)
          if ((double)n_f * 32.0 > (double)nv) {
            hipLaunchKernelGGL(k_frontier_from_dist<V>, dim3(grid_for((nv + 63) / 64, kBlock / 64, 4096)), dim3(kBlock),
                               0, s, dist, nv, depth, INF, vis.data(), fr.data(), pred, a.nmap);
          } else {
            hipLaunchKernelGGL(k_mark_queues<V>, dim3(grid_for(n_f, kBlock, 4096)), dim3(kBlock), 0, s, qa[0].data(),
                               ncur[0], qa[1].data(), ncur[1], qa[2].data(), ncur[2], vis.data(), fr.data(), nullptr,
                               pred, a.nmap);
          }
          CGX_LAUNCH_CHECK();
          have_bitmap = true;
        }
        bool const probe_path = a.order == nullptr;  // (else the one-pass k_bottomup: no identity order)
        auto bu_level = [&](bfs_args<V, E> const& x) {
          if (probe_path) {  // probe + residual (identity order)
            // (measured and rejected: two chunks per wave in flight, 337K vs 370K MTEPS on
            // RMAT-24 -- the probe is not bound by one wave's load chain)
            unsigned const pg = grid_for((nv + 63) / 64, kBlock / 64, probe_grid);
            if (x.head && x.head2)
              hipLaunchKernelGGL((k_bu_probe<V, E, false, true, true>), dim3(pg), dim3(kBlock), 0, s, x, qb[0].data());
            else if (x.head)
              hipLaunchKernelGGL((k_bu_probe<V, E, false, true, false>), dim3(pg), dim3(kBlock), 0, s, x, qb[0].data());
            else if (probe_vec)
              hipLaunchKernelGGL((k_bu_probe<V, E, true, false, false>), dim3(pg), dim3(kBlock), 0, s, x, qb[0].data());
            else
              hipLaunchKernelGGL((k_bu_probe<V, E, false, false, false>), dim3(pg), dim3(kBlock), 0, s, x, qb[0].data());
            CGX_LAUNCH_CHECK();
            hipLaunchKernelGGL((k_bu_residual<V, E>), dim3(residual_grid), dim3(kBlock), 0, s, x, qb[0].data());
          } else {
            HIP_CHECK(hipMemsetAsync(x.nxt, 0, nwords * 4, s));  // (the probe writes every word itself)
            hipLaunchKernelGGL((k_bottomup<V, E>), dim3(adj.num_items), dim3(kBlock), 0, s, x);
          }
          CGX_LAUNCH_CHECK();
        };
        bu_level(a);
        // A bottom-up phase's first level is followed by two more bottom-up levels (the
        // first two levels leave frontiers far above nv / beta on every bench root):
        // those are launched at once, each on the bitmap the level before writes and
        // with its own counters, and all three come back with one host round trip.
        // The direction changes no result, so a wrong guess costs time only.  RMAT-24:
        // 0.669-0.672 ms per traversal against 0.682 with one speculated level (same box).
        int const nspec = dir_opt && bu_phase == 0 ? (int)std::min<long long>(2, (long long)limit - depth - 1) : 0;
        if (nspec > 0) {
          bfs_ctr* const sctr[2] = {ctr3.data(), ctr4.data()};
          bfs_args<V, E> x       = a;
          for (int j = 0; j < nspec; ++j) {
            x.depth = (V)(depth + 1 + j);
            x.ctr   = sctr[j];
            std::swap(x.fr, x.nxt);  // reads the level before's discoveries, rewrites the older bitmap whole
            bu_level(x);
          }
          read_ctr(nullptr, ctr3.data(), nullptr, nspec > 1 ? ctr4.data() : nullptr);
          bfs_ctr_hdr const lv[3] = {*hctr, pctr[1], pctr[2]};
          bool over = false;
          for (int j = 0; j < nspec; ++j) {
            n_f = lv[j].next_n;
            m_f = lv[j].next_m;
            if (dbg)
              std::fprintf(stderr, "[bfs] level %d bottom-up n_f=%llu m_f=%llu m_u=%llu (speculated next)\n",
                           (int)depth, n_f, m_f, m_u);
            m_u = m_u > m_f ? m_u - m_f : 0;
            ++depth;
            ++levels;
            ++bu_steps;
            if (n_f == 0) {  // (the later levels ran on an empty frontier)
              over = true;
              break;
            }
          }
          if (over) break;
          n_f = lv[nspec].next_n;  // the last level's
          m_f = lv[nspec].next_m;
          if (nspec % 2 == 0) {  // an odd number of levels: the frontier is in nxt
            std::swap(a.fr, a.nxt);
            std::swap(fr, nxt);
          }
          have_queue = false;
          bu_phase += nspec + 1;
        } else {
          read_ctr();
          std::swap(a.fr, a.nxt);
          std::swap(fr, nxt);
          have_queue = false;
          n_f = hctr->next_n;
          m_f = hctr->next_m;
          ++bu_phase;
        }
        ++bu_steps;
      } else {
        bu_phase = 0;
        if (!have_queue) {
          // frontier bitmap -> queues with no host round trip: the conversion counts
          // into ctr2, k_topdown reads the queue lengths from there and the grid is
          // sized for all n_f frontier vertices in every degree class
          for (int c = 0; c < 3; ++c) a.qnext[c] = qa[c].data();
          HIP_CHECK(hipMemsetAsync(ctr2.data(), 0, sizeof(bfs_ctr), s));
          bfs_args<V, E> ac = a;
          ac.ctr            = ctr2.data();
          hipLaunchKernelGGL((k_bitmap_to_queues<V, E>), dim3(grid_for(nwords, kBlock, 4096)), dim3(kBlock), 0, s,
                             ac, fr.data(), nwords);
          CGX_LAUNCH_CHECK();
          for (int c = 0; c < 3; ++c) ncur[c] = n_f;
          a.ncur_dev = reinterpret_cast<unsigned long long const*>(ctr2.data());  // bfs_ctr::qlen, offset 0
          have_queue = true;
        }
        for (int c = 0; c < 3; ++c) {
          a.qcur[c]  = qa[c].data();
          a.ncur[c]  = ncur[c];
          a.qnext[c] = qb[c].data();
        }
        long long nb_large = ncur[2] ? (long long)std::min<unsigned long long>(std::max<unsigned long long>(ncur[2] * 8, 256), 4096) : 0;
        long long nb_mid   = (long long)std::min<unsigned long long>((ncur[1] + 3) / 4, 4096);
        long long nb_small = (long long)std::min<unsigned long long>((ncur[0] + 63) / 64, 8192);
        nb_large = std::min(nb_large, td_cap);
        nb_mid   = std::min(nb_mid, td_cap);
        nb_small = std::min(nb_small, td_cap);
        a.blk_mid_start    = nb_large;
        a.blk_small_start  = nb_large + nb_mid;
        long long grid     = nb_large + nb_mid + nb_small;
        if (grid > 0) {
          hipLaunchKernelGGL((k_topdown<V, E>), dim3(grid), dim3(kBlock), 0, s, a);
          CGX_LAUNCH_CHECK();
        }
        a.ncur_dev = nullptr;
        // Speculative next level: once a bottom-up phase is over the frontier only
        // shrinks, so the level after this one is launched top-down before this one's
        // counters are read (its queue lengths read on the device, its grid that of
        // this level, every class at least one segment), and both levels come back
        // with one host round trip.  Results do not depend on the direction schedule
        // (smallest-id parent either way), so a wrong guess costs time only.
        bool const spec = bu_steps > 0 && !pending_src && depth + 1 < limit;
        if (spec) {
          // this level's new frontier is the next level's visited set
          hipLaunchKernelGGL(k_mark_queues<V>, dim3(grid_for(n_f, kBlock, 4096)), dim3(kBlock), 0, s, qb[0].data(),
                             0ull, qb[1].data(), 0ull, qb[2].data(), 0ull, vis.data(), nullptr, ctr.data(), pred,
                             a.nmap);
          CGX_LAUNCH_CHECK();
          bfs_args<V, E> b = a;
          b.depth          = (V)(depth + 1);
          b.ctr            = ctr3.data();
          b.ncur_dev       = reinterpret_cast<unsigned long long const*>(ctr.data());
          for (int c = 0; c < 3; ++c) {
            b.qcur[c]  = qb[c].data();
            b.qnext[c] = qa[c].data();
          }
          long long const sl = std::max(nb_large, 8ll), sm = std::max(nb_mid, 8ll), ss = std::max(nb_small, 8ll);
          b.blk_mid_start    = sl;
          b.blk_small_start  = sl + sm;
          hipLaunchKernelGGL((k_topdown<V, E>), dim3(sl + sm + ss), dim3(kBlock), 0, s, b);
          CGX_LAUNCH_CHECK();
          read_ctr(nullptr, ctr3.data());
          bfs_ctr_hdr const l2 = pctr[1];
          unsigned long long const n1 = hctr->qlen[0] + hctr->qlen[1] + hctr->qlen[2];
          unsigned long long const m1 = hctr->next_m;
          if (dbg)
            std::fprintf(stderr, "[bfs] level %d top-down n_f=%llu m_f=%llu m_u=%llu (speculated next)\n", (int)depth,
                         n1, m1, m_u);
          m_u = m_u > m1 ? m_u - m1 : 0;
          ++depth;
          ++levels;
          // the speculative level (empty when this one found nothing): its output is in qa
          for (int c = 0; c < 3; ++c) ncur[c] = l2.qlen[c];
          n_f = ncur[0] + ncur[1] + ncur[2];
          m_f = l2.next_m;
          if (n1 == 0) {  // nothing was discovered: the traversal is over
            n_f = 0;
            m_f = 0;
            break;
          }
          unsigned long long const m_u_next = m_u > m_f ? m_u - m_f : 0;
          bool const next_bu = next_dir_bu(false, n_f, m_f, m_u_next);
          bool const last    = n_f == 0 || depth + 1 >= limit;
          if (!last && !next_bu) {
            hipLaunchKernelGGL(k_mark_queues<V>, dim3(grid_for(n_f, kBlock, 4096)), dim3(kBlock), 0, s,
                               qa[0].data(), ncur[0], qa[1].data(), ncur[1], qa[2].data(), ncur[2], vis.data(),
                               nullptr, nullptr, pred, a.nmap);
            CGX_LAUNCH_CHECK();
          }
          have_bitmap = false;
          if (dbg)
            std::fprintf(stderr, "[bfs] level %d top-down n_f=%llu m_f=%llu m_u=%llu (speculative)\n", (int)depth,
                         n_f, m_f, m_u);
          m_u = m_u > m_f ? m_u - m_f : 0;
          ++depth;
          ++levels;
          continue;
        }
        read_ctr(pending_src ? bad.data() : nullptr, nullptr, pending_src ? ctr2.data() : nullptr);
        if (pending_src) {  // level 0 also brought back the source check and the sources' edge count
          CGX_INPUT(pctr->pad[1] == 0, "Invalid input argument: sources have invalid vertex IDs.");
          unsigned long long const m_src = pctr->pad[2];
          m_u         = m_u > m_src ? m_u - m_src : 0;
          pending_src = false;
        }
        for (int c = 0; c < 3; ++c) ncur[c] = hctr->qlen[c];
        n_f = ncur[0] + ncur[1] + ncur[2];
        m_f = hctr->next_m;
        // The new frontier's visited bits are needed only by a next top-down level: a
        // next bottom-up level marks them with its frontier bitmap (queues -> bitmap
        // above), and after the last level nothing reads them
        unsigned long long const m_u_next = m_u > m_f ? m_u - m_f : 0;
        bool const next_bu   = next_dir_bu(false, n_f, m_f, m_u_next);
        bool const last      = n_f == 0 || depth + 1 >= limit;
        if (!last && !next_bu) {
          hipLaunchKernelGGL(k_mark_queues<V>, dim3(grid_for(n_f, kBlock, 4096)), dim3(kBlock), 0, s, qb[0].data(),
                             ncur[0], qb[1].data(), ncur[1], qb[2].data(), ncur[2], vis.data(), nullptr, nullptr,
                             pred, a.nmap);
          CGX_LAUNCH_CHECK();
        }
        for (int c = 0; c < 3; ++c) std::swap(qa[c], qb[c]);
        have_bitmap = false;
      }
      if (dbg)
        std::fprintf(stderr, "[bfs] level %d %s n_f=%llu m_f=%llu m_u=%llu %.1f us\n", (int)depth,
                     bottom_up ? "bottom-up" : "top-down", n_f, m_f, m_u,
                     1e6 * std::chrono::duration<double>(std::chrono::steady_clock::now() - tl).count());
      m_u = m_u > m_f ? m_u - m_f : 0;
      ++depth;
      ++levels;
    }
    if (pending_src) {  // no level ran (depth limit 0): the source check is still owed
      read_ctr(bad.data());
      CGX_INPUT(pctr->pad[1] == 0, "Invalid input argument: sources have invalid vertex IDs.");
    }
    // a depth limit ended the loop on a top-down level's discoveries: their
    // predecessors to external ids (bottom-up levels wrote external ids already)
    if (a.nmap && have_queue && n_f > 0 && levels > 0) {
      hipLaunchKernelGGL(k_mark_queues<V>, dim3(grid_for(n_f, kBlock, 4096)), dim3(kBlock), 0, s, qa[0].data(),
                         ncur[0], qa[1].data(), ncur[1], qa[2].data(), ncur[2], vis.data(), nullptr, nullptr, pred,
                         a.nmap);
      CGX_LAUNCH_CHECK();
    }
    h.last_bfs_levels    = levels;
    h.last_bfs_bottom_up = bu_steps;
  } catch (...) {
    throw;
  }
}

}  // namespace

void run_bfs(handle_t& h, graph_t& g, array_view_t* sources, bool direction_optimizing, size_t depth_limit,
             bool compute_predecessors, bool expensive, paths_result_t& res)
{
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    bfs_impl<typename T::vertex_t, typename T::edge_t, typename T::weight_t>(
      h, g, sources, direction_optimizing, depth_limit, compute_predecessors, expensive, res);
  });
}

}  // namespace cgx
