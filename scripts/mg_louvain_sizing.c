// Sizing model for multi-GPU Louvain at the configs' scale (measurement aid, not product).
//
// For the symmetrised Graph500 R-MAT graph of the bench (oracle/rmat.py's generator:
// a=.57 b=c=.19, edge factor 16, seed 42, scrambled ids) and P ranks, with the
// library's vertex owner (mg_owner_of_ext, csrc/mg_graph.hpp:45-52), it counts per rank:
//
//   1D partition by source owner (this library's MG Louvain, csrc/louvain.hip MG section):
//     rows (owned vertices with edges), edges, ghosts (distinct remote destinations),
//     mirror entries (how many other ranks hold each owned vertex as a ghost);
//   2D partition R x C (the reference's graph_view_t, C = row communicator size):
//     the block's edges and distinct destinations.
//
// and prints the first sweep's exchange bytes per rank (every vertex its own cluster:
// the sweep that references the most clusters):
//   1D: view  = remote referenced clusters (= ghosts) x 20 B (two key lookups of 4 B,
//               answers of 8 + 4 B: collect_by_key of afix and pcnt, mg_view)
//       advance = f x rows x 32 B x (P-1)/P (two weight deltas of 4 + 8 + 4 B per moved
//               row, mg_advance) + f x mirror entries of moved rows x 8 B
//   2D (per_v_transform_reduce_dst_key_aggregated_outgoing_e.cuh:506-611,736-753,
//       louvain_impl.cuh:91-103):
//       minor clusters  = (R-1) x V/P x 4 B (the column's destinations' clusters)
//       major clusters  = (C-1) x V/P x 4 B (the row's sources' clusters)
//       aggregated pairs = (C-1)/C x block edges x 16 B (src, cluster, weight to the
//               source's owner; every (src, dst) pair is its own key in the first sweep)
//       cluster weights = (P-1)/P x distinct destinations x 12 B (key + weight)
//       moves           = f x rows x 24 B x (P-1)/P
// with f the fraction of rows that move (1 = upper bound).  Edge counts include the
// generator's few duplicate edges (dedup removes ~2 % at scale 24-26); vertex and
// ghost counts are exact (bitmaps).
//
// build: gcc -O3 -fopenmp -o /tmp/mg_louvain_sizing scripts/mg_louvain_sizing.c
// usage: /tmp/mg_louvain_sizing SCALE [P] [C] [f]
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t splitmix64(uint64_t x)
{
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z          = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z          = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline uint64_t scramble(uint64_t v, int scale, uint64_t seed)
{
  uint64_t const mask = (scale >= 64) ? ~0ull : ((1ull << scale) - 1);
  int const h         = (scale + 1) / 2;
  v = (v * 0x9E3779B1ull + seed) & mask;
  v ^= v >> h;
  v = (v * 0x85EBCA77ull) & mask;
  v ^= v >> h;
  return v;
}

static inline int owner_of_ext(int64_t x, int P)  // csrc/mg_graph.hpp mg_owner_of_ext
{
  unsigned long long z = (unsigned long long)x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (int)(z % (unsigned long long)P);
}

static inline void set_bit(uint64_t* b, uint64_t i) { __atomic_fetch_or(&b[i >> 6], 1ull << (i & 63), __ATOMIC_RELAXED); }
static inline int get_bit(uint64_t const* b, uint64_t i) { return (int)((b[i >> 6] >> (i & 63)) & 1ull); }

int main(int argc, char** argv)
{
  if (argc < 2) {
    fprintf(stderr, "usage: %s SCALE [P=8] [C=2] [f=1.0]\n", argv[0]);
    return 2;
  }
  int const scale = atoi(argv[1]);
  int const P     = argc > 2 ? atoi(argv[2]) : 8;
  int const C     = argc > 3 ? atoi(argv[3]) : 2;
  double const f  = argc > 4 ? atof(argv[4]) : 1.0;
  int const R     = P / C;
  uint64_t const seed = 42, V = 1ull << scale, nedge = 16ull << scale;
  double const a = 0.57, b = 0.19, c = 0.19, tab = a + b, tabc = a + b + c;
  size_t const words = (size_t)((V + 63) / 64);
  uint64_t* present = calloc(words, 8);
  uint64_t** ghost  = malloc(P * sizeof(uint64_t*));   // ghost[p]: remote destinations of rank p's rows
  uint64_t** bdst   = malloc(P * sizeof(uint64_t*));   // bdst[blk]: destinations of 2D block blk
  for (int p = 0; p < P; ++p) {
    ghost[p] = calloc(words, 8);
    bdst[p]  = calloc(words, 8);
  }
  int64_t* e1d = calloc(P, 8);
  int64_t* e2d = calloc(P, 8);
  int const T  = omp_get_max_threads();
  int64_t* te1 = calloc((size_t)T * P, 8);
  int64_t* te2 = calloc((size_t)T * P, 8);
#pragma omp parallel
  {
    int const t = omp_get_thread_num();
#pragma omp for schedule(static, 1 << 16)
    for (int64_t e = 0; e < (int64_t)nedge; ++e) {
      uint64_t s = 0, d = 0;
      for (int l = 0; l < scale; ++l) {
        uint64_t const z = splitmix64((seed * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)e * 64ull + (uint64_t)l));
        double const r   = (double)(z >> 11) * (1.0 / 9007199254740992.0);
        uint64_t const sb = r >= tab, db = ((r >= a) && (r < tab)) || (r >= tabc);
        s |= sb << (scale - 1 - l);
        d |= db << (scale - 1 - l);
      }
      s = scramble(s, scale, seed);
      d = scramble(d, scale, seed);
      set_bit(present, s);
      set_bit(present, d);
      for (int dir = 0; dir < (s == d ? 1 : 2); ++dir) {
        uint64_t const u = dir ? d : s, v = dir ? s : d;
        int const ou = owner_of_ext((int64_t)u, P), ov = owner_of_ext((int64_t)v, P);
        te1[(size_t)t * P + ou]++;
        if (ov != ou) set_bit(ghost[ou], v);
        int const blk = (ou / C) * C + (ov % C);  // row of owner(u), column of owner(v)
        te2[(size_t)t * P + blk]++;
        set_bit(bdst[blk], v);
      }
    }
  }
  for (int t = 0; t < T; ++t)
    for (int p = 0; p < P; ++p) {
      e1d[p] += te1[(size_t)t * P + p];
      e2d[p] += te2[(size_t)t * P + p];
    }
  int64_t *rows = calloc(P, 8), *gh = calloc(P, 8), *mir = calloc(P, 8), *bd = calloc(P, 8);
  int64_t nv = 0;
#pragma omp parallel for reduction(+ : nv)
  for (int64_t v = 0; v < (int64_t)V; ++v) {
    if (!get_bit(present, (uint64_t)v)) continue;
    ++nv;
    int const o = owner_of_ext(v, P);
    __atomic_fetch_add(&rows[o], 1, __ATOMIC_RELAXED);
    int m = 0;
    for (int q = 0; q < P; ++q) {
      if (get_bit(ghost[q], (uint64_t)v)) {
        ++m;
        __atomic_fetch_add(&gh[q], 1, __ATOMIC_RELAXED);
      }
      if (get_bit(bdst[q], (uint64_t)v)) __atomic_fetch_add(&bd[q], 1, __ATOMIC_RELAXED);
    }
    __atomic_fetch_add(&mir[o], m, __ATOMIC_RELAXED);
  }
  int64_t E = 0;
  for (int p = 0; p < P; ++p) E += e1d[p];
  printf("RMAT-%d: V=%lld (vertices with edges), stored edges %lld (both directions, duplicates kept), P=%d, 2D %dx%d, "
         "moved fraction f=%.2f\n", scale, (long long)nv, (long long)E, P, R, C, f);
  printf("rank | 1D: rows edges ghosts mirror-entries | sweep bytes: view advance total | 2D: block edges dst | sweep "
         "bytes: minor major pairs weights moves total\n");
  double s1 = 0, s2 = 0;
  for (int p = 0; p < P; ++p) {
    double const view = (double)gh[p] * 20.0;
    double const adv  = f * rows[p] * 32.0 * (P - 1) / P + f * mir[p] * 8.0;
    double const vp   = (double)nv / P;
    double const mn = (R - 1) * vp * 4.0, mj = (C - 1) * vp * 4.0;
    double const pairs = (double)(C - 1) / C * e2d[p] * 16.0;
    double const wts   = (double)(P - 1) / P * bd[p] * 12.0;
    double const mv    = f * rows[p] * 24.0 * (P - 1) / P;
    s1 = view + adv > s1 ? view + adv : s1;
    s2 = mn + mj + pairs + wts + mv > s2 ? mn + mj + pairs + wts + mv : s2;
    printf("%4d | %10lld %11lld %10lld %11lld | %8.1f %8.1f %8.1f MB | %11lld %10lld | %7.1f %7.1f %8.1f %7.1f %7.1f "
           "%8.1f MB\n",
           p, (long long)rows[p], (long long)e1d[p], (long long)gh[p], (long long)mir[p], view / 1e6, adv / 1e6,
           (view + adv) / 1e6, (long long)e2d[p], (long long)bd[p], mn / 1e6, mj / 1e6, pairs / 1e6, wts / 1e6,
           mv / 1e6, (mn + mj + pairs + wts + mv) / 1e6);
  }
  printf("max over ranks, first sweep: 1D %.1f MB, 2D %.1f MB per rank\n", s1 / 1e6, s2 / 1e6);
  return 0;
}
