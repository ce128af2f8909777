/*
 * Compiled CPU restatement of the reference's own CPU references (TEST
 * INFRASTRUCTURE ONLY -- see oracle/__init__.py): the secondary CPU baseline of
 * SURVEY.md §8d ("the build's compiled single-thread C++ restatement of the
 * reference CPU references, plus an OpenMP variant with its core count stated").
 * bench.py's cpu_baseline leg is the only caller; nothing in the product links it.
 *
 *  - cpu_pagerank: cpp/tests/link_analysis/pagerank_test.cpp:43-130
 *    (pagerank_reference): per iteration a dangling sum, a pull over the CSC
 *    (pr[v] = sum alpha * old[u] * w / outw[u] + (dangling*alpha + 1-alpha)/V)
 *    and an L1 difference, in result_t = float as the reference instantiates it.
 *    The loop over destinations is the one OpenMP splits (static schedule over
 *    vertices, reductions for the two sums); threads = 1 is the scalar restatement.
 *  - cpu_bfs: cpp/tests/traversal/bfs_test.cpp:41-79 (bfs_reference): queue-based
 *    level-synchronous top-down BFS.  With threads > 1 each level's frontier is
 *    split over threads that claim vertices with an atomic compare-and-swap on the
 *    distance and append to thread-local queues.
 *
 *  - cpu_pagerank_f64: the oracle's PageRank (oracle/pagerank.py, i.e.
 *    pagerank_impl.cuh:48-293 in float64: dangling mass, x~ = pr / outw, pull
 *    SpMV, stop on L1 < epsilon) compiled with OpenMP, so tests can check the GPU
 *    at the benchmark sizes (RMAT-22/24) in seconds.  Checked against the numpy
 *    oracle by tests/test_cpu_baseline.py.
 *
 * Build (oracle/Makefile): gcc -O3 -fopenmp -shared -fPIC -o oracle/_build/libcpu_baseline.so
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static double now_s(void) { return omp_get_wtime(); }

/* Runs `iterations` power iterations (no stop test, a bounded sample) from the
 * uniform start and returns the seconds they took; pr receives the last iterate.
 * off/idx: CSC (row v lists the sources u of its in-edges), out-degree counted
 * from idx (unweighted graphs).  Out-weight computation is outside the timing,
 * as the GPU timing excludes graph preparation. */
double cpu_pagerank(const int64_t* off, const int32_t* idx, int64_t nv, int iterations, double alpha, int threads,
                    float* pr)
{
  if (nv <= 0) return 0.0;
  if (threads > 0) omp_set_num_threads(threads);
  float* outw = (float*)calloc((size_t)nv, sizeof(float));
  float* old  = (float*)malloc((size_t)nv * sizeof(float));
  if (!outw || !old) {
    free(outw);
    free(old);
    return -1.0;
  }
  int64_t const ne = off[nv];
  for (int64_t e = 0; e < ne; ++e) outw[idx[e]] += 1.0f;
  for (int64_t v = 0; v < nv; ++v) pr[v] = 1.0f / (float)nv;
  float const a = (float)alpha;
  double t0     = now_s();
  for (int it = 0; it < iterations; ++it) {
    memcpy(old, pr, (size_t)nv * sizeof(float));
    float dangling = 0.0f;
#pragma omp parallel for schedule(static) reduction(+ : dangling) if (threads != 1)
    for (int64_t v = 0; v < nv; ++v)
      if (outw[v] == 0.0f) dangling += old[v];
    float const base = (dangling * a + (1.0f - a)) / (float)nv;
    float diff       = 0.0f;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : diff) if (threads != 1)
    for (int64_t v = 0; v < nv; ++v) {
      float s = 0.0f;
      for (int64_t j = off[v]; j < off[v + 1]; ++j) {
        int32_t const u = idx[j];
        s += a * old[u] * (1.0f / outw[u]);
      }
      pr[v] = s + base;
      diff += fabsf(pr[v] - old[v]);
    }
    (void)diff;  /* the reference stops on diff < epsilon; the sample runs a fixed count */
  }
  double t = now_s() - t0;
  free(outw);
  free(old);
  return t;
}

/* BFS from `source` over the CSR; dist = INT32_MAX / pred = -1 for unreached.
 * Returns seconds.  threads == 1: the reference's sequential queue loop. */
double cpu_bfs(const int64_t* off, const int32_t* idx, int64_t nv, int32_t source, int threads, int32_t* dist,
               int32_t* pred)
{
  if (nv <= 0) return 0.0;
  if (threads > 0) omp_set_num_threads(threads);
  for (int64_t v = 0; v < nv; ++v) {
    dist[v] = INT32_MAX;
    pred[v] = -1;
  }
  int32_t* cur = (int32_t*)malloc((size_t)nv * sizeof(int32_t));
  int32_t* nxt = (int32_t*)malloc((size_t)nv * sizeof(int32_t));
  if (!cur || !nxt) {
    free(cur);
    free(nxt);
    return -1.0;
  }
  double t0    = now_s();
  int64_t ncur = 1, nnext = 0;
  cur[0]       = source;
  dist[source] = 0;
  int32_t depth = 0;
  while (ncur > 0) {
    nnext = 0;
    if (threads == 1) {
      for (int64_t i = 0; i < ncur; ++i) {
        int32_t const row = cur[i];
        for (int64_t j = off[row]; j < off[row + 1]; ++j) {
          int32_t const nbr = idx[j];
          if (dist[nbr] == INT32_MAX) {
            dist[nbr]      = depth + 1;
            pred[nbr]      = row;
            nxt[nnext++]   = nbr;
          }
        }
      }
    } else {
#pragma omp parallel
      {
        int32_t local[1024];
        int nl = 0;
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < ncur; ++i) {
          int32_t const row = cur[i];
          for (int64_t j = off[row]; j < off[row + 1]; ++j) {
            int32_t const nbr = idx[j];
            if (__atomic_load_n(&dist[nbr], __ATOMIC_RELAXED) != INT32_MAX) continue;
            int32_t expect = INT32_MAX;
            if (__atomic_compare_exchange_n(&dist[nbr], &expect, depth + 1, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
              pred[nbr]   = row;
              local[nl++] = nbr;
              if (nl == 1024) {
                int64_t at = __atomic_fetch_add(&nnext, nl, __ATOMIC_RELAXED);
                memcpy(nxt + at, local, sizeof(local));
                nl = 0;
              }
            }
          }
        }
        if (nl) {
          int64_t at = __atomic_fetch_add(&nnext, nl, __ATOMIC_RELAXED);
          memcpy(nxt + at, local, (size_t)nl * sizeof(int32_t));
        }
      }
    }
    int32_t* tmp = cur;
    cur          = nxt;
    nxt          = tmp;
    ncur         = nnext;
    ++depth;
  }
  double t = now_s() - t0;
  free(cur);
  free(nxt);
  return t;
}

/* fp64 oracle PageRank on the CSC (unweighted): returns iterations run (> 0), or
 * -1 when max_iterations is reached without L1 < epsilon, -2 on allocation failure.
 * pr receives the ranks by internal id. */
int cpu_pagerank_f64(const int64_t* off, const int32_t* idx, int64_t nv, double alpha, double epsilon,
                     int max_iterations, int threads, double* pr)
{
  if (nv <= 0) return 0;
  if (threads > 0) omp_set_num_threads(threads);
  double* outw = (double*)calloc((size_t)nv, sizeof(double));
  double* xt   = (double*)malloc((size_t)nv * sizeof(double));
  if (!outw || !xt) {
    free(outw);
    free(xt);
    return -2;
  }
  int64_t const ne = off[nv];
  for (int64_t e = 0; e < ne; ++e) outw[idx[e]] += 1.0;
#pragma omp parallel for schedule(static)
  for (int64_t v = 0; v < nv; ++v) pr[v] = 1.0 / (double)nv;
  int it = 0;
  while (1) {
    double dangling = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : dangling)
    for (int64_t v = 0; v < nv; ++v) {
      if (outw[v] == 0.0) dangling += pr[v];
      xt[v] = pr[v] / (outw[v] == 0.0 ? 1.0 : outw[v]);
    }
    double const base = (dangling * alpha + (1.0 - alpha)) / (double)nv;
    double diff       = 0.0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : diff)
    for (int64_t v = 0; v < nv; ++v) {
      double s = 0.0;
      for (int64_t j = off[v]; j < off[v + 1]; ++j) s += xt[idx[j]] * alpha;
      double const nw = base + s;
      diff += fabs(nw - pr[v]);
      pr[v] = nw;  /* pr[v] is read only by this iteration's diff: xt holds the sources */
    }
    ++it;
    if (diff < epsilon) break;
    if (it >= max_iterations) {
      it = -1;
      break;
    }
  }
  free(outw);
  free(xt);
  return it;
}
