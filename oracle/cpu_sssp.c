/*
 * Compiled near-far SSSP (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py): the
 * checker of the GPU SSSP at the reference's test and benchmark sizes
 * (cpp/tests/traversal/sssp_test.cpp:305 runs RMAT(20, 32); the numpy oracle
 * oracle/sssp.py is a frontier Bellman-Ford, too slow there) and bench.py's SSSP CPU
 * baseline.  Checked against oracle/sssp.py by tests/test_cpu_baseline.py.
 *
 * Restates detail::sssp, cpp/src/traversal/sssp_impl.cuh:79-270, one thread:
 *  - distances start at numeric_limits<weight_t>::max(), 0 at the source (:99-120);
 *  - delta = warp_size * average edge weight / average degree, warp_size = 32 as the
 *    reference's raft::warp_size() (:143-157; sums taken in double here -- delta only
 *    orders the work, the distances are the fixed point either way);
 *  - three buckets, current near / next near / far (:161-167); a push from u to v
 *    with new = dist[u] + w in weight_t is kept iff new < min(cutoff, dist[v])
 *    (e_op_t, :49-72), and goes to next near if new < threshold, else to far
 *    (update_v_frontier's v_op, :199-221);
 *  - near empty: threshold += delta and the far bucket is split -- entries below the
 *    old threshold dropped (already settled), below the new one to current near,
 *    the rest stay far -- repeated with threshold += delta until near is non-empty or
 *    far is empty (split_bucket, :226-262).
 *  Serial relaxation reads distances as they improve inside a round (the reference
 *  reads them after update_v_frontier); fp addition of non-negative weights is
 *  monotone, so both reach the same fixed point: the minimum over paths of the
 *  left-folded weight_t sums below the cutoff.
 *  Predecessors: the build's deterministic rule (oracle/sssp.py): the smallest
 *  internal id among the tight in-neighbours (dist[u] + w == dist[v]); -1 when
 *  unreached or the source.
 *
 * Returns the number of relaxation rounds; *seconds = the traversal's time
 * (allocation excluded).  -2 on allocation failure.
 */
#include <float.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CGX_SSSP(NAME, W, WMAX)                                                                                   \
  int NAME(const int64_t* off, const int32_t* idx, const W* wgt, int64_t nv, int32_t source, double cutoff,       \
           W* dist, int32_t* pred, double* seconds)                                                               \
  {                                                                                                               \
    int64_t const ne = nv > 0 ? off[nv] : 0;                                                                      \
    for (int64_t v = 0; v < nv; ++v) dist[v] = WMAX;                                                              \
    for (int64_t v = 0; v < nv; ++v) pred[v] = -1;                                                                \
    *seconds = 0.0;                                                                                               \
    if (nv <= 0 || source < 0 || source >= nv) return 0;                                                          \
    int32_t* cur   = (int32_t*)malloc((size_t)nv * sizeof(int32_t));                                              \
    int32_t* nxt   = (int32_t*)malloc((size_t)nv * sizeof(int32_t));                                              \
    int64_t far_cap = nv + 1;                                                                                     \
    int32_t* far   = (int32_t*)malloc((size_t)far_cap * sizeof(int32_t));                                         \
    int32_t* far2  = (int32_t*)malloc((size_t)far_cap * sizeof(int32_t));                                         \
    int32_t* stamp = (int32_t*)malloc((size_t)nv * sizeof(int32_t));                                              \
    if (!cur || !nxt || !far || !far2 || !stamp) {                                                                \
      free(cur); free(nxt); free(far); free(far2); free(stamp);                                                   \
      return -2;                                                                                                  \
    }                                                                                                             \
    for (int64_t v = 0; v < nv; ++v) stamp[v] = -1;                                                               \
    double t0 = omp_get_wtime();                                                                                  \
    double wsum = 0.0;                                                                                            \
    for (int64_t e = 0; e < ne; ++e) wsum += (double)wgt[e];                                                      \
    double const avg_w = ne ? wsum / (double)ne : 0.0, avg_deg = (double)ne / (double)nv;                        \
    W const delta = (W)(avg_deg > 0 ? 32.0 * avg_w / avg_deg : 1.0);                                              \
    W const cut   = (cutoff >= (double)WMAX || cutoff != cutoff) ? WMAX : (W)cutoff;                              \
    dist[source] = (W)0;                                                                                          \
    int64_t ncur = 1, nnxt = 0, nfar = 0;                                                                         \
    cur[0] = source;                                                                                              \
    W thr = delta;                                                                                                \
    int32_t round = 0, tag = 0;                                                                                   \
    while (1) {                                                                                                   \
      ++round;                                                                                                    \
      ++tag;                                                                                                      \
      nnxt = 0;                                                                                                   \
      for (int64_t i = 0; i < ncur; ++i) {                                                                        \
        int32_t const u = cur[i];                                                                                 \
        W const du      = dist[u];                                                                                \
        for (int64_t e = off[u]; e < off[u + 1]; ++e) {                                                           \
          int32_t const v = idx[e];                                                                               \
          W const nd      = (W)(du + wgt[e]);                                                                     \
          W const lim     = dist[v] < cut ? dist[v] : cut;                                                        \
          if (!(nd < lim)) continue;                                                                              \
          dist[v] = nd;                                                                                           \
          if (nd < thr) {                                                                                         \
            if (stamp[v] != tag) {                                                                                \
              stamp[v]    = tag;                                                                                  \
              nxt[nnxt++] = v;                                                                                    \
            }                                                                                                     \
          } else {                                                                                                \
            if (nfar == far_cap) {                                                                                \
              far_cap *= 2;                                                                                       \
              int32_t* f = (int32_t*)realloc(far, (size_t)far_cap * sizeof(int32_t));                             \
              int32_t* g = (int32_t*)realloc(far2, (size_t)far_cap * sizeof(int32_t));                            \
              if (!f || !g) {                                                                                     \
                free(f ? f : far); free(g ? g : far2); free(cur); free(nxt); free(stamp);                         \
                return -2;                                                                                        \
              }                                                                                                   \
              far = f; far2 = g;                                                                                  \
            }                                                                                                     \
            far[nfar++] = v;                                                                                      \
          }                                                                                                       \
        }                                                                                                         \
      }                                                                                                           \
      if (nnxt > 0) {                                                                                             \
        int32_t* t = cur; cur = nxt; nxt = t;                                                                     \
        ncur = nnxt;                                                                                              \
        continue;                                                                                                 \
      }                                                                                                           \
      if (nfar == 0) break;                                                                                       \
      W const old = thr;                                                                                          \
      thr         = (W)(thr + delta);                                                                             \
      ++tag;                                                                                                      \
      while (1) {                                                                                                 \
        int64_t n2 = 0;                                                                                           \
        ncur       = 0;                                                                                           \
        for (int64_t i = 0; i < nfar; ++i) {                                                                      \
          int32_t const v = far[i];                                                                               \
          W const d       = dist[v];                                                                              \
          if (!(d >= old)) continue;                                                                              \
          if (d < thr) {                                                                                          \
            if (stamp[v] != tag) {                                                                                \
              stamp[v]    = tag;                                                                                  \
              cur[ncur++] = v;                                                                                    \
            }                                                                                                     \
          } else {                                                                                                \
            far2[n2++] = v;                                                                                       \
          }                                                                                                       \
        }                                                                                                         \
        int32_t* t = far; far = far2; far2 = t;                                                                   \
        nfar = n2;                                                                                                \
        if (ncur > 0 || nfar == 0) break;                                                                         \
        thr = (W)(thr + delta);                                                                                   \
      }                                                                                                           \
      if (ncur == 0 && nfar == 0) break;                                                                          \
    }                                                                                                             \
    *seconds = omp_get_wtime() - t0;                                                                              \
    for (int64_t u = 0; u < nv; ++u) {                                                                            \
      W const du = dist[u];                                                                                       \
      if (du == WMAX) continue;                                                                                   \
      for (int64_t e = off[u]; e < off[u + 1]; ++e) {                                                             \
        int32_t const v = idx[e];                                                                                 \
        if (v == source || (W)(du + wgt[e]) != dist[v]) continue;                                                 \
        if (pred[v] < 0 || u < pred[v]) pred[v] = (int32_t)u;                                                     \
      }                                                                                                           \
    }                                                                                                             \
    free(cur); free(nxt); free(far); free(far2); free(stamp);                                                     \
    return round;                                                                                                 \
  }

CGX_SSSP(cpu_sssp_f32, float, FLT_MAX)
CGX_SSSP(cpu_sssp_f64, double, DBL_MAX)
