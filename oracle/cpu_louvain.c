/*
 * Compiled oracle Louvain (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).
 *
 * The same algorithm and arithmetic as oracle/louvain.py, compiled with OpenMP so
 * the GPU can be checked at the reference's own Louvain usecase size
 * (cpp/tests/community/louvain_test.cpp:430-442, RMAT(20, 32)) in seconds.  Both
 * restate the reference:
 *  - level loop: louvain_impl.cuh:46-237 (vertex weights k, every vertex a cluster
 *    key, Q of the singleton clustering, `while new_Q > cur_Q + 1e-4` sweeps with the
 *    up/down restriction alternating, a level keeps the clustering only when Q
 *    improved, stop when cur_Q <= best), flatten :239-255;
 *  - local move: common_methods.cuh:200-356 (old-cluster sum without self loops,
 *    self loops subtracted from the own cluster's aggregated sum :270-292 / :49-74,
 *    gain 2*((new - old)/m - gamma*(a_new*k - a_old*k + k*k)/m^2), a_new = FLT_MAX
 *    for a cluster that is not a key :331-346, best = max gain with ties to the
 *    smaller cluster id :77-94, move only if gain > 0 in the up/down direction
 *    :97-109);
 *  - cluster weights :358-382 (by the source's cluster; only clusters with out-edges
 *    are keys), modularity :121-170 (internal / m - gamma * sum a_c^2 / m^2);
 *  - contraction: structure/coarsen_graph_impl.cuh:527-632 (parallel edges summed,
 *    the used labels renumbered by descending coarse out-degree, ties by label).
 *
 * Every expression is evaluated in the same order as the numpy oracle (compile with
 * -ffp-contract=off: no fused multiply-add).  Sums are taken in another order than
 * numpy's, so the two agree bit for bit whenever the sums are exact -- integer
 * weights whose totals stay below 2^53 -- and to rounding otherwise
 * (tests/test_cpu_baseline.py checks both).
 *
 * Build: oracle/Makefile (into oracle/_build/libcpu_baseline.so).
 */
#include <float.h>
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int64_t nv, ne;
  int64_t* off;  /* [nv + 1], rows = sources */
  int64_t* dst;  /* [ne] */
  double* w;     /* [ne] */
} lv_graph;

static void lv_free(lv_graph* g)
{
  free(g->off);
  free(g->dst);
  free(g->w);
  memset(g, 0, sizeof(*g));
}

/* compute_modularity: internal weight and sum of squared present cluster weights */
static double lv_modularity(lv_graph const* g, int64_t const* c, uint8_t const* present, double const* a, double m,
                            double gamma)
{
  double internal = 0.0, sum_sq = 0.0;
#pragma omp parallel for schedule(dynamic, 1024) reduction(+ : internal)
  for (int64_t u = 0; u < g->nv; ++u)
    for (int64_t e = g->off[u]; e < g->off[u + 1]; ++e)
      if (c[u] == c[g->dst[e]]) internal += g->w[e];
#pragma omp parallel for schedule(static) reduction(+ : sum_sq)
  for (int64_t x = 0; x < g->nv; ++x)
    if (present[x]) sum_sq += a[x] * a[x];
  return internal / m - (gamma * sum_sq) / (m * m);
}

/* compute_cluster_keys_and_values: a[c] = sum of w over edges whose source is in c */
static void lv_cluster_weights(lv_graph const* g, int64_t const* c, uint8_t* present, double* a)
{
  memset(present, 0, (size_t)g->nv);
  memset(a, 0, (size_t)g->nv * sizeof(double));
  for (int64_t u = 0; u < g->nv; ++u)
    for (int64_t e = g->off[u]; e < g->off[u + 1]; ++e) {  /* edge order, as np.add.at */
      a[c[u]] += g->w[e];
      present[c[u]] = 1;
    }
}

/* per-thread scratch of the local move: a dense accumulator and seen flag per cluster
 * id and the list of clusters a row touches (stride = level-0 vertex count) */
typedef struct {
  int64_t stride;
  double* acc;
  uint8_t* seen;
  int64_t* list;
} lv_scratch;

/* one synchronous local-move sweep (update_clustering_by_delta_modularity) */
static void lv_update(lv_graph const* g, int64_t const* c, uint8_t const* present, double const* a, double const* k,
                      double m, double gamma, int up_down, int64_t* out, lv_scratch const* S)
{
  int64_t const nv = g->nv;
#pragma omp parallel
  {
    int const t      = omp_get_thread_num();
    double* acc      = S->acc + (size_t)t * S->stride;
    uint8_t* sn      = S->seen + (size_t)t * S->stride;
    int64_t* list    = S->list + (size_t)t * S->stride;
#pragma omp for schedule(dynamic, 256)
    for (int64_t u = 0; u < nv; ++u) {
      out[u] = c[u];
      int64_t const b = g->off[u], e_end = g->off[u + 1];
      if (b == e_end) continue;
      double old_sum = 0.0, self = 0.0;
      int64_t nl = 0;
      for (int64_t e = b; e < e_end; ++e) {
        int64_t const v = g->dst[e];
        if (v == u) self += g->w[e];
        else if (c[v] == c[u]) old_sum += g->w[e];
        int64_t const cv = c[v];
        if (!sn[cv]) {
          sn[cv]     = 1;
          acc[cv]    = 0.0;
          list[nl++] = cv;
        }
        acc[cv] += g->w[e];
      }
      double const kk    = k[u];
      double const a_old = a[c[u]];
      double best_dq     = -INFINITY;
      int64_t best_c     = INT64_MAX;
      for (int64_t i = 0; i < nl; ++i) {
        int64_t const pc = list[i];
        double psum      = acc[pc];
        if (pc == c[u]) psum = psum - self;
        double const a_new = present[pc] ? a[pc] : (double)FLT_MAX;
        double const dq =
          2.0 * (((psum - old_sum) / m) - gamma * (a_new * kk - a_old * kk + kk * kk) / (m * m));
        if (dq > best_dq || (dq == best_dq && pc < best_c)) {
          best_dq = dq;
          best_c  = pc;
        }
        sn[pc] = 0;
      }
      if (best_dq > 0.0 && ((best_c > c[u]) == (up_down != 0))) out[u] = best_c;
    }
  }
}

static int cmp_i64(void const* x, void const* y)
{
  int64_t const a = *(int64_t const*)x, b = *(int64_t const*)y;
  return a < b ? -1 : a > b;
}

/* coarsen by labels (values in [0, nv)): returns the coarse graph, relabels[v] = new id */
static void lv_contract(lv_graph const* g, int64_t const* labels, lv_graph* out, int64_t* relabel)
{
  int64_t const nv = g->nv;
  /* used labels, sorted */
  uint8_t* used = (uint8_t*)calloc((size_t)nv, 1);
  for (int64_t v = 0; v < nv; ++v) used[labels[v]] = 1;
  /* group edges by the source's label (counting sort) */
  int64_t* cnt = (int64_t*)calloc((size_t)nv + 1, sizeof(int64_t));
  for (int64_t u = 0; u < nv; ++u) cnt[labels[u] + 1] += g->off[u + 1] - g->off[u];
  for (int64_t x = 0; x < nv; ++x) cnt[x + 1] += cnt[x];
  int64_t* pos = (int64_t*)malloc((size_t)nv * sizeof(int64_t));
  memcpy(pos, cnt, (size_t)nv * sizeof(int64_t));
  int64_t* gd = (int64_t*)malloc((size_t)(g->ne ? g->ne : 1) * sizeof(int64_t));
  double* gw  = (double*)malloc((size_t)(g->ne ? g->ne : 1) * sizeof(double));
  for (int64_t u = 0; u < nv; ++u)
    for (int64_t e = g->off[u]; e < g->off[u + 1]; ++e) {
      int64_t const p = pos[labels[u]]++;
      gd[p]           = labels[g->dst[e]];
      gw[p]           = g->w[e];
    }
  /* per source label: distinct destination labels (ascending) with summed weights */
  double* acc      = (double*)calloc((size_t)nv, sizeof(double));
  uint8_t* sn      = (uint8_t*)calloc((size_t)nv, 1);
  int64_t* list    = (int64_t*)malloc((size_t)nv * sizeof(int64_t));
  int64_t* coff    = (int64_t*)calloc((size_t)nv + 1, sizeof(int64_t)); /* by label */
  int64_t* cd      = (int64_t*)malloc((size_t)(g->ne ? g->ne : 1) * sizeof(int64_t));
  double* cw       = (double*)malloc((size_t)(g->ne ? g->ne : 1) * sizeof(double));
  int64_t ncoarse  = 0;
  for (int64_t x = 0; x < nv; ++x) {
    coff[x]    = ncoarse;
    int64_t nl = 0;
    for (int64_t p = cnt[x]; p < cnt[x + 1]; ++p) {
      int64_t const y = gd[p];
      if (!sn[y]) {
        sn[y]      = 1;
        acc[y]     = 0.0;
        list[nl++] = y;
      }
      acc[y] += gw[p];
    }
    qsort(list, (size_t)nl, sizeof(int64_t), cmp_i64);
    for (int64_t i = 0; i < nl; ++i) {
      cd[ncoarse]   = list[i];
      cw[ncoarse++] = acc[list[i]];
      sn[list[i]]   = 0;
    }
  }
  coff[nv] = ncoarse;
  /* new ids: used labels by descending coarse out-degree, ties by ascending label */
  int64_t nu = 0;
  for (int64_t x = 0; x < nv; ++x) nu += used[x];
  int64_t maxdeg = 0;
  for (int64_t x = 0; x < nv; ++x)
    if (used[x] && coff[x + 1] - coff[x] > maxdeg) maxdeg = coff[x + 1] - coff[x];
  int64_t* dcnt = (int64_t*)calloc((size_t)maxdeg + 2, sizeof(int64_t));
  for (int64_t x = 0; x < nv; ++x)
    if (used[x]) dcnt[maxdeg - (coff[x + 1] - coff[x]) + 1]++;
  for (int64_t i = 0; i <= maxdeg; ++i) dcnt[i + 1] += dcnt[i];
  int64_t* new_of = (int64_t*)malloc((size_t)nv * sizeof(int64_t));
  int64_t* lab_of = (int64_t*)malloc((size_t)(nu ? nu : 1) * sizeof(int64_t));
  for (int64_t x = 0; x < nv; ++x) /* ascending label within a degree: stable counting sort */
    if (used[x]) {
      int64_t const id = dcnt[maxdeg - (coff[x + 1] - coff[x])]++;
      new_of[x]        = id;
      lab_of[id]       = x;
    }
  out->nv  = nu;
  out->ne  = ncoarse;
  out->off = (int64_t*)calloc((size_t)nu + 1, sizeof(int64_t));
  out->dst = (int64_t*)malloc((size_t)(ncoarse ? ncoarse : 1) * sizeof(int64_t));
  out->w   = (double*)malloc((size_t)(ncoarse ? ncoarse : 1) * sizeof(double));
  /* a coarse row keeps its edges in ascending old destination label, as the numpy
   * oracle's level arrays do (sorted by (label(u), label(v)), then relabelled) */
  int64_t q = 0;
  for (int64_t id = 0; id < nu; ++id) {
    int64_t const x = lab_of[id];
    out->off[id]    = q;
    for (int64_t p = coff[x]; p < coff[x + 1]; ++p) {
      out->dst[q] = new_of[cd[p]];
      out->w[q++] = cw[p];
    }
  }
  out->off[nu] = q;
  for (int64_t v = 0; v < nv; ++v) relabel[v] = new_of[labels[v]];
  free(used);
  free(cnt);
  free(pos);
  free(gd);
  free(gw);
  free(acc);
  free(sn);
  free(list);
  free(coff);
  free(cd);
  free(cw);
  free(dcnt);
  free(new_of);
  free(lab_of);
}

/*
 * Louvain on the CSR (off[nv + 1], idx[ne] sorted within rows, w[ne]) of the level-0
 * graph in internal ids.  Writes the flattened clustering (nv entries), the best
 * modularity and the dendrogram's level count.  Returns 0, or -2 on allocation
 * failure.
 */
int cpu_louvain(int64_t nv, int64_t const* off, int32_t const* idx, double const* w, int max_level,
                double resolution, int threads, int64_t* clustering, double* q_out, int* levels_out)
{
  if (threads > 0) omp_set_num_threads(threads);
  lv_graph g;
  g.nv  = nv;
  g.ne  = off[nv];
  g.off = (int64_t*)malloc((size_t)(nv + 1) * sizeof(int64_t));
  g.dst = (int64_t*)malloc((size_t)(g.ne ? g.ne : 1) * sizeof(int64_t));
  g.w   = (double*)malloc((size_t)(g.ne ? g.ne : 1) * sizeof(double));
  if (!g.off || !g.dst || !g.w) return -2;
  memcpy(g.off, off, (size_t)(nv + 1) * sizeof(int64_t));
  for (int64_t e = 0; e < g.ne; ++e) {
    g.dst[e] = idx[e];
    g.w[e]   = w[e];
  }
  double m = 0.0;
  for (int64_t e = 0; e < g.ne; ++e) m += g.w[e];
  int const nt = omp_get_max_threads();
  lv_scratch S;
  S.stride = nv > 0 ? nv : 1;
  S.acc    = (double*)calloc((size_t)nt * (size_t)S.stride, sizeof(double));
  S.seen   = (uint8_t*)calloc((size_t)nt * (size_t)S.stride, 1);
  S.list   = (int64_t*)malloc((size_t)nt * (size_t)S.stride * sizeof(int64_t));
  if (!S.acc || !S.seen || !S.list) return -2;
  for (int64_t v = 0; v < nv; ++v) clustering[v] = v;
  double best = -1.0;
  int levels  = 0;
  while (levels < max_level) {
    int64_t const V = g.nv;
    int64_t* level  = (int64_t*)malloc((size_t)(V ? V : 1) * sizeof(int64_t));
    int64_t* c      = (int64_t*)malloc((size_t)(V ? V : 1) * sizeof(int64_t));
    int64_t* nc     = (int64_t*)malloc((size_t)(V ? V : 1) * sizeof(int64_t));
    double* k       = (double*)calloc((size_t)(V ? V : 1), sizeof(double));
    double* a       = (double*)malloc((size_t)(V ? V : 1) * sizeof(double));
    uint8_t* pres   = (uint8_t*)malloc((size_t)(V ? V : 1));
    ++levels;
    for (int64_t v = 0; v < V; ++v) {
      level[v] = v;
      c[v]     = v;
      for (int64_t e = g.off[v]; e < g.off[v + 1]; ++e) k[v] += g.w[e];
      a[v]    = k[v];
      pres[v] = 1;
    }
    double new_q = lv_modularity(&g, c, pres, a, m, resolution);
    double cur_q = new_q - 1.0;
    int up_down  = 1;
    while (new_q > cur_q + 0.0001) {
      cur_q = new_q;
      lv_update(&g, c, pres, a, k, m, resolution, up_down, nc, &S);
      int64_t* t = c;
      c          = nc;
      nc         = t;
      lv_cluster_weights(&g, c, pres, a);
      up_down = !up_down;
      new_q   = lv_modularity(&g, c, pres, a, m, resolution);
      if (new_q > cur_q) memcpy(level, c, (size_t)V * sizeof(int64_t));
    }
    int const stop = cur_q <= best;
    if (!stop) {
      best = cur_q;
      lv_graph coarse;
      int64_t* relabel = (int64_t*)malloc((size_t)(V ? V : 1) * sizeof(int64_t));
      lv_contract(&g, level, &coarse, relabel);
      memcpy(level, relabel, (size_t)V * sizeof(int64_t));
      free(relabel);
      lv_free(&g);
      g = coarse;
    }
    for (int64_t v = 0; v < nv; ++v) clustering[v] = level[clustering[v]];
    free(c);
    free(nc);
    free(k);
    free(a);
    free(pres);
    free(level);
    if (stop) break;
  }
  lv_free(&g);
  free(S.acc);
  free(S.seen);
  free(S.list);
  *q_out      = best;
  *levels_out = levels;
  return 0;
}
