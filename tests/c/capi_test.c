/*
 * Plain-C client of libcugraph_c, compiled against the include/cugraph_c headers only
 * (no HIP, no C++).  It exercises the boundary the way the reference's own C
 * tests do (cpp/tests/c_api/pagerank_test.c, bfs_test.c, sssp_test.c, louvain_test.c): build a graph
 * from host edge arrays copied into type-erased device arrays, run the
 * algorithm, copy the result views back and compare with the reference's
 * expected vectors (the same numbers as tests/golden/reference_vectors.json).
 * It also covers the error contract (CUGRAPH_INVALID_INPUT with a message) and
 * the array release entry points (array.h:95,212).
 *
 * Build: gcc -std=c99 -I include tests/c/capi_test.c -L <lib> -lcugraph_c
 * Run:   ./capi_test            (needs a GPU; exit status = number of failures)
 */
#include <cugraph_c/algorithms.h>
#include <cugraph_c/array.h>
#include <cugraph_c/graph.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int g_failures = 0;

#define CHECK(cond, ...)                                                   \
  do {                                                                     \
    if (!(cond)) {                                                         \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                 \
      fprintf(stderr, __VA_ARGS__);                                        \
      fprintf(stderr, "\n");                                               \
      ++g_failures;                                                        \
      return 1;                                                            \
    }                                                                      \
  } while (0)

#define CHECK_RC(rc, err, what)                                                          \
  CHECK((rc) == CUGRAPH_SUCCESS, "%s failed (%d): %s", what, (int)(rc),                   \
        (err) ? cugraph_error_message(err) : "(no message)")

/* relative closeness as the reference C tests use it (c_test_utils.h nearlyEqual) */
static int close_rel(double a, double b, double tol)
{
  double d = fabs(a - b), m = fabs(a) > fabs(b) ? fabs(a) : fabs(b);
  return d <= tol * (m > 1e-30 ? m : 1.0);
}

/* the 6-vertex edge set shared by most reference C tests */
static const int32_t E6_SRC[8] = {0, 1, 1, 2, 2, 2, 3, 4};
static const int32_t E6_DST[8] = {1, 3, 4, 0, 1, 3, 5, 5};
static const float E6_W[8]     = {0.1f, 2.1f, 1.1f, 5.1f, 3.1f, 4.1f, 7.2f, 3.2f};

/* device copy of a host array; returns the owning array (view via *view) */
static cugraph_type_erased_device_array_t* to_device(const cugraph_resource_handle_t* h, const void* host,
                                                     size_t n, data_type_id_t t,
                                                     cugraph_type_erased_device_array_view_t** view)
{
  cugraph_type_erased_device_array_t* arr = NULL;
  cugraph_error_t* err                    = NULL;
  if (cugraph_type_erased_device_array_create(h, n, t, &arr, &err) != CUGRAPH_SUCCESS) {
    cugraph_error_free(err);
    return NULL;
  }
  *view = cugraph_type_erased_device_array_view(arr);
  if (cugraph_type_erased_device_array_view_copy_from_host(h, *view, (const byte_t*)host, &err) !=
      CUGRAPH_SUCCESS) {
    cugraph_error_free(err);
    cugraph_type_erased_device_array_view_free(*view);
    cugraph_type_erased_device_array_free(arr);
    return NULL;
  }
  return arr;
}

typedef struct {
  cugraph_type_erased_device_array_t *src, *dst, *wgt;
  cugraph_type_erased_device_array_view_t *src_v, *dst_v, *wgt_v;
  cugraph_graph_t* graph;
} test_graph_t;

static void free_graph(test_graph_t* g)
{
  if (g->graph) cugraph_sg_graph_free(g->graph);
  if (g->src_v) cugraph_type_erased_device_array_view_free(g->src_v);
  if (g->dst_v) cugraph_type_erased_device_array_view_free(g->dst_v);
  if (g->wgt_v) cugraph_type_erased_device_array_view_free(g->wgt_v);
  if (g->src) cugraph_type_erased_device_array_free(g->src);
  if (g->dst) cugraph_type_erased_device_array_free(g->dst);
  if (g->wgt) cugraph_type_erased_device_array_free(g->wgt);
  memset(g, 0, sizeof(*g));
}

static cugraph_error_code_t make_graph(const cugraph_resource_handle_t* h, const int32_t* s, const int32_t* d,
                                       const float* w, size_t ne, bool_t store_transposed, bool_t symmetric,
                                       test_graph_t* g, cugraph_error_t** err)
{
  memset(g, 0, sizeof(*g));
  *err                            = NULL;
  cugraph_graph_properties_t prop = {symmetric, FALSE};
  g->src                          = to_device(h, s, ne, INT32, &g->src_v);
  g->dst                          = to_device(h, d, ne, INT32, &g->dst_v);
  g->wgt                          = to_device(h, w, ne, FLOAT32, &g->wgt_v);
  if (!g->src || !g->dst || !g->wgt) return CUGRAPH_ALLOC_ERROR;
  return cugraph_sg_graph_create(h, &prop, g->src_v, g->dst_v, g->wgt_v, NULL, NULL, store_transposed, FALSE,
                                 FALSE, &g->graph, err);
}

/* cpp/tests/c_api/pagerank_test.c:211-229 and :250-268 */
static int pagerank_case(const int32_t* s, const int32_t* d, const float* w, size_t ne, size_t nv,
                         const float* expected, double alpha, double eps, size_t max_it, bool_t transposed)
{
  cugraph_resource_handle_t* h = cugraph_create_resource_handle(NULL);
  CHECK(h != NULL, "resource handle");
  test_graph_t g;
  cugraph_error_t* err = NULL;
  cugraph_error_code_t rc = make_graph(h, s, d, w, ne, transposed, FALSE, &g, &err);
  CHECK_RC(rc, err, "sg_graph_create");
  cugraph_centrality_result_t* res = NULL;
  rc = cugraph_pagerank(h, g.graph, NULL, NULL, NULL, NULL, alpha, eps, max_it, FALSE, &res, &err);
  CHECK_RC(rc, err, "cugraph_pagerank");
  int32_t vert[16];
  float val[16];
  cugraph_type_erased_device_array_view_t* vv = cugraph_centrality_result_get_vertices(res);
  cugraph_type_erased_device_array_view_t* pv = cugraph_centrality_result_get_values(res);
  CHECK(cugraph_type_erased_device_array_view_size(pv) == nv, "result size");
  CHECK(cugraph_type_erased_device_array_view_type(pv) == FLOAT32, "result dtype");
  rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)vert, vv, &err);
  CHECK_RC(rc, err, "copy vertices");
  rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)val, pv, &err);
  CHECK_RC(rc, err, "copy values");
  for (size_t i = 0; i < nv; ++i)
    CHECK(close_rel(expected[vert[i]], val[i], 1e-3), "pagerank[%d] = %g, expected %g", vert[i], val[i],
          expected[vert[i]]);
  cugraph_type_erased_device_array_view_free(vv);
  cugraph_type_erased_device_array_view_free(pv);
  cugraph_centrality_result_free(res);
  free_graph(&g);
  cugraph_free_resource_handle(h);
  return 0;
}

static int test_pagerank(void)
{
  static const float exp6[6] = {0.0915528f, 0.168382f, 0.0656831f, 0.191468f, 0.120677f, 0.362237f};
  static const int32_t ps[3] = {0, 1, 2}, pd[3] = {1, 2, 3};
  static const float pw[3]   = {1, 1, 1};
  static const float exp4[4] = {0.11615585f, 0.21488841f, 0.2988108f, 0.3701449f};
  int r = 0;
  r |= pagerank_case(E6_SRC, E6_DST, E6_W, 8, 6, exp6, 0.95, 1e-4, 20, FALSE);
  r |= pagerank_case(E6_SRC, E6_DST, E6_W, 8, 6, exp6, 0.95, 1e-4, 20, TRUE);
  r |= pagerank_case(ps, pd, pw, 3, 4, exp4, 0.85, 1e-6, 500, FALSE);
  return r;
}

/* cpp/tests/c_api/pagerank_test.c:288-310 */
static int test_personalized_pagerank(void)
{
  static const int32_t s[3] = {0, 1, 2}, d[3] = {1, 2, 3};
  static const float w[3]   = {1, 1, 1};
  static const int32_t pv[4] = {0, 1, 2, 3};
  static const float pval[4] = {0.1f, 0.2f, 0.3f, 0.4f};
  static const float expd[4] = {0.0559233f, 0.159381f, 0.303244f, 0.481451f};
  cugraph_resource_handle_t* h = cugraph_create_resource_handle(NULL);
  test_graph_t g;
  cugraph_error_t* err = NULL;
  cugraph_error_code_t rc = make_graph(h, s, d, w, 3, FALSE, FALSE, &g, &err);
  CHECK_RC(rc, err, "sg_graph_create");
  cugraph_type_erased_device_array_view_t *pv_v, *pval_v;
  cugraph_type_erased_device_array_t* pv_a   = to_device(h, pv, 4, INT32, &pv_v);
  cugraph_type_erased_device_array_t* pval_a = to_device(h, pval, 4, FLOAT32, &pval_v);
  CHECK(pv_a && pval_a, "personalization arrays");
  cugraph_centrality_result_t* res = NULL;
  rc = cugraph_personalized_pagerank(h, g.graph, NULL, NULL, NULL, NULL, pv_v, pval_v, 0.85, 1e-6, 500, FALSE,
                                     &res, &err);
  CHECK_RC(rc, err, "cugraph_personalized_pagerank");
  int32_t vert[4];
  float val[4];
  cugraph_type_erased_device_array_view_t* vv = cugraph_centrality_result_get_vertices(res);
  cugraph_type_erased_device_array_view_t* rv = cugraph_centrality_result_get_values(res);
  rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)vert, vv, &err);
  CHECK_RC(rc, err, "copy vertices");
  rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)val, rv, &err);
  CHECK_RC(rc, err, "copy values");
  for (int i = 0; i < 4; ++i)
    CHECK(close_rel(expd[vert[i]], val[i], 1e-3), "ppr[%d] = %g, expected %g", vert[i], val[i], expd[vert[i]]);
  cugraph_type_erased_device_array_view_free(vv);
  cugraph_type_erased_device_array_view_free(rv);
  cugraph_centrality_result_free(res);
  cugraph_type_erased_device_array_view_free(pv_v);
  cugraph_type_erased_device_array_view_free(pval_v);
  cugraph_type_erased_device_array_free(pv_a);
  cugraph_type_erased_device_array_free(pval_a);
  free_graph(&g);
  cugraph_free_resource_handle(h);
  return 0;
}

/* cpp/tests/c_api/bfs_test.c:118-143 */
static int test_bfs(void)
{
  static const int32_t exp_d[6] = {0, 1, 2147483647, 2, 2, 3};
  static const int32_t exp_p[6] = {-1, 0, -1, 1, 1, 3};
  static const int32_t src[1]   = {0};
  for (int t = 0; t < 2; ++t) {
    cugraph_resource_handle_t* h = cugraph_create_resource_handle(NULL);
    test_graph_t g;
    cugraph_error_t* err = NULL;
    cugraph_error_code_t rc = make_graph(h, E6_SRC, E6_DST, E6_W, 8, t ? TRUE : FALSE, FALSE, &g, &err);
    CHECK_RC(rc, err, "sg_graph_create");
    cugraph_type_erased_device_array_view_t* sv;
    cugraph_type_erased_device_array_t* sa = to_device(h, src, 1, INT32, &sv);
    CHECK(sa != NULL, "sources");
    cugraph_paths_result_t* res = NULL;
    rc = cugraph_bfs(h, g.graph, sv, FALSE, 10, TRUE, FALSE, &res, &err);
    CHECK_RC(rc, err, "cugraph_bfs");
    int32_t vert[6], dist[6], pred[6];
    cugraph_type_erased_device_array_view_t* vv = cugraph_paths_result_get_vertices(res);
    cugraph_type_erased_device_array_view_t* dv = cugraph_paths_result_get_distances(res);
    cugraph_type_erased_device_array_view_t* pv = cugraph_paths_result_get_predecessors(res);
    CHECK(cugraph_type_erased_device_array_view_size(dv) == 6, "bfs result size");
    rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)vert, vv, &err);
    CHECK_RC(rc, err, "copy");
    rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)dist, dv, &err);
    CHECK_RC(rc, err, "copy");
    rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)pred, pv, &err);
    CHECK_RC(rc, err, "copy");
    for (int i = 0; i < 6; ++i) {
      CHECK(dist[i] == exp_d[vert[i]], "bfs distance[%d] = %d, expected %d", vert[i], dist[i], exp_d[vert[i]]);
      CHECK(pred[i] == exp_p[vert[i]], "bfs predecessor[%d] = %d, expected %d", vert[i], pred[i],
            exp_p[vert[i]]);
    }
    cugraph_type_erased_device_array_view_free(vv);
    cugraph_type_erased_device_array_view_free(dv);
    cugraph_type_erased_device_array_view_free(pv);
    cugraph_paths_result_free(res);
    cugraph_type_erased_device_array_view_free(sv);
    cugraph_type_erased_device_array_free(sa);
    free_graph(&g);
    cugraph_free_resource_handle(h);
  }
  return 0;
}

/* cpp/tests/c_api/sssp_test.c:178-200 */
static int test_sssp(void)
{
  static const float exp_d[6]   = {0.0f, 0.1f, 3.4028235e38f, 2.2f, 1.2f, 4.4f};
  static const int32_t exp_p[6] = {-1, 0, -1, 1, 1, 4};
  cugraph_resource_handle_t* h  = cugraph_create_resource_handle(NULL);
  test_graph_t g;
  cugraph_error_t* err = NULL;
  cugraph_error_code_t rc = make_graph(h, E6_SRC, E6_DST, E6_W, 8, FALSE, FALSE, &g, &err);
  CHECK_RC(rc, err, "sg_graph_create");
  cugraph_paths_result_t* res = NULL;
  rc = cugraph_sssp(h, g.graph, 0, 10.0, TRUE, FALSE, &res, &err);
  CHECK_RC(rc, err, "cugraph_sssp");
  int32_t vert[6], pred[6];
  float dist[6];
  cugraph_type_erased_device_array_view_t* vv = cugraph_paths_result_get_vertices(res);
  cugraph_type_erased_device_array_view_t* dv = cugraph_paths_result_get_distances(res);
  cugraph_type_erased_device_array_view_t* pv = cugraph_paths_result_get_predecessors(res);
  rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)vert, vv, &err);
  CHECK_RC(rc, err, "copy");
  rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)dist, dv, &err);
  CHECK_RC(rc, err, "copy");
  rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)pred, pv, &err);
  CHECK_RC(rc, err, "copy");
  for (int i = 0; i < 6; ++i) {
    CHECK(close_rel(exp_d[vert[i]], dist[i], 1e-6), "sssp distance[%d] = %g, expected %g", vert[i], dist[i],
          exp_d[vert[i]]);
    CHECK(pred[i] == exp_p[vert[i]], "sssp predecessor[%d] = %d, expected %d", vert[i], pred[i], exp_p[vert[i]]);
  }
  cugraph_type_erased_device_array_view_free(vv);
  cugraph_type_erased_device_array_view_free(dv);
  cugraph_type_erased_device_array_view_free(pv);
  cugraph_paths_result_free(res);
  free_graph(&g);
  cugraph_free_resource_handle(h);
  return 0;
}

/* cpp/tests/c_api/louvain_test.c:101-127 (the 8 listed edges, symmetric graph) */
static int test_louvain(void)
{
  static const int32_t exp_c[6] = {0, 1, 0, 1, 1, 1};
  cugraph_resource_handle_t* h  = cugraph_create_resource_handle(NULL);
  test_graph_t g;
  cugraph_error_t* err = NULL;
  cugraph_error_code_t rc = make_graph(h, E6_SRC, E6_DST, E6_W, 8, FALSE, TRUE, &g, &err);
  CHECK_RC(rc, err, "sg_graph_create");
  cugraph_heirarchical_clustering_result_t* res = NULL;
  rc = cugraph_louvain(h, g.graph, 10, 1.0, FALSE, &res, &err);
  CHECK_RC(rc, err, "cugraph_louvain");
  int32_t vert[6], clus[6];
  cugraph_type_erased_device_array_view_t* vv = cugraph_heirarchical_clustering_result_get_vertices(res);
  cugraph_type_erased_device_array_view_t* cv = cugraph_heirarchical_clustering_result_get_clusters(res);
  double q = cugraph_heirarchical_clustering_result_get_modularity(res);
  rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)vert, vv, &err);
  CHECK_RC(rc, err, "copy");
  rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)clus, cv, &err);
  CHECK_RC(rc, err, "copy");
  for (int i = 0; i < 6; ++i)
    CHECK(clus[i] == exp_c[vert[i]], "louvain cluster[%d] = %d, expected %d", vert[i], clus[i], exp_c[vert[i]]);
  CHECK(close_rel(q, 0.218166, 1e-3), "modularity %g, expected 0.218166", q);
  cugraph_type_erased_device_array_view_free(vv);
  cugraph_type_erased_device_array_view_free(cv);
  cugraph_heirarchical_clustering_result_free(res);
  free_graph(&g);
  cugraph_free_resource_handle(h);
  return 0;
}

/* error contract: CAPI_EXPECTS failures come back as CUGRAPH_INVALID_INPUT with a message */
static int test_errors(void)
{
  cugraph_resource_handle_t* h = cugraph_create_resource_handle(NULL);
  test_graph_t g;
  cugraph_error_t* err = NULL;
  cugraph_error_code_t rc = make_graph(h, E6_SRC, E6_DST, E6_W, 8, TRUE, FALSE, &g, &err);
  CHECK_RC(rc, err, "sg_graph_create");
  cugraph_centrality_result_t* res = (cugraph_centrality_result_t*)&rc;  /* must be reset to NULL */
  rc = cugraph_pagerank(h, g.graph, NULL, NULL, NULL, NULL, 1.5, 1e-6, 100, FALSE, &res, &err);
  CHECK(rc == CUGRAPH_INVALID_INPUT, "alpha 1.5 gave %d", (int)rc);
  CHECK(res == NULL, "result not reset on error");
  CHECK(err != NULL && strlen(cugraph_error_message(err)) > 0, "no error message");
  cugraph_error_free(err);
  err = NULL;
  /* non-convergence is CUGRAPH_UNKNOWN_ERROR (pagerank_impl.cuh:287-291) */
  rc = cugraph_pagerank(h, g.graph, NULL, NULL, NULL, NULL, 0.95, 1e-30, 2, FALSE, &res, &err);
  CHECK(rc == CUGRAPH_UNKNOWN_ERROR, "non-convergence gave %d", (int)rc);
  cugraph_error_free(err);
  free_graph(&g);
  cugraph_free_resource_handle(h);
  return 0;
}

/* array.h:95 / :212: the caller takes ownership of the raw buffers */
static int test_release(void)
{
  cugraph_resource_handle_t* h = cugraph_create_resource_handle(NULL);
  cugraph_type_erased_device_array_view_t* v;
  int32_t host[5] = {7, 8, 9, 10, 11};
  cugraph_type_erased_device_array_t* a = to_device(h, host, 5, INT32, &v);
  CHECK(a != NULL, "device array");
  cugraph_type_erased_device_array_view_free(v);
  void* raw = cugraph_type_erased_device_array_release(a);
  CHECK(raw != NULL, "device release gave NULL");
  /* still readable through a fresh view over caller-owned memory */
  cugraph_type_erased_device_array_view_t* rv = cugraph_type_erased_device_array_view_create(raw, 5, INT32);
  int32_t back[5] = {0};
  cugraph_error_t* err = NULL;
  cugraph_error_code_t rc = cugraph_type_erased_device_array_view_copy_to_host(h, (byte_t*)back, rv, &err);
  CHECK_RC(rc, err, "copy released");
  CHECK(memcmp(back, host, sizeof(host)) == 0, "released device data differs");
  cugraph_type_erased_device_array_view_free(rv);
  /* the caller frees `raw` with hipFree; this C client has no HIP runtime linked, so the
   * block is left to process exit (the allocator no longer tracks it) */

  cugraph_type_erased_host_array_t* ha = NULL;
  rc = cugraph_type_erased_host_array_create(h, 3, FLOAT64, &ha, &err);
  CHECK_RC(rc, err, "host array");
  cugraph_type_erased_host_array_view_t* hv = cugraph_type_erased_host_array_view(ha);
  double* p = (double*)cugraph_type_erased_host_array_pointer(hv);
  p[0] = 1.5; p[1] = 2.5; p[2] = 3.5;
  cugraph_type_erased_host_array_view_free(hv);
  double* hr = (double*)cugraph_type_erased_host_array_release(ha);
  CHECK(hr && hr[0] == 1.5 && hr[2] == 3.5, "host release");
  free(hr);
  cugraph_free_resource_handle(h);
  return 0;
}

int main(void)
{
  struct { const char* name; int (*fn)(void); } tests[] = {
    {"pagerank", test_pagerank}, {"personalized_pagerank", test_personalized_pagerank},
    {"bfs", test_bfs},           {"sssp", test_sssp},
    {"louvain", test_louvain},   {"errors", test_errors},
    {"release", test_release},
  };
  for (size_t i = 0; i < sizeof(tests) / sizeof(tests[0]); ++i) {
    int before = g_failures;
    tests[i].fn();
    printf("%s %s\n", g_failures == before ? "PASS" : "FAIL", tests[i].name);
  }
  printf("%d failure(s)\n", g_failures);
  return g_failures;
}
