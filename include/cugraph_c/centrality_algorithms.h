/*
 * libcugraph_c centrality entry points on the hot path -- MI355X build.
 * ABI-compatible with the reference cpp/include/cugraph_c/centrality_algorithms.h:36-171.
 */
#pragma once
#include <cugraph_c/array.h>
#include <cugraph_c/error.h>
#include <cugraph_c/graph.h>
#include <cugraph_c/resource_handle.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { int32_t align_; } cugraph_centrality_result_t;

/* reference centrality_algorithms.h:46 -- external vertex ids (the number map) */
cugraph_type_erased_device_array_view_t* cugraph_centrality_result_get_vertices(
  cugraph_centrality_result_t* result);

/* reference centrality_algorithms.h:55 */
cugraph_type_erased_device_array_view_t* cugraph_centrality_result_get_values(
  cugraph_centrality_result_t* result);

/* reference centrality_algorithms.h:63 */
void cugraph_centrality_result_free(cugraph_centrality_result_t* result);

/*
 * reference centrality_algorithms.h:102-114 (implementation c_api/pagerank.cpp:244-304,
 * algorithm link_analysis/pagerank_impl.cuh:48-293).  Converges when the L1
 * difference of two consecutive iterates is < epsilon (plain epsilon, as the
 * reference implementation does); otherwise CUGRAPH_UNKNOWN_ERROR
 * ("PageRank failed to converge.") after max_iterations.
 */
cugraph_error_code_t cugraph_pagerank(
  const cugraph_resource_handle_t* handle,
  cugraph_graph_t* graph,
  const cugraph_type_erased_device_array_view_t* precomputed_vertex_out_weight_vertices,
  const cugraph_type_erased_device_array_view_t* precomputed_vertex_out_weight_sums,
  const cugraph_type_erased_device_array_view_t* initial_guess_vertices,
  const cugraph_type_erased_device_array_view_t* initial_guess_values,
  double alpha,
  double epsilon,
  size_t max_iterations,
  bool_t do_expensive_check,
  cugraph_centrality_result_t** result,
  cugraph_error_t** error);

/* reference centrality_algorithms.h:157-171 */
cugraph_error_code_t cugraph_personalized_pagerank(
  const cugraph_resource_handle_t* handle,
  cugraph_graph_t* graph,
  const cugraph_type_erased_device_array_view_t* precomputed_vertex_out_weight_vertices,
  const cugraph_type_erased_device_array_view_t* precomputed_vertex_out_weight_sums,
  const cugraph_type_erased_device_array_view_t* initial_guess_vertices,
  const cugraph_type_erased_device_array_view_t* initial_guess_values,
  const cugraph_type_erased_device_array_view_t* personalization_vertices,
  const cugraph_type_erased_device_array_view_t* personalization_values,
  double alpha,
  double epsilon,
  size_t max_iterations,
  bool_t do_expensive_check,
  cugraph_centrality_result_t** result,
  cugraph_error_t** error);

/*
 * Eigenvector centrality, reference centrality_algorithms.h:191-197
 * (centrality/eigenvector_centrality_impl.cuh): power method, L2 normalised,
 * stop when the L1 change < |V| * epsilon, else CUGRAPH_UNKNOWN_ERROR.
 */
cugraph_error_code_t cugraph_eigenvector_centrality(const cugraph_resource_handle_t* handle,
                                                    cugraph_graph_t* graph,
                                                    double epsilon,
                                                    size_t max_iterations,
                                                    bool_t do_expensive_check,
                                                    cugraph_centrality_result_t** result,
                                                    cugraph_error_t** error);

/*
 * Katz centrality, reference centrality_algorithms.h:224-233 (c_api/katz.cpp):
 * betas (optional) are indexed by external vertex id; results are L2 normalised.
 */
cugraph_error_code_t cugraph_katz_centrality(const cugraph_resource_handle_t* handle,
                                             cugraph_graph_t* graph,
                                             const cugraph_type_erased_device_array_view_t* betas,
                                             double alpha,
                                             double beta,
                                             double epsilon,
                                             size_t max_iterations,
                                             bool_t do_expensive_check,
                                             cugraph_centrality_result_t** result,
                                             cugraph_error_t** error);

/* HITS result, reference centrality_algorithms.h:238-290 */
typedef struct {
  int32_t align_;
} cugraph_hits_result_t;

cugraph_type_erased_device_array_view_t* cugraph_hits_result_get_vertices(cugraph_hits_result_t* result);
cugraph_type_erased_device_array_view_t* cugraph_hits_result_get_hubs(cugraph_hits_result_t* result);
cugraph_type_erased_device_array_view_t* cugraph_hits_result_get_authorities(cugraph_hits_result_t* result);
double cugraph_hits_result_get_hub_score_differences(cugraph_hits_result_t* result);
size_t cugraph_hits_result_get_number_of_iterations(cugraph_hits_result_t* result);
void cugraph_hits_result_free(cugraph_hits_result_t* result);

/* HITS, reference centrality_algorithms.h:322-332 (link_analysis/hits_impl.cuh) */
cugraph_error_code_t cugraph_hits(
  const cugraph_resource_handle_t* handle,
  cugraph_graph_t* graph,
  double epsilon,
  size_t max_iterations,
  const cugraph_type_erased_device_array_view_t* initial_hubs_guess_vertices,
  const cugraph_type_erased_device_array_view_t* initial_hubs_guess_values,
  bool_t normalize,
  bool_t do_expensive_check,
  cugraph_hits_result_t** result,
  cugraph_error_t** error);

#ifdef __cplusplus
}
#endif
