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

#ifdef __cplusplus
}
#endif
