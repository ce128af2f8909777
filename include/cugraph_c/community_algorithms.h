/*
 * libcugraph_c community entry points on the hot path -- MI355X build.
 * ABI-compatible with the reference cpp/include/cugraph_c/community_algorithms.h:83-136.
 */
#pragma once
#include <cugraph_c/error.h>
#include <cugraph_c/graph.h>
#include <cugraph_c/resource_handle.h>

#ifdef __cplusplus
extern "C" {
#endif

/* [sic] "heirarchical", as in the reference ABI */
typedef struct { int32_t align_; } cugraph_heirarchical_clustering_result_t;

/*
 * reference community_algorithms.h:105-111 (implementation c_api/louvain.cpp:152,
 * algorithm community/louvain_impl.cuh:46-301).
 */
cugraph_error_code_t cugraph_louvain(const cugraph_resource_handle_t* handle,
                                     cugraph_graph_t* graph,
                                     size_t max_level,
                                     double resolution,
                                     bool_t do_expensive_check,
                                     cugraph_heirarchical_clustering_result_t** result,
                                     cugraph_error_t** error);

/* reference community_algorithms.h:116 */
cugraph_type_erased_device_array_view_t* cugraph_heirarchical_clustering_result_get_vertices(
  cugraph_heirarchical_clustering_result_t* result);

/* reference community_algorithms.h:122 */
cugraph_type_erased_device_array_view_t* cugraph_heirarchical_clustering_result_get_clusters(
  cugraph_heirarchical_clustering_result_t* result);

/* reference community_algorithms.h:128 */
double cugraph_heirarchical_clustering_result_get_modularity(
  cugraph_heirarchical_clustering_result_t* result);

/* reference community_algorithms.h:136 */
void cugraph_heirarchical_clustering_result_free(cugraph_heirarchical_clustering_result_t* result);

#ifdef __cplusplus
}
#endif
