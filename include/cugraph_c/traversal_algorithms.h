/*
 * libcugraph_c traversal entry points on the hot path -- MI355X build.
 * ABI-compatible with the reference cpp/include/cugraph_c/traversal_algorithms.h:38-145.
 */
#pragma once
#include <cugraph_c/array.h>
#include <cugraph_c/error.h>
#include <cugraph_c/graph.h>
#include <cugraph_c/resource_handle.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { int32_t align_; } cugraph_paths_result_t;

/* reference traversal_algorithms.h:48 */
cugraph_type_erased_device_array_view_t* cugraph_paths_result_get_vertices(
  cugraph_paths_result_t* result);

/* reference traversal_algorithms.h:57 */
cugraph_type_erased_device_array_view_t* cugraph_paths_result_get_distances(
  cugraph_paths_result_t* result);

/* reference traversal_algorithms.h:68 -- empty when predecessors were not computed */
cugraph_type_erased_device_array_view_t* cugraph_paths_result_get_predecessors(
  cugraph_paths_result_t* result);

/* reference traversal_algorithms.h:76 */
void cugraph_paths_result_free(cugraph_paths_result_t* result);

/*
 * reference traversal_algorithms.h:105-115 (implementation c_api/bfs.cpp:187,
 * algorithm traversal/bfs_impl.cuh:94-287).  sources are renumbered in place
 * (as the reference does).  direction_optimizing=TRUE requires a symmetric
 * graph (the reference throws "unimplemented"; this build implements it).
 * Predecessor = the frontier neighbour with the smallest internal id.
 */
cugraph_error_code_t cugraph_bfs(
  const cugraph_resource_handle_t* handle,
  cugraph_graph_t* graph,
  cugraph_type_erased_device_array_view_t* sources,
  bool_t direction_optimizing,
  size_t depth_limit,
  bool_t compute_predecessors,
  bool_t do_expensive_check,
  cugraph_paths_result_t** result,
  cugraph_error_t** error);

/*
 * reference traversal_algorithms.h:138-145 (implementation c_api/sssp.cpp:146,
 * algorithm traversal/sssp_impl.cuh:79-270).
 */
cugraph_error_code_t cugraph_sssp(const cugraph_resource_handle_t* handle,
                                  cugraph_graph_t* graph,
                                  size_t source,
                                  double cutoff,
                                  bool_t compute_predecessors,
                                  bool_t do_expensive_check,
                                  cugraph_paths_result_t** result,
                                  cugraph_error_t** error);

/* extract_paths result, reference traversal_algorithms.h:147-204 */
typedef struct {
  int32_t align_;
} cugraph_extract_paths_result_t;

/*
 * Paths from a BFS/SSSP result back to the source (reference traversal_algorithms.h:173-180,
 * traversal/extract_bfs_paths_impl.cuh): row-major [destinations x max_path_length]
 * matrix of external vertex ids, -1 padded.
 */
cugraph_error_code_t cugraph_extract_paths(const cugraph_resource_handle_t* handle,
                                           cugraph_graph_t* graph,
                                           const cugraph_type_erased_device_array_view_t* sources,
                                           const cugraph_paths_result_t* paths_result,
                                           const cugraph_type_erased_device_array_view_t* destinations,
                                           cugraph_extract_paths_result_t** result,
                                           cugraph_error_t** error);
size_t cugraph_extract_paths_result_get_max_path_length(cugraph_extract_paths_result_t* result);
cugraph_type_erased_device_array_view_t* cugraph_extract_paths_result_get_paths(
  cugraph_extract_paths_result_t* result);
void cugraph_extract_paths_result_free(cugraph_extract_paths_result_t* result);

#ifdef __cplusplus
}
#endif
