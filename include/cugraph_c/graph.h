/*
 * libcugraph_c graph objects -- MI355X build.
 * ABI-compatible with the reference cpp/include/cugraph_c/graph.h:25-131.
 */
#pragma once
#include <cugraph_c/array.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { int32_t align_; } cugraph_graph_t;

/* reference graph.h:29-32 */
typedef struct {
  bool_t is_symmetric;
  bool_t is_multigraph;
} cugraph_graph_properties_t;

/*
 * reference graph.h:61-75 (implementation c_api/graph_sg.cpp:231).
 * src/dst: device arrays of INT32 or INT64 (same type); weights: FLOAT32/FLOAT64
 * or NULL (unweighted, treated as 1.0).  renumber=TRUE orders vertices by
 * descending major degree and drops ids that appear in no edge; FALSE keeps ids
 * and uses max(id)+1 vertices.  edge_ids/edge_types must both be NULL here.
 */
cugraph_error_code_t cugraph_sg_graph_create(
  const cugraph_resource_handle_t* handle,
  const cugraph_graph_properties_t* properties,
  const cugraph_type_erased_device_array_view_t* src,
  const cugraph_type_erased_device_array_view_t* dst,
  const cugraph_type_erased_device_array_view_t* weights,
  const cugraph_type_erased_device_array_view_t* edge_ids,
  const cugraph_type_erased_device_array_view_t* edge_types,
  bool_t store_transposed,
  bool_t renumber,
  bool_t check,
  cugraph_graph_t** graph,
  cugraph_error_t** error);

/* reference graph.h:82 */
void cugraph_sg_graph_free(cugraph_graph_t* graph);

/*
 * reference graph.h:110-124 (implementation c_api/graph_mg.cpp:239).
 * Collective over the communicator carried by the handle: every rank passes
 * its local slice of the edge list; edges are shuffled to their owners of the
 * 2D (row x col) partition.  num_edges is the global edge count.
 */
cugraph_error_code_t cugraph_mg_graph_create(
  const cugraph_resource_handle_t* handle,
  const cugraph_graph_properties_t* properties,
  const cugraph_type_erased_device_array_view_t* src,
  const cugraph_type_erased_device_array_view_t* dst,
  const cugraph_type_erased_device_array_view_t* weights,
  const cugraph_type_erased_device_array_view_t* edge_ids,
  const cugraph_type_erased_device_array_view_t* edge_types,
  bool_t store_transposed,
  size_t num_edges,
  bool_t check,
  cugraph_graph_t** graph,
  cugraph_error_t** error);

/* reference graph.h:131 */
void cugraph_mg_graph_free(cugraph_graph_t* graph);

#ifdef __cplusplus
}
#endif
