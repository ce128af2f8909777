/*
 * MI355X build extensions around the libcugraph_c boundary.
 *
 * These are the data formats either side of the hot path that the reference
 * provides through other layers (RAFT's R-MAT generator behind
 * cugraph.generators.rmat, cudf-based symmetrize/dedup behind
 * cugraph.Graph.from_cudf_edgelist) plus measurement hooks.  Nothing here is
 * needed by a caller that only uses the reference ABI.
 */
#pragma once
#include <cugraph_c/algorithms.h>

#ifdef __cplusplus
extern "C" {
#endif

/*
 * Counter-based Graph500 R-MAT edge generator (definition in oracle/rmat.py;
 * role of the reference cpp/src/generators/generate_rmat_edgelist.cu:36-103).
 * Edges [first_edge, first_edge + num_edges) of the stream for `seed`.
 * vertex_dtype: INT32 or INT64.
 */
cugraph_error_code_t cugraph_amd_generate_rmat_edgelist(const cugraph_resource_handle_t* handle,
                                                        size_t scale,
                                                        size_t num_edges,
                                                        double a,
                                                        double b,
                                                        double c,
                                                        uint64_t seed,
                                                        bool_t clip_and_flip,
                                                        bool_t scramble_vertex_ids,
                                                        size_t first_edge,
                                                        data_type_id_t vertex_dtype,
                                                        cugraph_type_erased_device_array_t** src,
                                                        cugraph_type_erased_device_array_t** dst,
                                                        cugraph_error_t** error);

/* Uniform [0,1) edge weights, 24-bit exact (oracle/rmat.py rmat_weights). */
cugraph_error_code_t cugraph_amd_generate_edge_weights(const cugraph_resource_handle_t* handle,
                                                       size_t num_edges,
                                                       uint64_t seed,
                                                       size_t first_edge,
                                                       data_type_id_t weight_dtype,
                                                       cugraph_type_erased_device_array_t** weights,
                                                       cugraph_error_t** error);

/*
 * cugraph.Graph edge-list preprocessing on the device
 * (python/cugraph/cugraph/structure/symmetrize.py:78-93): optionally append
 * reversed edges, then drop duplicate (src, dst) pairs keeping the minimum
 * weight.  Output is sorted by (src, dst).  weights may be NULL.
 */
cugraph_error_code_t cugraph_amd_symmetrize_dedup(const cugraph_resource_handle_t* handle,
                                                  const cugraph_type_erased_device_array_view_t* src,
                                                  const cugraph_type_erased_device_array_view_t* dst,
                                                  const cugraph_type_erased_device_array_view_t* weights,
                                                  bool_t symmetrize,
                                                  cugraph_type_erased_device_array_t** src_out,
                                                  cugraph_type_erased_device_array_t** dst_out,
                                                  cugraph_type_erased_device_array_t** weights_out,
                                                  cugraph_error_t** error);

/* Graph introspection (vertex count after renumbering, stored edge count). */
int64_t cugraph_amd_graph_get_number_of_vertices(const cugraph_graph_t* graph);
int64_t cugraph_amd_graph_get_number_of_edges(const cugraph_graph_t* graph);
bool_t cugraph_amd_graph_is_symmetric(const cugraph_graph_t* graph);

/*
 * Copy the graph's compressed adjacency to caller device buffers (for tests):
 * transposed=FALSE gives CSR (out-edges), TRUE gives CSC (in-edges), in the
 * graph's internal (renumbered) ids.  Pass NULL to query sizes only.
 */
cugraph_error_code_t cugraph_amd_graph_get_adjacency(const cugraph_resource_handle_t* handle,
                                                     cugraph_graph_t* graph,
                                                     bool_t transposed,
                                                     cugraph_type_erased_device_array_t** offsets,
                                                     cugraph_type_erased_device_array_t** indices,
                                                     cugraph_type_erased_device_array_t** weights,
                                                     cugraph_error_t** error);

/*
 * Copy the graph's per-vertex out-weight sums (weight_t[V], internal order; the
 * out-degree for unweighted graphs) -- compute_out_weight_sums of
 * pagerank_impl.cuh:158-164, as PageRank computes and caches them -- to a new
 * device array (for tests).
 */
cugraph_error_code_t cugraph_amd_graph_get_out_weight_sums(const cugraph_resource_handle_t* handle,
                                                           cugraph_graph_t* graph,
                                                           cugraph_type_erased_device_array_t** sums,
                                                           cugraph_error_t** error);

/*
 * Copy n device array views (dst[i] <- src[i], same type and size) with one
 * stream synchronize at the end: the batched form of
 * cugraph_type_erased_device_array_view_copy (array.h) for result extraction.
 */
cugraph_error_code_t cugraph_amd_device_array_views_copy(const cugraph_resource_handle_t* handle,
                                                         size_t n,
                                                         cugraph_type_erased_device_array_view_t* const* dst,
                                                         const cugraph_type_erased_device_array_view_t* const* src,
                                                         cugraph_error_t** error);

/*
 * Measurement hooks.  When profiling is on, algorithms record HIP events
 * around every launch of their dominant kernel (on the handle's stream) and
 * keep the total; stats are per handle and reset by each algorithm call.
 */
void cugraph_amd_set_profiling(cugraph_resource_handle_t* handle, bool_t enable);
size_t cugraph_amd_last_iterations(const cugraph_resource_handle_t* handle);
/*
 * Measurement / A-B switches, per handle (the reference's tuning constants are
 * constexpr; these select the alternatives DESIGN.md measured, for A/B scripts and
 * the bitwise-equality tests).  Names: pr_win_bits (0 | 12 | 13 | 14 | 15), pr_packed,
 * pr_whole, pr_calib, pr_deal_global, pr_unit_w, pr_fuse, pr_enc, pr_hub, pr_band_cut (-1 | 0 | cut),
 * mg_bfs_alpha, mg_bfs_beta, mg_bfs_pipelined (1 | 0), pr_fast_build, pr_share_div (0 | n),
 * mg_chunks, bfs_alpha, bfs_beta, bfs_probe_vec, bfs_head, bfs_res_grid,
 * bfs_probe_grid, bfs_td_cap, louvain_hash, louvain_big_hash, louvain_big_cap,
 * louvain_big_maxdeg, louvain_wide_keys, sssp_delta (0 | scale: delta = scale * average weight /
 * average degree), sssp_pull (0 by size | -1 never | n); "defaults" resets them all.  Booleans
 * are 0 / 1.  Unknown names: CUGRAPH_INVALID_INPUT.
 */
cugraph_error_code_t cugraph_amd_set_option(cugraph_resource_handle_t* handle, const char* name, double value,
                                            cugraph_error_t** error);
double cugraph_amd_last_hot_kernel_ms(const cugraph_resource_handle_t* handle);
size_t cugraph_amd_last_hot_kernel_launches(const cugraph_resource_handle_t* handle);
/* BFS: edges examined, levels, top-down/bottom-up steps of the last call */
size_t cugraph_amd_last_bfs_levels(const cugraph_resource_handle_t* handle);
size_t cugraph_amd_last_bfs_bottom_up_steps(const cugraph_resource_handle_t* handle);
/* Louvain: levels of the last call */
size_t cugraph_amd_last_louvain_levels(const cugraph_resource_handle_t* handle);
/* Multi-GPU Louvain: average bytes this rank sent per local-move sweep (cluster
 * lookups, weight deltas, ghost updates) in the last call; 0 on one GPU */
double cugraph_amd_last_louvain_sweep_bytes(const cugraph_resource_handle_t* handle);
/* Multi-GPU Louvain: this rank's level-0 share of the 1D partition in the last call --
 * its edges (the rows it owns) and its ghosts (distinct destinations owned elsewhere,
 * whose clusters it mirrors); 0 and 0 on one GPU */
void cugraph_amd_last_louvain_partition(const cugraph_resource_handle_t* handle, int64_t* local_edges,
                                        int64_t* ghosts);
/* Louvain dendrogram (the reference C++ API returns Dendrogram<vertex_t>,
 * louvain_impl.cuh:280-301; the C ABI only exposes the flattened clustering).
 * Level i holds the cluster of every level-i vertex this rank owns, in global-id
 * order (a rank's level-i vertices are one contiguous id range, ranks in order);
 * its values are level-(i+1) vertex ids.  The view lives as long as the result. */
size_t cugraph_amd_heirarchical_clustering_result_get_num_levels(cugraph_heirarchical_clustering_result_t* result);
cugraph_type_erased_device_array_view_t* cugraph_amd_heirarchical_clustering_result_get_level(
  cugraph_heirarchical_clustering_result_t* result, size_t level);

/* Return every cached HBM block of libcugraph_c's caching allocator to the driver
 * (synchronises the device).  Returns the bytes released.  The reference's
 * equivalent is releasing its RMM pool. */
size_t cugraph_amd_trim_device_cache(void);

/* The caching allocator's counters since the process started: out[0] driver
 * allocations (hipMalloc), out[1] their bytes, out[2] the seconds spent in them,
 * out[3] out-of-memory trims (every cached block released, then one retry),
 * out[4] bytes cached now.  Measurement aid. */
void cugraph_amd_allocator_stats(double* out);

/* Measured HBM ceiling: a 16-B-per-lane grid-stride copy of `bytes` (nontemporal
 * loads and stores), `reps` launches timed with HIP events on the handle's stream.
 * Returns (read + write bytes) / time in GB/s, or a negative value on error. */
double cugraph_amd_measure_copy_bandwidth(const cugraph_resource_handle_t* handle, size_t bytes, int reps);

/* Library build string, e.g. "cugraph-forked_amd gfx950 <date>". */
const char* cugraph_amd_version(void);

#ifdef __cplusplus
}
#endif
