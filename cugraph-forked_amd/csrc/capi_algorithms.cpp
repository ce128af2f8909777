// libcugraph_c algorithm entry points on the hot path (MI355X build):
// PageRank, personalised PageRank, BFS, SSSP, Louvain and their result objects.
//
// Argument checks and error behaviour follow cpp/src/c_api/{pagerank.cpp:244-304,
// bfs.cpp:187-230, sssp.cpp:146-190, louvain.cpp:152-190} and the result getters
// cpp/src/c_api/{centrality_result.cpp, paths_result.cpp, louvain.cpp}.
#include "capi.hpp"

#include <cugraph_amd/ext.h>

using namespace cgx;

namespace cgx {
void run_pagerank(handle_t& h, graph_t& g, array_view_t const* pow_v, array_view_t const* pow_s,
                  array_view_t const* guess_v, array_view_t const* guess_s, array_view_t const* pers_v,
                  array_view_t const* pers_s, double alpha, double eps, size_t max_iter, bool expensive,
                  centrality_result_t& res);
void run_bfs(handle_t& h, graph_t& g, array_view_t* sources, bool direction_optimizing, size_t depth_limit,
             bool compute_predecessors, bool expensive, paths_result_t& res);
void run_sssp(handle_t& h, graph_t& g, size_t source, double cutoff, bool compute_predecessors, bool expensive,
              paths_result_t& res);
void run_louvain(handle_t& h, graph_t& g, size_t max_level, double resolution, bool expensive,
                 clustering_result_t& res);
void run_katz(handle_t& h, graph_t& g, array_view_t const* betas, double alpha, double beta, double eps,
              size_t max_iter, bool expensive, centrality_result_t& res);
void run_eigenvector(handle_t& h, graph_t& g, double eps, size_t max_iter, bool expensive, centrality_result_t& res);
void run_hits(handle_t& h, graph_t& g, double eps, size_t max_iter, array_view_t const* guess_v,
              array_view_t const* guess_s, bool normalize, bool expensive, hits_result_t& res);
void run_extract_paths(handle_t& h, graph_t& g, paths_result_t const& pr, array_view_t const* dests,
                       extract_paths_result_t& res);
void mg_run_pagerank(handle_t& h, graph_t& g, array_view_t const* pow_v, array_view_t const* pow_s,
                     array_view_t const* guess_v, array_view_t const* guess_s, array_view_t const* pers_v,
                     array_view_t const* pers_s, double alpha, double eps, size_t max_iter, bool expensive,
                     centrality_result_t& res);
void mg_run_bfs(handle_t& h, graph_t& g, array_view_t* sources, bool direction_optimizing, size_t depth_limit,
                bool compute_predecessors, bool expensive, paths_result_t& res);
void mg_run_sssp(handle_t& h, graph_t& g, size_t source, double cutoff, bool compute_predecessors, bool expensive,
                 paths_result_t& res);
}  // namespace cgx

namespace {

template <typename R>
R* out_ptr(R** p)
{
  *p = nullptr;
  return nullptr;
}

cugraph_error_code_t pagerank_common(const cugraph_resource_handle_t* handle,
                                     cugraph_graph_t* graph,
                                     const cugraph_type_erased_device_array_view_t* pow_v,
                                     const cugraph_type_erased_device_array_view_t* pow_s,
                                     const cugraph_type_erased_device_array_view_t* guess_v,
                                     const cugraph_type_erased_device_array_view_t* guess_s,
                                     const cugraph_type_erased_device_array_view_t* pers_v,
                                     const cugraph_type_erased_device_array_view_t* pers_s,
                                     double alpha,
                                     double epsilon,
                                     size_t max_iterations,
                                     bool_t do_expensive_check,
                                     cugraph_centrality_result_t** result,
                                     cugraph_error_t** error)
{
  *result = nullptr;
  *error  = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    CGX_INPUT(graph != nullptr, "Invalid input argument: graph is NULL");
    auto& g = *G(graph);
    // dtype checks of c_api/pagerank.cpp:260-290
    CGX_INPUT(!pow_v || AV(pow_v)->type == g.vertex_type,
              "vertex type of graph and precomputed_vertex_out_weight_vertices must match");
    CGX_INPUT(!pow_s || AV(pow_s)->type == g.weight_type,
              "weight type of graph and precomputed_vertex_out_weight_sums must match");
    CGX_INPUT(!guess_v || AV(guess_v)->type == g.vertex_type,
              "vertex type of graph and initial_guess_vertices must match");
    CGX_INPUT(!guess_s || AV(guess_s)->type == g.weight_type, "weight type of graph and initial_guess_values must match");
    CGX_INPUT(!pers_v || AV(pers_v)->type == g.vertex_type,
              "vertex type of graph and personalization_vertices must match");
    CGX_INPUT(!pers_s || AV(pers_s)->type == g.weight_type,
              "weight type of graph and personalization_values must match");
    auto res = std::make_unique<centrality_result_t>();
    auto f   = g.multi_gpu ? mg_run_pagerank : run_pagerank;
    f(*H(handle), g, pow_v ? AV(pow_v) : nullptr, pow_s ? AV(pow_s) : nullptr, guess_v ? AV(guess_v) : nullptr,
      guess_s ? AV(guess_s) : nullptr, pers_v ? AV(pers_v) : nullptr, pers_s ? AV(pers_s) : nullptr, alpha, epsilon,
      max_iterations, do_expensive_check == TRUE, *res);
    HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    *result = reinterpret_cast<cugraph_centrality_result_t*>(res.release());
  });
}

}  // namespace

// ============================================================== PageRank
extern "C" cugraph_error_code_t cugraph_pagerank(
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
  cugraph_error_t** error)
{
  return pagerank_common(handle, graph, precomputed_vertex_out_weight_vertices, precomputed_vertex_out_weight_sums,
                         initial_guess_vertices, initial_guess_values, nullptr, nullptr, alpha, epsilon,
                         max_iterations, do_expensive_check, result, error);
}

extern "C" cugraph_error_code_t cugraph_personalized_pagerank(
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
  cugraph_error_t** error)
{
  return pagerank_common(handle, graph, precomputed_vertex_out_weight_vertices, precomputed_vertex_out_weight_sums,
                         initial_guess_vertices, initial_guess_values, personalization_vertices,
                         personalization_values, alpha, epsilon, max_iterations, do_expensive_check, result, error);
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_centrality_result_get_vertices(
  cugraph_centrality_result_t* result)
{
  return new_view(reinterpret_cast<centrality_result_t*>(result)->vertices.get());
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_centrality_result_get_values(
  cugraph_centrality_result_t* result)
{
  return new_view(reinterpret_cast<centrality_result_t*>(result)->values.get());
}

extern "C" void cugraph_centrality_result_free(cugraph_centrality_result_t* result)
{
  delete reinterpret_cast<centrality_result_t*>(result);
}

// ============================================================== BFS / SSSP
extern "C" cugraph_error_code_t cugraph_bfs(const cugraph_resource_handle_t* handle,
                                           cugraph_graph_t* graph,
                                           cugraph_type_erased_device_array_view_t* sources,
                                           bool_t direction_optimizing,
                                           size_t depth_limit,
                                           bool_t compute_predecessors,
                                           bool_t do_expensive_check,
                                           cugraph_paths_result_t** result,
                                           cugraph_error_t** error)
{
  *result = nullptr;
  *error  = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    CGX_INPUT(graph != nullptr && sources != nullptr, "Invalid input argument: graph/sources is NULL");
    auto& g = *G(graph);
    // c_api/bfs.cpp:196-200
    CGX_INPUT(AV(sources)->type == g.vertex_type, "vertex type of graph and sources must match");
    auto res = std::make_unique<paths_result_t>();
    auto f   = g.multi_gpu ? mg_run_bfs : run_bfs;
    f(*H(handle), g, AV(sources), direction_optimizing == TRUE, depth_limit, compute_predecessors == TRUE,
      do_expensive_check == TRUE, *res);
    HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    *result = reinterpret_cast<cugraph_paths_result_t*>(res.release());
  });
}

extern "C" cugraph_error_code_t cugraph_sssp(const cugraph_resource_handle_t* handle,
                                            cugraph_graph_t* graph,
                                            size_t source,
                                            double cutoff,
                                            bool_t compute_predecessors,
                                            bool_t do_expensive_check,
                                            cugraph_paths_result_t** result,
                                            cugraph_error_t** error)
{
  *result = nullptr;
  *error  = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    CGX_INPUT(graph != nullptr, "Invalid input argument: graph is NULL");
    auto& g = *G(graph);
    auto res = std::make_unique<paths_result_t>();
    (g.multi_gpu ? mg_run_sssp : run_sssp)(*H(handle), g, source, cutoff, compute_predecessors == TRUE,
                                           do_expensive_check == TRUE, *res);
    HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    *result = reinterpret_cast<cugraph_paths_result_t*>(res.release());
  });
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_paths_result_get_vertices(cugraph_paths_result_t* result)
{
  return new_view(reinterpret_cast<paths_result_t*>(result)->vertices.get());
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_paths_result_get_distances(cugraph_paths_result_t* result)
{
  return new_view(reinterpret_cast<paths_result_t*>(result)->distances.get());
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_paths_result_get_predecessors(
  cugraph_paths_result_t* result)
{
  return new_view(reinterpret_cast<paths_result_t*>(result)->predecessors.get());
}

extern "C" void cugraph_paths_result_free(cugraph_paths_result_t* result)
{
  delete reinterpret_cast<paths_result_t*>(result);
}

// ============================================================== Louvain
extern "C" cugraph_error_code_t cugraph_louvain(const cugraph_resource_handle_t* handle,
                                               cugraph_graph_t* graph,
                                               size_t max_level,
                                               double resolution,
                                               bool_t do_expensive_check,
                                               cugraph_heirarchical_clustering_result_t** result,
                                               cugraph_error_t** error)
{
  *result = nullptr;
  *error  = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    CGX_INPUT(graph != nullptr, "Invalid input argument: graph is NULL");
    auto& g = *G(graph);
    auto res = std::make_unique<clustering_result_t>();
    run_louvain(*H(handle), g, max_level, resolution, do_expensive_check == TRUE, *res);
    HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    *result = reinterpret_cast<cugraph_heirarchical_clustering_result_t*>(res.release());
  });
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_heirarchical_clustering_result_get_vertices(
  cugraph_heirarchical_clustering_result_t* result)
{
  return new_view(reinterpret_cast<clustering_result_t*>(result)->vertices.get());
}

extern "C" size_t cugraph_amd_heirarchical_clustering_result_get_num_levels(
  cugraph_heirarchical_clustering_result_t* result)
{
  return reinterpret_cast<clustering_result_t*>(result)->levels.size();
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_amd_heirarchical_clustering_result_get_level(
  cugraph_heirarchical_clustering_result_t* result, size_t level)
{
  auto* r = reinterpret_cast<clustering_result_t*>(result);
  return level < r->levels.size() ? new_view(r->levels[level].get()) : nullptr;
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_heirarchical_clustering_result_get_clusters(
  cugraph_heirarchical_clustering_result_t* result)
{
  return new_view(reinterpret_cast<clustering_result_t*>(result)->clusters.get());
}

extern "C" double cugraph_heirarchical_clustering_result_get_modularity(
  cugraph_heirarchical_clustering_result_t* result)
{
  return reinterpret_cast<clustering_result_t*>(result)->modularity;
}

extern "C" void cugraph_heirarchical_clustering_result_free(cugraph_heirarchical_clustering_result_t* result)
{
  delete reinterpret_cast<clustering_result_t*>(result);
}

// ---------------------------------------------------------------- Katz / eigenvector / HITS
// (reference c_api/katz.cpp, eigenvector_centrality.cpp, hits.cpp)
extern "C" cugraph_error_code_t cugraph_katz_centrality(const cugraph_resource_handle_t* handle,
                                                       cugraph_graph_t* graph,
                                                       const cugraph_type_erased_device_array_view_t* betas,
                                                       double alpha,
                                                       double beta,
                                                       double epsilon,
                                                       size_t max_iterations,
                                                       bool_t do_expensive_check,
                                                       cugraph_centrality_result_t** result,
                                                       cugraph_error_t** error)
{
  *result = nullptr;
  *error  = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    CGX_INPUT(graph != nullptr, "Invalid input argument: graph is NULL");
    auto& g = *G(graph);
    CGX_EXPECTS(!g.multi_gpu, CUGRAPH_NOT_IMPLEMENTED, "multi-GPU Katz centrality is not implemented in this build");
    auto res = std::make_unique<centrality_result_t>();
    run_katz(*H(handle), g, betas ? AV(betas) : nullptr, alpha, beta, epsilon, max_iterations,
             do_expensive_check == TRUE, *res);
    HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    *result = reinterpret_cast<cugraph_centrality_result_t*>(res.release());
  });
}

extern "C" cugraph_error_code_t cugraph_eigenvector_centrality(const cugraph_resource_handle_t* handle,
                                                              cugraph_graph_t* graph,
                                                              double epsilon,
                                                              size_t max_iterations,
                                                              bool_t do_expensive_check,
                                                              cugraph_centrality_result_t** result,
                                                              cugraph_error_t** error)
{
  *result = nullptr;
  *error  = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    CGX_INPUT(graph != nullptr, "Invalid input argument: graph is NULL");
    auto& g = *G(graph);
    CGX_EXPECTS(!g.multi_gpu, CUGRAPH_NOT_IMPLEMENTED,
                "multi-GPU eigenvector centrality is not implemented in this build");
    auto res = std::make_unique<centrality_result_t>();
    run_eigenvector(*H(handle), g, epsilon, max_iterations, do_expensive_check == TRUE, *res);
    HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    *result = reinterpret_cast<cugraph_centrality_result_t*>(res.release());
  });
}

extern "C" cugraph_error_code_t cugraph_hits(const cugraph_resource_handle_t* handle,
                                            cugraph_graph_t* graph,
                                            double epsilon,
                                            size_t max_iterations,
                                            const cugraph_type_erased_device_array_view_t* initial_hubs_guess_vertices,
                                            const cugraph_type_erased_device_array_view_t* initial_hubs_guess_values,
                                            bool_t normalize,
                                            bool_t do_expensive_check,
                                            cugraph_hits_result_t** result,
                                            cugraph_error_t** error)
{
  *result = nullptr;
  *error  = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    CGX_INPUT(graph != nullptr, "Invalid input argument: graph is NULL");
    CGX_INPUT((initial_hubs_guess_vertices == nullptr) == (initial_hubs_guess_values == nullptr),
              "Invalid input argument: initial hubs guess vertices and values must be given together");
    auto& g = *G(graph);
    CGX_EXPECTS(!g.multi_gpu, CUGRAPH_NOT_IMPLEMENTED, "multi-GPU HITS is not implemented in this build");
    auto res = std::make_unique<hits_result_t>();
    run_hits(*H(handle), g, epsilon, max_iterations,
             initial_hubs_guess_vertices ? AV(initial_hubs_guess_vertices) : nullptr,
             initial_hubs_guess_values ? AV(initial_hubs_guess_values) : nullptr, normalize == TRUE,
             do_expensive_check == TRUE, *res);
    HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    *result = reinterpret_cast<cugraph_hits_result_t*>(res.release());
  });
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_hits_result_get_vertices(cugraph_hits_result_t* result)
{
  return new_view(reinterpret_cast<hits_result_t*>(result)->vertices.get());
}
extern "C" cugraph_type_erased_device_array_view_t* cugraph_hits_result_get_hubs(cugraph_hits_result_t* result)
{
  return new_view(reinterpret_cast<hits_result_t*>(result)->hubs.get());
}
extern "C" cugraph_type_erased_device_array_view_t* cugraph_hits_result_get_authorities(cugraph_hits_result_t* result)
{
  return new_view(reinterpret_cast<hits_result_t*>(result)->authorities.get());
}
extern "C" double cugraph_hits_result_get_hub_score_differences(cugraph_hits_result_t* result)
{
  return reinterpret_cast<hits_result_t*>(result)->hub_score_differences;
}
extern "C" size_t cugraph_hits_result_get_number_of_iterations(cugraph_hits_result_t* result)
{
  return reinterpret_cast<hits_result_t*>(result)->number_of_iterations;
}
extern "C" void cugraph_hits_result_free(cugraph_hits_result_t* result)
{
  delete reinterpret_cast<hits_result_t*>(result);
}

// ---------------------------------------------------------------- extract paths (c_api/extract_paths.cpp)
extern "C" cugraph_error_code_t cugraph_extract_paths(const cugraph_resource_handle_t* handle,
                                                     cugraph_graph_t* graph,
                                                     const cugraph_type_erased_device_array_view_t* sources,
                                                     const cugraph_paths_result_t* paths_result,
                                                     const cugraph_type_erased_device_array_view_t* destinations,
                                                     cugraph_extract_paths_result_t** result,
                                                     cugraph_error_t** error)
{
  *result = nullptr;
  *error  = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    CGX_INPUT(graph != nullptr && paths_result != nullptr && destinations != nullptr,
              "Invalid input argument: graph, paths result and destinations must be given");
    (void)sources;
    auto& g = *G(graph);
    CGX_EXPECTS(!g.multi_gpu, CUGRAPH_NOT_IMPLEMENTED, "multi-GPU extract_paths is not implemented in this build");
    auto res = std::make_unique<extract_paths_result_t>();
    run_extract_paths(*H(handle), g, *reinterpret_cast<paths_result_t const*>(paths_result), AV(destinations), *res);
    *result = reinterpret_cast<cugraph_extract_paths_result_t*>(res.release());
  });
}

extern "C" size_t cugraph_extract_paths_result_get_max_path_length(cugraph_extract_paths_result_t* result)
{
  return reinterpret_cast<extract_paths_result_t*>(result)->max_path_length;
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_extract_paths_result_get_paths(
  cugraph_extract_paths_result_t* result)
{
  return new_view(reinterpret_cast<extract_paths_result_t*>(result)->paths.get());
}

extern "C" void cugraph_extract_paths_result_free(cugraph_extract_paths_result_t* result)
{
  delete reinterpret_cast<extract_paths_result_t*>(result);
}
