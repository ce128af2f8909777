// Entry points whose HIP implementation lands in a later commit of this round.
#include "capi.hpp"

namespace cgx {
void mg_run_pagerank(handle_t&, graph_t&, array_view_t const*, array_view_t const*, array_view_t const*,
                     array_view_t const*, array_view_t const*, array_view_t const*, double, double, size_t, bool,
                     centrality_result_t&)
{
  fail(CUGRAPH_NOT_IMPLEMENTED, "MG PageRank: not built yet");
}
void mg_run_bfs(handle_t&, graph_t&, array_view_t*, bool, size_t, bool, bool, paths_result_t&)
{
  fail(CUGRAPH_NOT_IMPLEMENTED, "MG BFS: not built yet");
}
void* comm_from_raft_handle(void* p) { return p; }
int comm_rank(comm_t*) { return 0; }
}  // namespace cgx

extern "C" cugraph_error_code_t cugraph_mg_graph_create(const cugraph_resource_handle_t*,
                                                       const cugraph_graph_properties_t*,
                                                       const cugraph_type_erased_device_array_view_t*,
                                                       const cugraph_type_erased_device_array_view_t*,
                                                       const cugraph_type_erased_device_array_view_t*,
                                                       const cugraph_type_erased_device_array_view_t*,
                                                       const cugraph_type_erased_device_array_view_t*,
                                                       bool_t,
                                                       size_t,
                                                       bool_t,
                                                       cugraph_graph_t** graph,
                                                       cugraph_error_t** error)
{
  *graph = nullptr;
  *error = nullptr;
  return cgx::guarded(error, [&] { cgx::fail(CUGRAPH_NOT_IMPLEMENTED, "MG graph: not built yet"); });
}
extern "C" void cugraph_mg_graph_free(cugraph_graph_t* graph) { delete cgx::G(graph); }
