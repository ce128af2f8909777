// Entry points whose HIP implementation lands in a later commit of this round.
#include "capi.hpp"

namespace cgx {
void mg_run_bfs(handle_t&, graph_t&, array_view_t*, bool, size_t, bool, bool, paths_result_t&)
{
  fail(CUGRAPH_NOT_IMPLEMENTED, "MG BFS: not built yet");
}
}  // namespace cgx

