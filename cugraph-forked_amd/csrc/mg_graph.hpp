// Multi-GPU graph: vertex partition, 2D edge partition and id lookups.
//
// Reference: create_graph_from_edgelist_impl.cuh:194-555 (MG build),
// renumber_edgelist_impl.cuh:95-452, c_api/graph_mg.cpp:138-239 (edge shuffle by
// GPU id), partition_manager.hpp (2D grid).  Layout here:
//
//  * P = R x C ranks, rank p = r * C + c (C = row communicator size).
//  * Vertex owner of an external id: a hash (mg_owner_of_ext).  Each owner sorts its
//    vertices by descending degree (ties: ascending external id) and numbers them
//    voff[p] .. voff[p+1]-1: global ids are dense and every rank's range is
//    contiguous, hubs first.
//  * Edge (u, v) (global ids) lives on rank (row of owner(u), column of owner(v)):
//    row r holds the sources of ranks r*C .. r*C+C-1 (one contiguous id range),
//    column c the destinations of ranks c, C+c, 2C+c, ...  A PageRank iteration
//    then needs an allgather of x~ inside the row and a reduce-scatter of partial
//    sums inside the column.
#pragma once

#include "capi.hpp"
#include "comm.hpp"

#include <vector>

namespace cgx {

struct mg_graph_t {
  int P = 1, p = 0, R = 1, C = 1;
  std::vector<int64_t> voff;  // P + 1 global vertex offsets
  int64_t n_own() const { return voff[p + 1] - voff[p]; }
  int owner_of_global(int64_t x) const;  // host
  // owned vertices: external ids sorted ascending and their global ids (ext -> global lookup)
  buffer own_ext_sorted;  // vertex_t[n_own]
  buffer own_gid;         // vertex_t[n_own]
  // this rank's 2D block of edges (global ids), weights optional
  int64_t ne = 0;
  buffer src, dst, w;
  // per-algorithm caches (pagerank.hip, mg_bfs.hip, mg_sssp.hip)
  std::shared_ptr<void> pr_block;
  std::shared_ptr<void> bfs_rows;
  std::shared_ptr<void> bfs_block;  // the 2D block as a CSR over the row's sources (mg_bfs.hip)
  std::shared_ptr<void> sssp_rows;  // weighted out-rows by source owner (mg_sssp.hip)
  // every vertex's external id on every rank (global -> external, and external ids
  // sorted with their global ids): id translation of traversal results and sources
  // without a query exchange (V x 3 ids per rank: RMAT-26 394 MB of 288 GB); built on
  // first use by mg_ensure_replicated_ids
  bool rep_valid = false;
  buffer rep_nmap, rep_ext_sorted, rep_gid;
};

// owner of an external vertex id (hash), host and device
__host__ __device__ inline int mg_owner_of_ext(int64_t x, int P)
{
  unsigned long long z = (unsigned long long)x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (int)(z % (unsigned long long)P);
}

// owner rank of a global id: last p with voff[p] <= x (voff device array of P+1)
__device__ inline int mg_owner_of_global(int64_t x, int64_t const* voff, int P)
{
  int lo = 0, hi = P - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (voff[mid] <= x) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Build the MG graph (every rank calls with its local edge list, external ids).
void build_mg_graph(handle_t& h, graph_t& g, array_view_t const& src, array_view_t const& dst,
                    array_view_t const* weights);

// external ids (graph vertex type, device, n) -> global ids in place; collective.
// Unknown ids become -1 (check: throw CUGRAPH_INVALID_INPUT instead).
void mg_ext_to_global(handle_t& h, graph_t& g, void* ids, size_t n, bool check);
// global ids -> external ids in place (values outside [0, V) untouched); collective.
void mg_global_to_ext(handle_t& h, graph_t& g, void* ids, size_t n);
// The replicated id maps (mg_graph_t::rep_*): collective on first use, then local.
void mg_ensure_replicated_ids(handle_t& h, graph_t& g);
// The same translations through the replicated maps: no communication (after the
// maps exist); unknown external ids become -1
void mg_global_to_ext_local(handle_t& h, graph_t& g, void* ids, size_t n);
void mg_ext_to_global_local(handle_t& h, graph_t& g, void* ids, size_t n);

}  // namespace cgx
