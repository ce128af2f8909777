// Degree-binned work schedule shared by the pull SpMV (PageRank) and the
// bottom-up BFS kernels.
//
// The reference splits majors into segments [deg >= 1024 | >= 32 | >= 1 | 0]
// after renumbering by descending degree (cpp/include/cugraph/graph_view.hpp:255-263,
// renumber_edgelist_impl.cuh:392-451) and runs block / warp(32) / thread kernels
// per segment (prims/per_v_transform_reduce_incoming_outgoing_e.cuh:194-479).
// For 64-wide CDNA4 wavefronts we use finer power-of-two bins: a vertex of
// degree d in [2^k, 2^(k+1)) is served by a lane group of width
// min(64, 2^(k-1)) so every lane issues 2-3 gathers, a whole 256-thread block
// serves degree >= 4096.  Vertices are visited in descending-degree order, so
// every bin is one contiguous range and a work item is (width, [begin, end)).
#pragma once

#include <cstdint>

namespace cgx {

constexpr int kSchedBins = 9;
// lower degree bound of each bin, descending
constexpr int64_t kBinLo[kSchedBins] = {4096, 128, 64, 32, 16, 8, 4, 1, 0};
// lanes per vertex; 256 = whole block
constexpr int kBinWidth[kSchedBins] = {256, 64, 32, 16, 8, 4, 2, 1, 1};

struct work_item {
  int32_t width;  // lanes per vertex (1..64) or 256 (block per vertex)
  int32_t bin;
  int64_t begin;  // positions in processing order
  int64_t end;
};

}  // namespace cgx
