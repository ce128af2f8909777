/*
 * Umbrella header (reference cpp/include/cugraph_c/algorithms.h).  This build
 * provides the hot-path families only.
 */
#pragma once
#include <cugraph_c/array.h>
#include <cugraph_c/centrality_algorithms.h>
#include <cugraph_c/community_algorithms.h>
#include <cugraph_c/error.h>
#include <cugraph_c/graph.h>
#include <cugraph_c/resource_handle.h>
#include <cugraph_c/traversal_algorithms.h>
