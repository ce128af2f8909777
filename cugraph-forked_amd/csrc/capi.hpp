// Internal representations behind the opaque libcugraph_c handles (MI355X build).
//
// Layout mirrors what the reference keeps behind the same opaque pointers
// (cpp/src/c_api/{resource_handle,array,error,graph}.hpp) but the storage is our
// own: a graph owns its compressed adjacency in one or both orientations
// (out-edges "CSR", in-edges "CSC"; one shared object when the graph is
// symmetric), the number map, and lazily-built per-orientation scheduling data
// for the degree-binned kernels.
#pragma once

#include "common.hpp"

#include <cugraph_c/algorithms.h>

#include <memory>
#include <string>
#include <cstring>
#include <vector>

namespace cgx {

struct mg_graph_t;  // mg_graph.hpp
struct mg_context;  // comm.hpp (multi-GPU); nullptr for single GPU

// Measurement / A-B switches of the kernels, per handle (cugraph_amd_set_option,
// include/cugraph_amd/ext.h).  The defaults are the production choices; the other
// values select the measured alternatives DESIGN.md records, for the A/B scripts and
// the bitwise-equality tests.  Nothing here is read from the environment.
// Schedule-time switches (pr_win_bits, pr_packed, pr_whole) apply to schedules built
// after they are set: the push schedule is cached on the graph.
struct tuning_t {
  int pr_win_bits      = 0;     // 0: by size (push_win_bits); 12 / 13 / 14 / 15 force 4K / 8K / 16K / 32K windows
                                // (15: single-GPU symmetric unweighted schedules only, else 14)
  bool pr_packed       = true;  // 16-bit entries for unweighted graphs (else 32-bit)
  bool pr_whole        = true;  // windows summed by one item are stored, not added
  bool pr_calib        = true;  // measured-cost queues after the first launch
  bool pr_deal_global  = false; // measured items in one longest-first queue instead of 8 XCD queues
  bool pr_unit_w       = true;  // all-ones weights run the unweighted push
  bool pr_fuse         = true;  // apply fused into the 16K-window push
  bool pr_enc          = true;  // x~ as fixed-point words (fp32 single GPU)
  bool pr_hub          = true;  // hub x~ staged in LDS (16K windows)
  int64_t pr_band_cut  = -1;    // banded push source cut (-1: by size, 0: no bands)
  int pr_share_div     = 0;     // items per push block on average (0: kShareDiv); windows above 1.5x are shared
  bool pr_fast_build   = true;  // symmetric unweighted schedules through one-word keys (else the general build)
  int mg_chunks        = 0;     // MG overlap chunks (0: one chunk, no overlap)
  double bfs_alpha     = 40.0;  // direction switch (Beamer's alpha / beta)
  double bfs_beta      = 64.0;
  double mg_bfs_alpha  = 40.0;  // multi-GPU BFS direction switch (mg_bfs.hip; one-rank RMAT-24: 40 / 64
  double mg_bfs_beta   = 64.0;  // 2.92 vs Beamer's 14 / 24 3.20 ms per traversal)
  int mg_bfs_pipelined = 1;     // MG BFS: bottom-up levels enqueued a level ahead, counts read late (mg_bfs.hip bu_state)
  bool bfs_probe_vec   = true;  // bottom-up probe by 16-byte loads
  bool bfs_head        = true;  // bottom-up probe's head table
  int bfs_res_grid     = 1024;  // residual scan blocks
  int bfs_probe_grid   = 4096;  // probe blocks
  int64_t bfs_td_cap   = 1024;  // top-down blocks per degree-class segment
  bool louvain_hash    = true;  // LDS-hash local move (else sort + reduce-by-key)
  bool louvain_big_hash = true; // heavy rows on the LDS passes (else the sort path)
  int louvain_big_cap  = 0;     // (row, bucket) table cap below the built-in one (tests of the fallback)
  int64_t louvain_big_maxdeg = 0;  // heavy rows above this degree on the sort path (0: the table limit)
  bool louvain_wide_keys = false;  // 64-bit hash keys below 2^24 ids (tests)
  double sssp_delta    = 0;     // SSSP delta = sssp_delta * average weight / average degree (0: sssp.hip kDeltaScale)
  int sssp_pull        = 0;     // SSSP dense rounds by pull: 0 by size (sssp.hip kPullDiv), -1 never, n: list > part / n
};

struct handle_t {
  int device         = 0;
  hipStream_t stream = nullptr;
  mg_context* mg     = nullptr;
  bool profiling     = false;
  tuning_t tune;
  // statistics of the last algorithm call (see include/cugraph_amd/ext.h)
  size_t last_iterations     = 0;
  double last_hot_ms         = 0;
  size_t last_hot_launches   = 0;
  size_t last_bfs_levels     = 0;
  size_t last_bfs_bottom_up  = 0;
  size_t last_louvain_levels = 0;
  double last_louvain_sweep_bytes = 0;  // MG: average bytes sent per sweep by this rank
  int64_t last_louvain_local_edges = 0;  // MG: this rank's level-0 edges (rows it owns)
  int64_t last_louvain_ghosts      = 0;  // MG: its level-0 ghosts (distinct remote destinations)
  // Host-pinned scratch for the per-level / per-chunk device state reads and a pool
  // of profiling events, both kept for the handle's lifetime: hipHostMalloc +
  // hipHostFree per call measured ~250 us of host stall per BFS traversal.
  void* pinned = nullptr;
  std::vector<hipEvent_t> events;
  template <typename T>
  T* pinned_as()
  {
    static_assert(sizeof(T) <= kPinnedBytes, "pinned scratch too small");
    if (!pinned) HIP_CHECK(hipHostMalloc(&pinned, kPinnedBytes, hipHostMallocDefault));
    return static_cast<T*>(pinned);
  }
  // Coherent (fine-grained) pinned block the host polls while the stream runs on:
  // a kernel publishes values and then a sequence number with system-scope stores.
  // It must stay hipHostMallocCoherent (uncached): bfs.hip k_publish_seq orders the
  // words before the sequence number with a vmcnt wait only, no release.
  void* polled = nullptr;
  template <typename T>
  T* polled_as()
  {
    static_assert(sizeof(T) <= kPinnedBytes, "polled scratch too small");
    if (!polled) {
      HIP_CHECK(hipHostMalloc(&polled, kPinnedBytes, hipHostMallocCoherent));
      std::memset(polled, 0, kPinnedBytes);
    }
    return static_cast<T*>(polled);
  }
  hipEvent_t event(size_t i)  // the i-th pooled event (created on first use)
  {
    while (events.size() <= i) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreate(&e));
      events.push_back(e);
    }
    return events[i];
  }
  static constexpr size_t kPinnedBytes = 4096;
  ~handle_t()
  {
    if (pinned) (void)hipHostFree(pinned);
    if (polled) (void)hipHostFree(polled);
    for (auto e : events) (void)hipEventDestroy(e);
  }
};

struct array_view_t {  // reference c_api/array.hpp:30-35
  void* data           = nullptr;
  size_t size          = 0;
  size_t num_bytes     = 0;
  data_type_id_t type  = INT32;
  template <typename T>
  T* as() const
  {
    return static_cast<T*>(data);
  }
};

struct device_array_t {
  buffer buf;
  size_t size         = 0;
  data_type_id_t type = INT32;
  device_array_t(size_t n, data_type_id_t t, hipStream_t s) : buf(n * dtype_size(t), s), size(n), type(t) {}
  array_view_t view() const { return array_view_t{buf.data(), size, size * dtype_size(type), type}; }
};

struct host_array_t {
  std::vector<std::byte> data;
  size_t size         = 0;
  data_type_id_t type = INT32;
};

struct err_t {
  std::string message;
};

// PageRank windowed-push schedule of one edge set (pagerank.hip): packed entries
// sorted by (destination window, source), work units and fixed-point accumulators
struct pr_push_t {
  bool built = false;
  bool ok    = false;  // ids and edge positions fit the 32-bit packing
  int win_bits = 12;   // destination window = 2^win_bits consecutive rows
  buffer ent;          // uint32[E + unit]: (source - unit's first source) << win_bits | (row - window base)
  buffer ew;           // weight_t[E + unit] for weighted graphs
  bool packed = false; // 16-bit entries (unweighted): ent16 + seg_base instead of ent
  buffer ent16;        // uint16[E' + unit]: delta << win_bits | slot, or a source jump
  buffer seg_base;     // uint32[nunits * 16]: running source before each 512-entry wave segment
  buffer units;        // push_unit[nunits], in (window, source) order
  int64_t nunits = 0;
  buffer acc;          // u64[nacc] fixed-point sums by row; windows stored whole by one item are
                       // overwritten each iteration, the others (win_multi) are cleared by the apply
  int64_t nacc = 0;
  buffer items;        // int64[nitems + 1]: first unit of every item (a window or a share of one)
  buffer queue;        // int64[nitems]: item ids of queue 0, 1, ..., 7
  std::vector<int64_t> qoff;  // queue q = queue[qoff[q], qoff[q + 1])
  int64_t nitems = 0;
  int64_t nwin   = 0;
  buffer tile_ctr;     // uint32 queue heads (128 B apart); zero between iterations
  buffer win_multi;    // uint8[nwin]: 1 = window summed by several items (flushes add), 0 = one item stores it
  // fused apply (pagerank.hip fused_finish): items per window, windows without items
  buffer win_items;       // uint32[nwin]
  buffer win_left;        // uint32[nwin]: win_items between iterations
  buffer empty_wins;      // int64[nempty]
  int64_t nempty = 0, nwin_items = 0;
  // measured-cost queues (pagerank.hip calibrate_queues): the first launch on a schedule
  // records every item's duration, the host then re-deals the items by those costs
  buffer item_ticks;      // uint32[nitems], s_memrealtime ticks
  int calib = 0;          // 0 not yet, 1 recorded (re-deal pending), 2 done or off
  // source bands (pagerank.hip, banded push): every window's entries are split at a
  // source cut into two virtual windows, vw = band * nwin_real + window; the stream
  // and the items are band-major, so the whole grid sweeps the low sources first
  bool bands = false;
  int64_t nwin_real = 0;  // real windows (nwin counts the virtual ones)
  buffer win_pub;         // uint32[nwin_real]: items of the window that published this iteration
  buffer carry;           // uint32[nacc]: 32K windows' carry words (push_args::carry), zero between iterations
  // the last call's iteration count (plain calls: no guess, no personalization) with
  // its alpha and epsilon: the first chunk of the next such call (pagerank.hip)
  int last_iters = 0;
  double last_alpha = -1.0, last_eps = -1.0;
};

// One orientation of the adjacency: majors (rows) -> minors (indices).
constexpr int64_t kIdxPad = 16;  // entries past the end of adjacency_t::indices (vector loads)

struct adjacency_t {
  buffer offsets;  // edge_t[V+1]
  buffer indices;  // vertex_t[E], ascending within each row (+ kIdxPad entries when idx_padded)
  buffer weights;  // weight_t[E] or empty
  bool idx_padded = false;
  // degree-binned schedule (built on first use, see schedule.hpp)
  bool degree_sorted = false;  // majors already in descending-degree order (renumbered build)
  int64_t max_degree = -1;     // cached on first use (BFS), -1 = not known yet
  int unit_weights   = -1;     // weighted: 1 if every weight is exactly 1 (PageRank: unweighted push), -1 unknown
  bool sched_valid   = false;
  buffer order;                         // vertex_t[V] processing order if !degree_sorted
  std::vector<int64_t> bin_begin;       // positions (in processing order) where each bin starts
  buffer items;                         // work items for the SpMV-like kernels
  int64_t num_items = 0;
  // BFS bottom-up probe's head table: 16 B per vertex (16 * kHeadQ, bfs.hip k_bfs_head; RMAT-24 142 MB),
  // built on the first direction-optimising BFS and kept for the adjacency's lifetime like pr and
  // items (freed with the graph; trim_device_cache returns only the allocator's free blocks)
  buffer bfs_head;
  double wsum = -1;  // SSSP: sum of the weights (delta), cached on first use; -1 = not known yet
  // SSSP (sssp.hip): the light (w < delta) and heavy edges as two CSRs, with each part's
  // chunk rows, for one delta
  double sssp_delta = -1;
  int64_t sssp_eL = 0, sssp_eH = 0;
  buffer sssp_offL, sssp_offH, sssp_idxL, sssp_wL, sssp_idxH, sssp_wH, sssp_crowL, sssp_crowH;
  pr_push_t pr;  // PageRank windowed-push schedule (pagerank.hip), built on first use
};

struct graph_t {
  data_type_id_t vertex_type = INT32;
  data_type_id_t edge_type   = INT32;
  data_type_id_t weight_type = FLOAT32;
  bool store_transposed      = false;  // orientation the user asked for (the reference mutates it)
  bool symmetric             = false;
  bool multigraph            = false;
  bool weighted              = false;
  bool renumbered            = false;
  bool multi_gpu             = false;
  int64_t num_vertices       = 0;
  int64_t num_edges          = 0;
  std::shared_ptr<adjacency_t> out;  // CSR (may be null until built)
  std::shared_ptr<adjacency_t> in;   // CSC (== out when symmetric)
  buffer number_map;                 // vertex_t[V]: internal -> external id
  // cached external -> internal lookup (sorted external ids + their internal ids)
  bool ext_lookup_valid = false;
  buffer ext_sorted;    // vertex_t[V]
  buffer ext_internal;  // vertex_t[V]
  // cached per-vertex out-weight sums (weight_t[V]) and their dangling mask source
  bool outw_valid = false;
  buffer outw;
  std::shared_ptr<mg_graph_t> mg;  // multi-GPU partition state (mg_graph.hpp); null for SG
};

struct centrality_result_t {
  std::unique_ptr<device_array_t> vertices;
  std::unique_ptr<device_array_t> values;
};

struct paths_result_t {
  std::unique_ptr<device_array_t> vertices;
  std::unique_ptr<device_array_t> distances;
  std::unique_ptr<device_array_t> predecessors;
};

struct extract_paths_result_t {
  size_t max_path_length = 0;
  std::unique_ptr<device_array_t> paths;  // [destinations x max_path_length], row major
};

struct hits_result_t {
  std::unique_ptr<device_array_t> vertices;
  std::unique_ptr<device_array_t> hubs;
  std::unique_ptr<device_array_t> authorities;
  double hub_score_differences = 0;
  size_t number_of_iterations  = 0;
};

struct clustering_result_t {
  std::unique_ptr<device_array_t> vertices;
  std::unique_ptr<device_array_t> clusters;
  double modularity = 0;
  // dendrogram (reference Dendrogram<vertex_t>, dendrogram.hpp): level i holds the
  // cluster of every level-i vertex this rank owns, in global-id order; its values
  // are level-(i+1) vertex ids (the last level: that level's cluster ids)
  std::vector<std::unique_ptr<device_array_t>> levels;
};

// ------------------------------------------------------------------ helpers
inline handle_t* H(cugraph_resource_handle_t const* h) { return reinterpret_cast<handle_t*>(const_cast<cugraph_resource_handle_t*>(h)); }
inline graph_t* G(cugraph_graph_t* g) { return reinterpret_cast<graph_t*>(g); }
inline graph_t const* G(cugraph_graph_t const* g) { return reinterpret_cast<graph_t const*>(g); }
inline array_view_t const* AV(cugraph_type_erased_device_array_view_t const* v)
{
  return reinterpret_cast<array_view_t const*>(v);
}
inline array_view_t* AV(cugraph_type_erased_device_array_view_t* v) { return reinterpret_cast<array_view_t*>(v); }

inline cugraph_type_erased_device_array_view_t* new_view(device_array_t const* a)
{
  return reinterpret_cast<cugraph_type_erased_device_array_view_t*>(new array_view_t(a->view()));
}

// Run `f` converting every exception into the reference's error protocol
// (cpp/src/c_api/utils.hpp:24-56): cgx::error keeps its code, anything else is
// CUGRAPH_UNKNOWN_ERROR; the message goes into a fresh error object.
template <typename F>
cugraph_error_code_t guarded(cugraph_error_t** error, F&& f)
{
  try {
    f();
    return CUGRAPH_SUCCESS;
  } catch (cgx::error const& e) {
    if (error) *error = reinterpret_cast<cugraph_error_t*>(new err_t{e.what()});
    return e.code;
  } catch (std::bad_alloc const& e) {
    if (error) *error = reinterpret_cast<cugraph_error_t*>(new err_t{std::string("allocation failed: ") + e.what()});
    return CUGRAPH_ALLOC_ERROR;
  } catch (std::exception const& e) {
    if (error) *error = reinterpret_cast<cugraph_error_t*>(new err_t{e.what()});
    return CUGRAPH_UNKNOWN_ERROR;
  }
}

// ------------------------------------------------------------------ shared graph services
// (graph_build.hip)
void build_sg_graph(handle_t& h, graph_t& g, array_view_t const& src, array_view_t const& dst,
                    array_view_t const* weights, bool renumber);
adjacency_t& ensure_adjacency(handle_t& h, graph_t& g, bool transposed);  // builds the other orientation
void ensure_schedule(handle_t& h, graph_t& g, adjacency_t& adj);
// external ids (device, graph vertex type) -> internal ids, in place; throws on unknown ids
void renumber_ext_to_int(handle_t& h, graph_t& g, void* ids, size_t n, bool check);
// the same lookup with no check and no host sync: ids not in the graph become -1,
// for callers that range-check the internal ids on the device anyway (BFS sources)
void renumber_ext_to_int_unchecked(handle_t& h, graph_t& g, void* ids, size_t n);
// sorted external ids + their internal ids (g.ext_sorted / g.ext_internal), renumbered graphs
void ensure_ext_lookup(handle_t& h, graph_t& g);
// internal ids -> external ids (values < 0 or >= V are left untouched), in place
void unrenumber_int_to_ext(handle_t& h, graph_t& g, void* ids, size_t n);
// copy of the number map as a result array
std::unique_ptr<device_array_t> number_map_copy(handle_t& h, graph_t& g);
// per-vertex out-weight sums in weight_t (cached on the graph)
void const* out_weight_sums(handle_t& h, graph_t& g);

}  // namespace cgx
