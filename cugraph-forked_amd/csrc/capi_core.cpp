// libcugraph_c core entry points: resource handle, errors, type-erased arrays,
// SG graph create/free (MI355X build).
//
// Semantics follow the reference implementation files
//   cpp/src/c_api/resource_handle.cpp, error.cpp, array.cpp, graph_sg.cpp:231-330
// (argument checks, error codes, ownership); the storage behind them is our own.
#include "capi.hpp"
#include "comm.hpp"

#include <cugraph_amd/ext.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

using namespace cgx;

namespace {

// Process-wide pool of handle streams.  A stream is never destroyed: memory
// cached on it by the caching allocator (alloc.cpp) may be freed after the
// handle that owned it is gone.
std::mutex g_stream_mutex;
std::vector<std::pair<int, hipStream_t>> g_free_streams;

void release_stream(int device, hipStream_t s)
{
  std::lock_guard<std::mutex> lk(g_stream_mutex);
  g_free_streams.emplace_back(device, s);
}

hipStream_t make_stream(int& device)
{
  HIP_CHECK(hipGetDevice(&device));
  {
    std::lock_guard<std::mutex> lk(g_stream_mutex);
    for (size_t i = 0; i < g_free_streams.size(); ++i) {
      if (g_free_streams[i].first == device) {
        hipStream_t s = g_free_streams[i].second;
        g_free_streams.erase(g_free_streams.begin() + i);
        return s;
      }
    }
  }
  // keep freed blocks cached in the device pool (stream-ordered allocator)
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
    uint64_t threshold = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &threshold);
  }
  hipStream_t s;
  // a blocking stream: orders after work on the legacy null stream (e.g. torch's default)
  HIP_CHECK(hipStreamCreate(&s));
  return s;
}

void set_err(cugraph_error_t** error, char const* msg)
{
  if (error) *error = reinterpret_cast<cugraph_error_t*>(new err_t{msg});
}

}  // namespace


// ============================================================== resource handle
extern "C" cugraph_resource_handle_t* cugraph_create_resource_handle(void* raft_handle)
{
  try {
    auto* h   = new handle_t{};
    h->stream = make_stream(h->device);
    h->mg     = static_cast<mg_context*>(raft_handle);  // cugraph_amd_mg_context_t (comm.h) or NULL
    return reinterpret_cast<cugraph_resource_handle_t*>(h);
  } catch (...) {
    return nullptr;
  }
}

extern "C" int cugraph_resource_handle_get_rank(const cugraph_resource_handle_t* handle)
{
  auto* h = H(handle);
  return (h && h->mg) ? h->mg->rank() : 0;
}

extern "C" void cugraph_free_resource_handle(cugraph_resource_handle_t* handle)
{
  auto* h = H(handle);
  if (!h) return;
  (void)hipStreamSynchronize(h->stream);
  release_stream(h->device, h->stream);
  delete h;
}

// ============================================================== errors
extern "C" const char* cugraph_error_message(const cugraph_error_t* error)
{
  return error ? reinterpret_cast<err_t const*>(error)->message.c_str() : nullptr;
}

extern "C" void cugraph_error_free(cugraph_error_t* error) { delete reinterpret_cast<err_t*>(error); }

// ============================================================== device arrays
extern "C" cugraph_error_code_t cugraph_type_erased_device_array_create(const cugraph_resource_handle_t* handle,
                                                                       size_t n_elems,
                                                                       data_type_id_t dtype,
                                                                       cugraph_type_erased_device_array_t** array,
                                                                       cugraph_error_t** error)
{
  *array = nullptr;
  *error = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    CGX_INPUT(dtype >= INT32 && dtype < NTYPES, "Invalid input argument: invalid data type.");
    auto* a = new device_array_t(n_elems, dtype, H(handle)->stream);
    HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    *array = reinterpret_cast<cugraph_type_erased_device_array_t*>(a);
  });
}

extern "C" cugraph_error_code_t cugraph_type_erased_device_array_create_from_view(
  const cugraph_resource_handle_t* handle,
  const cugraph_type_erased_device_array_view_t* view,
  cugraph_type_erased_device_array_t** array,
  cugraph_error_t** error)
{
  *array = nullptr;
  *error = nullptr;
  return guarded(error, [&] {
    auto const* v = AV(view);
    auto* a       = new device_array_t(v->size, v->type, H(handle)->stream);
    if (v->num_bytes)
      HIP_CHECK(hipMemcpyAsync(a->buf.data(), v->data, v->num_bytes, hipMemcpyDefault, H(handle)->stream));
    HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    *array = reinterpret_cast<cugraph_type_erased_device_array_t*>(a);
  });
}

extern "C" void cugraph_type_erased_device_array_free(cugraph_type_erased_device_array_t* p)
{
  auto* a = reinterpret_cast<device_array_t*>(p);
  if (!a) return;
  delete a;  // freed on the null stream (common.hpp buffer::release)
}

// reference array.h:95 (declared under `#if 0` there, array.cpp:111-122: RMM buffers
// cannot give up their memory).  Blocks of the caching allocator can: the block
// leaves the allocator's books (never cached, never reused), its stream is
// synchronised, and the caller owns the pointer and frees it with hipFree.
extern "C" void* cugraph_type_erased_device_array_release(cugraph_type_erased_device_array_t* p)
{
  auto* a = reinterpret_cast<device_array_t*>(p);
  if (!a) return nullptr;
  hipStream_t const s = a->buf.stream();
  void* raw           = a->buf.detach();
  delete a;
  return raw ? cgx::device_forget(raw, s) : nullptr;
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_type_erased_device_array_view(
  cugraph_type_erased_device_array_t* array)
{
  return new_view(reinterpret_cast<device_array_t*>(array));
}

extern "C" cugraph_error_code_t cugraph_type_erased_device_array_view_as_type(
  cugraph_type_erased_device_array_t* array,
  data_type_id_t dtype,
  cugraph_type_erased_device_array_view_t** result_view,
  cugraph_error_t** error)
{
  *result_view = nullptr;
  *error       = nullptr;
  auto* a      = reinterpret_cast<device_array_t*>(array);
  if (dtype_size(dtype) != dtype_size(a->type)) {
    set_err(error, "Invalid input argument: dtype size mismatch");
    return CUGRAPH_INVALID_INPUT;
  }
  *result_view = reinterpret_cast<cugraph_type_erased_device_array_view_t*>(
    new array_view_t{a->buf.data(), a->size, a->size * dtype_size(dtype), dtype});
  return CUGRAPH_SUCCESS;
}

extern "C" cugraph_type_erased_device_array_view_t* cugraph_type_erased_device_array_view_create(void* pointer,
                                                                                                 size_t n_elems,
                                                                                                 data_type_id_t dtype)
{
  return reinterpret_cast<cugraph_type_erased_device_array_view_t*>(
    new array_view_t{pointer, n_elems, n_elems * dtype_size(dtype), dtype});
}

extern "C" void cugraph_type_erased_device_array_view_free(cugraph_type_erased_device_array_view_t* p)
{
  delete AV(p);
}

extern "C" size_t cugraph_type_erased_device_array_view_size(const cugraph_type_erased_device_array_view_t* p)
{
  return AV(p)->size;
}

extern "C" data_type_id_t cugraph_type_erased_device_array_view_type(const cugraph_type_erased_device_array_view_t* p)
{
  return AV(p)->type;
}

extern "C" const void* cugraph_type_erased_device_array_view_pointer(const cugraph_type_erased_device_array_view_t* p)
{
  return AV(p)->data;
}

extern "C" cugraph_error_code_t cugraph_type_erased_device_array_view_copy_from_host(
  const cugraph_resource_handle_t* handle,
  cugraph_type_erased_device_array_view_t* dst,
  const byte_t* h_src,
  cugraph_error_t** error)
{
  *error = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    auto* d = AV(dst);
    if (d->num_bytes) {
      HIP_CHECK(hipMemcpyAsync(d->data, h_src, d->num_bytes, hipMemcpyHostToDevice, H(handle)->stream));
      HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    }
  });
}

extern "C" cugraph_error_code_t cugraph_type_erased_device_array_view_copy_to_host(
  const cugraph_resource_handle_t* handle,
  byte_t* h_dst,
  const cugraph_type_erased_device_array_view_t* src,
  cugraph_error_t** error)
{
  *error = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    auto const* v = AV(src);
    if (v->num_bytes) {
      HIP_CHECK(hipMemcpyAsync(h_dst, v->data, v->num_bytes, hipMemcpyDeviceToHost, H(handle)->stream));
      HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    }
  });
}

extern "C" cugraph_error_code_t cugraph_type_erased_device_array_view_copy(
  const cugraph_resource_handle_t* handle,
  cugraph_type_erased_device_array_view_t* dst,
  const cugraph_type_erased_device_array_view_t* src,
  cugraph_error_t** error)
{
  *error = nullptr;
  return guarded(error, [&] {
    auto* d       = AV(dst);
    auto const* v = AV(src);
    CGX_INPUT(d->type == v->type, "Invalid input argument: type mismatch");
    CGX_INPUT(d->size == v->size, "Invalid input argument: size mismatch");
    if (v->num_bytes) {
      HIP_CHECK(hipMemcpyAsync(d->data, v->data, v->num_bytes, hipMemcpyDefault, H(handle)->stream));
      HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
    }
  });
}

// ============================================================== host arrays
extern "C" cugraph_error_code_t cugraph_type_erased_host_array_create(const cugraph_resource_handle_t*,
                                                                     size_t n_elems,
                                                                     data_type_id_t dtype,
                                                                     cugraph_type_erased_host_array_t** array,
                                                                     cugraph_error_t** error)
{
  *array = nullptr;
  *error = nullptr;
  return guarded(error, [&] {
    auto* a = new host_array_t{};
    a->data.resize(n_elems * dtype_size(dtype));
    a->size = n_elems;
    a->type = dtype;
    *array  = reinterpret_cast<cugraph_type_erased_host_array_t*>(a);
  });
}

extern "C" void cugraph_type_erased_host_array_free(cugraph_type_erased_host_array_t* p)
{
  delete reinterpret_cast<host_array_t*>(p);
}

// reference array.h:212 (also `#if 0` there, array.cpp:210-217).  The bytes move to
// a malloc'd block the caller frees with free(); an empty array gives NULL.
extern "C" void* cugraph_type_erased_host_array_release(cugraph_type_erased_host_array_t* p)
{
  auto* a = reinterpret_cast<host_array_t*>(p);
  if (!a) return nullptr;
  void* raw = nullptr;
  if (!a->data.empty()) {
    raw = std::malloc(a->data.size());
    if (raw) std::memcpy(raw, a->data.data(), a->data.size());
  }
  delete a;
  return raw;
}

extern "C" cugraph_type_erased_host_array_view_t* cugraph_type_erased_host_array_view(
  cugraph_type_erased_host_array_t* array)
{
  auto* a = reinterpret_cast<host_array_t*>(array);
  return reinterpret_cast<cugraph_type_erased_host_array_view_t*>(
    new array_view_t{a->data.data(), a->size, a->data.size(), a->type});
}

extern "C" cugraph_type_erased_host_array_view_t* cugraph_type_erased_host_array_view_create(void* pointer,
                                                                                             size_t n_elems,
                                                                                             data_type_id_t dtype)
{
  return reinterpret_cast<cugraph_type_erased_host_array_view_t*>(
    new array_view_t{pointer, n_elems, n_elems * dtype_size(dtype), dtype});
}

extern "C" void cugraph_type_erased_host_array_view_free(cugraph_type_erased_host_array_view_t* p)
{
  delete reinterpret_cast<array_view_t*>(p);
}

extern "C" size_t cugraph_type_erased_host_array_size(const cugraph_type_erased_host_array_view_t* p)
{
  return reinterpret_cast<array_view_t const*>(p)->size;
}

extern "C" data_type_id_t cugraph_type_erased_host_array_type(const cugraph_type_erased_host_array_view_t* p)
{
  return reinterpret_cast<array_view_t const*>(p)->type;
}

extern "C" void* cugraph_type_erased_host_array_pointer(const cugraph_type_erased_host_array_view_t* p)
{
  return reinterpret_cast<array_view_t const*>(p)->data;
}

extern "C" cugraph_error_code_t cugraph_type_erased_host_array_view_copy(const cugraph_resource_handle_t*,
                                                                        cugraph_type_erased_host_array_view_t* dst,
                                                                        const cugraph_type_erased_host_array_view_t* src,
                                                                        cugraph_error_t** error)
{
  *error  = nullptr;
  auto* d = reinterpret_cast<array_view_t*>(dst);
  auto* v = reinterpret_cast<array_view_t const*>(src);
  if (d->type != v->type || d->size != v->size) {
    set_err(error, "Invalid input argument: host array type/size mismatch");
    return CUGRAPH_INVALID_INPUT;
  }
  if (v->num_bytes) std::memcpy(d->data, v->data, v->num_bytes);
  return CUGRAPH_SUCCESS;
}

// ============================================================== graphs
extern "C" cugraph_error_code_t cugraph_sg_graph_create(const cugraph_resource_handle_t* handle,
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
                                                       cugraph_error_t** error)
{
  *graph = nullptr;
  *error = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    auto const* ps = AV(src);
    auto const* pd = AV(dst);
    auto const* pw = weights ? AV(weights) : nullptr;
    // argument checks of c_api/graph_sg.cpp:257-300
    CGX_INPUT(ps->size == pd->size, "Invalid input arguments: src size != dst size.");
    CGX_INPUT(ps->type == pd->type, "Invalid input arguments: src type != dst type.");
    CGX_INPUT(!pw || pw->size == ps->size, "Invalid input arguments: src size != weights size.");
    CGX_INPUT((edge_ids == nullptr) == (edge_types == nullptr),
              "Invalid input arguments: either none or both of edge ids and edge types must be provided.");
    CGX_EXPECTS(edge_ids == nullptr, CUGRAPH_NOT_IMPLEMENTED, "edge ids / edge types are not supported by this build");
    CGX_EXPECTS(ps->type == INT32 || ps->type == INT64, CUGRAPH_UNSUPPORTED_TYPE_COMBINATION,
                "vertex type must be INT32 or INT64");
    auto g              = std::make_unique<graph_t>();
    g->vertex_type      = ps->type;
    g->edge_type        = ps->size < (size_t)INT32_MAX ? ps->type : INT64;  // graph_sg.cpp:276-283
    g->weight_type      = pw ? pw->type : FLOAT32;
    g->weighted         = pw != nullptr;
    g->store_transposed = store_transposed == TRUE;
    g->symmetric        = properties ? properties->is_symmetric == TRUE : false;
    g->multigraph       = properties ? properties->is_multigraph == TRUE : false;
    build_sg_graph(*H(handle), *g, *ps, *pd, pw, renumber == TRUE);
    // check: the reference forwards it to create_graph_from_edgelist
    // (graph_sg.cpp:161-162), whose expensive_check_edgelist tests only a vertex list
    // (create_graph_from_edgelist_impl.cuh:71-84, :169-190) -- and the SG C API passes
    // none (graph_sg.cpp:155: std::nullopt), so on this path it checks nothing there
    // either; the size and type checks above run regardless
    (void)check;
    *graph = reinterpret_cast<cugraph_graph_t*>(g.release());
  });
}

extern "C" void cugraph_sg_graph_free(cugraph_graph_t* graph)
{
  auto* g = G(graph);
  if (!g) return;
  (void)hipDeviceSynchronize();
  delete g;
}

// ============================================================== extensions: introspection
extern "C" int64_t cugraph_amd_graph_get_number_of_vertices(const cugraph_graph_t* graph)
{
  return G(graph)->num_vertices;
}
extern "C" int64_t cugraph_amd_graph_get_number_of_edges(const cugraph_graph_t* graph) { return G(graph)->num_edges; }
extern "C" bool_t cugraph_amd_graph_is_symmetric(const cugraph_graph_t* graph)
{
  return G(graph)->symmetric ? TRUE : FALSE;
}

extern "C" cugraph_error_code_t cugraph_amd_device_array_views_copy(
  const cugraph_resource_handle_t* handle,
  size_t n,
  cugraph_type_erased_device_array_view_t* const* dst,
  const cugraph_type_erased_device_array_view_t* const* src,
  cugraph_error_t** error)
{
  *error = nullptr;
  return guarded(error, [&] {
    for (size_t i = 0; i < n; ++i) {
      auto* d       = AV(dst[i]);
      auto const* v = AV(src[i]);
      CGX_INPUT(d->type == v->type, "Invalid input argument: type mismatch");
      CGX_INPUT(d->size == v->size, "Invalid input argument: size mismatch");
    }
    for (size_t i = 0; i < n; ++i) {
      auto* d       = AV(dst[i]);
      auto const* v = AV(src[i]);
      if (v->num_bytes) HIP_CHECK(hipMemcpyAsync(d->data, v->data, v->num_bytes, hipMemcpyDefault, H(handle)->stream));
    }
    HIP_CHECK(hipStreamSynchronize(H(handle)->stream));
  });
}

extern "C" cugraph_error_code_t cugraph_amd_graph_get_adjacency(const cugraph_resource_handle_t* handle,
                                                               cugraph_graph_t* graph,
                                                               bool_t transposed,
                                                               cugraph_type_erased_device_array_t** offsets,
                                                               cugraph_type_erased_device_array_t** indices,
                                                               cugraph_type_erased_device_array_t** weights,
                                                               cugraph_error_t** error)
{
  *error = nullptr;
  return guarded(error, [&] {
    auto& h          = *H(handle);
    auto& g          = *G(graph);
    CGX_EXPECTS(!g.multi_gpu, CUGRAPH_NOT_IMPLEMENTED, "adjacency export is single-GPU only");
    adjacency_t& adj = ensure_adjacency(h, g, transposed == TRUE);
    size_t nv = (size_t)g.num_vertices, ne = (size_t)g.num_edges;
    auto o = new device_array_t(nv + 1, g.edge_type, h.stream);
    auto i = new device_array_t(ne, g.vertex_type, h.stream);
    HIP_CHECK(hipMemcpyAsync(o->buf.data(), adj.offsets.data(), (nv + 1) * dtype_size(g.edge_type),
                             hipMemcpyDeviceToDevice, h.stream));
    if (ne)
      HIP_CHECK(hipMemcpyAsync(i->buf.data(), adj.indices.data(), ne * dtype_size(g.vertex_type),
                               hipMemcpyDeviceToDevice, h.stream));
    *offsets = reinterpret_cast<cugraph_type_erased_device_array_t*>(o);
    *indices = reinterpret_cast<cugraph_type_erased_device_array_t*>(i);
    if (weights) {
      *weights = nullptr;
      if (g.weighted) {
        auto w = new device_array_t(ne, g.weight_type, h.stream);
        if (ne)
          HIP_CHECK(hipMemcpyAsync(w->buf.data(), adj.weights.data(), ne * dtype_size(g.weight_type),
                                   hipMemcpyDeviceToDevice, h.stream));
        *weights = reinterpret_cast<cugraph_type_erased_device_array_t*>(w);
      }
    }
    HIP_CHECK(hipStreamSynchronize(h.stream));
  });
}

extern "C" cugraph_error_code_t cugraph_amd_graph_get_out_weight_sums(const cugraph_resource_handle_t* handle,
                                                                     cugraph_graph_t* graph,
                                                                     cugraph_type_erased_device_array_t** sums,
                                                                     cugraph_error_t** error)
{
  *error = nullptr;
  *sums  = nullptr;
  return guarded(error, [&] {
    auto& h = *H(handle);
    auto& g = *G(graph);
    CGX_EXPECTS(!g.multi_gpu, CUGRAPH_NOT_IMPLEMENTED, "out-weight sums export is single-GPU only");
    size_t const nv = (size_t)g.num_vertices;
    void const* src = nv ? out_weight_sums(h, g) : nullptr;
    auto a          = new device_array_t(nv, g.weight_type, h.stream);
    if (nv)
      HIP_CHECK(hipMemcpyAsync(a->buf.data(), src, nv * dtype_size(g.weight_type), hipMemcpyDeviceToDevice, h.stream));
    HIP_CHECK(hipStreamSynchronize(h.stream));
    *sums = reinterpret_cast<cugraph_type_erased_device_array_t*>(a);
  });
}

// ============================================================== extensions: measurement
extern "C" void cugraph_amd_set_profiling(cugraph_resource_handle_t* handle, bool_t enable)
{
  H(handle)->profiling = enable == TRUE;
}

// measurement / A-B switches (tuning_t, capi.hpp): name -> field
extern "C" cugraph_error_code_t cugraph_amd_set_option(cugraph_resource_handle_t* handle, const char* name,
                                                       double value, cugraph_error_t** error)
{
  *error = nullptr;
  return guarded(error, [&] {
    CGX_INPUT(handle && name, "Invalid input argument: handle and name must not be NULL");
    tuning_t& t = H(handle)->tune;
    std::string const n(name);
    auto b   = [&](bool& f) { f = value != 0.0; };
    auto i32 = [&](int& f) { f = (int)value; };
    if (n == "pr_win_bits") {
      CGX_INPUT(value == 0 || value == 12 || value == 13 || value == 14 || value == 15,
                "Invalid input argument: pr_win_bits must be 0, 12, 13, 14 or 15");
      i32(t.pr_win_bits);
    } else if (n == "pr_packed") b(t.pr_packed);
    else if (n == "pr_whole") b(t.pr_whole);
    else if (n == "pr_calib") b(t.pr_calib);
    else if (n == "pr_deal_global") b(t.pr_deal_global);
    else if (n == "pr_unit_w") b(t.pr_unit_w);
    else if (n == "pr_fuse") b(t.pr_fuse);
    else if (n == "pr_enc") b(t.pr_enc);
    else if (n == "pr_hub") b(t.pr_hub);
    else if (n == "pr_band_cut") t.pr_band_cut = (int64_t)value;
    else if (n == "pr_fast_build") b(t.pr_fast_build);
    else if (n == "pr_share_div") i32(t.pr_share_div);
    else if (n == "mg_chunks") i32(t.mg_chunks);
    else if (n == "sssp_pull") i32(t.sssp_pull);
    else if (n == "sssp_delta") {
      CGX_INPUT(value >= 0, "Invalid input argument: sssp_delta must be >= 0");
      t.sssp_delta = value;
    }
    else if (n == "bfs_alpha") t.bfs_alpha = value;
    else if (n == "bfs_beta") t.bfs_beta = value;
    else if (n == "mg_bfs_alpha") t.mg_bfs_alpha = value;
    else if (n == "mg_bfs_beta") t.mg_bfs_beta = value;
    else if (n == "mg_bfs_pipelined") i32(t.mg_bfs_pipelined);
    else if (n == "bfs_probe_vec") b(t.bfs_probe_vec);
    else if (n == "bfs_head") b(t.bfs_head);
    else if (n == "bfs_res_grid") i32(t.bfs_res_grid);
    else if (n == "bfs_probe_grid") i32(t.bfs_probe_grid);
    else if (n == "bfs_td_cap") t.bfs_td_cap = (int64_t)value;
    else if (n == "louvain_hash") b(t.louvain_hash);
    else if (n == "louvain_big_hash") b(t.louvain_big_hash);
    else if (n == "louvain_big_cap") i32(t.louvain_big_cap);
    else if (n == "louvain_big_maxdeg") t.louvain_big_maxdeg = (int64_t)value;
    else if (n == "louvain_wide_keys") b(t.louvain_wide_keys);
    else if (n == "defaults") t = tuning_t{};
    else fail(CUGRAPH_INVALID_INPUT, "Invalid input argument: unknown option " + n);
  });
}
extern "C" size_t cugraph_amd_last_iterations(const cugraph_resource_handle_t* handle)
{
  return H(handle)->last_iterations;
}
extern "C" double cugraph_amd_last_hot_kernel_ms(const cugraph_resource_handle_t* handle)
{
  return H(handle)->last_hot_ms;
}
extern "C" size_t cugraph_amd_last_hot_kernel_launches(const cugraph_resource_handle_t* handle)
{
  return H(handle)->last_hot_launches;
}
extern "C" size_t cugraph_amd_last_bfs_levels(const cugraph_resource_handle_t* handle)
{
  return H(handle)->last_bfs_levels;
}
extern "C" size_t cugraph_amd_last_bfs_bottom_up_steps(const cugraph_resource_handle_t* handle)
{
  return H(handle)->last_bfs_bottom_up;
}
extern "C" size_t cugraph_amd_last_louvain_levels(const cugraph_resource_handle_t* handle)
{
  return H(handle)->last_louvain_levels;
}
extern "C" double cugraph_amd_last_louvain_sweep_bytes(const cugraph_resource_handle_t* handle)
{
  return H(handle)->last_louvain_sweep_bytes;
}
extern "C" void cugraph_amd_last_louvain_partition(const cugraph_resource_handle_t* handle, int64_t* local_edges,
                                                   int64_t* ghosts)
{
  *local_edges = H(handle)->last_louvain_local_edges;
  *ghosts      = H(handle)->last_louvain_ghosts;
}
extern "C" size_t cugraph_amd_trim_device_cache(void) { return cgx::device_cache_trim(); }
extern "C" void cugraph_amd_allocator_stats(double* out) { cgx::device_alloc_stats(out); }
extern "C" const char* cugraph_amd_version(void) { return "cugraph-forked_amd libcugraph_c gfx950 " __DATE__; }
