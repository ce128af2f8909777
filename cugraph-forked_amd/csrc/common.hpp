// Core runtime pieces shared by every translation unit of libcugraph_c (MI355X build):
// error type, HIP checks, stream-ordered device buffers, type dispatch.
//
// Replaces the roles RAFT/RMM play for the reference (raft::handle_t streams,
// rmm::device_uvector, CUGRAPH_EXPECTS in cpp/include/cugraph/utilities/error.hpp:22-58).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>

#include <cugraph_c/resource_handle.h>
#include <cugraph_c/error.h>

namespace cgx {

// ---------------------------------------------------------------- errors
struct error : public std::runtime_error {
  cugraph_error_code_t code;
  error(cugraph_error_code_t c, std::string const& msg) : std::runtime_error(msg), code(c) {}
};

[[noreturn]] inline void fail(cugraph_error_code_t code, std::string const& msg) { throw error(code, msg); }

#define CGX_EXPECTS(cond, code, msg)            \
  do {                                          \
    if (!(cond)) ::cgx::fail((code), (msg));    \
  } while (0)

#define CGX_INPUT(cond, msg) CGX_EXPECTS(cond, CUGRAPH_INVALID_INPUT, msg)

#define HIP_CHECK(expr)                                                                        \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) {                                                                    \
      ::cgx::fail(e_ == hipErrorOutOfMemory ? CUGRAPH_ALLOC_ERROR : CUGRAPH_UNKNOWN_ERROR,     \
                  std::string("HIP error ") + hipGetErrorString(e_) + " at " + __FILE__ + ":" + \
                    std::to_string(__LINE__) + " (" #expr ")");                                \
    }                                                                                          \
  } while (0)

// ---------------------------------------------------------------- dtypes
inline size_t dtype_size(data_type_id_t t)
{
  switch (t) {
    case INT32: return 4;
    case INT64: return 8;
    case FLOAT32: return 4;
    case FLOAT64: return 8;
    default: fail(CUGRAPH_INVALID_INPUT, "invalid data type id");
  }
}

template <typename T>
constexpr data_type_id_t dtype_of()
{
  if constexpr (std::is_same_v<T, int32_t>) return INT32;
  else if constexpr (std::is_same_v<T, int64_t>) return INT64;
  else if constexpr (std::is_same_v<T, float>) return FLOAT32;
  else return FLOAT64;
}

// ---------------------------------------------------------------- device buffer
// HBM blocks come from a stream-ordered caching allocator (alloc.cpp): a freed
// block goes back to a per-stream cache and the next allocation of the same size
// class on that stream takes it without a driver call.  (The reference runs on an
// RMM pool for the same reason; hipFreeAsync of multi-GB blocks measured 250 ms
// stalls per Louvain sweep on MI355X, see DESIGN.md.)
void* device_alloc(size_t bytes, hipStream_t s);
void device_free(void* p, hipStream_t s);
size_t device_cache_trim();  // returns the cached bytes released
void device_alloc_stats(double* out);  // [5]: driver allocations, their bytes and seconds, OOM trims, cached bytes
// Hand a live block to the caller: the allocator stops tracking it (it is never
// cached or reused) and the stream is synchronised; the caller frees it with hipFree.
void* device_forget(void* p, hipStream_t s);

// compute units of the current device (persistent grids: resident blocks per CU x
// this), queried once per device
inline int device_cu_count()
{
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0) d = 0;
  static int cache[64] = {};
  if (d < 64 && cache[d] > 0) return cache[d];
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || n <= 0) n = 256;
  if (d < 64) cache[d] = n;
  return n;
}

class buffer {
 public:
  buffer() = default;
  buffer(size_t bytes, hipStream_t s) : stream_(s) { resize(bytes); }
  buffer(buffer const&) = delete;
  buffer& operator=(buffer const&) = delete;
  buffer(buffer&& o) noexcept { swap(o); }
  buffer& operator=(buffer&& o) noexcept
  {
    if (this != &o) {
      release();
      swap(o);
    }
    return *this;
  }
  ~buffer() { release(); }

  void resize(size_t bytes)
  {
    release();
    bytes_ = bytes;
    if (bytes) {
      ptr_ = device_alloc(bytes, stream_);
      if (!ptr_) {
        bytes_ = 0;
        fail(CUGRAPH_ALLOC_ERROR, "device allocation failed (" + std::to_string(bytes) + " bytes)");
      }
    }
  }
  void set_stream(hipStream_t s) { stream_ = s; }
  // Frees are stream-ordered on the allocating stream.  Handle streams come from a
  // process-wide pool and are never destroyed (capi_core.cpp), so a buffer may
  // outlive the handle that allocated it (graphs/results freed after their handle).
  void release()
  {
    if (ptr_) device_free(ptr_, stream_);
    ptr_   = nullptr;
    bytes_ = 0;
  }
  // give up ownership (caller frees with device_free)
  void* detach()
  {
    void* p = ptr_;
    ptr_    = nullptr;
    bytes_  = 0;
    return p;
  }
  template <typename T = void>
  T* data() const
  {
    return static_cast<T*>(ptr_);
  }
  size_t bytes() const { return bytes_; }
  hipStream_t stream() const { return stream_; }
  bool empty() const { return ptr_ == nullptr; }

 private:
  void swap(buffer& o) noexcept
  {
    std::swap(ptr_, o.ptr_);
    std::swap(bytes_, o.bytes_);
    std::swap(stream_, o.stream_);
  }
  void* ptr_          = nullptr;
  size_t bytes_       = 0;
  hipStream_t stream_ = nullptr;
};

template <typename T>
struct dbuf {  // typed view over a buffer
  buffer b;
  size_t n = 0;
  dbuf() = default;
  dbuf(size_t count, hipStream_t s) : b(count * sizeof(T), s), n(count) {}
  T* data() const { return b.data<T>(); }
  size_t size() const { return n; }
  void resize(size_t count, hipStream_t s)
  {
    b.set_stream(s);
    b.resize(count * sizeof(T));
    n = count;
  }
  void free()  // release the block now (stream-ordered), before the dbuf goes out of scope
  {
    b.release();
    n = 0;
  }
};

// ---------------------------------------------------------------- launch helpers
inline unsigned grid_for(size_t n, unsigned block, unsigned max_blocks = 1u << 16)
{
  size_t g = (n + block - 1) / block;
  if (g == 0) g = 1;
  if (g > max_blocks) g = max_blocks;
  return static_cast<unsigned>(g);
}

#define CGX_LAUNCH_CHECK() HIP_CHECK(hipGetLastError())

// ---------------------------------------------------------------- type dispatch
template <typename V, typename E, typename W>
struct types3 {
  using vertex_t = V;
  using edge_t   = E;
  using weight_t = W;
};

// Valid combinations follow cpp/include/cugraph/utilities/graph_traits.hpp:40-57:
// vertex in {i32,i64}, edge in {i32,i64}, sizeof(vertex) <= sizeof(edge), weight in {f32,f64}.
template <typename F>
decltype(auto) dispatch_vew(data_type_id_t v, data_type_id_t e, data_type_id_t w, F&& f)
{
  if (w != FLOAT32 && w != FLOAT64)
    fail(CUGRAPH_UNSUPPORTED_TYPE_COMBINATION, "weight type must be FLOAT32 or FLOAT64");
  if (v == INT32 && e == INT32) {
    if (w == FLOAT32) return f(types3<int32_t, int32_t, float>{});
    return f(types3<int32_t, int32_t, double>{});
  }
  if (v == INT32 && e == INT64) {
    if (w == FLOAT32) return f(types3<int32_t, int64_t, float>{});
    return f(types3<int32_t, int64_t, double>{});
  }
  if (v == INT64 && e == INT64) {
    if (w == FLOAT32) return f(types3<int64_t, int64_t, float>{});
    return f(types3<int64_t, int64_t, double>{});
  }
  fail(CUGRAPH_UNSUPPORTED_TYPE_COMBINATION, "unsupported vertex/edge type combination");
}

}  // namespace cgx
