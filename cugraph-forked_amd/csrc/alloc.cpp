// Stream-ordered caching allocator for HBM (the role RMM's pool resource plays
// under the reference, cpp/include/cugraph/... via rmm::mr::device_memory_resource).
//
// Blocks are rounded to size classes (4 per power of two, <= 25 % slack).  A
// freed block is cached on the stream it was freed on; an allocation on the same
// stream reuses a cached block of its class (or up to twice its class) with no
// driver call and no synchronisation -- stream order already places the new
// user's work after the old user's.  Blocks never move between streams.  When the
// driver is out of memory the device is synchronised, every cached block is
// returned, and the allocation is retried once.
#include "common.hpp"

#include <chrono>
#include <map>
#include <mutex>
#include <unordered_map>

namespace cgx {

namespace {

struct cache_t {
  std::mutex mu;
  std::unordered_map<hipStream_t, std::multimap<size_t, void*>> free_blocks;
  std::unordered_map<void*, size_t> live;  // block -> class size
  size_t cached = 0;
  // statistics (cugraph_amd_allocator_stats): driver allocations, their bytes and
  // seconds, and out-of-memory trims (every cached block returned, then a retry)
  size_t n_malloc = 0, malloc_bytes = 0, n_oom = 0;
  double malloc_s = 0.0;
};

cache_t& cache()
{
  static cache_t* c = new cache_t();  // never destroyed: frees may run during static teardown
  return *c;
}

size_t size_class(size_t b)
{
  if (b <= 512) return 512;
  int const e       = 63 - __builtin_clzll((unsigned long long)(b - 1));  // 2^e < b <= 2^(e+1)
  size_t const step = (size_t)1 << (e >= 2 ? e - 2 : 0);
  return (b + step - 1) / step * step;
}

size_t trim_locked(cache_t& c)
{
  if (c.cached == 0) return 0;
  (void)hipDeviceSynchronize();
  size_t freed = 0;
  for (auto& kv : c.free_blocks)
    for (auto& blk : kv.second) {
      (void)hipFree(blk.second);
      freed += blk.first;
    }
  c.free_blocks.clear();
  c.cached = 0;
  return freed;
}

// CGX_POISON=1 (debugging only): every allocation is filled with 0xff bytes on its
// stream, so a read of memory nobody wrote gives the same garbage on every run
bool poison_enabled()
{
  static bool const on = std::getenv("CGX_POISON") != nullptr;
  return on;
}

void* poisoned(void* p, size_t bytes, hipStream_t s)
{
  if (p && poison_enabled()) (void)hipMemsetAsync(p, 0xff, bytes, s);
  return p;
}

void* device_alloc_raw(size_t bytes, hipStream_t s)
{
  cache_t& c       = cache();
  size_t const cls = size_class(bytes);
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.free_blocks.find(s);
  if (it != c.free_blocks.end()) {
    auto& m = it->second;
    auto b  = m.lower_bound(cls);
    if (b != m.end() && b->first <= 2 * cls) {
      void* p = b->second;
      c.live[p] = b->first;
      c.cached -= b->first;
      m.erase(b);
      return p;
    }
  }
  void* p = nullptr;
  auto const t0 = std::chrono::steady_clock::now();
  if (hipMalloc(&p, cls) != hipSuccess) {
    (void)hipGetLastError();
    ++c.n_oom;
    trim_locked(c);
    if (hipMalloc(&p, cls) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
  }
  c.malloc_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  ++c.n_malloc;
  c.malloc_bytes += cls;
  c.live[p] = cls;
  return p;
}

}  // namespace

void* device_alloc(size_t bytes, hipStream_t s) { return poisoned(device_alloc_raw(bytes, s), size_class(bytes), s); }

void device_free(void* p, hipStream_t s)
{
  if (!p) return;
  cache_t& c = cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.live.find(p);
  if (it == c.live.end()) return;  // not ours
  size_t const cls = it->second;
  c.live.erase(it);
  c.free_blocks[s].emplace(cls, p);
  c.cached += cls;
}

void* device_forget(void* p, hipStream_t s)
{
  if (!p) return nullptr;
  cache_t& c = cache();
  {
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(p);
    if (it == c.live.end()) return nullptr;  // not ours
    c.live.erase(it);
  }
  // pending work on the block's stream finishes before the caller may hipFree it
  if (hipStreamSynchronize(s) != hipSuccess) (void)hipGetLastError();
  return p;
}

void device_alloc_stats(double* out)
{
  cache_t& c = cache();
  std::lock_guard<std::mutex> lk(c.mu);
  out[0] = (double)c.n_malloc;
  out[1] = (double)c.malloc_bytes;
  out[2] = c.malloc_s;
  out[3] = (double)c.n_oom;
  out[4] = (double)c.cached;
}

size_t device_cache_trim()
{
  cache_t& c = cache();
  std::lock_guard<std::mutex> lk(c.mu);
  return trim_locked(c);
}

}  // namespace cgx
