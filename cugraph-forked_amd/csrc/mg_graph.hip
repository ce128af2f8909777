// Multi-GPU graph construction and id lookups (see mg_graph.hpp for the layout).
// C entry points: cugraph_mg_graph_create / cugraph_mg_graph_free
// (reference cpp/src/c_api/graph_mg.cpp:138-259).
#include "mg_graph.hpp"

#include "prims.hpp"

#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_select.hpp>

#include <algorithm>
#include <numeric>

namespace cgx {

int mg_graph_t::owner_of_global(int64_t x) const
{
  return (int)(std::upper_bound(voff.begin(), voff.end(), x) - voff.begin()) - 1;
}

namespace {

inline unsigned blocks(int64_t n) { return grid_for(n > 0 ? n : 1, kBlock, 16384); }

template <typename T>
__device__ int64_t lower_bound_dev(T const* a, int64_t n, T x)
{
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

template <typename T>
dbuf<T> sort_unique(T const* in, size_t n, hipStream_t s)
{
  dbuf<T> a(std::max<size_t>(n, 1), s), b(std::max<size_t>(n, 1), s), out(std::max<size_t>(n, 1), s);
  out.n = 0;
  if (!n) return out;
  HIP_CHECK(hipMemcpyAsync(a.data(), in, n * sizeof(T), hipMemcpyDeviceToDevice, s));
  radix_sort_keys<T>(a.data(), b.data(), n, 0, 8 * sizeof(T), s);
  dbuf<size_t> cnt(1, s);
  size_t tmp = 0;
  HIP_CHECK(rocprim::unique(nullptr, tmp, b.data(), out.data(), cnt.data(), n, rocprim::equal_to<T>(), s));
  buffer t(tmp, s);
  HIP_CHECK(rocprim::unique(t.data(), tmp, b.data(), out.data(), cnt.data(), n, rocprim::equal_to<T>(), s));
  out.n = to_host_scalar(cnt.data(), s);
  return out;
}

// runs of a sorted array: unique keys and int64 counts
template <typename T>
void run_lengths(T const* sorted, size_t n, dbuf<T>& keys, dbuf<int64_t>& counts, hipStream_t s)
{
  keys.resize(std::max<size_t>(n, 1), s);
  counts.resize(std::max<size_t>(n, 1), s);
  keys.n = counts.n = 0;
  if (!n) return;
  dbuf<size_t> nr(1, s);
  size_t tmp = 0;
  HIP_CHECK(rocprim::run_length_encode(nullptr, tmp, sorted, n, keys.data(), counts.data(), nr.data(), s));
  buffer t(tmp, s);
  HIP_CHECK(rocprim::run_length_encode(t.data(), tmp, sorted, n, keys.data(), counts.data(), nr.data(), s));
  keys.n = counts.n = to_host_scalar(nr.data(), s);
}

template <typename V>
__global__ void k_owner_ext(V const* x, size_t n, int P, int* dest)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dest[i] = mg_owner_of_ext((int64_t)x[i], P);
}

template <typename V>
__global__ void k_owner_global(V const* x, size_t n, int64_t const* voff, int P, int self, int* dest)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int64_t v = (int64_t)x[i];
    dest[i]   = (v >= 0 && v < voff[P]) ? mg_owner_of_global(v, voff, P) : self;
  }
}

// per-rank counts of a destination-sorted array: two binary searches per rank (a
// per-element atomicAdd onto the P counters serialised at the memory side: 14 ms for
// 2.4M elements on one rank, RMAT-22's predecessor routing in the MG BFS)
__global__ void k_rank_counts(int const* dest_sorted, int64_t n, int P, int64_t* cnt)
{
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < P; q += gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = n;  // first position with dest >= q
    while (lo < hi) {
      int64_t const mid = (lo + hi) >> 1;
      if (dest_sorted[mid] < q) lo = mid + 1;
      else hi = mid;
    }
    int64_t a = lo, b = n;  // first position with dest >= q + 1
    while (a < b) {
      int64_t const mid = (a + b) >> 1;
      if (dest_sorted[mid] < q + 1) a = mid + 1;
      else b = mid;
    }
    cnt[q] = a - lo;
  }
}

template <typename T, typename I>
__global__ void k_gather_by(T const* in, I const* idx, size_t n, T* out)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[idx[i]];
}

template <typename T, typename I>
__global__ void k_scatter_by(T const* in, I const* idx, size_t n, T* out)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[idx[i]] = in[i];
}

// Order positions [0, n) by destination rank; per-rank counts on the host.
struct routing {
  dbuf<int64_t> perm;  // sorted position -> original position
  std::vector<size_t> counts;
};

routing route_by(int const* dest, size_t n, int P, hipStream_t s)
{
  routing rt;
  rt.perm.resize(std::max<size_t>(n, 1), s);
  rt.counts.assign(P, 0);
  if (!n) return rt;
  dbuf<int> d2(n, s);
  dbuf<int64_t> iv(n, s);
  iota<int64_t>(iv.data(), n, 0, s);
  radix_sort_pairs<int, int64_t>(dest, d2.data(), iv.data(), rt.perm.data(), n, 0, bits_for(P), s);
  dbuf<int64_t> cnt(P, s);
  hipLaunchKernelGGL(k_rank_counts, dim3(1), dim3(64), 0, s, d2.data(), (int64_t)n, P, cnt.data());
  CGX_LAUNCH_CHECK();
  auto h = to_host(cnt.data(), P, s);
  for (int q = 0; q < P; ++q) rt.counts[q] = (size_t)h[q];
  return rt;
}

template <typename T>
dbuf<T> permute(T const* in, dbuf<int64_t> const& perm, size_t n, hipStream_t s)
{
  dbuf<T> out(std::max<size_t>(n, 1), s);
  if (n)
    hipLaunchKernelGGL((k_gather_by<T, int64_t>), dim3(blocks(n)), dim3(kBlock), 0, s, in, perm.data(), n, out.data());
  CGX_LAUNCH_CHECK();
  return out;
}

// ---------------------------------------------------------------- build kernels
template <typename V>
__global__ void k_add_degrees(V const* ids, int64_t const* cnt, size_t n, V const* owned, int64_t nown, int64_t* deg)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int64_t pos = lower_bound_dev<V>(owned, nown, ids[i]);
    if (pos < nown && owned[pos] == ids[i]) atomicAdd((unsigned long long*)(deg + pos), (unsigned long long)cnt[i]);
  }
}

template <typename V>
__global__ void k_number(V const* owned, int64_t const* order, int64_t n, int64_t base, V* nmap, V* gid_of_owned)
{
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t o       = order[i];
    nmap[i]         = owned[o];
    gid_of_owned[o] = (V)(base + i);
  }
}

// answer: external id -> global id (or -1)
template <typename V>
__global__ void k_answer_ext(V const* q, size_t n, V const* owned, V const* gid, int64_t nown, V* out)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int64_t pos = lower_bound_dev<V>(owned, nown, q[i]);
    out[i]      = (pos < nown && owned[pos] == q[i]) ? gid[pos] : (V)-1;
  }
}

// answer: global id -> external id (ids outside this rank's range pass through)
template <typename V>
__global__ void k_answer_global(V const* q, size_t n, V const* nmap, int64_t lo, int64_t hi, V* out)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int64_t v = (int64_t)q[i];
    out[i]    = (v >= lo && v < hi) ? nmap[v - lo] : q[i];
  }
}

template <typename V>
__global__ void k_relabel(V* x, size_t n, V const* keys, V const* vals, int64_t nk)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int64_t pos = lower_bound_dev<V>(keys, nk, x[i]);
    x[i]        = vals[pos];
  }
}

template <typename V>
__global__ void k_edge_target(V const* src, V const* dst, size_t n, int64_t const* voff, int P, int C, int* dest)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int ou  = mg_owner_of_global((int64_t)src[i], voff, P);
    int ov  = mg_owner_of_global((int64_t)dst[i], voff, P);
    dest[i] = (ou / C) * C + (ov % C);
  }
}

__global__ void k_count_bad(int64_t const* x, size_t n, int* bad)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (x[i] < 0) atomicAdd(bad, 1);
}

template <typename V>
__global__ void k_count_neg(V const* x, size_t n, int* bad)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (x[i] < 0) atomicAdd(bad, 1);
}

// Route `q` (n keys) to `dest` ranks, have the owner compute `answer(recv, m, out)`,
// return the answers in the original order (into `out`).
template <typename V, typename F>
void route_query(comm_t& comm, V const* q, int const* dest, size_t n, V* out, F&& answer, hipStream_t s)
{
  int P   = comm.size;
  auto rt = route_by(dest, n, P, s);
  auto qs = permute<V>(q, rt.perm, n, s);
  std::vector<size_t> rc, back_rc;
  auto got = exchange<V>(comm, qs.data(), rt.counts, rc, s);
  dbuf<V> ans(std::max<size_t>(got.n, 1), s);
  if (got.n) answer(got.data(), got.n, ans.data());
  auto back = exchange<V>(comm, ans.data(), rc, back_rc, s);
  if (n)
    hipLaunchKernelGGL((k_scatter_by<V, int64_t>), dim3(blocks(n)), dim3(kBlock), 0, s, back.data(), rt.perm.data(), n,
                       out);
  CGX_LAUNCH_CHECK();
}

template <typename V, typename R>
void build_mg_impl(handle_t& h, graph_t& g, array_view_t const& srcv, array_view_t const& dstv,
                   array_view_t const* wv)
{
  hipStream_t s = h.stream;
  mg_context& ctx = *h.mg;
  comm_t& comm    = *ctx.world;
  int const P = comm.size, p = comm.rank;
  size_t const n = srcv.size;
  auto mg        = std::make_shared<mg_graph_t>();
  mg->P = P, mg->p = p, mg->R = ctx.R, mg->C = ctx.C;

  V const* src = srcv.as<V>();
  V const* dst = dstv.as<V>();
  {  // ids must be non-negative (every rank agrees before going on)
    dbuf<int> bad(1, s);
    fill<int>(bad.data(), 1, 0, s);
    if (n) {
      hipLaunchKernelGGL(k_count_neg<V>, dim3(blocks(n)), dim3(kBlock), 0, s, src, n, bad.data());
      hipLaunchKernelGGL(k_count_neg<V>, dim3(blocks(n)), dim3(kBlock), 0, s, dst, n, bad.data());
    }
    CGX_LAUNCH_CHECK();
    int64_t nb = comm.host_allreduce<int64_t>((int64_t)to_host_scalar(bad.data(), s), CGX_COMM_SUM, s);
    CGX_INPUT(nb == 0, "Invalid input argument: vertex ids must be non-negative");
  }

  // 1. local endpoints, 2. to their owners
  dbuf<V> cat(std::max<size_t>(2 * n, 1), s);
  if (n) {
    HIP_CHECK(hipMemcpyAsync(cat.data(), src, n * sizeof(V), hipMemcpyDeviceToDevice, s));
    HIP_CHECK(hipMemcpyAsync(cat.data() + n, dst, n * sizeof(V), hipMemcpyDeviceToDevice, s));
  }
  auto L = sort_unique<V>(cat.data(), 2 * n, s);
  cat    = dbuf<V>();
  size_t nL = L.n;
  dbuf<int> dest(std::max<size_t>(nL, 1), s);
  if (nL) hipLaunchKernelGGL(k_owner_ext<V>, dim3(blocks(nL)), dim3(kBlock), 0, s, L.data(), nL, P, dest.data());
  CGX_LAUNCH_CHECK();
  auto rtL = route_by(dest.data(), nL, P, s);
  auto Lo  = permute<V>(L.data(), rtL.perm, nL, s);
  std::vector<size_t> rcL;
  auto Rr = exchange<V>(comm, Lo.data(), rtL.counts, rcL, s);
  // 3. owned vertex set
  auto O         = sort_unique<V>(Rr.data(), Rr.n, s);
  int64_t const nO = (int64_t)O.n;

  // 4. degrees of the owned vertices (majors: destinations when transposed)
  dbuf<int64_t> deg(std::max<int64_t>(nO, 1), s);
  fill<int64_t>(deg.data(), std::max<int64_t>(nO, 1), 0, s);
  {
    V const* maj = g.store_transposed ? dst : src;
    dbuf<V> ms(std::max<size_t>(n, 1), s), ms2(std::max<size_t>(n, 1), s);
    if (n) {
      HIP_CHECK(hipMemcpyAsync(ms.data(), maj, n * sizeof(V), hipMemcpyDeviceToDevice, s));
      radix_sort_keys<V>(ms.data(), ms2.data(), n, 0, 8 * sizeof(V), s);
    }
    dbuf<V> mu;
    dbuf<int64_t> mc;
    run_lengths<V>(ms2.data(), n, mu, mc, s);
    size_t nm = mu.n;
    dbuf<int> md(std::max<size_t>(nm, 1), s);
    if (nm) hipLaunchKernelGGL(k_owner_ext<V>, dim3(blocks(nm)), dim3(kBlock), 0, s, mu.data(), nm, P, md.data());
    CGX_LAUNCH_CHECK();
    auto rt  = route_by(md.data(), nm, P, s);
    auto mus = permute<V>(mu.data(), rt.perm, nm, s);
    auto mcs = permute<int64_t>(mc.data(), rt.perm, nm, s);
    std::vector<size_t> rc1, rc2;
    auto rid = exchange<V>(comm, mus.data(), rt.counts, rc1, s);
    auto rcn = exchange<int64_t>(comm, mcs.data(), rt.counts, rc2, s);
    if (rid.n)
      hipLaunchKernelGGL(k_add_degrees<V>, dim3(blocks(rid.n)), dim3(kBlock), 0, s, rid.data(), rcn.data(), rid.n,
                         O.data(), nO, deg.data());
    CGX_LAUNCH_CHECK();
  }

  // 5. number the owned vertices: descending degree, ties by ascending external id
  auto counts = comm.host_allgather<int64_t>(nO, s);
  mg->voff.assign(P + 1, 0);
  for (int q = 0; q < P; ++q) mg->voff[q + 1] = mg->voff[q] + counts[q];
  int64_t const V_total = mg->voff[P];
  CGX_EXPECTS(g.vertex_type == INT64 || V_total < (int64_t)INT32_MAX, CUGRAPH_INVALID_INPUT,
              "Invalid input argument: too many vertices for int32 ids");
  g.number_map.set_stream(s);
  g.number_map.resize(std::max<int64_t>(nO, 1) * sizeof(V));
  mg->own_ext_sorted.set_stream(s);
  mg->own_ext_sorted.resize(std::max<int64_t>(nO, 1) * sizeof(V));
  mg->own_gid.set_stream(s);
  mg->own_gid.resize(std::max<int64_t>(nO, 1) * sizeof(V));
  if (nO) {
    dbuf<int64_t> deg2(nO, s), iv(nO, s), order(nO, s);
    iota<int64_t>(iv.data(), nO, 0, s);
    radix_sort_pairs<int64_t, int64_t>(deg.data(), deg2.data(), iv.data(), order.data(), nO, 0, 64, s,
                                       /*descending=*/true);
    hipLaunchKernelGGL(k_number<V>, dim3(blocks(nO)), dim3(kBlock), 0, s, O.data(), order.data(), nO, mg->voff[p],
                       g.number_map.data<V>(), mg->own_gid.data<V>());
    CGX_LAUNCH_CHECK();
    HIP_CHECK(hipMemcpyAsync(mg->own_ext_sorted.data(), O.data(), nO * sizeof(V), hipMemcpyDeviceToDevice, s));
  }

  // 6. answer the endpoint queries, 7. relabel the local edges
  dbuf<V> ans(std::max<size_t>(Rr.n, 1), s);
  if (Rr.n)
    hipLaunchKernelGGL(k_answer_ext<V>, dim3(blocks(Rr.n)), dim3(kBlock), 0, s, Rr.data(), Rr.n,
                       mg->own_ext_sorted.data<V>(), mg->own_gid.data<V>(), nO, ans.data());
  CGX_LAUNCH_CHECK();
  std::vector<size_t> rcb;
  auto gLo = exchange<V>(comm, ans.data(), rcL, rcb, s);  // global ids of Lo, in Lo order
  dbuf<V> Lk(std::max<size_t>(nL, 1), s), Lg(std::max<size_t>(nL, 1), s);
  if (nL) radix_sort_pairs<V, V>(Lo.data(), Lk.data(), gLo.data(), Lg.data(), nL, 0, 8 * sizeof(V), s);
  dbuf<V> s2(std::max<size_t>(n, 1), s), d2(std::max<size_t>(n, 1), s);
  if (n) {
    HIP_CHECK(hipMemcpyAsync(s2.data(), src, n * sizeof(V), hipMemcpyDeviceToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d2.data(), dst, n * sizeof(V), hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_relabel<V>, dim3(blocks(n)), dim3(kBlock), 0, s, s2.data(), n, Lk.data(), Lg.data(),
                       (int64_t)nL);
    hipLaunchKernelGGL(k_relabel<V>, dim3(blocks(n)), dim3(kBlock), 0, s, d2.data(), n, Lk.data(), Lg.data(),
                       (int64_t)nL);
  }
  CGX_LAUNCH_CHECK();

  // 8. edges to their 2D block
  dbuf<int64_t> voff_d(P + 1, s);
  HIP_CHECK(hipMemcpyAsync(voff_d.data(), mg->voff.data(), (P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  dbuf<int> ed(std::max<size_t>(n, 1), s);
  if (n)
    hipLaunchKernelGGL(k_edge_target<V>, dim3(blocks(n)), dim3(kBlock), 0, s, s2.data(), d2.data(), n,
                       voff_d.data(), P, ctx.C, ed.data());
  CGX_LAUNCH_CHECK();
  auto rtE = route_by(ed.data(), n, P, s);
  std::vector<size_t> rce;
  {
    auto ps = permute<V>(s2.data(), rtE.perm, n, s);
    auto rs = exchange<V>(comm, ps.data(), rtE.counts, rce, s);
    mg->ne  = (int64_t)rs.n;
    mg->src = std::move(rs.b);
  }
  {
    auto pd = permute<V>(d2.data(), rtE.perm, n, s);
    auto rd = exchange<V>(comm, pd.data(), rtE.counts, rce, s);
    mg->dst = std::move(rd.b);
  }
  if (wv) {
    auto pw = permute<R>(wv->as<R>(), rtE.perm, n, s);
    auto rw = exchange<R>(comm, pw.data(), rtE.counts, rce, s);
    mg->w   = std::move(rw.b);
  }
  HIP_CHECK(hipStreamSynchronize(s));
  g.num_vertices = V_total;
  g.num_edges    = comm.host_allreduce<int64_t>((int64_t)n, CGX_COMM_SUM, s);
  g.mg           = std::move(mg);
}

}  // namespace

void build_mg_graph(handle_t& h, graph_t& g, array_view_t const& src, array_view_t const& dst,
                    array_view_t const* weights)
{
  dispatch_vew(g.vertex_type, g.edge_type, g.weight_type, [&](auto t) {
    using T = decltype(t);
    build_mg_impl<typename T::vertex_t, typename T::weight_t>(h, g, src, dst, weights);
  });
}

void mg_ext_to_global(handle_t& h, graph_t& g, void* ids, size_t n, bool check)
{
  hipStream_t s = h.stream;
  comm_t& comm  = *h.mg->world;
  mg_graph_t& mg = *g.mg;
  auto run = [&](auto tag) {
    using V = decltype(tag);
    V* x    = static_cast<V*>(ids);
    dbuf<int> dest(std::max<size_t>(n, 1), s);
    if (n) hipLaunchKernelGGL(k_owner_ext<V>, dim3(blocks(n)), dim3(kBlock), 0, s, x, n, mg.P, dest.data());
    CGX_LAUNCH_CHECK();
    int64_t nown = mg.n_own();
    route_query<V>(
      comm, x, dest.data(), n, x,
      [&](V const* q, size_t m, V* out) {
        hipLaunchKernelGGL(k_answer_ext<V>, dim3(blocks(m)), dim3(kBlock), 0, s, q, m, mg.own_ext_sorted.data<V>(),
                           mg.own_gid.data<V>(), nown, out);
        CGX_LAUNCH_CHECK();
      },
      s);
    if (check) {
      dbuf<int> bad(1, s);
      fill<int>(bad.data(), 1, 0, s);
      if (n) hipLaunchKernelGGL(k_count_neg<V>, dim3(blocks(n)), dim3(kBlock), 0, s, x, n, bad.data());
      CGX_LAUNCH_CHECK();
      int64_t nb = comm.host_allreduce<int64_t>((int64_t)to_host_scalar(bad.data(), s), CGX_COMM_SUM, s);
      CGX_INPUT(nb == 0, "Invalid input argument: vertex id not in the graph");
    }
  };
  if (g.vertex_type == INT32) run(int32_t{});
  else run(int64_t{});
}

void mg_global_to_ext(handle_t& h, graph_t& g, void* ids, size_t n)
{
  hipStream_t s = h.stream;
  comm_t& comm  = *h.mg->world;
  mg_graph_t& mg = *g.mg;
  dbuf<int64_t> voff_d(mg.P + 1, s);
  HIP_CHECK(hipMemcpyAsync(voff_d.data(), mg.voff.data(), (mg.P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  auto run = [&](auto tag) {
    using V = decltype(tag);
    V* x    = static_cast<V*>(ids);
    dbuf<int> dest(std::max<size_t>(n, 1), s);
    if (n)
      hipLaunchKernelGGL(k_owner_global<V>, dim3(blocks(n)), dim3(kBlock), 0, s, x, n, voff_d.data(), mg.P, mg.p,
                         dest.data());
    CGX_LAUNCH_CHECK();
    int64_t lo = mg.voff[mg.p], hi = mg.voff[mg.p + 1];
    route_query<V>(
      comm, x, dest.data(), n, x,
      [&](V const* q, size_t m, V* out) {
        hipLaunchKernelGGL(k_answer_global<V>, dim3(blocks(m)), dim3(kBlock), 0, s, q, m, g.number_map.data<V>(), lo,
                           hi, out);
        CGX_LAUNCH_CHECK();
      },
      s);
  };
  if (g.vertex_type == INT32) run(int32_t{});
  else run(int64_t{});
  HIP_CHECK(hipStreamSynchronize(s));
}

namespace {

// rank q's slice of the padded allgather (stride mx) -> its global range
template <typename V>
__global__ void k_compact_slices(V const* gath, int64_t mx, int64_t const* voff, int P, int64_t V_total, V* out)
{
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < V_total; g += (int64_t)gridDim.x * blockDim.x) {
    int const q = mg_owner_of_global(g, voff, P);
    out[g]      = gath[q * mx + (g - voff[q])];
  }
}

template <typename V>
__global__ void k_global_to_ext_rep(V* x, size_t n, V const* nmap, int64_t V_total)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int64_t const v = (int64_t)x[i];
    if (v >= 0 && v < V_total) x[i] = nmap[v];
  }
}

template <typename V>
void ensure_rep_impl(handle_t& h, graph_t& g)
{
  mg_graph_t& mg = *g.mg;
  hipStream_t s  = h.stream;
  comm_t& comm   = *h.mg->world;
  int64_t const Vt = g.num_vertices;
  int64_t mx       = 1;
  for (int q = 0; q < mg.P; ++q) mx = std::max<int64_t>(mx, mg.voff[q + 1] - mg.voff[q]);
  dbuf<V> pad(mx, s), gath(mx * mg.P, s);
  if (mg.n_own())
    HIP_CHECK(hipMemcpyAsync(pad.data(), g.number_map.data(), mg.n_own() * sizeof(V), hipMemcpyDeviceToDevice, s));
  comm.allgather<V>(pad.data(), gath.data(), (size_t)mx, s);
  dbuf<int64_t> voff_d(mg.P + 1, s);
  HIP_CHECK(hipMemcpyAsync(voff_d.data(), mg.voff.data(), (mg.P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  for (buffer* b : {&mg.rep_nmap, &mg.rep_ext_sorted, &mg.rep_gid}) {
    b->set_stream(s);
    b->resize(std::max<int64_t>(Vt, 1) * sizeof(V));
  }
  if (Vt) {
    hipLaunchKernelGGL(k_compact_slices<V>, dim3(blocks(Vt)), dim3(kBlock), 0, s, gath.data(), mx, voff_d.data(),
                       mg.P, Vt, mg.rep_nmap.data<V>());
    CGX_LAUNCH_CHECK();
    dbuf<V> iv(Vt, s);
    iota<V>(iv.data(), Vt, V(0), s);
    radix_sort_pairs<V, V>(mg.rep_nmap.data<V>(), mg.rep_ext_sorted.data<V>(), iv.data(), mg.rep_gid.data<V>(), Vt, 0,
                           8 * sizeof(V), s);
  }
  HIP_CHECK(hipStreamSynchronize(s));
  mg.rep_valid = true;
}

}  // namespace

void mg_ensure_replicated_ids(handle_t& h, graph_t& g)
{
  if (g.mg->rep_valid) return;
  if (g.vertex_type == INT32) ensure_rep_impl<int32_t>(h, g);
  else ensure_rep_impl<int64_t>(h, g);
}

void mg_global_to_ext_local(handle_t& h, graph_t& g, void* ids, size_t n)
{
  mg_ensure_replicated_ids(h, g);
  if (!n) return;
  auto run = [&](auto tag) {
    using V = decltype(tag);
    hipLaunchKernelGGL(k_global_to_ext_rep<V>, dim3(blocks(n)), dim3(kBlock), 0, h.stream, static_cast<V*>(ids), n,
                       g.mg->rep_nmap.data<V>(), g.num_vertices);
    CGX_LAUNCH_CHECK();
  };
  if (g.vertex_type == INT32) run(int32_t{});
  else run(int64_t{});
}

void mg_ext_to_global_local(handle_t& h, graph_t& g, void* ids, size_t n)
{
  mg_ensure_replicated_ids(h, g);
  if (!n) return;
  auto run = [&](auto tag) {
    using V = decltype(tag);
    hipLaunchKernelGGL(k_answer_ext<V>, dim3(blocks(n)), dim3(kBlock), 0, h.stream, static_cast<V const*>(ids), n,
                       g.mg->rep_ext_sorted.data<V>(), g.mg->rep_gid.data<V>(), g.num_vertices, static_cast<V*>(ids));
    CGX_LAUNCH_CHECK();
  };
  if (g.vertex_type == INT32) run(int32_t{});
  else run(int64_t{});
}

}  // namespace cgx

using namespace cgx;

extern "C" cugraph_error_code_t cugraph_mg_graph_create(const cugraph_resource_handle_t* handle,
                                                       const cugraph_graph_properties_t* properties,
                                                       const cugraph_type_erased_device_array_view_t* src,
                                                       const cugraph_type_erased_device_array_view_t* dst,
                                                       const cugraph_type_erased_device_array_view_t* weights,
                                                       const cugraph_type_erased_device_array_view_t* edge_ids,
                                                       const cugraph_type_erased_device_array_view_t* edge_types,
                                                       bool_t store_transposed,
                                                       size_t /*num_edges*/,
                                                       bool_t /*check*/,
                                                       cugraph_graph_t** graph,
                                                       cugraph_error_t** error)
{
  *graph = nullptr;
  *error = nullptr;
  return guarded(error, [&] {
    CGX_EXPECTS(handle != nullptr, CUGRAPH_INVALID_HANDLE, "invalid resource handle");
    handle_t& h = *H(handle);
    CGX_INPUT(h.mg != nullptr, "Invalid input argument: the resource handle has no multi-GPU communicator");
    CGX_INPUT(src && dst && properties, "Invalid input argument: src, dst and properties must be given");
    CGX_EXPECTS(edge_ids == nullptr && edge_types == nullptr, CUGRAPH_NOT_IMPLEMENTED,
                "edge ids / edge types are not supported by this build");
    auto const* s = AV(src);
    auto const* d = AV(dst);
    // graph_mg.cpp:239-259 type checks
    CGX_INPUT(s->type == d->type, "Invalid input argument: vertex type mismatch between src and dst");
    CGX_INPUT(s->size == d->size, "Invalid input argument: src and dst sizes differ");
    CGX_EXPECTS(s->type == INT32 || s->type == INT64, CUGRAPH_UNSUPPORTED_TYPE_COMBINATION,
                "Unsupported vertex type");
    auto const* w = weights ? AV(weights) : nullptr;
    if (w) {
      CGX_INPUT(w->size == s->size, "Invalid input argument: weights size differs from src");
      CGX_EXPECTS(w->type == FLOAT32 || w->type == FLOAT64, CUGRAPH_UNSUPPORTED_TYPE_COMBINATION,
                  "Unsupported weight type");
    }
    auto g              = std::make_unique<graph_t>();
    g->vertex_type      = s->type;
    g->weight_type      = w ? w->type : FLOAT32;
    g->store_transposed = store_transposed == TRUE;
    g->symmetric        = properties->is_symmetric == TRUE;
    g->multigraph       = properties->is_multigraph == TRUE;
    g->weighted         = w != nullptr;
    g->renumbered       = true;
    g->multi_gpu        = true;
    // edge_t: int64 when the global edge count may reach INT32_MAX (graph_sg.cpp:246 rule)
    int64_t ne_total = h.mg->world->host_allreduce<int64_t>((int64_t)s->size, CGX_COMM_SUM, h.stream);
    g->edge_type     = (ne_total >= (int64_t)INT32_MAX || s->type == INT64) ? INT64 : INT32;
    build_mg_graph(h, *g, *s, *d, w);
    *graph = reinterpret_cast<cugraph_graph_t*>(g.release());
  });
}

extern "C" void cugraph_mg_graph_free(cugraph_graph_t* graph) { delete G(graph); }
