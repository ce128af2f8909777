// Communicator implementations (RCCL, host callbacks) and the context C entry
// points of include/cugraph_amd/comm.h.
#include "comm.hpp"

#include "capi.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>

namespace cgx {

namespace {
template <typename T>
void put_scalar(T* d, T v, hipStream_t st)
{
  HIP_CHECK(hipMemcpyAsync(d, &v, sizeof(T), hipMemcpyHostToDevice, st));
  HIP_CHECK(hipStreamSynchronize(st));
}
}  // namespace

size_t comm_dtype_size(int dt)
{
  switch (dt) {
    case CGX_COMM_U8: return 1;
    case CGX_COMM_I32:
    case CGX_COMM_F32: return 4;
    default: return 8;
  }
}

template <typename T>
T comm_t::host_allreduce(T v, int op, hipStream_t st)
{
  dbuf<T> d(1, st);
  put_scalar(d.data(), v, st);
  allreduce(d.data(), d.data(), 1, op, st);
  T out{};
  HIP_CHECK(hipMemcpyAsync(&out, d.data(), sizeof(T), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  return out;
}

template <typename T>
std::vector<T> comm_t::host_allgather(T v, hipStream_t st)
{
  dbuf<T> d(1, st), all(size, st);
  put_scalar(d.data(), v, st);
  allgather(d.data(), all.data(), 1, st);
  std::vector<T> out(size);
  HIP_CHECK(hipMemcpyAsync(out.data(), all.data(), size * sizeof(T), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  return out;
}

template int64_t comm_t::host_allreduce<int64_t>(int64_t, int, hipStream_t);
template double comm_t::host_allreduce<double>(double, int, hipStream_t);
template std::vector<int64_t> comm_t::host_allgather<int64_t>(int64_t, hipStream_t);

std::vector<size_t> exchange_counts(comm_t& comm, std::vector<size_t> const& counts, hipStream_t st)
{
  int P = comm.size;
  std::vector<int64_t> mine(counts.begin(), counts.end());
  dbuf<int64_t> d(P, st), all((size_t)P * P, st);
  HIP_CHECK(hipMemcpyAsync(d.data(), mine.data(), P * sizeof(int64_t), hipMemcpyHostToDevice, st));
  comm.allgather(d.data(), all.data(), (size_t)P, st);
  std::vector<int64_t> h((size_t)P * P);
  HIP_CHECK(hipMemcpyAsync(h.data(), all.data(), h.size() * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  std::vector<size_t> r(P);
  for (int q = 0; q < P; ++q) r[q] = (size_t)h[(size_t)q * P + comm.rank];
  return r;
}

template <typename T>
dbuf<T> exchange(comm_t& comm, T const* send, std::vector<size_t> const& counts, std::vector<size_t>& rcounts,
                 hipStream_t st)
{
  rcounts = exchange_counts(comm, counts, st);
  return exchange_known<T>(comm, send, counts, rcounts, st);
}

template <typename T>
dbuf<T> exchange_known(comm_t& comm, T const* send, std::vector<size_t> const& counts,
                       std::vector<size_t> const& rcounts, hipStream_t st)
{
  int P = comm.size;
  std::vector<size_t> sd(P), rd(P);
  size_t tot = 0;
  for (int q = 0; q < P; ++q) {
    sd[q] = q ? sd[q - 1] + counts[q - 1] : 0;
    rd[q] = tot;
    tot += rcounts[q];
  }
  dbuf<T> out(std::max<size_t>(tot, 1), st);
  comm.alltoallv((void const*)send, counts.data(), sd.data(), (void*)out.data(), rcounts.data(), rd.data(),
                 comm_dtype<T>(), st);
  out.n = tot;
  return out;
}

#define CGX_EXCHANGE_KNOWN(T)                                                                                \
  template dbuf<T> exchange_known<T>(comm_t&, T const*, std::vector<size_t> const&, std::vector<size_t> const&, \
                                     hipStream_t);
CGX_EXCHANGE_KNOWN(int32_t)
CGX_EXCHANGE_KNOWN(int64_t)
CGX_EXCHANGE_KNOWN(float)
CGX_EXCHANGE_KNOWN(double)
CGX_EXCHANGE_KNOWN(uint32_t)
CGX_EXCHANGE_KNOWN(unsigned long long)
CGX_EXCHANGE_KNOWN(long long)
#undef CGX_EXCHANGE_KNOWN

template dbuf<int32_t> exchange<int32_t>(comm_t&, int32_t const*, std::vector<size_t> const&, std::vector<size_t>&,
                                         hipStream_t);
template dbuf<int64_t> exchange<int64_t>(comm_t&, int64_t const*, std::vector<size_t> const&, std::vector<size_t>&,
                                         hipStream_t);
template dbuf<float> exchange<float>(comm_t&, float const*, std::vector<size_t> const&, std::vector<size_t>&,
                                     hipStream_t);
template dbuf<double> exchange<double>(comm_t&, double const*, std::vector<size_t> const&, std::vector<size_t>&,
                                       hipStream_t);
template dbuf<uint32_t> exchange<uint32_t>(comm_t&, uint32_t const*, std::vector<size_t> const&,
                                           std::vector<size_t>&, hipStream_t);
template dbuf<unsigned long long> exchange<unsigned long long>(comm_t&, unsigned long long const*,
                                                               std::vector<size_t> const&, std::vector<size_t>&,
                                                               hipStream_t);

namespace {

#define NCCL_CHECK(x)                                                                               \
  do {                                                                                              \
    ncclResult_t r_ = (x);                                                                          \
    if (r_ != ncclSuccess) fail(CUGRAPH_UNKNOWN_ERROR, std::string("RCCL: ") + ncclGetErrorString(r_)); \
  } while (0)

ncclDataType_t nccl_dt(int dt)
{
  switch (dt) {
    case CGX_COMM_U8: return ncclUint8;
    case CGX_COMM_I32: return ncclInt32;
    case CGX_COMM_I64: return ncclInt64;
    case CGX_COMM_U64: return ncclUint64;
    case CGX_COMM_F32: return ncclFloat32;
    default: return ncclFloat64;
  }
}
ncclRedOp_t nccl_op(int op) { return op == CGX_COMM_MIN ? ncclMin : op == CGX_COMM_MAX ? ncclMax : ncclSum; }

class rccl_comm final : public comm_t {
 public:
  ncclComm_t comm = nullptr;
  ~rccl_comm() override
  {
    if (comm) (void)ncclCommDestroy(comm);
  }
  void allreduce(void const* s, void* r, size_t n, int dt, int op, hipStream_t st) override
  {
    NCCL_CHECK(ncclAllReduce(s, r, n, nccl_dt(dt), nccl_op(op), comm, st));
  }
  void allgather(void const* s, void* r, size_t n, int dt, hipStream_t st) override
  {
    NCCL_CHECK(ncclAllGather(s, r, n, nccl_dt(dt), comm, st));
  }
  void reduce_scatter(void const* s, void* r, size_t n, int dt, int op, hipStream_t st) override
  {
    NCCL_CHECK(ncclReduceScatter(s, r, n, nccl_dt(dt), nccl_op(op), comm, st));
  }
  void alltoallv(void const* s, size_t const* sc, size_t const* sd, void* r, size_t const* rc, size_t const* rd,
                 int dt, hipStream_t st) override
  {
    size_t const es = comm_dtype_size(dt);
    // this rank's own share is a device copy, not a send to itself; a peer's share
    // goes in pieces of at most kPiece bytes (both sides cut it alike: the sender's
    // count is the receiver's).  Measured on MI355X (RCCL 2.27.7, ROCm 7.2,
    // scripts/ubench/rccl_self.hip, gpurun_out/r05a-b): one ncclSend/ncclRecv pair of a
    // rank to itself is byte-exact up to 2^30 bytes and wrong from 2^30 + 8 on -- the
    // second half of the buffer, whatever the element type (uint8 / int32 / int64
    // counts alike); the same sizes in 2^30-byte pieces inside one group are exact.
    // So kPiece is that limit (peer sends could not be tested: one GPU per box).
    constexpr size_t kPiece = size_t(1) << 30;
    size_t const pe         = kPiece / es;
    if (sc[rank]) {
      CGX_EXPECTS(sc[rank] == rc[rank], CUGRAPH_UNKNOWN_ERROR, "alltoallv: self counts differ");
      HIP_CHECK(hipMemcpyAsync((char*)r + rd[rank] * es, (char const*)s + sd[rank] * es, sc[rank] * es,
                               hipMemcpyDeviceToDevice, st));
    }
    NCCL_CHECK(ncclGroupStart());
    for (int q = 0; q < size; ++q) {
      if (q == rank) continue;
      for (size_t o = 0; o < sc[q]; o += pe)
        NCCL_CHECK(ncclSend((char const*)s + (sd[q] + o) * es, std::min(pe, sc[q] - o), nccl_dt(dt), q, comm, st));
      for (size_t o = 0; o < rc[q]; o += pe)
        NCCL_CHECK(ncclRecv((char*)r + (rd[q] + o) * es, std::min(pe, rc[q] - o), nccl_dt(dt), q, comm, st));
    }
    NCCL_CHECK(ncclGroupEnd());
  }
};

class ops_comm final : public comm_t {
 public:
  cugraph_amd_comm_ops_t ops{};
  explicit ops_comm(cugraph_amd_comm_ops_t const& o) : ops(o)
  {
    rank = o.rank;
    size = o.size;
  }
  static void check(int rc, char const* what)
  {
    if (rc != 0) fail(CUGRAPH_UNKNOWN_ERROR, std::string("communicator callback failed: ") + what);
  }
  void allreduce(void const* s, void* r, size_t n, int dt, int op, hipStream_t st) override
  {
    check(ops.allreduce(ops.ctx, s, r, n, dt, op, (void*)st), "allreduce");
  }
  void allgather(void const* s, void* r, size_t n, int dt, hipStream_t st) override
  {
    check(ops.allgather(ops.ctx, s, r, n, dt, (void*)st), "allgather");
  }
  void reduce_scatter(void const* s, void* r, size_t n, int dt, int op, hipStream_t st) override
  {
    check(ops.reduce_scatter(ops.ctx, s, r, n, dt, op, (void*)st), "reduce_scatter");
  }
  void alltoallv(void const* s, size_t const* sc, size_t const* sd, void* r, size_t const* rc, size_t const* rd,
                 int dt, hipStream_t st) override
  {
    check(ops.alltoallv(ops.ctx, s, sc, sd, r, rc, rd, dt, (void*)st), "alltoallv");
  }
};

void check_grid(int world, int row_size)
{
  CGX_INPUT(world >= 1 && row_size >= 1 && world % row_size == 0,
            "Invalid input argument: row_comm_size must divide the number of ranks");
}

}  // namespace

}  // namespace cgx

using namespace cgx;

extern "C" size_t cugraph_amd_comm_unique_id_size(void) { return sizeof(ncclUniqueId); }

extern "C" cugraph_error_code_t cugraph_amd_comm_get_unique_id(void* unique_id, cugraph_error_t** error)
{
  *error = nullptr;
  return guarded(error, [&] {
    ncclUniqueId id;
    NCCL_CHECK(ncclGetUniqueId(&id));
    std::memcpy(unique_id, &id, sizeof(id));
  });
}

extern "C" cugraph_error_code_t cugraph_amd_mg_context_create_rccl(const void* unique_id, int world_size, int rank,
                                                                   int row_comm_size,
                                                                   cugraph_amd_mg_context_t** context,
                                                                   cugraph_error_t** error)
{
  *context = nullptr;
  *error   = nullptr;
  return guarded(error, [&] {
    check_grid(world_size, row_comm_size);
    auto ctx = std::make_unique<mg_context>();
    ctx->C   = row_comm_size;
    ctx->R   = world_size / row_comm_size;
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    auto w = std::make_unique<rccl_comm>();
    NCCL_CHECK(ncclCommInitRank(&w->comm, world_size, id, rank));
    w->rank = rank;
    w->size = world_size;
    auto r  = std::make_unique<rccl_comm>();
    NCCL_CHECK(ncclCommSplit(w->comm, rank / row_comm_size, rank % row_comm_size, &r->comm, nullptr));
    r->rank = rank % row_comm_size;
    r->size = row_comm_size;
    auto c  = std::make_unique<rccl_comm>();
    NCCL_CHECK(ncclCommSplit(w->comm, rank % row_comm_size, rank / row_comm_size, &c->comm, nullptr));
    c->rank    = rank / row_comm_size;
    c->size    = ctx->R;
    ctx->world = std::move(w);
    ctx->row   = std::move(r);
    ctx->col   = std::move(c);
    *context   = reinterpret_cast<cugraph_amd_mg_context_t*>(ctx.release());
  });
}

extern "C" cugraph_error_code_t cugraph_amd_mg_context_create_ops(const cugraph_amd_comm_ops_t* world,
                                                                  const cugraph_amd_comm_ops_t* row,
                                                                  const cugraph_amd_comm_ops_t* col,
                                                                  int row_comm_size,
                                                                  cugraph_amd_mg_context_t** context,
                                                                  cugraph_error_t** error)
{
  *context = nullptr;
  *error   = nullptr;
  return guarded(error, [&] {
    CGX_INPUT(world && row && col, "Invalid input argument: communicator tables must not be NULL");
    check_grid(world->size, row_comm_size);
    CGX_INPUT(row->size == row_comm_size && col->size == world->size / row_comm_size &&
                row->rank == world->rank % row_comm_size && col->rank == world->rank / row_comm_size,
              "Invalid input argument: row/column communicators do not match the grid");
    auto ctx   = std::make_unique<mg_context>();
    ctx->C     = row_comm_size;
    ctx->R     = world->size / row_comm_size;
    ctx->world = std::make_unique<ops_comm>(*world);
    ctx->row   = std::make_unique<ops_comm>(*row);
    ctx->col   = std::make_unique<ops_comm>(*col);
    *context   = reinterpret_cast<cugraph_amd_mg_context_t*>(ctx.release());
  });
}

extern "C" void cugraph_amd_mg_context_free(cugraph_amd_mg_context_t* context)
{
  delete reinterpret_cast<mg_context*>(context);
}
