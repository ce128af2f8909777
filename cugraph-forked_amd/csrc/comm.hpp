// Communicators for the multi-GPU path (include/cugraph_amd/comm.h).
//
// The reference reaches NCCL through raft::comms with 2D row/column
// sub-communicators (cpp/include/cugraph/partition_manager.hpp,
// cpp/tests/utilities/mg_utilities.cpp:52-68).  Here a comm_t is either an RCCL
// communicator (one process per GPU, xGMI) or a table of host callbacks (tests:
// several ranks on one GPU over torch.distributed/gloo).  All collectives are
// stream-ordered on the caller's stream.
#pragma once

#include "common.hpp"

#include <cugraph_amd/comm.h>

#include <memory>
#include <vector>

namespace cgx {

template <typename T>
constexpr int comm_dtype()
{
  if constexpr (std::is_same_v<T, uint8_t> || std::is_same_v<T, int8_t>) return CGX_COMM_U8;
  else if constexpr (std::is_same_v<T, int32_t> || std::is_same_v<T, uint32_t>) return CGX_COMM_I32;
  else if constexpr (std::is_same_v<T, int64_t> || std::is_same_v<T, long long>) return CGX_COMM_I64;
  else if constexpr (std::is_same_v<T, uint64_t> || std::is_same_v<T, unsigned long long>) return CGX_COMM_U64;
  else if constexpr (std::is_same_v<T, float>) return CGX_COMM_F32;
  else return CGX_COMM_F64;
}

size_t comm_dtype_size(int dt);

class comm_t {
 public:
  virtual ~comm_t() = default;
  int rank = 0;
  int size = 1;
  virtual void allreduce(void const* s, void* r, size_t n, int dt, int op, hipStream_t st)                = 0;
  virtual void allgather(void const* s, void* r, size_t n, int dt, hipStream_t st)                        = 0;
  virtual void reduce_scatter(void const* s, void* r, size_t n, int dt, int op, hipStream_t st)           = 0;
  virtual void alltoallv(void const* s, size_t const* sc, size_t const* sd, void* r, size_t const* rc,
                         size_t const* rd, int dt, hipStream_t st)                                          = 0;

  // typed helpers
  template <typename T>
  void allreduce(T const* s, T* r, size_t n, int op, hipStream_t st)
  {
    allreduce((void const*)s, (void*)r, n, comm_dtype<T>(), op, st);
  }
  template <typename T>
  void allgather(T const* s, T* r, size_t n, hipStream_t st)
  {
    allgather((void const*)s, (void*)r, n, comm_dtype<T>(), st);
  }
  template <typename T>
  void reduce_scatter(T const* s, T* r, size_t n, int op, hipStream_t st)
  {
    reduce_scatter((void const*)s, (void*)r, n, comm_dtype<T>(), op, st);
  }
  // host scalar allreduce (one element per call)
  template <typename T>
  T host_allreduce(T v, int op, hipStream_t st);
  // all ranks' values of one host scalar
  template <typename T>
  std::vector<T> host_allgather(T v, hipStream_t st);
};

struct mg_context {
  std::unique_ptr<comm_t> world, row, col;
  int R = 1, C = 1;  // grid rows x columns; rank = r * C + c; row comm = the C ranks of row r (rank c)
  int rank() const { return world->rank; }
  int size() const { return world->size; }
  int r() const { return world->rank / C; }
  int c() const { return world->rank % C; }
};

// Exchange variable-length blocks: `send` holds `counts[q]` elements for rank q in
// rank order; returns the received elements (rank order) and their counts.
template <typename T>
dbuf<T> exchange(comm_t& comm, T const* send, std::vector<size_t> const& counts, std::vector<size_t>& rcounts,
                 hipStream_t st);

// The same with the receive counts already known (a reply to an exchange: its
// send counts are the request's receive counts), so no count exchange is needed.
template <typename T>
dbuf<T> exchange_known(comm_t& comm, T const* send, std::vector<size_t> const& counts,
                       std::vector<size_t> const& rcounts, hipStream_t st);

// recv counts from send counts (every rank's count vector)
std::vector<size_t> exchange_counts(comm_t& comm, std::vector<size_t> const& counts, hipStream_t st);

}  // namespace cgx
