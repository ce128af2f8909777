/*
 * Multi-GPU communicator context for the libcugraph_c MG entry points.
 *
 * The reference passes a raft::handle_t (NCCL comms + the 2D row/column
 * sub-communicators built by raft::comms / cugraph::partition_2d, see
 * cpp/tests/utilities/mg_utilities.cpp:52-68) as the `void* raft_handle` of
 * cugraph_create_resource_handle (cugraph_c/resource_handle.h:50).  Here that
 * pointer is a cugraph_amd_mg_context_t created below:
 *
 *   - RCCL (production): one process per GPU; rank 0 makes a unique id, the
 *     caller broadcasts its bytes (e.g. torch.distributed), every rank calls
 *     cugraph_amd_mg_context_create_rccl.  The row and column communicators of
 *     the R x C grid (rank = r * C + c, C = row_comm_size) are ncclCommSplit
 *     children of the world communicator.
 *   - host callbacks: the caller supplies the collectives (used by the tests to
 *     run the MG path with several ranks on one GPU over torch.distributed/gloo,
 *     which RCCL forbids).  Buffers passed to the callbacks are device pointers;
 *     `stream` is the hipStream_t the data is ordered on (the callee must
 *     synchronise it before reading and leave results ready before returning).
 *
 * Every collective is issued by all ranks of the communicator in the same order.
 */
#pragma once
#include <cugraph_c/algorithms.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int32_t align_;
} cugraph_amd_mg_context_t;

/* element types / reduction ops of the callback interface */
enum cugraph_amd_comm_dtype { CGX_COMM_U8 = 0, CGX_COMM_I32, CGX_COMM_I64, CGX_COMM_U64, CGX_COMM_F32, CGX_COMM_F64 };
enum cugraph_amd_comm_op { CGX_COMM_SUM = 0, CGX_COMM_MIN, CGX_COMM_MAX };

typedef struct {
  void* ctx;
  int rank;
  int size;
  /* recv[i] = op over ranks of send[i], i < count */
  int (*allreduce)(void* ctx, const void* send, void* recv, size_t count, int dtype, int op, void* stream);
  /* recv = concatenation over ranks of `count` elements each */
  int (*allgather)(void* ctx, const void* send, void* recv, size_t count, int dtype, void* stream);
  /* recv = segment `rank` (recvcount elements) of the op over ranks of send (size * recvcount) */
  int (*reduce_scatter)(void* ctx, const void* send, void* recv, size_t recvcount, int dtype, int op, void* stream);
  /* element counts / displacements (host arrays of `size` entries) */
  int (*alltoallv)(void* ctx, const void* send, const size_t* sendcounts, const size_t* sdispls, void* recv,
                   const size_t* recvcounts, const size_t* rdispls, int dtype, void* stream);
} cugraph_amd_comm_ops_t;

/* RCCL unique id (ncclUniqueId, 128 bytes) */
size_t cugraph_amd_comm_unique_id_size(void);
cugraph_error_code_t cugraph_amd_comm_get_unique_id(void* unique_id, cugraph_error_t** error);

cugraph_error_code_t cugraph_amd_mg_context_create_rccl(const void* unique_id,
                                                        int world_size,
                                                        int rank,
                                                        int row_comm_size,
                                                        cugraph_amd_mg_context_t** context,
                                                        cugraph_error_t** error);

/* world, row (size row_comm_size, rank c) and column (size world/row_comm_size, rank r) */
cugraph_error_code_t cugraph_amd_mg_context_create_ops(const cugraph_amd_comm_ops_t* world,
                                                       const cugraph_amd_comm_ops_t* row,
                                                       const cugraph_amd_comm_ops_t* col,
                                                       int row_comm_size,
                                                       cugraph_amd_mg_context_t** context,
                                                       cugraph_error_t** error);

void cugraph_amd_mg_context_free(cugraph_amd_mg_context_t* context);

#ifdef __cplusplus
}
#endif
