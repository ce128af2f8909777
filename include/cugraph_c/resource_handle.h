/*
 * libcugraph_c resource handle -- MI355X build.
 * ABI-compatible with the reference cpp/include/cugraph_c/resource_handle.h:28-69.
 *
 * The handle owns one HIP stream on the current device.  In the reference the
 * void* argument is a raft::handle_t*; here it is either NULL (single GPU) or a
 * communicator created by cugraph_amd_comm_create() (include/cugraph_amd/comm.h).
 */
#pragma once
#include <cugraph_c/error.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum bool_ { FALSE = 0, TRUE = 1 } bool_t;

typedef int8_t byte_t;

/* reference resource_handle.h:30 */
typedef enum data_type_id_ { INT32 = 0, INT64, FLOAT32, FLOAT64, NTYPES } data_type_id_t;

typedef struct cugraph_resource_handle_ {
  int32_t align_;
} cugraph_resource_handle_t;

/* reference resource_handle.h:50 */
cugraph_resource_handle_t* cugraph_create_resource_handle(void* raft_handle);

/* reference resource_handle.h:60 -- rank in the communicator (0 for SG) */
int cugraph_resource_handle_get_rank(const cugraph_resource_handle_t* handle);

/* reference resource_handle.h:67 */
void cugraph_free_resource_handle(cugraph_resource_handle_t* handle);

#ifdef __cplusplus
}
#endif
