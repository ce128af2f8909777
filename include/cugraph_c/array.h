/*
 * libcugraph_c type-erased arrays -- MI355X build.
 * ABI-compatible with the reference cpp/include/cugraph_c/array.h:25-326.
 * Device arrays live in HBM, allocated on the handle's stream from
 * libcugraph_c's stream-ordered caching allocator (csrc/alloc.cpp); views wrap
 * caller memory and never own it.
 */
#pragma once
#include <cugraph_c/resource_handle.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { int32_t align_; } cugraph_type_erased_device_array_t;
typedef struct { int32_t align_; } cugraph_type_erased_device_array_view_t;
typedef struct { int32_t align_; } cugraph_type_erased_host_array_t;
typedef struct { int32_t align_; } cugraph_type_erased_host_array_view_t;

/* reference array.h:52 */
cugraph_error_code_t cugraph_type_erased_device_array_create(
  const cugraph_resource_handle_t* handle,
  size_t n_elems,
  data_type_id_t dtype,
  cugraph_type_erased_device_array_t** array,
  cugraph_error_t** error);

/* reference array.h:67 */
cugraph_error_code_t cugraph_type_erased_device_array_create_from_view(
  const cugraph_resource_handle_t* handle,
  const cugraph_type_erased_device_array_view_t* view,
  cugraph_type_erased_device_array_t** array,
  cugraph_error_t** error);

/* reference array.h:78 */
void cugraph_type_erased_device_array_free(cugraph_type_erased_device_array_t* p);

/* reference array.h:95 (compiled out there with `#if 0`; implemented here).
 * Gives up ownership: the array handle is freed, its stream synchronised, and the
 * returned device pointer belongs to the caller, who frees it with hipFree. */
void* cugraph_type_erased_device_array_release(cugraph_type_erased_device_array_t* p);

/* reference array.h:97 -- view of an owning array (lives as long as the array) */
cugraph_type_erased_device_array_view_t* cugraph_type_erased_device_array_view(
  cugraph_type_erased_device_array_t* array);

/* reference array.h:111 */
cugraph_error_code_t cugraph_type_erased_device_array_view_as_type(
  cugraph_type_erased_device_array_t* array,
  data_type_id_t dtype,
  cugraph_type_erased_device_array_view_t** result_view,
  cugraph_error_t** error);

/* reference array.h:126 -- wraps caller device memory */
cugraph_type_erased_device_array_view_t* cugraph_type_erased_device_array_view_create(
  void* pointer, size_t n_elems, data_type_id_t dtype);

/* reference array.h:134 */
void cugraph_type_erased_device_array_view_free(cugraph_type_erased_device_array_view_t* p);

/* reference array.h:142 */
size_t cugraph_type_erased_device_array_view_size(const cugraph_type_erased_device_array_view_t* p);

/* reference array.h:150 */
data_type_id_t cugraph_type_erased_device_array_view_type(
  const cugraph_type_erased_device_array_view_t* p);

/* reference array.h:159 */
const void* cugraph_type_erased_device_array_view_pointer(
  const cugraph_type_erased_device_array_view_t* p);

/* reference array.h:172 */
cugraph_error_code_t cugraph_type_erased_host_array_create(const cugraph_resource_handle_t* handle,
                                                           size_t n_elems,
                                                           data_type_id_t dtype,
                                                           cugraph_type_erased_host_array_t** array,
                                                           cugraph_error_t** error);

/* reference array.h:183 */
void cugraph_type_erased_host_array_free(cugraph_type_erased_host_array_t* p);

/* reference array.h:212 (compiled out there with `#if 0`; implemented here).
 * The array handle is freed and its bytes returned in a malloc'd block the caller
 * frees with free(); NULL for an empty array. */
void* cugraph_type_erased_host_array_release(cugraph_type_erased_host_array_t* p);

/* reference array.h:202 */
cugraph_type_erased_host_array_view_t* cugraph_type_erased_host_array_view(
  cugraph_type_erased_host_array_t* array);

/* reference array.h:213 */
cugraph_type_erased_host_array_view_t* cugraph_type_erased_host_array_view_create(
  void* pointer, size_t n_elems, data_type_id_t dtype);

/* reference array.h:221 */
void cugraph_type_erased_host_array_view_free(cugraph_type_erased_host_array_view_t* p);

/* reference array.h:229 */
size_t cugraph_type_erased_host_array_size(const cugraph_type_erased_host_array_view_t* p);

/* reference array.h:237 */
data_type_id_t cugraph_type_erased_host_array_type(const cugraph_type_erased_host_array_view_t* p);

/* reference array.h:245 */
void* cugraph_type_erased_host_array_pointer(const cugraph_type_erased_host_array_view_t* p);

/* reference array.h:258 */
cugraph_error_code_t cugraph_type_erased_host_array_view_copy(
  const cugraph_resource_handle_t* handle,
  cugraph_type_erased_host_array_view_t* dst,
  const cugraph_type_erased_host_array_view_t* src,
  cugraph_error_t** error);

/* reference array.h:275 */
cugraph_error_code_t cugraph_type_erased_device_array_view_copy_from_host(
  const cugraph_resource_handle_t* handle,
  cugraph_type_erased_device_array_view_t* dst,
  const byte_t* h_src,
  cugraph_error_t** error);

/* reference array.h:292 */
cugraph_error_code_t cugraph_type_erased_device_array_view_copy_to_host(
  const cugraph_resource_handle_t* handle,
  byte_t* h_dst,
  const cugraph_type_erased_device_array_view_t* src,
  cugraph_error_t** error);

/* reference array.h:309 */
cugraph_error_code_t cugraph_type_erased_device_array_view_copy(
  const cugraph_resource_handle_t* handle,
  cugraph_type_erased_device_array_view_t* dst,
  const cugraph_type_erased_device_array_view_t* src,
  cugraph_error_t** error);

#ifdef __cplusplus
}
#endif
