/*
 * libcugraph_c error objects -- MI355X build.
 * ABI-compatible with the reference cpp/include/cugraph_c/error.h:25-52.
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* reference error.h:25-33 */
typedef enum cugraph_error_code_ {
  CUGRAPH_SUCCESS = 0,
  CUGRAPH_UNKNOWN_ERROR,
  CUGRAPH_INVALID_HANDLE,
  CUGRAPH_ALLOC_ERROR,
  CUGRAPH_INVALID_INPUT,
  CUGRAPH_NOT_IMPLEMENTED,
  CUGRAPH_UNSUPPORTED_TYPE_COMBINATION
} cugraph_error_code_t;

/* opaque, reference error.h:35 */
typedef struct cugraph_error_ {
  int32_t align_;
} cugraph_error_t;

/* reference error.h:45 -- message of an error returned by any entry point */
const char* cugraph_error_message(const cugraph_error_t* error);

/* reference error.h:52 -- NULL is allowed */
void cugraph_error_free(cugraph_error_t* error);

#ifdef __cplusplus
}
#endif
