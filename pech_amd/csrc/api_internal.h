// api_internal.h -- library-private hooks shared by crc32c_api.cpp and
// crc32c_async.cpp (hidden visibility: not exported by libpech_crc32c.so).
#ifndef PECH_API_INTERNAL_H
#define PECH_API_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "layout.h"

#define PECH_HIDDEN __attribute__((visibility("hidden")))

// plan + main kernels for n device descriptors on `stream`, explicit
// workspace (pech_ws_bytes(n) bytes, 256-byte aligned); current device
PECH_HIDDEN int pech_internal_launch(const pech_desc *d_descs, uint32_t *d_out, unsigned int n, void *ws,
				     size_t ws_bytes, hipStream_t stream);
// set the thread's crc32c_last_error() text
PECH_HIDDEN void pech_internal_set_err(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

#endif
