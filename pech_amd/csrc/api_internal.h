// api_internal.h -- library-private hooks shared by crc32c_api.cpp and
// crc32c_async.cpp (hidden visibility: not exported by libpech_crc32c.so).
#ifndef PECH_API_INTERNAL_H
#define PECH_API_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "layout.h"

#define PECH_HIDDEN __attribute__((visibility("hidden")))

// The kernels for n device descriptors on `stream` (small: the direct
// kernel; else flat, or plan + main), explicit workspace (pech_ws_bytes(n)
// bytes, 256-byte aligned); current device.  hout (a device-visible pinned
// host array of n words, or NULL): returns 1 when the results are stored
// there by the kernel itself, 0 when they are in d_out (the caller copies),
// a negative errno on failure.
// hstat (the device view of a coherent pinned host word, or NULL): a flat
// launch's status word (layout.h PECH_FLAT_PUB / PECH_FLAT_ERR); *flat_tag:
// that launch's tag, 0 when the batch did not run as one flat launch.
// host_resident: every buffer is pinned host memory read in place (a
// zero-copy slot; the flat kernel's interleaved rows, PECH_FLAT_F_IL).
PECH_HIDDEN int pech_internal_launch(const pech_desc *d_descs, uint32_t *d_out, unsigned int n, void *ws,
				     size_t ws_bytes, hipStream_t stream, bool small = false, uint32_t *hout = nullptr,
				     uint64_t *hstat = nullptr, uint64_t *flat_tag = nullptr, bool host_resident = false);
// The GPUs a multi-device caller spreads over: PECH_DEVICES="0,0,..." (a
// repeated id puts several shards or contexts on one GPU: how one-GPU boxes
// rehearse eight) or every visible device.  Count, or a negative errno.
PECH_HIDDEN int pech_internal_device_list(int *devs, int max, int max_per_dev);
// set the thread's crc32c_last_error() text
PECH_HIDDEN void pech_internal_set_err(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

// crc32c_cpu.c: the host routine of the drop-in (small calls, GPU-failure
// fallback) and the per-thread library stack every HIP-calling entry point
// runs on (pech's coroutines have 64 KiB stacks, src/sched.c:16)
extern "C" {
PECH_HIDDEN uint32_t pech_cpu_crc32c(uint32_t crc, const void *data, size_t n);
PECH_HIDDEN uint32_t pech_cpu_crc32c_portable(uint32_t crc, const void *data, size_t n);
PECH_HIDDEN int pech_cpu_has_sse42(void);
PECH_HIDDEN void pech_stack_call(void (*fn)(void *), void *arg);
PECH_HIDDEN int pech_on_lib_stack(void);
}

// f() on the library stack; returns what f returns
template <class F> static inline auto on_lib_stack(F &&f) -> decltype(f())
{
	using R = decltype(f());
	struct Box {
		F *f;
		R r;
	} box{&f, R{}};
	pech_stack_call([](void *p) { Box *b = (Box *)p; b->r = (*b->f)(); }, &box);
	return box.r;
}

// Fault injection for the failure-path tests (tests/test_faults.py):
// pech_fault(site) is true on the countdown-th call at that site after
// crc32c_test_inject(site, countdown) armed it.
enum pech_fault_site {
	PECH_FAULT_DROPIN_GPU = 0, // drop-in crc32c(): its GPU launch fails
	PECH_FAULT_ASYNC_LAUNCH = 1, // async: a slot's kernel launch fails
	PECH_FAULT_ASYNC_DMA = 2,    // async: a payload's H2D DMA fails
	PECH_FAULT_ASYNC_STREAM = 3, // async: a launched batch's stream fails (no host function, query error)
	PECH_FAULT_FLAT_TIMEOUT = 4, // a flat launch's waves time out waiting for out[] (PECH_FLAT_T_TIMEOUT)
	PECH_FAULT_FLAT_NOPUB = 5,   // a flat launch skips its async slot's publication (PECH_FLAT_T_NOPUB)
	PECH_FAULT_SITES = 6
};
PECH_HIDDEN bool pech_fault(int site);

#endif
