/*
 * pech_crc32c_async.h -- the messenger-facing layer of libpech_crc32c.so
 * (SURVEY.md §8f rows 1-3): payload checksums that complete through an
 * eventfd on pech's epoll loop, DMA-able payload pages, and CRC reuse by
 * concatenation.  Every result equals the reference's
 * crc32c(seed, buf, len) (/root/reference/include/crc32c.h:88-96).
 *
 * Reference interfaces these serve (file:line in /root/reference):
 *   crc32c_async_*  -- replaces the per-<=4 KiB-piece ceph_crc32c_iov() chain
 *                      (src/ceph/messenger.c:1734-1740) of read_partial_msg_data
 *                      (:2649-2684, verified at the footer :2836-2842) and
 *                      write_partial_message_data (:1748-1803) with ONE
 *                      submission per completed payload; completion is an
 *                      eventfd an event_item watches (include/event.h:7-28),
 *                      so the single-threaded loop never blocks on the GPU.
 *   crc32c_pages_*  -- alloc_pages()/__free_pages() (src/page.c:73-146):
 *                      same 2^order-page sizes and per-order free lists
 *                      (orders 0..11, 32 MiB cached per order), but pinned,
 *                      GPU-mapped host memory, so payload bytes received into
 *                      them reach the GPU by DMA (or are read by the kernel
 *                      in place) with no staging copy.  Backs alloc_bvec() in
 *                      osds_alloc_msg() (src/ceph/osd_server.c:2317-2381).
 *   crc32c_concat   -- the data CRC of a message whose data section is a
 *                      concatenation of already-checksummed segments: the
 *                      REPOP fan-out re-sends the request's op data through
 *                      nested cursors (osd_server.c:1119, sent per replica
 *                      at :1972) and would otherwise re-scan the same bytes
 *                      once per replica.
 *
 * Threading: an async context belongs to ONE caller thread (pech has one,
 * README:11-16).  The HIP runtime signals the eventfd from its own thread;
 * callbacks only ever run inside crc32c_async_complete() on the caller's
 * thread.  Errors: 0 or a negative errno (include/err.h style), as in
 * pech_crc32c.h; no CPU fallback.
 */
#ifndef PECH_CRC32C_ASYNC_H
#define PECH_CRC32C_ASYNC_H

#include <stddef.h>
#include <stdint.h>

#include "pech_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- DMA-able payload pages (src/page.c:73-146) ------------------------ */
#define CRC32C_PAGE_SHIFT 12u
#define CRC32C_PAGE_SIZE (1u << CRC32C_PAGE_SHIFT)
#define CRC32C_PAGES_MAX_ORDER 11u /* src/page.c:5; larger orders are not cached */

/* (4096 << order) bytes of pinned, GPU-mapped host memory, page aligned;
 * NULL on failure (crc32c_last_error()).  Orders <= 11 come from a free list
 * when one is cached. */
void *crc32c_pages_alloc(unsigned int order);
/* Return pages from crc32c_pages_alloc(order); cached up to 32 MiB per order
 * (src/page.c:6), released to the driver beyond that. */
void crc32c_pages_free(void *pages, unsigned int order);
/* 1 if [p, p + len) lies inside ONE live crc32c_pages_alloc() allocation. */
int crc32c_pages_is_pinned(const void *p, size_t len);
/* Release every cached free page (deinit_pages(), src/page.c:46-58). */
void crc32c_pages_trim(void);

/* ---- asynchronous payload checksums ------------------------------------ */
struct crc32c_async;

/* Completion callback: crc = crc32c(seed, buf, len) of the submission, or
 * err < 0 if the GPU work failed (crc is then 0 and must not be used). */
typedef void (*crc32c_done_fn)(void *arg, uint32_t crc, int err);

/* flags for crc32c_async_create().
 * Default (0): payloads in crc32c_pages memory are read by the kernel in
 * place over the host link: no H2D copy and no per-payload DMA call, so the
 * caller's thread pays about a microsecond per payload at any size
 * (DESIGN.md 6.4).  Pageable payloads are packed into pinned staging. */
#define CRC32C_ASYNC_DEFAULT 0u
/* The default since round 4; accepted for callers written before. */
#define CRC32C_ASYNC_ZEROCOPY 1u
/* crc32c_pages payloads from 32 KiB up are DMA'd to device staging instead:
 * more host-link bandwidth for large payloads (MI355X: 42 against 36 GiB/s
 * at 4 MiB, for 5 against 4 us of the caller's CPU per payload; but 5
 * against 19 GiB/s at 64 KiB).  The copies are recorded at
 * submit and issued together when the slot launches (one batched call where
 * the HIP runtime has hipMemcpyBatchAsync).  One slot's copies are in flight
 * at a time: a filled slot waits, without a HIP call, and launches from
 * crc32c_async_complete() (or a wait for a free slot, or drain) once the
 * slots before it are harvested.  Not with ZEROCOPY. */
#define CRC32C_ASYNC_DMA 2u

/* A context on the current device: its own HIP stream, staging slots and
 * eventfd.  NULL on failure.  Every later call on the context runs on that
 * device and restores the caller's current device, so one thread can drive
 * one context per GPU (independent payloads shard over GPUs with no
 * collective). */
struct crc32c_async *crc32c_async_create(unsigned int flags);

/* The same on GPU `device` (the caller's current device is left as it was). */
struct crc32c_async *crc32c_async_create_on(int device, unsigned int flags);

/* The GPUs a caller that spreads its payloads over several contexts should
 * use, one context each: every visible device, or the PECH_DEVICES list
 * ("0,0" repeats a device: two contexts on one GPU, how a one-GPU machine
 * rehearses a node).  Fills up to max entries of devs; returns the count, or
 * a negative errno (-ENODEV: no GPU, -EINVAL: a bad list). */
int crc32c_async_devices(int *devs, int max);

/* The eventfd (EFD_NONBLOCK | EFD_CLOEXEC): readable while finished batches
 * wait for crc32c_async_complete().  Owned by the context. */
int crc32c_async_fd(const struct crc32c_async *a);

/* Queue crc32c(seed, buf, len) of HOST memory `buf` (pageable, or
 * crc32c_pages memory: read in place, or DMA'd with CRC32C_ASYNC_DMA; no CPU
 * copy).  The caller
 * keeps `buf` unchanged and alive until `done` runs (hold a ceph_msg_get()
 * reference, messenger.c:3907-3924).  Any length < 2^32, including 0.  A
 * full batch is launched automatically; otherwise call crc32c_async_flush(). */
int crc32c_async_submit(struct crc32c_async *a, const void *buf, unsigned int len, uint32_t seed,
			crc32c_done_fn done, void *arg);

/* Launch everything queued (asynchronous; returns at once). */
int crc32c_async_flush(struct crc32c_async *a);

/* Run the callbacks of every finished batch, in submission order, on the
 * calling thread; clears the eventfd.  Returns the number of callbacks run
 * (>= 0) or a negative errno.  Never blocks.  A batch whose stream failed
 * after the launch never signals the eventfd (HIP skips its host function);
 * complete() finds it by querying the stream and fails its payloads (err
 * -EIO).  So the loop calls complete() when the fd fires AND from a timer
 * (pech: a timer_list of a few ms) while crc32c_async_pending() > 0. */
int crc32c_async_complete(struct crc32c_async *a);

/* Flush and wait until every submission's callback has run (shutdown, tests). */
int crc32c_async_drain(struct crc32c_async *a);

/* Submissions queued or in flight whose callbacks have not run yet. */
unsigned int crc32c_async_pending(const struct crc32c_async *a);

/* Drain, then free the context (its eventfd is closed). */
void crc32c_async_destroy(struct crc32c_async *a);

/* Per-context counters (no HIP call). */
struct crc32c_async_stats {
	int device;             /* the GPU the context runs on                    */
	uint64_t submitted;     /* accepted submissions                           */
	uint64_t launches;      /* batches launched                               */
	unsigned int inflight;  /* batches launched and not yet harvested         */
	unsigned int queued;    /* CRC32C_ASYNC_DMA: filled slots waiting to launch */
	uint64_t host_out;      /* launches whose kernel stored the results in host memory itself */
	uint64_t polled;        /* launches whose completion the context's thread polled */
	uint64_t faults;        /* flat launches whose results the kernel voided: their
	                           payloads failed with -EIO (no CRC delivered)       */
	uint64_t pub_missing;   /* flat launches whose in-kernel results publication
	                           was missing: the results were copied from the GPU
	                           instead (never a previous batch's)                 */
};
int crc32c_async_get_stats(const struct crc32c_async *a, struct crc32c_async_stats *st);

/* ---- CRC reuse by concatenation (host algebra, no data pass) ----------- */
/* crc32c(seed, S_0 || S_1 || ... || S_{n-1}) from the segments' zero-seeded
 * CRCs crcs[i] = crc32c(0, S_i, lens[i]).  n == 0 returns seed. */
uint32_t crc32c_concat(uint32_t seed, const uint32_t *crcs, const uint64_t *lens, unsigned int n);

#ifdef __cplusplus
}
#endif

#endif /* PECH_CRC32C_ASYNC_H */
