/*
 * pech_crc32c.h -- batch / device / algebra API of libpech_crc32c.so.
 *
 * Every entry point computes exactly what the reference's per-buffer
 * crc32c(seed, buf, len) (/root/reference/include/crc32c.h:88-96) returns;
 * what changes is how many buffers one call covers and where the bytes live.
 *
 * Reference interfaces these replace or extend (file:line in /root/reference):
 *   crc32c_batch          -- the per-payload loop of ceph_crc32c_iov()
 *                            (src/ceph/messenger.c:1734-1740, driven from
 *                            read_partial_msg_data :2677 and
 *                            write_partial_message_data :1788): one call per
 *                            completed payload instead of one per <=4 KiB
 *                            piece (bit-identical by the chaining law).
 *   crc32c_dev_batch_*    -- same, over device-resident buffers (GPU-resident
 *                            object data; no reference counterpart).
 *   crc32c_dev_copy_batch_* -- CRC fused with the copy memstore makes of the
 *                            same bytes (src/ceph/memstore.c:306, :445).
 *   crc32c_combine/_shift -- CRC reuse across replica sends
 *                            (src/ceph/osd_server.c:1119 nested cursor,
 *                            :1972 per-replica ceph_con_send) and page-piece
 *                            joins (src/iov_iter.c:188-207).
 *
 * Conventions (pech style, include/err.h): int-returning calls give 0 or a
 * negative errno: -EINVAL bad arguments, -ENOMEM allocation failure, -EIO a
 * HIP failure (crc32c_last_error() has the text), -ENODEV no usable GPU.
 * Batch, device and async calls never fall back to the CPU: without a GPU
 * they fail loudly.  Only the drop-in crc32c() (crc32c.h) stays total.
 * Threading: any thread may call; pech uses one (README:11-16).  Every entry
 * point that calls HIP runs on a per-thread 8 MiB library stack, so pech's
 * 64 KiB coroutine stacks (src/sched.c:16) need no change.
 * The internal workspace of crc32c_dev_[copy_]batch_async serves one launch
 * at a time: a launch on another stream than the previous one waits for it
 * (use the _ws_ forms with one workspace per stream for concurrency).
 */
#ifndef PECH_CRC32C_H
#define PECH_CRC32C_H

#include <stddef.h>
#include <stdint.h>

#include "crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One device-resident buffer of a device batch (16 bytes, AoS). */
struct crc32c_desc {
	uint64_t addr; /* device address of the first byte (any alignment) */
	uint32_t len;  /* bytes; 0 => result is seed                        */
	uint32_t seed; /* incoming register, as crc32c()'s first argument    */
};

/* flags for crc32c_batch() */
#define CRC32C_F_HOST 0u   /* bufs are pageable host memory                */
#define CRC32C_F_DEVICE 1u /* bufs are device memory on the current device */
#define CRC32C_F_PINNED 2u /* bufs are pinned host memory (read in place)   */
#define CRC32C_F_ALL_DEVICES 4u /* with CRC32C_F_PINNED: shard over every GPU */

/*
 * out[i] = crc32c(seeds ? seeds[i] : 0, bufs[i], lens[i]) for i < n.
 * Synchronous.  Pageable host buffers are moved with hipMemcpyAsync through
 * pinned staging (double-buffered, one copy stream per slot, overlapped with
 * the kernel).  Pinned buffers (CRC32C_F_PINNED: hipHostMalloc'd, registered
 * or crc32c_pages memory) of 1 MiB or more are DMA'd straight from their
 * pages; smaller ones are read by the kernel in place through their device
 * mapping (zero-copy: no host memcpy, no per-buffer DMA call), falling back
 * to staging if a buffer has no mapping.  Results come back with one D2H
 * copy per sub-batch.
 * CRC32C_F_PINNED | CRC32C_F_ALL_DEVICES: the batch is split into contiguous,
 * byte-balanced shards, one per visible GPU, each read in place over its own
 * host link; all shards are issued from the calling thread before any is
 * waited for (pech's one thread drives a whole node).  A
 * buffer of at least 16 MiB that exceeds one GPU's share of the batch is cut
 * into per-GPU segments whose CRCs are combined on the host.  Every
 * buffer must be mapped on every GPU (hipHostMalloc / crc32c_pages memory);
 * otherwise -EINVAL and nothing is launched.  Other flag combinations with
 * CRC32C_F_ALL_DEVICES are -EINVAL.
 */
int crc32c_batch(const void *const *bufs, const unsigned int *lens, const uint32_t *seeds,
		 uint32_t *out, unsigned int n, unsigned int flags);

/*
 * Device batch, asynchronous on `stream` (a hipStream_t, NULL = default
 * stream): d_out[i] = crc32c(d_descs[i].seed, d_descs[i].addr, d_descs[i].len).
 * The lengths of one call must total below 512 GiB (the kernels count 128-byte
 * rows in 32 bits); more than HBM holds, so only descriptors aliasing the same
 * memory can reach it -- split such batches (the synchronous crc32c_batch
 * does this itself).
 * d_descs and d_out are device memory of the current device; the call only
 * enqueues work (no host synchronisation, no allocation once the internal
 * workspace is large enough: see crc32c_dev_reserve()).  Buffers and
 * descriptors must stay valid and unmodified until the stream reaches the
 * end of the enqueued work.
 */
int crc32c_dev_batch_async(const struct crc32c_desc *d_descs, uint32_t *d_out, unsigned int n,
			   void *stream);

/*
 * Small-buffer device batch: as crc32c_dev_batch_async, in ONE kernel launch
 * with no workspace (no plan kernel; the descriptors are read where they
 * lie), so any number of streams may use it concurrently and it can be
 * captured in a graph.  Balanced for batches whose buffers are all below
 * 32 KiB (the messenger's front/middle/data segments and small-object
 * payloads); correct for any batch, but a larger buffer is walked by one
 * 8-lane group alone -- route those to crc32c_dev_batch_async.  The results
 * are stored (d_out needs no initialisation).
 */
int crc32c_dev_batch_small_async(const struct crc32c_desc *d_descs, uint32_t *d_out, unsigned int n,
				 void *stream);

/* Workspace the device batch needs for n buffers, and the explicit-workspace
 * form (for concurrent streams or graph capture; the internal-workspace forms
 * are refused inside a capture, -EINVAL).  d_workspace must be
 * 256-byte aligned (hipMalloc memory is) and used by one launch at a time. */
size_t crc32c_dev_workspace_bytes(unsigned int n);
int crc32c_dev_batch_ws_async(const struct crc32c_desc *d_descs, uint32_t *d_out, unsigned int n,
			      void *d_workspace, size_t workspace_bytes, void *stream);

/*
 * Fused CRC + copy, device batch, asynchronous on `stream`:
 *   d_out[i] = crc32c(d_descs[i].seed, d_descs[i].addr, d_descs[i].len)  and
 *   the len bytes at d_descs[i].addr are copied to d_dsts[i]
 * in ONE pass over the source bytes (each read once from HBM, written once).
 * Replaces the CRC pass plus the separate gathers of memstore's write path
 * (copy_from_iter into 64 KiB blocks, src/ceph/memstore.c:306) and read path
 * (memcpy gather, :445).  Any source / destination alignment; destination
 * ranges must not overlap any source range of the batch (as for memcpy).
 * Same workspace rules as crc32c_dev_batch_*.
 */
int crc32c_dev_copy_batch_async(const struct crc32c_desc *d_descs, const uint64_t *d_dsts, uint32_t *d_out,
				unsigned int n, void *stream);
int crc32c_dev_copy_batch_ws_async(const struct crc32c_desc *d_descs, const uint64_t *d_dsts, uint32_t *d_out,
				   unsigned int n, void *d_workspace, size_t workspace_bytes, void *stream);
/* Fused CRC + copy of a small-buffer batch: as crc32c_dev_copy_batch_async,
 * in ONE launch with no workspace (the direct kernel, as
 * crc32c_dev_batch_small_async: balanced for buffers below 32 KiB, correct
 * for any; graph-capturable; d_out needs no initialisation). */
int crc32c_dev_copy_batch_small_async(const struct crc32c_desc *d_descs, const uint64_t *d_dsts, uint32_t *d_out,
				      unsigned int n, void *stream);

/* Device batches (crc32c_dev_batch_async / _ws_async, and the batches the
 * synchronous and async host paths launch) of at most n buffers run as ONE
 * kernel launch with no plan kernel; larger ones, fused copies and batches
 * captured in a graph take the two-launch plan + main path (pech_crc32c_flat
 * up to 256 buffers, pech_crc32c_flatg up to 4,096).  Default and maximum
 * 4,096; 0 = always plan + main.
 * Results are identical either way.  Returns the previous value. */
unsigned int crc32c_set_flat_max(unsigned int n);

/* Pre-size the internal workspace of the current device for n buffers. */
int crc32c_dev_reserve(unsigned int n);

/* Algebra (no data pass):
 *   crc32c_shift(v, n)        == crc32c(v, <n zero bytes>, n)
 *   crc32c_combine(a, b, lb)  == crc32c(s, A||B)  given a = crc32c(s, A),
 *                                b = crc32c(0, B), lb = |B|.               */
uint32_t crc32c_shift(uint32_t v, uint64_t nbytes);
uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* Drop-in routing: crc32c() calls of at most `bytes` bytes are computed on
 * the host CPU, larger ones on the GPU (0 = every non-empty call on the GPU).
 * Default 4 MiB, or the PECH_CRC32C_CPU_MAX environment variable.  Returns
 * the previous value. */
unsigned int crc32c_set_cpu_max(unsigned int bytes);

/* Process-wide counters of the drop-in crc32c(). */
struct crc32c_stats {
	uint64_t cpu_calls, cpu_bytes;  /* computed on the host (incl. fallbacks) */
	uint64_t gpu_calls, gpu_bytes;  /* computed by the gfx950 kernels          */
	uint64_t gpu_fallbacks;         /* GPU path failed, recomputed on the host */
	uint64_t gpu_faults;            /* flat launches whose results the kernel itself
	                                   voided (a wave's wait for out[]'s
	                                   initialisation timed out): the synchronous
	                                   and async paths discard them; a device
	                                   entry point's caller must too */
};
int crc32c_get_stats(struct crc32c_stats *st);

/* Eagerly initialise the current device (tables, streams).  Optional. */
int crc32c_device_init(void);

/* Kernel timing: when enabled, every main-kernel launch carries a pair of
 * HIP events stamped by its own dispatch packet (hipExtLaunchKernel: kernel
 * start and end on its stream, no launch boundary included);
 * crc32c_timing_read() synchronises on them and returns the summed kernel
 * milliseconds and launch count since the last read. */
int crc32c_timing(int enable);
int crc32c_timing_read(double *kernel_ms, uint64_t *launches);
/* Per-launch milliseconds collected by the last crc32c_timing_read():
 * copies up to `max` into `ms`, returns how many there were. */
int crc32c_timing_samples(float *ms, unsigned int max);

/* Text of the last error (thread-local), "" if none. */
const char *crc32c_last_error(void);

/* Library / kernel identification, e.g. "pech_crc32c gfx950 rows128 ...". */
const char *crc32c_version(void);

#ifdef __cplusplus
}
#endif

#endif /* PECH_CRC32C_H */
