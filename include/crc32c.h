/*
 * crc32c.h -- drop-in replacement for pech's include/crc32c.h.
 *
 * Replaces /root/reference/include/crc32c.h:88-96:
 *     static inline u32 crc32c(u32 crc, const void *data_, unsigned int length)
 * with the same identifier, argument meaning and result, exported with C
 * linkage from libpech_crc32c.so (the reference's version is static inline,
 * so no caller depends on a symbol; src/ceph/messenger.c:6 keeps including
 * "crc32c.h" and its six call sites compile unchanged).
 *
 * Semantics (bit-exact with the reference): reflected CRC-32C (polynomial
 * 0x1EDC6F41, reflected 0x82F63B78), byte-wise raw register update, NO pre-
 * or post-inversion; `crc` is the incoming register (the messenger passes 0);
 * length 0 returns `crc`; any alignment; `data` is read only.  Chaining holds
 * exactly: crc32c(crc32c(s, A, |A|), B, |B|) == crc32c(s, A||B, |A|+|B|).
 *
 * `data` is HOST memory.  The call is synchronous and, like the reference,
 * cannot fail.  Calls of up to crc32c_set_cpu_max() bytes (default 4 MiB:
 * every header, front/middle section and <=4 KiB data piece the messenger
 * hashes) run on the host (SSE4.2 crc32, 3 streams,
 * ~0.01 us for a 49-byte header); larger ones are staged to the GPU and
 * checksummed by the gfx950 kernel, on a library-owned stack (safe from
 * pech's 64 KiB coroutine stacks, src/sched.c:16).  If the GPU path fails
 * the bytes are recomputed on the host (crc32c_get_stats() counts it).
 * Throughput belongs to the batch / async APIs (pech_crc32c*.h).
 */
#ifndef _CRC32C_H
#define _CRC32C_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* replaces include/crc32c.h:88 (static inline u32 crc32c(u32, const void *, unsigned int)) */
uint32_t crc32c(uint32_t crc, const void *data, unsigned int length);

#ifdef __cplusplus
}
#endif

#endif /* _CRC32C_H */
