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
 * `data` is HOST memory.  The bytes are staged to the GPU and checksummed by
 * the gfx950 kernel; the call is synchronous and cannot fail (a HIP failure
 * aborts the process with a message -- the library has no CPU fallback).
 * For throughput use the batch API in pech_crc32c.h.
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
