/*
 * layout.h -- geometry shared by the host library and the gfx950 kernels.
 *
 * Virtual row space.  Every buffer (addr, len) is viewed as a run of 16-byte
 * aligned "pieces" [a0, a1), a0 = addr & ~15, a1 = align16(addr + max(len,4)),
 * grouped into 128-byte "rows" (8 pieces, one HBM cache line) that are
 * RIGHT-aligned to a1.  Pieces of the first row that lie below a0 are
 * virtual zeros (leading zeros do not change R(0, .)); bytes of real pieces
 * outside [addr, addr+len) are masked to zero; the z = a1 - (addr+len)
 * trailing zeros are undone by a final multiply with x^(-8z).  The seed is
 * xored into bytes [addr, addr+4) (gf2.h identities).
 *
 * One 8-lane "group" of a wave owns a contiguous range of rows of the
 * concatenated row space of a batch; lane g8 of the group holds piece g8 of
 * each row as four 4-byte "streams".
 */
#ifndef PECH_CRC32C_LAYOUT_H
#define PECH_CRC32C_LAYOUT_H

#include <stdint.h>

#define PECH_ROW_BYTES 128u
#define PECH_PIECE_BYTES 16u
#define PECH_GROUP_LANES 8u
#define PECH_WG_THREADS 1024u
#define PECH_GROUPS_PER_WG (PECH_WG_THREADS / PECH_GROUP_LANES)
#define PECH_CHUNK 1024u          /* buffers per plan chunk (one plan WG)  */
#define PECH_MAX_CHUNKS 1024u     /* => at most 2^20 buffers per launch    */
#define PECH_MAX_BATCH (PECH_CHUNK * PECH_MAX_CHUNKS)
#define PECH_RPG_MIN 32u          /* min rows per group (4 KiB)            */

/* constants block (u32 words), built on the host, uploaded once per device */
#define PECH_C_TAB128 0u    /* A_128 byte tables, 4 x 256  (Horner step)   */
#define PECH_C_TAB4 1024u   /* A_4   byte tables           (lane combine)  */
#define PECH_C_TAB16 2048u  /* A_16                        (butterfly 1)   */
#define PECH_C_TAB32 3072u  /* A_32                        (butterfly 2)   */
#define PECH_C_TAB64 4096u  /* A_64                        (butterfly 3)   */
#define PECH_C_POWR 5120u   /* x^(1024*j*64^i), i<5, j<64  (row shifts)    */
#define PECH_C_XINV 5440u   /* x^(-8z), z<32               (tail undo)     */
#define PECH_C_WORDS 5472u

/* device batch descriptor (matches struct crc32c_desc in include/) */
struct pech_desc {
	uint64_t addr;
	uint32_t len;
	uint32_t seed;
};

#ifdef __HIPCC__
#define LAYOUT_FN __host__ __device__ inline
#else
#define LAYOUT_FN static inline
#endif

/* rows of buffer (addr, len) in the virtual row space; 0 for len == 0 */
LAYOUT_FN uint32_t pech_rows(uint64_t addr, uint32_t len)
{
	if (len == 0)
		return 0;
	uint64_t a0 = addr & ~(uint64_t)15;
	uint64_t e4 = addr + (len < 4 ? 4u : len);
	uint64_t a1 = (e4 + 15) & ~(uint64_t)15;
	uint32_t pieces = (uint32_t)((a1 - a0) >> 4);
	return (pieces + 7) >> 3;
}

#endif /* PECH_CRC32C_LAYOUT_H */
