/*
 * layout.h -- geometry shared by the host library and the gfx950 kernels.
 *
 * Split of one buffer D = (addr, len, seed) (gf2.h identities):
 *   head h = [addr, cs)        cs = align16(addr)              (< 16 bytes)
 *   core c = [cs, ce)          ce = align16_down(addr + len)   (16-byte pieces)
 *   tail t = [ce, addr + len)                                  (< 16 bytes)
 *   crc32c(seed, D) = x^(8|t|) * R(0, c)                      <- main kernel
 *                   ^ x^(8 len) * seed
 *                   ^ x^(8(|c|+|t|)) * R(0, h) ^ R(0, t)      <- plan kernel
 * Buffers with no full aligned piece (len < 16 or spanning < one aligned
 * 16-byte block) are checksummed entirely by the plan kernel (<= 30 bytes).
 *
 * Row space.  The core's 16-byte pieces are grouped in 128-byte ROWS (8
 * pieces), on the 128-byte line grid, so every row load is one whole HBM
 * line: row 0 is the line holding cs (vbase = align128_down(cs)), its first
 * vp pieces (vp < 8) are virtual leading zeros, which do not change R(0, .);
 * the last row's last zt pieces (zt < 8) lie past ce, still inside that
 * line, and are read as zeros -- trailing zeros multiply R by x^(128 zt),
 * which the run's final shift undoes (x^(8 |t| - 128 zt), inverse powers
 * when negative).  (Until v0.12 rows were right-aligned to ce, so a core
 * whose end was not line-aligned put every row across two lines: +15 %
 * HBM traffic and +13 % time on such batches.)  One 8-lane GROUP of a wave
 * walks rows of one buffer; lane g8 of the group holds piece g8 of every
 * row as four 4-byte register "streams".
 */
#ifndef PECH_CRC32C_LAYOUT_H
#define PECH_CRC32C_LAYOUT_H

#include <stddef.h>
#include <stdint.h>

#define PECH_ROW_BYTES 128u
#define PECH_PIECE_BYTES 16u
#define PECH_GROUP_LANES 8u
#define PECH_WG_THREADS 1024u
#define PECH_WAVES_PER_WG (PECH_WG_THREADS / 64u)
#define PECH_CHUNK 1024u          /* buffers per plan chunk (one plan WG)  */
#define PECH_MAX_CHUNKS 1024u     /* => at most 2^20 buffers per launch    */
#define PECH_MAX_BATCH (PECH_CHUNK * PECH_MAX_CHUNKS)
#define PECH_RPW_MIN 64u          /* min rows per wave (8 KiB)             */
#define PECH_LARGE_ROWS 2048u     /* size-class cap for the plan's ordering  */
#define PECH_SPLIT_ROWS 256u      /* >= this: a buffer is split over 8 groups */
#ifndef PECH_ITEM_ROWS
#define PECH_ITEM_ROWS 256u       /* uniform batches: rows per pooled work item */
#endif
#ifndef PECH_POOL_ROWS
#define PECH_POOL_ROWS 512u       /* uniform batches: at most this many of a wave's rows are pooled */
#endif
#define PECH_NZ_UNIFORM 0x80000000u /* nzs[] flag: every buffer of the chunk has a core of the same rows */
#define PECH_SMALL_MAX 65536u     /* drop-in crc32c(): one-launch path up to this */
#define PECH_DROPIN_CPU_MAX_DEFAULT (4u << 20) /* drop-in crc32c(): host routine up to this */
/* payload of one launch: rows (128 B) are counted in 32 bits, so < 512 GiB */
#define PECH_LAUNCH_MAX_BYTES (256ull << 30)

/* constants block (u32 words), built on the host, uploaded once per device */
#define PECH_C_TAB128 0u    /* A_128 byte tables, 4 x 256  (row Horner step)  */
#define PECH_C_TAB4 1024u   /* A_4   byte tables           (lane fold)        */
#define PECH_C_TAB16 2048u  /* A_16                        (butterfly 1)      */
#define PECH_C_TAB32 3072u  /* A_32                        (butterfly 2)      */
#define PECH_C_TAB64 4096u  /* A_64                        (butterfly 3)      */
#define PECH_C_POWB 5120u   /* x^(8*j*64^i), i<6, j<64     (byte shifts)      */
#define PECH_C_TAB1 5504u   /* A_1 = the reference table, include/crc32c.h:16 */
#define PECH_C_XINV 5760u   /* x^(-8k), k < 128 (trailing virtual zeros)      */
#define PECH_C_WORDS 5888u

/* device batch descriptor (matches struct crc32c_desc in include/) */
struct pech_desc {
	uint64_t addr;
	uint32_t len;
	uint32_t seed;
};

/* per-buffer core descriptor written by the plan kernel, in row-space order */
struct pech_core {
	uint64_t vbase; /* address of row 0, piece 0 (may precede the core)      */
	uint32_t rows;  /* rows of the core (0: buffer fully done by the plan)   */
	uint32_t meta;  /* orig (bits 0-19) | vp (20-22) | tail (24-27) | zt (28-30) */
};

#define PECH_META(orig, vp, t, zt) \
	((orig) | ((uint32_t)(vp) << 20) | ((uint32_t)(t) << 24) | ((uint32_t)(zt) << 28))
#define PECH_META_ORIG(m) ((m) & 0xFFFFFu)
#define PECH_META_VP(m) (((m) >> 20) & 7u)
#define PECH_META_TAIL(m) (((m) >> 24) & 15u)
#define PECH_META_ZT(m) (((m) >> 28) & 7u)

#ifdef __HIPCC__
#define LAYOUT_FN __host__ __device__ inline
#else
#define LAYOUT_FN static inline
#endif

/* rows (128-byte lines) holding the core of buffer (addr, len); 0 if it has
 * no full aligned piece */
LAYOUT_FN uint32_t pech_core_rows(uint64_t addr, uint32_t len)
{
	const uint64_t cs = (addr + 15) & ~(uint64_t)15;
	const uint64_t ce = (addr + len) & ~(uint64_t)15;
	if (ce <= cs)
		return 0;
	return (uint32_t)((ce - (cs & ~(uint64_t)127) + 127) >> 7);
}

/* size class used to order buffers inside a plan chunk (similar row counts
 * become neighbours, so the 8 groups of a wave get similar work) */
LAYOUT_FN uint32_t pech_size_class(uint32_t rows)
{
	if (rows >= PECH_LARGE_ROWS)
		return 12;
	uint32_t c = 0;
	while ((2u << c) <= rows)
		++c;
	return c; /* floor(log2(rows)), 0..10 */
}
#define PECH_NCLASS 13u

/* Device workspace of one launch of m <= PECH_MAX_BATCH descriptors,
 * carved in this order (each array 256-byte aligned):
 *   cores    pech_core[slots]        sorted core descriptors per chunk
 *   lrs      u32[slots]              chunk-local exclusive row scan
 *   partials u32[PECH_MAX_CHUNKS]    rows per chunk
 *   nzs      u32[PECH_MAX_CHUNKS]    non-empty cores per chunk | PECH_NZ_UNIFORM
 *   deltas   i64[slots]              fused copy: destination - source per buffer
 * slots = nch * PECH_CHUNK, nch = ceil(m / PECH_CHUNK). */
struct pech_ws {
	struct pech_core *cores;
	uint32_t *lrs, *partials, *nzs;
	int64_t *deltas;
};

static inline size_t pech_ws_align(size_t x) { return (x + 255u) & ~(size_t)255u; }

static inline size_t pech_ws_bytes(uint32_t m)
{
	const size_t nch = (m + PECH_CHUNK - 1u) / PECH_CHUNK, slots = nch * PECH_CHUNK;
	return pech_ws_align(slots * sizeof(struct pech_core)) + pech_ws_align(slots * 4u) +
	       2u * pech_ws_align(PECH_MAX_CHUNKS * 4u) + pech_ws_align(slots * 8u);
}

static inline struct pech_ws pech_ws_carve(void *base, uint32_t m)
{
	const size_t nch = (m + PECH_CHUNK - 1u) / PECH_CHUNK, slots = nch * PECH_CHUNK;
	char *p = (char *)base;
	struct pech_ws w;
	w.cores = (struct pech_core *)p;
	p += pech_ws_align(slots * sizeof(struct pech_core));
	w.lrs = (uint32_t *)p;
	p += pech_ws_align(slots * 4u);
	w.partials = (uint32_t *)p;
	p += pech_ws_align(PECH_MAX_CHUNKS * 4u);
	w.nzs = (uint32_t *)p;
	p += pech_ws_align(PECH_MAX_CHUNKS * 4u);
	w.deltas = (int64_t *)p;
	return w;
}

#endif /* PECH_CRC32C_LAYOUT_H */
