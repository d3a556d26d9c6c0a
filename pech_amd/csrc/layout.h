/*
 * layout.h -- geometry shared by the host library and the gfx950 kernels.
 *
 * Split of one buffer D = (addr, len, seed) (v0.16):
 *   core c = [addr, ce)    ce = align16_down(addr + len)   <- main kernel
 *   tail t = [ce, addr + len)                (< 16 bytes)  <- plan kernel
 *   crc32c(seed, D) = x^(8|t|) * R(0, c) ^ R(0, t) ^ x^(8 len) * seed
 * The core is viewed on the 128-byte line grid: ROWS are the lines holding
 * it, row 0 at vbase = align128_down(addr), so every row load is one whole
 * HBM line.  One 8-lane GROUP of a wave walks rows of one buffer; lane g8 of
 * the group holds 16-byte piece g8 of every row as four 4-byte register
 * "streams".  The rows' bytes outside the core are read as zeros:
 *   lb = addr - vbase leading bytes of row 0 -- pieces below lb/16 wholly,
 *        the first lb%16 bytes of piece lb/16: leading zeros do not change
 *        R(0, .) (gf2.h), so a head costs nothing;
 *   zt whole trailing pieces of the last row past ce: trailing zeros
 *        multiply R by x^(128 zt), which the last run's final shift undoes
 *        (x^(8|t| - 128 zt), inverse powers when negative).
 * A buffer with no core (it lies inside one aligned 16-byte block) is
 * checksummed entirely by the plan kernel.  The plan kernel reads one block
 * per buffer with an unaligned end (its tail) and no other payload byte.
 * (Until v0.15 it also checksummed the < 16-byte head from a second block,
 * with a GF(2) shift of up to six 32-step multiplies: 13.6 us of plan and 5 %
 * more HBM traffic on unaligned 4,100-byte buffers.  Until v0.12 rows were
 * right-aligned to the core end instead of the line grid: +15 % traffic.)
 * The fused copy stores only whole pieces in the main kernel; its plan
 * kernel copies the bytes of a partial first piece and of the tail.
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
#ifndef PECH_IL_COPY
#define PECH_IL_COPY 1            /* fused copy's interleaved mode (profiles/r03/ab_copy_interleaved.txt) */
#endif
#ifndef PECH_EARLY_FILL_ROWS
#define PECH_EARLY_FILL_ROWS 4096u /* CRC kernel: tables published before the start search up to this many rows per workgroup */
#endif
#ifndef PECH_IL_CRC
#define PECH_IL_CRC 0             /* the same for the CRC-only kernel (A/B: reads gained nothing in the probe) */
#endif
#ifndef PECH_IL_MIN_ROWS
#define PECH_IL_MIN_ROWS 1024u    /* fused copy: uniform batches of buffers this large walk interleaved rows */
#endif
#ifndef PECH_IL_GROUPS
#define PECH_IL_GROUPS 128u       /* lane groups of a main-kernel workgroup (8 x waves): the interleave stride */
#endif
#ifndef PECH_POOL_MIN_SHARE
#define PECH_POOL_MIN_SHARE 1024u /* uniform batches pool only shares of at least this many rows */
#endif
#ifndef PECH_POOL_ROWS
#define PECH_POOL_ROWS 1536u      /* uniform batches: at most this many of a wave's rows are pooled */
#endif
#define PECH_NZ_UNIFORM 0x80000000u /* nzs[] flag: every buffer of the chunk has a core of the same rows */
#define PECH_NZ_MASK 0x7FFu         /* nzs[] bits 0-10: non-empty cores of the chunk */
#define PECH_NS_SHIFT 11u           /* nzs[] bits 11-21: of them, cores below PECH_SPLIT_ROWS (sorted first) */
#ifndef PECH_FLAT_MAX
#define PECH_FLAT_MAX 256u        /* device batches of up to this many buffers: one launch, no plan kernel */
#endif
#define PECH_FLATG_MAX 4096u      /* ... and up to this many: one launch of pech_crc32c_flatg (descriptors read in place) */
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
#define PECH_C_TAB16K 5888u /* A_16384 byte tables (fused copy, interleaved rows) */
#define PECH_C_ROWPOW 6912u /* x^(8*128*k), k < PECH_ROWPOW_N (run-end shifts by whole rows, global) */
#define PECH_ROWPOW_BITS 18u
#define PECH_ROWPOW_N (1u << PECH_ROWPOW_BITS) /* 1 MiB: shifts of up to 32 MiB in one table read */
#define PECH_C_WORDS (PECH_C_ROWPOW + PECH_ROWPOW_N)

/* device batch descriptor (matches struct crc32c_desc in include/) */
struct pech_desc {
	uint64_t addr;
	uint32_t len;
	uint32_t seed;
};

/* per-buffer core descriptor written by the plan kernel, in row-space order */
struct pech_core {
	uint64_t addr;  /* first byte of the buffer (and core); row 0 at addr & ~127 */
	uint32_t rows;  /* lines holding the core (0: none, done by the plan)     */
	uint32_t meta;  /* orig (bits 0-19) | zt (20-22) | tail (23-26)          */
};

#define PECH_META(orig, zt, t) ((orig) | ((uint32_t)(zt) << 20) | ((uint32_t)(t) << 23))
#define PECH_META_ORIG(m) ((m) & 0xFFFFFu)
#define PECH_META_ZT(m) (((m) >> 20) & 7u)
#define PECH_META_TAIL(m) (((m) >> 23) & 15u)

#ifdef __HIPCC__
#define LAYOUT_FN __host__ __device__ inline
#else
#define LAYOUT_FN static inline
#endif

/* rows (128-byte lines) holding the core [addr, align16_down(addr + len))
 * of buffer (addr, len); 0 if it has none */
LAYOUT_FN uint32_t pech_core_rows(uint64_t addr, uint32_t len)
{
	const uint64_t ce = (addr + len) & ~(uint64_t)15;
	return ce > addr ? (uint32_t)(((addr & 127u) + (ce - addr) + 127u) >> 7) : 0u;
}

/* whole 16-byte pieces of the core's last row past its end (0..7) */
LAYOUT_FN uint32_t pech_core_zt(uint64_t addr, uint32_t len, uint32_t rows)
{
	const uint64_t ce = (addr + len) & ~(uint64_t)15;
	return (uint32_t)(((uint64_t)rows * 128u - (addr & 127u) - (ce - addr)) >> 4);
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
 *   nzs      u32[PECH_MAX_CHUNKS]    non-empty cores per chunk | small ones << 11 | PECH_NZ_UNIFORM
 *   deltas   i64[slots]              fused copy: destination - source per buffer
 * slots = nch * PECH_CHUNK, nch = ceil(m / PECH_CHUNK).
 * A flat launch (m <= PECH_FLAT_MAX, no plan kernel) uses only the first
 * PECH_FLAT_WS_BYTES bytes, three u64 words (crc32c_kernels.hip,
 * pech_crc32c_flat): [0] the claim/publication word of out[]'s
 * initialisation (tag << 1 | done), [1] (low half) the count of workgroups
 * done before an async slot's results are published, [2] the tag of a launch
 * one of whose waves gave up waiting for out[] (its results are void). */
struct pech_ws {
	struct pech_core *cores;
	uint32_t *lrs, *partials, *nzs;
	int64_t *deltas;
};

#define PECH_FLAT_WS_BYTES 24u

/* A flat launch's status word (hstat, coherent pinned host memory, read by
 * the library after the launch has completed): PECH_FLAT_PUB(tag) once an
 * async slot's results are stored in its host array, PECH_FLAT_ERR(tag) when
 * a wave's wait for out[]'s initialisation timed out (the results are void);
 * anything else is an earlier launch's word.  Tags are below 2^62. */
#define PECH_FLAT_PUB(tag) (((uint64_t)(tag) << 2) | 1u)
#define PECH_FLAT_ERR(tag) (((uint64_t)(tag) << 2) | 2u)
/* test library only (crc32c_test_inject): the kernel's fault bits */
#define PECH_FLAT_T_TIMEOUT 1u /* every wave that waits for out[] times out at once */
#define PECH_FLAT_T_NOPUB 2u   /* the async slot's publication is skipped */
/* ... and the library's mode bit: the batch is read from pinned host memory
 * (an async zero-copy slot): uniform batches of large buffers walk interleaved
 * rows, the access shape that reads the host link at the copy engines' rate */
#define PECH_FLAT_F_IL 4u

static inline size_t pech_ws_align(size_t x) { return (x + 255u) & ~(size_t)255u; }

static inline size_t pech_ws_bytes(uint32_t m)
{
	const size_t nch = (m + PECH_CHUNK - 1u) / PECH_CHUNK, slots = nch * PECH_CHUNK;
	return pech_ws_align(slots * sizeof(struct pech_core)) + pech_ws_align(slots * 4u) +
	       2u * pech_ws_align(PECH_MAX_CHUNKS * 4u) + pech_ws_align(slots * 8u);
}

#if defined(__cplusplus) && __cplusplus >= 201103L
static_assert(PECH_FLAT_WS_BYTES <= 256u, "the flat words fit the first aligned array of any workspace");
#endif

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
