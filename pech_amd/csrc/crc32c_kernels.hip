// crc32c_kernels.hip -- gfx950 (CDNA4) kernels for batched CRC32C.
//
// For every descriptor (addr, len, seed) of a batch, computes exactly the
// reference's crc32c(seed, addr, len) (/root/reference/include/crc32c.h:88-96)
// over device-resident bytes.  Two launches per batch on the caller's stream:
//
//  pech_crc32c_plan  one 1024-thread workgroup per chunk of 1024 buffers:
//      splits each buffer into head / core / tail (layout.h), checksums the
//      <16-byte head and tail and the seed term itself (byte loop on the
//      reference table + GF(2) shifts) and writes that partial result to out[],
//      orders the chunk's buffers by size class (LDS counting sort) and writes
//      core descriptors + the chunk-local exclusive scan of core rows.
//
//  pech_crc32c_main  persistent, one 1024-thread workgroup per CU (the LDS
//      tables take 144 KiB).  Each wave owns a contiguous range of the batch's
//      row space and walks it in "steps"; a step gives each of the wave's 8
//      lane-groups a run of rows of one buffer -- eight neighbouring buffers
//      (small ones), or eight slices of one large buffer.  Per row and lane:
//      one 16-byte load of its piece (rows = 128-byte lines, fully coalesced
//      per group), then for its 4 word streams  s <- A_128(s) ^ w, where
//      A_128 ("advance 128 zero bytes") is 4 byte-indexed table lookups.  The
//      A_128 tables sit in LDS once per bank (32 copies), so lane l (mod 32)
//      only ever reads bank l: conflict-free whatever the data; the byte ->
//      LDS address step is ONE v_perm_b32.  Loads run PECH_U rows ahead with
//      unconditional (clamped) addresses so waits are counted, not drained.
//      At a run's end the 32 stream registers of a group are folded (A_4, then
//      an A_16/A_32/A_64 butterfly over the 8 lanes), shifted to the buffer's
//      end (x^(8m), power tables) and xor-ed atomically into out[].
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf2.h"
#include "layout.h"

#ifndef PECH_U
#define PECH_U 8 // rows in flight per lane
#endif
#ifndef PECH_U_DCOPY
#define PECH_U_DCOPY 8 // rows per block, direct fused copy (block discipline; 12 spills there)
#endif
#ifndef PECH_U_COPY
#define PECH_U_COPY 12 // rows per block, fused-copy variant (block discipline, 128 VGPRs)
#endif
#ifndef PECH_SPLIT_MIN
#define PECH_SPLIT_MIN 8u // rows of a large buffer a step splits over the 8 groups (plan_step; >= 8: a row each)
#endif
static_assert(PECH_SPLIT_MIN >= 8u, "every slice of a split step needs a row");
#ifndef PECH_DEAL_BLOCKS
#define PECH_DEAL_BLOCKS 32u // small launches: a workgroup's live shares lie this many apart (wave_share)
#endif
#ifndef PECH_LIVE_WAVES
#define PECH_LIVE_WAVES 4u // small launches: the live waves per CU wave_share aims at
#endif
#ifndef PECH_MAIN_WAVES
#define PECH_MAIN_WAVES 16 // waves per main-kernel workgroup (one workgroup per CU)
#endif
#define PECH_MAIN_THREADS (64u * PECH_MAIN_WAVES)
// Diagnostic switches that change results exist only with PECH_DIAG (A/B
// builds, tools/build_ab.sh): a product build that sees one fails here.
#if (defined(PECH_AB_NOLDS) || defined(PECH_AB_NOLOAD) || defined(PECH_AB_NOATOMIC) || defined(PECH_AB_NOSHIFT)) && !defined(PECH_DIAG)
#error "PECH_AB_NOLDS / PECH_AB_NOLOAD / PECH_AB_NOATOMIC / PECH_AB_NOSHIFT produce wrong CRCs: diagnostic builds must also define PECH_DIAG"
#endif

// Split-step results are XORed into a workgroup table in LDS and reach out[]
// with one global atomic per (workgroup, buffer), issued by the workgroup's
// last wave to finish: the
// waves of a 4 MiB buffer (16 per workgroup, 64 in a 256 MiB launch) then no
// longer queue on one address (measured: 4 MiB class 52.0 -> 50.0 us).
#define PECH_DEFER_SLOTS 64u
#define PECH_DEFER_EMPTY 0xFFFFFFFFu

// ---- LDS map of the main kernel (bytes) ---------------------------------
#define L_REP 0u                 // 128 KiB: A_128, 32 bank copies
#define L_TAB4 131072u           // 4 KiB each, single copy
#define L_TAB16 (L_TAB4 + 4096u)
#define L_TAB32 (L_TAB16 + 4096u)
#define L_TAB64 (L_TAB32 + 4096u)
#define L_POWB (L_TAB64 + 4096u) // 1536 B
#define L_NZ (L_POWB + 1536u)    // 4 KiB: chunk non-empty counts
#define L_DEFER (L_NZ + 4096u)   // 512 B: split-step results, keyed by output slot
#define L_DEFER_DONE (L_DEFER + 8u * PECH_DEFER_SLOTS) // waves of the workgroup done
#define L_XINV (L_DEFER_DONE + 16u) // 512 B: x^(-8k), k < 128
#define L_POOL (L_XINV + 512u)   // 16 B: the workgroup's next pooled item (uniform batches)
#define L_BYTES (L_POOL + 16u)
#define L_SCAN L_BYTES           // 256 B: the large flat prologue's per-wave totals and flags (prologue_flatg)
#define L_BYTES_G (L_SCAN + 256u) // pech_crc32c_flatg only (the other kernels keep their LDS footprint)
static_assert(L_BYTES_G <= 160u * 1024u, "flatg LDS budget");
static_assert(L_BYTES <= 160u * 1024u, "main kernel LDS over 160 KiB");

static_assert(L_POWB - L_TAB4 == 4u * (PECH_C_POWB - PECH_C_TAB4), "LDS/consts layout mismatch");
static_assert(L_BYTES <= 160u * 1024u, "LDS budget");

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) const uint8_t g_u8;

// ---- helpers --------------------------------------------------------------
__device__ __forceinline__ uint32_t uni(uint32_t v)
{
	return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ uint64_t uni64(uint64_t v)
{
	return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

// Inclusive add-scan over the 64 lanes by DPP moves (no LDS round trips, which
// is what __shfl_up compiles to: ds_bpermute): Hillis-Steele inside each
// 16-lane row (row_shr 1, 2, 4, 8 with zero fill), then row 15's sum into
// rows 1 and 3 (row_bcast:15) and lane 31's into rows 2 and 3 (row_bcast:31).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x)
{
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
	return x;
}

// The last lane with a nonzero `c`, for lane values that are a monotone
// prefix (every lane before it nonzero): a ballot instead of a reduction.
__device__ __forceinline__ uint32_t last_lane_with(uint32_t c)
{
	const uint64_t m = __ballot(c != 0u);
	return 63u - (uint32_t)__builtin_clzll(m | 1ull);
}

__device__ __forceinline__ uint32_t lane_value(uint32_t v, uint32_t lane)
{
	return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// NT-thread exclusive scan; scratch = NT/64 LDS words
template <uint32_t NT = PECH_WG_THREADS>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *scratch, uint32_t *total)
{
	const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
	const uint32_t x = wave_incl_scan(v);
	if (lane == 63u)
		scratch[wave] = x;
	__syncthreads();
	uint32_t off = 0, tot = 0;
#pragma unroll
	for (uint32_t w = 0; w < NT / 64u; ++w) {
		const uint32_t t = scratch[w];
		off += (w < wave) ? t : 0u;
		tot += t;
	}
	*total = tot;
	__syncthreads();
	return off + x - v;
}

__device__ __forceinline__ uint32_t lds_u32(const uint32_t *lds, uint32_t byte_off)
{
	return *(const uint32_t *)((const char *)lds + byte_off);
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// A_128(s) ^ w from the bank-replicated tables.  lreg = (lane&31)*4 | 1<<16.
// Table k, entry e, bank copy c lives at (k>>1)*64K + e*256 + (k&1)*128 + 4c.
// Five-operand XOR as two bitop3s.
__device__ __forceinline__ uint32_t adv128(const uint32_t *lds, uint32_t s, uint32_t lreg, uint32_t w)
{
#ifdef PECH_AB_NOLDS // diagnostic build only: no table lookups (wrong CRCs)
	return (s << 1) ^ (s >> 3) ^ lreg ^ w;
#endif
	const uint32_t a0 = __builtin_amdgcn_perm(s, lreg, 0x0C0C0400u);
	const uint32_t a1 = __builtin_amdgcn_perm(s, lreg, 0x0C0C0500u);
	const uint32_t a2 = __builtin_amdgcn_perm(s, lreg, 0x0C020600u);
	const uint32_t a3 = __builtin_amdgcn_perm(s, lreg, 0x0C020700u);
	return xor3(xor3(lds_u32(lds, a0), lds_u32(lds, a1 + 128u), w), lds_u32(lds, a2), lds_u32(lds, a3 + 128u));
}

// single-copy byte tables (4 x 256 words at byte offset `tab`)
__device__ __forceinline__ uint32_t adv_tab(const uint32_t *lds, uint32_t tab, uint32_t v)
{
	const uint32_t *t = lds + (tab >> 2);
	return xor3(t[v & 0xFFu], t[256u + ((v >> 8) & 0xFFu)], t[512u + ((v >> 16) & 0xFFu)] ^ t[768u + (v >> 24)]);
}

// a * b mod P on the GPU, five VALU ops per bit of a: the bit of a as a
// mask (v_bfe_i32), p ^= b & mask and b = b*x as one v_bitop3 each (0x78:
// S0 ^ (S1 & S2)), with the shift and the carry mask of b.  The generic loop
// of gf2.h compiles to seven; the run-end shifts are ~1 us of every split
// step (profiles/r04/ab_shift_early.txt).
__device__ __forceinline__ uint32_t gf2_mulmod_dev(uint32_t a, uint32_t b)
{
#ifdef PECH_MULMOD_GENERIC // A/B: the gf2.h loop
	return gf2_mulmod(a, b);
#endif
	uint32_t p = 0;
#pragma unroll
	for (int i = 31; i >= 0; --i) {
		const uint32_t ma = (uint32_t)((int32_t)(a << (31 - i)) >> 31);
		p = __builtin_amdgcn_bitop3_b32(p, b, ma, 0x78);
		const uint32_t mb = (uint32_t)((int32_t)(b << 31) >> 31);
		b = __builtin_amdgcn_bitop3_b32(b >> 1, mb, CRC32C_POLY_REFLECTED, 0x78);
	}
	return p;
}

// v * x^(8m) mod P with the 64-ary power table POWB[i][j] = x^(8 j 64^i)
__device__ __forceinline__ uint32_t shift_bytes(const uint32_t *powb, uint64_t m, uint32_t v)
{
#ifdef PECH_AB_NOSHIFT // diagnostic build only: the run-end shifts skipped (wrong CRCs)
	if (m != 0x9E3779B9u)
		return v;
#endif
#pragma unroll
	for (uint32_t i = 0; i < 6; ++i) {
		const uint32_t d = (uint32_t)(m >> (6u * i)) & 63u;
		if (d)
			v = gf2_mulmod_dev(powb[64u * i + d], v);
	}
	return v;
}

// ---- plan kernel ----------------------------------------------------------
// byte-wise reference update (include/crc32c.h:92-93) on the LDS table, over
// bytes [lo, hi) of a 16-byte block held in registers (0 <= lo <= hi <= 16)
__device__ __forceinline__ uint32_t crc_block(const uint32_t *t1, uint32_t crc, u32x4 v, uint32_t lo, uint32_t hi)
{
#pragma unroll
	for (uint32_t k = 0; k < 16; ++k) {
		const uint32_t w = k < 4 ? v.x : (k < 8 ? v.y : (k < 12 ? v.z : v.w));
		const uint32_t byte = (w >> (8u * (k & 3u))) & 0xFFu;
		if (k >= lo && k < hi)
			crc = t1[(crc ^ byte) & 0xFFu] ^ (crc >> 8);
	}
	return crc;
}

// fused-copy variant: bytes [lo, hi) of the block whose first byte is at
// `dst` in the destination (a partial first piece, the tail, or a buffer
// without a core; the main kernel stores only whole pieces)
__device__ __forceinline__ void copy_block(u32x4 v, uint32_t lo, uint32_t hi, uint64_t dst)
{
	__attribute__((address_space(1))) uint8_t *d = (__attribute__((address_space(1))) uint8_t *)dst;
#pragma unroll
	for (uint32_t k = 0; k < 16; ++k) {
		const uint32_t w = k < 4 ? v.x : (k < 8 ? v.y : (k < 12 ? v.z : v.w));
		if (k >= lo && k < hi)
			d[k] = (uint8_t)(w >> (8u * (k & 3u)));
	}
}

// Per buffer: its row-space descriptor (layout.h) and the part of its CRC
// outside the core -- the tail R(0, t) (one block load, only for an
// unaligned end), the seed term x^(8 len) seed (0 for the messenger's zero
// seeds), or the whole CRC of a buffer without a core.  No GF(2) shift of
// data: a head is masked in the main kernel.  COPY: also dst[b] <- the
// bytes of a partial first piece (a second block load) and of the tail,
// and dl = dst - src for the main kernel.
template <bool COPY>
__device__ __forceinline__ void plan_body(const pech_desc *__restrict__ descs, uint32_t n, pech_core *__restrict__ cores,
					  uint32_t *__restrict__ lrs, uint32_t *__restrict__ partials,
					  uint32_t *__restrict__ nzs, const uint32_t *__restrict__ consts,
					  uint32_t *__restrict__ out, const uint64_t *__restrict__ dsts,
					  int64_t *__restrict__ deltas)
{
	__shared__ uint32_t t1[256];
	__shared__ uint32_t powb[384];
	__shared__ uint32_t wcnt[PECH_NCLASS * PECH_WAVES_PER_WG]; // per (class, wave): buffers, then their offset
	__shared__ uint32_t rows_at[PECH_CHUNK];
	__shared__ uint32_t scratch[PECH_WAVES_PER_WG];
	__shared__ uint32_t rmax; // largest core of the chunk (uniformity flag)
	const uint32_t tid = threadIdx.x;
#ifdef PECH_KARGS_AT_ENTRY
	asm volatile("" ::"s"(descs), "s"(n), "s"(cores), "s"(lrs), "s"(partials), "s"(nzs), "s"(consts), "s"(out), "s"(dsts),
		     "s"(deltas)); // one kernarg round (main_body)
#endif
	const uint32_t b = blockIdx.x * PECH_CHUNK + tid;
	// loads unconditional (clamped indices) so they are in flight together:
	// loads under exec-masked branches each got a vmcnt(0) at the join
	pech_desc d = descs[min(b, n - 1u)];
	const uint32_t tv1 = consts[PECH_C_TAB1 + (tid & 255u)];
	const uint32_t tvp = consts[PECH_C_POWB + min(tid, 383u)];
	if (b >= n)
		d.len = 0;
	// The tail lies in the aligned 16-byte block at ce (an aligned block never
	// crosses a page, so it is readable whenever one of its bytes is).  A
	// buffer with nothing to read there (an aligned end, an empty buffer
	// whose address may be anything) loads its own descriptor instead.
	const uint64_t safe = (uint64_t)(descs + min(b, n - 1u));
	const uint64_t end = d.addr + d.len, ce = end & ~(uint64_t)15, a0 = d.addr & ~(uint64_t)15;
	const bool needT = d.len != 0 && (end & 15u) != 0;
	// (skipping this round trip in waves without an unaligned end measured
	// neutral on c4-64k / C4 steps: profiles/r06/ab_copy_plan.txt)
	const u32x4 vT = *(g_u32x4 *)(needT ? ce : safe);
	u32x4 vA = (u32x4)(0u);
	const bool hp = COPY && d.len != 0 && (d.addr & 15u) != 0 && a0 != ce; // partial first piece of a core
	if (COPY)
		vA = *(g_u32x4 *)(hp ? a0 : safe);
	if (tid < 256)
		t1[tid] = tv1;
	if (tid < 384)
		powb[tid] = tvp;
	rows_at[tid] = 0;
	if (tid == 0)
		rmax = 0;
	__syncthreads();

	uint32_t rows = 0, cls = 0;
	pech_core core = {0, 0, 0};
	if (b < n) {
		rows = pech_core_rows(d.addr, d.len);
		const uint32_t t = (uint32_t)(end - ce);
		int64_t dl = 0;
		if (COPY) {
			dl = (int64_t)(dsts[b] - d.addr);
			deltas[b] = dl;
		}
		uint32_t res;
		if (rows == 0) {
			// no core: the buffer lies inside the block at ce (<= 15 bytes)
			res = d.len ? crc_block(t1, d.seed, vT, (uint32_t)(d.addr - ce), t) : d.seed;
			if (COPY && d.len)
				copy_block(vT, (uint32_t)(d.addr - ce), t, ce + dl);
		} else {
			// seed term R(s, D) = x^(8|D|) s ^ R(0, D), and the tail R(0, t)
			res = d.seed ? shift_bytes(powb, d.len, d.seed) : 0u;
			if (t)
				res ^= crc_block(t1, 0, vT, 0u, t);
			if (COPY) {
				if (hp)
					copy_block(vA, (uint32_t)(d.addr - a0), 16u, a0 + dl);
				if (t)
					copy_block(vT, 0u, t, ce + dl);
			}
			core.addr = d.addr;
			core.rows = rows;
			core.meta = PECH_META(b, pech_core_zt(d.addr, d.len, rows), t);
			cls = pech_size_class(rows);
		}
		out[b] = res;
	}
	{ // the chunk's largest core: a wave max by lane swaps, then one LDS atomic per wave
		uint32_t m = rows;
#pragma unroll
		for (uint32_t off = 32; off; off >>= 1)
			m = max(m, (uint32_t)__shfl_xor((int)m, (int)off));
		if ((tid & 63u) == 0 && m)
			atomicMax(&rmax, m);
	}
	// Order the chunk's buffers by size class, STABLY (descriptor order inside
	// a class): per-wave ballots, then one scan over (class, wave).
	const uint32_t lane = tid & 63u, wave = tid >> 6;
	uint32_t rank = 0;
#pragma unroll
	for (uint32_t c = 0; c < PECH_NCLASS; ++c) {
		const uint64_t m = __ballot(rows != 0 && cls == c);
		if (rows != 0 && cls == c)
			rank = (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
		if (lane == 0)
			wcnt[c * PECH_WAVES_PER_WG + wave] = (uint32_t)__builtin_popcountll(m);
	}
	__syncthreads();
	uint32_t nz;
	{
		const uint32_t v = tid < PECH_NCLASS * PECH_WAVES_PER_WG ? wcnt[tid] : 0u;
		const uint32_t ex = block_excl_scan(v, scratch, &nz); // (barriers inside)
		if (tid < PECH_NCLASS * PECH_WAVES_PER_WG)
			wcnt[tid] = ex;
		__syncthreads();
		if (rows) {
			// Inside every full block of 16 same-class buffers below the split
			// size, ranks 0,2,..,14 take positions 0..7 and ranks 1,3,..,15
			// positions 8..15.  The main kernel hands 8 consecutive positions
			// to the 8 lane groups of a step, so group g reads buffer 2g in one
			// step and 2g+1 in the next: for buffers laid out back to back
			// (arrays of pages) every group walks one contiguous 2-buffer range
			// instead of 8 groups jumping to fresh 4 KiB blocks each step --
			// measured 7-8% faster for 4 KiB buffers on the bare read stream
			// (tools/sched_probe.hip "column steps" vs "static steps").
			const uint32_t c0 = wcnt[cls * PECH_WAVES_PER_WG];
			const uint32_t c1 = cls + 1u < PECH_NCLASS ? wcnt[(cls + 1u) * PECH_WAVES_PER_WG] : nz;
			uint32_t r = wcnt[cls * PECH_WAVES_PER_WG + wave] + rank - c0;
			if (rows < PECH_SPLIT_ROWS && (r | 15u) < c1 - c0)
				r = (r & ~15u) | ((r & 1u) << 3) | ((r >> 1) & 7u);
			const uint32_t pos = c0 + r;
			cores[blockIdx.x * PECH_CHUNK + pos] = core;
			rows_at[pos] = rows;
		}
	}
	__syncthreads();
	uint32_t total;
	const uint32_t ex = block_excl_scan(rows_at[tid], scratch, &total);
	lrs[blockIdx.x * PECH_CHUNK + tid] = ex;
	if (tid == 0) {
		partials[blockIdx.x] = total;
		// uniform chunk: every buffer has a core and all cores have the
		// largest one's rows (sum == count x max); the main kernel then
		// locates any row by division and pools its work (PECH_ITEM_ROWS)
		const uint32_t cnt = min(PECH_CHUNK, n - blockIdx.x * PECH_CHUNK);
		const bool uni = nz == cnt && (uint64_t)nz * rmax == (uint64_t)total && total != 0;
		// the small cores (< PECH_SPLIT_ROWS rows: classes 0-7) come first
		const uint32_t nsmall = wcnt[8u * PECH_WAVES_PER_WG];
		nzs[blockIdx.x] = nz | (nsmall << PECH_NS_SHIFT) | (uni ? PECH_NZ_UNIFORM : 0u);
	}
}

extern "C" __global__ __launch_bounds__(PECH_WG_THREADS) void pech_crc32c_plan(
	const pech_desc *__restrict__ descs, uint32_t n, pech_core *__restrict__ cores, uint32_t *__restrict__ lrs,
	uint32_t *__restrict__ partials, uint32_t *__restrict__ nzs, const uint32_t *__restrict__ consts,
	uint32_t *__restrict__ out)
{
	plan_body<false>(descs, n, cores, lrs, partials, nzs, consts, out, nullptr, nullptr);
}

extern "C" __global__ __launch_bounds__(PECH_WG_THREADS) void pech_crc32c_plan_copy(
	const pech_desc *__restrict__ descs, uint32_t n, pech_core *__restrict__ cores, uint32_t *__restrict__ lrs,
	uint32_t *__restrict__ partials, uint32_t *__restrict__ nzs, const uint32_t *__restrict__ consts,
	uint32_t *__restrict__ out, const uint64_t *__restrict__ dsts, int64_t *__restrict__ deltas)
{
	plan_body<true>(descs, n, cores, lrs, partials, nzs, consts, out, dsts, deltas);
}

// ---- single small buffer (the drop-in crc32c()) ---------------------------
// One workgroup, one launch: the buffer (<= PECH_SMALL_MAX bytes) is read in
// place from pinned host staging (zero-copy: no DMA, no plan kernel), 16 B
// per lane into LDS, then thread t runs the reference byte loop
// (include/crc32c.h:92-93) over its contiguous segment, shifts its register
// to the buffer end (x^(8m)) and the segments are XOR-reduced; the seed term
// is x^(8 len) * seed.  The result goes straight to pinned host memory.
#define PECH_SMALL_THREADS 1024u
static_assert(PECH_SMALL_MAX % 16u == 0u, "small path: whole 16-byte loads");
extern "C" __global__ __launch_bounds__(PECH_SMALL_THREADS) void pech_crc32c_small(
	const uint8_t *__restrict__ src, uint32_t len, uint32_t seed, const uint32_t *__restrict__ consts,
	uint32_t *__restrict__ out, uint32_t ticket)
{
	__shared__ __attribute__((aligned(16))) uint8_t data[PECH_SMALL_MAX];
	__shared__ uint32_t t1[256];
	__shared__ uint32_t powb[384];
	__shared__ uint32_t red[PECH_SMALL_THREADS / 64u];
	const uint32_t tid = threadIdx.x;
	if (tid < 256u)
		t1[tid] = consts[PECH_C_TAB1 + tid];
	if (tid < 384u)
		powb[tid] = consts[PECH_C_POWB + tid];
	// the staging buffer is 16-byte aligned and at least PECH_SMALL_MAX long:
	// whole 16-byte loads past len stay inside it and are never used
	constexpr uint32_t LPT = PECH_SMALL_MAX / 16u / PECH_SMALL_THREADS; // loads per thread, all in flight at once
	u32x4 w[LPT];
#pragma unroll
	for (uint32_t k = 0; k < LPT; ++k) {
		const uint32_t i = tid + k * PECH_SMALL_THREADS;
		if (i * 16u < len)
			w[k] = *(const g_u32x4 *)(src + 16u * i);
	}
#pragma unroll
	for (uint32_t k = 0; k < LPT; ++k) {
		const uint32_t i = tid + k * PECH_SMALL_THREADS;
		if (i * 16u < len)
			*(u32x4 *)(data + 16u * i) = w[k];
	}
	__syncthreads();
	// segments of whole 16-byte words, read as such (byte reads at a stride
	// of the segment length hit the same LDS banks from every lane)
	const uint32_t seg = ((len + PECH_SMALL_THREADS - 1u) / PECH_SMALL_THREADS + 15u) & ~15u;
	const uint32_t b0 = min(len, tid * seg), b1 = min(len, b0 + seg);
	uint32_t c = 0;
	for (uint32_t j = b0; j < b1; j += 16u) {
		const u32x4 q = *(const u32x4 *)(data + j);
		const uint32_t e = min(16u, b1 - j);
#pragma unroll
		for (uint32_t k = 0; k < 16u; ++k) {
			const uint32_t byte = (q[k >> 2] >> (8u * (k & 3u))) & 0xFFu;
			if (k < e)
				c = t1[(c ^ byte) & 0xFFu] ^ (c >> 8);
		}
	}
	uint32_t v = (b1 > b0 && len > b1) ? shift_bytes(powb, len - b1, c) : c;
	for (uint32_t d = 1; d < 64; d <<= 1)
		v ^= __shfl_xor(v, d);
	if ((tid & 63u) == 0)
		red[tid >> 6] = v;
	__syncthreads();
	if (tid == 0) {
		uint32_t r = seed ? shift_bytes(powb, len, seed) : 0u;
		for (uint32_t w = 0; w < PECH_SMALL_THREADS / 64u; ++w)
			r ^= red[w];
		// result, then the caller's ticket: the host polls out[1] (system scope)
		__builtin_nontemporal_store(r, out);
		__threadfence_system();
		__builtin_nontemporal_store(ticket, out + 1);
		__threadfence_system();
	}
}

// ---- main kernel ----------------------------------------------------------
#ifdef PECH_STAMPS // diagnostic build: per-wave entry/start/end s_memrealtime stamps
#define PECH_MAX_STAMPS 8192u
#define PECH_NSTAMP 12u // start, end, tag, entry, scan, find, plan, fill, 25/50/75% of the first step, loads issued
__device__ uint64_t pech_stamps[PECH_NSTAMP * PECH_MAX_STAMPS];
#define STAMP(v) const uint64_t v = __builtin_amdgcn_s_memrealtime()
extern "C" int pech_read_stamps(uint64_t *host, uint32_t n)
{
	return hipMemcpyFromSymbol(host, HIP_SYMBOL(pech_stamps), sizeof(uint64_t) * PECH_NSTAMP * n) == hipSuccess ? 0 : -1;
}
#else
#define STAMP(v)
#endif
// A step gives each 8-lane group of a wave one run of rows of one buffer.
// Per lane: `ad` = address of this lane's piece in the run's first row, `nl`
// rows to load (>= 1), `nu` rows to use (0 = idle group: its loads repeat
// another group's rows and its state is ignored), `zoff` != 0 = the first
// row's piece lies wholly before the buffer (row 0 is loaded from ad + zoff
// -- the first real piece -- and zeroed), `zh` = its first zh bytes lie
// before the buffer (zeroed), `zl` = the lane's piece of the run's last row
// lies past the core's end (a trailing virtual piece, zeroed), `m` = bytes
// from the run's end to the buffer's end (final shift; negative when the
// run ends in the core's last row and its zt trailing virtual pieces
// outnumber the tail bytes), `orig` = output slot.  Zeroed bytes are never
// stored by the fused copy.
// Uniform: T / nmin = max / min of nu over the active groups (T == 0: no
// step), and the wave's cursor after the step.
struct Step {
	uint64_t ad;
	uint32_t mp;  // rows after the run << 7 | zt << 4 | tail   (m = 128 rows + tail - 16 zt; mp_bits)
	uint32_t nl, nu;
	uint32_t oz;  // orig | (zoff / 16) << 20 | zh << 23 | zl << 27 | ra bit 25 << 29   (zoff <= 112, zh < 16)
	uint32_t T, nmin;
	uint32_t pos, lr, rem;
	uint64_t dad; // fused copy: destination of this lane's piece in row 0 (ad + dst - src)
#ifdef PECH_DEBUG_BOUNDS
	uint64_t blo, bhi; // core of the buffer this lane loads from
#endif
};

// The address is laundered through an empty asm: row 0 of a virtual piece is
// zeroed after its load, and without the barrier LLVM treats the load's
// address as "don't care" in that case and folds ad + zoff back to ad -- a
// read before the buffer (seen in the ISA; a GPU fault at allocation starts).
__device__ __forceinline__ uint64_t row_addr(uint64_t ad, uint32_t row, uint32_t zoff, uint32_t rs = PECH_ROW_BYTES)
{
	uint64_t a = ad + (uint64_t)row * rs + (row == 0 ? zoff : 0u);
	asm("" : "+v"(a));
	return a;
}

#ifdef PECH_DEBUG_BOUNDS
// debug build: every ring load is checked against the core [lo, hi) of the
// buffer being walked; a violation is printed and redirected to lo.
__device__ __forceinline__ u32x4 ld_piece(uint64_t a, uint64_t lo, uint64_t hi, uint32_t tag)
{
	if (a < lo || a + 16u > hi) {
		printf("PECH OOB tag %u blk %u tid %u addr %llx lo %llx hi %llx\n", tag, blockIdx.x, threadIdx.x,
		       (unsigned long long)a, (unsigned long long)lo, (unsigned long long)hi);
		a = lo;
	}
	return *(g_u32x4 *)a;
}
#define LD_PIECE(S, a, tag) ld_piece((a), (S).blo, (S).bhi, (tag))
#elif defined(PECH_AB_NOLOAD) // diagnostic build only: no HBM reads (wrong CRCs)
#define LD_PIECE(S, a, tag) ((u32x4)((uint32_t)(a)))
#else // payload bytes are read once: nontemporal (measured +8-10 % HBM rate)
#define LD_PIECE(S, a, tag) (__builtin_nontemporal_load((g_u32x4 *)(a)))
#endif

static_assert(PECH_MAIN_WAVES % 4 == 0 && PECH_MAIN_WAVES <= 16, "waves per workgroup: 4, 8, 12 or 16");
// the interleaved fused copy's row stride and the direct kernel's position
// stride are the workgroup's lane groups: one constant for both
static_assert(PECH_IL_GROUPS == PECH_GROUP_LANES * PECH_MAIN_WAVES, "PECH_IL_GROUPS = 8 groups x PECH_MAIN_WAVES");

// Step.oz bits of lane g8 when its run starts at the buffer's row 0 (first):
// lb leading bytes of the row lie before the buffer -- pieces below lb/16
// wholly (zoff redirect), lb%16 bytes of piece lb/16 (zh)
__device__ __forceinline__ uint32_t head_bits(bool first, uint32_t g8, uint32_t lb)
{
	const uint32_t vp = lb >> 4;
	if (!first)
		return 0u;
	return g8 < vp ? (vp - g8) << 20 : (g8 == vp ? (lb & 15u) << 23 : 0u);
}

// ... and when it ends the core (last): the last zt pieces of the row lie
// past it (trailing virtual pieces, zeroed)
__device__ __forceinline__ uint32_t tail_bits(bool last, uint32_t g8, uint32_t zt)
{
	return last && g8 >= 8u - zt ? 1u << 27 : 0u;
}

// Step.mp of a run with `ra` rows of its buffer after it: ra << 7 | zt << 4 |
// tail.  ra reaches 2^25 (a core of 2^25 + 1 rows: a buffer within 255 bytes
// of 4 GiB, whose first row is a run of its own), which wraps 32 bits after
// the shift, so bit 25 of ra goes to Step.oz bit 29 (ra_bit) -- ADVICE r3.
#define PECH_OZ_RA25 (1u << 29)
__device__ __forceinline__ uint32_t mp_bits(uint32_t ra, uint32_t meta)
{
	return (ra << 7) | (meta >> 16 & 0x70u) | PECH_META_TAIL(meta);
}
__device__ __forceinline__ uint32_t ra_bit(uint32_t ra) { return (ra >> 25 & 1u) << 29; }

// v with its bytes [0, kb) kept and [kb, 16) zeroed (0 <= kb <= 16)
__device__ __forceinline__ u32x4 keep_below(u32x4 v, uint32_t kb)
{
	u32x4 r;
#pragma unroll
	for (uint32_t j = 0; j < 4; ++j) {
		const uint32_t k = min(kb - min(kb, 4u * j), 4u);
		r[j] = v[j] & (k >= 4u ? 0xFFFFFFFFu : (1u << (8u * k)) - 1u);
	}
	return r;
}

// one descriptor per lane group (a step's speculative descriptors)
__device__ __forceinline__ pech_core load_spec(const pech_core *__restrict__ cores, uint32_t p)
{
	const u32x4 v = ((const u32x4 *)cores)[p];
	pech_core c;
	c.addr = ((uint64_t)v.y << 32) | v.x;
	c.rows = v.z;
	c.meta = v.w;
	return c;
}

// ---- flat batches (pech_crc32c_flat): n <= PECH_FLAT_MAX, no plan kernel ----
// Every wave reads the batch's descriptors itself and keeps them in LDS as
// {addr, rows, meta} per position, in descriptor order (L_FLAT, the chunk
// table's space: a flat launch has no chunks).  rows are the 128-byte lines
// holding ALL of the buffer's bytes, as in the direct kernel: no tail block
// and no plan kernel.  meta = position | T << 20, with T (0..127) the zero
// bytes after the buffer in its last line.  A run that ends its buffer keeps
// kb bytes of each lane's piece of that line (Step.oz bits 12-16; the
// position then has 12 bits) and is multiplied by x^(-8 T) at its end:
// m = 128 ra - T.
#define L_FLAT L_NZ
#define PECH_FLAT_T(meta) (((meta) >> 20) & 127u)
#define PECH_FLAT_KB_SHIFT 12u
static_assert(PECH_FLAT_MAX * 16u <= 4096u && PECH_FLAT_MAX <= 4096u, "flat table: 16 B per position in L_NZ, 12-bit positions");

__device__ __forceinline__ pech_core flat_core(const uint32_t *lds, uint32_t p)
{
	const u32x4 v = *(const u32x4 *)(lds + L_FLAT / 4u + 4u * p);
	pech_core c;
	c.addr = ((uint64_t)v.y << 32) | v.x;
	c.rows = v.z;
	c.meta = v.w;
	return c;
}

// Large flat batches (pech_crc32c_flatg, PECH_FLAT_MAX < n <= PECH_FLATG_MAX):
// no LDS table -- 16 B per position would not fit beside the A_128 tables --
// so a step's descriptors come from the caller's array itself (`g`: the
// crc32c_desc array, L2-resident after the prologue read it), each turned
// into the LDS table's {addr, rows, meta}: a split step's one descriptor by a
// scalar load at its wave-uniform position (lgkmcnt: the ring's vector loads
// are never drained for it); a small-buffer step's eight, one per lane group,
// from a vector prefetch issued a step ahead (plan_step's PRE), or on a miss
// by a vector load (main_body).
__device__ __forceinline__ pech_core flatg_conv(u32x4 v, uint32_t p) // v: {addr lo, addr hi, len, seed}
{
	pech_core c;
	c.addr = ((uint64_t)v.y << 32) | v.x;
	const uint32_t lb = v.x & (PECH_ROW_BYTES - 1u), len = v.z;
	c.rows = len ? (uint32_t)(((uint64_t)lb + len + PECH_ROW_BYTES - 1u) >> 7) : 0u;
	c.meta = p | (c.rows ? c.rows * PECH_ROW_BYTES - lb - len : 0u) << 20; // (T mod 2^32: exact, < 128)
	return c;
}
// A descriptor loaded by a vector load and read only in part (flatg_conv
// ignores the seed, the prologue the address's high word): its unread
// registers were free for reuse while the load was in flight, and the
// reuse waited for the load with a vmcnt(0) -- draining the tables' loads
// at entry and the ring at a step's end.  Marking the whole vector read
// where it is consumed keeps its registers until then.
__device__ __forceinline__ void keep_whole(const u32x4 &v)
{
	asm volatile("" ::"v"(v));
}
__device__ __forceinline__ pech_core flatg_core(const pech_core *__restrict__ g, uint32_t p)
{
	return flatg_conv(((const u32x4 *)g)[uni(p)], p);
}

// Step.oz bits of lane g8 for a run that ends its buffer (last): the zl flag
// and the bytes kb of the lane's last-line piece that are the buffer's
template <bool FLAT>
__device__ __forceinline__ uint32_t tail_of(bool last, uint32_t g8, uint32_t meta)
{
	if (!FLAT)
		return tail_bits(last, g8, PECH_META_ZT(meta));
	const uint32_t e = 128u - PECH_FLAT_T(meta), lo = 16u * g8;
	const uint32_t kb = e > lo ? min(e - lo, 16u) : 0u;
	return last ? (1u << 27) | (kb << PECH_FLAT_KB_SHIFT) : 0u;
}

template <bool FLAT>
__device__ __forceinline__ uint32_t mp_of(uint32_t ra, uint32_t meta)
{
	return FLAT ? (ra << 7) | PECH_FLAT_T(meta) : mp_bits(ra, meta);
}

// Work out the wave's next step from its cursor (pos, lr, rem).  COPY: also
// the destination offset of each group's buffer (deltas[orig], scalar loads).
// PRE: `spec` holds cores[ppos + grp] (loaded at kernel entry); a step that
// starts at ppos takes its descriptors from it instead of loading them.
// grid: static shares, whose small-buffer steps lie on a grid of 8 positions.
// FLAT: the descriptors come from the wave's LDS table (flat_core) for
// positions < nflat, empty buffers included (skipped here).
// FLATG: the same from the caller's descriptors (`cores` is then the
// crc32c_desc array; flatg_core); with PRE, `spec` holds position ppos + grp
// already converted (flatg_conv).
template <bool COPY, bool PRE = false, bool FLAT = false, bool FLATG = false>
__device__ __forceinline__ Step plan_step(const pech_core *__restrict__ cores, const int64_t *__restrict__ deltas,
					  const uint32_t *lds, uint32_t pos, uint32_t lr, uint32_t rem, uint32_t lane,
					  uint32_t g8, uint32_t grp, bool grid, const pech_core &spec = pech_core{},
					  uint32_t ppos = 0, uint32_t nflat = 0)
{
	static_assert(!(FLAT && (COPY || (PRE && !FLATG))), "flat batches: CRC only, descriptors from LDS (flatg: or speculated)");
	Step S;
	int64_t dl = 0;
	S.T = 0;
	S.nmin = 0;
	S.ad = 0;
	S.mp = 0;
	S.nl = 1;
	S.nu = 0;
	S.oz = 0;
#ifdef PECH_DEBUG_BOUNDS
	S.blo = S.bhi = 0;
#endif
	for (;;) {
		if (rem == 0)
			break;
		uint32_t c, nzc;
		if (FLAT) {
			if (pos >= nflat) { // (never while rows remain)
#ifdef PECH_DEBUG_BOUNDS
				printf("PECH OOB flat cursor pos %u n %u rem %u\n", pos, nflat, rem);
#endif
				break;
			}
			c = 0;
			nzc = nflat;
		} else {
			c = pos >> 10;
			nzc = uni(lds[L_NZ / 4u + c]);
			if ((pos & 1023u) >= nzc) {
				pos = (c + 1u) << 10;
				continue;
			}
		}
		const bool hit = PRE && pos == ppos; // wave-uniform
		pech_core cd;
		if (FLATG)
			cd = hit ? spec : flatg_core(cores, pos); // (hit: uni() below reads lane 0, group 0's = pos)
		else if (FLAT)
			cd = flat_core(lds, pos);
		else if (hit)
			cd = spec; // lanes 0-7 (group 0) hold cores[pos]; uni() reads lane 0
		else
			cd = cores[pos];
#ifdef PECH_DEBUG_BOUNDS
		if (FLATG && hit) {
			const uint32_t pj = min(pos + grp, nflat - 1u);
			const pech_core e = flatg_conv(((const u32x4 *)cores)[pj], pj);
			if (spec.rows != e.rows || spec.addr != e.addr || spec.meta != e.meta)
				printf("PECH OOB speculated flatg descriptor pos %u grp %u\n", pos, grp);
		} else if (hit && (cd.rows != cores[pos + grp].rows || cd.addr != cores[pos + grp].addr))
			printf("PECH OOB preloaded descriptor pos %u grp %u\n", pos, grp);
#endif
		const uint32_t rows0 = uni(cd.rows);
		if (FLAT && rows0 == 0u) { // an empty buffer (flat batches keep them in place; lr is 0 here)
			++pos;
			continue;
		}
		const uint64_t a0 = uni64(cd.addr);
		const uint64_t vb0 = a0 & ~(uint64_t)(PECH_ROW_BYTES - 1u);
		const uint32_t lb0 = (uint32_t)a0 & (PECH_ROW_BYTES - 1u);
		const uint32_t meta0 = uni(cd.meta);
		const uint32_t avail0 = rows0 - lr;
		// A large buffer (or what is left of it) goes to 8 slices when at least
		// PECH_SPLIT_MIN (8) of its rows are to be walked, so every slice has a
		// row.  A remainder walked by group 0 alone left 7 groups idle: below
		// PECH_SPLIT_ROWS, 19 % of the row slots of a C4-like mix
		// (tests/kernel_model.py); below 64 rows (v0.17-v0.30), every share
		// that ends a few rows into a buffer or starts a few rows before its
		// end -- launches whose rows per wave do not divide the buffers: 8 x
		// 4,100,000 B took 21.0 us against 14.2 us for 8 x 4 MiB
		// (profiles/r05/launch_sizes.txt).  The slices' folds and shifts run
		// side by side, so short slices cost no more than one group's run.
		if (rows0 >= PECH_SPLIT_ROWS && min(avail0, rem) >= PECH_SPLIT_MIN) {
			// one large buffer (portion): 8 contiguous slices, one per group
			const uint32_t P = min(avail0, rem);
			const uint32_t q = P >> 3, rm = P & 7u;
			const uint32_t st = lr + grp * q + min(grp, rm);
			const uint32_t nn = q + (grp < rm ? 1u : 0u);
			S.ad = vb0 + (uint64_t)st * PECH_ROW_BYTES + 16u * g8;
			S.nl = nn;
			S.nu = nn;
			S.oz = PECH_META_ORIG(meta0) | head_bits(st == 0, g8, lb0) | ra_bit(rows0 - st - nn) |
			       tail_of<FLAT>(st + nn == rows0, g8, meta0); // the first / this slice ends the buffer
			S.mp = mp_of<FLAT>(rows0 - st - nn, meta0);
			S.T = q + (rm ? 1u : 0u);
			S.nmin = q;
			if (COPY)
				dl = deltas[PECH_META_ORIG(meta0)];
#ifdef PECH_DEBUG_BOUNDS
			S.blo = vb0 + 16u * (lb0 >> 4);
			S.bhi = vb0 + (uint64_t)rows0 * PECH_ROW_BYTES;
#endif
			rem -= P;
			if (P == avail0) {
				++pos;
				lr = 0;
			} else {
				lr += P;
			}
		} else {
			// up to 8 neighbouring buffers, one per group.  Their descriptors
			// come in by SCALAR loads (lgkmcnt), so waiting for them never
			// drains the vector-load prefetch queue (vmcnt is in order).
			// pos+7 may run past the chunk (or the cores array into lrs, still
			// workspace memory); such entries are never used.
			uint32_t vlo = 0, vhi = 0, mrows = 0, mmeta = 0;
			int64_t mdl = 0;
			if (FLATG && hit) { // each group its own speculated entry
				vlo = (uint32_t)spec.addr;
				vhi = (uint32_t)(spec.addr >> 32);
				mrows = spec.rows;
				mmeta = spec.meta;
			} else if (FLATG) {
				// each group its own entry by a vector load (a miss: the
				// planner's prefetch a step ahead normally hits).  Eight scalar
				// loads and selects here made the compiler schedule the row
				// loops' lookups one pair at a time (c4-64k 53.3 -> ~49 us)
				const uint32_t pj = min(pos + grp, nflat - 1u);
				const pech_core dj = flatg_conv(((const u32x4 *)cores)[pj], pj);
				vlo = (uint32_t)dj.addr;
				vhi = (uint32_t)(dj.addr >> 32);
				mrows = dj.rows;
				mmeta = dj.meta;
			} else if (FLAT) { // each group its own entry (LDS: no scalar-load selects)
				const pech_core dj = flat_core(lds, min(pos + grp, nflat - 1u));
				vlo = (uint32_t)dj.addr;
				vhi = (uint32_t)(dj.addr >> 32);
				mrows = dj.rows;
				mmeta = dj.meta;
			} else if (hit) {
				vlo = (uint32_t)spec.addr;
				vhi = (uint32_t)(spec.addr >> 32);
				mrows = spec.rows;
				mmeta = spec.meta;
				if (COPY) {
					const uint32_t pj = pos + grp;
					const bool okj = (pj & 1023u) < nzc && (pj >> 10) == c;
					mdl = deltas[okj ? PECH_META_ORIG(spec.meta) : 0u];
				}
			} else {
#pragma unroll
				for (uint32_t j = 0; j < 8; ++j) {
					const pech_core dj = cores[pos + j];
					const bool mine = grp == j;
					vlo = mine ? uni((uint32_t)dj.addr) : vlo;
					vhi = mine ? uni((uint32_t)(dj.addr >> 32)) : vhi;
					mrows = mine ? uni(dj.rows) : mrows;
					mmeta = mine ? uni(dj.meta) : mmeta;
					if (COPY) {
						// entries past the chunk are garbage: never index with them
						const uint32_t pj = pos + j;
						const bool okj = (pj & 1023u) < nzc && (pj >> 10) == c;
						const int64_t dj_dl = deltas[okj ? PECH_META_ORIG(uni(dj.meta)) : 0u];
						mdl = mine ? dj_dl : mdl;
					}
				}
			}
			pech_core my;
			my.addr = ((uint64_t)vhi << 32) | vlo;
			my.rows = mrows;
			my.meta = mmeta;
			const uint32_t myp = pos + grp;
			const bool inchunk = FLAT ? myp < nflat : (myp & 1023u) < nzc && (myp >> 10) == c;
			const uint32_t myrows = inchunk ? my.rows : 0u;
			// cut at the first non-first group whose buffer is split or out of chunk
			const bool cut = grp > 0 && (!inchunk || myrows >= PECH_SPLIT_ROWS);
			const uint64_t cutm = __ballot(cut && g8 == 0);
			const uint32_t kcut = cutm ? (uint32_t)(__builtin_ctzll(cutm) >> 3) : 8u;
			const uint32_t mylr = grp ? 0u : lr;
			const uint32_t avail = grp < kcut ? myrows - mylr : 0u;
			// exclusive prefix of avail over groups (one contribution per
			// group, from its lane 0), by DPP: no LDS round trips
			const uint32_t incl = wave_incl_scan(g8 == 0 ? avail : 0u);
			const uint32_t pre = incl - avail;
			// grid (static shares): a step of small buffers is walked whole
			// by the wave whose share holds its middle row (the first row of
			// its position kcut/2; prologue in main_body), else not at all
			const bool whole = grid && rows0 < PECH_SPLIT_ROWS;
			const bool own = lane_value(pre, 8u * (kcut >> 1)) < rem;
			const uint32_t nu = whole ? (own ? avail : 0u) : (pre >= rem ? 0u : min(avail, rem - pre));
			// the step's longest and shortest run: 8 lane reads (group-uniform values)
			uint32_t tmax = 0, tmin = 0xFFFFFFFFu;
#pragma unroll
			for (uint32_t j = 0; j < 8; ++j) {
				const uint32_t v = lane_value(nu, 8u * j);
				tmax = max(tmax, v);
				tmin = v ? min(tmin, v) : tmin;
			}
			S.T = tmax;
			S.nmin = tmin;
			// (whole: the share's rest at most; a step not owned ends the range)
			const uint32_t used = whole && !own ? rem : min(lane_value(incl, 63), rem);
			const uint32_t mylb = (uint32_t)my.addr & (PECH_ROW_BYTES - 1u);
			const uint64_t myvb = my.addr & ~(uint64_t)(PECH_ROW_BYTES - 1u);
			if (nu) {
				S.ad = myvb + (uint64_t)mylr * PECH_ROW_BYTES + 16u * g8;
				S.nl = nu;
				S.oz = PECH_META_ORIG(my.meta) | head_bits(mylr == 0, g8, mylb) | ra_bit(myrows - mylr - nu) |
				       tail_of<FLAT>(mylr + nu == myrows, g8, my.meta); // the run ends the buffer
			} else {
				// idle groups reload group 0's rows (valid memory: the redirect
				// of row 0's pieces before the buffer kept), state ignored
				S.ad = vb0 + (uint64_t)lr * PECH_ROW_BYTES + 16u * g8;
				S.nl = min(avail0, rem);
				S.oz = head_bits(lr == 0, g8, lb0) & (7u << 20);
			}
			S.nu = nu;
			dl = mdl;
			S.mp = mp_of<FLAT>(myrows - mylr - nu, my.meta);
#ifdef PECH_DEBUG_BOUNDS
			const uint64_t bv = nu ? myvb : vb0;
			S.blo = bv + 16u * ((nu ? mylb : lb0) >> 4);
			S.bhi = bv + (uint64_t)(nu ? myrows : rows0) * PECH_ROW_BYTES;
#endif
			rem -= used;
			if (rem) { // then every group < kcut finished its buffer
				pos += kcut;
				lr = 0;
			}
		}
		break;
	}
	S.pos = pos;
	S.lr = lr;
	S.rem = rem;
	S.dad = S.ad + (uint64_t)dl;
	return S;
}

// Fused copy, interleaved rows (uniform batches of buffers of at least
// PECH_IL_MIN_ROWS rows): the workgroup's 128 lane groups walk the portion
// [lr, lr + P) of one buffer together, group j taking rows lr + j,
// lr + j + 128, ... (`ad` steps 16 KiB per row; Horner over rows 128 apart
// is A_16384, the LDS table in this mode).  One row step of the workgroup
// reads and writes 16 KiB contiguous, so the CU's accesses in flight form
// one window instead of 128 scattered slices (copy probe: 389.5 against
// 407.0 us per GiB, profiles/r03/copyshape_probe.json).  The cursor is the
// workgroup's, the same in all its waves.
// FLAT (pech_crc32c_flat on host-resident slots, PECH_FLAT_F_IL): the
// descriptors from the wave's LDS table, the last line's bytes kept below kb.
template <bool COPY, bool FLAT = false>
__device__ __forceinline__ Step plan_il(const pech_core *__restrict__ cores, const int64_t *__restrict__ deltas,
					uint32_t pos, uint32_t lr, uint32_t rem, uint32_t j, uint32_t g8,
					const uint32_t *lds = nullptr)
{
	static_assert(!(FLAT && COPY), "flat batches: CRC only");
	Step S;
	int64_t dl = 0;
	S.T = 0;
	S.nmin = 0;
	S.ad = 0;
	S.mp = 0;
	S.nl = 1;
	S.nu = 0;
	S.oz = 0;
#ifdef PECH_DEBUG_BOUNDS
	S.blo = S.bhi = 0;
#endif
	// A portion of at most j0 rows (the wave's first group) gives the whole
	// wave nothing to do: it moves on to the next portion instead of ending
	// its walk -- the workgroup's range goes on, and a range that starts in a
	// buffer's last rows (P < 120) left waves 1-15 without their rows of every
	// later portion (fused copy and flat interleaved mode; found by
	// test_zero_copy_slots_interleaved_rows: 3 x 1,025-row buffers, a range
	// starting 4 rows before a buffer's end)
	const uint32_t j0 = j & ~7u;
	while (rem) {
		const pech_core cd = FLAT ? flat_core(lds, pos) : cores[pos]; // wave-uniform (scalar loads when planned)
		const uint32_t rows0 = uni(cd.rows);
		const uint64_t a0 = uni64(cd.addr);
		const uint64_t vb0 = a0 & ~(uint64_t)(PECH_ROW_BYTES - 1u);
		const uint32_t lb0 = (uint32_t)a0 & (PECH_ROW_BYTES - 1u);
		const uint32_t meta0 = uni(cd.meta);
		const uint32_t zt0 = PECH_META_ZT(meta0);
		const uint32_t P = min(rows0 - lr, rem);
		if (P <= j0) { // no row of this portion for any group of the wave
			rem -= P;
			if (lr + P == rows0) {
				++pos;
				lr = 0;
			} else {
				lr += P;
			}
			continue;
		}
		const uint32_t nn = P > j ? (P - j + PECH_IL_GROUPS - 1u) / PECH_IL_GROUPS : 0u;
		const uint32_t st = lr + j;
		// the wave's 8 groups are j0..j0+7: counts nonincreasing in the group
		S.T = (P - j0 + PECH_IL_GROUPS - 1u) / PECH_IL_GROUPS;
		uint32_t tmin = S.T;
#pragma unroll
		for (uint32_t g = 1; g < 8; ++g) {
			const uint32_t c = P > j0 + g ? (P - j0 - g + PECH_IL_GROUPS - 1u) / PECH_IL_GROUPS : 0u;
			tmin = c ? c : tmin;
		}
		S.nmin = tmin;
		if (nn) {
			const uint32_t last = st + PECH_IL_GROUPS * (nn - 1u);
			S.ad = vb0 + (uint64_t)st * PECH_ROW_BYTES + 16u * g8;
			S.nl = nn;
			S.nu = nn;
			S.oz = PECH_META_ORIG(meta0) | head_bits(st == 0, g8, lb0) | ra_bit(rows0 - last - 1u) |
			       (FLAT ? tail_of<true>(last == rows0 - 1u, g8, meta0) : tail_bits(last == rows0 - 1u, g8, zt0));
			S.mp = mp_of<FLAT>(rows0 - last - 1u, meta0);
		} else {
			// an idle group reloads the portion's first row (valid memory,
			// the redirect of row 0's pieces before the buffer kept), ignored
			S.ad = vb0 + (uint64_t)lr * PECH_ROW_BYTES + 16u * g8;
			S.oz = head_bits(lr == 0, g8, lb0) & (7u << 20);
		}
		if (COPY)
			dl = deltas[PECH_META_ORIG(meta0)];
#ifdef PECH_DEBUG_BOUNDS
		S.blo = vb0 + 16u * (lb0 >> 4);
		S.bhi = vb0 + (uint64_t)rows0 * PECH_ROW_BYTES;
#endif
		rem -= P;
		if (lr + P == rows0) {
			++pos;
			lr = 0;
		} else {
			lr += P;
		}
		break;
	}
	S.pos = pos;
	S.lr = lr;
	S.rem = rem;
	S.dad = S.ad + (uint64_t)dl;
	return S;
}

#define STEP_ZOFF(S) (((S).oz >> 16) & 0x70u) // (zoff/16) << 20 -> zoff
#define STEP_ORIG(S) ((S).oz & 0xFFFFFu)
#define STEP_ZH(S) (((S).oz >> 23) & 15u)
#define STEP_HEAD(S) (((S).oz >> 20) & 0x7Fu) // row 0's piece is not wholly the buffer's (zoff or zh)
#define STEP_ZL(S) ((S).oz & (1u << 27)) // bit 28: STEP_SLOW (direct kernel), bit 29: PECH_OZ_RA25
#define STEP_RA(S) ((uint64_t)((S).mp >> 7) | (uint64_t)((S).oz & PECH_OZ_RA25) >> 4) // rows after the run
#define STEP_M(S) ((int64_t)(STEP_RA(S) * PECH_ROW_BYTES + ((S).mp & 15u)) - (int64_t)((S).mp & 0x70u))
// flat batches: m = 128 ra - T, and the position in bits 0-11 (kb above it)
template <bool FLAT>
__device__ __forceinline__ int64_t step_m(const Step &S)
{
	return FLAT ? (int64_t)(STEP_RA(S) * PECH_ROW_BYTES) - (int64_t)(S.mp & 127u) : STEP_M(S);
}
template <bool FLAT>
__device__ __forceinline__ uint32_t step_orig(const Step &S)
{
	return FLAT ? (S.oz & 0xFFFu) : STEP_ORIG(S);
}
// x^(8 * 128 * rows after the run), modulo the table's span (finish_run)
__device__ __forceinline__ uint32_t rowpow(const uint32_t *consts, const Step &S)
{
	return consts[PECH_C_ROWPOW + ((uint32_t)STEP_RA(S) & (PECH_ROWPOW_N - 1u))];
}

// a / b with a 32-bit quotient: one 32-bit division when a fits 32 bits
// (wave-uniform: a scalar branch), the 64-bit sequence otherwise
__device__ __forceinline__ uint64_t div_u64_u32(uint64_t a, uint32_t b)
{
	return (a >> 32) == 0u ? (uint64_t)((uint32_t)a / b) : a / b;
}

// Ring discipline: row k of a step lives in ring slot k % PECH_U and the
// lookahead is PECH_U-1 rows.  The iteration that consumes row k first issues
// the load of row k+PECH_U-1 into the slot row k-1 has just vacated, so no
// slot ever holds two live values: the register mapping is static across
// the loop back-edge (no copies, and no vmcnt(0) drain to make them).
// Priming loads rows 0..PECH_U-2 (clamped to the step's rows).
#define RING_PRIME_RS(S, ring, rs)                                                                     \
	do {                                                                                          \
		const uint32_t last_ = (S).nl - 1u;                                                   \
		_Pragma("unroll") for (uint32_t i = 0; i + 1 < U; ++i) (ring)[i] =                    \
			LD_PIECE((S), row_addr((S).ad, min(i, last_), STEP_ZOFF(S), (rs)), 1);           \
	} while (0)
#define RING_PRIME(S, ring) RING_PRIME_RS(S, ring, PECH_ROW_BYTES)

__device__ __forceinline__ void horner_row(const uint32_t *lds, uint32_t lreg, u32x4 w, uint32_t &s0, uint32_t &s1,
					   uint32_t &s2, uint32_t &s3)
{
	s0 = adv128(lds, s0, lreg, w.x);
	s1 = adv128(lds, s1, lreg, w.y);
	s2 = adv128(lds, s2, lreg, w.z);
	s3 = adv128(lds, s3, lreg, w.w);
}

__device__ __forceinline__ void horner_row_pred(const uint32_t *lds, uint32_t lreg, u32x4 w, bool ok, uint32_t &s0,
						uint32_t &s1, uint32_t &s2, uint32_t &s3)
{
	const uint32_t t0 = adv128(lds, s0, lreg, w.x);
	const uint32_t t1 = adv128(lds, s1, lreg, w.y);
	const uint32_t t2 = adv128(lds, s2, lreg, w.z);
	const uint32_t t3 = adv128(lds, s3, lreg, w.w);
	s0 = ok ? t0 : s0;
	s1 = ok ? t1 : s1;
	s2 = ok ? t2 : s2;
	s3 = ok ? t3 : s3;
}

// Fold a group's 32 stream registers into the CRC of its run (as a message
// ending at the run's last row), shift it to the buffer's core end plus the
// tail (m bytes), xor into out[orig].
template <bool ROWPOW>
__device__ __forceinline__ void finish_run(uint32_t *lds, uint32_t g8, uint32_t s0, uint32_t s1, uint32_t s2,
					   uint32_t s3, int64_t m, uint64_t ra, uint32_t tpow, bool active, uint32_t *out,
					   uint32_t orig)
{
	uint32_t u = adv_tab(lds, L_TAB4, s0) ^ s1;
	u = adv_tab(lds, L_TAB4, u) ^ s2;
	u = adv_tab(lds, L_TAB4, u) ^ s3;
	u = adv_tab(lds, L_TAB4, u);
	// Butterfly to the group's lane 0 only (the one that uses the result):
	// at each stage the lower lane of a pair folds in its partner's value,
	// read by a DPP row shift (lane i <- lane i + d, inside the 16-lane row
	// that holds the whole group) instead of an LDS permute.
	u = adv_tab(lds, L_TAB16, u) ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x101, 0xf, 0xf, true);
	u = adv_tab(lds, L_TAB32, u) ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x102, 0xf, 0xf, true);
	u = adv_tab(lds, L_TAB64, u) ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x104, 0xf, 0xf, true);
	uint32_t v = 0;
	if (ROWPOW) {
		// m = 128 ra + dl, dl in [-112, 15]: x^(8 dl) from the power table
		// (x^(-8k) for the trailing virtual zeros), x^(8 128 ra) read from
		// the row-power table one step ahead (tpow) -- at most two products,
		// one for aligned buffers, instead of one per 6-bit digit of m (up to
		// four for a 4 MiB buffer)
		if (active && g8 == 0) {
			const int32_t dl = (int32_t)(m - (int64_t)(ra * PECH_ROW_BYTES));
			v = u;
			if (dl != 0)
				v = gf2_mulmod_dev(dl > 0 ? lds[L_POWB / 4u + (uint32_t)dl] : lds[L_XINV / 4u + (uint32_t)(-dl)], v);
			if (ra != 0)
				v = gf2_mulmod_dev(tpow, v);
			if (ra >> PECH_ROWPOW_BITS) // buffers above 32 MiB: the rest by digits
				v = shift_bytes(lds + L_POWB / 4u, (ra >> PECH_ROWPOW_BITS) << (PECH_ROWPOW_BITS + 7u), v);
		}
	} else if (active && g8 == 0) { // m < 0: the run's trailing virtual zeros outweigh the tail
		v = m > 0 ? shift_bytes(lds + L_POWB / 4u, (uint64_t)m, u)
			  : (m < 0 ? gf2_mulmod_dev(lds[L_XINV / 4u + (uint32_t)(-m)], u) : u);
	}
	// A split step (every active group on one buffer) folds its 8 group
	// results in registers: one atomic per wave instead of 8 on one address.
	const uint32_t o0 = uni(orig);
	if (__ballot(active && orig != o0) == 0ull) {
		// groups 0+1, 2+3, 4+5, 6+7 by a DPP row shift, then four lane reads
		v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x108, 0xf, 0xf, true);
		v = lane_value(v, 0) ^ lane_value(v, 16) ^ lane_value(v, 32) ^ lane_value(v, 48);
		if ((threadIdx.x & 63u) == 0) {
			// the workgroup's table: slot o0 % 64, claimed by CAS; a slot
			// held by another buffer falls back to the global atomic
			uint32_t *keys = (uint32_t *)lds + L_DEFER / 4u, *vals = keys + PECH_DEFER_SLOTS;
			const uint32_t sl = o0 & (PECH_DEFER_SLOTS - 1u);
			const uint32_t prev = atomicCAS(keys + sl, PECH_DEFER_EMPTY, o0);
			if (prev == PECH_DEFER_EMPTY || prev == o0)
				atomicXor(vals + sl, v);
			else
				atomicXor(out + o0, v);
		}
	} else if (active && g8 == 0) {
#ifdef PECH_AB_NOATOMIC // diagnostic build only: run results of non-split steps dropped (wrong CRCs; the deferral flush too)
		if (v == 0x9E3779B9u)
#endif
		atomicXor(out + orig, v);
	}
}

// A trailing virtual piece (past the core's end, in the core's last row)
// counts as zero; only the ragged and last blocks of a step can hold a run's
// last row.  Flat batches: the lane keeps the first kb bytes of its piece of
// the buffer's last line (the rest lies past the buffer).
template <bool FLAT = false>
__device__ __forceinline__ u32x4 zl_mask(const Step &S, uint32_t row, u32x4 v)
{
	if (FLAT)
		return (STEP_ZL(S) && row == S.nu - 1u) ? keep_below(v, (S.oz >> PECH_FLAT_KB_SHIFT) & 31u) : v;
	return (STEP_ZL(S) && row == S.nu - 1u) ? (u32x4)(0u) : v;
}
__device__ __forceinline__ bool zl_keep(const Step &S, uint32_t row)
{
	return !(STEP_ZL(S) && row == S.nu - 1u);
}

// Fused copy: the consumed piece of row `row` of the lane's run goes to its
// destination (S.dad: source + dst - src).  Pieces not wholly the buffer's
// (row 0 with zoff or zh -- the plan kernel copies the bytes of a partial
// one --, trailing virtual pieces) and rows past nu (clamped prefetch, idle
// groups) are never stored.
template <bool COPY>
__device__ __forceinline__ void st_piece(const Step &S, uint32_t row, u32x4 v, bool ok, uint32_t rs = PECH_ROW_BYTES)
{
	typedef __attribute__((address_space(1))) u32x4 g_u32x4w;
	if (COPY && ok) // nontemporal: the destination is not re-read by this launch
		__builtin_nontemporal_store(v, (g_u32x4w *)(S.dad + (uint64_t)row * rs));
}

// Uniform batches: the end of share [a, b)'s head, which its owner walks
// first; the rest of the share (at most PECH_POOL_ROWS rows) is pooled.  The
// head is at least one item, or the whole share.
__device__ __forceinline__ uint32_t share_head(uint32_t a, uint32_t b)
{
	return min(b, max(a + PECH_ITEM_ROWS, b - min(PECH_POOL_ROWS, b - a)));
}

// Wave priority (s_setprio) from a static share's progress: 3 while more
// than 3/4 of the share's rows remain, then 2, 1, 0.  The SQ issues
// oldest-first among waves of equal priority, so with equal static shares a
// CU's four waves per SIMD finished in age order, up to 65 us apart (C4,
// busy p50 85 / 108 / 134 / 149 us by age slot, profiles/r05/stamps_c4.txt),
// and the CU's last quarter ran on a quarter of its waves.  Raising the
// waves that are behind keeps a CU's waves within about a quarter of a share
// of each other (profiles/r05/ab_prio.txt).  Pooled walks use the same
// levels over the rows a wave still holds once its pool is dry (main_body).
#ifndef PECH_PRIO_MIN_SHARE
#define PECH_PRIO_MIN_SHARE 1024u
#endif
struct Prio {
	uint32_t th1, th2, th3, cur;
};
__device__ __forceinline__ Prio prio_init(uint32_t tot)
{
	return Prio{tot / 4u, tot / 2u, tot - tot / 4u, 0xFFu};
}
__device__ __forceinline__ void prio_update(Prio &P, uint32_t rem_rows)
{
	const uint32_t q = (rem_rows > P.th1 ? 1u : 0u) + (rem_rows > P.th2 ? 1u : 0u) + (rem_rows > P.th3 ? 1u : 0u);
	if (q == P.cur)
		return;
	P.cur = q;
	if (q == 3u)
		__builtin_amdgcn_s_setprio(3);
	else if (q == 2u)
		__builtin_amdgcn_s_setprio(2);
	else if (q == 1u)
		__builtin_amdgcn_s_setprio(1);
	else
		__builtin_amdgcn_s_setprio(0);
}

// What a main-kernel wave knows after the chunk scan and the start search
// (prologue_start): all wave-uniform.
struct Start {
	uint32_t U0, wg_rows, r0, r1, jmax, rem_all, p0, lr0, jj, pjj, nzjj, nsjj;
	uint32_t nlive; // live workgroups of the launch (the same in every one)
	uint64_t wg0;
	bool uniform, il;
#ifdef PECH_STAMPS
	uint64_t t_scan;
#endif
};

// Every wave's equal share [r0, r1) of the batch's Rtot rows, the
// workgroup's static rows [wg0, wg0 + wg_rows), the pool size (jmax) and the
// rows the wave walks before pooling (rem_all); false when the whole
// workgroup is idle (small batch).  (Shared by the planned and the flat
// prologues.)
template <bool COPY>
__device__ __forceinline__ bool wave_share(uint32_t Rtot, uint32_t W, uint32_t rpw_min, uint32_t wave, bool uniform,
					   bool il, Start &st)
{
	// Every wave gets an equal share of the batch's rows (at least rpw_min).
	// Large batches: workgroup b gets rows [b Rtot / G, (b+1) Rtot / G) --
	// proportional, not b * ceil(Rtot / W): the rounding drifted by up to a
	// row per wave, a whole step of 8 small buffers after a few hundred
	// waves, so some waves walked an extra step (2 -> 3 on unaligned
	// 4,100-byte buffers) and set the launch's end.  Small batches: shares
	// of rpw rows, the last ones idle.  rpw grows with the launch from
	// rpw_min to 4 rpw_min, aiming at four live waves per CU (one per SIMD):
	// below ~128 MiB a launch is latency-bound, and fewer, longer waves
	// spend less of it in per-wave work (32 MiB: 15.2 -> 13.4 us,
	// profiles/r05/ab_wave_major.txt); from W 4 rpw_min rows on, every wave
	// of every CU streams its proportional share.
	const uint32_t G4 = PECH_LIVE_WAVES * gridDim.x;
	const uint32_t rpw_a = min(max((uint32_t)(((uint64_t)Rtot + G4 - 1u) / G4), rpw_min), 4u * rpw_min);
	const bool prop = (uint64_t)Rtot >= (uint64_t)W * rpw_a;
	const uint32_t rpw = prop ? 0u : rpw_a;
#ifdef PECH_FAST_DIV // A/B: 32-bit quotients when the products fit 32 bits (batches below 4 GiB / grid rows)
	const uint64_t wg0 = prop ? div_u64_u32((uint64_t)blockIdx.x * Rtot, gridDim.x)
				  : (uint64_t)blockIdx.x * PECH_MAIN_WAVES * rpw;
	const uint32_t wg_rows = prop ? (uint32_t)(div_u64_u32((uint64_t)(blockIdx.x + 1u) * Rtot, gridDim.x) - wg0)
				      : (uint32_t)min((uint64_t)PECH_MAIN_WAVES * rpw, (uint64_t)Rtot - wg0);
#else
	const uint64_t wg0 = prop ? (uint64_t)blockIdx.x * Rtot / gridDim.x : (uint64_t)blockIdx.x * PECH_MAIN_WAVES * rpw;
#endif
#ifndef PECH_WG_MAJOR_SMALL
	// Small batches, wave-major: share k = wave * G + blockIdx, so the live
	// shares spread one or two waves per CU over every CU instead of filling
	// the first CUs' 16 waves -- four waves to a SIMD took turns at the same
	// VALU work (prologue, fold, shift), and a 4 MiB launch's youngest waves
	// ended 3.5 us after its oldest (profiles/r05/stamps_flat_v29a.txt).  (Not
	// with interleaved rows: they walk the workgroup's range together.)
	st.nlive = prop ? gridDim.x : (uint32_t)min((uint64_t)gridDim.x, ((uint64_t)Rtot + rpw - 1u) / rpw);
	if (!prop && !il) {
#ifdef PECH_DEAL_FULL_GRID // A/B: the shares dealt over every workgroup (v0.29c-v0.31)
		const uint32_t Gd = gridDim.x;
#else
		// ... over just enough workgroups for PECH_LIVE_WAVES live waves each:
		// below 4 G rpw_min rows (8 MiB on 256 CUs) fewer workgroups carry the
		// launch, and each buffer's out[] word gets fewer cross-workgroup XORs
		// (a 4 MiB launch: 128 instead of 256 onto one word; those atomics cost
		// small launches 1.5-2 us, profiles/r05/ab_share_dealing.txt)
		const uint32_t nsh = (uint32_t)(((uint64_t)Rtot + rpw - 1u) / rpw);
		const uint32_t Gd = min(gridDim.x, (nsh + PECH_LIVE_WAVES - 1u) / PECH_LIVE_WAVES);
		st.nlive = min(st.nlive, Gd);
		if (blockIdx.x >= Gd)
			return false; // whole workgroup idle
#endif
#if PECH_DEAL_BLOCKS
		// ... in blocks of 4 S shares, S = PECH_DEAL_BLOCKS: a workgroup's live
		// shares lie S apart inside one block (one buffer as a rule, so the
		// workgroup's deferral table sends one atomic per buffer; not
		// neighbours: two waves of a CU on neighbouring ranges of a buffer
		// cost more than the atomics they save).  64 x 500 KiB 17.0 -> 14.0 us,
		// 4 MiB of 64 KiB buffers 10.1-10.5 -> 8.3-8.7 us
		// (profiles/r05/ab_deal_blocks.txt).  (-DPECH_DEAL_BLOCKS=0: strided.)
		constexpr uint32_t S = PECH_DEAL_BLOCKS;
		const uint64_t k = Gd % S == 0u && wave < PECH_LIVE_WAVES
					   ? (uint64_t)(blockIdx.x / S) * (PECH_LIVE_WAVES * S) + blockIdx.x % S + S * wave
					   : (uint64_t)wave * Gd + blockIdx.x;
		// live: the workgroups whose first share exists (every full block's S,
		// the last one's first ones; all Gd once there are more shares than
		// the blocks hold -- the waves past PECH_LIVE_WAVES take those)
		if (Gd % S == 0u)
			st.nlive = min(Gd, nsh / (PECH_LIVE_WAVES * S) * S + min(nsh % (PECH_LIVE_WAVES * S), S));
		if (Gd % S == 0u ? (uint64_t)(blockIdx.x / S) * (PECH_LIVE_WAVES * S) + blockIdx.x % S >= nsh
				 : (uint64_t)blockIdx.x * rpw >= Rtot)
			return false; // whole workgroup idle: its wave 0 has the lowest share
#else
		const uint64_t k = (uint64_t)wave * Gd + blockIdx.x;
		if ((uint64_t)blockIdx.x * rpw >= Rtot)
			return false; // whole workgroup idle: its wave 0 has the lowest share
#endif
		const uint64_t a = k * rpw;
		st.r0 = (uint32_t)min(a, (uint64_t)Rtot);
		st.r1 = (uint32_t)min(a + rpw, (uint64_t)Rtot);
		st.wg0 = 0;
		st.wg_rows = 0;
		st.jmax = 0;
		st.rem_all = st.r1 - st.r0;
		st.U0 = 0;
		st.uniform = uniform;
		st.il = il;
		return true;
	}
#endif
#ifdef PECH_WG_MAJOR_SMALL
	if (!prop)
#else
	if (!prop && il) // (interleaved rows keep workgroup-major shares: 16 rpw rows per live workgroup)
#endif
		st.nlive = (uint32_t)min((uint64_t)gridDim.x, ((uint64_t)Rtot + PECH_MAIN_WAVES * rpw - 1u) / (PECH_MAIN_WAVES * rpw));
	if (wg0 >= Rtot)
		return false; // whole workgroup idle (small batch)
	// The workgroup's static rows [wg0, wg0 + wg_rows) go to its waves in
	// equal contiguous pieces (age-weighted shares measured no better,
	// profiles/r01/ab_v5.txt).
#ifndef PECH_FAST_DIV
	const uint32_t wg_rows = prop ? (uint32_t)((uint64_t)(blockIdx.x + 1u) * Rtot / gridDim.x - wg0)
				      : (uint32_t)min((uint64_t)PECH_MAIN_WAVES * rpw, (uint64_t)Rtot - wg0);
#endif
	const uint32_t r0 = (uint32_t)(wg0 + (uint64_t)wg_rows * wave / PECH_MAIN_WAVES);
	const uint32_t r1 = (uint32_t)(wg0 + (uint64_t)wg_rows * (wave + 1u) / PECH_MAIN_WAVES);
	// Uniform batches: a wave starts on its share's head [r0, t) and then
	// takes items of PECH_ITEM_ROWS rows from the workgroup's pool of share
	// tails (at most PECH_POOL_ROWS of each share; an LDS counter, claim c is
	// tail item c/16 of share c%16, located by division), so the CU's 16
	// waves -- issued oldest-first, which made equal static shares finish up
	// to 60 us apart -- end together, and the CU is free for the next
	// launch's workgroup that much earlier.  (The fused copy keeps static
	// shares: pooled items cost it 9-14 % per launch, profiles/r02/ab_item_pool.txt.)
	// Shares below PECH_POOL_MIN_SHARE rows keep static shares too: a 512-row
	// share (256 MiB of 64 KiB-4 MiB buffers) pooled is a 256-row head and one
	// item, i.e. runs of 32 rows with a fold each; static, one step of 64-row
	// runs: 48.8 instead of 51.5-53.4 us per launch (profiles/r03/ab_pool_min_share.txt).
#ifdef PECH_NO_POOL // A/B: static shares for every batch
	const uint32_t jmax = 0u;
#else
	const uint32_t jmax = !COPY && !il && uniform && wg_rows >= PECH_MAIN_WAVES * PECH_POOL_MIN_SHARE
				      ? 1u + (min(PECH_POOL_ROWS, (wg_rows + PECH_MAIN_WAVES - 1u) /
										      PECH_MAIN_WAVES) + PECH_ITEM_ROWS - 1u) /
							     PECH_ITEM_ROWS
					       : 0u;
#endif
	st.U0 = 0;
	st.wg_rows = wg_rows;
	st.r0 = r0;
	st.r1 = r1;
	st.jmax = jmax;
	st.rem_all = jmax ? share_head(r0, r1) - r0 : r1 - r0;
	st.wg0 = wg0;
	st.uniform = uniform;
	st.il = il;
	return true;
}

// The main kernel's chunk scan and start search, with CPL chunks per lane
// (4: batches of up to 256 chunks, 16: up to PECH_MAX_CHUNKS).  Every wave
// scans the chunk totals itself (no workgroup scan, no barrier), takes its
// equal share [r0, r1) of the rows, and locates r0: first at the speculated
// position pg (exact for uniform batches), else by a search over the chunk
// prefixes and the start chunk's row offsets (lr4, reloaded when the
// speculated chunk was wrong).  It also writes the chunk non-empty counts to
// LDS for plan_step.  Returns false when the whole workgroup is idle.
template <bool COPY, uint32_t CPL>
__device__ __forceinline__ bool prologue_start(uint32_t *lds, const pech_core *__restrict__ cores,
					       const uint32_t *__restrict__ lrs, const uint32_t *__restrict__ partials,
					       const uint32_t *__restrict__ nzs, uint32_t n, uint32_t nchunks, uint32_t lane,
					       uint32_t wave, uint32_t W, uint32_t rpw_min, uint32_t pg, uint32_t cg,
					       uint32_t lrg, const pech_core &spec, u32x4 (&lr4)[4], Start &st)
{
	static_assert(CPL == 4u || CPL == 16u, "chunks per lane");
	static_assert(64u * 16u == PECH_MAX_CHUNKS, "16 chunks per lane cover every chunk");
	// (partials / nzs hold PECH_MAX_CHUNKS entries in the workspace: CPL = 4
	// reads the first 256 of each unconditionally, entries past nchunks are
	// masked)
	u32x4 pv4[CPL / 4u], nv4[CPL / 4u];
	if (CPL == 4u) {
		pv4[0] = ((const u32x4 *)partials)[lane];
		nv4[0] = ((const u32x4 *)nzs)[lane];
	} else {
#pragma unroll
		for (uint32_t k = 0; k < CPL / 4u; ++k) // defined values where nothing loads (a select of undef may fold)
			pv4[k] = nv4[k] = (u32x4)(0u);
		if (lane * CPL < nchunks) {
#pragma unroll
			for (uint32_t k = 0; k < CPL / 4u; ++k) {
				pv4[k] = ((const u32x4 *)partials)[lane * (CPL / 4u) + k];
				nv4[k] = ((const u32x4 *)nzs)[lane * (CPL / 4u) + k];
			}
		}
	}
	// the wave's own exclusive scan of the chunk totals
	uint32_t pc[CPL], nc[CPL], lsum = 0;
	bool uflag = true;
#pragma unroll
	for (uint32_t k = 0; k < CPL; ++k) {
		const bool real = lane * CPL + k < nchunks;
		const uint32_t nzf = real ? nv4[k >> 2][k & 3u] : PECH_NZ_UNIFORM;
		pc[k] = real ? pv4[k >> 2][k & 3u] : 0u;
		nc[k] = nzf & ~PECH_NZ_UNIFORM; // non-empty | small cores << PECH_NS_SHIFT
		uflag = uflag && (nzf & PECH_NZ_UNIFORM) != 0u;
		lsum += pc[k];
	}
	const uint32_t incl = wave_incl_scan(lsum);
	const uint32_t Rtot = lane_value(incl, 63);
	// Uniform batch (every chunk flagged by the plan kernel, all with chunk
	// 0's rows per buffer): position p holds rows [p U0, (p+1) U0), so any row
	// is located by a division, and the workgroup pools its rows in items.
	const uint32_t nz0 = lane_value(nc[0], 0) & PECH_NZ_MASK; // (lane values: wave-uniform, as the pool needs)
	const uint32_t U0 = nz0 ? lane_value(pc[0], 0) / nz0 : 0u;
	bool uok = uflag;
#pragma unroll
	for (uint32_t k = 0; k < CPL; ++k)
		uok = uok && (uint64_t)(nc[k] & PECH_NZ_MASK) * U0 == (uint64_t)pc[k];
	const bool uniform = U0 != 0u && __ballot(!uok) == 0ull;
	// fused copy of a uniform batch of large buffers: interleaved rows (plan_il)
	const bool il = (COPY ? PECH_IL_COPY : PECH_IL_CRC) && uniform && U0 >= PECH_IL_MIN_ROWS;
	STAMP(t_scan);
#ifdef PECH_STAMPS
	st.t_scan = t_scan;
#endif
	if (!wave_share<COPY>(Rtot, W, rpw_min, wave, uniform, il, st))
		return false; // whole workgroup idle (small batch)
	const uint32_t r0 = st.r0, rem_all = st.rem_all;
	// nz table for plan_step: every wave writes all of it (the same values)
	// and reads back only its own writes until the barrier below
#pragma unroll
	for (uint32_t k = 0; k < CPL / 4u; ++k)
		*(u32x4 *)(lds + L_NZ / 4u + lane * CPL + 4u * k) =
			u32x4{nc[4 * k], nc[4 * k + 1], nc[4 * k + 2], nc[4 * k + 3]} & PECH_NZ_MASK; // braces: a parenthesised list is a comma splat

	uint32_t p0 = 0, lr0 = 0;
	bool found = false;
	// the start chunk's prefix, non-empty and small cores, and rows (grid snap below)
	uint32_t jj = 0, pjj = 0, nzjj = 0, nsjj = 0;
	if (rem_all) {
		// The speculated position first, checked exactly: buffer pg holds
		// row r0 iff its global offset (chunk prefix + lrs[pg]) <= r0 <
		// offset + its rows.  Uniform batches start here without waiting for
		// the row-offset scan below.
		const uint32_t lc = cg / CPL, kc = cg % CPL;
		uint32_t prec = incl - lsum, nzc = 0;
#pragma unroll
		for (uint32_t k = 0; k < CPL; ++k) {
			prec += k < kc ? pc[k] : 0u;
			nzc = k == kc ? nc[k] : nzc;
		}
		const uint32_t og = lane_value(prec, lc) + uni(lrg);
		const uint32_t rg = uni(spec.rows); // lane 0: cores[pg]
		if (cg < nchunks && (pg & 1023u) < (lane_value(nzc, lc) & PECH_NZ_MASK) && og <= r0 && r0 - og < rg) {
			p0 = pg;
			lr0 = r0 - og;
			found = true;
			jj = cg;
			pjj = lane_value(prec, lc);
			nzjj = lane_value(nzc, lc);
			nsjj = nzjj >> PECH_NS_SHIFT;
			nzjj &= PECH_NZ_MASK;
		}
	}
	if (rem_all && !found) {
		// start chunk j: the last chunk whose prefix is <= r0 (non-empty,
		// since r0 < Rtot); its prefix and non-empty count
		uint32_t pre = incl - lsum, cnt = 0, pj = 0, nzj = 0;
#pragma unroll
		for (uint32_t k = 0; k < CPL; ++k) {
			const bool le = lane * CPL + k < nchunks && pre <= r0;
			cnt += le ? 1u : 0u;
			pj = le ? pre : pj;
			nzj = le ? nc[k] : nzj;
			pre += pc[k];
		}
		// (prefixes are nondecreasing: the lanes with cnt > 0 are a prefix)
		const uint32_t Lj = last_lane_with(cnt);
		const uint32_t j = Lj * CPL + lane_value(cnt, Lj) - 1u;
		pj = lane_value(pj, Lj);
		nzj = lane_value(nzj, Lj);
		nsjj = nzj >> PECH_NS_SHIFT;
		nzj &= PECH_NZ_MASK;
		jj = j;
		pjj = pj;
		nzjj = nzj;
		const uint32_t rr = r0 - pj;
#ifdef PECH_LR4_LAZY // A/B: no speculative row offsets (a whole 4 KiB per wave through the TA at entry)
		if (lane * 16u < nzj) {
#else
		if (j != cg && lane * 16u < nzj) { // speculation missed: the start chunk's row offsets now
#endif
#pragma unroll
			for (uint32_t k = 0; k < 4; ++k)
				lr4[k] = ((const u32x4 *)(lrs + j * PECH_CHUNK + lane * 16u))[k];
		}
		// position: the count of the chunk's offsets <= rr (nondecreasing
		// over its nz non-empty cores), and the row inside that buffer
		uint32_t c2 = 0, lo = 0;
#pragma unroll
		for (uint32_t k = 0; k < 16; ++k) {
			const uint32_t e = lr4[k >> 2][k & 3u];
			const bool ok = lane * 16u + k < nzj && e <= rr;
			c2 += ok ? 1u : 0u;
			lo = ok ? max(lo, e) : lo;
		}
		// (offsets increase over the non-empty cores: the lanes with c2 > 0
		// are a prefix, and the last of them holds the largest offset <= rr)
		const uint32_t Lp = last_lane_with(c2);
		const uint32_t cpos = Lp * 16u + lane_value(c2, Lp);
		p0 = j * PECH_CHUNK + cpos - 1u;
		lr0 = rr - lane_value(lo, Lp);
#ifdef PECH_DEBUG_BOUNDS
		if (lane == 0 && (j >= nchunks || cpos == 0 || cpos > nzj || lr0 >= cores[p0].rows))
			printf("PECH OOB prologue blk %u wave %u r0 %u j %u cg %u nchunks %u nzj %u cpos %u rr %u rows %u\n",
			       blockIdx.x, wave, r0, j, cg, nchunks, nzj, cpos, rr, cores[min(p0, nchunks * PECH_CHUNK - 1u)].rows);
#endif
	}
	st.U0 = U0;
	st.p0 = p0;
	st.lr0 = lr0;
	st.jj = jj;
	st.pjj = pjj;
	st.nzjj = nzjj;
	st.nsjj = nsjj;
	return true;
}

// The flat prologue (pech_crc32c_flat): lane l holds descriptors 4l .. 4l+3
// (dv, loaded at entry with the tables).  Every wave computes their rows,
// scans them itself (DPP), takes its share (wave_share) and finds the
// position holding its first row with one ballot -- no plan kernel, no
// workspace reads.  It also writes the batch's LDS table (flat_core): all of
// it, the same values in every wave, read back only from its own writes
// until the workgroup's barrier.  Rtot: the launch's rows (the early table
// fill's exact size).  Uniform (every buffer the same rows, none empty):
// position p holds rows [p U0, (p+1) U0), as the pool needs.
__device__ __forceinline__ bool prologue_flat(uint32_t *lds, const u32x4 (&dv)[4], uint32_t n, uint32_t lane,
					      uint32_t wave, uint32_t W, uint32_t rpw_min, Start &st, uint32_t &Rtot,
					      bool il_req)
{
	uint32_t rows[4], lsum = 0;
#pragma unroll
	for (uint32_t k = 0; k < 4; ++k) {
		const uint32_t p = 4u * lane + k, lb = dv[k].x & (PECH_ROW_BYTES - 1u), len = dv[k].z;
		rows[k] = p < n && len ? (uint32_t)(((uint64_t)lb + len + PECH_ROW_BYTES - 1u) >> 7) : 0u;
		lsum += rows[k];
		if (p < n) { // T: zero bytes after the buffer in its last line
			const uint32_t T = rows[k] ? rows[k] * PECH_ROW_BYTES - lb - len : 0u;
			*(u32x4 *)(lds + L_FLAT / 4u + 4u * p) = u32x4{dv[k].x, dv[k].y, rows[k], p | T << 20};
		}
	}
	const uint32_t incl = wave_incl_scan(lsum);
	Rtot = lane_value(incl, 63);
	STAMP(t_scan);
#ifdef PECH_STAMPS
	st.t_scan = t_scan;
#endif
	const uint32_t U0 = lane_value(rows[0], 0);
	bool uok = true;
#pragma unroll
	for (uint32_t k = 0; k < 4; ++k)
		uok = uok && (4u * lane + k >= n || rows[k] == U0);
	const bool uniform = U0 != 0u && __ballot(!uok) == 0ull;
	// host-resident slots (il_req): a uniform batch of buffers of at least
	// PECH_IL_MIN_ROWS rows walks interleaved rows, as the fused copy does
	// (the workgroup's 128 groups over one portion, 16 KiB per row step):
	// GPU reads of pinned host memory in static slices touch 32K pages at
	// once and reach 45-48 GB/s, interleaved 50-56 GB/s, the copy engines'
	// rate (tools/host_probe.hip, profiles/r06/host_probe.txt)
	const bool il = il_req && uniform && U0 >= PECH_IL_MIN_ROWS;
	if (!wave_share<false>(Rtot, W, rpw_min, wave, uniform, il, st))
		return false; // whole workgroup idle (small batch)
	st.U0 = U0;
	st.p0 = st.lr0 = 0;
	st.jj = st.pjj = st.nzjj = st.nsjj = 0;
	if (st.rem_all && !il) {
		// the one position p with prefix(p) <= r0 < prefix(p) + rows(p)
		const uint32_t r0 = st.r0;
		uint32_t pre = incl - lsum, hk = 4u, lr = 0;
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) {
			const bool h = rows[k] != 0u && pre <= r0 && r0 - pre < rows[k];
			hk = h ? k : hk;
			lr = h ? r0 - pre : lr;
			pre += rows[k];
		}
		const uint32_t L = (uint32_t)__builtin_ctzll(__ballot(hk < 4u) | (1ull << 63));
		st.p0 = 4u * L + lane_value(hk, L);
		st.lr0 = lane_value(lr, L);
#ifdef PECH_DEBUG_BOUNDS
		if (lane == 0 && (st.p0 >= n || lane_value(hk, L) >= 4u))
			printf("PECH OOB flat prologue blk %u wave %u r0 %u p0 %u n %u\n", blockIdx.x, wave, r0, st.p0, n);
#endif
	}
	return true;
}

// Large flat batches (pech_crc32c_flatg, n <= PECH_FLATG_MAX = 4,096): thread
// t of the workgroup holds positions 4t .. 4t+3 (dv, loaded at entry with the
// tables).  Each wave scans its threads' rows (DPP), writes its lanes'
// in-wave prefixes (L_FLAT, 4 KiB) and its total, smallest / largest row
// count and seed flag (L_SCAN); after ONE workgroup barrier every wave knows
// Rtot, the wave offsets and uniformity, takes its share (wave_share) and
// finds the position holding its first row: the last thread whose prefix
// is <= r0 (a count over the 1,024 prefixes, 16 per lane), then that thread's
// 4 descriptors by scalar loads.  No per-position table: steps read the
// descriptors themselves (flatg_core).  Nothing here is written by the
// tables' fill, so no second barrier.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v)
{
#pragma unroll
	for (uint32_t d = 1; d < 64u; d <<= 1)
		v = min(v, (uint32_t)__shfl_xor((int)v, (int)d));
	return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
#pragma unroll
	for (uint32_t d = 1; d < 64u; d <<= 1)
		v = max(v, (uint32_t)__shfl_xor((int)v, (int)d));
	return v;
}

__device__ __forceinline__ bool prologue_flatg(uint32_t *lds, const u32x4 (&dv)[4], const pech_desc *__restrict__ descs,
					       uint32_t n, uint32_t tid, uint32_t lane, uint32_t wave, uint32_t W,
					       uint32_t rpw_min, Start &st, uint32_t &Rtot, bool &seeds)
{
	static_assert(PECH_FLATG_MAX == 4u * PECH_MAIN_THREADS, "flatg: 4 positions per thread of the workgroup");
	uint32_t rows[4], tsum = 0, rmin = 0xFFFFFFFFu, rmax = 0;
	bool sd = false;
#pragma unroll
	for (uint32_t k = 0; k < 4; ++k) {
		const uint32_t p = 4u * tid + k, lb = dv[k].x & (PECH_ROW_BYTES - 1u), len = dv[k].z;
		rows[k] = p < n && len ? (uint32_t)(((uint64_t)lb + len + PECH_ROW_BYTES - 1u) >> 7) : 0u;
		tsum += rows[k];
		rmin = p < n ? min(rmin, rows[k]) : rmin;
		rmax = p < n ? max(rmax, rows[k]) : rmax;
		sd = sd || (p < n && dv[k].w != 0u);
		keep_whole(dv[k]);
	}
	const uint32_t incl = wave_incl_scan(tsum);
	lds[L_FLAT / 4u + tid] = incl - tsum; // the thread's prefix inside its wave
	rmin = wave_min_u32(rmin);
	rmax = wave_max_u32(rmax);
	const bool wsd = __ballot(sd) != 0ull;
	if (lane == 63u) {
		lds[L_SCAN / 4u + wave] = incl;
		lds[L_SCAN / 4u + 16u + wave] = rmin;
		lds[L_SCAN / 4u + 32u + wave] = rmax;
		lds[L_SCAN / 4u + 48u + wave] = wsd;
	}
	__syncthreads();
	STAMP(t_scan);
#ifdef PECH_STAMPS
	st.t_scan = t_scan;
#endif
	// one LDS word per lane (lanes 0-15 the waves' totals, 16-31 their
	// smallest and 32-47 their largest rows, 48-63 their seed flags) and lane
	// operations: 64 broadcast reads per wave, all 16 waves at once behind the
	// barrier, kept the LDS pipe busy ~0.8 us
	const uint32_t sw = lds[L_SCAN / 4u + lane];
	const uint32_t tw = lane < PECH_MAIN_WAVES ? sw : 0u;
	const uint32_t tinc = wave_incl_scan(tw);
	Rtot = lane_value(tinc, PECH_MAIN_WAVES - 1u);
	// the waves before the one of threads 16 lane .. 16 lane + 15 (lane >> 2)
	const uint32_t woff = (uint32_t)__shfl((int)(tinc - tw), (int)(lane >> 2));
	seeds = __ballot(lane >= 48u && sw != 0u) != 0ull;
	// uniform: every wave holding positions has min = max = wave 0's min
	const uint32_t nw = (n + 255u) >> 8, m0 = lane_value(sw, 16u);
	const bool mine = (lane >= 16u && lane < 16u + nw) || (lane >= 32u && lane < 32u + nw);
	const bool uniform = m0 != 0u && __ballot(mine && sw != m0) == 0ull;
	const uint32_t U0 = uniform ? m0 : uni(wave_min_u32(lane >= 16u && lane < 32u ? sw : 0xFFFFFFFFu));
	if (!wave_share<false>(Rtot, W, rpw_min, wave, uniform, false, st))
		return false; // whole workgroup idle (small batch)
	st.U0 = U0;
	st.p0 = st.lr0 = 0;
	st.jj = st.pjj = st.nzjj = st.nsjj = 0;
	if (st.rem_all && uniform) {
		// position p holds rows [p U0, (p+1) U0): no search, no loads
		st.p0 = st.r0 / U0;
		st.lr0 = st.r0 - st.p0 * U0;
	} else if (st.rem_all) {
		const uint32_t r0 = st.r0;
		// threads whose prefix is <= r0: the last of them holds r0 (a thread
		// with no rows before it shares the next one's prefix, which is > r0)
		uint32_t cnt = 0;
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q) {
			const u32x4 v = *(const u32x4 *)(lds + L_FLAT / 4u + 16u * lane + 4u * q);
			cnt += (woff + v.x <= r0) + (woff + v.y <= r0) + (woff + v.z <= r0) + (woff + v.w <= r0);
		}
		const uint32_t ts = lane_value(wave_incl_scan(cnt), 63) - 1u;
		// + the waves before ts's: lane ts / 16's woff (its 16 threads are ts's wave's)
		const uint32_t acc0 = uni(lds[L_FLAT / 4u + ts] + lane_value(woff, ts >> 4));
		uint32_t acc = acc0;
		uint32_t p0 = 4u * ts, lr0 = 0;
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) { // scalar loads: the thread's four descriptors
			const uint32_t p = 4u * ts + k;
			const u32x4 d = ((const u32x4 *)descs)[uni(min(p, n - 1u))];
			const uint32_t lb = d.x & (PECH_ROW_BYTES - 1u);
			const uint32_t r = p < n && d.z ? (uint32_t)(((uint64_t)lb + d.z + PECH_ROW_BYTES - 1u) >> 7) : 0u;
			const bool h = r != 0u && acc <= r0 && r0 - acc < r;
			p0 = h ? p : p0;
			lr0 = h ? r0 - acc : lr0;
			acc += r;
		}
		st.p0 = uni(p0);
		st.lr0 = uni(lr0);
#ifdef PECH_DEBUG_BOUNDS
		if (lane == 0 && (st.p0 >= n || ts >= PECH_MAIN_THREADS))
			printf("PECH OOB flatg prologue blk %u wave %u r0 %u p0 %u ts %u n %u\n", blockIdx.x, wave, r0, st.p0, ts, n);
#endif
	}
	return true;
}

// FLAT (pech_crc32c_flat): the same walk for n <= PECH_FLAT_MAX buffers with
// no plan kernel -- the descriptors are read at entry (descs) and kept in LDS
// (prologue_flat), and out[] is zeroed inside the launch, published through
// *flag (below).
//
// *flag, a word of the caller's workspace, holds FLAT_INIT(tag) while a wave
// of the launch initialises out[] and FLAT_DONE(tag) once it has; any other
// value is a previous launch's (or the garbage of a fresh workspace: the host
// gives every flat launch a fresh tag, below 2^62).  Workgroup 0's first
// wave claims the job at entry (an exchange); any wave that reaches its first
// XOR into out[] before FLAT_DONE and finds no claim of this launch claims it
// itself (a compare-and-swap from the value it read) -- so waves only ever
// wait for a wave that is running and initialising, never for workgroup 0 to
// be dispatched.  (Waiting for workgroup 0 deadlocked two concurrent flat
// launches on one GPU: each one's waiting workgroups held the CUs the other's
// workgroup 0 needed, until the wait's bound let them go on with out[]
// uninitialised -- found by test_torchrun_two_ranks_real_kernels.)
#define FLAT_INIT(tag) ((tag) << 1)
#define FLAT_DONE(tag) (((tag) << 1) | 1ull)

// The status word of a flat launch (hstat: coherent pinned host memory the
// caller reads after the launch has completed; layout.h PECH_FLAT_PUB/ERR).
// A wave that gave up waiting for out[]'s initialisation has XORed into
// words that may not have been zeroed: it records the launch's tag in the
// workspace's error word (ws word 2), counts the launch in pech_flat_faults
// (first wave only) and stores PECH_FLAT_ERR(tag) to hstat, so no caller
// takes the launch's results -- the library recomputes or fails the batch
// (the reference cannot produce a wrong CRC, and a wrong one
// would fault the connection: messenger.c:2826-2842).  The publisher of an
// async slot's results (flat_publish) ends with PECH_FLAT_PUB(tag), or with
// PECH_FLAT_ERR(tag) when the error word holds this launch's tag.
__device__ unsigned long long pech_flat_faults;
extern "C" int pech_read_flat_faults(uint64_t *host)
{
	return hipMemcpyFromSymbol(host, HIP_SYMBOL(pech_flat_faults), sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
__device__ __forceinline__ void flat_fault(uint64_t *flag, uint64_t *hstat, uint64_t tag, uint32_t lane)
{
	if (lane == 0) {
		const uint64_t prev = atomicExch((unsigned long long *)(flag + 2), (unsigned long long)tag);
		if (prev != tag)
			atomicAdd(&pech_flat_faults, 1ull);
		if (hstat)
			__hip_atomic_store(hstat, PECH_FLAT_ERR(tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	}
#ifdef PECH_DEBUG_BOUNDS
	if (lane == 0)
		printf("PECH OOB flat out[] never initialised blk %u\n", blockIdx.x);
#endif
}

// The claimed job: zeroes (device-scope atomic exchanges: every access to
// out[] in the launch is a device-scope atomic, ordered at the word itself),
// the seed terms x^(8 len) s of R(s, D) = x^(8|D|) s ^ R(0, D) after them (the
// seed itself for an empty buffer; the messenger's seeds are 0: nothing to
// do), then FLAT_DONE (a release store).  No acquire on the readers' side:
// they only XOR, after they read FLAT_DONE.  (An acquire there was an L2
// invalidate per wave: +6.5 us per C3 launch.)  (The descriptors are read
// again here, in this rare path, when there are seeds: kept in registers for
// it, they pushed the kernel past 128 VGPRs.)  NMAX: the kernel's batch limit
// (PECH_FLAT_MAX, or PECH_FLATG_MAX for pech_crc32c_flatg).
template <uint32_t NMAX>
__device__ __forceinline__ void flat_init(const pech_desc *__restrict__ descs, uint32_t n, uint32_t lane,
					  const uint32_t *__restrict__ consts, uint32_t *__restrict__ out, uint64_t *flag,
					  uint64_t tag, bool seeds)
{
	if constexpr (NMAX <= PECH_FLAT_MAX) {
#pragma unroll
		for (uint32_t k = 0; k < NMAX / 64u; ++k)
			if (64u * k + lane < n)
				(void)atomicExch(out + 64u * k + lane, 0u);
	} else {
		// flatg: up to 64 words per lane, in a loop over the batch's own words
		// (unrolled to NMAX, their addresses were hoisted out of the step loop
		// that calls this and spilled), four exchanges in flight per turn
		uint32_t *o = out + lane;
#pragma unroll 1
		for (uint32_t k = 0; 64u * k < n; k += 4u, o += 256u) {
#pragma unroll
			for (uint32_t j = 0; j < 4u; ++j)
				if (64u * (k + j) + lane < n)
					(void)atomicExch(o + 64u * j, 0u);
		}
	}
	if (seeds) {
		__threadfence(); // the zeroes are performed before the seed terms land on the same words
#pragma unroll 1
		for (uint32_t k = 0; k < NMAX / 64u; ++k) {
			const uint32_t p = 64u * k + lane;
			if (p >= n)
				break;
			const u32x4 d = ((const u32x4 *)descs)[p];
			if (d.w != 0u)
				atomicXor(out + p, d.z ? shift_bytes(consts + PECH_C_POWB, d.z, d.w) : d.w);
		}
	}
	if (lane == 0) {
		(void)atomicExch((uint32_t *)(flag + 1), 0u); // the publication count (flat_publish)
		__hip_atomic_store(flag, FLAT_DONE(tag), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
	}
}

// Before a wave's first XOR into out[]: `ready` once it has read FLAT_DONE
// (normally from its early load, issued with the ring's prime and looked at
// behind the tables' barrier, so it costs no wait); otherwise poll -- and
// claim the job when no wave of this launch has (see above).  Each poll is
// consumed before the loop can exit, so no load of this rare path is left
// pending at the step loop's join, where the compiler would wait for it with
// a vmcnt(0), i.e. drain the ring at every step end.  (Bounded: a wave never
// waits forever; after ~1 s it records the launch as faulted (flat_fault)
// and goes on, and no caller takes the launch's results.)  `test` (the
// test library's fault hook, 0 from the release library):
// PECH_FLAT_T_TIMEOUT makes every wave that reaches this wait take the
// timeout at once.
template <uint32_t NMAX>
__device__ __forceinline__ void flat_ready(uint64_t *flag, uint64_t tag, bool &ready,
					   const pech_desc *__restrict__ descs, uint32_t n, uint32_t lane,
					   const uint32_t *__restrict__ consts, uint32_t *__restrict__ out, bool seeds,
					   uint64_t *hstat, uint32_t test)
{
	if (ready)
		return;
	const bool force = test & PECH_FLAT_T_TIMEOUT;
	for (uint32_t spin = 0;; ++spin) {
		const uint64_t v = uni64(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
		if (v == FLAT_DONE(tag) && !force)
			break;
		if ((v >> 1) != tag) { // no claim of this launch: claim it
			uint64_t got = 0;
			if (lane == 0)
				got = atomicCAS((unsigned long long *)flag, (unsigned long long)v, (unsigned long long)FLAT_INIT(tag));
			if (uni64(got) == v) {
				flat_init<NMAX>(descs, n, lane, consts, out, flag, tag, seeds);
				break;
			}
			continue; // another wave claimed it first
		}
		if (spin >= (1u << 24) || force) {
			flat_fault(flag, hstat, tag, lane);
			break;
		}
		__builtin_amdgcn_s_sleep(2); // FLAT_INIT: a running wave is at it
	}
	ready = true;
}

// Flat launches for the async layer (hout != NULL): the results go to the
// slot's pinned host array from the kernel itself, instead of a copy after
// it (a blit kernel, 4.2-4.4 us per lone payload on the stream, plus its
// dispatch; profiles/r05/lat_prof.txt).  Each live workgroup's last wave,
// once every XOR of its workgroup is performed, counts itself in (flag + 1);
// the last of the nlive reads out[] at L2 and stores it to hout.  (The count
// is zeroed by flat_init, before FLAT_DONE, and a workgroup counts only
// after it has read FLAT_DONE.)  "Performed": each wave waits for its own
// atomics' acknowledgements (vm_done) before the workgroup's LDS count --
// device-scope atomics are performed at L2, where every later atomic and
// L2 load sees them.  An agent-scope release fence would do it too, but it
// writes L2 back (buffer_wbl2) in every wave: lone 1 MiB payloads 48 -> 86 us.
__device__ __forceinline__ void vm_done()
{
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// The results are followed by the launch's status word (hstat): the caller
// takes hout only when it reads PECH_FLAT_PUB(tag) there, so a publication
// that did not happen -- the nlive miscount of v0.32's first build, which
// left 137 of 200 msgr_sim payloads with a previous batch's results -- is a
// detected event, not stale CRCs.  The host reads hstat
// after the launch has completed, which orders every store of the kernel.
// (PECH_FLAT_T_NOPUB, test library only: the publication is skipped.)
template <uint32_t NMAX>
__device__ __forceinline__ void flat_publish(uint64_t *flag, uint32_t nlive, uint32_t n, uint32_t lane,
					     uint32_t *__restrict__ out, uint32_t *__restrict__ hout, uint64_t *hstat,
					     uint64_t tag, uint32_t test)
{
	vm_done(); // (the flush's XORs; or, with nlive 0, flat_init's zeroes and seeds)
	if (nlive) { // (0: a launch without rows, published by the wave that initialised out[])
		uint32_t c = 0;
		if (lane == 0)
			c = atomicAdd((uint32_t *)(flag + 1), 1u);
		if (uni(c) + 1u != nlive)
			return;
	}
	if (test & PECH_FLAT_T_NOPUB)
		return;
	asm volatile("" ::: "memory");
#pragma unroll(NMAX <= PECH_FLAT_MAX ? NMAX / 64u : 1u)
	for (uint32_t k = 0; 64u * k < n; ++k) {
		const uint32_t p = 64u * k + lane;
		if (p < n)
			hout[p] = __hip_atomic_load(out + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	if (lane == 0 && hstat) {
		// a wave of this launch that gave up on out[]'s initialisation has
		// recorded the tag before it counted in (its own vm_done)
		const uint64_t e = __hip_atomic_load(flag + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		__hip_atomic_store(hstat, e == tag ? PECH_FLAT_ERR(tag) : PECH_FLAT_PUB(tag), __ATOMIC_RELAXED,
				   __HIP_MEMORY_SCOPE_SYSTEM);
	}
}

template <bool COPY, uint32_t U, bool FLAT = false, bool FLATG = false, bool FIL = false>
__device__ __forceinline__ void main_body(uint32_t *lds, const pech_core *__restrict__ cores,
					  const uint32_t *__restrict__ lrs, const uint32_t *__restrict__ partials,
					  const uint32_t *__restrict__ nzs, uint32_t n,
					  const uint32_t *__restrict__ consts, uint32_t *__restrict__ out, uint32_t rpw_min,
					  const int64_t *__restrict__ deltas, const pech_desc *__restrict__ descs = nullptr,
					  uint64_t *flag = nullptr, uint64_t tag = 0, uint32_t *__restrict__ hout = nullptr,
					  uint64_t *hstat = nullptr, uint32_t test = 0u)
{
	static_assert(!(FLAT && COPY), "flat batches: CRC only");
	static_assert(FLAT || !FLATG, "FLATG is a flat mode");
	static_assert(!FIL || (FLAT && !FLATG), "FIL: the flat kernel's interleaved-rows variant");
	constexpr uint32_t NMAX = FLATG ? PECH_FLATG_MAX : PECH_FLAT_MAX; // flat: the launch's batch limit
	const uint32_t tid = threadIdx.x;
	// flat steps read {addr, rows, meta} per position: FLATG from the caller's
	// descriptors (flatg_core), FLAT from the wave's LDS table
	const pech_core *const gdesc = FLATG ? (const pech_core *)descs : cores;
	STAMP(t_entry);
#ifdef PECH_KARGS_AT_ENTRY
	// every kernel argument in SGPRs at entry, in one scalar round: on demand,
	// LLVM loaded them in three rounds, each gating the next group of the
	// prologue's vector loads (kernarg reads are scalar-cache misses at entry)
	asm volatile("" ::"s"(cores), "s"(lrs), "s"(partials), "s"(nzs), "s"(n), "s"(consts), "s"(out), "s"(rpw_min),
		     "s"(deltas));
#endif
	const uint32_t lane = tid & 63u, g8 = tid & 7u, grp = lane >> 3;
	const uint32_t lreg = ((lane & 31u) << 2) | (1u << 16);
	const uint32_t wave = uni(tid >> 6);
	const uint32_t W = gridDim.x * PECH_MAIN_WAVES;
	const uint32_t nchunks = (n + PECH_CHUNK - 1u) / PECH_CHUNK;
	// Flat: workgroup 0's first wave claims the initialisation of out[] first
	// thing (an exchange; its result is looked at once the descriptors are
	// in, which the seed terms need); see flat_init
	uint64_t claim0 = 0;
	bool seeds = false; // flat: some buffer of the batch has a seed
	if constexpr (FLAT) {
		if (blockIdx.x == 0 && wave == 0 && lane == 0)
			claim0 = atomicExch((unsigned long long *)flag, (unsigned long long)FLAT_INIT(tag));
	}

	// Prologue (v0.11): three dependent global rounds before the first data
	// instead of four, and no barrier until the ring is primed.  Every wave
	// issues at entry, all in flight together:
	//   the table constants (written to LDS only after the prime, from
	//   registers: issued first, their wait never drains the ring),
	//   every chunk's row total and non-empty count (16 chunks per lane: the
	//   wave scans them itself -- no workgroup scan, no barrier),
	//   the row offsets of the chunk it most likely starts in, and the
	//   descriptors of the 8 buffers at its likely start position
	//   (speculative: exact for uniform batches; reloaded if wrong).
	// Only the lanes whose entries exist load (every wave reads the same
	// chunk totals: whole-array loads were 32 MiB of L2 reads per launch).
	static_assert(1024u % PECH_MAIN_THREADS == 0u, "table fill: A_128 words split evenly over the threads");
	static_assert(PECH_MAX_CHUNKS == 64u * 16u, "wave scan: 16 chunks per lane");
	static_assert(PECH_CHUNK == 64u * 16u, "find: 16 row offsets per lane");
	constexpr uint32_t T128 = 1024u / PECH_MAIN_THREADS; // A_128 words per thread
	constexpr uint32_t NT4 = (PECH_C_TAB1 - PECH_C_TAB4) / 4u; // single-copy tables, 16-B words
	constexpr uint32_t TPT = (NT4 + PECH_MAIN_THREADS - 1u) / PECH_MAIN_THREADS;
	const u32x4 *c4 = (const u32x4 *)(consts + PECH_C_TAB4);
	uint32_t t128[T128], t16k[T128];
	u32x4 tv[TPT];
	uint32_t txi;
	static_assert(PECH_MAIN_THREADS >= 128u, "inverse powers: one word per thread");
	auto load_consts = [&]() {
#pragma unroll
		for (uint32_t j = 0; j < T128; ++j) {
			t128[j] = consts[PECH_C_TAB128 + tid + j * PECH_MAIN_THREADS];
			t16k[j] = COPY || PECH_IL_CRC || FIL ? consts[PECH_C_TAB16K + tid + j * PECH_MAIN_THREADS]
									   : 0u; // interleaved mode's table
		}
#pragma unroll
		for (uint32_t k = 0; k < TPT; ++k)
			tv[k] = c4[min(tid + k * PECH_MAIN_THREADS, NT4 - 1u)];
		txi = consts[PECH_C_XINV + (tid & 127u)];
	};
#ifndef PECH_CONSTS_LAST
	load_consts();
#endif
	uint32_t rows0 = 0, pg = 0, cg = 0, lrg = 0;
	pech_core spec = pech_core{};
	u32x4 lr4[4], dv[4], gspec = (u32x4)(0u);
	if constexpr (FLATG) {
		// the batch's descriptors, 4 per THREAD of the workgroup (64 contiguous bytes), with the tables
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k)
			dv[k] = ((const u32x4 *)descs)[min(4u * tid + k, n - 1u)];
		// and the first step's, one per lane group, at the likely start
		// position (exact for uniform batches, as the planned kernel's spec):
		// the step after the prologue's barrier then plans without a load
		pg = uni(min((uint32_t)((double)(blockIdx.x * PECH_MAIN_WAVES + wave) * (double)n / (double)W), n - 1u));
		gspec = ((const u32x4 *)descs)[min(pg + grp, n - 1u)];
	} else if constexpr (FLAT) {
		// the batch's descriptors, 4 per lane (64 contiguous bytes), with the tables
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k)
			dv[k] = ((const u32x4 *)descs)[min(4u * lane + k, n - 1u)];
	} else {
		rows0 = uni(partials[0]); // chunk 0's rows (the early fill's launch-size estimate)
		// the speculative start (below), its chunk's row offsets, then the chunk totals
		const uint32_t wglob = blockIdx.x * PECH_MAIN_WAVES + wave;
		// likely start position: exact for uniform batches (a double quotient of
		// integers is exact when it is one; a near miss only costs a reload)
		pg = uni(min((uint32_t)((double)wglob * (double)n / (double)W), n - 1u));
		cg = pg >> 10;   // and chunk
		lrg = lrs[pg]; // pg's row offset in its chunk
		// cores[pg + grp] (pg + 7 may run into lrs: workspace memory, used only if in the chunk)
		spec = load_spec(cores, pg + grp);

		// the speculative row offsets.  Unconditional -- a load under a branch
		// gets a vmcnt(0) at the join -- with lanes past the chunk's buffers
		// reading lane 0's lines (no extra traffic; masked later).
#ifndef PECH_LR4_LAZY
		{
			const uint32_t ll = lane * 16u < n - cg * PECH_CHUNK ? lane : 0u;
#pragma unroll
			for (uint32_t k = 0; k < 4; ++k)
				lr4[k] = ((const u32x4 *)(lrs + cg * PECH_CHUNK + ll * 16u))[k];
		}
#else
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k)
			lr4[k] = (u32x4)(0u);
#endif
	}
#ifdef PECH_CONSTS_LAST // A/B: the tables' loads after the ones the scan and the start search wait for
	load_consts();
#endif
	STAMP(t_issued);
	// The LDS tables.  A_128 once per bank: its 32 copies as 8 x 16 B; lane t
	// starts at copy group t mod 8 so neighbouring lanes, whose rows are
	// 256 B apart, write different banks.  Then the single-copy tables and
	// the empty deferral table.
	auto fill_tables = [&](bool il_tab) {
#pragma unroll
		for (uint32_t j = 0; j < T128; ++j) {
			const uint32_t w = tid + j * PECH_MAIN_THREADS, k = w >> 8, e = w & 0xFFu;
			const u32x4 v = (u32x4)(il_tab ? t16k[j] : t128[j]);
			char *dst = (char *)lds + (k >> 1) * 65536u + e * 256u + (k & 1u) * 128u;
#pragma unroll
			for (uint32_t q = 0; q < 8u; ++q)
				*(u32x4 *)(dst + 16u * ((q + w) & 7u)) = v;
		}
#pragma unroll
		for (uint32_t k = 0; k < TPT; ++k)
			if (tid + k * PECH_MAIN_THREADS < NT4)
				*(u32x4 *)((char *)lds + L_TAB4 + 16u * (tid + k * PECH_MAIN_THREADS)) = tv[k];
		if (tid < 128u)
			lds[L_XINV / 4u + tid] = txi;
		if (tid == 0)
			lds[L_POOL / 4u] = 0u;
		if (tid < PECH_DEFER_SLOTS) {
			lds[L_DEFER / 4u + tid] = PECH_DEFER_EMPTY;
			lds[L_DEFER / 4u + PECH_DEFER_SLOTS + tid] = 0u;
			if (tid == 0)
				lds[L_DEFER_DONE / 4u] = 0u;
		}
	};

	// The chunk scan and the start search (prologue_start): four chunks per
	// lane for batches of up to 256 chunks (262,144 buffers), sixteen beyond.
	// Every wave of the CU runs it, so its instruction count is the prologue's
	// cost: a wave64 VALU instruction issues every 4 cycles per SIMD and four
	// waves share a SIMD (the 16-per-lane loops alone were ~1 us of it).
	// Launches of up to about PECH_EARLY_FILL_ROWS rows per workgroup (128
	// MiB on 256 CUs; estimated from chunk 0's rows, exact for uniform
	// batches): the CRC kernel (one table set) writes and publishes the LDS
	// tables as soon as they arrive -- with the chunk totals the scan waits
	// for -- and each wave then streams as soon as its own prime lands.  With
	// the barrier after the prime every wave waits for the workgroup's
	// slowest prologue: 4 MiB launches 25.4 -> 21.7 us.  Larger launches keep
	// it, fill included: there a fill before the scan cost +1.2 us per
	// launch, and without the barrier the early starters took issue slots
	// from the waves still in their prologue and the tail grew
	// (profiles/r04/ab_early_fill.txt).  The copy kernel's table depends on
	// the scan (interleaved mode): late fill.
	// The estimate's limit: it is chunk 0's rows times the chunk
	// count, so a skewed batch -- small buffers in its first 1,024, large ones
	// after -- can take the early fill at a size where the late one is faster
	// (a tail ~1 us longer, never a wrong result).  The exact total would
	// need a load after the scan, i.e. a round trip before the fill on every
	// planned launch; the messenger's and the benchmarks' batches are not
	// skewed that way.  (Flat batches fill late at every size.)
	Start sv;
	bool early_fill, live;
	if constexpr (FLAT) {
		uint32_t Rtot;
		if constexpr (FLATG) {
			// the tables go in before the prologue's barrier, which publishes
			// them with the scan: flatg's only barrier (a fill behind the prime
			// would take a second one, 1.5 us p50 in 256 MiB launches)
			fill_tables(false);
			live = prologue_flatg(lds, dv, descs, n, tid, lane, wave, W, rpw_min, sv, Rtot, seeds);
		} else {
			live = prologue_flat(lds, dv, n, lane, wave, W, rpw_min, sv, Rtot, FIL && (test & PECH_FLAT_F_IL));
			seeds = __ballot((4u * lane < n && dv[0].w) || (4u * lane + 1u < n && dv[1].w) ||
					 (4u * lane + 2u < n && dv[2].w) || (4u * lane + 3u < n && dv[3].w)) != 0ull;
		}
		if (blockIdx.x == 0 && wave == 0) {
			// (lane 0's exchange: a claim of this launch already there -- another
			// wave got in first -- leaves the job to it; a FLAT_DONE it
			// overwrote goes back)
			const uint64_t c0 = lane_value((uint32_t)claim0, 0) | (uint64_t)lane_value((uint32_t)(claim0 >> 32), 0) << 32;
			if ((c0 >> 1) != tag)
				flat_init<NMAX>(descs, n, lane, consts, out, flag, tag, seeds);
			else if (c0 == FLAT_DONE(tag) && lane == 0)
				__hip_atomic_store(flag, FLAT_DONE(tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		if (hout && Rtot == 0u && blockIdx.x == 0 && wave == 0) // no rows at all: out[] holds the seeds (flat_init above)
			flat_publish<NMAX>(flag, 0u, n, lane, out, hout, hstat, tag, test);
		if (!live)
			return; // whole workgroup idle (small batch)
		// Flat launches fill late at every size: with the wave-major shares of
		// small launches only ~4 waves per CU stream, and the early fill's
		// barrier after all 16 prologues cost them more than the fill behind
		// their primes (32 MiB 14.1 -> 13.8 us, 4 MiB 10.7 -> 10.4 us,
		// profiles/r05/ab_curve_v30.txt; PECH_FLAT_EARLY_FILL: the old rule)
#ifdef PECH_FLAT_EARLY_FILL
		early_fill = !PECH_IL_CRC && Rtot <= (uint64_t)PECH_EARLY_FILL_ROWS * gridDim.x; // workgroup-uniform
#else
		early_fill = false;
#endif
		if (FLATG) {
			early_fill = true; // (filled and published above)
		} else if (early_fill) {
			fill_tables(false);
			__syncthreads();
		}
	} else {
		early_fill = !COPY && !PECH_IL_CRC &&
			     (uint64_t)rows0 * nchunks <= (uint64_t)PECH_EARLY_FILL_ROWS * gridDim.x; // workgroup-uniform
		if (early_fill) {
			fill_tables(false);
			__syncthreads();
		}
		live = nchunks <= 64u * 4u
			       ? prologue_start<COPY, 4>(lds, cores, lrs, partials, nzs, n, nchunks, lane, wave, W, rpw_min, pg,
							 cg, lrg, spec, lr4, sv)
			       : prologue_start<COPY, 16>(lds, cores, lrs, partials, nzs, n, nchunks, lane, wave, W, rpw_min,
							  pg, cg, lrg, spec, lr4, sv);
		if (!live)
			return; // whole workgroup idle (small batch)
	}
#ifdef PECH_STAMPS
	const uint64_t t_scan = sv.t_scan;
#endif
	const uint32_t U0 = sv.U0, wg_rows = sv.wg_rows, r0 = sv.r0, r1 = sv.r1, jmax = sv.jmax;
	const uint64_t wg0 = sv.wg0;
	// (the plain flat kernel never interleaves: a compile-time false keeps its
	// row stride an immediate -- a runtime one cost ~4 us per launch)
	const bool il = FLAT && !FIL ? false : sv.il;
	const uint32_t rsb = il ? PECH_IL_GROUPS * PECH_ROW_BYTES : PECH_ROW_BYTES; // bytes from one row of a run to the next
	uint32_t rem_all = sv.rem_all, p0 = sv.p0, lr0 = sv.lr0;
	const uint32_t jj = sv.jj, pjj = sv.pjj, nzjj = sv.nzjj, nsjj = sv.nsjj;
	u32x4 ring[U];
	// Static shares (no pool): the small cores of a chunk (its first nsjj
	// positions) are walked in whole steps of 8 positions on a grid from the
	// chunk start, each by the wave whose share holds the step's middle row
	// (the first row of its position cnt/2).  A wave starting inside a small
	// step walks it from its start if it owns it, else starts at the next
	// grid point.  Shares cut inside small buffers left a partial first and
	// last step per wave, with idle groups (unaligned 4,100-byte buffers: 2
	// steps per wave became 3, +37 % per launch), and ownership by the first
	// row flipped with +-1 row of jitter when shares and steps nearly align.
	const bool grid = !FLAT && jmax == 0u; // (flat batches keep descriptor order: no size classes)
	if (grid && rem_all) {
		const uint32_t local = p0 & 1023u;
		if (local < nsjj) {
			const uint32_t k0 = local & ~7u, cnt = min(8u, nsjj - k0), k1 = min(nsjj, k0 + 8u);
			// the step's middle row, its first row and the next grid point's,
			// by scalar loads issued together (wave-uniform addresses)
			const uint32_t *cl = lrs + jj * PECH_CHUNK;
			const uint32_t omid = uni(cl[k0 + cnt / 2u]), o0 = uni(cl[k0]);
			const uint32_t o1 = uni(k1 < nzjj ? cl[k1] : partials[jj]);
			const bool own = pjj + omid >= r0;
			const uint32_t roff = pjj + (own ? o0 : o1); // (before r0 if this wave owns the step)
			rem_all = r1 > roff ? r1 - roff : 0u;
			const uint32_t l2 = own ? k0 : k1;
			p0 = l2 < nzjj ? jj * PECH_CHUNK + l2 : (jj + 1u) * PECH_CHUNK;
			lr0 = 0;
		}
	}
	STAMP(t_find);
	if (il) { // the workgroup's whole range, walked by all its waves together
		p0 = (uint32_t)(wg0 / U0);
		lr0 = (uint32_t)(wg0 - (uint64_t)p0 * U0);
		rem_all = wg_rows;
	}
	Step S;
	if constexpr (FLATG) {
		keep_whole(gspec);
		S = plan_step<false, true, true, true>(gdesc, deltas, lds, p0, lr0, rem_all, lane, g8, grp, false,
						       flatg_conv(gspec, min(pg + grp, n - 1u)), pg, n);
	} else if constexpr (FLAT) {
		S = il ? plan_il<false, true>(cores, deltas, p0, lr0, rem_all, wave * 8u + grp, g8, lds)
		       : plan_step<false, false, true, false>(gdesc, deltas, lds, p0, lr0, rem_all, lane, g8, grp, false,
							      pech_core{}, 0u, n);
	} else {
		S = il ? plan_il<COPY>(cores, deltas, p0, lr0, rem_all, wave * 8u + grp, g8)
		       : plan_step<COPY, true>(cores, deltas, lds, p0, lr0, rem_all, lane, g8, grp, grid, spec, pg);
	}
	STAMP(t_plan);
	uint32_t tpow = COPY ? 0u : rowpow(consts, S); // x^(8 128 ra) of the step's run (finish_run)
	// Static shares walk on from where a step ends: the CRC kernel loads the
	// 8 descriptors there (one per group, as `spec`) when it plans a step, so
	// planning the step after it needs no dependent load (the copy kernel has
	// no VGPRs to spare).  nslots - 1 clamps a cursor at the batch end (the
	// 7 entries past it lie in lrs: workspace memory, never used).
	const uint32_t nslots = nchunks * PECH_CHUNK;
#ifndef PECH_NEXT_SPEC_FIRST
	uint32_t nppos = 0xFFFFFFFFu; // (the first step's successor plans with loads)
	pech_core nspec = pech_core{};
	// flatg: the raw descriptors where the first step ends, from the start
	// (a miss in its planner is a vector load, which waits behind the ring);
	// converted when used (flatg_conv)
	u32x4 nspec_g = (u32x4)(0u);
	if constexpr (FLATG) {
		nppos = min(S.pos, n - 1u);
		nspec_g = ((const u32x4 *)descs)[min(nppos + grp, n - 1u)];
	}
#else // A/B: prefetched from the first step on
	uint32_t nppos = COPY ? 0u : min(S.pos, nslots - 1u);
	pech_core nspec = COPY ? pech_core{} : load_spec(cores, nppos + grp);
#endif
	// Flat: workgroup 0 zeroed out[] itself (its first wave, before the
	// barrier below); every other wave reads the flag now, just before its
	// prime, and looks at it behind the tables' fill and barrier (below)
	uint64_t seen = 0;
	bool ready = !FLAT;
	if constexpr (FLAT) {
		// Unconditional, as one block: the flag's wait below then counts the
		// prime's loads after it (vmcnt(7)) and no ring copy joins a path
		// without them -- with a conditional prime the compiler copied the
		// first row's registers right after issuing it, i.e. waited for it
		// before the tables' fill and barrier.  A wave with no step primes
		// from the constants table (valid memory, never used).
		if (!S.T) {
			S.ad = (uint64_t)consts + 16u * g8;
			S.nl = 1;
			S.oz = 0;
#ifdef PECH_DEBUG_BOUNDS
			S.blo = S.ad;
			S.bhi = S.ad + 16u;
#endif
		}
		seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		RING_PRIME_RS(S, ring, rsb);
	} else if (S.T) {
		RING_PRIME_RS(S, ring, rsb);
	}

	// otherwise the tables are written while the prime is in flight
	if (!early_fill)
		fill_tables(il);
	STAMP(t_fill);
	if (!early_fill)
		__syncthreads(); // tables published; every wave's prime is already in flight
	// (looked at only now, the flag's round trip hides behind the fill and
	// the barrier)
	if (FLAT && S.T)
		ready = ready || (uni64(seen) == FLAT_DONE(tag) && !(test & PECH_FLAT_T_TIMEOUT));
	STAMP(t_start);
	// the wave's first pool claim, one item ahead (resolved when its first
	// item is done)
	uint32_t claim = 0, claim2 = 0;
	if (jmax > 1u && lane == 0) {
		claim = atomicAdd(lds + L_POOL / 4u, 1u);
		if (!COPY) // the CRC kernel claims two items ahead: the second one's descriptors are prefetched
			claim2 = atomicAdd(lds + L_POOL / 4u, 1u);
	}
#ifdef PECH_STAMPS
	uint64_t tq[3] = {0, 0, 0};
	uint32_t nstep = 0;
#endif
#ifdef PECH_NO_PRIO // A/B: every wave at the default priority
	constexpr bool prio_on = false;
#else
	// wave-uniform: static shares of at least PECH_PRIO_MIN_SHARE rows (256 MiB
	// launches, 512-row shares, lost 2 % with it: profiles/r05/ab_prio.txt)
	const bool prio_on = !COPY && jmax == 0u && !il && rem_all >= PECH_PRIO_MIN_SHARE;
#endif
	Prio prio = prio_init(rem_all);
#ifndef PECH_NO_PRIO_POOL
	// Pooled walks (uniform batches of buffers of >= PECH_SPLIT_ROWS rows):
	// once a wave's latest claim finds the pool dry, the waves holding the
	// most rows go first.  Claims run two items ahead, so the oldest waves
	// used to finish their last two items first and leave the CU to the
	// youngest: C3 end p50 131 / 141 / 148 / 154 us by age slot, per-CU end
	// spread 25 us; with it 11 us, 162.1 -> 160.6 us per launch, serial
	// +0.9 %, value unchanged (profiles/r05/ab_prio_pool.txt).  (1 GiB of
	// 4 KiB buffers lost 3-4 % of its sustained rate with it.)
	const bool prio_pool = !COPY && jmax > 1u && sv.U0 >= PECH_SPLIT_ROWS;
	if (prio_pool)
		prio = prio_init(2u * PECH_ITEM_ROWS);
	// rows this wave has left: unknown (max) while its latest claim still got an item
	auto pool_left = [&](uint32_t in_step) -> uint32_t {
		const uint32_t c1 = uni(claim), c2 = uni(claim2);
		if (1u + c2 / PECH_MAIN_WAVES < jmax)
			return 0xFFFFFFFFu;
		return in_step + (1u + c1 / PECH_MAIN_WAVES < jmax ? PECH_ITEM_ROWS : 0u);
	};
#else
	constexpr bool prio_pool = false;
	auto pool_left = [](uint32_t in_step) -> uint32_t { return in_step; };
#endif
	while (S.T) {
		if (prio_on)
			prio_update(prio, S.rem + 8u * S.T);
		if (prio_pool)
			prio_update(prio, pool_left(S.rem + 8u * S.T));
		uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
		// row 0's bytes before the buffer are zeros (free: leading zeros):
		// zoff -> the whole piece, zh -> its first zh bytes; on 64-bit halves
		{
			const uint32_t sh = STEP_ZOFF(S) ? 128u : 8u * STEP_ZH(S);
			uint64_t lo = ((uint64_t)ring[0].y << 32) | ring[0].x, hi = ((uint64_t)ring[0].w << 32) | ring[0].z;
			lo &= sh >= 64u ? 0ull : ~0ull << sh;
			hi &= sh >= 128u ? 0ull : (sh <= 64u ? ~0ull : ~0ull << (sh - 64u));
			ring[0] = u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
		}
		const uint32_t nblk = (S.T + U - 1) / U;
		const uint32_t last = S.nl - 1u;
		uint32_t blk = 0;
		// full blocks: every lane's rows valid, prefetch stays inside every run
		for (; blk + 1 < nblk && (blk + 2) * U <= S.nmin; ++blk) {
			const uint64_t base = S.ad + (uint64_t)blk * U * rsb;
			if (prio_on && blk)
				prio_update(prio, S.rem + 8u * (S.T - blk * U));
			if (prio_pool && blk)
				prio_update(prio, pool_left(S.rem + 8u * (S.T - blk * U)));
#if defined(PECH_STAMPS) && !defined(PECH_STAMP_FIN)
			if (nstep == 0 && (blk == nblk / 4u || blk == nblk / 2u || blk == 3u * nblk / 4u))
				tq[blk == nblk / 4u ? 0 : (blk == nblk / 2u ? 1 : 2)] = __builtin_amdgcn_s_memrealtime();
#endif
			if constexpr (COPY) {
				// Block discipline for the fused copy: the block's last row, its U
				// Horner rows, its U stores together, then the next block's first
				// U-1 rows.  vmcnt counts stores too and retires in issue order, so
				// in the rotating ring every load waited behind the stores issued
				// after it (half the lookahead); here a load waits only behind
				// stores issued before it.  Measured: C3 copy 449-465 -> 389-397 us
				// per launch (profiles/r02/ab_copy_block.txt).
				ring[U - 1] = LD_PIECE(S, base + (U - 1) * rsb, 2);
#pragma unroll
				for (uint32_t i = 0; i < U; ++i)
					horner_row(lds, lreg, ring[i], s0, s1, s2, s3);
#pragma unroll
				for (uint32_t i = 0; i < U; ++i)
					st_piece<COPY>(S, blk * U + i, ring[i], S.nu != 0 && (i != 0 || blk != 0 || !STEP_HEAD(S)), rsb);
#pragma unroll
				for (uint32_t i = 0; i + 1 < U; ++i)
					ring[i] = LD_PIECE(S, base + (U + i) * rsb, 2);
				continue;
			}
#pragma unroll
			for (uint32_t i = 0; i < U; ++i) {
				ring[(i + U - 1) % U] = LD_PIECE(S, base + (i + U - 1) * rsb, 2);
				horner_row(lds, lreg, ring[i], s0, s1, s2, s3);
				st_piece<COPY>(S, blk * U + i, ring[i], S.nu != 0 && (i != 0 || blk != 0 || !STEP_HEAD(S)), rsb);
			}
		}
		// ragged blocks: clamped prefetch, predicated update
		for (; blk + 1 < nblk; ++blk) {
			const uint32_t r = blk * U;
			if constexpr (COPY) { // block discipline (see the full blocks), clamped and predicated
				ring[U - 1] = LD_PIECE(S, row_addr(S.ad, min(r + U - 1, last), STEP_ZOFF(S), rsb), 3);
#pragma unroll
				for (uint32_t i = 0; i < U; ++i)
					horner_row_pred(lds, lreg, zl_mask(S, r + i, ring[i]), r + i < S.nu, s0, s1, s2, s3);
#pragma unroll
				for (uint32_t i = 0; i < U; ++i)
					st_piece<COPY>(S, r + i, ring[i],
						       r + i < S.nu && (r + i != 0 || !STEP_HEAD(S)) && zl_keep(S, r + i), rsb);
#pragma unroll
				for (uint32_t i = 0; i + 1 < U; ++i)
					ring[i] = LD_PIECE(S, row_addr(S.ad, min(r + U + i, last), STEP_ZOFF(S), rsb), 3);
				continue;
			}
#pragma unroll
			for (uint32_t i = 0; i < U; ++i) {
				ring[(i + U - 1) % U] =
					LD_PIECE(S, row_addr(S.ad, min(r + i + U - 1, last), STEP_ZOFF(S), rsb), 3);
				horner_row_pred(lds, lreg, zl_mask<FLAT>(S, r + i, ring[i]), r + i < S.nu, s0, s1, s2, s3);
				st_piece<COPY>(S, r + i, ring[i],
					       r + i < S.nu && (r + i != 0 || !STEP_HEAD(S)) && zl_keep(S, r + i), rsb);
			}
		}
		// last block: its first load is this step's last row, the rest
		// already fetch the next step's first rows
		const uint32_t r = blk * U;
		ring[U - 1] = LD_PIECE(S, row_addr(S.ad, min(r + U - 1, last), STEP_ZOFF(S), rsb), 4);
		// Flat: the out[] flag again, looked at when this step's run is
		// XORed (after the block): the early read at the prime came before
		// the claiming wave had zeroed out[] in most waves, and polling then
		// cost every wave a round trip at its first XOR (~1-2 us of busy time
		// in 256 MiB launches of 64 KiB buffers, profiles/r06/stamps_flatg.txt).
		// Unconditional, as one more load in the ring's count (vmcnt(7) at its
		// use, no drain).
		uint64_t seen_l = 0;
		if constexpr (FLAT)
			seen_l = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef PECH_STAMP_FIN // stamps build: time spent planning steps inside the loop (sum, 25 % stamp slot)
		const uint64_t t_pl0 = __builtin_amdgcn_s_memrealtime();
#endif
		uint32_t npos = S.pos, nlr = S.lr, nrem = S.rem;
		if (jmax > 1u && nrem == 0) {
			// item done: the next one from the pool (wave-uniform branch,
			// scalar work and an LDS atomic; the ring is untouched)
			for (;;) {
				const uint32_t c = uni(claim), j = 1u + c / PECH_MAIN_WAVES, sh = c % PECH_MAIN_WAVES;
				if (j >= jmax)
					break; // pool empty
				const uint32_t a = (uint32_t)(wg0 + (uint64_t)wg_rows * sh / PECH_MAIN_WAVES);
				const uint32_t b = (uint32_t)(wg0 + (uint64_t)wg_rows * (sh + 1u) / PECH_MAIN_WAVES);
				const uint32_t st = share_head(a, b) + (j - 1u) * PECH_ITEM_ROWS;
				if (COPY) {
					if (lane == 0)
						claim = atomicAdd(lds + L_POOL / 4u, 1u); // the next claim, one item ahead
				} else {
					claim = claim2; // (lane 0's)
					if (lane == 0)
						claim2 = atomicAdd(lds + L_POOL / 4u, 1u); // two items ahead
				}
				if (st < b) {
					npos = st / U0;
					nlr = st - npos * U0;
					nrem = min(PECH_ITEM_ROWS, b - st);
					break;
				}
			}
		}
#ifndef PECH_NO_NEXT_SPEC
		// (flatg: as the planned kernel, from descriptors prefetched by
		// vector loads a step ahead; its scalar loads for the N of every
		// step made the row loops' schedule serialise their LDS lookups,
		// c4-64k 53.3 against 48.9 us for the planned main)
		if constexpr (FLATG)
			keep_whole(nspec_g);
		const Step N = FLATG ? plan_step<false, true, true, true>(gdesc, deltas, lds, npos, nlr, nrem, lane, g8, grp, false,
									 flatg_conv(nspec_g, min(nppos + grp, n - 1u)), nppos, n)
			       : FLAT ? (il ? plan_il<false, true>(cores, deltas, npos, nlr, nrem, wave * 8u + grp, g8, lds)
				      : plan_step<false, false, true, false>(gdesc, deltas, lds, npos, nlr, nrem, lane, g8, grp,
									     false, pech_core{}, 0u, n))
			   : il ? plan_il<COPY>(cores, deltas, npos, nlr, nrem, wave * 8u + grp, g8)
			   : COPY ? plan_step<COPY>(cores, deltas, lds, npos, nlr, nrem, lane, g8, grp, grid)
				  : plan_step<COPY, true>(cores, deltas, lds, npos, nlr, nrem, lane, g8, grp, grid, nspec, nppos);
		if (!COPY && (!FLAT || FLATG)) { // the descriptors where the step after N starts (flat: they are in LDS)
			const uint32_t nlim = FLATG ? n : nslots;
			nppos = min(N.pos, nlim - 1u);
			if (jmax > 1u && N.rem == 0) {
				// N ends a pooled item: the next item is the pending claim's
				// (a guess: an item past its share's end moves on to the next
				// claim, and the plan then misses and loads)
				const uint32_t c = uni(claim), j = 1u + c / PECH_MAIN_WAVES, sh = c % PECH_MAIN_WAVES;
				const uint32_t a = (uint32_t)(wg0 + (uint64_t)wg_rows * sh / PECH_MAIN_WAVES);
				const uint32_t b = (uint32_t)(wg0 + (uint64_t)wg_rows * (sh + 1u) / PECH_MAIN_WAVES);
				const uint32_t st = share_head(a, b) + (j - 1u) * PECH_ITEM_ROWS;
				nppos = j < jmax && st < b ? min(st / U0, nlim - 1u) : nppos;
			}
			if constexpr (FLATG)
				nspec_g = ((const u32x4 *)descs)[min(nppos + grp, n - 1u)];
			else
				nspec = load_spec(cores, nppos + grp);
		}
#else // A/B: N's descriptors loaded when N is planned
		const Step N = FLAT ? (il ? plan_il<false, true>(cores, deltas, npos, nlr, nrem, wave * 8u + grp, g8, lds)
				      : plan_step<false, false, true, FLATG>(gdesc, deltas, lds, npos, nlr, nrem, lane, g8, grp,
									     false, pech_core{}, 0u, n))
			   : il ? plan_il<COPY>(cores, deltas, npos, nlr, nrem, wave * 8u + grp, g8)
				  : plan_step<COPY>(cores, deltas, lds, npos, nlr, nrem, lane, g8, grp, grid);
#endif
		const uint32_t tpow_n = COPY ? 0u : rowpow(consts, N); // (used when N ends)
#ifdef PECH_STAMP_FIN
		tq[0] += __builtin_amdgcn_s_memrealtime() - t_pl0;
#endif
		if constexpr (COPY) { // block discipline: this block's rows and stores, then the next step's loads
			const bool more = N.T != 0;
			const Step &L = more ? N : S;
			const uint32_t lrow0 = more ? 0u : last, lmax = more ? N.nl - 1u : last;
#pragma unroll
			for (uint32_t i = 0; i < U; ++i)
				horner_row_pred(lds, lreg, zl_mask(S, r + i, ring[i]), r + i < S.nu, s0, s1, s2, s3);
#pragma unroll
			for (uint32_t i = 0; i < U; ++i)
				st_piece<COPY>(S, r + i, ring[i], r + i < S.nu && (r + i != 0 || !STEP_HEAD(S)) && zl_keep(S, r + i), rsb);
#pragma unroll
			for (uint32_t i = 1; i < U; ++i)
				ring[i - 1] = LD_PIECE(L, row_addr(L.ad, min(lrow0 + i - 1, lmax), STEP_ZOFF(L), rsb), 5);
		} else {
			horner_row_pred(lds, lreg, zl_mask<FLAT>(S, r, ring[0]), r < S.nu, s0, s1, s2, s3);
			st_piece<COPY>(S, r, ring[0], r < S.nu && (r != 0 || !STEP_HEAD(S)) && zl_keep(S, r), rsb);
			// Branch-free on purpose: with no next step the prefetch re-reads
			// this step's last row (valid memory, never used).  An if/else here
			// let LLVM sink the shared Horner code into a join block, which
			// cost ring-register copies behind a vmcnt(0) at every step end.
			const bool more = N.T != 0;
			const Step &L = more ? N : S;
			const uint32_t lrow0 = more ? 0u : last, lmax = more ? N.nl - 1u : last;
#pragma unroll
			for (uint32_t i = 1; i < U; ++i) {
				ring[i - 1] = LD_PIECE(L, row_addr(L.ad, min(lrow0 + i - 1, lmax), STEP_ZOFF(L), rsb), 5);
				horner_row_pred(lds, lreg, zl_mask<FLAT>(S, r + i, ring[i]), r + i < S.nu, s0, s1, s2, s3);
				st_piece<COPY>(S, r + i, ring[i], r + i < S.nu && zl_keep(S, r + i), rsb);
			}
		}
#ifdef PECH_DEBUG_BOUNDS
		{ // debug build: an active group's output slot must lie in this launch's slots
			const bool bad = S.nu != 0 && step_orig<FLAT>(S) >= (FLAT ? n : nchunks * PECH_CHUNK);
			if (bad && g8 == 0)
				printf("PECH OOB out blk %u wave %u orig %u nu %u T %u pos %u\n", blockIdx.x, wave, step_orig<FLAT>(S),
				       S.nu, S.T, S.pos);
			if (bad)
				S.nu = 0;
		}
#endif
#ifdef PECH_STAMP_FIN // stamps build: the last step's fold + shift (75 % stamp -> its start)
		tq[2] = __builtin_amdgcn_s_memrealtime();
#endif
		if constexpr (FLAT) {
			ready = ready || (uni64(seen_l) == FLAT_DONE(tag) && !(test & PECH_FLAT_T_TIMEOUT));
			flat_ready<NMAX>(flag, tag, ready, descs, n, lane, consts, out, seeds, hstat, test);
		}
		finish_run<!COPY>(lds, g8, s0, s1, s2, s3, step_m<FLAT>(S), STEP_RA(S), tpow, S.nu != 0, out, step_orig<FLAT>(S));
		tpow = tpow_n;
#ifdef PECH_STAMP_FIN
		tq[1] = __builtin_amdgcn_s_memrealtime();
#endif
		S = N;
#ifdef PECH_STAMPS
		++nstep;
#endif
	}
	// The workgroup's last wave to finish flushes the deferred split-step
	// results (no barrier: the others exit).  A wave's LDS operations complete
	// in order and the fences keep the compiler from moving them, so every
	// earlier wave's table updates precede its count.
	{
		uint32_t done = 0;
		if (FLAT && hout) // this wave's XORs into out[] performed before the workgroup's count (flat_publish)
			vm_done();
		__threadfence_block(); // table updates before the count (compiler and LDS order)
		if (lane == 0)
			done = atomicAdd(lds + L_DEFER_DONE / 4u, 1u);
		done = lane_value(done, 0);
		__threadfence_block();
		static_assert(PECH_DEFER_SLOTS == 64u, "one slot per lane of the flushing wave");
		if (done == PECH_MAIN_WAVES - 1u) {
			if (FLAT)
				flat_ready<NMAX>(flag, tag, ready, descs, n, lane, consts, out, seeds, hstat, test);
			const uint32_t k = lds[L_DEFER / 4u + lane];
			bool flush = k != PECH_DEFER_EMPTY;
#ifdef PECH_DEBUG_BOUNDS
			if (flush && k >= (FLAT ? n : nchunks * PECH_CHUNK)) {
				printf("PECH OOB flush blk %u slot %u key %u\n", blockIdx.x, lane, k);
				flush = false;
			}
#endif
			if (flush)
#ifdef PECH_AB_NOATOMIC // diagnostic build only: the flush dropped too (wrong CRCs)
				if (k == 0x9E3779B9u)
#endif
				atomicXor(out + k, lds[L_DEFER / 4u + PECH_DEFER_SLOTS + lane]);
			if (FLAT && hout)
				flat_publish<NMAX>(flag, sv.nlive, n, lane, out, hout, hstat, tag, test);
		}
	}
#ifdef PECH_STAMPS
	const uint32_t wid = blockIdx.x * PECH_MAIN_WAVES + wave;
	if (lane == 0 && wid < PECH_MAX_STAMPS) {
		uint32_t xcc;
		asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
		uint64_t *st = pech_stamps + PECH_NSTAMP * wid;
		st[0] = t_start;
		st[1] = __builtin_amdgcn_s_memrealtime();
		st[2] = ((uint64_t)blockIdx.x << 8) | (xcc & 0xFu);
		st[3] = t_entry;
		st[4] = t_scan;
		st[5] = t_find;
		st[6] = t_plan;
		st[7] = t_fill;
		st[11] = t_issued;
		st[8] = tq[0];
		st[9] = tq[1];
		st[10] = tq[2];
	}
#endif
}

extern "C" __global__ __launch_bounds__(PECH_MAIN_THREADS, 1) void pech_crc32c_main(
	const pech_core *__restrict__ cores, const uint32_t *__restrict__ lrs, const uint32_t *__restrict__ partials,
	const uint32_t *__restrict__ nzs, uint32_t n, const uint32_t *__restrict__ consts, uint32_t *__restrict__ out,
	uint32_t rpw_min)
{
	__shared__ __attribute__((aligned(16))) uint32_t lds[L_BYTES / 4u];
	main_body<false, PECH_U>(lds, cores, lrs, partials, nzs, n, consts, out, rpw_min, nullptr);
}

// fused CRC + copy (include/pech_crc32c.h crc32c_dev_copy_batch_*): the same
// walk, every consumed 16-byte piece also stored to its destination
extern "C" __global__ __launch_bounds__(PECH_MAIN_THREADS, 1) void pech_crc32c_main_copy(
	const pech_core *__restrict__ cores, const uint32_t *__restrict__ lrs, const uint32_t *__restrict__ partials,
	const uint32_t *__restrict__ nzs, uint32_t n, const uint32_t *__restrict__ consts, uint32_t *__restrict__ out,
	uint32_t rpw_min, const int64_t *__restrict__ deltas)
{
	__shared__ __attribute__((aligned(16))) uint32_t lds[L_BYTES / 4u];
	main_body<true, PECH_U_COPY>(lds, cores, lrs, partials, nzs, n, consts, out, rpw_min, deltas);
}

// One-launch device batch of up to PECH_FLAT_MAX buffers (any sizes): the
// main kernel's walk with no plan kernel (main_body<FLAT>).  A batch of few
// buffers -- C3's 256 x 4 MiB, an async slot of large payloads, a single
// large message -- then costs one launch on the stream instead of two, and
// its prologue reads the descriptors themselves instead of the plan's
// workspace.  `flag` (8 bytes of the caller's workspace) and the per-launch
// `tag` publish workgroup 0's zeroed out[] to the other workgroups.
extern "C" __global__ __launch_bounds__(PECH_MAIN_THREADS, 1) void pech_crc32c_flat(
	const pech_desc *__restrict__ descs, uint32_t n, const uint32_t *__restrict__ consts, uint32_t *__restrict__ out,
	uint32_t rpw_min, uint64_t *__restrict__ flag, uint64_t tag, uint32_t *__restrict__ hout, uint64_t *hstat,
	uint32_t test)
{
	__shared__ __attribute__((aligned(16))) uint32_t lds[L_BYTES / 4u];
	main_body<false, PECH_U, true>(lds, nullptr, nullptr, nullptr, nullptr, n, consts, out, rpw_min, nullptr, descs, flag,
				       tag, hout, hstat, test);
}

// pech_crc32c_flat for host-resident batches (PECH_FLAT_F_IL: the async
// layer's zero-copy slots): uniform batches of rows >= PECH_IL_MIN_ROWS walk
// interleaved rows (plan_il), others static shares, as pech_crc32c_flat
extern "C" __global__ __launch_bounds__(PECH_MAIN_THREADS, 1) void pech_crc32c_flat_il(
	const pech_desc *__restrict__ descs, uint32_t n, const uint32_t *__restrict__ consts, uint32_t *__restrict__ out,
	uint32_t rpw_min, uint64_t *__restrict__ flag, uint64_t tag, uint32_t *__restrict__ hout, uint64_t *hstat,
	uint32_t test)
{
	__shared__ __attribute__((aligned(16))) uint32_t lds[L_BYTES / 4u];
	main_body<false, PECH_U, true, false, true>(lds, nullptr, nullptr, nullptr, nullptr, n, consts, out, rpw_min, nullptr,
						    descs, flag, tag, hout, hstat, test);
}

// The same for PECH_FLAT_MAX < n <= PECH_FLATG_MAX buffers (the messenger's
// slots of 64 KiB payloads, 512 to a 32 MiB slot; C4's 64 KiB class, 4,096
// per 256 MiB launch): one launch instead of plan + main.  Its prologue
// scans the rows over the whole workgroup (prologue_flatg) and its steps read
// the descriptors in place (flatg_core); out[] is initialised and published
// as in pech_crc32c_flat.
extern "C" __global__ __launch_bounds__(PECH_MAIN_THREADS, 1) void pech_crc32c_flatg(
	const pech_desc *__restrict__ descs, uint32_t n, const uint32_t *__restrict__ consts, uint32_t *__restrict__ out,
	uint32_t rpw_min, uint64_t *__restrict__ flag, uint64_t tag, uint32_t *__restrict__ hout, uint64_t *hstat,
	uint32_t test)
{
	__shared__ __attribute__((aligned(16))) uint32_t lds[L_BYTES_G / 4u];
	main_body<false, PECH_U, true, true>(lds, nullptr, nullptr, nullptr, nullptr, n, consts, out, rpw_min, nullptr, descs,
					     flag, tag, hout, hstat, test);
}

// ---- direct kernel: small-buffer batches without a plan kernel -------------
// crc32c_dev_batch_small_async (include/pech_crc32c.h): ONE launch and no
// workspace.  The batch's positions are split evenly over the waves; each
// wave walks its positions in steps of 8 (one buffer per group, all of its
// rows), reading the descriptors itself by scalar loads.  Balanced when the
// buffers are of similar size -- the caller's contract: every buffer below
// PECH_SPLIT_ROWS * 128 bytes (32 KiB) -- and correct for any batch (a larger
// buffer is walked by one group alone).  A buffer's rows cover ALL of its
// bytes: row 0's bytes before it are masked as in the main kernel (head), the
// last row's bytes after it are masked too (tail: piece by piece), and the
// trailing zeros are undone by one x^(-8 trail) multiply, trail < 128 -- no
// tail block load: an unaligned end costs nothing beyond the row it shares.
// Only a seed (or an empty buffer) takes the slow path, a descriptor reload
// at the run's end.  Results are stored, not XORed: out[] needs no
// initialisation.  This saves the plan launch and the main kernel's
// chunk-scan prologue on the messenger's small payloads.
#define STEP_SLOW(S) (((S).oz >> 28) & 1u) // the run's buffer has a seed, or no bytes
#define DSTEP_TRAIL(S) ((S).mp & 0x7Fu)     // zero bytes after the buffer in its last row
#define DSTEP_KB(S) (((S).mp >> 8) & 31u)    // bytes of the lane's piece kept in the last row

// Direct mode: the last row's piece keeps its bytes below DSTEP_KB (64-bit
// halves, as the head mask)
__device__ __forceinline__ u32x4 tail_keep(const Step &S, uint32_t row, u32x4 v)
{
	const uint32_t kb = row == S.nu - 1u ? DSTEP_KB(S) : 16u;
	uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
	lo &= kb >= 8u ? ~0ull : (1ull << (8u * kb)) - 1ull;
	hi &= kb >= 16u ? ~0ull : (kb <= 8u ? 0ull : (1ull << (8u * (kb - 8u))) - 1ull);
	return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}

// The next step of a direct-mode wave: positions [pos, end), interleaved in
// blocks of 16 (group g takes pos + 2g, then pos + 2g + 1: for buffers laid
// out back to back every group walks one contiguous 2-buffer range, as the
// plan kernel's order does), a plain run of up to 8 at the range's end.
template <bool COPY = false>
__device__ __forceinline__ Step plan_direct(const pech_desc *__restrict__ descs, const uint32_t *consts,
					    uint32_t &pos, uint32_t end, uint32_t &ph, uint32_t g8, uint32_t grp,
					    const uint64_t *__restrict__ dsts = nullptr)
{
	Step S;
	S.T = 0;
	S.nmin = 0;
	S.mp = 0;
	S.oz = 0;
	S.nl = 1;
	S.nu = 0;
	S.ad = (uint64_t)consts + 16u * g8; // idle groups: valid memory, state ignored
	S.pos = S.lr = S.rem = 0;
#ifdef PECH_DEBUG_BOUNDS
	S.blo = S.ad;
	S.bhi = S.ad + 16u;
#endif
	const uint32_t left = end - pos;
	if (left == 0) {
		S.dad = S.ad;
		return S;
	}
	const bool il = ph != 0u || left >= 16u;
	const uint32_t cnt = il ? 8u : min(left, 8u);
	// one descriptor per group by scalar loads (wave-uniform addresses)
	uint32_t alo = 0, ahi = 0, len = 0, seed = 0;
	uint64_t dst = 0;
#pragma unroll
	for (uint32_t j = 0; j < 8; ++j) {
		const uint32_t pj = il ? pos + 2u * j + ph : pos + min(j, cnt - 1u);
		const pech_desc dj = descs[pj];
		const bool mine = grp == j;
		alo = mine ? uni((uint32_t)dj.addr) : alo;
		ahi = mine ? uni((uint32_t)(dj.addr >> 32)) : ahi;
		len = mine ? uni(dj.len) : len;
		seed = mine ? uni(dj.seed) : seed;
		if (COPY)
			dst = mine ? uni64(dsts[pj]) : dst;
	}
	const uint32_t b = il ? pos + 2u * grp + ph : pos + grp;
	const bool have = grp < cnt;
	const uint64_t addr = ((uint64_t)ahi << 32) | alo;
	const uint32_t lb = alo & (PECH_ROW_BYTES - 1u);
	const uint32_t rows = have ? (uint32_t)(((uint64_t)lb + len + PECH_ROW_BYTES - 1u) >> 7) : 0u;
	const bool slow = have && (seed != 0u || rows == 0u);
	uint32_t tmax = 0, tmin = 0xFFFFFFFFu, anyslow = 0, dj = 0;
#pragma unroll
	for (uint32_t j = 0; j < 8; ++j) {
		const uint32_t v = lane_value(rows, 8u * j);
		dj = v > tmax ? j : dj;
		tmax = max(tmax, v);
		tmin = v ? min(tmin, v) : tmin;
		anyslow |= lane_value(slow ? 1u : 0u, 8u * j);
	}
	if (tmax) { // idle groups walk the longest buffer's rows (valid memory for the unclamped loop), ignored
		const uint64_t da = ((uint64_t)lane_value(ahi, 8u * dj) << 32) | lane_value(alo, 8u * dj);
		S.ad = (da & ~(uint64_t)(PECH_ROW_BYTES - 1u)) + 16u * g8;
		S.nl = tmax;
#ifdef PECH_DEBUG_BOUNDS
		S.blo = S.ad;
		S.bhi = (da & ~(uint64_t)(PECH_ROW_BYTES - 1u)) + (uint64_t)tmax * PECH_ROW_BYTES;
#endif
	}
	// a step of tiny buffers only (no rows) still runs once, for its slow path
	S.T = max(tmax, anyslow);
	S.nmin = tmin == 0xFFFFFFFFu ? 0u : tmin;
	if (rows) {
		S.ad = (addr & ~(uint64_t)(PECH_ROW_BYTES - 1u)) + 16u * g8;
		S.nl = rows;
		S.nu = rows;
		S.oz = head_bits(true, g8, lb);
		// mod 2^32: the true values are < 128 and in (0, 128]
		const uint32_t e = lb + len - (rows - 1u) * PECH_ROW_BYTES;
		S.mp = (rows * PECH_ROW_BYTES - lb - len) | (min(e - min(e, 16u * g8), 16u) << 8);
#ifdef PECH_DEBUG_BOUNDS
		S.blo = (addr & ~(uint64_t)(PECH_ROW_BYTES - 1u)) + 16u * (lb >> 4);
		S.bhi = (addr & ~(uint64_t)(PECH_ROW_BYTES - 1u)) + (uint64_t)rows * PECH_ROW_BYTES;
#endif
	}
	S.oz |= (have ? b : 0u) | (slow ? 1u << 28 : 0u);
	if (il) {
		pos += ph ? 16u : 0u;
		ph ^= 1u;
	} else {
		pos += cnt;
	}
	// fused copy: this lane's row-0 piece in the destination (a source byte
	// at a goes to a + dst - addr); groups without rows store nothing
	S.dad = COPY && rows ? S.ad + (dst - addr) : S.ad;
	return S;
}

// Direct fused copy: the bytes of row `row`'s piece that are the buffer's
// go to the destination -- a whole 16-byte store, or, for the partial pieces
// at the buffer's two ends (bytes before it in row 0, past it in the last
// row), byte stores.  Pieces wholly outside the buffer and rows past the run
// store nothing.
template <bool COPY>
__device__ __forceinline__ void st_direct(const Step &S, uint32_t row, u32x4 v)
{
	typedef __attribute__((address_space(1))) u32x4 g_u32x4w;
	if (!COPY || row >= S.nu)
		return;
	const uint32_t lo = row == 0u ? (STEP_ZOFF(S) ? 16u : STEP_ZH(S)) : 0u;
	const uint32_t hi = row == S.nu - 1u ? DSTEP_KB(S) : 16u;
	const uint64_t a = S.dad + (uint64_t)row * PECH_ROW_BYTES;
	if (lo == 0u && hi == 16u) {
		__builtin_nontemporal_store(v, (g_u32x4w *)a);
		return;
	}
#pragma unroll
	for (uint32_t i = 0; i < 16u; ++i)
		if (i >= lo && i < hi)
			*(__attribute__((address_space(1))) uint8_t *)(a + i) = (uint8_t)(v[i >> 2] >> (8u * (i & 3u)));
}

// Direct mode: fold as finish_run, undo the trailing zeros, add the seed's
// term (slow path) and store out[b].
__device__ __forceinline__ void finish_direct(uint32_t *lds, uint32_t g8, uint32_t s0, uint32_t s1, uint32_t s2,
					      uint32_t s3, const Step &S, const pech_desc *__restrict__ descs,
					      uint32_t *__restrict__ out)
{
	uint32_t u = adv_tab(lds, L_TAB4, s0) ^ s1;
	u = adv_tab(lds, L_TAB4, u) ^ s2;
	u = adv_tab(lds, L_TAB4, u) ^ s3;
	u = adv_tab(lds, L_TAB4, u);
	u = adv_tab(lds, L_TAB16, u) ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x101, 0xf, 0xf, true);
	u = adv_tab(lds, L_TAB32, u) ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x102, 0xf, 0xf, true);
	u = adv_tab(lds, L_TAB64, u) ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x104, 0xf, 0xf, true);
	const bool lead = g8 == 0u;
	uint32_t v = 0;
	if (S.nu != 0u && lead) {
		const uint32_t tr = DSTEP_TRAIL(S);
		v = tr ? gf2_mulmod_dev(lds[L_XINV / 4u + tr], u) : u;
	}
	const bool slow = STEP_SLOW(S) != 0u && lead;
	if (__ballot(slow) != 0ull && slow) { // the rare slow path: its load waits for the ring too
		const pech_desc d = descs[STEP_ORIG(S)];
		if (d.seed) // R(s, D) = x^(8|D|) s ^ R(0, D)
			v ^= d.len ? shift_bytes(lds + L_POWB / 4u, d.len, d.seed) : d.seed;
	}
	if ((S.nu != 0u || STEP_SLOW(S) != 0u) && lead)
		out[STEP_ORIG(S)] = v;
}

// Direct mode: a ring load past the run's last row (the unrolled tail of its
// last block, the final prefetch) only keeps the ring's counted order, so it
// reads the constants table (L2-resident) instead of the run's last line
// again.  (The bounds-checked build keeps the in-buffer clamp it can check.)
__device__ __forceinline__ uint64_t dload_addr(const Step &S, uint32_t row, uint32_t last, uint64_t dummy)
{
#if defined(PECH_DEBUG_BOUNDS) || defined(PECH_DIRECT_CLAMP) // (PECH_DIRECT_CLAMP: A/B, the v0.18 clamp)
	(void)dummy;
	return row_addr(S.ad, min(row, last), STEP_ZOFF(S));
#else
	const uint64_t a = row_addr(S.ad, min(row, last), STEP_ZOFF(S));
	return row <= last ? a : dummy;
#endif
}

template <uint32_t U, bool COPY = false>
__device__ __forceinline__ void direct_body(uint32_t *lds, const pech_desc *__restrict__ descs, uint32_t n,
					    const uint32_t *__restrict__ consts, uint32_t *__restrict__ out,
					    const uint64_t *__restrict__ dsts = nullptr)
{
	const uint32_t tid = threadIdx.x;
#ifdef PECH_KARGS_AT_ENTRY
	asm volatile("" ::"s"(descs), "s"(n), "s"(consts), "s"(out), "s"(dsts)); // one kernarg round (main_body)
#endif
	const uint32_t lane = tid & 63u, g8 = tid & 7u, grp = lane >> 3;
	const uint32_t lreg = ((lane & 31u) << 2) | (1u << 16);
	const uint32_t wave = uni(tid >> 6);
	constexpr uint32_t T128 = 1024u / PECH_MAIN_THREADS;
	constexpr uint32_t NT4 = (PECH_C_TAB1 - PECH_C_TAB4) / 4u;
	constexpr uint32_t TPT = (NT4 + PECH_MAIN_THREADS - 1u) / PECH_MAIN_THREADS;
	const u32x4 *c4 = (const u32x4 *)(consts + PECH_C_TAB4);
	uint32_t t128[T128];
#pragma unroll
	for (uint32_t j = 0; j < T128; ++j)
		t128[j] = consts[PECH_C_TAB128 + tid + j * PECH_MAIN_THREADS];
	u32x4 tv[TPT];
#pragma unroll
	for (uint32_t k = 0; k < TPT; ++k)
		tv[k] = c4[min(tid + k * PECH_MAIN_THREADS, NT4 - 1u)];
	const uint32_t txi = consts[PECH_C_XINV + (tid & 127u)];
	// the wave's positions: an equal split of the batch
	const uint32_t wglob = blockIdx.x * PECH_MAIN_WAVES + wave;
#ifndef PECH_DIRECT_WAVE_SHARES
	// Workgroup-interleaved positions (v0.21): step k of wave w takes
	// positions wb + 128 k + 8 w .. + 7 of the workgroup's range [wb, we), so
	// the workgroup's 128 lane groups are on 128 consecutive buffers (one
	// window per CU) and its waves end together; per launch equal, two-stream
	// value +3-5 % (profiles/r03/ab_direct_wg_interleave.txt).
	const uint32_t wb = (uint32_t)((uint64_t)blockIdx.x * n / gridDim.x);
	const uint32_t we = (uint32_t)((uint64_t)(blockIdx.x + 1u) * n / gridDim.x);
	uint32_t kstep = 0;
	auto next_step = [&]() {
		const uint32_t e0 = min(wb + PECH_IL_GROUPS * kstep + 8u * wave + 8u, we);
		uint32_t p = min(wb + PECH_IL_GROUPS * kstep + 8u * wave, e0), ph0 = 0;
		++kstep;
		return plan_direct<COPY>(descs, consts, p, e0, ph0, g8, grp, dsts);
	};
#else // A/B: each wave an equal share of the positions, in blocks of 16 (v0.17-v0.20)
	const uint32_t W = gridDim.x * PECH_MAIN_WAVES;
	uint32_t pos = (uint32_t)((uint64_t)wglob * n / W), ph = 0;
	const uint32_t pend = (uint32_t)((uint64_t)(wglob + 1u) * n / W);
	auto next_step = [&]() { return plan_direct<COPY>(descs, consts, pos, pend, ph, g8, grp, dsts); };
#endif
	// (spread over 128 lines of the table: one line for every wave was an L2 hot spot)
	const uint64_t dummy = (uint64_t)consts + (uint64_t)((wglob * 8u + grp) & 127u) * PECH_ROW_BYTES + 16u * g8;
	static_assert(128u * PECH_ROW_BYTES <= PECH_C_WORDS * 4u, "dummy lines inside the constants");
	Step S = next_step();
	u32x4 ring[U];
	if (S.T)
		RING_PRIME(S, ring);
#pragma unroll
	for (uint32_t j = 0; j < T128; ++j) {
		const uint32_t w = tid + j * PECH_MAIN_THREADS, k = w >> 8, e = w & 0xFFu;
		const u32x4 v = (u32x4)(t128[j]);
		char *dst = (char *)lds + (k >> 1) * 65536u + e * 256u + (k & 1u) * 128u;
#pragma unroll
		for (uint32_t q = 0; q < 8u; ++q)
			*(u32x4 *)(dst + 16u * ((q + w) & 7u)) = v;
	}
#pragma unroll
	for (uint32_t k = 0; k < TPT; ++k)
		if (tid + k * PECH_MAIN_THREADS < NT4)
			*(u32x4 *)((char *)lds + L_TAB4 + 16u * (tid + k * PECH_MAIN_THREADS)) = tv[k];
	if (tid < 128u)
		lds[L_XINV / 4u + tid] = txi;
	__syncthreads(); // tables published; every wave's prime is already in flight
	while (S.T) {
		uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
		{ // row 0's bytes before the buffer are zeros (as in main_body)
			const uint32_t sh = STEP_ZOFF(S) ? 128u : 8u * STEP_ZH(S);
			uint64_t lo = ((uint64_t)ring[0].y << 32) | ring[0].x, hi = ((uint64_t)ring[0].w << 32) | ring[0].z;
			lo &= sh >= 64u ? 0ull : ~0ull << sh;
			hi &= sh >= 128u ? 0ull : (sh <= 64u ? ~0ull : ~0ull << (sh - 64u));
			ring[0] = u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
		}
		const uint32_t nblk = (S.T + U - 1) / U;
		const uint32_t last = S.nl - 1u;
		uint32_t blk = 0;
		for (; blk + 1 < nblk && (blk + 2) * U <= S.nmin; ++blk) {
			const uint64_t base = S.ad + (uint64_t)blk * U * PECH_ROW_BYTES;
			if constexpr (COPY) { // block discipline, as the main copy kernel (vmcnt counts stores in order)
				ring[U - 1] = LD_PIECE(S, base + (U - 1) * PECH_ROW_BYTES, 2);
#pragma unroll
				for (uint32_t i = 0; i < U; ++i)
					horner_row(lds, lreg, ring[i], s0, s1, s2, s3);
#pragma unroll
				for (uint32_t i = 0; i < U; ++i)
					st_direct<COPY>(S, blk * U + i, ring[i]);
#pragma unroll
				for (uint32_t i = 0; i + 1 < U; ++i)
					ring[i] = LD_PIECE(S, base + (U + i) * PECH_ROW_BYTES, 2);
				continue;
			}
#pragma unroll
			for (uint32_t i = 0; i < U; ++i) {
				ring[(i + U - 1) % U] = LD_PIECE(S, base + (i + U - 1) * PECH_ROW_BYTES, 2);
				horner_row(lds, lreg, ring[i], s0, s1, s2, s3);
			}
		}
		for (; blk + 1 < nblk; ++blk) {
			const uint32_t r = blk * U;
			if constexpr (COPY) {
				ring[U - 1] = LD_PIECE(S, dload_addr(S, r + U - 1, last, dummy), 3);
#pragma unroll
				for (uint32_t i = 0; i < U; ++i)
					horner_row_pred(lds, lreg, tail_keep(S, r + i, ring[i]), r + i < S.nu, s0, s1, s2, s3);
#pragma unroll
				for (uint32_t i = 0; i < U; ++i)
					st_direct<COPY>(S, r + i, ring[i]);
#pragma unroll
				for (uint32_t i = 0; i + 1 < U; ++i)
					ring[i] = LD_PIECE(S, dload_addr(S, r + U + i, last, dummy), 3);
				continue;
			}
#pragma unroll
			for (uint32_t i = 0; i < U; ++i) {
				ring[(i + U - 1) % U] = LD_PIECE(S, dload_addr(S, r + i + U - 1, last, dummy), 3);
				horner_row_pred(lds, lreg, tail_keep(S, r + i, ring[i]), r + i < S.nu, s0, s1, s2, s3);
			}
		}
		const uint32_t r = blk * U;
		ring[U - 1] = LD_PIECE(S, dload_addr(S, r + U - 1, last, dummy), 4);
		const Step N = next_step();
		if constexpr (COPY) { // this block's rows and stores, then the next step's first loads
			const bool more = N.T != 0;
			const Step &L = more ? N : S;
			const uint32_t lmax = more ? N.nl - 1u : last;
#pragma unroll
			for (uint32_t i = 0; i < U; ++i)
				if (r + i < S.T)
					horner_row_pred(lds, lreg, tail_keep(S, r + i, ring[i]), r + i < S.nu, s0, s1, s2, s3);
#pragma unroll
			for (uint32_t i = 0; i < U; ++i)
				if (r + i < S.T)
					st_direct<COPY>(S, r + i, ring[i]);
#pragma unroll
			for (uint32_t i = 1; i < U; ++i)
				ring[i - 1] = LD_PIECE(L, dload_addr(L, more ? i - 1 : lmax + 1u, lmax, dummy), 5);
			finish_direct(lds, g8, s0, s1, s2, s3, S, descs, out);
			S = N;
			continue;
		}
		// the last block's rows past every group's run (S.T, wave-uniform)
		// are skipped by a scalar branch: their loads keep the ring's order
		if (r < S.T)
			horner_row_pred(lds, lreg, tail_keep(S, r, ring[0]), r < S.nu, s0, s1, s2, s3);
		// branch-free: with no next step the prefetch reads the constants
		const bool more = N.T != 0;
		const Step &L = more ? N : S;
		const uint32_t lmax = more ? N.nl - 1u : last;
#pragma unroll
		for (uint32_t i = 1; i < U; ++i) {
			ring[i - 1] = LD_PIECE(L, dload_addr(L, more ? i - 1 : lmax + 1u, lmax, dummy), 5);
			if (r + i < S.T)
				horner_row_pred(lds, lreg, tail_keep(S, r + i, ring[i]), r + i < S.nu, s0, s1, s2, s3);
		}
		finish_direct(lds, g8, s0, s1, s2, s3, S, descs, out);
		S = N;
	}
}

extern "C" __global__ __launch_bounds__(PECH_MAIN_THREADS, 1) void pech_crc32c_direct(
	const pech_desc *__restrict__ descs, uint32_t n, const uint32_t *__restrict__ consts, uint32_t *__restrict__ out)
{
	__shared__ __attribute__((aligned(16))) uint32_t lds[L_BYTES / 4u];
	direct_body<PECH_U>(lds, descs, n, consts, out);
}

// fused CRC + copy of a small-buffer batch (crc32c_dev_copy_batch_small_async):
// the direct kernel with every consumed piece also stored to its destination
extern "C" __global__ __launch_bounds__(PECH_MAIN_THREADS, 1) void pech_crc32c_direct_copy(
	const pech_desc *__restrict__ descs, uint32_t n, const uint32_t *__restrict__ consts, uint32_t *__restrict__ out,
	const uint64_t *__restrict__ dsts)
{
	__shared__ __attribute__((aligned(16))) uint32_t lds[L_BYTES / 4u];
	direct_body<PECH_U_DCOPY, true>(lds, descs, n, consts, out, dsts);
}

// ---- host-side launchers (used by crc32c_api.cpp) -------------------------
extern "C" hipError_t pech_launch_small(const void *src, uint32_t len, uint32_t seed, const uint32_t *consts,
					uint32_t *out, uint32_t ticket, hipStream_t stream)
{
	if (len > PECH_SMALL_MAX)
		return hipErrorInvalidValue;
	hipLaunchKernelGGL(pech_crc32c_small, dim3(1), dim3(PECH_SMALL_THREADS), 0, stream, (const uint8_t *)src, len,
			   seed, consts, out, ticket);
	return hipGetLastError();
}

// dsts != NULL: the fused-copy variant (destination address per descriptor)
extern "C" hipError_t pech_launch_plan(const pech_desc *descs, uint32_t n, const pech_ws *ws, const uint32_t *consts,
				       uint32_t *out, const uint64_t *dsts, hipStream_t stream)
{
	const uint32_t nch = (n + PECH_CHUNK - 1) / PECH_CHUNK;
	if (dsts)
		hipLaunchKernelGGL(pech_crc32c_plan_copy, dim3(nch), dim3(PECH_WG_THREADS), 0, stream, descs, n, ws->cores,
				   ws->lrs, ws->partials, ws->nzs, consts, out, dsts, ws->deltas);
	else
		hipLaunchKernelGGL(pech_crc32c_plan, dim3(nch), dim3(PECH_WG_THREADS), 0, stream, descs, n, ws->cores,
				   ws->lrs, ws->partials, ws->nzs, consts, out);
	return hipGetLastError();
}

// ev_start/ev_stop (optional): stamped by the kernel's own dispatch packet
// (hipExtLaunchKernel), so their interval is the kernel's execution alone,
// as rocprofv3's kernel trace reports it -- no launch boundary included.
extern "C" hipError_t pech_launch_main(uint32_t n, const pech_ws *ws, const uint32_t *consts, uint32_t *out,
				       uint32_t ncu, uint32_t rpw_min, int copy, hipStream_t stream, hipEvent_t ev_start,
				       hipEvent_t ev_stop)
{
	if (copy)
		hipExtLaunchKernelGGL(pech_crc32c_main_copy, dim3(ncu), dim3(PECH_MAIN_THREADS), 0, stream, ev_start, ev_stop,
				      0u, (const pech_core *)ws->cores, (const uint32_t *)ws->lrs,
				      (const uint32_t *)ws->partials, (const uint32_t *)ws->nzs, n, consts, out, rpw_min,
				      (const int64_t *)ws->deltas);
	else
		hipExtLaunchKernelGGL(pech_crc32c_main, dim3(ncu), dim3(PECH_MAIN_THREADS), 0, stream, ev_start, ev_stop,
				      0u, (const pech_core *)ws->cores, (const uint32_t *)ws->lrs,
				      (const uint32_t *)ws->partials, (const uint32_t *)ws->nzs, n, consts, out, rpw_min);
	return hipGetLastError();
}

// flat kernel (one launch, 1 <= n <= PECH_FLAT_MAX); ev_start/ev_stop as
// pech_launch_main; flag: 8-byte aligned device word, tag: fresh per launch
extern "C" hipError_t pech_launch_flat(const pech_desc *descs, uint32_t n, const uint32_t *consts, uint32_t *out,
				       uint32_t ncu, uint32_t rpw_min, uint64_t *flag, uint64_t tag, hipStream_t stream,
				       hipEvent_t ev_start, hipEvent_t ev_stop, uint32_t *hout, uint64_t *hstat, uint32_t test)
{
	if (n == 0 || n > PECH_FLATG_MAX || ((uintptr_t)flag & 7u))
		return hipErrorInvalidValue;
	if (n <= PECH_FLAT_MAX && (test & PECH_FLAT_F_IL))
		hipExtLaunchKernelGGL(pech_crc32c_flat_il, dim3(ncu), dim3(PECH_MAIN_THREADS), 0, stream, ev_start, ev_stop,
				      0u, descs, n, consts, out, rpw_min, flag, tag, hout, hstat, test);
	else if (n <= PECH_FLAT_MAX)
		hipExtLaunchKernelGGL(pech_crc32c_flat, dim3(ncu), dim3(PECH_MAIN_THREADS), 0, stream, ev_start, ev_stop, 0u,
				      descs, n, consts, out, rpw_min, flag, tag, hout, hstat, test);
	else
		hipExtLaunchKernelGGL(pech_crc32c_flatg, dim3(ncu), dim3(PECH_MAIN_THREADS), 0, stream, ev_start, ev_stop, 0u,
				      descs, n, consts, out, rpw_min, flag, tag, hout, hstat, test);
	return hipGetLastError();
}

// direct kernel (no plan, no workspace); ev_start/ev_stop as pech_launch_main;
// dsts != NULL: the fused-copy variant
extern "C" hipError_t pech_launch_direct(const pech_desc *descs, uint32_t n, const uint32_t *consts, uint32_t *out,
					 uint32_t ncu, hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop,
					 const uint64_t *dsts)
{
	if (dsts)
		hipExtLaunchKernelGGL(pech_crc32c_direct_copy, dim3(ncu), dim3(PECH_MAIN_THREADS), 0, stream, ev_start,
				      ev_stop, 0u, descs, n, consts, out, dsts);
	else
		hipExtLaunchKernelGGL(pech_crc32c_direct, dim3(ncu), dim3(PECH_MAIN_THREADS), 0, stream, ev_start, ev_stop,
				      0u, descs, n, consts, out);
	return hipGetLastError();
}

#define PECH_STR2(x) #x
#define PECH_STR(x) PECH_STR2(x)
extern "C" const char *pech_kernel_tag(void)
{
	return "pech_crc32c 0.36 gfx950 rows128 wave-steps(8x8-lane groups) prio-by-progress(static,pool-dry) split>=8rows small-deal<=4waves/wg,blocks32 grid-small-steps masked-heads flat<=" PECH_STR(PECH_FLAT_MAX) "(host:il),flatg<=" PECH_STR(PECH_FLATG_MAX) "(status-word) direct-small-batches(past-end-consts,wg-interleaved,copy) lds-bank-replicated-A128 mulmod-bitop3 rowpow next-spec(pool 2-ahead) early-fill<=" PECH_STR(PECH_EARLY_FILL_ROWS) "rows/wg U" PECH_STR(
		PECH_U) " waves/CU " PECH_STR(PECH_MAIN_WAVES) " copy-blocks U" PECH_STR(PECH_U_COPY) " copy-il" PECH_STR(PECH_IL_COPY) " uniform-pool " PECH_STR(PECH_POOL_ROWS) "/" PECH_STR(PECH_ITEM_ROWS) " from " PECH_STR(PECH_POOL_MIN_SHARE);
}
