// crc32c_kernels.hip -- gfx950 (CDNA4) kernels for batched CRC32C.
//
// Computes, for every descriptor (addr, len, seed) of a batch, exactly the
// value of the reference crc32c(seed, addr, len)
// (/root/reference/include/crc32c.h:88-96), over device-resident bytes.
//
// Two launches per batch, both on the caller's stream:
//   pech_crc32c_plan : one 1024-thread workgroup per chunk of 1024 buffers;
//                      rows per buffer (layout.h), chunk-local exclusive scan
//                      -> lrs[], chunk totals -> partials[], out[] initialised
//                      (0, or the seed for len == 0: crc32c.h:92 loop never runs).
//   pech_crc32c_main : persistent, one 1024-thread workgroup per CU (the LDS
//                      tables take 144 KiB).  Each 8-lane group walks a
//                      contiguous range of rows of the batch's row space.
//
// Hot loop (per lane, per 128-byte row): one coalesced 16-byte load of its
// piece, then for each of its 4 word streams  s <- A_128(s) ^ w, where
// A_128 (advance 128 zero bytes) is four byte-indexed table lookups.  The
// tables are replicated 32x in LDS, one copy per bank, so a lookup is
// conflict-free whatever the data: lane l (mod 32) only ever touches bank l.
// The byte -> LDS address step is ONE v_perm_b32 (byte k of s lands in
// address byte 1, the lane's bank offset in byte 0).
// A segment ends at a buffer end or at the group's range end; its 32 stream
// registers are folded with single-copy A_4/A_16/A_32/A_64 tables, shifted
// to the buffer's end with the power tables, and stored (whole buffer) or
// xor-ed atomically (buffer split over groups) into out[].
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf2.h"
#include "layout.h"

// ---- LDS map (bytes) ------------------------------------------------------
#define L_REP 0u                      // 128 KiB: A_128 tables, 32 bank copies
#define L_TAB4 131072u                // 4 KiB each, single copy
#define L_TAB16 (L_TAB4 + 4096u)
#define L_TAB32 (L_TAB16 + 4096u)
#define L_TAB64 (L_TAB32 + 4096u)
#define L_POWR (L_TAB64 + 4096u)      // 1280 B
#define L_XINV (L_POWR + 1280u)       // 128 B
#define L_CHUNK (L_XINV + 128u)       // 4 KiB: chunk row offsets
#define L_MISC (L_CHUNK + 4096u)      // scan scratch
#define L_BYTES (L_MISC + 128u)

static_assert(L_CHUNK == 131072u + 4u * (PECH_C_WORDS - PECH_C_TAB4), "LDS/consts layout mismatch");
static_assert(L_BYTES <= 160u * 1024u, "LDS budget");

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;

// 16-byte descriptor load through the global (not flat) address space
__device__ __forceinline__ pech_desc load_desc(const pech_desc *descs, uint32_t b)
{
	const u32x4 v = *(g_u32x4 *)(descs + b);
	pech_desc d;
	d.addr = (uint64_t)v.x | ((uint64_t)v.y << 32);
	d.len = v.z;
	d.seed = v.w;
	return d;
}

// ---- helpers --------------------------------------------------------------
// 1024-thread exclusive scan; scratch = 16 LDS words
__device__ inline uint32_t block_excl_scan(uint32_t v, uint32_t *scratch, uint32_t *total)
{
	const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
	uint32_t x = v;
#pragma unroll
	for (uint32_t d = 1; d < 64; d <<= 1) {
		uint32_t y = __shfl_up(x, d);
		if (lane >= d)
			x += y;
	}
	if (lane == 63u)
		scratch[wave] = x;
	__syncthreads();
	uint32_t off = 0, tot = 0;
#pragma unroll
	for (uint32_t w = 0; w < PECH_WG_THREADS / 64u; ++w) {
		uint32_t t = scratch[w];
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

// A_128(s) from the bank-replicated tables.  lreg = (lane&31)*4 | 1<<16.
// table k, entry e, bank copy c lives at (k>>1)*64K + e*256 + (k&1)*128 + 4c.
__device__ __forceinline__ uint32_t adv128(const uint32_t *lds, uint32_t s, uint32_t lreg)
{
	const uint32_t a0 = __builtin_amdgcn_perm(s, lreg, 0x0C0C0400u);
	const uint32_t a1 = __builtin_amdgcn_perm(s, lreg, 0x0C0C0500u);
	const uint32_t a2 = __builtin_amdgcn_perm(s, lreg, 0x0C020600u);
	const uint32_t a3 = __builtin_amdgcn_perm(s, lreg, 0x0C020700u);
	return lds_u32(lds, a0) ^ lds_u32(lds, a1 + 128u) ^ lds_u32(lds, a2) ^ lds_u32(lds, a3 + 128u);
}

// single-copy byte tables (4 x 256 words at byte offset `tab`)
__device__ __forceinline__ uint32_t adv_tab(const uint32_t *lds, uint32_t tab, uint32_t v)
{
	const uint32_t *t = lds + (tab >> 2);
	return t[v & 0xFFu] ^ t[256u + ((v >> 8) & 0xFFu)] ^ t[512u + ((v >> 16) & 0xFFu)] ^ t[768u + (v >> 24)];
}

__device__ __forceinline__ uint32_t bytes_mask(int t) // low t bytes set, t in [0,4]
{
	return t >= 4 ? 0xFFFFFFFFu : ((1u << (8 * t)) - 1u);
}

// Mask bytes of the piece at pa that lie outside [ptr, ptr+len) and xor the
// seed into bytes [ptr, ptr+4).  Only rows at a buffer's edges get here.
__device__ inline u32x4 fix_piece(u32x4 w, uint64_t pa, uint64_t ptr, uint32_t len, uint32_t seed)
{
	const int64_t dlo = (int64_t)(ptr - pa);
	const int64_t dhi = (int64_t)(ptr + len - pa);
	const int lo = (int)(dlo < 0 ? 0 : (dlo > 16 ? 16 : dlo));
	const int hi = (int)(dhi < 0 ? 0 : (dhi > 16 ? 16 : dhi));
	uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const int a = max(lo - 4 * k, 0), b = min(hi - 4 * k, 4);
		const uint32_t m = (b <= a) ? 0u : (bytes_mask(b) & ~bytes_mask(a));
		ws[k] &= m;
		const int64_t ds = dlo - 4 * k;
		if (ds >= 0 && ds <= 3)
			ws[k] ^= seed << (8 * (int)ds);
		else if (ds >= -3 && ds < 0)
			ws[k] ^= seed >> (-8 * (int)ds);
	}
	return (u32x4){ws[0], ws[1], ws[2], ws[3]};
}

// ---- plan kernel ----------------------------------------------------------
extern "C" __global__ __launch_bounds__(PECH_WG_THREADS) void pech_crc32c_plan(
	const pech_desc *__restrict__ descs, uint32_t n, uint32_t *__restrict__ lrs,
	uint32_t *__restrict__ partials, uint32_t *__restrict__ out)
{
	__shared__ uint32_t scratch[PECH_WG_THREADS / 64u];
	const uint32_t b = blockIdx.x * PECH_CHUNK + threadIdx.x;
	uint32_t rows = 0;
	if (b < n) {
		const pech_desc d = descs[b];
		rows = pech_rows(d.addr, d.len);
		out[b] = d.len ? 0u : d.seed;
	}
	uint32_t total;
	const uint32_t ex = block_excl_scan(rows, scratch, &total);
	if (b < n)
		lrs[b] = ex;
	if (threadIdx.x == 0)
		partials[blockIdx.x] = total;
}

// ---- main kernel ----------------------------------------------------------
#ifndef PECH_PREFETCH
#define PECH_PREFETCH 4 // rows in flight per lane
#endif

struct LoadCur {
	uint64_t pa;   // this lane's piece in the current row
	uint64_t a0;   // pieces below a0 are virtual zeros
	uint32_t left; // rows left in the buffer, current included
	uint32_t b;
	pech_desc nd;  // prefetched descriptor of buffer b+1
};

struct CompCur {
	uint64_t pa;
	uint64_t ptr;
	uint32_t len, seed;
	uint32_t lr, rows, z;
	uint32_t b, seg0;
	uint32_t edge;
	pech_desc nd;
};

extern "C" __global__ __launch_bounds__(PECH_WG_THREADS, 1) void pech_crc32c_main(
	const pech_desc *__restrict__ descs, uint32_t n, const uint32_t *__restrict__ lrs,
	const uint32_t *__restrict__ partials, uint32_t nchunks, const uint32_t *__restrict__ consts,
	uint32_t *__restrict__ out, uint32_t rpg_min)
{
	__shared__ __attribute__((aligned(16))) uint32_t lds[L_BYTES / 4u];
	const uint32_t tid = threadIdx.x;

	// chunk row offsets and the batch's total row count
	uint32_t Rtot;
	{
		const uint32_t pv = tid < nchunks ? partials[tid] : 0u;
		const uint32_t ex = block_excl_scan(pv, lds + L_MISC / 4u, &Rtot);
		lds[L_CHUNK / 4u + tid] = ex;
	}
	const uint64_t G = (uint64_t)gridDim.x * PECH_GROUPS_PER_WG;
	uint64_t rpg64 = ((uint64_t)Rtot + G - 1) / G;
	const uint32_t rpg = (uint32_t)(rpg64 < rpg_min ? rpg_min : rpg64);
	if ((uint64_t)blockIdx.x * PECH_GROUPS_PER_WG * rpg >= Rtot)
		return; // whole workgroup idle (small batch)

	// stage the tables: A_128 replicated once per bank, the rest single copy
	for (uint32_t j = tid; j < 8192u; j += PECH_WG_THREADS) {
		const uint32_t A = j << 4;
		const uint32_t k = ((A >> 16) << 1) | ((A >> 7) & 1u);
		const uint32_t v = consts[PECH_C_TAB128 + k * 256u + ((A >> 8) & 0xFFu)];
		*(uint4 *)((char *)lds + A) = make_uint4(v, v, v, v);
	}
	{
		const uint4 *c4 = (const uint4 *)(consts + PECH_C_TAB4);
		for (uint32_t j = tid; j < (PECH_C_WORDS - PECH_C_TAB4) / 4u; j += PECH_WG_THREADS)
			*(uint4 *)((char *)lds + L_TAB4 + 16u * j) = c4[j];
	}
	__syncthreads();

	const uint32_t lane = tid & 63u, g8 = tid & 7u;
	const uint32_t lreg = ((lane & 31u) << 2) | (1u << 16);
	const uint64_t r0 = ((uint64_t)blockIdx.x * PECH_GROUPS_PER_WG + (tid >> 3)) * rpg;
	if (r0 >= Rtot)
		return;
	uint32_t rem = (uint32_t)(((uint64_t)Rtot - r0) < rpg ? ((uint64_t)Rtot - r0) : rpg);

	// locate the first buffer: chunk by binary search in LDS, then an 8-ary
	// search over the chunk's row offsets with the group's 8 lanes
	uint32_t clo = 0, chi = nchunks;
	while (chi - clo > 1) {
		const uint32_t mid = (clo + chi) >> 1;
		if (lds[L_CHUNK / 4u + mid] <= r0)
			clo = mid;
		else
			chi = mid;
	}
	const uint32_t rr = (uint32_t)(r0 - lds[L_CHUNK / 4u + clo]);
	uint32_t blo = clo * PECH_CHUNK, bhi = min(n, blo + PECH_CHUNK);
	while (bhi - blo > 1) {
		const uint32_t step = (bhi - blo + 7u) >> 3;
		const uint32_t p = blo + g8 * step;
		const bool ok = p < bhi && lrs[p] <= rr;
		const uint64_t bal = __ballot(ok);
		const uint32_t cnt = __popc((uint32_t)(bal >> (lane & ~7u)) & 0xFFu);
		blo = blo + (cnt - 1u) * step;
		bhi = min(bhi, blo + step);
	}

	CompCur C;
	LoadCur L;
	{
		const pech_desc d = load_desc(descs, blo);
		const uint32_t lr = rr - lrs[blo];
		const uint32_t rows = pech_rows(d.addr, d.len);
		const uint64_t a1 = (d.addr + (d.len < 4u ? 4u : d.len) + 15u) & ~(uint64_t)15;
		const uint64_t vb = a1 - (uint64_t)PECH_ROW_BYTES * rows;
		C.pa = vb + (uint64_t)PECH_ROW_BYTES * lr + 16u * g8;
		C.ptr = d.addr;
		C.len = d.len;
		C.seed = d.seed;
		C.lr = lr;
		C.rows = rows;
		C.z = (uint32_t)(a1 - (d.addr + d.len));
		C.b = blo;
		C.seg0 = lr;
		C.edge = (((d.addr | (d.addr + d.len)) & 15u) != 0) || d.seed != 0;
		L.pa = C.pa;
		L.a0 = d.addr & ~(uint64_t)15;
		L.left = rows - lr;
		L.b = blo;
		if (blo + 1 < n) {
			L.nd = load_desc(descs, blo + 1);
			C.nd = L.nd;
		} else {
			L.nd = pech_desc{0, 0, 0};
			C.nd = L.nd;
		}
	}

	const uint32_t total = rem;
	u32x4 ring[PECH_PREFETCH];
	uint32_t issued = 0;
#pragma unroll
	for (int i = 0; i < PECH_PREFETCH; ++i) {
		ring[i] = (u32x4)(0u);
		if (issued < total) {
			if (L.pa >= L.a0)
				ring[i] = *(g_u32x4 *)L.pa;
			++issued;
			if (issued < total) {
				// advance the load cursor one row
				L.pa += PECH_ROW_BYTES;
				if (--L.left == 0) {
					uint32_t b = L.b + 1;
					pech_desc d = L.nd;
					while (d.len == 0) {
						++b;
						d = load_desc(descs, b);
					}
					const uint32_t rows = pech_rows(d.addr, d.len);
					const uint64_t a1 = (d.addr + (d.len < 4u ? 4u : d.len) + 15u) & ~(uint64_t)15;
					L.pa = a1 - (uint64_t)PECH_ROW_BYTES * rows + 16u * g8;
					L.a0 = d.addr & ~(uint64_t)15;
					L.left = rows;
					L.b = b;
					if (b + 1 < n)
						L.nd = load_desc(descs, b + 1);
				}
			}
		}
	}

	uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
	uint32_t done = 0;
	while (done < total) {
#pragma unroll
		for (int i = 0; i < PECH_PREFETCH; ++i) {
			if (done < total) {
				u32x4 w = ring[i];
				if (issued < total) {
					u32x4 v = (u32x4)(0u);
					if (L.pa >= L.a0)
						v = *(g_u32x4 *)L.pa;
					ring[i] = v;
					++issued;
					if (issued < total) {
						L.pa += PECH_ROW_BYTES;
						if (--L.left == 0) {
							uint32_t b = L.b + 1;
							pech_desc d = L.nd;
							while (d.len == 0) {
								++b;
								d = load_desc(descs, b);
							}
							const uint32_t rows = pech_rows(d.addr, d.len);
							const uint64_t a1 = (d.addr + (d.len < 4u ? 4u : d.len) + 15u) & ~(uint64_t)15;
							L.pa = a1 - (uint64_t)PECH_ROW_BYTES * rows + 16u * g8;
							L.a0 = d.addr & ~(uint64_t)15;
							L.left = rows;
							L.b = b;
							if (b + 1 < n)
								L.nd = load_desc(descs, b + 1);
						}
					}
				}

				if (C.edge && (C.lr <= 1u || C.lr + 1u == C.rows))
					w = fix_piece(w, C.pa, C.ptr, C.len, C.seed);
				s0 = adv128(lds, s0, lreg) ^ w.x;
				s1 = adv128(lds, s1, lreg) ^ w.y;
				s2 = adv128(lds, s2, lreg) ^ w.z;
				s3 = adv128(lds, s3, lreg) ^ w.w;
				++C.lr;
				C.pa += PECH_ROW_BYTES;
				++done;

				if (C.lr == C.rows || done == total) {
					// fold the 4 streams of the lane, then the 8 lanes of the row
					uint32_t u = adv_tab(lds, L_TAB4, s0) ^ s1;
					u = adv_tab(lds, L_TAB4, u) ^ s2;
					u = adv_tab(lds, L_TAB4, u) ^ s3;
					u = adv_tab(lds, L_TAB4, u);
					uint32_t o, lo, hi;
					o = __shfl_xor(u, 1);
					lo = (g8 & 1u) ? o : u;
					hi = (g8 & 1u) ? u : o;
					u = adv_tab(lds, L_TAB16, lo) ^ hi;
					o = __shfl_xor(u, 2);
					lo = (g8 & 2u) ? o : u;
					hi = (g8 & 2u) ? u : o;
					u = adv_tab(lds, L_TAB32, lo) ^ hi;
					o = __shfl_xor(u, 4);
					lo = (g8 & 4u) ? o : u;
					hi = (g8 & 4u) ? u : o;
					u = adv_tab(lds, L_TAB64, lo) ^ hi;
					// shift to the buffer's end, undo the z trailing zeros
					const uint32_t k = C.rows - C.lr;
					if (C.z)
						u = gf2_mulmod(lds[L_XINV / 4u + C.z], u);
#pragma unroll
					for (uint32_t i6 = 0; i6 < 5; ++i6) {
						const uint32_t dg = (k >> (6u * i6)) & 63u;
						if (dg)
							u = gf2_mulmod(lds[L_POWR / 4u + 64u * i6 + dg], u);
					}
					if (g8 == 0) {
						if (C.seg0 == 0 && k == 0)
							out[C.b] = u;
						else
							atomicXor(out + C.b, u);
					}
					s0 = s1 = s2 = s3 = 0;
					if (done < total) {
						// next buffer
						uint32_t b = C.b + 1;
						pech_desc d = C.nd;
						while (d.len == 0) {
							++b;
							d = load_desc(descs, b);
						}
						const uint32_t rows = pech_rows(d.addr, d.len);
						const uint64_t a1 = (d.addr + (d.len < 4u ? 4u : d.len) + 15u) & ~(uint64_t)15;
						C.pa = a1 - (uint64_t)PECH_ROW_BYTES * rows + 16u * g8;
						C.ptr = d.addr;
						C.len = d.len;
						C.seed = d.seed;
						C.lr = 0;
						C.rows = rows;
						C.z = (uint32_t)(a1 - (d.addr + d.len));
						C.b = b;
						C.seg0 = 0;
						C.edge = (((d.addr | (d.addr + d.len)) & 15u) != 0) || d.seed != 0;
						if (b + 1 < n)
							C.nd = load_desc(descs, b + 1);
					}
				}
			}
		}
	}
}

// ---- host-side launchers (used by crc32c_api.cpp) -------------------------
extern "C" hipError_t pech_launch_plan(const pech_desc *descs, uint32_t n, uint32_t *lrs, uint32_t *partials,
				       uint32_t *out, hipStream_t stream)
{
	const uint32_t nch = (n + PECH_CHUNK - 1) / PECH_CHUNK;
	hipLaunchKernelGGL(pech_crc32c_plan, dim3(nch), dim3(PECH_WG_THREADS), 0, stream, descs, n, lrs, partials,
			   out);
	return hipGetLastError();
}

extern "C" hipError_t pech_launch_main(const pech_desc *descs, uint32_t n, const uint32_t *lrs,
				       const uint32_t *partials, const uint32_t *consts, uint32_t *out,
				       uint32_t ncu, uint32_t rpg_min, hipStream_t stream)
{
	const uint32_t nch = (n + PECH_CHUNK - 1) / PECH_CHUNK;
	hipLaunchKernelGGL(pech_crc32c_main, dim3(ncu), dim3(PECH_WG_THREADS), 0, stream, descs, n, lrs, partials,
			   nch, consts, out, rpg_min);
	return hipGetLastError();
}
