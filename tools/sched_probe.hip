// sched_probe.hip -- work-distribution probes on the GPU box (not product
// code).  A pure nontemporal read stream with the CRC kernel's access shape
// (8-lane groups walking 128-byte rows, 8 rows in flight per lane, one
// 1024-thread workgroup per CU, 16 waves), over 1 GiB, with three schedules:
//   static   every wave reads an equal contiguous share (the r01 schedule)
//   claims   the same shares, but each wave claims its next S rows with a
//            64-bit atomicAdd on its own control word one step ahead
//            (measures what the claims cost while the chip streams)
//   steal    claims + work stealing: a wave whose share is exhausted samples
//            64 other waves' control words in one vector load, takes half of
//            the largest remainder from its end with a 64-bit CAS, and
//            continues (its own word then holds the stolen range, so it can
//            be stolen from in turn)
//   xcd      static shares per XCD in proportion to weights the host
//            recalibrates from the previous launches' per-XCD finish times
//            (each workgroup takes a slot on its XCD with one atomicAdd at
//            entry; s_memrealtime telemetry per workgroup)
// and a read+write copy probe (same shape, nontemporal loads and stores):
// the denominator for the fused CRC + copy kernel.
// Build: make build/sched_probe.  Output: one JSON object.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) u32x4 g_u32x4w;

#define CHECK(x)                                                               \
	do {                                                                   \
		hipError_t e = (x);                                            \
		if (e != hipSuccess) {                                         \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
			exit(1);                                               \
		}                                                              \
	} while (0)

#define D 8          // rows in flight per lane
#define WAVES 16     // per workgroup
#define ROW 128u

__device__ __forceinline__ uint32_t uni(uint32_t v)
{
	return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ u32x4 ld(const uint8_t *p, uint64_t row, uint32_t g8)
{
	return __builtin_nontemporal_load((g_u32x4 *)(p + row * ROW + 16u * g8));
}

__device__ __forceinline__ uint64_t ctl_pack(uint32_t b, uint32_t e)
{
	return ((uint64_t)e << 32) | b;
}

// One step = rows [b, b + n) of the row space, the 8 groups taking 8
// contiguous slices.  Per lane: first row and count.
struct PStep {
	uint32_t row, n; // this lane's group slice
	uint32_t T;      // max slice length (loop trip count), 0 = no step
};

__device__ __forceinline__ PStep make_step(uint32_t b, uint32_t n, uint32_t grp)
{
	PStep s;
	const uint32_t q = n >> 3, rm = n & 7u;
	s.row = b + grp * q + min(grp, rm);
	s.n = q + (grp < rm ? 1u : 0u);
	s.T = n ? q + (rm ? 1u : 0u) : 0u;
	return s;
}

// steal: returns the first step of the stolen range (T == 0: nothing found)
template <bool STEAL>
__device__ __forceinline__ PStep steal(uint64_t *ctl, uint32_t W, uint32_t w, uint32_t S, uint32_t lane, uint32_t grp,
				       uint32_t *nsteal)
{
	PStep none;
	none.T = 0;
	none.row = none.n = 0;
	if (!STEAL)
		return none;
	for (uint32_t attempt = 0; attempt < 4; ++attempt) {
		const uint32_t cand = (w + 1u + (lane + 64u * attempt) * 67u) % W;
		const uint64_t v = __hip_atomic_load(ctl + cand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const uint32_t b = (uint32_t)v, e = (uint32_t)(v >> 32);
		uint32_t rem = e > b ? e - b : 0u;
		// wave max of rem, and the lowest lane holding it
		uint32_t m = rem;
#pragma unroll
		for (uint32_t d = 1; d < 64; d <<= 1)
			m = max(m, (uint32_t)__shfl_xor(m, d));
		m = uni(m);
		if (m < 2u * S)
			continue;
		const uint64_t hit = __ballot(rem == m);
		const uint32_t src = (uint32_t)__builtin_ctzll(hit);
		const uint32_t vc = uni(__shfl(cand, src));
		uint64_t cur = __shfl(v, src);
		for (uint32_t tries = 0; tries < 3; ++tries) {
			const uint32_t cb = uni((uint32_t)cur), ce = uni((uint32_t)(cur >> 32));
			if (ce <= cb || ce - cb < 2u * S)
				break;
			const uint32_t K = ((ce - cb) / 2u) / S * S;
			uint64_t prev = 0;
			if (lane == 0) {
				uint64_t expct = cur;
				__hip_atomic_compare_exchange_strong(ctl + vc, &expct, ctl_pack(cb, ce - K), __ATOMIC_RELAXED,
								     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				prev = expct; // the value seen (== cur on success)
			}
			prev = ((uint64_t)uni((uint32_t)(__shfl(prev, 0) >> 32)) << 32) | uni((uint32_t)__shfl(prev, 0));
			if (prev == cur) {
				// [ce - K, ce) is ours; the first S rows are taken now
				const uint32_t s0 = ce - K;
				if (lane == 0) {
					__hip_atomic_exchange(ctl + w, ctl_pack(s0 + S, ce), __ATOMIC_RELAXED,
							      __HIP_MEMORY_SCOPE_AGENT);
					atomicAdd(nsteal, 1u);
				}
				return make_step(s0, S, grp);
			}
			cur = prev;
		}
	}
	return none;
}

// MODE 4: like 3, but the wave's share is cut the other way: step j gives
// group g rows [r0 + g * (share / 8) + j * S / 8, + S / 8) -- every group
// walks ONE contiguous range of the share across the steps (as 2 consecutive
// 4 KiB buffers per group would), instead of a fresh 32-row block per step.
__device__ __forceinline__ PStep make_step_cols(uint32_t r0, uint32_t share, uint32_t j, uint32_t S, uint32_t grp)
{
	PStep s;
	const uint32_t per = share / 8u, k = S / 8u;
	s.row = r0 + grp * per + j * k;
	s.n = min(k, per - min(per, j * k));
	s.T = s.n ? k : 0u;
	return s;
}

template <int MODE> // 0 static, 1 claims, 2 steal, 3 static in steps of S rows (no atomics), 4 see above
__global__ __launch_bounds__(1024, 1) void k_sched(const uint8_t *p, uint32_t R, uint64_t *ctl, uint32_t S,
						    uint32_t *out, uint32_t *nsteal)
{
	const uint32_t W = gridDim.x * WAVES;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t r0 = (uint32_t)((uint64_t)R * w / W), r1 = (uint32_t)((uint64_t)R * (w + 1u) / W);
	u32x4 acc = (u32x4)(0u), ring[D];
	PStep cur;
	uint32_t next_r = r0;
	if (MODE == 5) { // static, after an idle prologue of about S microseconds (s_memrealtime: 100 MHz)
		const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
		while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * S)
			__builtin_amdgcn_s_sleep(8);
	}
	if (MODE == 0 || MODE == 5) {
		cur = make_step(r0, r1 - r0, grp); // the whole share is one step
	} else if (MODE == 3) {
		const uint32_t n0 = min(S, r1 - r0);
		cur = make_step(r0, n0, grp);
		next_r = r0 + n0;
	} else if (MODE == 4) {
		cur = make_step_cols(r0, r1 - r0, 0, S, grp);
		next_r = 1; // next step index
	} else {
		const uint32_t n0 = min(S, r1 - r0);
		if (lane == 0)
			__hip_atomic_exchange(ctl + w, ctl_pack(r0 + n0, r1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		cur = make_step(r0, n0, grp);
	}
	if (cur.T == 0)
		return;
#pragma unroll
	for (int i = 0; i + 1 < D; ++i)
		ring[i] = ld(p, cur.row + min((uint32_t)i, cur.n - 1u), g8);
	while (cur.T) {
		// claim the step after this one now: consumed at this step's end
		uint64_t fut = 0;
		if (MODE != 0 && MODE != 3 && MODE != 4 && lane == 0)
			fut = __hip_atomic_fetch_add(ctl + w, (uint64_t)S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const uint32_t nblk = (cur.T + D - 1) / D;
		uint32_t blk = 0;
		for (; blk + 1 < nblk; ++blk) {
#pragma unroll
			for (int i = 0; i < D; ++i) {
				const uint32_t r = blk * D + i;
				ring[(i + D - 1) % D] = ld(p, cur.row + min(r + D - 1, cur.n - 1u), g8);
				acc ^= ring[i];
			}
		}
		// next step
		PStep nxt;
		nxt.T = 0;
		nxt.row = nxt.n = 0;
		if (MODE == 3) {
			if (next_r < r1) {
				nxt = make_step(next_r, min(S, r1 - next_r), grp);
				next_r += min(S, r1 - next_r);
			}
		} else if (MODE == 4) {
			nxt = make_step_cols(r0, r1 - r0, next_r++, S, grp);
			nxt.T = uni(nxt.T);
		} else if (MODE != 0) {
			fut = __shfl(fut, 0);
			const uint32_t b = uni((uint32_t)fut), e = uni((uint32_t)(fut >> 32));
			if (b < e)
				nxt = make_step(b, min(S, e - b), grp);
			else
				nxt = steal<MODE == 2>(ctl, W, w, S, lane, grp, nsteal);
		}
		const bool more = nxt.T != 0;
		const uint32_t r = blk * D;
#pragma unroll
		for (int i = 0; i < D; ++i) {
			const uint32_t ri = r + i;
			// the last block's prefetch already fetches the next step's first rows
			const uint32_t lr = ri + D - 1;
			if (i == 0)
				ring[D - 1] = ld(p, cur.row + min(lr, cur.n - 1u), g8);
			else
				ring[i - 1] = more ? ld(p, nxt.row + min((uint32_t)(i - 1), nxt.n - 1u), g8)
						   : ld(p, cur.row + cur.n - 1u, g8);
			if (ri < cur.n)
				acc ^= ring[i];
		}
		cur = nxt;
	}
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (x == 0x12345678u)
		out[w] = x;
}

// XCD-weighted static: XCD x streams rows [X[x], X[x+1]) split over the
// workgroups that land on it (slot from a per-XCD counter), 16 waves each
__global__ __launch_bounds__(1024, 1) void k_xcd(const uint8_t *p, uint32_t R, const uint32_t *X, uint32_t *slots,
						 uint32_t nslot, uint64_t *tele, uint32_t *out)
{
	__shared__ uint32_t s_slot, s_xcc;
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t wv = threadIdx.x / 64u;
	const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
	if (threadIdx.x == 0) {
		uint32_t xcc;
		asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
		s_xcc = xcc & 7u;
		s_slot = atomicAdd(slots + (xcc & 7u), 1u);
	}
	__syncthreads();
	const uint32_t xcc = s_xcc, slot = s_slot;
	u32x4 acc = (u32x4)(0u), ring[D];
	if (slot < nslot) {
		const uint32_t a = X[xcc], b = X[xcc + 1];
		const uint32_t ws0 = a + (uint32_t)((uint64_t)(b - a) * slot / nslot);
		const uint32_t ws1 = a + (uint32_t)((uint64_t)(b - a) * (slot + 1) / nslot);
		const uint32_t r0 = ws0 + (uint32_t)((uint64_t)(ws1 - ws0) * wv / WAVES);
		const uint32_t r1 = ws0 + (uint32_t)((uint64_t)(ws1 - ws0) * (wv + 1) / WAVES);
		const PStep s = make_step(r0, r1 - r0, grp);
		if (s.T) {
#pragma unroll
			for (int i = 0; i + 1 < D; ++i)
				ring[i] = ld(p, s.row + min((uint32_t)i, s.n - 1u), g8);
			for (uint32_t r = 0; r < s.T; r += D) {
#pragma unroll
				for (int i = 0; i < D; ++i) {
					ring[(i + D - 1) % D] = ld(p, s.row + min(r + i + D - 1, s.n - 1u), g8);
					if (r + i < s.n)
						acc ^= ring[i];
				}
			}
		}
	}
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (x == 0x12345678u)
		out[blockIdx.x] = x;
	__syncthreads();
	if (threadIdx.x == 0) {
		tele[3 * blockIdx.x] = t0;
		tele[3 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
		tele[3 * blockIdx.x + 2] = ((uint64_t)slot << 8) | xcc;
	}
}

// Global pool: units of S rows, handed out by NC counters (counter k serves
// units k, k + NC, ...; wave w draws from counter w % NC, so every counter
// sees waves of every XCD).  Each wave keeps AHEAD claims in flight: the
// claim for step i + AHEAD is issued when step i starts, so an atomic's
// latency under streaming load (~10-20 us) is covered by AHEAD steps.
template <int AHEAD>
__global__ __launch_bounds__(1024, 1) void k_pool(const uint8_t *p, uint32_t R, uint32_t *ctr, uint32_t S, uint32_t NC,
						  uint32_t *out)
{
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t k = w % NC;
	const uint32_t nunits = (R + S - 1) / S;
	uint32_t q[AHEAD + 1]; // claimed unit indices, oldest first (lane 0's results)
#pragma unroll
	for (int i = 0; i <= AHEAD; ++i)
		q[i] = lane == 0 ? atomicAdd(ctr + k, 1u) : 0u;
	auto unit_step = [&](uint32_t c) {
		const uint32_t u = k + NC * uni(__shfl(c, 0));
		PStep s;
		if (u >= nunits) {
			s.T = 0;
			s.row = s.n = 0;
			return s;
		}
		return make_step(u * S, min(S, R - u * S), grp);
	};
	PStep cur = unit_step(q[0]);
	u32x4 acc = (u32x4)(0u), ring[D];
	if (cur.T == 0)
		return;
#pragma unroll
	for (int i = 0; i + 1 < D; ++i)
		ring[i] = ld(p, cur.row + min((uint32_t)i, cur.n - 1u), g8);
	while (cur.T) {
		// shift the claim queue, claim one more
#pragma unroll
		for (int i = 0; i < AHEAD; ++i)
			q[i] = q[i + 1];
		q[AHEAD] = lane == 0 ? atomicAdd(ctr + k, 1u) : 0u;
		const uint32_t nblk = (cur.T + D - 1) / D;
		uint32_t blk = 0;
		for (; blk + 1 < nblk; ++blk) {
#pragma unroll
			for (int i = 0; i < D; ++i) {
				const uint32_t r = blk * D + i;
				ring[(i + D - 1) % D] = ld(p, cur.row + min(r + D - 1, cur.n - 1u), g8);
				acc ^= ring[i];
			}
		}
		const PStep nxt = unit_step(q[0]);
		const bool more = nxt.T != 0;
		const uint32_t r = blk * D;
#pragma unroll
		for (int i = 0; i < D; ++i) {
			const uint32_t ri = r + i;
			if (i == 0)
				ring[D - 1] = ld(p, cur.row + min(ri + D - 1, cur.n - 1u), g8);
			else
				ring[i - 1] = more ? ld(p, nxt.row + min((uint32_t)(i - 1), nxt.n - 1u), g8)
						   : ld(p, cur.row + cur.n - 1u, g8);
			if (ri < cur.n)
				acc ^= ring[i];
		}
		cur = nxt;
	}
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (x == 0x12345678u)
		out[w] = x;
}

// Workgroup pool: the workgroup's contiguous range (an equal 1/grid share of
// the rows) is cut into items of S rows; its 16 waves take items in order
// with an LDS counter (ds_add_rtn, no device atomics), each wave claiming its
// next item AHEAD one item early.  Waves of one CU then finish within about
// one item of each other, whatever their issue priority.
__global__ __launch_bounds__(1024, 1) void k_wgpool(const uint8_t *p, uint32_t R, uint32_t S, uint32_t *out)
{
	__shared__ uint32_t next_item;
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t b0 = (uint32_t)((uint64_t)R * blockIdx.x / gridDim.x);
	const uint32_t b1 = (uint32_t)((uint64_t)R * (blockIdx.x + 1) / gridDim.x);
	const uint32_t nitems = (b1 - b0 + S - 1) / S;
	if (threadIdx.x == 0)
		next_item = WAVES; // items 0..15 go to waves 0..15 without a claim
	__syncthreads();
	const uint32_t wv = threadIdx.x / 64u;
	auto item_step = [&](uint32_t it) {
		PStep s;
		if (it >= nitems) {
			s.T = 0;
			s.row = s.n = 0;
			return s;
		}
		const uint32_t a = b0 + it * S;
		return make_step(a, min(S, b1 - a), grp);
	};
	PStep cur = item_step(wv);
	u32x4 acc = (u32x4)(0u), ring[D];
	if (cur.T) {
#pragma unroll
		for (int i = 0; i + 1 < D; ++i)
			ring[i] = ld(p, cur.row + min((uint32_t)i, cur.n - 1u), g8);
	}
	while (cur.T) {
		uint32_t claim = 0;
		if (lane == 0)
			claim = atomicAdd(&next_item, 1u);
		const uint32_t nblk = (cur.T + D - 1) / D;
		uint32_t blk = 0;
		for (; blk + 1 < nblk; ++blk) {
#pragma unroll
			for (int i = 0; i < D; ++i) {
				const uint32_t r = blk * D + i;
				ring[(i + D - 1) % D] = ld(p, cur.row + min(r + D - 1, cur.n - 1u), g8);
				acc ^= ring[i];
			}
		}
		const PStep nxt = item_step(uni(__shfl(claim, 0)));
		const bool more = nxt.T != 0;
		const uint32_t r = blk * D;
#pragma unroll
		for (int i = 0; i < D; ++i) {
			const uint32_t ri = r + i;
			if (i == 0)
				ring[D - 1] = ld(p, cur.row + min(ri + D - 1, cur.n - 1u), g8);
			else
				ring[i - 1] = more ? ld(p, nxt.row + min((uint32_t)(i - 1), nxt.n - 1u), g8)
						   : ld(p, cur.row + cur.n - 1u, g8);
			if (ri < cur.n)
				acc ^= ring[i];
		}
		cur = nxt;
	}
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (x == 0x12345678u)
		out[w] = x;
}

// static shares, each wave's share read starting at a pseudo-random row of
// it and wrapping around (ROT 1: one offset per wave, shared by its 8
// groups; ROT 2: one offset per group): do the streams' aligned starts cost?
template <int ROT>
__global__ __launch_bounds__(1024, 1) void k_rot(const uint8_t *p, uint32_t R, uint32_t *out)
{
	const uint32_t W = gridDim.x * WAVES;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t r0 = (uint32_t)((uint64_t)R * w / W), r1 = (uint32_t)((uint64_t)R * (w + 1u) / W);
	const PStep s = make_step(r0, r1 - r0, grp);
	const uint32_t key = ROT == 1 ? w : w * 8u + grp;
	const uint32_t off = s.n ? (key * 2654435761u >> 7) % s.n : 0u;
	u32x4 acc = (u32x4)(0u), ring[D];
	for (uint32_t r = 0; r < s.T; r += D) {
#pragma unroll
		for (int i = 0; i < D; ++i) {
			uint32_t q = min(r + i, s.n - 1u) + off;
			q = q >= s.n ? q - s.n : q;
			ring[i] = ld(p, s.row + q, g8);
		}
#pragma unroll
		for (int i = 0; i < D; ++i)
			if (r + i < s.n)
				acc ^= ring[i];
	}
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (x == 0x12345678u)
		out[w] = x;
}

// read+write copy, static shares, same shape
__global__ __launch_bounds__(1024, 1) void k_copy(const uint8_t *p, uint8_t *q, uint32_t R)
{
	const uint32_t W = gridDim.x * WAVES;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t r0 = (uint32_t)((uint64_t)R * w / W), r1 = (uint32_t)((uint64_t)R * (w + 1u) / W);
	const PStep s = make_step(r0, r1 - r0, grp);
	u32x4 ring[D];
	for (uint32_t r = 0; r < s.n; r += D) {
#pragma unroll
		for (int i = 0; i < D; ++i)
			ring[i] = ld(p, s.row + min(r + i, s.n - 1u), g8);
#pragma unroll
		for (int i = 0; i < D; ++i)
			if (r + i < s.n)
				__builtin_nontemporal_store(ring[i], (g_u32x4w *)(q + (uint64_t)(s.row + r + i) * ROW + 16u * g8));
	}
}

// read+write copy, static shares, but each wave-instruction covers 1 KiB of
// consecutive rows (lane l: row 8k + l/8, piece l%8) instead of 8 rows of 8
// separate streams
template <bool NT>
__global__ __launch_bounds__(1024, 1) void k_copy_wide(const uint8_t *p, uint8_t *q, uint32_t R)
{
	const uint32_t W = gridDim.x * WAVES;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u;
	const uint32_t r0 = (uint32_t)((uint64_t)R * w / W), r1 = (uint32_t)((uint64_t)R * (w + 1u) / W);
	const uint64_t lo = (uint64_t)r0 * ROW + 16u * lane, hi = (uint64_t)r1 * ROW;
	u32x4 ring[D];
	for (uint64_t a = lo; a < hi; a += D * 1024u) {
#pragma unroll
		for (int i = 0; i < D; ++i) {
			const uint64_t ai = min(a + i * 1024u, hi - 16u);
			ring[i] = NT ? __builtin_nontemporal_load((g_u32x4 *)(p + ai)) : *(g_u32x4 *)(p + ai);
		}
#pragma unroll
		for (int i = 0; i < D; ++i)
			if (a + i * 1024u < hi) {
				if (NT)
					__builtin_nontemporal_store(ring[i], (g_u32x4w *)(q + a + i * 1024u));
				else
					*(g_u32x4w *)(q + a + i * 1024u) = ring[i];
			}
	}
}

// static shares read with the rows interleaved over the groups: group g walks
// rows g, g+8, g+16, ... of the wave's share, so each wave-instruction reads
// 8 consecutive rows (1 KiB contiguous, the grid's per-instruction footprint)
// inside the persistent shape; DD rows in flight per lane
template <int DD>
__global__ __launch_bounds__(1024, 1) void k_wide(const uint8_t *p, uint32_t R, uint32_t *out)
{
	const uint32_t W = gridDim.x * WAVES;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t r0 = (uint32_t)((uint64_t)R * w / W), r1 = (uint32_t)((uint64_t)R * (w + 1u) / W);
	const uint32_t n = r1 - r0, T = (n + 7u) / 8u;
	const uint32_t ng = n > grp ? (n - grp + 7u) / 8u : 0u;
	if (T == 0)
		return;
	const uint32_t last = ng ? ng - 1u : 0u, base = ng ? r0 + grp : r0;
	u32x4 acc = (u32x4)(0u), ring[DD];
#pragma unroll
	for (int i = 0; i + 1 < DD; ++i)
		ring[i] = ld(p, base + 8u * min((uint32_t)i, last), g8);
	for (uint32_t j = 0; j < T; j += DD) {
#pragma unroll
		for (int i = 0; i < DD; ++i) {
			ring[(i + DD - 1) % DD] = ld(p, base + 8u * min(j + i + DD - 1, last), g8);
			if (j + i < ng)
				acc ^= ring[i];
		}
	}
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (x == 0x12345678u)
		out[w] = x;
}

// plain one-element-per-thread float4 copy over a large grid (not persistent)
template <bool NT>
__global__ __launch_bounds__(256) void k_copy_grid(const uint8_t *p, uint8_t *q, uint64_t n16)
{
	const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
	if (i < n16) {
		const u32x4 v = NT ? __builtin_nontemporal_load((g_u32x4 *)(p + 16u * i)) : *(g_u32x4 *)(p + 16u * i);
		if (NT)
			__builtin_nontemporal_store(v, (g_u32x4w *)(q + 16u * i));
		else
			*(g_u32x4w *)(q + 16u * i) = v;
	}
}

// plain one-element-per-thread read over a large grid (not persistent)
template <bool NT>
__global__ __launch_bounds__(256) void k_read_grid(const uint8_t *p, uint64_t n16, uint32_t *out)
{
	const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
	if (i < n16) {
		const u32x4 v = NT ? __builtin_nontemporal_load((g_u32x4 *)(p + 16u * i)) : *(g_u32x4 *)(p + 16u * i);
		if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u)
			out[i & 1023u] = 1u;
	}
}

// persistent waves over interleaved tiles: wave w takes tiles w, w + W, ...
// of TR rows; in a tile its 8 groups each walk TR/8 consecutive rows (the
// CRC kernel's group shape), D rows in flight.  All waves stay inside a
// window of about W tiles, moving through memory together (DRAM locality),
// instead of 32K streams spread over the whole batch.
template <bool COPY, uint32_t TR>
__global__ __launch_bounds__(1024, 1) void k_tiles(const uint8_t *p, uint8_t *q, uint32_t R, uint32_t *out)
{
	const uint32_t W = gridDim.x * WAVES;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	constexpr uint32_t PER = TR / 8u;
	static_assert(PER % D == 0, "tile slice: whole ring blocks");
	u32x4 acc = (u32x4)(0u), ring[D];
	for (uint32_t t = w; (uint64_t)t * TR < R; t += W) {
		const uint32_t row0 = t * TR + grp * PER;
		for (uint32_t r = 0; r < PER; r += D) {
#pragma unroll
			for (int i = 0; i < D; ++i)
				ring[i] = ld(p, min(row0 + r + i, R - 1u), g8);
#pragma unroll
			for (int i = 0; i < D; ++i) {
				if (COPY) {
					if (row0 + r + i < R)
						__builtin_nontemporal_store(ring[i], (g_u32x4w *)(q + (uint64_t)(row0 + r + i) * ROW + 16u * g8));
				} else {
					acc ^= ring[i];
				}
			}
		}
	}
	if (!COPY && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
		out[w] = 1u;
}

// The in-flight address window (round 3): the grid copy with one float4 per
// thread runs at 335 us, with 4 / 16 per thread at 366 / 401, i.e. as slow as
// the static persistent copy -- the wider the set of addresses in flight at
// once, the slower, with no store waits in any of them.  Persistent tiles
// (k_tiles) should give the grid's narrow window, but waves drift apart
// (oldest-first issue), so here every wave runs the same number of tile
// steps with a workgroup barrier after each: a CU's 16 waves stay on 16
// adjacent tiles and the chip on a window of about W tiles.  144 KiB of LDS
// as the CRC kernel, so one workgroup per CU.
template <bool COPY, uint32_t TR, bool SYNC>
__global__ __launch_bounds__(1024, 1) void k_tiles_sync(const uint8_t *p, uint8_t *q, uint32_t R, uint32_t *out)
{
	__shared__ uint32_t pad[36 * 1024];
	const uint32_t W = gridDim.x * WAVES;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	constexpr uint32_t PER = TR / 8u;
	static_assert(PER % D == 0, "tile slice: whole ring blocks");
	pad[threadIdx.x] = lane;
	const uint32_t ntiles = (R + TR - 1u) / TR, steps = (ntiles + W - 1u) / W;
	u32x4 acc = (u32x4)(0u), ring[D];
	for (uint32_t k = 0; k < steps; ++k) {
		const uint32_t t = k * W + w;
		if (t < ntiles) {
			const uint32_t row0 = t * TR + grp * PER;
			for (uint32_t r = 0; r < PER; r += D) {
#pragma unroll
				for (int i = 0; i < D; ++i)
					ring[i] = ld(p, min(row0 + r + i, R - 1u), g8);
#pragma unroll
				for (int i = 0; i < D; ++i) {
					if (COPY) {
						if (row0 + r + i < R)
							__builtin_nontemporal_store(ring[i],
										    (g_u32x4w *)(q + (uint64_t)(row0 + r + i) * ROW + 16u * g8));
					} else {
						acc ^= ring[i];
					}
				}
			}
		}
		if (SYNC)
			__syncthreads();
	}
	if (!COPY && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
		out[w] = pad[(threadIdx.x + 1u) & 1023u];
}

// The grid also deals consecutive 4 KiB pieces to consecutive workgroups, i.e.
// round robin over the XCDs; k_tiles gives a workgroup 16 consecutive tiles.
// Here tile t goes to workgroup t mod G first (wave (t / G) mod 16 of it), so
// neighbouring tiles are on different XCDs, as in the grid.
template <bool COPY, uint32_t TR>
__global__ __launch_bounds__(1024, 1) void k_tiles_xcd(const uint8_t *p, uint8_t *q, uint32_t R, uint32_t *out)
{
	__shared__ uint32_t pad[36 * 1024];
	const uint32_t G = gridDim.x, W = G * WAVES;
	const uint32_t wave = uni(threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	constexpr uint32_t PER = TR / 8u;
	static_assert(PER % D == 0, "tile slice: whole ring blocks");
	pad[threadIdx.x] = lane;
	u32x4 acc = (u32x4)(0u), ring[D];
	// this wave's tiles: t = k W + wave G + blockIdx.x
	for (uint32_t t = wave * G + blockIdx.x; (uint64_t)t * TR < R; t += W) {
		const uint32_t row0 = t * TR + grp * PER;
		for (uint32_t r = 0; r < PER; r += D) {
#pragma unroll
			for (int i = 0; i < D; ++i)
				ring[i] = ld(p, min(row0 + r + i, R - 1u), g8);
#pragma unroll
			for (int i = 0; i < D; ++i) {
				if (COPY) {
					if (row0 + r + i < R)
						__builtin_nontemporal_store(ring[i],
									    (g_u32x4w *)(q + (uint64_t)(row0 + r + i) * ROW + 16u * g8));
				} else {
					acc ^= ring[i];
				}
			}
		}
	}
	if (!COPY && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
		out[blockIdx.x] = pad[(threadIdx.x + 1u) & 1023u];
}

// The other explanation: static shares start on 256 KiB multiples (and their
// group slices on 32 KiB multiples), so the 32K streams may step through the
// same HBM channels in phase.  Here each group walks its slice from a hashed
// starting row (a multiple of D) and wraps around: same shares, same bytes,
// streams de-phased.
template <bool COPY, bool ROT>
__global__ __launch_bounds__(1024, 1) void k_rotated(const uint8_t *p, uint8_t *q, uint32_t R, uint32_t *out)
{
	__shared__ uint32_t pad[36 * 1024];
	const uint32_t W = gridDim.x * WAVES;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t r0 = (uint32_t)((uint64_t)R * w / W), r1 = (uint32_t)((uint64_t)R * (w + 1u) / W);
	const PStep s = make_step(r0, r1 - r0, grp);
	pad[threadIdx.x] = lane;
	const uint32_t blocks = s.n / D;
	const uint32_t o = ROT && blocks ? ((((w * 8u + grp) * 2654435761u) >> 9) % blocks) * D : 0u;
	u32x4 acc = (u32x4)(0u), ring[D];
	for (uint32_t r = 0; r < s.n; r += D) {
		uint32_t rows[D];
#pragma unroll
		for (int i = 0; i < D; ++i) {
			uint32_t j = o + r + i;
			j = j >= s.n ? j - s.n : j;
			rows[i] = s.row + min(j, s.n - 1u);
			ring[i] = ld(p, rows[i], g8);
		}
#pragma unroll
		for (int i = 0; i < D; ++i) {
			if (COPY) {
				if (r + i < s.n)
					__builtin_nontemporal_store(ring[i], (g_u32x4w *)(q + (uint64_t)rows[i] * ROW + 16u * g8));
			} else if (r + i < s.n) {
				acc ^= ring[i];
			}
		}
	}
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
		out[w] = pad[(threadIdx.x + 1u) & 1023u];
}

// Split roles: waves 0-7 of a workgroup only load (their vmcnt never holds a
// store), stage each 8-row block in LDS and hand it to their partner wave
// 8-15, which only stores (and so never waits for anything but its LDS
// slot).  Two 8 KiB slots per pair, LDS flags polled with s_sleep.  Tests
// whether the persistent copy's deficit against the grid is a wave waiting
// on its own store acknowledgements.
__global__ __launch_bounds__(1024, 1) void k_copy_split(const uint8_t *p, uint8_t *q, uint32_t R)
{
	__shared__ __attribute__((aligned(16))) u32x4 stage[8][2][D * 64]; // 128 KiB
	__shared__ uint32_t flag[8][2];
	const uint32_t wave = uni(threadIdx.x / 64u), pair = wave & 7u;
	const bool reader = wave < 8u;
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t W = gridDim.x * 8u, w = blockIdx.x * 8u + pair; // shares per pair
	const uint32_t r0 = (uint32_t)((uint64_t)R * w / W), r1 = (uint32_t)((uint64_t)R * (w + 1u) / W);
	const PStep s = make_step(r0, r1 - r0, grp);
	if (threadIdx.x < 16u)
		flag[threadIdx.x >> 1][threadIdx.x & 1u] = 0u;
	__syncthreads();
	const uint32_t nb = (s.T + D - 1u) / D; // blocks (wave-uniform: T)
	for (uint32_t b = 0; b < nb; ++b) {
		const uint32_t k = b & 1u, r = b * D;
		volatile uint32_t *f = &flag[pair][k];
		if (reader) {
			u32x4 v[D];
#pragma unroll
			for (int i = 0; i < D; ++i)
				v[i] = ld(p, s.row + min(r + i, s.n - 1u), g8);
			while (*f != 0u)
				__builtin_amdgcn_s_sleep(1);
#pragma unroll
			for (int i = 0; i < D; ++i)
				stage[pair][k][i * 64 + lane] = v[i];
			__builtin_amdgcn_s_waitcnt(0xc07f); // lgkmcnt(0): the slot's writes are done
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
			if (lane == 0)
				*f = 1u;
		} else {
			while (*f != 1u)
				__builtin_amdgcn_s_sleep(1);
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
			u32x4 v[D];
#pragma unroll
			for (int i = 0; i < D; ++i)
				v[i] = stage[pair][k][i * 64 + lane];
			__builtin_amdgcn_s_waitcnt(0xc07f);
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
			if (lane == 0)
				*f = 0u;
#pragma unroll
			for (int i = 0; i < D; ++i)
				if (r + i < s.n)
					__builtin_nontemporal_store(v[i], (g_u32x4w *)(q + (uint64_t)(s.row + r + i) * ROW + 16u * g8));
		}
	}
}

// Workgroup-interleaved rows: workgroup b owns a contiguous share of the
// batch, and its 128 lane groups walk it together -- group j of the
// workgroup takes rows j, j + 128, j + 256, ... of the share, so one row
// step of the workgroup reads (and writes) 16 KiB contiguous, and the CU's
// footprint in flight is one contiguous window.  (A CRC run over rows 128
// apart is Horner with x^(8 * 16 KiB) instead of x^(8 * 128): the same table
// size.)  D rows in flight per lane.
template <bool COPY, bool SYNC = false>
__global__ __launch_bounds__(1024, 1) void k_wg_interleave(const uint8_t *p, uint8_t *q, uint32_t R, uint32_t *out)
{
	__shared__ uint32_t pad[36 * 1024];
	const uint32_t G = gridDim.x, b = blockIdx.x;
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u;
	const uint32_t j = threadIdx.x >> 3; // lane group of the workgroup, 0..127
	const uint32_t r0 = (uint32_t)((uint64_t)R * b / G), r1 = (uint32_t)((uint64_t)R * (b + 1u) / G);
	pad[threadIdx.x] = lane;
	const uint32_t n = r1 - r0, steps = (n + 127u) / 128u; // row steps of the workgroup
	u32x4 acc = (u32x4)(0u), ring[D];
	for (uint32_t k = 0; k < steps; k += D) {
#pragma unroll
		for (int i = 0; i < D; ++i) {
			const uint32_t rr = (k + i) * 128u + j;
			ring[i] = ld(p, r0 + min(rr, n - 1u), g8);
		}
#pragma unroll
		for (int i = 0; i < D; ++i) {
			const uint32_t rr = (k + i) * 128u + j;
			if (rr < n) {
				if (COPY)
					__builtin_nontemporal_store(ring[i], (g_u32x4w *)(q + (uint64_t)(r0 + rr) * ROW + 16u * g8));
				else
					acc ^= ring[i];
			}
		}
		if (SYNC)
			__syncthreads(); // the workgroup's 16 waves stay on one window
	}
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
		out[b] = pad[(threadIdx.x + 1u) & 1023u];
}

// Small buffers (4 KiB = 32 rows, one per lane group per step, as the CRC
// kernels walk them): static shares (wave w takes buffers [w S, (w+1) S), 8
// per step) or workgroup-interleaved (step k of wave w takes buffers
// base + 128 k + 8 w .. + 7 of its workgroup's range: the workgroup's 128
// groups are on 128 consecutive buffers, one 512 KiB window per step).
template <bool COPY, bool IL>
__global__ __launch_bounds__(1024, 1) void k_small(const uint8_t *p, uint8_t *q, uint32_t R, uint32_t *out)
{
	__shared__ uint32_t pad[36 * 1024];
	constexpr uint32_t BR = 32u; // rows per buffer
	const uint32_t wave = uni(threadIdx.x / 64u), lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t nbuf = R / BR, G = gridDim.x;
	const uint32_t b0 = (uint32_t)((uint64_t)nbuf * blockIdx.x / G), b1 = (uint32_t)((uint64_t)nbuf * (blockIdx.x + 1u) / G);
	const uint32_t per = b1 - b0; // buffers of this workgroup
	pad[threadIdx.x] = lane;
	u32x4 acc = (u32x4)(0u), ring[D];
	const uint32_t steps = (per + 127u) / 128u;
	for (uint32_t k = 0; k < steps; ++k) {
		uint32_t b;
		bool ok;
		if (IL) {
			b = 128u * k + 8u * wave + grp;
			ok = b < per;
		} else {
			const uint32_t ws = (per + 15u) / 16u; // the wave's share, 8 buffers per step
			b = ws * wave + 8u * k + grp;
			ok = 8u * k + grp < ws && b < per;
		}
		const uint32_t row0 = (b0 + (ok ? b : 0u)) * BR;
		for (uint32_t r = 0; r < BR; r += D) {
#pragma unroll
			for (int i = 0; i < D; ++i)
				ring[i] = ld(p, row0 + r + i, g8);
#pragma unroll
			for (int i = 0; i < D; ++i) {
				if (COPY) {
					if (ok)
						__builtin_nontemporal_store(ring[i], (g_u32x4w *)(q + (uint64_t)(row0 + r + i) * ROW + 16u * g8));
				} else {
					acc ^= ring[i];
				}
			}
		}
	}
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
		out[blockIdx.x] = pad[(threadIdx.x + 1u) & 1023u];
}

// grid copy with one float4 per thread, workgroups of NT threads holding
// PADW words of LDS (occupancy control)
template <int NT, int PADW>
__global__ __launch_bounds__(NT) void k_copy_grid_pad(const uint8_t *p, uint8_t *q, uint64_t n16)
{
	__shared__ uint32_t pad[PADW];
	const uint64_t i = blockIdx.x * (uint64_t)NT + threadIdx.x;
	pad[threadIdx.x % PADW] = threadIdx.x;
	if (i < n16) {
		u32x4 v = __builtin_nontemporal_load((g_u32x4 *)(p + 16u * i));
		if (pad[(threadIdx.x + 1) % PADW] == 0x12345678u)
			v.x = 0;
		__builtin_nontemporal_store(v, (g_u32x4w *)(q + 16u * i));
	}
}

// static copy whose stores lag one block: block k+1's loads are issued before
// block k's stores, so a wait for a load never covers the stores just issued
// (vmcnt retires loads and stores in issue order).  Two DD-row buffers.
template <int DD>
__global__ __launch_bounds__(1024, 1) void k_copy_lag(const uint8_t *p, uint8_t *q, uint32_t R)
{
	__shared__ uint32_t pad[36 * 1024];
	const uint32_t W = gridDim.x * WAVES;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t r0 = (uint32_t)((uint64_t)R * w / W), r1 = (uint32_t)((uint64_t)R * (w + 1u) / W);
	const PStep s = make_step(r0, r1 - r0, grp);
	pad[threadIdx.x] = lane;
	if (s.n == 0)
		return;
	u32x4 a[DD], b[DD];
#pragma unroll
	for (int i = 0; i < DD; ++i)
		a[i] = ld(p, s.row + min((uint32_t)i, s.n - 1u), g8);
	for (uint32_t r = 0; r < s.n; r += 2 * DD) {
#pragma unroll
		for (int i = 0; i < DD; ++i)
			b[i] = ld(p, s.row + min(r + DD + i, s.n - 1u), g8);
#pragma unroll
		for (int i = 0; i < DD; ++i)
			if (r + i < s.n)
				__builtin_nontemporal_store(a[i], (g_u32x4w *)(q + (uint64_t)(s.row + r + i) * ROW + 16u * g8));
#pragma unroll
		for (int i = 0; i < DD; ++i)
			a[i] = ld(p, s.row + min(r + 2 * DD + i, s.n - 1u), g8);
#pragma unroll
		for (int i = 0; i < DD; ++i)
			if (r + DD + i < s.n)
				__builtin_nontemporal_store(b[i], (g_u32x4w *)(q + (uint64_t)(s.row + r + DD + i) * ROW + 16u * g8));
	}
	if (pad[(threadIdx.x + 1u) & 1023u] == 0x12345678u)
		q[0] = 0;
}

// copy variants for the occupancy question: the static copy with DD rows in
// flight and MINB workgroups per CU (MINB 2: 32 waves per CU, <= 64 VGPRs)
template <int DD, int MINB>
__global__ __launch_bounds__(1024, MINB) void k_copy_occ(const uint8_t *p, uint8_t *q, uint32_t R)
{
	const uint32_t W = gridDim.x * WAVES;
	const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	const uint32_t r0 = (uint32_t)((uint64_t)R * w / W), r1 = (uint32_t)((uint64_t)R * (w + 1u) / W);
	const PStep s = make_step(r0, r1 - r0, grp);
	u32x4 ring[DD];
	for (uint32_t r = 0; r < s.n; r += DD) {
#pragma unroll
		for (int i = 0; i < DD; ++i)
			ring[i] = ld(p, s.row + min(r + i, s.n - 1u), g8);
#pragma unroll
		for (int i = 0; i < DD; ++i)
			if (r + i < s.n)
				__builtin_nontemporal_store(ring[i], (g_u32x4w *)(q + (uint64_t)(s.row + r + i) * ROW + 16u * g8));
	}
}

// grid copy, K float4 per thread (grid-stride inside the workgroup's block)
template <int K>
__global__ __launch_bounds__(256) void k_copy_gridk(const uint8_t *p, uint8_t *q, uint64_t n16)
{
	const uint64_t b = blockIdx.x * 256ull * K + threadIdx.x;
	u32x4 v[K];
#pragma unroll
	for (int k = 0; k < K; ++k)
		v[k] = __builtin_nontemporal_load((g_u32x4 *)(p + 16u * min(b + 256u * k, n16 - 1u)));
#pragma unroll
	for (int k = 0; k < K; ++k)
		if (b + 256u * k < n16)
			__builtin_nontemporal_store(v[k], (g_u32x4w *)(q + 16u * (b + 256u * k)));
}

// The grid copy carrying a stand-in for a per-tile partial CRC:
// 256-thread workgroups, one float4 per thread (4 KiB tile), TABW words of
// tables filled into LDS per workgroup from global memory (L2-resident), 16
// byte lookups per thread (dependent for TABW < 4096, slice-by-16 otherwise),
// a 6-round cross-lane fold with 4 lookups a round, one partial per wave.
template <int TABW>
__global__ __launch_bounds__(256) void k_copy_tilecrc(const uint8_t *p, uint8_t *q, uint64_t n16, const uint32_t *tab,
						      uint32_t *part)
{
	__shared__ uint32_t t[TABW];
	for (uint32_t k = threadIdx.x; k < (uint32_t)TABW; k += 256u)
		t[k] = tab[k];
	const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
	const u32x4 v = __builtin_nontemporal_load((g_u32x4 *)(p + 16u * min(i, n16 - 1u)));
	if (i < n16)
		__builtin_nontemporal_store(v, (g_u32x4w *)(q + 16u * i));
	__syncthreads();
	const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
	uint32_t c = 0;
#pragma unroll
	for (int j = 0; j < 16; ++j) {
		const uint32_t b = (w4[j >> 2] >> (8 * (j & 3))) & 255u;
		if (TABW >= 4096)
			c ^= t[(15 - j) * 256 + b];
		else
			c = t[((c ^ b) & 255u) | ((j & (TABW / 256 - 1)) << 8)] ^ (c >> 8);
	}
	for (int off = 1; off < 64; off <<= 1) {
		const uint32_t o = __shfl_xor(c, off);
		c = o ^ t[c & 255u] ^ t[((c >> 8) & 255u) | (256u % TABW)] ^ t[((c >> 16) & 255u) | (512u % TABW)] ^
		    t[(c >> 24) | (768u % TABW)];
	}
	if ((threadIdx.x & 63u) == 0 && i < n16)
		part[i >> 6] = c;
}

// folds 64 consecutive partials into one word (the batch's second launch)
__global__ __launch_bounds__(256) void k_tile_fold(const uint32_t *part, uint64_t nout, uint32_t *out)
{
	const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
	if (i >= nout)
		return;
	uint32_t c = 0;
	for (int k = 0; k < 64; ++k)
		c = (c << 1 | c >> 31) ^ part[64u * i + k];
	out[i] = c;
}

// Static shares for the first ncu workgroups over rows [0, Rs), then X
// extra workgroups over [Rs, R) in equal pieces: the dispatcher hands each
// extra workgroup to the first CU whose static workgroup has exited (one
// workgroup per CU at 1024 threads + the kernel's LDS), balancing the end of
// the launch with no atomics.  Extra workgroups idle `idle` us first (the CRC
// kernel's prologue).  Same read loop for both kinds.
__global__ __launch_bounds__(1024, 1) void k_extra(const uint8_t *p, uint32_t R, uint32_t ncu, uint32_t Rs, uint32_t X,
						   uint32_t idle, uint32_t *out)
{
	__shared__ uint32_t pad[36 * 1024]; // 144 KiB: one workgroup per CU, as the CRC kernel
	const uint32_t b = blockIdx.x, wave = threadIdx.x / 64u;
	const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
	uint64_t lo, hi;
	uint32_t wi, nw;
	if (b < ncu) {
		lo = 0;
		hi = Rs;
		wi = b * WAVES + wave;
		nw = ncu * WAVES;
	} else {
		const uint64_t k = b - ncu;
		lo = Rs + (uint64_t)(R - Rs) * k / X;
		hi = Rs + (uint64_t)(R - Rs) * (k + 1) / X;
		wi = wave;
		nw = WAVES;
		const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
		while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * idle)
			__builtin_amdgcn_s_sleep(8);
	}
	const uint32_t r0 = (uint32_t)(lo + (hi - lo) * wi / nw), r1 = (uint32_t)(lo + (hi - lo) * (wi + 1) / nw);
	const PStep s = make_step(r0, r1 - r0, grp);
	u32x4 acc = (u32x4)(0u), ring[D];
	if (s.T) {
#pragma unroll
		for (int i = 0; i + 1 < D; ++i)
			ring[i] = ld(p, s.row + min((uint32_t)i, s.n - 1u), g8);
		for (uint32_t r = 0; r < s.T; r += D) {
#pragma unroll
			for (int i = 0; i < D; ++i) {
				ring[(i + D - 1) % D] = ld(p, s.row + min(r + i + D - 1, s.n - 1u), g8);
				if (r + i < s.n)
					acc ^= ring[i];
			}
		}
	}
	pad[threadIdx.x] = acc.x;
	__syncthreads();
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w ^ pad[(threadIdx.x + 1u) & 1023u];
	if (x == 0x12345678u)
		out[b] = x;
}

static int g_entries;
static const char *sep(void)
{
	return g_entries++ ? ",\n" : "";
}

// launch-cost probe: an empty kernel of the CRC kernel's launch
// shape, the same with its LDS footprint, the LDS table fill alone (27 KiB of
// constants -> 128 KiB of bank-replicated tables, one barrier), and a fill
// followed by the static read of `R` rows
__global__ __launch_bounds__(1024, 1) void k_empty(uint32_t *out)
{
	if (threadIdx.x == 1023u && blockIdx.x == 0x7FFFFFFFu)
		out[0] = 1u;
}

template <bool READ>
__global__ __launch_bounds__(1024, 1) void k_fill(const uint32_t *tab, const uint8_t *p, uint32_t R, uint32_t *out)
{
	extern __shared__ uint32_t lds[];
	const uint32_t tid = threadIdx.x;
	uint32_t t[4];
#pragma unroll
	for (int j = 0; j < 4; ++j)
		t[j] = tab[tid + j * 1024u]; // 16 KiB of it per workgroup, as the kernel's A_128 tables
#pragma unroll
	for (int j = 0; j < 4; ++j)
#pragma unroll
		for (int c = 0; c < 8; ++c) // 32 bank copies of 4 KiB = 128 KiB
			lds[((tid + j * 1024u) * 8u + c) & (32768u - 1u)] = t[j] ^ c;
	__syncthreads();
	uint32_t acc = lds[(tid * 37u) & 32767u];
	if (READ) {
		const uint32_t W = gridDim.x * WAVES;
		const uint32_t w = uni(blockIdx.x * WAVES + threadIdx.x / 64u);
		const uint32_t lane = threadIdx.x & 63u, g8 = lane & 7u, grp = lane >> 3;
		const uint32_t r0 = (uint32_t)((uint64_t)R * w / W), r1 = (uint32_t)((uint64_t)R * (w + 1u) / W);
		// the wave's share in 8 group slices, D loads in flight
		const uint32_t n = r1 - r0, q = n >> 3, rm = n & 7u;
		const uint32_t st = r0 + grp * q + min(grp, rm), nn = q + (grp < rm ? 1u : 0u);
		u32x4 v = (u32x4)(0u);
		for (uint32_t r = 0; r < nn; r += D) {
			u32x4 ring[D];
#pragma unroll
			for (int i = 0; i < D; ++i)
				ring[i] = ld(p, st + min(r + i, nn - 1u), g8);
#pragma unroll
			for (int i = 0; i < D; ++i)
				v ^= ring[i];
		}
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x12345678u)
		out[tid] = acc;
}

// instruction-fetch probe: the same count of VALU instructions as straight-
// line code (NI x 8-byte v_add3_u32, cold in the instruction cache at every
// dispatch?) or as a loop over 256 of them (2 KiB of code)
template <int NI, bool LOOP>
__global__ __launch_bounds__(1024) void k_code(uint32_t *out)
{
	uint32_t a = threadIdx.x, b = blockIdx.x, c = 7u;
#define ADD3_8 "v_add3_u32 %0, %0, %1, %2\n" "v_add3_u32 %0, %0, %1, %2\n" "v_add3_u32 %0, %0, %1, %2\n" \
	"v_add3_u32 %0, %0, %1, %2\n" "v_add3_u32 %0, %0, %1, %2\n" "v_add3_u32 %0, %0, %1, %2\n" \
	"v_add3_u32 %0, %0, %1, %2\n" "v_add3_u32 %0, %0, %1, %2\n"
#define ADD3_64 ADD3_8 ADD3_8 ADD3_8 ADD3_8 ADD3_8 ADD3_8 ADD3_8 ADD3_8
	if (LOOP) {
#pragma unroll 1
		for (int it = 0; it < NI / 256; ++it) {
#pragma unroll
			for (int i = 0; i < 4; ++i)
				asm volatile(ADD3_64 : "+v"(a) : "v"(b), "v"(c));
		}
	} else {
#pragma unroll
		for (int i = 0; i < NI / 64; ++i)
			asm volatile(ADD3_64 : "+v"(a) : "v"(b), "v"(c));
	}
	if (a == 0x12345678u)
		out[threadIdx.x] = a;
}

// usage: sched_probe [reps] [all|read|copy] [MiB per launch, default 1024]
// (read: the static read stream only)
int main(int argc, char **argv)
{
	const char *which = argc > 2 ? argv[2] : "all";
	const bool all = !strcmp(which, "all"), only_read = !strcmp(which, "read"), only_copy = !strcmp(which, "copy");
	const size_t bytes = (size_t)(argc > 3 ? atoi(argv[3]) : 1024) << 20;
	const uint32_t R = (uint32_t)(bytes / ROW);
	hipDeviceProp_t prop;
	CHECK(hipGetDeviceProperties(&prop, 0));
	const int ncu = prop.multiProcessorCount;
	const uint32_t W = ncu * WAVES;
	uint8_t *buf[3];
	for (int i = 0; i < 3; ++i) {
		CHECK(hipMalloc(&buf[i], bytes));
		CHECK(hipMemset(buf[i], i + 1, bytes));
	}
	uint64_t *ctl;
	uint32_t *out, *nsteal;
	CHECK(hipMalloc(&ctl, W * 8u));
	CHECK(hipMalloc(&out, W * 4u));
	CHECK(hipMalloc(&nsteal, 4u));
	const int reps = argc > 1 ? atoi(argv[1]) : 20;
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	struct {
		const char *name;
		int mode;
		uint32_t S;
	} runs[] = {{"static", 0, 0},         {"claims S256", 1, 256},  {"steal S256", 2, 256},
		    {"steal S128", 2, 128},     {"steal S64", 2, 64},     {"claims S128", 1, 128},
		    {"static steps S256", 3, 256}, {"static steps S128", 3, 128}, {"column steps S256", 4, 256},
		    {"column steps S128", 4, 128}, {"static after 3 us idle", 5, 3}, {"static after 6 us idle", 5, 6},
		    {"static (again)", 0, 0}};
	printf("{\"device\": \"%s\", \"cus\": %d, \"bytes\": %zu, \"results\": [\n", prop.name, ncu, bytes);
	for (size_t k = 0; k < sizeof(runs) / sizeof(runs[0]); ++k) {
		const int md = runs[k].mode;
		const bool pick = all || (only_read && md == 0) || (!strcmp(which, "steps") && (md == 0 || md == 3 || md == 4)) ||
				  (!strcmp(which, "idle") && (md == 0 || md == 5));
		if (!pick)
			continue;
		float tot = 0, best = 1e9f;
		uint32_t steals = 0;
		for (int r = -2; r < reps; ++r) {
			CHECK(hipMemsetAsync(ctl, 0, W * 8u, 0));
			CHECK(hipMemsetAsync(nsteal, 0, 4u, 0));
			CHECK(hipEventRecord(e0, 0));
			const uint8_t *p = buf[(r + 4) % 2];
			if (runs[k].mode == 0)
				hipLaunchKernelGGL(k_sched<0>, dim3(ncu), dim3(1024), 0, 0, p, R, ctl, runs[k].S, out, nsteal);
			else if (runs[k].mode == 1)
				hipLaunchKernelGGL(k_sched<1>, dim3(ncu), dim3(1024), 0, 0, p, R, ctl, runs[k].S, out, nsteal);
			else if (runs[k].mode == 3)
				hipLaunchKernelGGL(k_sched<3>, dim3(ncu), dim3(1024), 0, 0, p, R, ctl, runs[k].S, out, nsteal);
			else if (runs[k].mode == 4)
				hipLaunchKernelGGL(k_sched<4>, dim3(ncu), dim3(1024), 0, 0, p, R, ctl, runs[k].S, out, nsteal);
			else if (runs[k].mode == 5)
				hipLaunchKernelGGL(k_sched<5>, dim3(ncu), dim3(1024), 0, 0, p, R, ctl, runs[k].S, out, nsteal);
			else
				hipLaunchKernelGGL(k_sched<2>, dim3(ncu), dim3(1024), 0, 0, p, R, ctl, runs[k].S, out, nsteal);
			CHECK(hipEventRecord(e1, 0));
			CHECK(hipEventSynchronize(e1));
			float ms;
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			if (r >= 0) {
				tot += ms;
				best = ms < best ? ms : best;
			}
			CHECK(hipMemcpy(&steals, nsteal, 4, hipMemcpyDeviceToHost));
		}
		printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"best_us\": %.2f, \"GBps\": %.1f, \"steals_last\": %u}",
		       sep(), runs[k].name, tot / reps * 1e3, best * 1e3, bytes / (tot / reps * 1e-3) / 1e9, steals);
	}
	if (all || !strcmp(which, "rot")) {
		for (int pass = 0; pass < 2; ++pass)
			for (int mode = 0; mode < 3; ++mode) {
				float tot = 0;
				for (int r = -2; r < reps; ++r) {
					CHECK(hipEventRecord(e0, 0));
					const uint8_t *p = buf[(r + 4) % 2];
					if (mode == 0)
						hipLaunchKernelGGL(k_rot<0>, dim3(ncu), dim3(1024), 0, 0, p, R, out);
					else if (mode == 1)
						hipLaunchKernelGGL(k_rot<1>, dim3(ncu), dim3(1024), 0, 0, p, R, out);
					else
						hipLaunchKernelGGL(k_rot<2>, dim3(ncu), dim3(1024), 0, 0, p, R, out);
					CHECK(hipEventRecord(e1, 0));
					CHECK(hipEventSynchronize(e1));
					float ms;
					CHECK(hipEventElapsedTime(&ms, e0, e1));
					if (r >= 0)
						tot += ms;
				}
				static const char *nm[] = {"static, no rotation (no prefetch ring)", "rotated per wave",
							   "rotated per group"};
				printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}", sep(), nm[mode], tot / reps * 1e3,
				       bytes / (tot / reps * 1e-3) / 1e9);
			}
	}
	if (all || !strcmp(which, "wgpool")) {
		// workgroup pools: items of S rows claimed through LDS
		const uint32_t Ss[] = {512, 256, 128, 64};
		for (int pass = 0; pass < 2; ++pass)
			for (uint32_t S : Ss) {
				float tot = 0, best = 1e9f;
				for (int r = -2; r < reps; ++r) {
					CHECK(hipEventRecord(e0, 0));
					hipLaunchKernelGGL(k_wgpool, dim3(ncu), dim3(1024), 0, 0, buf[(r + 4) % 2], R, S, out);
					CHECK(hipEventRecord(e1, 0));
					CHECK(hipEventSynchronize(e1));
					float ms;
					CHECK(hipEventElapsedTime(&ms, e0, e1));
					if (r >= 0) {
						tot += ms;
						best = ms < best ? ms : best;
					}
				}
				printf("%s  {\"probe\": \"wgpool S%u\", \"us\": %.2f, \"best_us\": %.2f, \"GBps\": %.1f}", sep(), S,
				       tot / reps * 1e3, best * 1e3, bytes / (tot / reps * 1e-3) / 1e9);
			}
	}
	if (all) {
		// global pool with claims AHEAD steps ahead
		uint32_t *ctr;
		CHECK(hipMalloc(&ctr, 64 * 4));
		struct {
			const char *name;
			int ahead;
			uint32_t S, NC;
		} pr[] = {{"pool S256 ahead1 nc8", 1, 256, 8},  {"pool S256 ahead2 nc8", 2, 256, 8},
			  {"pool S128 ahead2 nc8", 2, 128, 8},  {"pool S128 ahead3 nc8", 3, 128, 8},
			  {"pool S64 ahead3 nc16", 3, 64, 16},  {"pool S256 ahead2 nc32", 2, 256, 32},
			  {"pool S128 ahead3 nc32", 3, 128, 32}};
		for (size_t k = 0; k < sizeof(pr) / sizeof(pr[0]); ++k) {
			float tot = 0, best = 1e9f;
			for (int r = -2; r < reps; ++r) {
				CHECK(hipMemsetAsync(ctr, 0, 64 * 4, 0));
				CHECK(hipEventRecord(e0, 0));
				const uint8_t *p = buf[(r + 4) % 2];
				if (pr[k].ahead == 1)
					hipLaunchKernelGGL(k_pool<1>, dim3(ncu), dim3(1024), 0, 0, p, R, ctr, pr[k].S, pr[k].NC, out);
				else if (pr[k].ahead == 2)
					hipLaunchKernelGGL(k_pool<2>, dim3(ncu), dim3(1024), 0, 0, p, R, ctr, pr[k].S, pr[k].NC, out);
				else
					hipLaunchKernelGGL(k_pool<3>, dim3(ncu), dim3(1024), 0, 0, p, R, ctr, pr[k].S, pr[k].NC, out);
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0) {
					tot += ms;
					best = ms < best ? ms : best;
				}
			}
			printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"best_us\": %.2f, \"GBps\": %.1f}", sep(), pr[k].name,
			       tot / reps * 1e3, best * 1e3, bytes / (tot / reps * 1e-3) / 1e9);
		}
	}
	if (all) {
		// XCD-weighted static, weights recalibrated after every launch
		uint32_t *X, *slots;
		uint64_t *tele;
		CHECK(hipMalloc(&X, 9 * 4));
		CHECK(hipMalloc(&slots, 8 * 4));
		CHECK(hipMalloc(&tele, (size_t)ncu * 3 * 8));
		std::vector<uint64_t> ht((size_t)ncu * 3);
		double w[8];
		for (int x = 0; x < 8; ++x)
			w[x] = 1.0 / 8;
		const uint32_t nslot = (ncu + 7) / 8;
		const int cal = 20;
		float tot = 0, first = 0;
		char hist[4096];
		int hl = 0;
		for (int r = 0; r < cal + reps; ++r) {
			uint32_t hx[9];
			double acc = 0;
			hx[0] = 0;
			for (int x = 0; x < 8; ++x) {
				acc += w[x];
				hx[x + 1] = x == 7 ? R : (uint32_t)(acc * R);
			}
			CHECK(hipMemcpy(X, hx, 9 * 4, hipMemcpyHostToDevice));
			CHECK(hipMemset(slots, 0, 8 * 4));
			CHECK(hipEventRecord(e0, 0));
			hipLaunchKernelGGL(k_xcd, dim3(ncu), dim3(1024), 0, 0, buf[r % 2], R, X, slots, nslot, tele, out);
			CHECK(hipEventRecord(e1, 0));
			CHECK(hipEventSynchronize(e1));
			float ms;
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			if (r == 0)
				first = ms;
			if (r >= cal)
				tot += ms;
			CHECK(hipMemcpy(ht.data(), tele, ht.size() * 8, hipMemcpyDeviceToHost));
			uint64_t tmin = ~0ull, tend[8] = {0};
			for (int b = 0; b < ncu; ++b) {
				tmin = ht[3 * b] < tmin ? ht[3 * b] : tmin;
				const int x = (int)(ht[3 * b + 2] & 7u);
				tend[x] = ht[3 * b + 1] > tend[x] ? ht[3 * b + 1] : tend[x];
			}
			double rate[8], rs = 0;
			for (int x = 0; x < 8; ++x) {
				rate[x] = w[x] / (double)(tend[x] - tmin);
				rs += rate[x];
			}
			for (int x = 0; x < 8; ++x)
				w[x] = 0.5 * w[x] + 0.5 * rate[x] / rs;
			if (r < 6 || r == cal + reps - 1) {
				hl += snprintf(hist + hl, sizeof(hist) - hl, "%s[%.1f", hl ? ", " : "", ms * 1e3);
				for (int x = 0; x < 8; ++x)
					hl += snprintf(hist + hl, sizeof(hist) - hl, ", %.1f", (tend[x] - tmin) / 100.0);
				hl += snprintf(hist + hl, sizeof(hist) - hl, "]");
			}
		}
		printf("%s  {\"probe\": \"xcd-weighted static\", \"us\": %.2f, \"first_us\": %.2f, \"GBps\": %.1f, "
		       "\"weights\": [%.4f, %.4f, %.4f, %.4f, %.4f, %.4f, %.4f, %.4f], "
		       "\"launch_us_and_xcd_end_us\": [%s]}",
		       sep(), tot / reps * 1e3, first * 1e3, bytes / (tot / reps * 1e-3) / 1e9, w[0], w[1], w[2], w[3], w[4], w[5],
		       w[6], w[7], hist);
	}
	if (all || only_copy) {
		float tot = 0;
		for (int r = -2; r < reps; ++r) {
			CHECK(hipEventRecord(e0, 0));
			hipLaunchKernelGGL(k_copy, dim3(ncu), dim3(1024), 0, 0, buf[(r + 4) % 2], buf[2], R);
			CHECK(hipEventRecord(e1, 0));
			CHECK(hipEventSynchronize(e1));
			float ms;
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			if (r >= 0)
				tot += ms;
		}
		printf("%s  {\"probe\": \"copy static (read+write)\", \"us\": %.2f, \"GBps_read_plus_write\": %.1f}",
		       sep(), tot / reps * 1e3, 2.0 * bytes / (tot / reps * 1e-3) / 1e9);
		const char *names[4] = {"copy wide 1 KiB/wave nt", "copy wide 1 KiB/wave", "copy grid float4 nt", "copy grid float4"};
		for (int v = 0; v < 4; ++v) {
			tot = 0;
			for (int r = -2; r < reps; ++r) {
				CHECK(hipEventRecord(e0, 0));
				const uint8_t *src = buf[(r + 4) % 2];
				if (v == 0)
					hipLaunchKernelGGL(k_copy_wide<true>, dim3(ncu), dim3(1024), 0, 0, src, buf[2], R);
				else if (v == 1)
					hipLaunchKernelGGL(k_copy_wide<false>, dim3(ncu), dim3(1024), 0, 0, src, buf[2], R);
				else if (v == 2)
					hipLaunchKernelGGL(k_copy_grid<true>, dim3((unsigned)(bytes / 16 / 256)), dim3(256), 0, 0, src, buf[2],
							   (uint64_t)(bytes / 16));
				else
					hipLaunchKernelGGL(k_copy_grid<false>, dim3((unsigned)(bytes / 16 / 256)), dim3(256), 0, 0, src, buf[2],
							   (uint64_t)(bytes / 16));
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0)
					tot += ms;
			}
			printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"GBps_read_plus_write\": %.1f}", sep(), names[v],
			       tot / reps * 1e3, 2.0 * bytes / (tot / reps * 1e-3) / 1e9);
		}
	}
	if (all || !strcmp(which, "locality")) {
		const char *names[] = {"read grid float4 nt", "read tiles 8 KiB", "read tiles 32 KiB", "read tiles 128 KiB",
				       "copy tiles 8 KiB", "copy tiles 32 KiB", "copy tiles 128 KiB"};
		for (int v = 0; v < 7; ++v) {
			float tot = 0;
			for (int r = -2; r < reps; ++r) {
				CHECK(hipEventRecord(e0, 0));
				const uint8_t *src = buf[(r + 4) % 2];
				switch (v) {
				case 0:
					hipLaunchKernelGGL(k_read_grid<true>, dim3((unsigned)(bytes / 16 / 256)), dim3(256), 0, 0, src,
							   (uint64_t)(bytes / 16), out);
					break;
				case 1: hipLaunchKernelGGL((k_tiles<false, 64>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 2: hipLaunchKernelGGL((k_tiles<false, 256>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 3: hipLaunchKernelGGL((k_tiles<false, 1024>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 4: hipLaunchKernelGGL((k_tiles<true, 64>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 5: hipLaunchKernelGGL((k_tiles<true, 256>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				default: hipLaunchKernelGGL((k_tiles<true, 1024>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				}
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0)
					tot += ms;
			}
			const double f = v >= 4 ? 2.0 : 1.0;
			printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"GBps%s\": %.1f}", sep(), names[v], tot / reps * 1e3,
			       v >= 4 ? "_read_plus_write" : "", f * bytes / (tot / reps * 1e-3) / 1e9);
		}
	}
	if (!strcmp(which, "extra")) {
		struct {
			uint32_t permille, X, idle;
		} ex[] = {{0, 0, 0}, {50, 256, 0}, {100, 256, 0}, {100, 512, 0}, {200, 512, 0}, {100, 256, 4},
			  {100, 512, 4}, {200, 512, 4}, {200, 1024, 4}, {0, 0, 0}};
		for (size_t v = 0; v < sizeof(ex) / sizeof(ex[0]); ++v) {
			float tot = 0;
			const uint32_t Rs = (uint32_t)((uint64_t)R * (1000u - ex[v].permille) / 1000u);
			for (int r = -2; r < reps; ++r) {
				CHECK(hipEventRecord(e0, 0));
				hipLaunchKernelGGL(k_extra, dim3(ncu + ex[v].X), dim3(1024), 0, 0, buf[(r + 4) % 2], R, (uint32_t)ncu, Rs,
						   ex[v].X, ex[v].idle, out);
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0)
					tot += ms;
			}
			printf("%s  {\"probe\": \"static + %u extra WGs over the last %.1f%% (idle %u us)\", \"us\": %.2f, \"GBps\": %.1f}",
			       sep(), ex[v].X, ex[v].permille / 10.0, ex[v].idle, tot / reps * 1e3, bytes / (tot / reps * 1e-3) / 1e9);
		}
	}
	if (!strcmp(which, "pipe")) {
		// Pipelined rate: 40 launches alternating over two streams (the bench's
		// `value` pass), each persistent launch holding 144 KiB of LDS per
		// workgroup as the CRC kernel does (one workgroup per CU), so a CU takes
		// the next launch's workgroup only once all 16 waves of the current one
		// have exited.  Static shares vs the intra-workgroup pool (waves of a CU
		// finish together), and the grid for reference.
		hipStream_t st[2];
		CHECK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
		CHECK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
		const size_t lds = 144u * 1024u;
		CHECK(hipFuncSetAttribute((const void *)k_sched<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		CHECK(hipFuncSetAttribute((const void *)k_wgpool, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		const char *names[] = {"pipe static", "pipe wgpool S512", "pipe wgpool S256", "pipe grid float4 nt",
				       "serial static", "serial wgpool S512"};
		const int nl = 40;
		for (int pass = 0; pass < 2; ++pass)
			for (int v = 0; v < 6; ++v) {
				double best = 1e30;
				for (int rep = 0; rep < 3; ++rep) {
					CHECK(hipDeviceSynchronize());
					const auto t0 = std::chrono::steady_clock::now();
					for (int i = 0; i < nl; ++i) {
						hipStream_t s = v >= 4 ? st[0] : st[i & 1];
						const uint8_t *src = buf[i & 1];
						if (v == 0 || v == 4)
							hipLaunchKernelGGL(k_sched<0>, dim3(ncu), dim3(1024), lds, s, src, R, ctl, 0u, out, nsteal);
						else if (v == 1 || v == 5)
							hipLaunchKernelGGL(k_wgpool, dim3(ncu), dim3(1024), lds, s, src, R, 512u, out);
						else if (v == 2)
							hipLaunchKernelGGL(k_wgpool, dim3(ncu), dim3(1024), lds, s, src, R, 256u, out);
						else
							hipLaunchKernelGGL(k_read_grid<true>, dim3((unsigned)(bytes / 16 / 256)), dim3(256), 0, s,
									   src, (uint64_t)(bytes / 16), out);
					}
					CHECK(hipDeviceSynchronize());
					const double us =
						std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / nl;
					best = us < best ? us : best;
				}
				printf("%s  {\"probe\": \"%s\", \"us_per_launch\": %.2f, \"GBps\": %.1f}", sep(), names[v], best,
				       bytes / (best * 1e-6) / 1e9);
			}
	}
	if (!strcmp(which, "wide")) { // group-sliced static vs row-interleaved static vs the grid, two passes
		const char *names[] = {"read static (group slices)", "read static wide D8 (rows interleaved over groups)",
				       "read static wide D12", "read grid float4 nt"};
		for (int pass = 0; pass < 2; ++pass)
			for (int v = 0; v < 4; ++v) {
				float tot = 0;
				for (int r = -2; r < reps; ++r) {
					CHECK(hipEventRecord(e0, 0));
					const uint8_t *src = buf[(r + 4) % 2];
					if (v == 0)
						hipLaunchKernelGGL(k_sched<0>, dim3(ncu), dim3(1024), 0, 0, src, R, ctl, 0u, out, nsteal);
					else if (v == 1)
						hipLaunchKernelGGL(k_wide<8>, dim3(ncu), dim3(1024), 0, 0, src, R, out);
					else if (v == 2)
						hipLaunchKernelGGL(k_wide<12>, dim3(ncu), dim3(1024), 0, 0, src, R, out);
					else
						hipLaunchKernelGGL(k_read_grid<true>, dim3((unsigned)(bytes / 16 / 256)), dim3(256), 0, 0,
								   src, (uint64_t)(bytes / 16), out);
					CHECK(hipEventRecord(e1, 0));
					CHECK(hipEventSynchronize(e1));
					float ms;
					CHECK(hipEventElapsedTime(&ms, e0, e1));
					if (r >= 0)
						tot += ms;
				}
				printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}", sep(), names[v], tot / reps * 1e3,
				       bytes / (tot / reps * 1e-3) / 1e9);
			}
	}
	if (!strcmp(which, "launch")) {
		// packet-level durations (hipExtLaunchKernelGGL start/stop events, as
		// the library times its main kernel) against launch size
		hipEvent_t a0, a1;
		CHECK(hipEventCreate(&a0));
		CHECK(hipEventCreate(&a1));
		uint32_t *tab;
		CHECK(hipMalloc(&tab, 6912u * 4u));
		CHECK(hipMemset(tab, 7, 6912u * 4u));
		const size_t lds = 144u << 10;
		CHECK(hipFuncSetAttribute((const void *)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		CHECK(hipFuncSetAttribute((const void *)k_fill<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		CHECK(hipFuncSetAttribute((const void *)k_fill<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		CHECK(hipFuncSetAttribute((const void *)k_sched<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		const int mibs[] = {0, 4, 32, 128, 256, 1024};
		const char *names[] = {"empty, no LDS", "empty, 144 KiB LDS", "table fill only", "static read, no LDS",
				       "static read, 144 KiB LDS", "table fill + static read", "grid read float4"};
		for (int v = 0; v < 7; ++v)
			for (int mi = 0; mi < 6; ++mi) {
				const int mib = mibs[mi];
				if ((v < 3) != (mib == 0))
					continue;
				const size_t sz = (size_t)mib << 20;
				const uint32_t Rs = (uint32_t)(sz / ROW);
				const size_t regions = sz ? (2 * bytes) / sz : 1;
				float tot = 0;
				for (int r = -2; r < reps; ++r) {
					const size_t reg = (size_t)(r + 2) % regions;
					const uint8_t *pp = sz ? buf[(reg * sz) / bytes] + (reg * sz) % bytes : buf[0];
					switch (v) {
					case 0: hipExtLaunchKernelGGL(k_empty, dim3(ncu), dim3(1024), 0, 0, a0, a1, 0, out); break;
					case 1: hipExtLaunchKernelGGL(k_empty, dim3(ncu), dim3(1024), lds, 0, a0, a1, 0, out); break;
					case 2: hipExtLaunchKernelGGL(k_fill<false>, dim3(ncu), dim3(1024), lds, 0, a0, a1, 0, tab, pp, Rs, out); break;
					case 3: hipExtLaunchKernelGGL(k_sched<0>, dim3(ncu), dim3(1024), 0, 0, a0, a1, 0, pp, Rs, ctl, 0u, out, nsteal); break;
					case 4: hipExtLaunchKernelGGL(k_sched<0>, dim3(ncu), dim3(1024), lds, 0, a0, a1, 0, pp, Rs, ctl, 0u, out, nsteal); break;
					case 5: hipExtLaunchKernelGGL(k_fill<true>, dim3(ncu), dim3(1024), lds, 0, a0, a1, 0, tab, pp, Rs, out); break;
					default: hipExtLaunchKernelGGL(k_read_grid<true>, dim3((unsigned)(sz / 16 / 256)), dim3(256), 0, 0, a0, a1, 0, pp, (uint64_t)(sz / 16), out); break;
					}
					CHECK(hipEventSynchronize(a1));
					float ms;
					CHECK(hipEventElapsedTime(&ms, a0, a1));
					if (r >= 0)
						tot += ms;
				}
				printf("%s  {\"probe\": \"%s\", \"MiB\": %d, \"us\": %.2f, \"GBps\": %.1f}", sep(), names[v], mib,
				       tot / reps * 1e3, sz ? sz / (tot / reps * 1e-3) / 1e9 : 0.0);
			}
	}
	if (!strcmp(which, "icache")) {
		hipEvent_t a0, a1;
		CHECK(hipEventCreate(&a0));
		CHECK(hipEventCreate(&a1));
		for (int threads = 256; threads <= 1024; threads *= 4)
			for (int v = 0; v < 6; ++v) {
				float tot = 0;
				for (int r = -2; r < reps; ++r) {
					switch (v) {
					case 0: hipExtLaunchKernelGGL((k_code<1024, false>), dim3(ncu), dim3(threads), 0, 0, a0, a1, 0, out); break;
					case 1: hipExtLaunchKernelGGL((k_code<1024, true>), dim3(ncu), dim3(threads), 0, 0, a0, a1, 0, out); break;
					case 2: hipExtLaunchKernelGGL((k_code<4096, false>), dim3(ncu), dim3(threads), 0, 0, a0, a1, 0, out); break;
					case 3: hipExtLaunchKernelGGL((k_code<4096, true>), dim3(ncu), dim3(threads), 0, 0, a0, a1, 0, out); break;
					case 4: hipExtLaunchKernelGGL((k_code<8192, false>), dim3(ncu), dim3(threads), 0, 0, a0, a1, 0, out); break;
					default: hipExtLaunchKernelGGL((k_code<8192, true>), dim3(ncu), dim3(threads), 0, 0, a0, a1, 0, out); break;
					}
					CHECK(hipEventSynchronize(a1));
					float ms;
					CHECK(hipEventElapsedTime(&ms, a0, a1));
					if (r >= 0)
						tot += ms;
				}
				static const int ni[] = {1024, 1024, 4096, 4096, 8192, 8192};
				printf("%s  {\"probe\": \"%d VALU instrs, %s\", \"threads\": %d, \"code_KiB\": %d, \"us\": %.2f}", sep(), ni[v],
				       v & 1 ? "loop of 256" : "straight-line", threads, v & 1 ? 2 : ni[v] * 8 / 1024, tot / reps * 1e3);
			}
	}
	if (!strcmp(which, "grid")) { // the best shapes measured: one float4 per thread, non-persistent grid, nt
		for (int v = 0; v < 2; ++v) {
			float tot = 0;
			const uint64_t n16 = bytes / 16;
			for (int r = -2; r < reps; ++r) {
				CHECK(hipEventRecord(e0, 0));
				const uint8_t *src = buf[(r + 4) % 2];
				if (v == 0)
					hipLaunchKernelGGL(k_read_grid<true>, dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, n16, out);
				else
					hipLaunchKernelGGL(k_copy_grid<true>, dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, buf[2], n16);
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0)
					tot += ms;
			}
			printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}", sep(),
			       v ? "copy grid float4 nt (read+write)" : "read grid float4 nt", tot / reps * 1e3,
			       (v ? 2.0 : 1.0) * bytes / (tot / reps * 1e-3) / 1e9);
		}
	}
	if (all || !strcmp(which, "copyocc")) {
		const char *names[] = {"copy static D8 16 waves/CU", "copy static D4 16 waves/CU", "copy static D16 16 waves/CU",
				       "copy static D8 32 waves/CU", "copy static D4 32 waves/CU", "copy grid 1 float4/thread",
				       "copy grid 4 float4/thread", "copy grid 16 float4/thread"};
		for (int v = 0; v < 8; ++v) {
			float tot = 0;
			for (int r = -2; r < reps; ++r) {
				CHECK(hipEventRecord(e0, 0));
				const uint8_t *src = buf[(r + 4) % 2];
				const uint64_t n16 = bytes / 16;
				switch (v) {
				case 0: hipLaunchKernelGGL((k_copy_occ<8, 1>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				case 1: hipLaunchKernelGGL((k_copy_occ<4, 1>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				case 2: hipLaunchKernelGGL((k_copy_occ<16, 1>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				case 3: hipLaunchKernelGGL((k_copy_occ<8, 2>), dim3(2 * ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				case 4: hipLaunchKernelGGL((k_copy_occ<4, 2>), dim3(2 * ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				case 5: hipLaunchKernelGGL((k_copy_gridk<1>), dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, buf[2], n16); break;
				case 6: hipLaunchKernelGGL((k_copy_gridk<4>), dim3((unsigned)(n16 / 1024)), dim3(256), 0, 0, src, buf[2], n16); break;
				default: hipLaunchKernelGGL((k_copy_gridk<16>), dim3((unsigned)(n16 / 4096)), dim3(256), 0, 0, src, buf[2], n16); break;
				}
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0)
					tot += ms;
			}
			printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"GBps_read_plus_write\": %.1f}", sep(), names[v],
			       tot / reps * 1e3, 2.0 * bytes / (tot / reps * 1e-3) / 1e9);
		}
	}
	if (!strcmp(which, "small")) { // 4 KiB buffers (run with a 256 MiB size: the C2 batch)
		const char *names[] = {"copy 4 KiB buffers, static shares", "copy 4 KiB buffers, workgroup-interleaved",
				       "read 4 KiB buffers, static shares", "read 4 KiB buffers, workgroup-interleaved"};
		for (int v = 0; v < 4; ++v) {
			float tot = 0;
			for (int r = -2; r < reps; ++r) {
				CHECK(hipEventRecord(e0, 0));
				const uint8_t *src = buf[(r + 4) % 2];
				switch (v) {
				case 0: hipLaunchKernelGGL((k_small<true, false>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 1: hipLaunchKernelGGL((k_small<true, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 2: hipLaunchKernelGGL((k_small<false, false>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				default: hipLaunchKernelGGL((k_small<false, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				}
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0)
					tot += ms;
			}
			const bool cp = v < 2;
			printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"%s\": %.1f}", sep(), names[v], tot / reps * 1e3,
			       cp ? "GBps_read_plus_write" : "GBps", (cp ? 2.0 : 1.0) * bytes / (tot / reps * 1e-3) / 1e9);
		}
	}
	if (!strcmp(which, "copyshape")) {
		const char *names[] = {"copy static D8", "copy grid 1 float4/thread (256-thread WGs)",
				       "copy grid 1 float4/thread, 1024-thread WGs", "copy grid 1 float4/thread, 256 threads + 40 KiB LDS (4 WGs/CU)",
				       "copy grid 1 float4/thread, 1024 threads + 144 KiB LDS (1 WG/CU)",
				       "copy workgroup-interleaved rows (128 groups, 16 KiB per row step)",
				       "read workgroup-interleaved rows", "read static (pad)", "read grid float4 nt",
				       "read workgroup-interleaved rows, barrier per 8-row block",
				       "copy workgroup-interleaved rows, barrier per 8-row block",
				       "read tiles 8 KiB, WG lockstep"};
		const int nv = (int)(sizeof(names) / sizeof(names[0]));
		for (int v = 0; v < nv; ++v) {
			float tot = 0;
			for (int r = -2; r < reps; ++r) {
				CHECK(hipEventRecord(e0, 0));
				const uint8_t *src = buf[(r + 4) % 2];
				const uint64_t n16 = bytes / 16;
				switch (v) {
				case 0: hipLaunchKernelGGL((k_copy_occ<8, 1>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				case 1: hipLaunchKernelGGL((k_copy_gridk<1>), dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, buf[2], n16); break;
				case 2: hipLaunchKernelGGL((k_copy_grid_pad<1024, 64>), dim3((unsigned)(n16 / 1024)), dim3(1024), 0, 0, src, buf[2], n16); break;
				case 3: hipLaunchKernelGGL((k_copy_grid_pad<256, 10 * 1024>), dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, buf[2], n16); break;
				case 4: hipLaunchKernelGGL((k_copy_grid_pad<1024, 36 * 1024>), dim3((unsigned)(n16 / 1024)), dim3(1024), 0, 0, src, buf[2], n16); break;
				case 5: hipLaunchKernelGGL((k_wg_interleave<true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 6: hipLaunchKernelGGL((k_wg_interleave<false>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 7: hipLaunchKernelGGL((k_rotated<false, false>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 8: hipLaunchKernelGGL(k_read_grid<true>, dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, n16, out); break;
				case 9: hipLaunchKernelGGL((k_wg_interleave<false, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 10: hipLaunchKernelGGL((k_wg_interleave<true, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				default: hipLaunchKernelGGL((k_tiles_sync<false, 64, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				}
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0)
					tot += ms;
			}
			const bool cp = v <= 5 || v == 10;
			printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"%s\": %.1f}", sep(), names[v], tot / reps * 1e3,
			       cp ? "GBps_read_plus_write" : "GBps", (cp ? 2.0 : 1.0) * bytes / (tot / reps * 1e-3) / 1e9);
		}
	}
	if (!strcmp(which, "copysplit")) {
		const char *names[] = {"copy static D8", "copy split roles (8 loading + 8 storing waves, LDS hand-off)",
				       "copy grid 1 float4/thread"};
		for (int v = 0; v < 3; ++v) {
			float tot = 0;
			for (int r = -2; r < reps; ++r) {
				CHECK(hipEventRecord(e0, 0));
				const uint8_t *src = buf[(r + 4) % 2];
				const uint64_t n16 = bytes / 16;
				switch (v) {
				case 0: hipLaunchKernelGGL((k_copy_occ<8, 1>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				case 1: hipLaunchKernelGGL(k_copy_split, dim3(ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				default: hipLaunchKernelGGL((k_copy_gridk<1>), dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, buf[2], n16); break;
				}
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0)
					tot += ms;
			}
			printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"GBps_read_plus_write\": %.1f}", sep(), names[v],
			       tot / reps * 1e3, 2.0 * bytes / (tot / reps * 1e-3) / 1e9);
		}
		// the split copy's destination must equal its source
		std::vector<uint8_t> h0(1 << 20), h1(1 << 20);
		hipLaunchKernelGGL(k_copy_split, dim3(ncu), dim3(1024), 0, 0, buf[0], buf[2], R);
		CHECK(hipDeviceSynchronize());
		for (size_t off = 0; off < bytes; off += bytes / 7) {
			const size_t o = off & ~(size_t)((1 << 20) - 1);
			CHECK(hipMemcpy(h0.data(), buf[0] + o, 1 << 20, hipMemcpyDeviceToHost));
			CHECK(hipMemcpy(h1.data(), buf[2] + o, 1 << 20, hipMemcpyDeviceToHost));
			if (memcmp(h0.data(), h1.data(), 1 << 20)) {
				printf("\n  {\"error\": \"split copy differs at %zu\"}", o);
				break;
			}
		}
	}
	if (!strcmp(which, "tilecrc")) { // can the grid copy carry a per-tile CRC?
		const char *names[] = {"copy grid 1 float4/thread", "tile copy + CRC stand-in, 1 KiB table, dependent lookups",
				       "tile copy + CRC stand-in, 4 KiB tables, dependent lookups",
				       "tile copy + CRC stand-in, 16 KiB tables, slice-by-16",
				       "tile copy + CRC stand-in, 4 KiB tables, + fold launch"};
		const uint64_t n16 = bytes / 16, nparts = n16 / 64 + 1, nout = n16 / 64 / 64;
		uint32_t *tab, *part, *fold;
		CHECK(hipMalloc(&tab, 4096 * 4));
		CHECK(hipMemset(tab, 0x5a, 4096 * 4));
		CHECK(hipMalloc(&part, nparts * 4));
		CHECK(hipMalloc(&fold, (nout + 1) * 4));
		const int nv = (int)(sizeof(names) / sizeof(names[0]));
		for (int v = 0; v < nv; ++v) {
			float tot = 0;
			for (int r = -2; r < reps; ++r) {
				CHECK(hipEventRecord(e0, 0));
				const uint8_t *src = buf[(r + 4) % 2];
				const dim3 g((unsigned)(n16 / 256));
				switch (v) {
				case 0: hipLaunchKernelGGL((k_copy_gridk<1>), g, dim3(256), 0, 0, src, buf[2], n16); break;
				case 1: hipLaunchKernelGGL((k_copy_tilecrc<256>), g, dim3(256), 0, 0, src, buf[2], n16, tab, part); break;
				case 3: hipLaunchKernelGGL((k_copy_tilecrc<4096>), g, dim3(256), 0, 0, src, buf[2], n16, tab, part); break;
				default: hipLaunchKernelGGL((k_copy_tilecrc<1024>), g, dim3(256), 0, 0, src, buf[2], n16, tab, part); break;
				}
				if (v == 4)
					hipLaunchKernelGGL(k_tile_fold, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0, 0, part, nout, fold);
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0)
					tot += ms;
			}
			printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"GBps_read_plus_write\": %.1f}", sep(), names[v], tot / reps * 1e3,
			       2.0 * bytes / (tot / reps * 1e-3) / 1e9);
		}
		CHECK(hipFree(tab));
		CHECK(hipFree(part));
		CHECK(hipFree(fold));
	}
	if (all || !strcmp(which, "window")) {
		const char *names[] = {"read tiles 8 KiB (drifting)", "read tiles 8 KiB, WG lockstep",
				       "read tiles 32 KiB, WG lockstep", "read grid float4 nt",
				       "copy tiles 8 KiB (drifting)", "copy tiles 8 KiB, WG lockstep",
				       "copy tiles 32 KiB, WG lockstep", "copy static, stores lag a block, 2x8 rows",
				       "copy static, stores lag a block, 2x4 rows", "copy static D8",
				       "copy grid 1 float4/thread", "read static (pad)", "read static, hashed slice starts",
				       "copy static (pad)", "copy static, hashed slice starts",
				       "read tiles 8 KiB, XCD round robin", "copy tiles 8 KiB, XCD round robin",
				       "copy tiles 32 KiB, XCD round robin"};
		const int nv = (int)(sizeof(names) / sizeof(names[0]));
		for (int v = 0; v < nv; ++v) {
			float tot = 0;
			for (int r = -2; r < reps; ++r) {
				CHECK(hipEventRecord(e0, 0));
				const uint8_t *src = buf[(r + 4) % 2];
				const uint64_t n16 = bytes / 16;
				switch (v) {
				case 0: hipLaunchKernelGGL((k_tiles_sync<false, 64, false>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 1: hipLaunchKernelGGL((k_tiles_sync<false, 64, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 2: hipLaunchKernelGGL((k_tiles_sync<false, 256, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 3: hipLaunchKernelGGL(k_read_grid<true>, dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, n16, out); break;
				case 4: hipLaunchKernelGGL((k_tiles_sync<true, 64, false>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 5: hipLaunchKernelGGL((k_tiles_sync<true, 64, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 6: hipLaunchKernelGGL((k_tiles_sync<true, 256, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 7: hipLaunchKernelGGL((k_copy_lag<8>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				case 8: hipLaunchKernelGGL((k_copy_lag<4>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				case 9: hipLaunchKernelGGL((k_copy_occ<8, 1>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R); break;
				case 10: hipLaunchKernelGGL((k_copy_gridk<1>), dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, buf[2], n16); break;
				case 11: hipLaunchKernelGGL((k_rotated<false, false>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 12: hipLaunchKernelGGL((k_rotated<false, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 13: hipLaunchKernelGGL((k_rotated<true, false>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 14: hipLaunchKernelGGL((k_rotated<true, true>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 15: hipLaunchKernelGGL((k_tiles_xcd<false, 64>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				case 16: hipLaunchKernelGGL((k_tiles_xcd<true, 64>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				default: hipLaunchKernelGGL((k_tiles_xcd<true, 256>), dim3(ncu), dim3(1024), 0, 0, src, buf[2], R, out); break;
				}
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 0)
					tot += ms;
			}
			const bool cp = (v >= 4 && v <= 10) || v == 13 || v == 14 || v >= 16;
			printf("%s  {\"probe\": \"%s\", \"us\": %.2f, \"%s\": %.1f}", sep(), names[v], tot / reps * 1e3,
			       cp ? "GBps_read_plus_write" : "GBps", (cp ? 2.0 : 1.0) * bytes / (tot / reps * 1e-3) / 1e9);
		}
	}
	printf("\n]}\n");
	return 0;
}
