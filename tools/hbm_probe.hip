// hbm_probe.hip -- read-bandwidth probes on the GPU box (not product code).
// Measures what HBM read rate different access shapes reach on MI355X, as
// context for the CRC kernel's roofline:
//   stream   : grid-stride, every wave reads contiguous 1 KiB per instruction
//   groupG   : the CRC kernel's shape -- G-lane groups, each walking its own
//              contiguous range in (G*16)-byte rows, D rows in flight per lane
// Build: hipcc -O3 --offload-arch=gfx950 tools/hbm_probe.hip -o build/hbm_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;

#define CHECK(x)                                                                   \
	do {                                                                       \
		hipError_t e = (x);                                                \
		if (e != hipSuccess) {                                             \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));     \
			exit(1);                                                   \
		}                                                                  \
	} while (0)

template <int UNROLL>
__global__ __launch_bounds__(1024) void k_stream(const u32x4 *p, size_t n16, uint32_t *out)
{
	const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
	const size_t stride = (size_t)gridDim.x * blockDim.x;
	u32x4 acc = (u32x4)(0u);
	size_t i = tid;
	for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
		u32x4 v[UNROLL];
#pragma unroll
		for (int u = 0; u < UNROLL; ++u)
			v[u] = *(g_u32x4 *)(p + i + u * stride);
#pragma unroll
		for (int u = 0; u < UNROLL; ++u)
			acc ^= v[u];
	}
	for (; i < n16; i += stride)
		acc ^= *(g_u32x4 *)(p + i);
	const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (r == 0x12345678u)
		out[tid] = r;
}

// G lanes per group, each group a contiguous range of `rows` rows of G*16 B
template <bool NT>
__device__ __forceinline__ u32x4 ldp(const uint8_t *a)
{
	if (NT)
		return __builtin_nontemporal_load((g_u32x4 *)a);
	return *(g_u32x4 *)a;
}

// same as k_group but each group starts its walk at a pseudo-random row of
// its range and wraps around (breaks the alignment of all streams modulo the
// range size)
template <int G, int D>
__global__ __launch_bounds__(1024) void k_group_rot(const uint8_t *p, uint32_t rows_per_group, uint32_t *out)
{
	const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / G;
	const uint32_t gl = threadIdx.x % G;
	const uint8_t *base = p + (size_t)gid * rows_per_group * (G * 16) + gl * 16;
	const uint32_t off = (gid * 2654435761u) % rows_per_group;
	u32x4 acc = (u32x4)(0u);
	for (uint32_t r = 0; r < rows_per_group; r += D) {
		u32x4 v[D];
#pragma unroll
		for (int d = 0; d < D; ++d) {
			uint32_t row = r + d + off;
			row = row >= rows_per_group ? row - rows_per_group : row;
			v[d] = __builtin_nontemporal_load((g_u32x4 *)(base + (size_t)row * G * 16));
		}
#pragma unroll
		for (int d = 0; d < D; ++d)
			acc ^= v[d];
	}
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (x == 0x12345678u)
		out[gid] = x;
}

// interleaved: group g of NG reads rows g, g+NG, ... (each wave-instruction
// covers consecutive 128-byte rows)
template <int D>
__global__ __launch_bounds__(1024) void k_interleaved(const uint8_t *p, uint32_t total_rows, uint32_t *out)
{
	const uint32_t ng = gridDim.x * blockDim.x / 8;
	const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / 8;
	const uint32_t gl = threadIdx.x % 8;
	u32x4 acc = (u32x4)(0u);
	for (uint32_t r = gid; r < total_rows; r += D * ng) {
		u32x4 v[D];
#pragma unroll
		for (int d = 0; d < D; ++d) {
			const uint32_t row = min(r + d * ng, total_rows - 1);
			v[d] = __builtin_nontemporal_load((g_u32x4 *)(p + (size_t)row * 128 + gl * 16));
		}
#pragma unroll
		for (int d = 0; d < D; ++d)
			acc ^= v[d];
	}
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (x == 0x12345678u)
		out[gid] = x;
}

template <int G, int D, bool NT = false>
__global__ __launch_bounds__(1024) void k_group(const uint8_t *p, uint32_t rows_per_group, uint32_t *out)
{
	const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / G;
	const uint32_t gl = threadIdx.x % G;
	const uint8_t *base = p + (size_t)gid * rows_per_group * (G * 16) + gl * 16;
	u32x4 acc = (u32x4)(0u);
	u32x4 ring[D];
#pragma unroll
	for (int d = 0; d < D; ++d)
		ring[d] = ldp<NT>(base + (size_t)d * G * 16);
	uint32_t r = D;
	for (; r + D <= rows_per_group; r += D) {
#pragma unroll
		for (int d = 0; d < D; ++d) {
			acc ^= ring[d];
			ring[d] = ldp<NT>(base + (size_t)(r + d) * G * 16);
		}
	}
#pragma unroll
	for (int d = 0; d < D; ++d)
		acc ^= ring[d];
	for (; r < rows_per_group; ++r)
		acc ^= ldp<NT>(base + (size_t)r * G * 16);
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (x == 0x12345678u)
		out[gid] = x;
}

// k_group<8, D, nt> restricted to the workgroups that land on the XCCs in
// `xmask` (HW_REG_XCC_ID; the others exit at once): per-XCD read bandwidth
// with the rest of the chip idle
template <int D>
__global__ __launch_bounds__(1024) void k_group_xcc(const uint8_t *p, uint32_t rows_per_group, uint32_t *out,
						    uint32_t xmask)
{
	uint32_t xcc;
	asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
	if (!((xmask >> (xcc & 7u)) & 1u))
		return;
	const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / 8;
	const uint32_t gl = threadIdx.x % 8;
	const uint8_t *base = p + (size_t)gid * rows_per_group * 128 + gl * 16;
	u32x4 acc = (u32x4)(0u);
	u32x4 ring[D];
#pragma unroll
	for (int d = 0; d < D; ++d)
		ring[d] = ldp<true>(base + (size_t)d * 128);
	uint32_t r = D;
	for (; r + D <= rows_per_group; r += D) {
#pragma unroll
		for (int d = 0; d < D; ++d) {
			acc ^= ring[d];
			ring[d] = ldp<true>(base + (size_t)(r + d) * 128);
		}
	}
#pragma unroll
	for (int d = 0; d < D; ++d)
		acc ^= ring[d];
	for (; r < rows_per_group; ++r)
		acc ^= ldp<true>(base + (size_t)r * 128);
	const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
	if (x == 0x12345678u)
		out[gid] = x;
}

static float time_it(void (*launch)(void *), void *arg, int reps)
{
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	launch(arg);
	CHECK(hipDeviceSynchronize());
	CHECK(hipEventRecord(a));
	for (int i = 0; i < reps; ++i)
		launch(arg);
	CHECK(hipEventRecord(b));
	CHECK(hipEventSynchronize(b));
	float ms;
	CHECK(hipEventElapsedTime(&ms, a, b));
	return ms / reps;
}

struct Args {
	uint8_t *buf[2];
	size_t bytes;
	uint32_t *out;
	int ncu;
	int it;
};

template <int U> static void launch_stream(void *v)
{
	Args *a = (Args *)v;
	const uint8_t *p = a->buf[a->it++ & 1];
	hipLaunchKernelGGL(k_stream<U>, dim3(a->ncu * 4), dim3(1024), 0, 0, (const u32x4 *)p, a->bytes / 16, a->out);
}

template <int G, int D, bool NT = false> static void launch_group(void *v)
{
	Args *a = (Args *)v;
	const uint8_t *p = a->buf[a->it++ & 1];
	const uint32_t groups = a->ncu * 1024 / G;
	const uint32_t rpg = (uint32_t)(a->bytes / (G * 16) / groups);
	hipLaunchKernelGGL((k_group<G, D, NT>), dim3(a->ncu), dim3(1024), 0, 0, p, rpg, a->out);
}

template <int G, int D> static void launch_group_rot(void *v)
{
	Args *a = (Args *)v;
	const uint8_t *p = a->buf[a->it++ & 1];
	const uint32_t groups = a->ncu * 1024 / G;
	const uint32_t rpg = (uint32_t)(a->bytes / (G * 16) / groups);
	hipLaunchKernelGGL((k_group_rot<G, D>), dim3(a->ncu), dim3(1024), 0, 0, p, rpg, a->out);
}

template <int D> static void launch_interleaved(void *v)
{
	Args *a = (Args *)v;
	const uint8_t *p = a->buf[a->it++ & 1];
	hipLaunchKernelGGL((k_interleaved<D>), dim3(a->ncu), dim3(1024), 0, 0, p, (uint32_t)(a->bytes / 128), a->out);
}

int main(int argc, char **argv)
{
	Args a;
	a.bytes = (size_t)1 << 30;
	hipDeviceProp_t prop;
	CHECK(hipGetDeviceProperties(&prop, 0));
	a.ncu = prop.multiProcessorCount;
	a.it = 0;
	for (int i = 0; i < 2; ++i) {
		CHECK(hipMalloc(&a.buf[i], a.bytes));
		CHECK(hipMemset(a.buf[i], i + 1, a.bytes));
	}
	CHECK(hipMalloc(&a.out, (size_t)a.ncu * 4096 * 4));
	const int reps = 20;
	struct {
		const char *name;
		void (*fn)(void *);
	} probes[] = {
		{"stream u4 (grid 4/CU)", launch_stream<4>},
		{"stream u8 (grid 4/CU)", launch_stream<8>},
		{"group8  D4", launch_group<8, 4>},
		{"group8  D8", launch_group<8, 8>},
		{"group16 D4", launch_group<16, 4>},
		{"group32 D4", launch_group<32, 4>},
		{"group64 D4", launch_group<64, 4>},
		{"group64 D8", launch_group<64, 8>},
		{"group8  D8 nt", launch_group<8, 8, true>},
		{"group8  D4 nt", launch_group<8, 4, true>},
		{"group64 D8 nt", launch_group<64, 8, true>},
		{"group8  D12 nt", launch_group<8, 12, true>},
		{"group8  D8 nt rotated", launch_group_rot<8, 8>},
		{"interleaved8 D8 nt", launch_interleaved<8>},
		{"group8  D8 nt (again)", launch_group<8, 8, true>},
	};
	printf("{\"device\": \"%s\", \"cus\": %d, \"bytes\": %zu, \"results\": [\n", prop.name, a.ncu, a.bytes);
	for (size_t i = 0; i < sizeof(probes) / sizeof(probes[0]); ++i) {
		const float ms = time_it(probes[i].fn, &a, reps);
		printf("  {\"probe\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}%s\n", probes[i].name, ms * 1e3,
		       a.bytes / (ms * 1e-3) / 1e9, i + 1 < sizeof(probes) / sizeof(probes[0]) ? "," : "");
	}
	printf("]");
	// per-XCD rates: only the workgroups on the XCCs of each mask read
	// (bytes read = bytes x popcount(mask) / 8: workgroups are placed on
	// XCCs round-robin, 32 per XCC)
	const uint32_t masks[] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x55, 0xAA, 0x0F, 0xF0, 0xFF};
	printf(",\n\"per_xcd\": [\n");
	for (size_t i = 0; i < sizeof(masks) / sizeof(masks[0]); ++i) {
		const uint32_t rpg = (uint32_t)(a.bytes / 128 / ((size_t)a.ncu * 128));
		hipEvent_t e0, e1;
		CHECK(hipEventCreate(&e0));
		CHECK(hipEventCreate(&e1));
		hipLaunchKernelGGL((k_group_xcc<8>), dim3(a.ncu), dim3(1024), 0, 0, a.buf[0], rpg, a.out, masks[i]);
		CHECK(hipDeviceSynchronize());
		CHECK(hipEventRecord(e0));
		for (int r = 0; r < reps; ++r)
			hipLaunchKernelGGL((k_group_xcc<8>), dim3(a.ncu), dim3(1024), 0, 0, a.buf[r & 1], rpg, a.out,
					   masks[i]);
		CHECK(hipEventRecord(e1));
		CHECK(hipEventSynchronize(e1));
		float ms;
		CHECK(hipEventElapsedTime(&ms, e0, e1));
		ms /= reps;
		const double rd = (double)a.bytes * __builtin_popcount(masks[i]) / 8.0;
		printf("  {\"xcc_mask\": \"0x%02x\", \"us\": %.2f, \"GBps\": %.1f}%s\n", masks[i], ms * 1e3,
		       rd / (ms * 1e-3) / 1e9, i + 1 < sizeof(masks) / sizeof(masks[0]) ? "," : "");
	}
	printf("]}\n");
	return 0;
}
