// atomic_probe.hip -- device-scope atomic latency/throughput on MI355X (not
// product code).  Context for the main kernel's work-distribution design:
// one lane per wave performs K dependent atomicAdd's (each waits for the
// previous return) on
//   one   : a single counter shared by every wave of the chip
//   xcd   : one counter per XCD (8 counters, 256 B apart), by HW_REG_XCC_ID
//   wave  : a private counter per wave (no contention)
// and, for scale, the same with K dependent global loads (latency only).
// Build: hipcc -O3 --offload-arch=gfx950 tools/atomic_probe.hip -o build/atomic_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                   \
	do {                                                                       \
		hipError_t e = (x);                                                \
		if (e != hipSuccess) {                                             \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));     \
			exit(1);                                                   \
		}                                                                  \
	} while (0)

template <int MODE>
__global__ __launch_bounds__(1024) void k_atomic(uint32_t *ctr, int K, uint32_t *sink)
{
	const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	if ((threadIdx.x & 63u) != 0)
		return;
	uint32_t xcc;
	asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
	uint32_t *c = MODE == 0 ? ctr : MODE == 1 ? ctr + 64u * (xcc & 7u) : ctr + 64u * (8u + wave);
	uint32_t acc = 0;
	for (int k = 0; k < K; ++k)
		acc += atomicAdd(c + (acc & 0u), 1u);
	if (acc == 0xFFFFFFFFu)
		sink[wave] = acc;
}

// scalar (SMEM) atomics: counted on lgkmcnt, independent of the vector queue
template <int MODE>
__global__ __launch_bounds__(1024) void k_satomic(uint32_t *ctr, int K, uint32_t *sink)
{
	const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	uint32_t xcc;
	asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
	uint32_t *c = MODE == 0 ? ctr : ctr + 64u * (xcc & 7u);
	uint32_t acc = 0;
	for (int k = 0; k < K; ++k) {
		uint32_t r = 1u;
		asm volatile("s_atomic_add %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "+s"(r) : "s"(c) : "memory");
		acc += r;
	}
	if ((threadIdx.x & 63u) == 0 && acc == 0xFFFFFFFFu)
		sink[wave] = acc;
}

__global__ __launch_bounds__(1024) void k_chase(const uint32_t *next, int K, uint32_t *sink)
{
	const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	if ((threadIdx.x & 63u) != 0)
		return;
	uint32_t i = wave * 64u;
	for (int k = 0; k < K; ++k)
		i = __builtin_nontemporal_load(next + i);
	if (i == 0xFFFFFFFFu)
		sink[wave] = i;
}

int main()
{
	hipDeviceProp_t prop;
	CHECK(hipGetDeviceProperties(&prop, 0));
	const int ncu = prop.multiProcessorCount;
	const int waves = ncu * 16;
	uint32_t *ctr, *sink, *next;
	CHECK(hipMalloc(&ctr, (size_t)(8 + waves) * 256));
	CHECK(hipMalloc(&sink, (size_t)waves * 4));
	const size_t nn = (size_t)waves * 64;
	CHECK(hipMalloc(&next, nn * 4));
	uint32_t *h = (uint32_t *)malloc(nn * 4);
	for (size_t i = 0; i < nn; ++i) // each wave walks its own 256 B-strided cycle
		h[i] = (uint32_t)((i / 64) * 64 + ((i % 64) + 1) % 64);
	CHECK(hipMemcpy(next, h, nn * 4, hipMemcpyHostToDevice));
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	const int K = 64;
	printf("{\"cus\": %d, \"waves\": %d, \"K\": %d, \"results\": [\n", ncu, waves, K);
	for (int mode = 0; mode < 6; ++mode) {
		float best = 1e30f;
		for (int rep = 0; rep < 5; ++rep) {
			CHECK(hipMemset(ctr, 0, (size_t)(8 + waves) * 256));
			CHECK(hipEventRecord(a));
			if (mode == 0)
				hipLaunchKernelGGL(k_atomic<0>, dim3(ncu), dim3(1024), 0, 0, ctr, K, sink);
			else if (mode == 1)
				hipLaunchKernelGGL(k_atomic<1>, dim3(ncu), dim3(1024), 0, 0, ctr, K, sink);
			else if (mode == 2)
				hipLaunchKernelGGL(k_atomic<2>, dim3(ncu), dim3(1024), 0, 0, ctr, K, sink);
			else if (mode == 3)
				hipLaunchKernelGGL(k_chase, dim3(ncu), dim3(1024), 0, 0, next, K, sink);
			else if (mode == 4)
				hipLaunchKernelGGL(k_satomic<0>, dim3(ncu), dim3(1024), 0, 0, ctr, K, sink);
			else
				hipLaunchKernelGGL(k_satomic<1>, dim3(ncu), dim3(1024), 0, 0, ctr, K, sink);
			CHECK(hipEventRecord(b));
			CHECK(hipEventSynchronize(b));
			float ms;
			CHECK(hipEventElapsedTime(&ms, a, b));
			best = ms < best ? ms : best;
		}
		uint32_t hv[8 * 64];
		CHECK(hipMemcpy(hv, ctr, sizeof(hv), hipMemcpyDeviceToHost));
		uint64_t tot = 0;
		for (int x = 0; x < 8; ++x)
			tot += hv[64 * x];
		const bool counted = mode == 0 || mode == 1 || mode == 4 || mode == 5;
		const char *name[] = {"one counter", "per-XCD counter", "per-wave counter", "dependent load chain",
				      "scalar atomic, one counter", "scalar atomic, per-XCD counter"};
		printf("  {\"probe\": \"%s\", \"us\": %.2f, \"us_per_op_per_wave\": %.3f, \"Mops_per_s\": %.1f%s}%s\n",
		       name[mode], best * 1e3, best * 1e3 / K, (double)waves * K / (best * 1e-3) / 1e6,
		       !counted ? "" : (tot == (uint64_t)waves * K ? ", \"count_ok\": true" : ", \"count_ok\": false"),
		       mode < 5 ? "," : "");
	}
	printf("]}\n");
	return 0;
}
