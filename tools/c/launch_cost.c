/*
 * Host CPU cost of the HIP calls one async-layer slot makes (GPU box):
 * wall microseconds inside each call (call_us; the calls do not block), issued
 * back to back on one stream with a synchronize every 64 calls (a flush's
 * worth; the _incl_sync figures add the spin of that wait), so the
 * messenger's per-payload cost can be split into its launch parts.
 *   build/launch_cost [iters]
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pech_crc32c.h"

static double thread_cpu_s(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static double wall_s(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void noop(void *arg)
{
	(void)arg;
}

#define CHECK(x)                                                                    \
	do {                                                                        \
		if ((x) != 0) {                                                     \
			fprintf(stderr, "%s failed at %s:%d\n", #x, __FILE__, __LINE__); \
			exit(1);                                                    \
		}                                                                   \
	} while (0)

enum { N_DESC = 64, BUF = 4096 };

int main(int argc, char **argv)
{
	const int iters = argc > 1 ? atoi(argv[1]) : 20000;
	hipStream_t st;
	struct crc32c_desc *h_desc, *d_desc, *m_desc;
	uint32_t *d_out, *h_out, *m_out;
	uint8_t *d_buf, *h_big, *h_big2, *d_big;
	const char *names[] = {"small_async(64 descs)", "dev_batch_async(64 descs, plan+main)",
			       "memcpy D2H 256 B", "memcpy H2D 1 KiB", "hipLaunchHostFunc(noop)",
			       "small_async on mapped host descs + out", "hipEventRecord", "hipGetDevice",
			       "hipSetDevice(same)", "hipStreamQuery(idle)", "memcpy H2D 1 MiB (pinned, mapped)",
			       "memcpy H2D 4 MiB (pinned, mapped)", "memcpy H2D 1 MiB (pinned, default flags)"};
	int dev;
	hipEvent_t ev;
	int k, i;

	CHECK(hipSetDevice(0));
	CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
	CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
	CHECK(hipMalloc((void **)&d_buf, N_DESC * BUF));
	CHECK(hipMalloc((void **)&d_desc, N_DESC * sizeof(*d_desc)));
	CHECK(hipMalloc((void **)&d_out, N_DESC * 4));
	CHECK(hipHostMalloc((void **)&h_desc, N_DESC * sizeof(*h_desc), 0));
	CHECK(hipHostMalloc((void **)&h_out, N_DESC * 4, 0));
	CHECK(hipHostGetDevicePointer((void **)&m_desc, h_desc, 0));
	CHECK(hipHostGetDevicePointer((void **)&m_out, h_out, 0));
	CHECK(hipMemset(d_buf, 0x5A, N_DESC * BUF));
	/* crc32c_pages memory is hipHostMalloc(Mapped | Portable) */
	CHECK(hipHostMalloc((void **)&h_big, 4u << 20, hipHostMallocMapped | hipHostMallocPortable));
	CHECK(hipHostMalloc((void **)&h_big2, 1u << 20, 0));
	CHECK(hipMalloc((void **)&d_big, 4u << 20));
	memset(h_big, 1, 4u << 20);
	memset(h_big2, 2, 1u << 20);
	for (i = 0; i < N_DESC; i++) {
		h_desc[i].addr = (uint64_t)(uintptr_t)(d_buf + (size_t)i * BUF);
		h_desc[i].len = BUF;
		h_desc[i].seed = 0;
	}
	CHECK(hipMemcpy(d_desc, h_desc, N_DESC * sizeof(*d_desc), hipMemcpyHostToDevice));
	CHECK(crc32c_dev_reserve(N_DESC));
	for (k = 0; k < 13; k++) {
		double c0 = 0, w0 = 0, in_call = 0;
		int pass;

		for (pass = 0; pass < 2; pass++) { /* pass 0: warm-up */
			const int n = pass ? (k >= 10 ? iters / 20 : iters) : 256;

			if (pass) {
				c0 = thread_cpu_s();
				w0 = wall_s();
				in_call = 0;
			}
			for (i = 0; i < n; i++) {
				const double a = wall_s();

				switch (k) {
				case 0: CHECK(crc32c_dev_batch_small_async(d_desc, d_out, N_DESC, st)); break;
				case 1: CHECK(crc32c_dev_batch_async(d_desc, d_out, N_DESC, st)); break;
				case 2: CHECK(hipMemcpyAsync(h_out, d_out, 256, hipMemcpyDeviceToHost, st)); break;
				case 3: CHECK(hipMemcpyAsync(d_desc, h_desc, 1024, hipMemcpyHostToDevice, st)); break;
				case 4: CHECK(hipLaunchHostFunc(st, noop, NULL)); break;
				case 5: CHECK(crc32c_dev_batch_small_async(m_desc, m_out, N_DESC, st)); break;
				case 6: CHECK(hipEventRecord(ev, st)); break;
				case 7: CHECK(hipGetDevice(&dev)); break;
				case 8: CHECK(hipSetDevice(0)); break;
				case 9: CHECK(hipStreamQuery(st)); break;
				case 10: CHECK(hipMemcpyAsync(d_big, h_big, 1u << 20, hipMemcpyHostToDevice, st)); break;
				case 11: CHECK(hipMemcpyAsync(d_big, h_big, 4u << 20, hipMemcpyHostToDevice, st)); break;
				case 12: CHECK(hipMemcpyAsync(d_big, h_big2, 1u << 20, hipMemcpyHostToDevice, st)); break;
				}
				in_call += wall_s() - a;
				if (i % 64 == 63)
					CHECK(hipStreamSynchronize(st));
			}
			CHECK(hipStreamSynchronize(st));
		}
		printf("{\"call\": \"%s\", \"call_us\": %.3f, \"thread_cpu_us_incl_sync\": %.3f, "
		       "\"wall_us_incl_sync\": %.3f}\n", names[k], in_call / (k >= 10 ? iters / 20 : iters) * 1e6,
		       (thread_cpu_s() - c0) / (k >= 10 ? iters / 20 : iters) * 1e6,
		       (wall_s() - w0) / (k >= 10 ? iters / 20 : iters) * 1e6);
	}
	for (i = 0; i < N_DESC; i++)
		if (h_out[i] != h_out[0]) {
			fprintf(stderr, "mapped-output results differ\n");
			return 1;
		}
	return 0;
}
