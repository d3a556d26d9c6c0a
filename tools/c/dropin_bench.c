/*
 * dropin_bench.c -- per-call latency of the drop-in crc32c() from C, the
 * way messenger.c calls it (BENCH TOOL, not product code; links the test
 * oracle as the reference-loop column and as the checker).
 *
 * For each size: mean microseconds per synchronous call over pageable host
 * memory, for
 *   "host"  the default routing (crc32c_set_cpu_max default: host routine),
 *   "gpu"   every call through the gfx950 kernels (crc32c_set_cpu_max(0)),
 *   "ref"   the reference byte loop (include/crc32c.h:88-96 restated by
 *           oracle/crc32c_oracle.c, same compiler flags as pech).
 * Every route's result is compared with the reference; exit 1 on mismatch.
 * Output: one JSON object on stdout.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "pech_crc32c.h"

uint32_t oracle_crc32c(uint32_t crc, const void *data, unsigned int length);

static double now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

typedef uint32_t (*crc_fn)(uint32_t, const void *, unsigned int);

/* mean us per call over >= min_s seconds (and >= 3 calls) */
static double per_call(crc_fn f, const unsigned char *p, unsigned int n, double min_s, uint32_t *res)
{
	double t0, t;
	unsigned long k = 0, reps = 1;
	volatile uint32_t sink = 0;

	sink ^= f(0, p, n); /* warm */
	t0 = now();
	do {
		unsigned long i;
		for (i = 0; i < reps; i++)
			sink ^= f(0, p, n);
		k += reps;
		reps *= 2;
		t = now() - t0;
	} while (t < min_s || k < 3);
	*res = f(0, p, n);
	(void)sink;
	return t / k * 1e6;
}

int main(int argc, char **argv)
{
	static const unsigned int sizes[] = {49, 200, 4096, 65536, 1u << 20, 4u << 20, 16u << 20, 64u << 20};
	const double min_s = argc > 1 ? atof(argv[1]) : 0.2;
	const unsigned int nsz = sizeof(sizes) / sizeof(sizes[0]);
	unsigned char *buf = malloc((64u << 20) + 64);
	unsigned int i, bad = 0, prev;
	struct crc32c_stats st;

	if (!buf)
		return 2;
	for (i = 0; i < (64u << 20) + 64; i++)
		buf[i] = (unsigned char)((i * 2654435761u) >> 11);
	printf("{\"unit\": \"us_per_call\", \"sizes\": {");
	for (i = 0; i < nsz; i++) {
		const unsigned int n = sizes[i];
		uint32_t r_host, r_gpu, r_ref;
		double host, gpu, ref;

		prev = crc32c_set_cpu_max(4u << 20);
		host = per_call(crc32c, buf + 1, n, min_s, &r_host);
		crc32c_set_cpu_max(0);
		gpu = per_call(crc32c, buf + 1, n, min_s, &r_gpu);
		crc32c_set_cpu_max(prev);
		ref = per_call(oracle_crc32c, buf + 1, n, n > (1u << 20) ? min_s / 4 : min_s, &r_ref);
		if (r_host != r_ref || r_gpu != r_ref)
			bad++;
		printf("%s\"%u\": {\"host\": %.4f, \"gpu\": %.3f, \"ref\": %.4f}", i ? ", " : "", n, host, gpu, ref);
	}
	crc32c_get_stats(&st);
	printf("}, \"mismatches\": %u, \"gpu_fallbacks\": %llu}\n", bad, (unsigned long long)st.gpu_fallbacks);
	return bad || st.gpu_fallbacks ? 1 : 0;
}
