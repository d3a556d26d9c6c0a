/*
 * crc32c_hw.c -- TEST INFRASTRUCTURE ONLY (a CPU context baseline).
 *
 * CRC32C with the x86 SSE4.2 `crc32` instruction, the fastest CPU path a
 * Ceph host could use instead of pech's byte-table loop
 * (/root/reference/include/crc32c.h:88-96).  The instruction computes the same
 * reflected Castagnoli update on the raw register -- no pre- or
 * post-inversion -- so hw_crc32c(s, D) == crc32c(s, D) for every seed and
 * length; tests/test_oracle.py checks that against the golden vectors.
 *
 * bench.py reports it beside the reference in cpu_baseline (`sse42`), on one
 * thread and on the GPU's share of host cores.  It is never the product path:
 * nothing under pech_amd/ or include/ links or calls it.
 *
 * Three independent streams hide the instruction's 3-cycle latency; their
 * registers are joined with the GF(2) shift of SURVEY.md Appendix B:
 * R(s, A||B||C) = x^(8(|B|+|C|)) R(s,A) ^ x^(8|C|) R(0,B) ^ R(0,C).
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define HW_POLY 0x82F63B78u

static uint32_t hw_mulmod(uint32_t a, uint32_t b)
{
	uint32_t p = 0;
	int i;

	for (i = 31; i >= 0; i--) {
		if ((a >> i) & 1u)
			p ^= b;
		b = (b & 1u) ? (b >> 1) ^ HW_POLY : b >> 1;
	}
	return p;
}

static uint32_t hw_x8n(uint64_t n)
{
	uint32_t r = 0x80000000u, sq = 0x00800000u;

	while (n) {
		if (n & 1)
			r = hw_mulmod(r, sq);
		sq = hw_mulmod(sq, sq);
		n >>= 1;
	}
	return r;
}

__attribute__((target("sse4.2"))) static uint32_t hw_serial(uint32_t c, const unsigned char *p, size_t n)
{
	uint64_t c64;

	while (n && ((uintptr_t)p & 7u)) {
		c = __builtin_ia32_crc32qi(c, *p++);
		n--;
	}
	c64 = c;
	while (n >= 8) {
		uint64_t w;
		memcpy(&w, p, 8);
		c64 = __builtin_ia32_crc32di(c64, w);
		p += 8;
		n -= 8;
	}
	c = (uint32_t)c64;
	while (n--)
		c = __builtin_ia32_crc32qi(c, *p++);
	return c;
}

/* per-thread memo of the last stream length's shift constant */
struct hw_memo {
	size_t len;
	uint32_t k1, k2; /* x^(8L), x^(16L) */
};

#define HW_MIN3 1024u /* below this a single stream */

__attribute__((target("sse4.2"))) static uint32_t hw_crc(uint32_t c, const unsigned char *p, size_t n,
							 struct hw_memo *m)
{
	size_t L, i;
	uint64_t a, b, d;

	if (n < HW_MIN3)
		return hw_serial(c, p, n);
	while ((uintptr_t)p & 7u) { /* align the streams' words */
		c = __builtin_ia32_crc32qi(c, *p++);
		n--;
	}
	L = (n / 3u) & ~(size_t)7u;
	a = c;
	b = 0;
	d = 0;
	for (i = 0; i < L; i += 8) {
		uint64_t wa, wb, wd;
		memcpy(&wa, p + i, 8);
		memcpy(&wb, p + L + i, 8);
		memcpy(&wd, p + 2 * L + i, 8);
		a = __builtin_ia32_crc32di(a, wa);
		b = __builtin_ia32_crc32di(b, wb);
		d = __builtin_ia32_crc32di(d, wd);
	}
	if (m->len != L) {
		m->len = L;
		m->k1 = hw_x8n(L);
		m->k2 = hw_mulmod(m->k1, m->k1);
	}
	c = hw_mulmod(m->k2, (uint32_t)a) ^ hw_mulmod(m->k1, (uint32_t)b) ^ (uint32_t)d;
	return hw_serial(c, p + 3 * L, n - 3 * L);
}

uint32_t hw_crc32c(uint32_t crc, const void *data, unsigned int length)
{
	struct hw_memo m = {0, 0, 0};

	return hw_crc(crc, data, length, &m);
}

struct hw_job {
	const unsigned char *base;
	const uint64_t *offs;
	const uint32_t *lens;
	uint32_t *out;
	unsigned int lo, hi, reps;
};

static void *hw_worker(void *arg)
{
	struct hw_job *j = arg;
	struct hw_memo m = {0, 0, 0};
	unsigned int r, i;

	for (r = 0; r < j->reps; r++)
		for (i = j->lo; i < j->hi; i++)
			j->out[i] = hw_crc(0, j->base + j->offs[i], j->lens[i], &m);
	return 0;
}

/* buffer i = base + offs[i], lens[i] bytes, seed 0; `threads` POSIX threads
 * over contiguous slices, `reps` passes.  Returns 0, or -1 if a thread failed
 * to start. */
int hw_crc32c_batch_mt(const void *base, const uint64_t *offs, const uint32_t *lens, uint32_t *out, unsigned int n,
		       unsigned int threads, unsigned int reps)
{
	pthread_t tid[256];
	struct hw_job job[256];
	unsigned int t, started = 0;

	if (threads < 1 || threads > 256)
		return -1;
	for (t = 0; t < threads; t++) {
		job[t].base = base;
		job[t].offs = offs;
		job[t].lens = lens;
		job[t].out = out;
		job[t].lo = (unsigned int)((uint64_t)n * t / threads);
		job[t].hi = (unsigned int)((uint64_t)n * (t + 1) / threads);
		job[t].reps = reps;
		if (pthread_create(&tid[t], 0, hw_worker, &job[t]))
			break;
		started++;
	}
	for (t = 0; t < started; t++)
		pthread_join(tid[t], 0);
	return started == threads ? 0 : -1;
}
