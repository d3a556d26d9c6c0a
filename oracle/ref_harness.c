/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/).
 *
 * Compiles the reference's own header /root/reference/include/crc32c.h
 * (included by path through -iquote, never copied -- -iquote, not -I, so
 * pech's include/sched.h cannot shadow the system one pthread.h needs) into
 * a tiny shared library so tests and the golden-vector generator can call the
 * reference algorithm itself.  Only built when /root/reference is present (this container); the
 * resulting oracle/_ref/libref_crc32c.so travels to the GPU box with the
 * snapshot, for bench.py's cpu_baseline leg ("kind": "reference").
 */
#include <pthread.h>

#include "crc32c.h" /* /root/reference/include/crc32c.h */

/* exported wrapper around the static inline crc32c() of crc32c.h:88 */
u32 ref_crc32c(u32 crc, const void *data, unsigned int length)
{
	return crc32c(crc, data, length);
}

/* exported copy of crc32c_table (crc32c.h:16) for the table-regeneration test */
void ref_table_copy(u32 out[256])
{
	int i;

	for (i = 0; i < 256; i++)
		out[i] = crc32c_table[i];
}

/* strided batch, same shape as oracle_crc32c_strided() */
void ref_crc32c_strided(const void *base, unsigned long stride, unsigned int len,
			u32 *out, unsigned int n)
{
	unsigned int i;

	for (i = 0; i < n; i++)
		out[i] = crc32c(0, (const u8 *)base + (unsigned long)i * stride, len);
}

/* multi-threaded batch for bench.py's cpu_baseline leg (the
 * reference on 1 thread -- pech's model -- and on the box's cores over
 * independent buffers): buffer i is base + offs[i], lens[i] bytes, seed 0;
 * `threads` POSIX threads take contiguous slices of the batch, `reps` passes. */
struct mt_job {
	const u8 *base;
	const unsigned long *offs;
	const unsigned int *lens;
	u32 *out;
	unsigned int lo, hi, reps;
};

static void *mt_worker(void *arg)
{
	struct mt_job *j = arg;
	unsigned int r, i;

	for (r = 0; r < j->reps; r++)
		for (i = j->lo; i < j->hi; i++)
			j->out[i] = crc32c(0, j->base + j->offs[i], j->lens[i]);
	return 0;
}

int ref_crc32c_batch_mt(const void *base, const unsigned long *offs, const unsigned int *lens, u32 *out,
			unsigned int n, unsigned int threads, unsigned int reps)
{
	pthread_t tid[256];
	struct mt_job job[256];
	unsigned int t, started = 0;

	if (threads < 1 || threads > 256)
		return -1;
	for (t = 0; t < threads; t++) {
		job[t].base = base;
		job[t].offs = offs;
		job[t].lens = lens;
		job[t].out = out;
		job[t].lo = (unsigned int)((unsigned long)n * t / threads);
		job[t].hi = (unsigned int)((unsigned long)n * (t + 1) / threads);
		job[t].reps = reps;
		if (pthread_create(&tid[t], 0, mt_worker, &job[t]))
			break;
		started++;
	}
	for (t = 0; t < started; t++)
		pthread_join(tid[t], 0);
	return started == threads ? 0 : -1;
}
