/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/).
 *
 * Compiles the reference's own header /root/reference/include/crc32c.h
 * (included by path through -I, never copied) into a tiny shared library so
 * tests and the golden-vector generator can call the reference algorithm
 * itself.  Only built when /root/reference is present (this container); the
 * resulting oracle/_ref/libref_crc32c.so travels to the GPU box with the
 * snapshot, for bench.py's cpu_baseline leg ("kind": "reference").
 */
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
