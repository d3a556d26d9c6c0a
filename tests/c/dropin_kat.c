/*
 * dropin_kat.c -- the drop-in crc32c() called from C exactly as pech's
 * messenger calls the inline original (TEST PROGRAM, not product code).
 *
 * Compiled as pech compiles messenger.c (gnu89, -Wall -Werror) against this
 * repo's include/crc32c.h and linked with libpech_crc32c.so.  For each
 * "len:seed" argument it generates SURVEY Appendix A's bytes (xorshift32,
 * state 0x2545F491) and prints three results on one line:
 *   whole   crc32c(seed, buf, len)                      one call
 *   pieces  the ceph_crc32c_iov chain over <=4096-byte page pieces
 *           (/root/reference/src/ceph/messenger.c:1734-1740,
 *            src/iov_iter.c:188-207)
 *   hdr     crc32c(0, buf, min(len, 49))  -- a header-sized call
 *           (messenger.c:1403, :2714: offsetof(ceph_msg_header, crc) = 49)
 * tests/test_abi.py compares them with tests/golden/kat.json.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crc32c.h"

static void gen(unsigned char *p, unsigned long n)
{
	unsigned int s = 0x2545F491u;
	unsigned long i;

	for (i = 0; i < n; i++) {
		s ^= s << 13;
		s ^= s >> 17;
		s ^= s << 5;
		p[i] = (unsigned char)(s & 0xFF);
	}
}

int main(int argc, char **argv)
{
	int a;

	for (a = 1; a < argc; a++) {
		unsigned long len = strtoul(argv[a], NULL, 10);
		const char *c = strchr(argv[a], ':');
		unsigned int seed = c ? (unsigned int)strtoul(c + 1, NULL, 16) : 0;
		unsigned char *buf = malloc(len ? len : 1);
		unsigned int whole, pieces, hdr;
		unsigned long off;

		if (!buf)
			return 2;
		gen(buf, len);
		whole = crc32c(seed, buf, (unsigned int)len);
		pieces = seed;
		for (off = 0; off < len; off += 4096) {
			unsigned long n = len - off < 4096 ? len - off : 4096;
			pieces = crc32c(pieces, buf + off, (unsigned int)n);
		}
		hdr = crc32c(0, buf, (unsigned int)(len < 49 ? len : 49));
		printf("%lu %08x %08x %08x %08x\n", len, seed, whole, pieces, hdr);
		free(buf);
	}
	return 0;
}
