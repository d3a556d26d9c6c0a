/*
 * gf2.h -- CRC-32C algebra over GF(2), shared by host and device code.
 *
 * Domain: the raw CRC register of /root/reference/include/crc32c.h:88-96
 * (reflected Castagnoli polynomial, no pre/post inversion).  Bit 31 of a
 * register value is the coefficient of x^0, bit 0 that of x^31, so the
 * element "1" is 0x80000000 and multiplying by x is a right shift with a
 * conditional xor of the reflected polynomial.
 *
 * Identities the kernels rely on:
 *   R(v, 0^n)        = v * x^(8n) mod P                       (A_n(v))
 *   R(s, A || B)     = A_|B|(R(s, A)) ^ R(0, B)                 (chaining)
 *   R(s, D)          = R(0, D ^ s)   |D| >= 4, s xored into D[0..4) LE
 *   R(0, 0^k || D)   = R(0, D)                                  (leading zeros)
 *   R(0, D || 0^z)   = A_z(R(0, D)), A_z invertible             (trailing zeros)
 */
#ifndef PECH_CRC32C_GF2_H
#define PECH_CRC32C_GF2_H

#include <stdint.h>

#ifdef __HIPCC__
#define GF2_FN __host__ __device__ __forceinline__
#else
#define GF2_FN static inline
#endif

#define CRC32C_POLY_REFLECTED 0x82F63B78u /* 0x1EDC6F41, include/crc32c.h:11 */
#define CRC32C_ONE 0x80000000u            /* x^0 */
#define CRC32C_X8 0x00800000u             /* x^8 */
#define CRC32C_XINV 0x05EC76F1u           /* x^-1: mulx(0x05EC76F1) == 1 */

/* v * x mod P */
GF2_FN uint32_t gf2_mulx(uint32_t v)
{
	return (v >> 1) ^ (CRC32C_POLY_REFLECTED & (0u - (v & 1u)));
}

/* a * b mod P.  Branch-free, 32 steps over the bits of a (x^0 first). */
GF2_FN uint32_t gf2_mulmod(uint32_t a, uint32_t b)
{
	uint32_t p = 0;
	for (int i = 31; i >= 0; --i) {
		p ^= b & (0u - ((a >> i) & 1u));
		b = gf2_mulx(b);
	}
	return p;
}

/* x^(8n) mod P by square-and-multiply (host-side table building and the
 * rare generic shifts; the kernels use the precomputed power tables). */
GF2_FN uint32_t gf2_x8n(uint64_t n)
{
	uint32_t r = CRC32C_ONE, sq = CRC32C_X8;
	while (n) {
		if (n & 1u)
			r = gf2_mulmod(r, sq);
		sq = gf2_mulmod(sq, sq);
		n >>= 1;
	}
	return r;
}

/* A_n(v) = R(v, 0^n) */
GF2_FN uint32_t gf2_shift(uint32_t v, uint64_t nbytes)
{
	return gf2_mulmod(gf2_x8n(nbytes), v);
}

/* x^(-8z) mod P */
GF2_FN uint32_t gf2_xinv8n(uint32_t z)
{
	uint32_t xinv8 = CRC32C_ONE;
	for (int i = 0; i < 8; ++i)
		xinv8 = gf2_mulmod(xinv8, CRC32C_XINV);
	uint32_t r = CRC32C_ONE;
	for (uint32_t i = 0; i < z; ++i)
		r = gf2_mulmod(r, xinv8);
	return r;
}

#endif /* PECH_CRC32C_GF2_H */
