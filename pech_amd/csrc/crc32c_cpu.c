/*
 * crc32c_cpu.c -- the host-side pieces of the drop-in crc32c() that never
 * touch the GPU (product code, plain C, built by gcc; nothing here links or
 * includes oracle/):
 *
 *  1. pech_cpu_crc32c(): the reference's function (include/crc32c.h:88-96:
 *     raw register in, raw register out, no inversion) for the calls that
 *     SURVEY.md §8(a) rows a7/a8 keep on the CPU -- the 49-byte header and
 *     the front/middle sections (src/ceph/messenger.c:1403,1412,1418,2641,
 *     2714) and the <=4 KiB data pieces (:1729) -- and the fallback that
 *     keeps crc32c() total when the GPU fails (§8(b) "Errors").
 *     x86-64 hosts with SSE4.2 use the crc32 instruction (it computes exactly
 *     the reference register update: reflected 0x82F63B78, no inversion):
 *     three independent streams over equal blocks hide its 3-cycle latency
 *     and are joined with the GF(2) shift x^(8n) (gf2.h) applied through
 *     byte tables.  Other hosts use slice-by-8 tables built from the
 *     polynomial at first use.
 *
 *  2. pech_stack_call(): runs a function on a per-thread library stack.
 *     pech calls crc32c() from coroutines on 64 KiB stacks (src/sched.c:16,
 *     entered by setjmp/longjmp at :120-128); HIP API calls are not sized
 *     for that, so every path of the library that calls HIP runs on an
 *     8 MiB stack of its own (guard page below, reserved lazily), and the
 *     messenger's TASK_STACK_SIZE stays as it is.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include "gf2.h"

#define PECH_HIDDEN __attribute__((visibility("hidden")))

/* ------------------------------------------------------------------------ */
/* tables, built once from the polynomial                                  */

static uint32_t g_slice[8][256];      /* g_slice[k][e]: byte e followed by k zero bytes */
static uint32_t g_shift_long[4][256]; /* v -> A_LONG(v), one table per register byte  */
static uint32_t g_shift_short[4][256];
static int g_have_sse42;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

enum { LONG_BLK = 8192, SHORT_BLK = 256 }; /* bytes per stream in one 3-stream round */

static void shift_table(uint32_t t[4][256], uint64_t nbytes)
{
	const uint32_t xn = gf2_x8n(nbytes);
	for (int k = 0; k < 4; ++k)
		for (uint32_t e = 0; e < 256; ++e)
			t[k][e] = gf2_mulmod(xn, e << (8 * k));
}

static void init_tables(void)
{
	/* byte table of the reference (crc32c.h:16-81): T[e] = e * x^8 mod P */
	for (uint32_t e = 0; e < 256; ++e)
		g_slice[0][e] = gf2_mulmod(CRC32C_X8, e);
	for (int k = 1; k < 8; ++k)
		for (uint32_t e = 0; e < 256; ++e)
			g_slice[k][e] = (g_slice[k - 1][e] >> 8) ^ g_slice[0][g_slice[k - 1][e] & 0xFFu];
	shift_table(g_shift_long, LONG_BLK);
	shift_table(g_shift_short, SHORT_BLK);
#if defined(__x86_64__)
	__builtin_cpu_init();
	g_have_sse42 = __builtin_cpu_supports("sse4.2");
#endif
}

static inline uint32_t apply_shift(uint32_t t[4][256], uint32_t v)
{
	return t[0][v & 0xFFu] ^ t[1][(v >> 8) & 0xFFu] ^ t[2][(v >> 16) & 0xFFu] ^ t[3][v >> 24];
}

static inline uint64_t load64(const unsigned char *p)
{
	uint64_t v;
	memcpy(&v, p, 8);
	return v;
}

/* ------------------------------------------------------------------------ */
/* portable: slice-by-8                                                     */

static uint32_t crc_slice8(uint32_t crc, const unsigned char *p, size_t n)
{
	while (n && ((uintptr_t)p & 7u)) {
		crc = g_slice[0][(crc ^ *p++) & 0xFFu] ^ (crc >> 8);
		--n;
	}
	for (; n >= 8; n -= 8, p += 8) {
		const uint64_t w = load64(p) ^ crc; /* little-endian host */
		crc = g_slice[7][w & 0xFFu] ^ g_slice[6][(w >> 8) & 0xFFu] ^ g_slice[5][(w >> 16) & 0xFFu] ^
		      g_slice[4][(w >> 24) & 0xFFu] ^ g_slice[3][(w >> 32) & 0xFFu] ^ g_slice[2][(w >> 40) & 0xFFu] ^
		      g_slice[1][(w >> 48) & 0xFFu] ^ g_slice[0][w >> 56];
	}
	while (n--)
		crc = g_slice[0][(crc ^ *p++) & 0xFFu] ^ (crc >> 8);
	return crc;
}

/* ------------------------------------------------------------------------ */
/* x86-64 SSE4.2: crc32 instruction, three streams                          */

#if defined(__x86_64__)
#define SSE42 __attribute__((target("sse4.2")))

SSE42 static inline uint32_t run8(uint32_t c, const unsigned char *p, size_t words)
{
	uint64_t r = c;
	for (size_t i = 0; i < words; ++i)
		r = __builtin_ia32_crc32di(r, load64(p + 8 * i));
	return (uint32_t)r;
}

/* `blk` bytes per stream, rounds of 3 * blk while they fit */
SSE42 static inline uint32_t three_streams(uint32_t crc, const unsigned char **pp, size_t *np, size_t blk,
					    uint32_t t[4][256])
{
	const unsigned char *p = *pp;
	size_t n = *np;
	while (n >= 3 * blk) {
		uint64_t a = crc, b = 0, c = 0;
		const unsigned char *pa = p, *pb = p + blk, *pc = p + 2 * blk;
		for (size_t i = 0; i < blk; i += 8) {
			a = __builtin_ia32_crc32di(a, load64(pa + i));
			b = __builtin_ia32_crc32di(b, load64(pb + i));
			c = __builtin_ia32_crc32di(c, load64(pc + i));
		}
		/* R(s, A||B||C) = A_blk(A_blk(R(s,A)) ^ R(0,B)) ^ R(0,C) */
		crc = apply_shift(t, apply_shift(t, (uint32_t)a) ^ (uint32_t)b) ^ (uint32_t)c;
		p += 3 * blk;
		n -= 3 * blk;
	}
	*pp = p;
	*np = n;
	return crc;
}

SSE42 static uint32_t crc_sse42(uint32_t crc, const unsigned char *p, size_t n)
{
	while (n && ((uintptr_t)p & 7u)) {
		crc = __builtin_ia32_crc32qi(crc, *p++);
		--n;
	}
	crc = three_streams(crc, &p, &n, LONG_BLK, g_shift_long);
	crc = three_streams(crc, &p, &n, SHORT_BLK, g_shift_short);
	crc = run8(crc, p, n >> 3);
	p += n & ~(size_t)7u;
	n &= 7u;
	while (n--)
		crc = __builtin_ia32_crc32qi(crc, *p++);
	return crc;
}
#endif

PECH_HIDDEN uint32_t pech_cpu_crc32c(uint32_t crc, const void *data, size_t n)
{
	pthread_once(&g_once, init_tables);
#if defined(__x86_64__)
	if (g_have_sse42)
		return crc_sse42(crc, (const unsigned char *)data, n);
#endif
	return crc_slice8(crc, (const unsigned char *)data, n);
}

/* test hook (tests/test_cpu_path.py): force the portable path */
PECH_HIDDEN uint32_t pech_cpu_crc32c_portable(uint32_t crc, const void *data, size_t n)
{
	pthread_once(&g_once, init_tables);
	return crc_slice8(crc, (const unsigned char *)data, n);
}

PECH_HIDDEN int pech_cpu_has_sse42(void)
{
	pthread_once(&g_once, init_tables);
	return g_have_sse42;
}

/* ------------------------------------------------------------------------ */
/* per-thread library stack                                                 */

#define LIB_STACK_BYTES ((size_t)8 << 20)

struct lib_stack {
	unsigned char *base; /* mapping, guard page first */
	size_t bytes;
	int depth;           /* >0 while this thread runs on it */
};

static __thread struct lib_stack g_stack;
static pthread_key_t g_stack_key;
static pthread_once_t g_stack_once = PTHREAD_ONCE_INIT;

static void stack_release(void *p)
{
	struct lib_stack *s = (struct lib_stack *)p;
	if (s && s->base)
		munmap(s->base, s->bytes);
}

static int g_switch_off; /* PECH_STACK_SWITCH=0: diagnostic (tests/c/coro_stack.c) */

static void stack_key_init(void)
{
	const char *e = getenv("PECH_STACK_SWITCH");
	g_switch_off = e && e[0] == '0';
	(void)pthread_key_create(&g_stack_key, stack_release);
}

#if defined(__x86_64__)
/* rdi = arg, rsi = fn, rdx = 16-byte aligned stack top.  rbp keeps the
 * caller's stack pointer (callee-saved, so fn preserves it); the CFI makes
 * the frame walkable from the library stack back to the caller's. */
__asm__(".text\n"
	".p2align 4\n"
	".type pech_stack_switch_call,@function\n"
	"pech_stack_switch_call:\n"
	".cfi_startproc\n"
	"pushq %rbp\n"
	".cfi_def_cfa_offset 16\n"
	".cfi_offset %rbp, -16\n"
	"movq %rsp, %rbp\n"
	".cfi_def_cfa_register %rbp\n"
	"movq %rdx, %rsp\n"
	"callq *%rsi\n"
	"movq %rbp, %rsp\n"
	"popq %rbp\n"
	".cfi_def_cfa %rsp, 8\n"
	"ret\n"
	".cfi_endproc\n"
	".size pech_stack_switch_call, .-pech_stack_switch_call\n");
void pech_stack_switch_call(void *arg, void (*fn)(void *), void *top);
#endif

/* fn(arg) on this thread's library stack (directly when already on it, or
 * when the stack cannot be mapped -- then on the caller's stack, as before). */
PECH_HIDDEN void pech_stack_call(void (*fn)(void *), void *arg)
{
#if defined(__x86_64__)
	struct lib_stack *s = &g_stack;
	pthread_once(&g_stack_once, stack_key_init);
	if (g_switch_off) {
		fn(arg);
		return;
	}
	if (s->depth == 0 && !s->base) {
		const long pg = sysconf(_SC_PAGESIZE);
		void *m = mmap(NULL, LIB_STACK_BYTES + (size_t)pg, PROT_READ | PROT_WRITE,
			       MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE | MAP_STACK, -1, 0);
		if (m != MAP_FAILED) {
			(void)mprotect(m, (size_t)pg, PROT_NONE); /* guard page below the stack */
			s->base = (unsigned char *)m;
			s->bytes = LIB_STACK_BYTES + (size_t)pg;
			(void)pthread_setspecific(g_stack_key, s);
		}
	}
	if (s->depth == 0 && s->base) {
		s->depth = 1;
		pech_stack_switch_call(arg, fn, s->base + s->bytes);
		s->depth = 0;
		return;
	}
#endif
	fn(arg);
}

/* 1 while the calling thread runs on its library stack (tests) */
PECH_HIDDEN int pech_on_lib_stack(void)
{
	return g_stack.depth > 0;
}
