/*
 * coro_stack.c -- the library called from a pech-style coroutine (TEST
 * PROGRAM, not product code; links the test oracle for expected values).
 *
 * pech runs the messenger on workqueue tasks with 64 KiB stacks
 * (/root/reference/src/sched.c:16 TASK_STACK_SIZE), entered once through
 * ucontext and then switched with setjmp/longjmp (:120-128, :175-230).  This
 * program builds the same kind of task on a 64 KiB mmap'd stack with a
 * PROT_NONE guard page below it, and from inside the task calls:
 *   crc32c() at 49 B, 4 KiB, 64 KiB + 1 and 8 MiB (host and GPU routes, and
 *   every size again with crc32c_set_cpu_max(0): all on the GPU),
 *   crc32c_batch() on 16 buffers,
 *   crc32c_async_create/submit/flush/drain/destroy (callbacks run on the
 *   task's stack).
 * Every result is checked against the oracle.  The stack is pre-filled with
 * a pattern; the deepest byte the task touched is its high-water mark,
 * printed as "hwm <bytes>".  Usage: coro_stack [stack_kib] (default 64).
 * Exit 0 = all results exact; a stack overflow faults on the guard page.
 */
#define _GNU_SOURCE
#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <ucontext.h>
#include <unistd.h>

#include "pech_crc32c_async.h"

uint32_t oracle_crc32c(uint32_t crc, const void *data, unsigned int length);

static jmp_buf main_ctx, task_ctx;
static ucontext_t oneshot, back_uc;
static int failures;
static unsigned char *big;

#define BIG (8u << 20)

static void check(const char *what, unsigned int n, uint32_t got, uint32_t want)
{
	if (got != want) {
		printf("FAIL %s n=%u got %08x want %08x\n", what, n, got, want);
		failures++;
	}
}

struct cb_state {
	int calls;
	uint32_t want[4];
	uint32_t got[4];
	int err[4];
};

static void on_done(void *arg, uint32_t crc, int err)
{
	struct cb_state *st = (struct cb_state *)arg;
	volatile char probe[256]; /* the callback runs on the task's stack */

	probe[0] = 1;
	(void)probe[0];
	st->got[st->calls] = crc;
	st->err[st->calls] = err;
	st->calls++;
}

static void task_body(void)
{
	static const unsigned int sizes[] = {49, 4096, 65537, BIG};
	unsigned int i, pass;
	const void *bufs[16];
	unsigned int lens[16];
	uint32_t out[16];
	struct cb_state st;
	struct crc32c_async *a;

	for (pass = 0; pass < 2; pass++) {
		unsigned int prev = 0;
		if (pass == 1)
			prev = crc32c_set_cpu_max(0); /* every call on the GPU */
		for (i = 0; i < sizeof(sizes) / sizeof(sizes[0]); i++) {
			unsigned int n = sizes[i];
			check(pass ? "crc32c(gpu)" : "crc32c", n, crc32c(0x1234u + i, big + i, n),
			      oracle_crc32c(0x1234u + i, big + i, n));
		}
		if (pass == 1)
			crc32c_set_cpu_max(prev);
	}
	for (i = 0; i < 16; i++) {
		bufs[i] = big + 4096u * i + i;
		lens[i] = 1000u * i + 7u;
	}
	if (crc32c_batch(bufs, lens, NULL, out, 16, CRC32C_F_HOST)) {
		printf("FAIL crc32c_batch: %s\n", crc32c_last_error());
		failures++;
	}
	for (i = 0; i < 16; i++)
		check("crc32c_batch", lens[i], out[i], oracle_crc32c(0, bufs[i], lens[i]));

	memset(&st, 0, sizeof(st));
	a = crc32c_async_create(CRC32C_ASYNC_DEFAULT);
	if (!a) {
		printf("FAIL crc32c_async_create: %s\n", crc32c_last_error());
		failures++;
		return;
	}
	for (i = 0; i < 4; i++) {
		unsigned int n = i == 3 ? (3u << 20) + 5u : 4096u * (i + 1);
		st.want[i] = oracle_crc32c(i, big + 7 * i, n);
		if (crc32c_async_submit(a, big + 7 * i, n, i, on_done, &st)) {
			printf("FAIL crc32c_async_submit: %s\n", crc32c_last_error());
			failures++;
		}
	}
	if (crc32c_async_flush(a) || crc32c_async_drain(a)) {
		printf("FAIL async flush/drain: %s\n", crc32c_last_error());
		failures++;
	}
	crc32c_async_destroy(a);
	if (st.calls != 4) {
		printf("FAIL async callbacks: %d of 4\n", st.calls);
		failures++;
	}
	for (i = 0; i < (unsigned int)st.calls; i++)
		check("async", i, st.err[i] ? 0xdeadu : st.got[i], st.want[i]);
}

static void task_entry(void)
{
	if (!setjmp(task_ctx))
		longjmp(main_ctx, 1); /* as task_trampoline: park, return to creator */
	task_body();
	longjmp(main_ctx, 2);
}

int main(int argc, char **argv)
{
	const size_t kib = argc > 1 ? strtoul(argv[1], NULL, 10) : 64;
	const size_t stack = kib << 10;
	const long pg = sysconf(_SC_PAGESIZE);
	unsigned char *m, *lo;
	size_t i, hwm;
	int r;

	big = malloc(BIG + 64);
	if (!big)
		return 2;
	for (i = 0; i < BIG + 64; i++)
		big[i] = (unsigned char)(i * 2654435761u >> 13);
	m = mmap(NULL, stack + pg, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	if (m == MAP_FAILED)
		return 2;
	mprotect(m, pg, PROT_NONE); /* guard page: an overflow faults */
	lo = m + pg;
	memset(lo, 0xA5, stack);

	getcontext(&oneshot);
	oneshot.uc_stack.ss_sp = lo;
	oneshot.uc_stack.ss_size = stack;
	oneshot.uc_link = NULL;
	makecontext(&oneshot, task_entry, 0);
	r = setjmp(main_ctx);
	if (r == 0)
		swapcontext(&back_uc, &oneshot); /* first entry, like task_create() */
	else if (r == 1)
		longjmp(task_ctx, 1); /* schedule() into the task */
	/* r == 2: the task finished */
	for (i = 0; i < stack && lo[i] == 0xA5; i++)
		;
	hwm = stack - i;
	printf("stack %zu hwm %zu failures %d\n", stack, hwm, failures);
	return failures ? 1 : 0;
}
