/*
 * msgr_sim.c -- TEST PROGRAM: pech's receive path on libpech_crc32c's async
 * layer, in pech's own dialect (gnu89 C, one OS thread, epoll loop).
 *
 * What it plays out (file:line in /root/reference):
 *   - osds_alloc_msg() -> alloc_bvec(): every message's data section is ONE
 *     contiguous 2^order-page buffer (src/ceph/osd_server.c:2317-2381,
 *     :208-215); here from crc32c_pages_alloc() (pinned) or, for every
 *     third message, plain malloc (pageable), both paths of the library.
 *   - read_partial_msg_data() (src/ceph/messenger.c:2649-2684): bytes arrive;
 *     the reference chains crc32c() per <=4 KiB piece as they come.  Here the
 *     payload is submitted ONCE when total_resid reaches 0.
 *   - the footer check (messenger.c:2836-2842): the callback compares the
 *     GPU result with footer.data_crc, which the sender computed with the
 *     reference per-piece chain (oracle_crc32c_pieces, the test oracle).
 *   - the event loop (src/event.c:52-70): epoll_wait on the context's
 *     eventfd, as an event_item would (include/event.h:7-28).
 *   - several GPUs from pech's one thread: argv[3] contexts,
 *     context k created on device k % device-count, messages dealt round
 *     robin, one eventfd each on the same epoll set.
 * Exit status 0 iff every message verified and none is left pending.
 *
 * Bench mode (bench.py's msgr_async leg for small payloads):
 *   msgr_sim bench <payload bytes> <count> <zerocopy> <passes>
 * submits <count> payloads of crc32c_pages memory per pass (carved from
 * order-11 blocks), flushing every 64, and drains through the eventfd; checks
 * every result of the first pass against the oracle, then prints one JSON
 * line with GiB/s and payloads/s over the timed passes.
 *
 * Build: `make build/msgr_sim` (part of `make all`; gnu89, -Wall -Werror).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "pech_crc32c_async.h"

/* the test oracle (oracle/crc32c_oracle.c): reference loop, per-piece chain */
uint32_t oracle_crc32c_pieces(uint32_t crc, const void *data, size_t length, unsigned int piece);

struct msg {
	unsigned char *data;
	unsigned int data_len;
	unsigned int order; /* pages order, or ~0u for malloc */
	uint32_t footer_data_crc; /* what the peer put on the wire */
	int verified;
};

static unsigned int nr_bad, nr_done;

static void data_crc_done(void *arg, uint32_t crc, int err)
{
	struct msg *m = arg;

	if (err || crc != m->footer_data_crc) {
		fprintf(stderr, "bad crc: len %u got %08x want %08x err %d\n", m->data_len, crc, m->footer_data_crc,
			err);
		nr_bad++;
	}
	m->verified = 1;
	nr_done++;
}

static unsigned int order_for(unsigned int len)
{
	unsigned int o = 0;

	while ((CRC32C_PAGE_SIZE << o) < len)
		o++;
	return o;
}

static uint32_t xs = 0x2545F491u;

static unsigned char next_byte(void)
{
	xs ^= xs << 13;
	xs ^= xs >> 17;
	xs ^= xs << 5;
	return (unsigned char)xs;
}

struct bench_slot {
	uint32_t want, got;
	int err;
};

static void bench_done(void *arg, uint32_t crc, int err)
{
	struct bench_slot *b = arg;

	b->got = crc;
	b->err = err;
}

static double now_s(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int bench_main(unsigned int size, unsigned int count, unsigned int zerocopy, unsigned int passes)
{
	const size_t block = (size_t)CRC32C_PAGE_SIZE << 11;
	const size_t stride = ((size_t)size + 255u) & ~(size_t)255u;
	const unsigned int per_block = (unsigned int)(block / (stride ? stride : 256u));
	unsigned int nblocks = (count + per_block - 1) / per_block, i, p, bad = 0;
	unsigned char **blocks = calloc(nblocks, sizeof(*blocks));
	struct bench_slot *slots = calloc(count, sizeof(*slots));
	struct crc32c_async *a = crc32c_async_create(zerocopy ? CRC32C_ASYNC_ZEROCOPY : CRC32C_ASYNC_DEFAULT);
	double t0 = 0, t1;

	if (!a || !blocks || !slots || !per_block)
		return 2;
	for (i = 0; i < nblocks; i++) {
		size_t k;

		blocks[i] = crc32c_pages_alloc(11);
		if (!blocks[i])
			return 2;
		for (k = 0; k < block; k++)
			blocks[i][k] = next_byte();
	}
	for (i = 0; i < count; i++)
		slots[i].want = oracle_crc32c_pieces(0, blocks[i / per_block] + (size_t)(i % per_block) * stride, size,
						     4096);
	for (p = 0; p <= passes; p++) {
		if (p == 1)
			t0 = now_s(); /* pass 0 is the warm-up */
		for (i = 0; i < count; i++) {
			if (crc32c_async_submit(a, blocks[i / per_block] + (size_t)(i % per_block) * stride, size, 0,
						bench_done, &slots[i]))
				return 2;
			if (i % 64 == 63 && crc32c_async_flush(a))
				return 2;
		}
		if (crc32c_async_drain(a))
			return 2;
		if (p == 0)
			for (i = 0; i < count; i++)
				bad += slots[i].err || slots[i].got != slots[i].want;
	}
	t1 = now_s();
	printf("{\"payload_bytes\": %u, \"payloads\": %u, \"passes\": %u, \"zerocopy\": %u, \"bad\": %u, "
	       "\"GiBps\": %.3f, \"payloads_per_s\": %.0f}\n",
	       size, count, passes, zerocopy, bad, (double)size * count * passes / (t1 - t0) / (1u << 30),
	       (double)count * passes / (t1 - t0));
	crc32c_async_destroy(a);
	for (i = 0; i < nblocks; i++)
		crc32c_pages_free(blocks[i], 11);
	crc32c_pages_trim();
	return bad ? 1 : 0;
}

int main(int argc, char **argv)
{
	static const unsigned int sizes[] = {0, 1, 100, 4096, 4097, 65536, 131072, 1 << 20, (4 << 20) + 3,
					     (40 << 20) + 17};
	unsigned int nmsgs = argc > 1 ? (unsigned int)atoi(argv[1]) : 300;
	unsigned int zerocopy = argc > 2 ? (unsigned int)atoi(argv[2]) : 0;
	unsigned int nctx = argc > 3 ? (unsigned int)atoi(argv[3]) : 1;
	struct crc32c_async *ctxs[16], *a;
	struct epoll_event ev, out[16];
	struct msg *msgs;
	unsigned int i, k, c;
	int ep, rc, ndev = 1;

	if (argc > 5 && !strcmp(argv[1], "bench"))
		return bench_main((unsigned int)atoi(argv[2]), (unsigned int)atoi(argv[3]), (unsigned int)atoi(argv[4]),
				  (unsigned int)atoi(argv[5]));
	if (nctx < 1 || nctx > 16)
		return 2;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
		ndev = 1;
	ep = epoll_create1(0);
	if (ep < 0) {
		perror("epoll_create1");
		return 2;
	}
	for (c = 0; c < nctx; c++) {
		/* the context keeps the device current at creation */
		if (hipSetDevice((int)(c % (unsigned int)ndev)) != hipSuccess)
			return 2;
		ctxs[c] = crc32c_async_create(zerocopy ? CRC32C_ASYNC_ZEROCOPY : CRC32C_ASYNC_DEFAULT);
		if (!ctxs[c]) {
			fprintf(stderr, "crc32c_async_create: %s\n", crc32c_last_error());
			return 2;
		}
		memset(&ev, 0, sizeof(ev));
		ev.events = EPOLLIN;
		ev.data.u32 = c;
		if (epoll_ctl(ep, EPOLL_CTL_ADD, crc32c_async_fd(ctxs[c]), &ev)) {
			perror("epoll_ctl");
			return 2;
		}
	}
	(void)hipSetDevice(0); /* the contexts switch devices themselves */
	msgs = calloc(nmsgs, sizeof(*msgs));
	for (i = 0; i < nmsgs; i++) {
		struct msg *m = &msgs[i];

		m->data_len = sizes[(i * 7u) % (sizeof(sizes) / sizeof(sizes[0]))];
		if (i % 3 == 2) {
			m->order = ~0u;
			m->data = malloc(m->data_len ? m->data_len : 1);
		} else {
			m->order = order_for(m->data_len);
			m->data = crc32c_pages_alloc(m->order);
		}
		if (!m->data) {
			fprintf(stderr, "alloc: %s\n", crc32c_last_error());
			return 2;
		}
		/* "receive" the payload, then the peer's footer */
		for (k = 0; k < m->data_len; k++)
			m->data[k] = next_byte();
		m->footer_data_crc = oracle_crc32c_pieces(0, m->data, m->data_len, 4096);
		/* total_resid == 0: one submission for the whole payload */
		a = ctxs[i % nctx];
		rc = crc32c_async_submit(a, m->data, m->data_len, 0, data_crc_done, m);
		if (rc) {
			fprintf(stderr, "submit: %d %s\n", rc, crc32c_last_error());
			return 2;
		}
		/* the connection's read burst ends every 16 messages: flush */
		if (i % 16 == 15 && (rc = crc32c_async_flush(a))) {
			fprintf(stderr, "flush: %d %s\n", rc, crc32c_last_error());
			return 2;
		}
		/* opportunistic completions between reads, without blocking */
		if (i % 5 == 0 && crc32c_async_complete(a) < 0)
			return 2;
	}
	for (c = 0; c < nctx; c++)
		if ((rc = crc32c_async_flush(ctxs[c]))) {
			fprintf(stderr, "flush: %d %s\n", rc, crc32c_last_error());
			return 2;
		}
	/* the event loop: wait for an eventfd, complete it, until nothing pending */
	for (;;) {
		unsigned int pending = 0;
		int n, j;

		for (c = 0; c < nctx; c++)
			pending += crc32c_async_pending(ctxs[c]);
		if (!pending)
			break;
		n = epoll_wait(ep, out, 16, 10000);
		if (n < 0) {
			perror("epoll_wait");
			return 2;
		}
		if (n == 0) {
			fprintf(stderr, "timeout: %u pending\n", pending);
			return 3;
		}
		for (j = 0; j < n; j++)
			if (crc32c_async_complete(ctxs[out[j].data.u32]) < 0) {
				fprintf(stderr, "complete: %s\n", crc32c_last_error());
				return 2;
			}
	}
	for (i = 0; i < nmsgs; i++) {
		if (!msgs[i].verified)
			nr_bad++;
		if (msgs[i].order == ~0u)
			free(msgs[i].data);
		else
			crc32c_pages_free(msgs[i].data, msgs[i].order);
	}
	for (c = 0; c < nctx; c++)
		crc32c_async_destroy(ctxs[c]);
	crc32c_pages_trim();
	printf("msgr_sim: %u messages, %u verified, %u bad (zerocopy %u, %u contexts on %d device(s))\n", nmsgs,
	       nr_done, nr_bad, zerocopy, nctx, ndev);
	return nr_bad ? 1 : 0;
}
