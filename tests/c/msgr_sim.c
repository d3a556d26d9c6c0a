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
 * Bench mode (bench.py's msgr_async leg):
 *   msgr_sim bench <payload bytes> <count> <mode> <passes>
 * mode 0 async DMA (CRC32C_ASYNC_DMA), 1 async zero-copy (the default), 2 messenger adapter, 3 host routine
 * (bench_main): <count> payloads of crc32c_pages memory per pass, flushed
 * every 64, completed from an epoll loop; checks every result against the
 * oracle, then prints one JSON line: GiB/s, payloads/s, CPU microseconds per
 * payload of the calling thread and of the process, submit -> result
 * latency p50/p99.
 *
 * Build: `make build/msgr_sim` (part of `make all`; gnu89, -Wall -Werror).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/resource.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "crc32c.h"
#include "pech_crc32c_async.h"
#include "pech_crc32c_msgr.h"

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
	int err, done;
	double t_sub, t_done;
};

static double now_s(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* CPU seconds of the calling thread (pech's one OS thread) */
static double thread_cpu_s(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* CPU seconds of the whole process (HIP runtime threads included) */
static double process_cpu_s(void)
{
	struct rusage ru;

	getrusage(RUSAGE_SELF, &ru);
	return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}

static void bench_done(void *arg, uint32_t crc, int err)
{
	struct bench_slot *b = arg;

	b->got = crc;
	b->err = err;
	b->done = 1;
	b->t_done = now_s();
}

static void bench_release(void *msg)
{
	(void)msg; /* the adapter never drops a verified-queue entry here */
}

static int cmp_double(const void *a, const void *b)
{
	const double x = *(const double *)a, y = *(const double *)b;

	return x < y ? -1 : x > y;
}

/* take verified messages off the adapter's queue (its dispatch loop) */
static int adapter_dispatch(struct crc32c_msgr_conn *conn, unsigned int *bad)
{
	void *msg;
	uint32_t crc;
	int rc, n = 0;

	while ((rc = crc32c_msgr_rx_next(conn, &msg, &crc)) != 0) {
		struct bench_slot *b = msg;

		if (rc < 0)
			(*bad)++;
		b->got = crc;
		b->done = 1;
		b->t_done = now_s();
		n++;
	}
	return n;
}

/*
 * Bench mode: <count> payloads of <size> bytes in crc32c_pages memory per
 * pass, submitted as a server's read bursts do (flush every 64), completed
 * from an epoll loop on the context's eventfd (non-blocking complete()
 * between bursts, epoll_wait at the end).  mode 0: async layer, DMA;
 * 1: async layer, zero-copy; 2: the messenger adapter (rx_queue / rx_next on
 * a zero-copy context, its size routing at its default); 3: the drop-in
 * crc32c() per payload (host routine).  Reports the calling thread's CPU
 * time per payload (pech's one OS thread), the process's (HIP runtime
 * threads included) and the submit -> result latency.
 */
static int bench_main(unsigned int size, unsigned int count, unsigned int mode, unsigned int passes)
{
	const size_t block = (size_t)CRC32C_PAGE_SIZE << 11;
	const size_t stride = ((size_t)size + 255u) & ~(size_t)255u;
	const unsigned int per_block = (unsigned int)(block >= stride ? block / (stride ? stride : 256u) : 0u);
	const unsigned int order = size > block ? order_for(size) : 11u;
	const unsigned int nblocks = per_block ? (count + per_block - 1) / per_block : count;
	unsigned int i, p, bad = 0, k;
	unsigned char **blocks = calloc(nblocks, sizeof(*blocks));
	struct bench_slot *slots = calloc(count, sizeof(*slots));
	double *lat = calloc((size_t)count * passes + 1, sizeof(double));
	struct crc32c_async *a = NULL;
	struct crc32c_msgr_conn *conn = NULL;
	double t0 = 0, c0 = 0, pc0 = 0, t1, c1, pc1;
	size_t nlat = 0;
	int ep = -1;

	if (!blocks || !slots || !lat)
		return 2;
	if (mode != 3) {
		struct epoll_event ev;

		a = crc32c_async_create(mode == 0 ? CRC32C_ASYNC_DMA : CRC32C_ASYNC_DEFAULT);
		if (!a)
			return 2;
		ep = epoll_create1(0);
		memset(&ev, 0, sizeof(ev));
		ev.events = EPOLLIN;
		if (ep < 0 || epoll_ctl(ep, EPOLL_CTL_ADD, crc32c_async_fd(a), &ev))
			return 2;
		if (mode == 2 && !(conn = crc32c_msgr_conn_create(a, count + 1u, NULL, NULL, bench_release)))
			return 2;
	}
	for (i = 0; i < nblocks; i++) {
		size_t nb = per_block ? block : (size_t)CRC32C_PAGE_SIZE << order;

		blocks[i] = crc32c_pages_alloc(per_block ? 11u : order);
		if (!blocks[i])
			return 2;
		for (k = 0; k < nb; k++)
			blocks[i][k] = next_byte();
	}
#define PAYLOAD(i) (per_block ? blocks[(i) / per_block] + (size_t)((i) % per_block) * stride : blocks[i])
	for (i = 0; i < count; i++)
		slots[i].want = oracle_crc32c_pieces(0, PAYLOAD(i), size, 4096);
	for (p = 0; p <= passes; p++) {
		unsigned int left = count;

		if (p == 1) { /* pass 0 is the warm-up */
			t0 = now_s();
			c0 = thread_cpu_s();
			pc0 = process_cpu_s();
		}
		for (i = 0; i < count; i++)
			slots[i].done = 0;
		for (i = 0; i < count; i++) {
			struct bench_slot *b = &slots[i];

			b->t_sub = now_s();
			if (mode == 3) {
				b->got = crc32c(0, PAYLOAD(i), size);
				b->done = 1;
				b->t_done = now_s();
				left--;
				continue;
			}
			if (mode == 2) {
				if (crc32c_msgr_rx_queue(conn, b, PAYLOAD(i), size, 1, b->want))
					return 2;
			} else if (crc32c_async_submit(a, PAYLOAD(i), size, 0, bench_done, b)) {
				return 2;
			}
			if (i % 64 == 63) { /* end of a read burst: flush, complete without blocking */
				if (crc32c_async_flush(a) || crc32c_async_complete(a) < 0)
					return 2;
				if (mode == 2)
					adapter_dispatch(conn, &bad);
			}
		}
		if (a && crc32c_async_flush(a))
			return 2;
		for (;;) { /* the event loop until every result is in */
			struct epoll_event ev;

			if (mode == 2)
				adapter_dispatch(conn, &bad);
			for (left = 0, i = 0; i < count; i++)
				left += !slots[i].done;
			if (!left)
				break;
			if (epoll_wait(ep, &ev, 1, 10000) <= 0)
				return 3;
			if (crc32c_async_complete(a) < 0)
				return 2;
		}
		for (i = 0; i < count; i++) {
			bad += slots[i].err || slots[i].got != slots[i].want;
			if (p > 0)
				lat[nlat++] = slots[i].t_done - slots[i].t_sub;
		}
	}
#undef PAYLOAD
	t1 = now_s();
	c1 = thread_cpu_s();
	pc1 = process_cpu_s();
	qsort(lat, nlat, sizeof(double), cmp_double);
	printf("{\"payload_bytes\": %u, \"payloads\": %u, \"passes\": %u, \"mode\": \"%s\", \"bad\": %u, "
	       "\"GiBps\": %.3f, \"payloads_per_s\": %.0f, \"thread_cpu_us_per_payload\": %.3f, "
	       "\"process_cpu_us_per_payload\": %.3f, \"latency_us_p50\": %.1f, \"latency_us_p99\": %.1f}\n",
	       size, count, passes, mode == 0 ? "async-dma" : mode == 1 ? "async-zerocopy" : mode == 2 ? "adapter" : "host",
	       bad, (double)size * count * passes / (t1 - t0) / (1u << 30), (double)count * passes / (t1 - t0),
	       (c1 - c0) / ((double)count * passes) * 1e6, (pc1 - pc0) / ((double)count * passes) * 1e6,
	       nlat ? lat[nlat / 2] * 1e6 : 0.0, nlat ? lat[(size_t)(nlat * 0.99)] * 1e6 : 0.0);
	crc32c_msgr_conn_destroy(conn);
	if (a)
		crc32c_async_destroy(a);
	for (i = 0; i < nblocks; i++)
		crc32c_pages_free(blocks[i], per_block ? 11u : order);
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
		ctxs[c] = crc32c_async_create(zerocopy ? CRC32C_ASYNC_DEFAULT : CRC32C_ASYNC_DMA);
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
