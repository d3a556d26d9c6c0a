/*
 * crc32c_msgr.c -- the messenger-side adapter (include/pech_crc32c_msgr.h):
 * per-connection receive verify queues and send-side deferred footers on top
 * of the async layer.  Plain C (gcc); the GPU work is the async layer's.
 *
 * Routing by size: a payload of at most crc32c_msgr_set_host_max() bytes
 * (default PECH_MSGR_HOST_MAX_DEFAULT) is checksummed at once on the host
 * (pech_cpu_crc32c, crc32c_cpu.c, SSE4.2): below that size the host routine
 * costs less CPU time than submitting, launching and completing the payload
 * through the GPU (measured).  The entry is then ready at
 * once and takes the same queue/footer path as a GPU payload, so the
 * messenger's sequencing does not depend on the route.
 *
 * Routing by queue depth: a payload of at most
 * crc32c_msgr_set_lone_max() bytes (default PECH_MSGR_LONE_MAX_DEFAULT) that
 * arrives while its context has nothing outstanding, and is the first such
 * since the context's last flush (pech at queue depth 1: one
 * read_partial_msg_data -> footer compare per con_work pass,
 * messenger.c:2649-2684; the patch flushes at the end of every pass), is
 * checksummed on the host too: alone, it cannot share a launch, so the GPU
 * route costs the thread ~10 us of submit / launch / complete and the
 * payload ~25-50 us of latency, which the host routine beats up to a few
 * hundred KiB.  The payloads after it in the same pass --
 * a burst -- batch on the GPU as before (throughput mode).
 *
 * A GPU failure never reaches the messenger as a wrong or missing CRC: a
 * submission the async layer refuses, or a batch that fails, is recomputed
 * on the host from the same bytes, which the adapter still owns at that point.
 *
 * Single-threaded by contract (pech runs one OS thread, README:11-16): the
 * connection state and the process-wide counters are plain data, touched only
 * by the caller's thread (callbacks run inside crc32c_async_complete()).
 */
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pech_crc32c_msgr.h"

#define PECH_HIDDEN __attribute__((visibility("hidden")))
PECH_HIDDEN uint32_t pech_cpu_crc32c(uint32_t crc, const void *data, size_t n);
/* crc32c_async.cpp: 1 (and taken) when the context has nothing outstanding
 * and no lone payload was host-routed since its last flush */
PECH_HIDDEN int pech_async_take_lone(struct crc32c_async *a);

#define PECH_MSGR_HOST_MAX_DEFAULT (8u << 10) /* profiles/r03/msgr_cutoff.txt */
#define PECH_MSGR_LONE_MAX_DEFAULT (256u << 10) /* lone payloads: thread CPU crossover, DESIGN.md §6.7 */
#define TX_BUCKETS 64u /* per connection, chained by msg address */

enum { ST_WAIT, ST_DONE };

struct rx_ent {
	struct rx_ent *next;
	struct crc32c_msgr_conn *conn; /* NULL: orphaned by a reset, released when its CRC lands */
	crc32c_msgr_release_fn release;
	void *msg;
	const void *data;
	unsigned int len;
	uint32_t want, got;
	int state, check;
	unsigned int skips; /* a marker (msg NULL): the consecutive skipped messages it stands for */
};

struct tx_ent {
	struct tx_ent *next;  /* send order */
	struct tx_ent **prev; /* the link that points here (send-order list) */
	struct tx_ent *hnext; /* hash chain */
	struct crc32c_msgr_conn *conn; /* NULL: orphaned (cancel/destroy), released when its CRC lands */
	crc32c_msgr_release_fn release;
	void *msg;
	const void *data;
	unsigned int len;
	uint32_t seed, crc;
	int state, waiting;
};

struct crc32c_msgr_conn {
	struct crc32c_async *a;
	unsigned int max_pending, npending;
	struct rx_ent *head, *tail;
	struct tx_ent *tx, **tx_tail; /* send order */
	struct tx_ent *tx_hash[TX_BUCKETS];
	crc32c_msgr_kick_fn kick;
	void *kick_arg;
	crc32c_msgr_release_fn release;
	struct rx_ent *rx_cache; /* retired receive entries for reuse (host-routed payloads churn them) */
	unsigned int nrx_cache;
};

#define RX_CACHE_MAX 256u

static struct crc32c_msgr_stats g_st;
static unsigned int g_host_max = PECH_MSGR_HOST_MAX_DEFAULT;
static int g_host_max_env;
static unsigned int g_lone_max = PECH_MSGR_LONE_MAX_DEFAULT;
static int g_lone_max_env;

/* a byte count from the environment (once), else *v unchanged */
static void env_bytes(const char *name, unsigned int *v, int *read)
{
	const char *e;

	if (*read)
		return;
	*read = 1;
	e = getenv(name);
	if (e && *e) {
		char *end = NULL;
		const unsigned long long x = strtoull(e, &end, 0);
		if (end != e)
			*v = x > 0xFFFFFFFFull ? 0xFFFFFFFFu : (unsigned int)x;
	}
}

static unsigned int host_max(void)
{
	env_bytes("PECH_CRC32C_MSGR_HOST_MAX", &g_host_max, &g_host_max_env);
	return g_host_max;
}

static unsigned int lone_max(void)
{
	env_bytes("PECH_CRC32C_MSGR_LONE_MAX", &g_lone_max, &g_lone_max_env);
	return g_lone_max;
}

unsigned int crc32c_msgr_set_host_max(unsigned int bytes)
{
	const unsigned int prev = host_max();

	g_host_max = bytes;
	return prev;
}

unsigned int crc32c_msgr_set_lone_max(unsigned int bytes)
{
	const unsigned int prev = lone_max();

	g_lone_max = bytes;
	return prev;
}

/* the route of one checked payload: 1 = host routine now (counted in *lone
 * when only because its context is idle), 0 = the GPU */
static int route_host(const struct crc32c_msgr_conn *c, unsigned int len, uint64_t *lone)
{
	if (!host_max())
		return 0; /* 0: every checked payload to the GPU (lone ones too) */
	if (len <= host_max())
		return 1;
	if (lone_max() && len <= lone_max() && pech_async_take_lone(c->a)) {
		(*lone)++;
		return 1;
	}
	return 0;
}

static void kick(struct crc32c_msgr_conn *c)
{
	if (c && c->kick)
		c->kick(c->kick_arg);
}

/* ---- receive ---------------------------------------------------------- */

static void rx_done(void *arg, uint32_t crc, int err)
{
	struct rx_ent *e = arg;

	if (err) /* the GPU failed: same bytes, host routine */
		crc = pech_cpu_crc32c(0, e->data, e->len);
	if (!e->conn) {
		if (e->msg)
			e->release(e->msg);
		g_st.rx_released++;
		free(e);
		return;
	}
	e->got = crc;
	e->state = ST_DONE;
	kick(e->conn);
}

struct crc32c_msgr_conn *crc32c_msgr_conn_create(struct crc32c_async *a, unsigned int max_pending,
						 crc32c_msgr_kick_fn kick_fn, void *kick_arg,
						 crc32c_msgr_release_fn release)
{
	struct crc32c_msgr_conn *c;

	if (!a || !max_pending || !release)
		return NULL;
	c = calloc(1, sizeof(*c));
	if (!c)
		return NULL;
	c->a = a;
	c->max_pending = max_pending;
	c->kick = kick_fn;
	c->kick_arg = kick_arg;
	c->release = release;
	c->tx_tail = &c->tx;
	return c;
}

static struct rx_ent *rx_alloc(struct crc32c_msgr_conn *c)
{
	struct rx_ent *e = c->rx_cache;

	if (!e)
		return calloc(1, sizeof(*e));
	c->rx_cache = e->next;
	c->nrx_cache--;
	memset(e, 0, sizeof(*e));
	return e;
}

/* a retired entry of connection c (never an orphan: those are freed where they land) */
static void rx_retire(struct crc32c_msgr_conn *c, struct rx_ent *e)
{
	if (c->nrx_cache >= RX_CACHE_MAX) {
		free(e);
		return;
	}
	e->next = c->rx_cache;
	c->rx_cache = e;
	c->nrx_cache++;
}

int crc32c_msgr_rx_queue(struct crc32c_msgr_conn *c, void *msg, const void *data, unsigned int len, int check,
			 uint32_t footer_crc)
{
	struct rx_ent *e;

	if (!c || (len && !data) || (!msg && check))
		return -EINVAL;
	if (c->npending >= c->max_pending && msg) /* skip markers hold no message: always taken */
		return -EAGAIN;
	if (!msg && c->tail && !c->tail->msg) {
		/* consecutive markers share an entry: entries stay bounded by
		 * 2 * max_pending + 1 while the head waits for its CRC */
		c->tail->skips++;
		c->npending++;
		g_st.rx_unchecked++;
		return 0;
	}
	e = rx_alloc(c);
	if (!e)
		return -ENOMEM;
	e->conn = c;
	e->release = c->release;
	e->msg = msg;
	e->data = data;
	e->len = len;
	e->want = footer_crc;
	e->check = check != 0;
	e->skips = msg ? 0u : 1u;
	e->state = e->check ? ST_WAIT : ST_DONE;
	if (c->tail)
		c->tail->next = e;
	else
		c->head = e;
	c->tail = e;
	c->npending++;
	if (!e->check) {
		g_st.rx_unchecked++;
		return 0;
	}
	if (route_host(c, len, &g_st.rx_lone)) { /* small or lone payload: the host routine is cheaper */
		g_st.rx_host++;
		e->got = pech_cpu_crc32c(0, data, len);
		e->state = ST_DONE;
		return 0;
	}
	g_st.rx_submitted++;
	if (crc32c_async_submit(c->a, data, len, 0, rx_done, e)) {
		/* refused (context error or no GPU): no callback will come; host routine now */
		g_st.rx_host++;
		e->got = pech_cpu_crc32c(0, data, len);
		e->state = ST_DONE;
	}
	return 0;
}

int crc32c_msgr_rx_next(struct crc32c_msgr_conn *c, void **msg, uint32_t *crc)
{
	struct rx_ent *e;
	int rc;

	if (!c || !msg || !crc)
		return -EINVAL;
	e = c->head;
	if (!e || e->state != ST_DONE)
		return 0;
	if (!e->msg && e->skips > 1) { /* one skipped message of a shared marker */
		e->skips--;
		c->npending--;
		*msg = NULL;
		*crc = 0u;
		return 1;
	}
	c->head = e->next;
	if (!c->head)
		c->tail = NULL;
	c->npending--;
	*msg = e->msg;
	*crc = e->check ? e->got : 0u;
	rc = 1;
	if (e->check && e->got != e->want) {
		g_st.rx_bad++;
		rc = -EBADMSG;
	} else if (e->check) {
		g_st.rx_verified++;
	}
	rx_retire(c, e);
	return rc;
}

unsigned int crc32c_msgr_rx_pending(const struct crc32c_msgr_conn *c)
{
	return c ? c->npending : 0u;
}

/* ---- send ------------------------------------------------------------- */

static unsigned int tx_bucket(const void *msg)
{
	uintptr_t h = (uintptr_t)msg;

	h ^= h >> 17; /* messages are heap objects: drop the alignment bits */
	h *= 0x9E3779B97F4A7C15ull;
	return (unsigned int)(h >> 58) & (TX_BUCKETS - 1u);
}

static struct tx_ent *tx_find(struct crc32c_msgr_conn *c, const void *msg)
{
	struct tx_ent *e;

	for (e = c->tx_hash[tx_bucket(msg)]; e; e = e->hnext)
		if (e->msg == msg)
			return e;
	return NULL;
}

/* take e off both of its connection's lists */
static void tx_unlink(struct crc32c_msgr_conn *c, struct tx_ent *e)
{
	struct tx_ent **pp;

	for (pp = &c->tx_hash[tx_bucket(e->msg)]; *pp != e; pp = &(*pp)->hnext)
		;
	*pp = e->hnext;
	*e->prev = e->next;
	if (e->next)
		e->next->prev = e->prev;
	else
		c->tx_tail = e->prev;
	e->next = e->hnext = NULL;
	e->prev = NULL;
}

static struct tx_ent *tx_new(struct crc32c_msgr_conn *c, void *msg)
{
	struct tx_ent *e = calloc(1, sizeof(*e));
	const unsigned int b = tx_bucket(msg);

	if (!e)
		return NULL;
	e->conn = c;
	e->release = c->release;
	e->msg = msg;
	e->prev = c->tx_tail; /* append: send order */
	*c->tx_tail = e;
	c->tx_tail = &e->next;
	e->hnext = c->tx_hash[b];
	c->tx_hash[b] = e;
	return e;
}

static void tx_done(void *arg, uint32_t crc, int err)
{
	struct tx_ent *e = arg;

	if (err)
		crc = pech_cpu_crc32c(e->seed, e->data, e->len);
	if (!e->conn) {
		e->release(e->msg);
		g_st.tx_released++;
		free(e);
		return;
	}
	e->crc = crc;
	e->state = ST_DONE;
	if (e->waiting)
		kick(e->conn);
}

int crc32c_msgr_tx_submit(struct crc32c_msgr_conn *c, void *msg, const void *data, unsigned int len, uint32_t seed)
{
	struct tx_ent *e;

	if (!c || (len && !data))
		return -EINVAL;
	if (tx_find(c, msg))
		return 1; /* resend: the bytes and so the CRC are unchanged; no new reference taken */
	e = tx_new(c, msg);
	if (!e)
		return -ENOMEM;
	e->data = data;
	e->len = len;
	e->seed = seed;
	e->state = ST_WAIT;
	if (route_host(c, len, &g_st.tx_lone)) {
		g_st.tx_host++;
		e->crc = pech_cpu_crc32c(seed, data, len);
		e->state = ST_DONE;
		return 0;
	}
	g_st.tx_submitted++;
	if (crc32c_async_submit(c->a, data, len, seed, tx_done, e)) {
		/* refused: no callback will come; host routine now */
		g_st.tx_host++;
		e->crc = pech_cpu_crc32c(seed, data, len);
		e->state = ST_DONE;
	}
	return 0;
}

int crc32c_msgr_tx_known(struct crc32c_msgr_conn *c, void *msg, uint32_t crc)
{
	struct tx_ent *e;

	if (!c)
		return -EINVAL;
	if (tx_find(c, msg))
		return 1;
	e = tx_new(c, msg);
	if (!e)
		return -ENOMEM;
	e->crc = crc;
	e->state = ST_DONE;
	g_st.tx_known++;
	return 0;
}

int crc32c_msgr_tx_has(const struct crc32c_msgr_conn *c, const void *msg)
{
	return c && tx_find((struct crc32c_msgr_conn *)c, msg) ? 1 : 0;
}

int crc32c_msgr_tx_footer(struct crc32c_msgr_conn *c, void *msg, uint32_t *crc)
{
	struct tx_ent *e;

	if (!c || !crc)
		return -EINVAL;
	e = tx_find(c, msg);
	if (!e)
		return -ENOENT;
	if (e->state != ST_DONE) {
		if (!e->waiting)
			g_st.tx_held++;
		e->waiting = 1;
		return 0;
	}
	*crc = e->crc;
	tx_unlink(c, e);
	free(e);
	return 1;
}

/* drop e: released now, or (its CRC still in flight) when the CRC lands */
static void tx_drop(struct crc32c_msgr_conn *c, struct tx_ent *e)
{
	tx_unlink(c, e);
	if (e->state == ST_WAIT) {
		e->conn = NULL; /* the GPU still reads its bytes: released in tx_done */
		return;
	}
	c->release(e->msg);
	g_st.tx_released++;
	free(e);
}

unsigned int crc32c_msgr_tx_cancel(struct crc32c_msgr_conn *c, void *msg)
{
	struct tx_ent *e;
	unsigned int n = 0;

	if (!c)
		return 0;
	if (msg) {
		e = tx_find(c, msg);
		if (e) {
			tx_drop(c, e);
			n = 1;
		}
		return n;
	}
	while (c->tx) {
		tx_drop(c, c->tx);
		++n;
	}
	return n;
}

void crc32c_msgr_conn_reset(struct crc32c_msgr_conn *c)
{
	struct rx_ent *e, *n;

	if (!c)
		return;
	for (e = c->head; e; e = n) {
		n = e->next;
		if (e->state == ST_WAIT) {
			e->conn = NULL; /* the GPU still reads its bytes: released in rx_done */
			e->next = NULL;
		} else {
			if (e->msg) /* NULL: an in-order skip marker */
				c->release(e->msg);
			g_st.rx_released++;
			rx_retire(c, e);
		}
	}
	c->head = c->tail = NULL;
	c->npending = 0;
}

struct crc32c_async *crc32c_msgr_conn_async(const struct crc32c_msgr_conn *c)
{
	return c ? c->a : NULL;
}

void crc32c_msgr_conn_destroy(struct crc32c_msgr_conn *c)
{
	if (!c)
		return;
	crc32c_msgr_conn_reset(c);
	crc32c_msgr_tx_cancel(c, NULL);
	while (c->rx_cache) {
		struct rx_ent *e = c->rx_cache;

		c->rx_cache = e->next;
		free(e);
	}
	free(c);
}

void crc32c_msgr_get_stats(struct crc32c_msgr_stats *st)
{
	if (st)
		*st = g_st;
}
