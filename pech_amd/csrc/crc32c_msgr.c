/*
 * crc32c_msgr.c -- the messenger-side adapter (include/pech_crc32c_msgr.h):
 * per-connection receive verify queues and send-side deferred footers on top
 * of the async layer.  Plain C (gcc); the GPU work is the async layer's.
 *
 * A GPU failure never reaches the messenger as a wrong or missing CRC: a
 * submission the async layer refuses, or a batch that fails, is recomputed
 * on the host (pech_cpu_crc32c, crc32c_cpu.c) from the same bytes, which the
 * adapter still owns at that point.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pech_crc32c_msgr.h"

#define PECH_HIDDEN __attribute__((visibility("hidden")))
PECH_HIDDEN uint32_t pech_cpu_crc32c(uint32_t crc, const void *data, size_t n);

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
};

struct tx_ent {
	struct tx_ent *next;
	struct crc32c_msgr_conn *conn; /* NULL: orphaned by destroy, released when its CRC lands */
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
	struct tx_ent *tx;
	crc32c_msgr_kick_fn kick;
	void *kick_arg;
	crc32c_msgr_release_fn release;
};

static struct crc32c_msgr_stats g_st;

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
	return c;
}

int crc32c_msgr_rx_queue(struct crc32c_msgr_conn *c, void *msg, const void *data, unsigned int len, int check,
			 uint32_t footer_crc)
{
	struct rx_ent *e;

	if (!c || (len && !data))
		return -EINVAL;
	if (c->npending >= c->max_pending)
		return -EAGAIN;
	e = calloc(1, sizeof(*e));
	if (!e)
		return -ENOMEM;
	e->conn = c;
	e->release = c->release;
	e->msg = msg;
	e->data = data;
	e->len = len;
	e->want = footer_crc;
	e->check = check != 0;
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
	g_st.rx_submitted++;
	if (crc32c_async_submit(c->a, data, len, 0, rx_done, e)) {
		/* refused (context error or no GPU): host routine now */
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
	free(e);
	return rc;
}

unsigned int crc32c_msgr_rx_pending(const struct crc32c_msgr_conn *c)
{
	return c ? c->npending : 0u;
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
			c->release(e->msg);
			g_st.rx_released++;
			free(e);
		}
	}
	c->head = c->tail = NULL;
	c->npending = 0;
}

/* ---- send ------------------------------------------------------------- */

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

static struct tx_ent *tx_find(struct crc32c_msgr_conn *c, void *msg, struct tx_ent ***link)
{
	struct tx_ent **pp;

	for (pp = &c->tx; *pp; pp = &(*pp)->next)
		if ((*pp)->msg == msg) {
			if (link)
				*link = pp;
			return *pp;
		}
	return NULL;
}

static struct tx_ent *tx_new(struct crc32c_msgr_conn *c, void *msg)
{
	struct tx_ent *e = calloc(1, sizeof(*e)), **pp;

	if (!e)
		return NULL;
	e->conn = c;
	e->release = c->release;
	e->msg = msg;
	for (pp = &c->tx; *pp; pp = &(*pp)->next) /* send order */
		;
	*pp = e;
	return e;
}

int crc32c_msgr_tx_submit(struct crc32c_msgr_conn *c, void *msg, const void *data, unsigned int len, uint32_t seed)
{
	struct tx_ent *e;

	if (!c || (len && !data))
		return -EINVAL;
	if (tx_find(c, msg, NULL))
		return 0; /* resend: the bytes and so the CRC are unchanged */
	e = tx_new(c, msg);
	if (!e)
		return -ENOMEM;
	e->data = data;
	e->len = len;
	e->seed = seed;
	e->state = ST_WAIT;
	g_st.tx_submitted++;
	if (crc32c_async_submit(c->a, data, len, seed, tx_done, e)) {
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
	if (tx_find(c, msg, NULL))
		return 0;
	e = tx_new(c, msg);
	if (!e)
		return -ENOMEM;
	e->crc = crc;
	e->state = ST_DONE;
	g_st.tx_known++;
	return 0;
}

int crc32c_msgr_tx_footer(struct crc32c_msgr_conn *c, void *msg, uint32_t *crc)
{
	struct tx_ent **link = NULL, *e;

	if (!c || !crc)
		return -EINVAL;
	e = tx_find(c, msg, &link);
	if (!e)
		return -ENOENT;
	if (e->state != ST_DONE) {
		if (!e->waiting)
			g_st.tx_held++;
		e->waiting = 1;
		return 0;
	}
	*crc = e->crc;
	*link = e->next;
	free(e);
	return 1;
}

void crc32c_msgr_conn_destroy(struct crc32c_msgr_conn *c)
{
	struct tx_ent *e, *n;

	if (!c)
		return;
	crc32c_msgr_conn_reset(c);
	for (e = c->tx; e; e = n) {
		n = e->next;
		if (e->state == ST_WAIT) {
			e->conn = NULL; /* the GPU still reads its bytes: released in tx_done */
		} else {
			c->release(e->msg);
			g_st.tx_released++;
			free(e);
		}
	}
	free(c);
}

void crc32c_msgr_get_stats(struct crc32c_msgr_stats *st)
{
	if (st)
		*st = g_st;
}
