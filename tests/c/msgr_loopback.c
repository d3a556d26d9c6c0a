/*
 * msgr_loopback.c -- TEST PROGRAM: the reference messenger ITSELF, patched
 * by integration/pech_crc32c_msgr.patch, carrying OSD_OP-shaped messages
 * over 127.0.0.1 between two ceph_messengers of one pech process.
 *
 * Nothing here restates the messenger: this file is only the caller.  It is
 * linked with every src/ and src/ceph/ object of pech (temp patched copies
 * of messenger.c / messenger.h / osd_server.c, compiled with the reference
 * CFLAGS by tests/pech_build.py; no reference source is kept in this repo)
 * and with libpech_crc32c.so, and it starts pech's runtime the way
 * src/main.c:228-273 does: pages, scheduler, event loop, workqueues,
 * modules (init_ceph_lib -> ceph_msgr_init, which the patch makes create the
 * async CRC context), then one task.  Without a usable GPU that context is
 * NULL and every connection checksums inline, as before the patch: the same
 * binary then runs the reference's own path (build container).
 *
 * The task (lb_task):
 *   - a "server" messenger listening on 0.0.0.0:<ephemeral>
 *     (messenger.c:3431 ceph_messenger_init, :3568 start_listen) with
 *     osd_server-like con ops (alloc_con/accept_con/get/put, alloc_msg with
 *     ONE contiguous bvec of ceph_msg_data_pages_alloc() pages as
 *     alloc_msg_with_bvec does (osd_server.c:2317), dispatch, fault = close
 *     + put as osds_fault (osd_server.c:2397));
 *   - a "client" messenger whose connection (:809 ceph_con_init, :777
 *     ceph_con_open) goes through tests/c/loopback_proxy.c, a TCP relay
 *     that can flip one bit of one chosen message on the wire; its fault op
 *     reopens the connection and resends every unanswered request, as the
 *     osd client does (osd_client.c:4030 osd_fault -> reopen_osd,
 *     kick_osd_requests);
 *   - requests (CEPH_MSG_OSD_OP) with 4 KiB .. 4 MiB data (:3709
 *     ceph_con_send), interleaved with CEPH_MSG_PING that the server's
 *     alloc_msg skips (the verify queue's in-order markers); the server
 *     answers each request with a CEPH_MSG_OSD_OPREPLY of the same data
 *     size, so payload CRCs run in both directions.
 * Checks (exit 0 iff all hold; one JSON line on stdout either way):
 *   - every request dispatched by the server, every reply by the client,
 *     with the exact bytes sent (a corrupted message is never dispatched);
 *   - per connection, requests dispatched in send order, none twice;
 *     without injected faults, each exactly once overall;
 *   - every received data footer equals the oracle's per-4 KiB-piece chain
 *     of the bytes (oracle/crc32c_oracle.c, the reference loop), or carries
 *     CEPH_MSG_FOOTER_NOCRC in the nocrc scenario;
 *   - every ceph_msg allocated (both sides, both directions, skipped and
 *     revoked ones included) is freed by teardown, after ceph_msgr_exit()
 *     has drained the async context;
 *   - with --expect-gpu: the adapter's counters show GPU submissions on
 *     both sides (payloads above its 8 KiB host cutoff), and none in nocrc;
 *   - with --expect-contexts N: the patch created N async contexts (one per
 *     entry of PECH_DEVICES, e.g. "0,0": two on one GPU) and, unless nocrc,
 *     every one of them took submissions -- the connections are spread
 *     over them (recorded by wrapping crc32c_async_create_on).
 *
 * Scenarios (argv[1]): basic | corrupt-req | corrupt-reply | revoke | nocrc
 */
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "types.h"
#include "sched.h"
#include "timer.h"
#include "event.h"
#include "workqueue.h"
#include "timedef.h"
#include "err.h"
#include "module.h"
#include "printk.h"
#include "page.h"
#include "slab.h"
#include "kref.h"
#include "getorder.h"
#include "net.h"

#include "ceph/libceph.h"
#include "ceph/messenger.h"
#include "ceph/ceph_features.h"

#include "pech_crc32c.h"
#include "pech_crc32c_msgr.h"
#include "loopback_proxy.h"

/* the test oracle (oracle/crc32c_oracle.c): reference loop, per-piece chain */
uint32_t oracle_crc32c_pieces(uint32_t crc, const void *data, size_t length, unsigned int piece);

#define LB_MAGIC 0x4c425054u /* front magic */
#define MAX_REQ 512
#define MARK_OFF 2048u      /* where a message's flip mark sits in its data */
#define DEADLINE_MS 90000

struct lb_front {
	__le32 magic, idx, len, dir;
	u8 pad[48];
};

struct lb_req {
	struct ceph_msg *m; /* our reference, until teardown */
	unsigned int len;
	int replied, revoked;
	int srv_seen;       /* dispatches by the server, over all connections */
	int srv_gen;        /* server connection of the last dispatch */
};

struct lb_srv_con {
	struct ceph_connection con;
	struct kref ref;
	int gen;
	int last_idx; /* dispatch order on this connection */
};

static struct {
	const char *scenario;
	int expect_gpu, nocrc, expect_ctx;
	struct crc32c_async *ctx[16]; /* the patch's async contexts, in creation order */
	int nctx;
	struct ceph_options *opt;
	struct ceph_messenger srv, cli;
	struct ceph_connection ccon;
	struct ceph_entity_addr peer; /* the server, reached through the relay */
	struct lb_req req[MAX_REQ];
	int nreq, stopping;
	int srv_gen, srv_live;
	long msgs_alloc, msgs_freed;
	int srv_dispatched, srv_dups, cli_dispatched, cli_dups;
	int srv_faults, cli_faults, cli_resent, pings;
	int bad_bytes, bad_footer, bad_order, bad_front;
	long revoke_polls, revoke_out_seen; /* revoke: polls of con->out_msg, distinct messages seen in it */
	struct ceph_msg *revoke_target;     /* revoke: the message to revoke mid-send */
	int revoke_queued, revoked_held;
	int revoke_armed;                   /* revoke: the target's send is held (below) until it is revoked */
	long held_writes, held_completes;   /* revoke: data writes / complete() calls held back */
	struct work_struct revoke_work;
	int ret;
} S;

static u64 mix(u64 x)
{
	x += 0x9E3779B97F4A7C15ull;
	x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
	x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
	return x ^ (x >> 31);
}

/* the data of message idx in direction dir: a byte stream of its own, with
 * the relay's flip mark at MARK_OFF when it has room for it */
static void lb_fill(u8 *p, unsigned int len, unsigned int idx, int dir)
{
	u64 s = mix(((u64)idx << 1) | (u64)dir), v = 0;
	unsigned int i;

	for (i = 0; i < len; i++) {
		if ((i & 7) == 0)
			v = s = mix(s);
		p[i] = (u8)(v >> (8 * (i & 7)));
	}
	if (len >= MARK_OFF + LB_MARK_BYTES + 256)
		lb_mark(p + MARK_OFF, dir, idx);
}

static int lb_check(const u8 *p, unsigned int len, unsigned int idx, int dir)
{
	u8 *want = malloc(len ? len : 1);
	int ok;

	lb_fill(want, len, idx, dir);
	ok = !memcmp(want, p, len);
	free(want);
	return ok;
}

static void lb_free_msg(struct ceph_msg *m)
{
	S.msgs_freed++;
}

/* ONE contiguous bvec of 2^order pages, as alloc_bvec (osd_server.c:187);
 * the patch's allocator hands out pinned, GPU-mapped pages.  The order is
 * passed as alloc_bvec passes it, from pech's get_order() (32 + the order
 * above one page, see the patch's msg_data_order); the bvec's length comes
 * from the true order. */
static int lb_add_data(struct ceph_msg *m, unsigned int len)
{
	struct ceph_bvec_iter it;
	struct bio_vec *bv;
	unsigned int order = 0;
	struct page *pg = ceph_msg_data_pages_alloc(get_order(len));

	while ((PAGE_SIZE << order) < len)
		order++;
	if (!pg)
		return -ENOMEM;
	bv = kmalloc(sizeof(*bv), GFP_KERNEL);
	if (!bv) {
		ceph_msg_data_pages_free(pg, order);
		return -ENOMEM;
	}
	bv->bv_page = pg;
	bv->bv_len = PAGE_SIZE << order;
	bv->bv_offset = 0;
	memset(&it, 0, sizeof(it));
	it.bvecs = bv;
	it.iter.bi_size = len;
	ceph_msg_data_add_bvecs(m, &it, 1, true);
	return 0;
}

static u8 *lb_data(struct ceph_msg *m)
{
	return page_address(m->data[0].bvec_pos.bvecs[0].bv_page) + m->data[0].bvec_pos.bvecs[0].bv_offset;
}

static struct ceph_msg *lb_new(int type, unsigned int idx, unsigned int len, int dir)
{
	struct ceph_msg *m = ceph_msg_new2(type, sizeof(struct lb_front), 1, GFP_KERNEL, false);
	struct lb_front *f;

	BUG_ON(!m);
	S.msgs_alloc++;
	m->free_msg = lb_free_msg;
	f = m->front.iov_base;
	memset(f, 0, sizeof(*f));
	f->magic = cpu_to_le32(LB_MAGIC);
	f->idx = cpu_to_le32(idx);
	f->len = cpu_to_le32(len);
	f->dir = cpu_to_le32(dir);
	if (len) {
		BUG_ON(lb_add_data(m, len));
		m->hdr.data_len = cpu_to_le32(len);
		lb_fill(lb_data(m), len, idx, dir);
	}
	return m;
}

/* a received message: front, bytes and footer against what was sent */
static int lb_verify(struct ceph_msg *m, int type, int dir, unsigned int *idx)
{
	const struct lb_front *f = m->front.iov_base;
	unsigned int len;

	if (le16_to_cpu(m->hdr.type) != type || m->front.iov_len != sizeof(*f) || le32_to_cpu(f->magic) != LB_MAGIC ||
	    le32_to_cpu(f->dir) != dir || le32_to_cpu(f->idx) >= (u32)S.nreq) {
		S.bad_front++;
		return -1;
	}
	*idx = le32_to_cpu(f->idx);
	len = le32_to_cpu(f->len);
	if (len != m->data_length || len != S.req[*idx].len) {
		S.bad_front++;
		return -1;
	}
	if (!len)
		return 0;
	if (!lb_check(lb_data(m), len, *idx, dir)) {
		S.bad_bytes++;
		return -1;
	}
	if (S.nocrc) {
		if (!(m->footer.flags & CEPH_MSG_FOOTER_NOCRC))
			S.bad_footer++;
	} else if (le32_to_cpu(m->footer.data_crc) != oracle_crc32c_pieces(0, lb_data(m), len, PAGE_SIZE)) {
		S.bad_footer++;
		return -1;
	}
	return 0;
}

/* ---- message allocation for both sides (alloc_msg_with_bvec) ---------- */
static struct ceph_msg *lb_alloc_msg(struct ceph_connection *con, struct ceph_msg_header *hdr, int *skip)
{
	const int type = le16_to_cpu(hdr->type);
	const u32 front_len = le32_to_cpu(hdr->front_len);
	const u32 data_len = le32_to_cpu(hdr->data_len);
	struct ceph_msg *m;

	*skip = 0;
	if (type == CEPH_MSG_PING) { /* osds_alloc_msg: skipped (osd_server.c:2367) */
		*skip = 1;
		return NULL;
	}
	m = ceph_msg_new2(type, front_len, 1, GFP_KERNEL, false);
	if (!m)
		return NULL;
	S.msgs_alloc++;
	if (data_len && lb_add_data(m, data_len)) {
		ceph_msg_put(m);
		return NULL;
	}
	return m;
}

/* ---- server side (osd_server.c:389-444, :2397) ------------------------- */
static struct lb_srv_con *to_srv(struct ceph_connection *con)
{
	return container_of(con, struct lb_srv_con, con);
}

static void srv_release(struct kref *ref)
{
	kfree(container_of(ref, struct lb_srv_con, ref));
	S.srv_live--;
}

static struct ceph_connection *srv_get(struct ceph_connection *con)
{
	kref_get(&to_srv(con)->ref);
	return con;
}

static void srv_put(struct ceph_connection *con)
{
	kref_put(&to_srv(con)->ref, srv_release);
}

static struct ceph_connection *srv_alloc_con(struct ceph_messenger *msgr)
{
	struct lb_srv_con *sc = kzalloc(sizeof(*sc), GFP_KERNEL);

	if (!sc)
		return NULL;
	kref_init(&sc->ref);
	sc->gen = ++S.srv_gen;
	sc->last_idx = -1;
	S.srv_live++;
	return &sc->con;
}

static int srv_accept_con(struct ceph_connection *con)
{
	return 0;
}

static void srv_dispatch(struct ceph_connection *con, struct ceph_msg *m)
{
	struct lb_srv_con *sc = to_srv(con);
	struct lb_req *r;
	unsigned int idx;

	if (lb_verify(m, CEPH_MSG_OSD_OP, LB_C2S, &idx) == 0) {
		r = &S.req[idx];
		if ((int)idx <= sc->last_idx || r->srv_gen == sc->gen)
			S.bad_order++; /* out of order, or twice on one connection */
		sc->last_idx = idx;
		if (r->srv_seen++)
			S.srv_dups++; /* a resend after a fault (osd_fault semantics) */
		r->srv_gen = sc->gen;
		S.srv_dispatched++;
		ceph_con_send(con, lb_new(CEPH_MSG_OSD_OPREPLY, idx, r->len, LB_S2C));
	}
	ceph_msg_put(m);
}

static void srv_fault(struct ceph_connection *con)
{
	S.srv_faults++;
	ceph_con_close(con);
	srv_put(con); /* the accept reference (osds_fault) */
}

static const struct ceph_connection_operations srv_ops = {
	.alloc_con = srv_alloc_con,
	.accept_con = srv_accept_con,
	.get = srv_get,
	.put = srv_put,
	.dispatch = srv_dispatch,
	.fault = srv_fault,
	.alloc_msg = lb_alloc_msg,
	.free_msg = lb_free_msg,
};

/* ---- client side (osd_client.c:4030 osd_fault) ------------------------- */
static struct ceph_connection *cli_get(struct ceph_connection *con)
{
	return con;
}

static void cli_put(struct ceph_connection *con)
{
}

static void cli_send(unsigned int i)
{
	ceph_con_send(&S.ccon, ceph_msg_get(S.req[i].m));
}

static void cli_dispatch(struct ceph_connection *con, struct ceph_msg *m)
{
	unsigned int idx;

	if (lb_verify(m, CEPH_MSG_OSD_OPREPLY, LB_S2C, &idx) == 0) {
		if (S.req[idx].replied++)
			S.cli_dups++;
		S.cli_dispatched++;
	}
	ceph_msg_put(m);
}

static void cli_fault(struct ceph_connection *con)
{
	int i;

	S.cli_faults++;
	if (S.stopping)
		return;
	/* reopen_osd + kick_osd_requests: a fresh session, every unanswered
	 * request sent again with new seqs */
	ceph_con_close(con);
	ceph_con_open(con, CEPH_ENTITY_TYPE_OSD, 0, &S.peer);
	for (i = 0; i < S.nreq; i++)
		if (!S.req[i].replied && !S.req[i].revoked) {
			cli_send(i);
			S.cli_resent++;
		}
}

static const struct ceph_connection_operations cli_ops = {
	.get = cli_get,
	.put = cli_put,
	.dispatch = cli_dispatch,
	.fault = cli_fault,
	.alloc_msg = lb_alloc_msg,
	.free_msg = lb_free_msg,
};

/* ---- revoke while the footer is held ------------------------------------
 * The link wraps the patched messenger's call of crc32c_msgr_tx_footer()
 * (-Wl,--wrap, tests/pech_build.py): when the revoke target's footer is held
 * for its GPU CRC, a work item is queued that revokes it as soon as the
 * connection's work function has let go of the mutex -- before the CRC
 * lands and the connection is kicked (a poll from the test task could miss
 * that window: the worker runs queued work back to back).  Inline (no GPU)
 * there is no held footer; the test task's poll of con->out_msg catches the
 * message between socket writes instead. */
int __real_crc32c_msgr_tx_footer(struct crc32c_msgr_conn *c, void *msg, uint32_t *crc);

int __wrap_crc32c_msgr_tx_footer(struct crc32c_msgr_conn *c, void *msg, uint32_t *crc)
{
	const int ret = __real_crc32c_msgr_tx_footer(c, msg, crc);

	if (ret == 0 && msg && msg == S.revoke_target && !S.revoke_queued) {
		S.revoke_queued = 1;
		queue_work(system_wq, &S.revoke_work);
	}
	return ret;
}

/* every async context the patch creates (crc_ctx_init: one per device) */
struct crc32c_async *__real_crc32c_async_create_on(int device, unsigned int flags);

struct crc32c_async *__wrap_crc32c_async_create_on(int device, unsigned int flags)
{
	struct crc32c_async *a = __real_crc32c_async_create_on(device, flags);

	if (a && S.nctx < (int)ARRAY_SIZE(S.ctx))
		S.ctx[S.nctx++] = a;
	return a;
}

/* ---- the target held in place until it is revoked ------
 * The revoke must land while the target is being sent; a poll racing the
 * socket writes could miss that window on a loaded host.  So the harness
 * holds the send itself:
 *   inline (no async context): the client socket's writes of the target's
 *   data report a full socket (-EAGAIN: ceph_tcp_sendiov returns 0 and the
 *   messenger waits for write space) while it is con->out_msg and not yet
 *   revoked, its header and front already sent -- the poll below always
 *   finds it there;
 *   adapter (async contexts): complete() delivers nothing while the target
 *   is con->out_msg and not yet revoked, so its GPU CRC cannot be ready at
 *   its footer -- the footer is held (tx_footer returns 0) and the work
 *   item above revokes it there.
 * Both end with the revoke; the hold cannot outlive it. */
static int lb_holding(void)
{
	int i;

	if (!S.revoke_armed || !S.revoke_target || S.ccon.out_msg != S.revoke_target)
		return 0;
	for (i = 0; i < S.nreq; i++)
		if (S.req[i].m == S.revoke_target)
			return !S.req[i].revoked;
	return 0;
}

int __real_sock_sendmsg(struct socket *sock, struct kmsghdr *kmsg);

/* the messenger's socket writes; held: the target's data pages
 * (ceph_tcp_sendiov over the bvec, write_partial_message_data), once its
 * header and front are on the wire */
int __wrap_sock_sendmsg(struct socket *sock, struct kmsghdr *kmsg)
{
	if (S.nctx == 0 && sock == S.ccon.sock && iov_iter_is_bvec(&kmsg->msg_iter) && lb_holding()) {
		S.held_writes++;
		return -EAGAIN;
	}
	return __real_sock_sendmsg(sock, kmsg);
}

int __real_crc32c_async_complete(struct crc32c_async *a);

int __wrap_crc32c_async_complete(struct crc32c_async *a)
{
	if (S.nctx > 0 && lb_holding()) {
		S.held_completes++;
		return 0;
	}
	return __real_crc32c_async_complete(a);
}

static void revoke_workfn(struct work_struct *w)
{
	struct lb_req *r;
	int i;

	for (i = 0; i < S.nreq; i++) {
		r = &S.req[i];
		if (r->m == S.revoke_target && S.ccon.out_msg == r->m && !r->revoked && !r->srv_seen) {
			r->revoked = 1;
			ceph_msg_revoke(r->m);
			S.revoked_held = 1;
		}
	}
}

/* ---- the scenario task -------------------------------------------------- */
static int all_answered(void)
{
	int i;

	for (i = 0; i < S.nreq; i++)
		if (!S.req[i].replied && !S.req[i].revoked)
			return 0;
	return 1;
}

static void send_ping(void)
{
	struct ceph_msg *p = ceph_msg_new2(CEPH_MSG_PING, 0, 0, GFP_KERNEL, false);

	BUG_ON(!p);
	S.msgs_alloc++;
	p->free_msg = lb_free_msg;
	ceph_con_send(&S.ccon, p);
	S.pings++;
}

static const unsigned int sizes[] = {
	4096, 65536, 1u << 20, 4u << 20, 4100, 100000, 8192, 16384, 12288, 300001, 2u << 20, 32768,
};

static int lb_task(void *arg)
{
	struct ceph_entity_addr myaddr;
	struct sockaddr_storage ss;
	struct sockaddr_in *sin;
	struct crc32c_msgr_stats st;
	struct crc32c_async_stats cst[16];
	u16 srv_port, relay_port;
	int i, ret, corrupt_idx = -1, revoke_idx = -1, revoked_mid = 0;
	struct ceph_msg *last_out = NULL;
	unsigned long deadline;

	S.opt = ceph_alloc_options();
	BUG_ON(!S.opt);
	if (S.nocrc)
		ceph_set_opt(S.opt, NO_DATA_CRC);

	/* server: 0.0.0.0 so the client accepts its banner through the relay
	 * (process_banner_on_client: a blank address with the same nonce) */
	memset(&myaddr, 0, sizeof(myaddr));
	myaddr.type = CEPH_ENTITY_ADDR_TYPE_LEGACY;
	memset(&ss, 0, sizeof(ss));
	sin = (struct sockaddr_in *)&ss;
	sin->sin_family = AF_INET;
	sin->sin_addr.s_addr = htonl(INADDR_ANY);
	memcpy(&myaddr.in_addr, &ss, sizeof(ss)); /* a packed member: no pointer into it */
	ceph_messenger_init(&S.srv, &myaddr, CEPH_ENTITY_TYPE_OSD, 0, S.opt, CEPH_FEATURES_SUPPORTED_DEFAULT,
			    CEPH_FEATURES_REQUIRED_DEFAULT);
	ret = ceph_messenger_start_listen(&S.srv, &srv_ops);
	BUG_ON(ret);
	memcpy(&ss, &S.srv.inst.addr.in_addr, sizeof(ss));
	srv_port = sin->sin_port;
	ret = lb_proxy_start(srv_port, &relay_port);
	BUG_ON(ret);

	ceph_messenger_init(&S.cli, NULL, CEPH_ENTITY_TYPE_CLIENT, 4242, S.opt, CEPH_FEATURES_SUPPORTED_DEFAULT,
			    CEPH_FEATURES_REQUIRED_DEFAULT);
	S.peer = S.srv.inst.addr;
	sin->sin_addr.s_addr = htonl(INADDR_LOOPBACK);
	sin->sin_port = relay_port;
	memcpy(&S.peer.in_addr, &ss, sizeof(ss));
	ceph_con_init(&S.ccon, NULL, &cli_ops, &S.cli);
	ceph_con_open(&S.ccon, CEPH_ENTITY_TYPE_OSD, 0, &S.peer);

	/* the requests: the size mix, then a burst of 16 KiB ones (verify
	 * queue depth), or fewer, larger ones for the revoke case */
	if (!strcmp(S.scenario, "revoke")) {
		S.nreq = 16;
		for (i = 0; i < S.nreq; i++)
			S.req[i].len = i % 4 == 1 ? 4u << 20 : sizes[i % 3];
		revoke_idx = 5;
	} else {
		S.nreq = 3 * (int)ARRAY_SIZE(sizes) + 160;
		for (i = 0; i < S.nreq; i++)
			S.req[i].len = i < 3 * (int)ARRAY_SIZE(sizes) ? sizes[i % ARRAY_SIZE(sizes)] : 16384u;
		S.req[7].len = 0; /* a message without data */
	}
	if (!strcmp(S.scenario, "corrupt-req")) {
		corrupt_idx = 13; /* 64 KiB */
		lb_proxy_arm(LB_C2S, corrupt_idx);
	} else if (!strcmp(S.scenario, "corrupt-reply")) {
		corrupt_idx = 15; /* 4 MiB */
		lb_proxy_arm(LB_S2C, corrupt_idx);
	}
	for (i = 0; i < S.nreq; i++)
		S.req[i].m = lb_new(CEPH_MSG_OSD_OP, i, S.req[i].len, LB_C2S);
	for (i = 0; i < S.nreq; i++) {
		cli_send(i);
		if (i % 5 == 2)
			send_ping();
	}

	deadline = jiffies + msecs_to_jiffies(DEADLINE_MS);
	if (revoke_idx >= 0) {
		/* the last request is revoked while still queued (nothing has run
		 * since ceph_con_open): taken off out_queue, never sent */
		S.req[S.nreq - 1].revoked = 1;
		ceph_msg_revoke(S.req[S.nreq - 1].m);
		INIT_WORK(&S.revoke_work, revoke_workfn);
		S.revoke_target = S.req[revoke_idx].m;
		/* revoke_idx while it is being written (con->out_msg: its data on
		 * the wire, or its footer held for the GPU CRC): the rest goes out
		 * as zeros (write_partial_skip), the server faults on it, and the
		 * client reconnects and resends everything else.  The harness holds
		 * the target's send until then (lb_holding), so the revoke always
		 * lands mid-send: inline from this poll, with the adapter from the
		 * held footer's work item (this poll leaves that case to it). */
		S.revoke_armed = 1;
		while (!revoked_mid && !S.revoked_held && time_before(jiffies, deadline) &&
		       !S.req[revoke_idx].srv_seen && !S.req[revoke_idx].replied) {
			S.revoke_polls++;
			if (S.ccon.out_msg && S.ccon.out_msg != last_out) {
				last_out = S.ccon.out_msg;
				S.revoke_out_seen++;
			}
			if (S.nctx == 0 && S.ccon.out_msg == S.req[revoke_idx].m) {
				S.req[revoke_idx].revoked = 1;
				ceph_msg_revoke(S.req[revoke_idx].m);
				revoked_mid = 1;
			}
			schedule();
		}
		revoked_mid |= S.revoked_held;
	}
	while (!all_answered() && time_before(jiffies, deadline))
		msleep(2);

	/* teardown: close the client, wait for the server side to see it */
	S.stopping = 1;
	ceph_con_close(&S.ccon);
	deadline = jiffies + msecs_to_jiffies(10000);
	while (S.srv_live && time_before(jiffies, deadline))
		msleep(2);
	ceph_messenger_stop_listen(&S.srv);
	lb_proxy_stop();
	for (i = 0; i < S.nreq; i++)
		ceph_msg_put(S.req[i].m);
	crc32c_msgr_get_stats(&st);
	for (i = 0; i < S.nctx; i++)
		crc32c_async_get_stats(S.ctx[i], &cst[i]);
	/* the patch's _ceph_msgr_exit: the async context is destroyed first
	 * (drained: orphaned CRCs land and release their messages) */
	ceph_msgr_exit();

	/* checks */
	{
		int unanswered = 0, seen_once = 1, ok;
		const int faults_expected = corrupt_idx >= 0 || revoke_idx >= 0;
		const u64 gpu_sub = st.rx_submitted + st.tx_submitted;

		for (i = 0; i < S.nreq; i++) {
			if (!S.req[i].revoked && (!S.req[i].replied || !S.req[i].srv_seen))
				unanswered++;
			if (S.req[i].revoked && (S.req[i].srv_seen || S.req[i].replied))
				unanswered++; /* a revoked message must never arrive */
			if (S.req[i].srv_seen != 1 || S.req[i].replied != 1)
				seen_once = 0;
		}
		ok = !unanswered && !S.bad_bytes && !S.bad_footer && !S.bad_order && !S.bad_front &&
		     S.msgs_alloc == S.msgs_freed && S.srv_live == 0 && (faults_expected || seen_once) &&
		     (!faults_expected || S.srv_faults + S.cli_faults > 0) &&
		     (corrupt_idx < 0 || lb_proxy_flips() == 1) && (revoke_idx < 0 || revoked_mid);
		if (S.expect_gpu)
			ok = ok && (S.nocrc ? gpu_sub == 0 : st.rx_submitted > 0 && st.tx_submitted > 0) &&
			     (corrupt_idx < 0 || st.rx_bad >= 1);
		if (S.expect_ctx) {
			ok = ok && S.nctx == S.expect_ctx;
			for (i = 0; i < S.nctx; i++)
				ok = ok && (S.nocrc ? cst[i].submitted == 0 : cst[i].submitted > 0);
		}
		printf("{\"contexts\": [");
		for (i = 0; i < S.nctx; i++)
			printf("%s{\"device\": %d, \"submitted\": %llu, \"launches\": %llu}", i ? ", " : "", cst[i].device,
			       (unsigned long long)cst[i].submitted, (unsigned long long)cst[i].launches);
		printf("]}\n");
		printf("{\"scenario\": \"%s\", \"ok\": %s, \"requests\": %d, \"unanswered\": %d, \"revoked_mid_send\": %d, "
		       "\"revoked_footer_held\": %d, "
		       "\"srv_dispatched\": %d, \"srv_dups\": %d, \"cli_dispatched\": %d, \"cli_dups\": %d, "
		       "\"pings_skipped\": %d, \"srv_faults\": %d, \"cli_faults\": %d, \"cli_resent\": %d, "
		       "\"revoke_polls\": %ld, \"revoke_out_seen\": %ld, \"held_writes\": %ld, \"held_completes\": %ld, "
		       "\"relay_conns\": %d, \"relay_flips\": %d, \"bad_bytes\": %d, \"bad_footer\": %d, "
		       "\"bad_order\": %d, \"bad_front\": %d, \"msgs_alloc\": %ld, \"msgs_freed\": %ld, "
		       "\"adapter\": {\"rx_submitted\": %llu, \"rx_host\": %llu, \"rx_unchecked\": %llu, "
		       "\"rx_verified\": %llu, \"rx_bad\": %llu, \"rx_released\": %llu, \"tx_submitted\": %llu, "
		       "\"tx_host\": %llu, \"tx_held\": %llu, \"tx_released\": %llu}}\n",
		       S.scenario, ok ? "true" : "false", S.nreq, unanswered, revoked_mid, S.revoked_held, S.srv_dispatched,
		       S.srv_dups,
		       S.cli_dispatched, S.cli_dups, S.pings, S.srv_faults, S.cli_faults, S.cli_resent,
		       S.revoke_polls, S.revoke_out_seen, S.held_writes, S.held_completes, lb_proxy_conns(), lb_proxy_flips(), S.bad_bytes, S.bad_footer, S.bad_order, S.bad_front,
		       S.msgs_alloc, S.msgs_freed, (unsigned long long)st.rx_submitted,
		       (unsigned long long)st.rx_host, (unsigned long long)st.rx_unchecked,
		       (unsigned long long)st.rx_verified, (unsigned long long)st.rx_bad,
		       (unsigned long long)st.rx_released, (unsigned long long)st.tx_submitted,
		       (unsigned long long)st.tx_host, (unsigned long long)st.tx_held,
		       (unsigned long long)st.tx_released);
		S.ret = ok ? 0 : 1;
	}
	ceph_destroy_options(S.opt);
	deinit_workqueue();
	deinit_event();
	return 0;
}

/* a BUG_ON() aborts: name where (the binary links with -rdynamic) */
static void on_abort(int sig)
{
	void *bt[64];
	int n = backtrace(bt, 64);

	backtrace_symbols_fd(bt, n, 2);
	signal(sig, SIG_DFL);
	raise(sig);
}

int main(int argc, char **argv)
{
	struct task_struct *task;
	int i;

	if (argc < 2) {
		fprintf(stderr, "usage: %s basic|corrupt-req|corrupt-reply|revoke|nocrc [--expect-gpu] [--expect-contexts N]\n",
			argv[0]);
		return 2;
	}
	memset(&S, 0, sizeof(S));
	S.scenario = argv[1];
	S.nocrc = !strcmp(S.scenario, "nocrc");
	for (i = 2; i < argc; i++)
		if (!strcmp(argv[i], "--expect-gpu"))
			S.expect_gpu = 1;
		else if (!strcmp(argv[i], "--expect-contexts") && i + 1 < argc)
			S.expect_ctx = atoi(argv[++i]);
	setvbuf(stdout, NULL, _IONBF, 0);
	signal(SIGABRT, on_abort);
	signal(SIGSEGV, on_abort);
	{
		/* pech's main blocks every signal (main.c:176 init_signals): a
		 * write to a socket the peer closed fails with EPIPE, it does not
		 * kill the process -- for the relay's thread as well */
		sigset_t set;

		sigemptyset(&set);
		sigaddset(&set, SIGPIPE);
		sigprocmask(SIG_BLOCK, &set, NULL);
	}
	S.ret = 1;

	/* src/main.c:228-237 */
	init_formatting();
	init_pages();
	init_sched();
	init_event();
	init_workqueue();
	init_modules(); /* init_ceph_lib -> ceph_msgr_init -> the patch's crc_ctx_init */

	task = task_create(lb_task, NULL);
	BUG_ON(!task);
	wake_up_process(task);
	while (tasks_to_run())
		schedule();
	deinit_pages();
	return S.ret;
}
