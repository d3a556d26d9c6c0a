/*
 * pech_crc32c_msgr.h -- the messenger-side adapter of libpech_crc32c.so:
 * GPU data CRCs that keep the messenger's sequencing and ack semantics.
 *
 * The async layer (pech_crc32c_async.h) completes payload CRCs later, on the
 * epoll loop.  The messenger cannot simply "verify in the callback":
 *  - process_message() consumes con->in_msg and bumps in_seq
 *    (/root/reference/src/ceph/messenger.c:2858-2869), and
 *    prepare_read_message() requires in_msg == NULL (:1882), so the next
 *    message cannot be read while one waits in in_msg;
 *  - in_seq is what prepare_write_ack() acknowledges (:1444-1454, :3013):
 *    acking a message whose data CRC has not been checked yet would let the
 *    peer drop it, and a later mismatch (:2838-2842) would lose it;
 *  - the footer goes on the wire after the data (:1793-1798), so the send
 *    side needs the CRC by the time the last data byte is written.
 * This adapter gives each connection
 *  RECEIVE: a verify queue.  When a message's footer has been read the
 *    messenger detaches it from in_msg into the queue (crc32c_msgr_rx_queue:
 *    the GPU CRC is submitted there), keeps reading, and dispatches from the
 *    queue head in arrival order (crc32c_msgr_rx_next) -- in_seq, and so the
 *    ack, advances only for verified messages.  A mismatch at the head is
 *    reported as -EBADMSG: the connection faults exactly as today, the peer
 *    resends everything unacked, and crc32c_msgr_conn_reset() drops the
 *    queue (buffers still being read by the GPU are released when their CRC
 *    completes, never before).
 *  SEND: the data CRC is submitted when the message is prepared
 *    (prepare_write_message, :1345-1439), before its first byte is sent, and
 *    collected at the footer (crc32c_msgr_tx_footer); if it is not ready the
 *    connection holds the footer and is kicked when it is.  A CRC known
 *    without a data pass -- the REPOP fan-out (osd_server.c:1119, :1972)
 *    forwards the verified request data to every replica -- is registered
 *    with crc32c_msgr_tx_known(): no GPU work per replica.
 * The option gates stay in the messenger (CEPH_OPT_NO_DATA_CRC, libceph.h:36):
 * with data CRCs off it passes check = 0 / never submits, and sets
 * CEPH_MSG_FOOTER_NOCRC as today.
 *
 * Ownership: every message handed to the adapter (rx_queue, tx_submit,
 * tx_known) comes back exactly once -- from rx_next, from tx_footer (1), or
 * through release() -- and its data must stay valid and unchanged until then.
 * GPU failures never reach the messenger: a refused submission or a failed
 * batch is recomputed on the host from the same bytes.
 * Threading: as the async layer -- one caller thread; the kick and release
 * callbacks run inside crc32c_async_complete() on that thread (release also
 * inside reset / cancel / destroy).  The adapter keeps no locks: its
 * connections and counters belong to that thread.
 * Errors: 0 / negative errno (include/err.h style).
 */
#ifndef PECH_CRC32C_MSGR_H
#define PECH_CRC32C_MSGR_H

#include <stdint.h>

#include "pech_crc32c_async.h"

#ifdef __cplusplus
extern "C" {
#endif

struct crc32c_msgr_conn;

/* kick(arg): a queued receive CRC or a held footer's CRC completed -- the
 * messenger queues the connection's work (queue_con, messenger.c).
 * release(msg): the adapter no longer references msg (reset or destroy),
 * the messenger drops its reference (ceph_msg_put). */
typedef void (*crc32c_msgr_kick_fn)(void *arg);
typedef void (*crc32c_msgr_release_fn)(void *msg);

/* A connection's adapter on async context `a` (shared by many connections;
 * results complete in submission order per context).  max_pending bounds
 * the receive queue (backpressure: rx_queue returns -EAGAIN when full). */
struct crc32c_msgr_conn *crc32c_msgr_conn_create(struct crc32c_async *a, unsigned int max_pending,
						 crc32c_msgr_kick_fn kick, void *kick_arg,
						 crc32c_msgr_release_fn release);

/* Fault / reconnect (con_fault): every queued receive message is released
 * (now, or when its in-flight CRC completes); send entries are kept (a
 * resent message reuses its CRC: the bytes are the same). */
void crc32c_msgr_conn_reset(struct crc32c_msgr_conn *c);

/* Reset, release the send entries too (crc32c_msgr_tx_cancel(c, NULL)),
 * free the adapter. */
void crc32c_msgr_conn_destroy(struct crc32c_msgr_conn *c);

/* The async context the connection submits to (NULL for NULL): a messenger
 * with one context per GPU flushes and completes only its connection's
 * after each pass of con_work. */
struct crc32c_async *crc32c_msgr_conn_async(const struct crc32c_msgr_conn *c);

/* Payloads of at most `bytes` (default 8 KiB, or PECH_CRC32C_MSGR_HOST_MAX
 * in the environment) are checksummed at once on the host instead of the
 * GPU: below the crossover the host routine costs less CPU time than the
 * GPU round trip.  Process-wide; returns the previous
 * value.  0 sends every checked payload to the GPU (lone ones too, below). */
unsigned int crc32c_msgr_set_host_max(unsigned int bytes);

/* Payloads of at most `bytes` (default 256 KiB, or PECH_CRC32C_MSGR_LONE_MAX
 * in the environment) that arrive while the connection's async context has
 * nothing outstanding (crc32c_async_pending() == 0: queue depth 1) are
 * checksummed on the host as well: a lone payload cannot share a launch, and
 * up to this size the host routine costs the thread less CPU than the GPU
 * round trip, at a fraction of its latency.  Process-wide;
 * returns the previous value.  0 turns the rule off. */
unsigned int crc32c_msgr_set_lone_max(unsigned int bytes);

/* RECEIVE, at the footer (read_partial_message :2816): queue msg, whose data
 * section is data[0, len).  check != 0 (do_datacrc and the footer has no
 * CEPH_MSG_FOOTER_NOCRC flag): crc32c(0, data, len) is computed (on the GPU,
 * or on the host up to crc32c_msgr_set_host_max()) and compared with
 * footer_crc; otherwise the message is ready at once.  msg may be NULL with
 * check == 0: an in-order marker for a message the messenger skipped, so
 * in_seq still advances in arrival order.  Markers are always taken, and
 * consecutive ones share one entry (a count), so the queue holds at most
 * 2 * max_pending + 1 entries however many messages are skipped while its
 * head waits.  The messenger must not modify or free data until
 * msg is returned by rx_next or released.  0, -EAGAIN (queue full: stop
 * reading, dispatch first), or < 0. */
int crc32c_msgr_rx_queue(struct crc32c_msgr_conn *c, void *msg, const void *data, unsigned int len, int check,
			 uint32_t footer_crc);

/* The queue head, in arrival order:
 *   1        *msg verified (or unchecked); *crc = its data CRC (0 unchecked):
 *            bump in_seq and dispatch it;
 *   0        head not verified yet, or queue empty;
 *   -EBADMSG *msg's data CRC differs from its footer (*crc = computed):
 *            fault the connection ("bad crc", messenger.c:3137-3139).
 * A message returned with 1 or -EBADMSG is no longer the adapter's. */
int crc32c_msgr_rx_next(struct crc32c_msgr_conn *c, void **msg, uint32_t *crc);

/* Messages queued and not yet returned. */
unsigned int crc32c_msgr_rx_pending(const struct crc32c_msgr_conn *c);

/* SEND: submit crc32c(seed, data, len) of outgoing msg (prepare_write_message;
 * seed = footer.data_crc, 0 for a new message).  0: a new entry (the adapter
 * now holds the caller's reference to msg, returned by tx_footer or
 * release); 1: msg already has an entry (resend after a fault, or
 * tx_known): nothing new is taken; < 0 error. */
int crc32c_msgr_tx_submit(struct crc32c_msgr_conn *c, void *msg, const void *data, unsigned int len, uint32_t seed);

/* SEND without a data pass: msg's data CRC is already known (REPOP fan-out:
 * the verified request CRC, or crc32c_concat() of segment CRCs).  Returns
 * as tx_submit. */
int crc32c_msgr_tx_known(struct crc32c_msgr_conn *c, void *msg, uint32_t crc);

/* 1 if msg has a send entry (submitted or known), else 0. */
int crc32c_msgr_tx_has(const struct crc32c_msgr_conn *c, const void *msg);

/* Drop msg's send entry (msg NULL: every send entry of c), for messages the
 * messenger discards unsent: reset_connection drops out_queue/out_sent
 * (messenger.c:724-731), ceph_msg_revoke (:3749).  Each dropped entry's
 * reference comes back through release(): now, or when its in-flight CRC
 * lands.  Returns the number of entries dropped. */
unsigned int crc32c_msgr_tx_cancel(struct crc32c_msgr_conn *c, void *msg);

/* At the end of msg's data (write_partial_message_data :1793): 1 and *crc
 * when ready (the entry is consumed), 0 when still running (hold the footer:
 * kick() fires on completion), -ENOENT no entry for msg. */
int crc32c_msgr_tx_footer(struct crc32c_msgr_conn *c, void *msg, uint32_t *crc);

/* Counters of this adapter (all connections of the process). */
struct crc32c_msgr_stats {
	uint64_t rx_submitted, rx_unchecked, rx_verified, rx_bad, rx_released;
	uint64_t tx_submitted, tx_known, tx_held, tx_released; /* held: footers that had to wait */
	uint64_t rx_host, tx_host; /* checksummed on the host: small payloads, refused submissions */
	uint64_t rx_lone, tx_lone; /* of them: payloads up to crc32c_msgr_set_lone_max() routed to the
	                              host because their context had nothing outstanding */
};
void crc32c_msgr_get_stats(struct crc32c_msgr_stats *st);

#ifdef __cplusplus
}
#endif

#endif /* PECH_CRC32C_MSGR_H */
