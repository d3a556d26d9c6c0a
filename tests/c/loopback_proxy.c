/*
 * loopback_proxy.c -- TEST PROGRAM part of build/msgr_loopback: a TCP relay
 * between the client messenger and the listening one, in its own thread
 * (plain POSIX, none of pech's headers), that can flip one byte of one
 * message's data section on the wire -- a corrupted transmission, which the
 * receiving messenger must catch with its data CRC (-EBADMSG, con_fault) and
 * never dispatch.
 *
 * The message to corrupt is found by content: the test writes a 16-byte mark
 * ("PECHFLIP" + direction + message index + filler) into that message's data
 * (msgr_loopback.c, lb_fill); the relay scans each direction's byte stream
 * for an armed mark, across read boundaries, and flips one bit FLIP_AFTER
 * bytes past it, inside the same data section.  Each armed mark is flipped
 * once: the resend after the fault passes clean.
 */
#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include "loopback_proxy.h"

#define MAX_PAIRS 8
#define BUF_BYTES (256u << 10)
#define FLIP_AFTER 64u

struct side {
	int fd;               /* read from here, write to the other side */
	unsigned long long pos; /* stream offset of the next byte read */
	unsigned char carry[LB_MARK_BYTES - 1]; /* last bytes of the previous read */
	unsigned int ncarry;
	unsigned long long flip_at; /* stream offset to flip, or ~0 */
};

struct pair {
	int live;
	struct side s[2]; /* s[LB_C2S]: client -> server, s[LB_S2C]: server -> client */
};

static struct {
	pthread_t thr;
	int lfd, stopfd;
	struct sockaddr_in target;
	struct pair pairs[MAX_PAIRS];
	pthread_mutex_t mu;
	unsigned char armed[2][LB_MARK_BYTES]; /* per direction: the mark to flip after */
	int arm[2];
	int flips, conns;
} P;

void lb_mark(unsigned char out[LB_MARK_BYTES], int dir, uint32_t idx)
{
	memcpy(out, "PECHFLIP", 8);
	out[8] = (unsigned char)dir;
	out[9] = (unsigned char)(idx >> 16);
	out[10] = (unsigned char)(idx >> 8);
	out[11] = (unsigned char)idx;
	memset(out + 12, 0xA5, 4);
}

void lb_proxy_arm(int dir, uint32_t idx)
{
	pthread_mutex_lock(&P.mu);
	lb_mark(P.armed[dir], dir, idx);
	P.arm[dir] = 1;
	pthread_mutex_unlock(&P.mu);
}

int lb_proxy_flips(void)
{
	int n;

	pthread_mutex_lock(&P.mu);
	n = P.flips;
	pthread_mutex_unlock(&P.mu);
	return n;
}

int lb_proxy_conns(void)
{
	int n;

	pthread_mutex_lock(&P.mu);
	n = P.conns;
	pthread_mutex_unlock(&P.mu);
	return n;
}

static int write_all(int fd, const unsigned char *p, size_t n)
{
	while (n) {
		ssize_t w = write(fd, p, n);

		if (w < 0 && errno == EINTR)
			continue;
		if (w <= 0)
			return -1;
		p += w;
		n -= (size_t)w;
	}
	return 0;
}

/* scan [carry || buf) for the armed mark of direction d; flip when due */
static void scan_flip(struct side *sd, int d, unsigned char *buf, size_t n)
{
	unsigned char win[LB_MARK_BYTES - 1 + BUF_BYTES];
	size_t i, m;

	pthread_mutex_lock(&P.mu);
	if (P.arm[d]) {
		memcpy(win, sd->carry, sd->ncarry);
		memcpy(win + sd->ncarry, buf, n);
		m = sd->ncarry + n;
		for (i = 0; i + LB_MARK_BYTES <= m; i++)
			if (win[i] == 'P' && !memcmp(win + i, P.armed[d], LB_MARK_BYTES)) {
				sd->flip_at = sd->pos - sd->ncarry + i + LB_MARK_BYTES + FLIP_AFTER;
				P.arm[d] = 0;
				break;
			}
	}
	if (sd->flip_at >= sd->pos && sd->flip_at < sd->pos + n) {
		buf[sd->flip_at - sd->pos] ^= 0x10;
		sd->flip_at = ~0ull;
		P.flips++;
	}
	pthread_mutex_unlock(&P.mu);
	/* keep the last bytes for a mark that straddles two reads */
	if (n >= LB_MARK_BYTES - 1) {
		memcpy(sd->carry, buf + n - (LB_MARK_BYTES - 1), LB_MARK_BYTES - 1);
		sd->ncarry = LB_MARK_BYTES - 1;
	} else {
		size_t keep = sd->ncarry + n > LB_MARK_BYTES - 1 ? LB_MARK_BYTES - 1 - n : sd->ncarry;

		memmove(sd->carry, sd->carry + sd->ncarry - keep, keep);
		memcpy(sd->carry + keep, buf, n);
		sd->ncarry = (unsigned int)(keep + n);
	}
	sd->pos += n;
}

static void pair_close(struct pair *pr)
{
	close(pr->s[0].fd);
	close(pr->s[1].fd);
	pr->live = 0;
}

static void nodelay(int fd)
{
	int one = 1;

	(void)setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

static void accept_one(void)
{
	int c = accept(P.lfd, NULL, NULL), s, k;

	if (c < 0)
		return;
	s = socket(AF_INET, SOCK_STREAM, 0);
	if (s < 0 || connect(s, (struct sockaddr *)&P.target, sizeof(P.target))) {
		close(c);
		if (s >= 0)
			close(s);
		return;
	}
	nodelay(c);
	nodelay(s);
	for (k = 0; k < MAX_PAIRS; k++)
		if (!P.pairs[k].live)
			break;
	if (k == MAX_PAIRS) {
		close(c);
		close(s);
		return;
	}
	memset(&P.pairs[k], 0, sizeof(P.pairs[k]));
	P.pairs[k].live = 1;
	P.pairs[k].s[LB_C2S].fd = c;
	P.pairs[k].s[LB_S2C].fd = s;
	P.pairs[k].s[0].flip_at = P.pairs[k].s[1].flip_at = ~0ull;
	pthread_mutex_lock(&P.mu);
	P.conns++;
	pthread_mutex_unlock(&P.mu);
}

static void *proxy_main(void *arg)
{
	static unsigned char buf[BUF_BYTES];
	struct pollfd pf[2 + 2 * MAX_PAIRS];
	int map[2 + 2 * MAX_PAIRS];
	(void)arg;

	for (;;) {
		int n = 0, k, r;

		pf[n].fd = P.stopfd;
		pf[n].events = POLLIN;
		map[n++] = -1;
		pf[n].fd = P.lfd;
		pf[n].events = POLLIN;
		map[n++] = -2;
		for (k = 0; k < MAX_PAIRS; k++)
			if (P.pairs[k].live) {
				pf[n].fd = P.pairs[k].s[0].fd;
				pf[n].events = POLLIN;
				map[n++] = 2 * k;
				pf[n].fd = P.pairs[k].s[1].fd;
				pf[n].events = POLLIN;
				map[n++] = 2 * k + 1;
			}
		r = poll(pf, (nfds_t)n, -1);
		if (r < 0 && errno == EINTR)
			continue;
		if (r < 0 || (pf[0].revents & POLLIN))
			break;
		if (pf[1].revents & POLLIN)
			accept_one();
		for (k = 2; k < n; k++) {
			struct pair *pr = &P.pairs[map[k] / 2];
			const int d = map[k] & 1;
			ssize_t got;

			if (!pr->live || !(pf[k].revents & (POLLIN | POLLHUP | POLLERR)))
				continue;
			got = read(pr->s[d].fd, buf, sizeof(buf));
			if (got <= 0) {
				/* one side closed or failed: the messenger faulted; end the pair */
				pair_close(pr);
				continue;
			}
			scan_flip(&pr->s[d], d, buf, (size_t)got);
			if (write_all(pr->s[d ^ 1].fd, buf, (size_t)got))
				pair_close(pr);
		}
	}
	for (int k = 0; k < MAX_PAIRS; k++)
		if (P.pairs[k].live)
			pair_close(&P.pairs[k]);
	return NULL;
}

int lb_proxy_start(uint16_t target_port_be, uint16_t *listen_port_be)
{
	struct sockaddr_in a;
	socklen_t al = sizeof(a);
	int one = 1;

	memset(&P, 0, sizeof(P));
	pthread_mutex_init(&P.mu, NULL);
	P.target.sin_family = AF_INET;
	P.target.sin_port = target_port_be;
	P.target.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
	P.lfd = socket(AF_INET, SOCK_STREAM, 0);
	if (P.lfd < 0)
		return -errno;
	(void)setsockopt(P.lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
	memset(&a, 0, sizeof(a));
	a.sin_family = AF_INET;
	a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
	if (bind(P.lfd, (struct sockaddr *)&a, sizeof(a)) || listen(P.lfd, 16) ||
	    getsockname(P.lfd, (struct sockaddr *)&a, &al))
		return -errno;
	*listen_port_be = a.sin_port;
	P.stopfd = eventfd(0, EFD_CLOEXEC);
	if (P.stopfd < 0)
		return -errno;
	return -pthread_create(&P.thr, NULL, proxy_main, NULL);
}

void lb_proxy_stop(void)
{
	const uint64_t one = 1;

	if (write(P.stopfd, &one, sizeof(one)) == sizeof(one))
		pthread_join(P.thr, NULL);
	close(P.stopfd);
	close(P.lfd);
}
