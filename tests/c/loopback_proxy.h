/* loopback_proxy.h -- the corrupting TCP relay of build/msgr_loopback
 * (tests/c/loopback_proxy.c).  Test code only. */
#ifndef LOOPBACK_PROXY_H
#define LOOPBACK_PROXY_H

#include <stdint.h>

#define LB_MARK_BYTES 16
#define LB_C2S 0 /* client -> server */
#define LB_S2C 1 /* server -> client */

/* relay 127.0.0.1:<port> -> 127.0.0.1:target_port (network byte order) */
int lb_proxy_start(uint16_t target_port_be, uint16_t *listen_port_be);
void lb_proxy_stop(void);
/* the 16-byte mark of message idx in direction dir */
void lb_mark(unsigned char out[LB_MARK_BYTES], int dir, uint32_t idx);
/* flip one bit of the next message of direction dir carrying idx's mark */
void lb_proxy_arm(int dir, uint32_t idx);
int lb_proxy_flips(void);
int lb_proxy_conns(void);

#endif
