/* wire.c -- see wire.h */
#define _GNU_SOURCE
#include "wire.h"

#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

int wire_send_all(int fd, const void *p, size_t n) {
    const char *c = (const char *)p;
    while (n) {
        ssize_t k = send(fd, c, n, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            return -1;
        }
        c += k;
        n -= (size_t)k;
    }
    return 0;
}

int wire_recv_all(int fd, void *p, size_t n) {
    char *c = (char *)p;
    while (n) {
        ssize_t k = recv(fd, c, n, 0);
        if (k == 0) return -1; /* peer closed (server.c:421 treats <= 0 as a dead worker) */
        if (k < 0) {
            if (errno == EINTR) continue;
            return -1;         /* includes EAGAIN after SO_RCVTIMEO: a hung worker */
        }
        c += k;
        n -= (size_t)k;
    }
    return 0;
}

int wire_set_nodelay(int fd) {
    int one = 1;
    return setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

int wire_set_recv_timeout(int fd, double seconds) {
    struct timeval tv;
    tv.tv_sec = (time_t)seconds;
    tv.tv_usec = (suseconds_t)((seconds - (double)tv.tv_sec) * 1e6);
    return setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
}

/* ------------------------------------------------------------------------------- v0 */
int wire_v0_send_chunk(int fd, const int32_t *keys, size_t n) {
    const size_t per = WIRE_V0_PIECE_BYTES / sizeof(int32_t);
    for (size_t off = 0; off < n; off += per) {
        size_t m = n - off < per ? n - off : per;
        if (wire_send_all(fd, keys + off, m * sizeof(int32_t))) return -1;
    }
    const int32_t end = WIRE_V0_END_MARKER;
    return wire_send_all(fd, &end, sizeof end);
}

int wire_v0_recv_sorted(int fd, int32_t *keys, size_t n) {
    return wire_recv_all(fd, keys, n * sizeof(int32_t));
}

int wire_v0_send_sorted(int fd, const int32_t *keys, size_t n) {
    return wire_send_all(fd, keys, n * sizeof(int32_t));
}

void wire_v0_reader_init(wire_v0_reader *r, int fd) {
    r->fd = fd;
    r->len = r->pos = 0;
}

int wire_v0_recv_chunk(wire_v0_reader *r, int32_t **buf, size_t *cap, size_t *n) {
    *n = 0;
    for (;;) {
        while (r->len - r->pos >= sizeof(int32_t)) {
            int32_t v;
            memcpy(&v, r->buf + r->pos, sizeof v);
            r->pos += sizeof v;
            if (v == WIRE_V0_END_MARKER) return 0;
            if (*n == *cap) {
                size_t nc = *cap ? *cap * 2 : 4096;
                int32_t *nb = (int32_t *)realloc(*buf, nc * sizeof(int32_t));
                if (!nb) return -1;
                *buf = nb;
                *cap = nc;
            }
            (*buf)[(*n)++] = v;
        }
        /* keep a partial int (a recv may end mid-key) and refill */
        size_t rest = r->len - r->pos;
        memmove(r->buf, r->buf + r->pos, rest);
        r->len = rest;
        r->pos = 0;
        ssize_t k;
        do {
            k = recv(r->fd, r->buf + r->len, sizeof(r->buf) - r->len, 0);
        } while (k < 0 && errno == EINTR);
        if (k <= 0) return -1;
        r->len += (size_t)k;
    }
}

/* ------------------------------------------------------------------------------- v1 */
int wire_v1_send(int fd, uint16_t type, uint32_t elem_bytes, int32_t status, const void *payload,
                 uint64_t count) {
    wire_hdr h;
    h.magic = WIRE_MAGIC;
    h.version = WIRE_VERSION;
    h.type = type;
    h.elem_bytes = elem_bytes;
    h.status = status;
    h.count = count;
    if (wire_send_all(fd, &h, sizeof h)) return -1;
    if (payload && count && elem_bytes)
        return wire_send_all(fd, payload, (size_t)count * elem_bytes);
    return 0;
}

int wire_v1_recv_hdr(int fd, wire_hdr *h) {
    if (wire_recv_all(fd, h, sizeof *h)) return -1;
    if (h->magic != WIRE_MAGIC || h->version != WIRE_VERSION) {
        errno = EPROTO;
        return -1;
    }
    return 0;
}
