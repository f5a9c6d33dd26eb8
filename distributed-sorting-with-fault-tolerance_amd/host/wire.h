/* wire.h -- master <-> worker wire protocol.
 *
 * v0 = the reference's protocol, kept bit-compatible so the build's master drives the
 *      reference's `client` and the reference's `server` drives the build's worker:
 *      TCP/IPv4, native-endian int32, no header.  The master sends a chunk in send()s of at most
 *      4096 bytes (server.c:351-352) followed by a separate 4-byte -1 end marker
 *      (server.c:405-406); the worker accumulates ints until it sees -1 (client.c:112-113), sorts
 *      and replies with exactly chunk_size int32 and no terminator (client.c:119).  One
 *      connection serves many chunks (client.c:94).  Consequence kept from the reference: a -1
 *      key cannot be sent.
 * v1 = length-prefixed frames (24-byte header + payload), TCP_NODELAY, int32 or int64 keys, the
 *      full key range, heartbeats and worker error reports.
 */
#ifndef DSORT_WIRE_H
#define DSORT_WIRE_H

#include <stddef.h>
#include <stdint.h>

#define WIRE_V0_PIECE_BYTES 4096 /* BUFFER_SIZE ints * 4, server.c:12 */
#define WIRE_V0_END_MARKER (-1)  /* server.c:405 / client.c:113 */

#define WIRE_MAGIC 0x54525344u /* "DSRT" little endian */
#define WIRE_VERSION 1

enum wire_type {
    WIRE_SORT = 1,   /* master -> worker: payload = count keys of elem_bytes each     */
    WIRE_RESULT = 2, /* worker -> master: payload = the sorted keys                   */
    WIRE_PING = 3,   /* master -> worker heartbeat                                    */
    WIRE_PONG = 4,   /* worker -> master heartbeat answer                             */
    WIRE_BYE = 5,    /* master -> worker: close the session                           */
    WIRE_ERROR = 6,  /* worker -> master: status = negative DSORT_E* code, no payload */
};

typedef struct wire_hdr {
    uint32_t magic;
    uint16_t version;
    uint16_t type;
    uint32_t elem_bytes;
    int32_t status;
    uint64_t count;
} wire_hdr;

/* Socket helpers: 0 on success, -1 on error / EOF / timeout (errno kept). */
int wire_send_all(int fd, const void *p, size_t n);
int wire_recv_all(int fd, void *p, size_t n);
int wire_set_nodelay(int fd);
int wire_set_recv_timeout(int fd, double seconds); /* 0 = no timeout */

/* v0, master side */
int wire_v0_send_chunk(int fd, const int32_t *keys, size_t n);
int wire_v0_recv_sorted(int fd, int32_t *keys, size_t n);

/* v0, worker side: buffered reader that splits the byte stream at -1 end markers. */
typedef struct wire_v0_reader {
    int fd;
    unsigned char buf[WIRE_V0_PIECE_BYTES + 4];
    size_t len; /* bytes held in buf */
    size_t pos; /* next unread byte */
} wire_v0_reader;
void wire_v0_reader_init(wire_v0_reader *r, int fd);
/* Reads one chunk (all ints before the next -1) into *buf (grown with realloc as needed).
 * Returns 0 with *n set, or -1 on EOF/error. */
int wire_v0_recv_chunk(wire_v0_reader *r, int32_t **buf, size_t *cap, size_t *n);
int wire_v0_send_sorted(int fd, const int32_t *keys, size_t n);

/* v1 */
int wire_v1_send(int fd, uint16_t type, uint32_t elem_bytes, int32_t status, const void *payload,
                 uint64_t count);
/* Receives and validates a header (magic, version).  0 / -1. */
int wire_v1_recv_hdr(int fd, wire_hdr *h);

#endif
