/* worker.c -- the GPU worker node (role of the reference's client.c).
 *
 *   dsort_worker [--proto v0|v1] [--device D] [--fault MODE:K] [--verbose] client.conf
 *   dsort_worker --mode samplesort --connect HOST:PORT --device D   (ss_worker.c)
 *
 * Connects to the master (client.c:68-88), then serves chunks until the master closes the
 * connection (client.c:94-134).  Where the reference calls merge_sort(chunk, 0, n-1)
 * (client.c:117) this worker calls dsort_sort_i32(), the MI355X sort of libdsort.
 * Differences from client.c: no 4096-key chunk cap (client.c:91 overflows past it), no per-key
 * printf, the GPU context is created once at start-up and a missing GPU is a hard error.
 *
 * Fault injection for the fault-tolerance tests (the reference has none):
 *   --fault exit-before-reply:K   exit after receiving the K-th chunk, without replying
 *                                 (the recv-fault path of the master, server.c:421)
 *   --fault hang-before-reply:K   stop answering after receiving the K-th chunk (detected only
 *                                 by the master's --timeout; the reference would hang forever)
 *   --fault exit-on-connect       connect, then exit before any chunk (send/recv fault path)
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "conf.h"
#include "dsort.h"
#include "wire.h"

enum fault_mode { FAULT_NONE, FAULT_EXIT_BEFORE_REPLY, FAULT_HANG_BEFORE_REPLY, FAULT_EXIT_ON_CONNECT };

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

static void usage(void) {
    fprintf(stderr, "usage: dsort_worker [--proto v0|v1] [--device D] [--fault MODE:K] [--verbose] client.conf\n");
    exit(2);
}

static void maybe_fault(enum fault_mode mode, long at, long chunk_no) {
    if (chunk_no != at) return;
    if (mode == FAULT_EXIT_BEFORE_REPLY) {
        fprintf(stderr, "worker: fault injection: exiting before replying to chunk %ld\n", chunk_no);
        _exit(0);
    }
    if (mode == FAULT_HANG_BEFORE_REPLY) {
        fprintf(stderr, "worker: fault injection: hanging before replying to chunk %ld\n", chunk_no);
        for (;;) pause();
    }
}

int samplesort_worker(const char *host, int port, int device, int verbose); /* ss_worker.c */

int main(int argc, char **argv) {
    int samplesort = 0;
    const char *connect_to = NULL;
    for (int i = 1; i + 1 < argc; ++i) {
        if (!strcmp(argv[i], "--mode") && !strcmp(argv[i + 1], "samplesort")) samplesort = 1;
        if (!strcmp(argv[i], "--connect")) connect_to = argv[i + 1];
    }
    if (samplesort) {
        int dev = 0;
        for (int i = 1; i + 1 < argc; ++i)
            if (!strcmp(argv[i], "--device")) dev = atoi(argv[i + 1]);
        const char *colon = connect_to ? strrchr(connect_to, ':') : NULL;
        if (!colon) usage();
        char host[64];
        snprintf(host, sizeof host, "%.*s", (int)(colon - connect_to), connect_to);
        return samplesort_worker(host, atoi(colon + 1), dev, 0);
    }
    int proto = 0, device = 0, verbose = 0;
    enum fault_mode fmode = FAULT_NONE;
    long fat = 0;
    const char *conf_path = NULL;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--proto") && i + 1 < argc) {
            ++i;
            if (!strcmp(argv[i], "v0")) proto = 0;
            else if (!strcmp(argv[i], "v1")) proto = 1;
            else usage();
        } else if (!strcmp(argv[i], "--device") && i + 1 < argc) {
            device = atoi(argv[++i]);
        } else if (!strcmp(argv[i], "--fault") && i + 1 < argc) {
            const char *m = argv[++i];
            const char *colon = strchr(m, ':');
            if (!strncmp(m, "exit-before-reply", 17)) fmode = FAULT_EXIT_BEFORE_REPLY;
            else if (!strncmp(m, "hang-before-reply", 17)) fmode = FAULT_HANG_BEFORE_REPLY;
            else if (!strcmp(m, "exit-on-connect")) fmode = FAULT_EXIT_ON_CONNECT;
            else usage();
            fat = colon ? atol(colon + 1) : 1;
        } else if (!strcmp(argv[i], "--verbose")) {
            verbose = 1;
        } else if (argv[i][0] == '-') {
            usage();
        } else {
            conf_path = argv[i];
        }
    }
    if (!conf_path) usage();
    signal(SIGPIPE, SIG_IGN);

    dsort_conf conf;
    if (dsort_conf_read(conf_path, 1, &conf)) return 1;

    dsort_ctx *ctx = NULL;
    int rc = dsort_init(&ctx, device);
    if (rc) {
        fprintf(stderr, "worker: dsort_init(device %d) failed (%d): a gfx950 GPU is required\n", device, rc);
        return 3;
    }

    int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) {
        perror("worker: socket");
        return 1;
    }
    struct sockaddr_in addr;
    memset(&addr, 0, sizeof addr);
    addr.sin_family = AF_INET;
    addr.sin_port = htons((uint16_t)conf.server_port);
    if (inet_pton(AF_INET, conf.server_ip, &addr.sin_addr) <= 0) {
        fprintf(stderr, "worker: bad SERVER_IP %s\n", conf.server_ip);
        return 1;
    }
    if (connect(fd, (struct sockaddr *)&addr, sizeof addr) < 0) {
        perror("worker: connect");
        return 1;
    }
    if (proto == 1) wire_set_nodelay(fd);
    printf("Connected to server at IP: %s PORT: %d (proto v%d, device %d)\n", conf.server_ip,
           conf.server_port, proto, device);
    fflush(stdout);
    if (fmode == FAULT_EXIT_ON_CONNECT) {
        fprintf(stderr, "worker: fault injection: exiting right after connect\n");
        _exit(0);
    }

    long chunk_no = 0;
    size_t cap = 0;
    void *buf = NULL;
    if (proto == 0) {
        wire_v0_reader rd;
        wire_v0_reader_init(&rd, fd);
        int32_t *keys = NULL;
        size_t n = 0;
        while (wire_v0_recv_chunk(&rd, &keys, &cap, &n) == 0) {
            ++chunk_no;
            maybe_fault(fmode, fat, chunk_no);
            double t0 = now_ms();
            rc = dsort_sort_i32(ctx, keys, n);
            if (rc) {
                fprintf(stderr, "worker: dsort_sort_i32 failed: %s\n", dsort_last_error(ctx));
                break; /* v0 has no error frame: closing the socket makes the master reassign */
            }
            if (wire_v0_send_sorted(fd, keys, n)) break;
            if (verbose) printf("worker: chunk %ld: %zu keys sorted in %.3f ms\n", chunk_no, n, now_ms() - t0);
        }
        buf = keys;
    } else {
        wire_hdr h;
        while (wire_v1_recv_hdr(fd, &h) == 0) {
            if (h.type == WIRE_BYE) break;
            if (h.type == WIRE_PING) {
                if (wire_v1_send(fd, WIRE_PONG, 0, 0, NULL, 0)) break;
                continue;
            }
            if (h.type != WIRE_SORT || (h.elem_bytes != 4 && h.elem_bytes != 8)) {
                fprintf(stderr, "worker: unexpected frame type %u\n", h.type);
                break;
            }
            size_t bytes = (size_t)h.count * h.elem_bytes;
            if (bytes > cap) {
                void *nb = realloc(buf, bytes);
                if (!nb) {
                    wire_v1_send(fd, WIRE_ERROR, 0, DSORT_ENOMEM, NULL, 0);
                    break;
                }
                buf = nb;
                cap = bytes;
            }
            if (bytes && wire_recv_all(fd, buf, bytes)) break;
            ++chunk_no;
            maybe_fault(fmode, fat, chunk_no);
            double t0 = now_ms();
            rc = h.elem_bytes == 4 ? dsort_sort_i32(ctx, (int32_t *)buf, (size_t)h.count)
                                   : dsort_sort_i64(ctx, (int64_t *)buf, (size_t)h.count);
            if (rc) {
                fprintf(stderr, "worker: sort failed: %s\n", dsort_last_error(ctx));
                wire_v1_send(fd, WIRE_ERROR, h.elem_bytes, rc, NULL, 0);
                continue;
            }
            if (wire_v1_send(fd, WIRE_RESULT, h.elem_bytes, 0, buf, h.count)) break;
            if (verbose)
                printf("worker: chunk %ld: %llu keys sorted in %.3f ms\n", chunk_no,
                       (unsigned long long)h.count, now_ms() - t0);
        }
    }
    printf("Connection closed by server\n");
    free(buf);
    close(fd);
    dsort_finalize(ctx);
    return 0;
}
