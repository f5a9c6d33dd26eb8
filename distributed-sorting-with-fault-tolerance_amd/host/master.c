/* master.c -- the master node (role of the reference's server.c) with a GPU merge.
 *
 *   dsort_master [--workers N] [--proto v0|v1] [--device D] [--timeout SEC]
 *                [--retry-delay-ms MS] [--reassign first|least-loaded] [--codec gpu|cpu]
 *                [--output PATH] server.conf
 *   dsort_master --mode samplesort --gpus N ...   the multi-GPU sample sort (ss_master.c)
 *
 * Same session model as server.c: accept exactly N worker connections (server.c:148-157), then
 * read file names from stdin until "exit" (server.c:160-168).  Per file:
 *   1. parse whitespace-separated %d keys (server.c:177-182, 212-214), on the GPU by default
 *      (dsort_parse_text_i32; --codec cpu keeps the host parser);
 *   2. split them into N contiguous chunks, chunk i holding n/N + (i < n%N) keys
 *      (server.c:185-216), and hand chunk i to worker i on its own thread (server.c:231-257);
 *   3. fault tolerance (server.c:297-477): a failed send or receive marks the worker dead and the
 *      whole chunk is re-sent, after a 100 ms pause (server.c:304), to a live worker; the sorted
 *      result always lands in the chunk's own slot (server.c:415); a per-worker mutex held over
 *      the whole send->receive transaction serialises two chunks on one worker (server.c:344);
 *   4. merge the N sorted chunks on the GPU with dsort_merge_i32 -- where server.c:266 calls
 *      merge_chunks() -- and write output.txt, one "%d\n" per key (server.c:517-519), formatted
 *      on the GPU by default (dsort_format_text_i32).
 * Differences: liveness state is mutex-protected (the reference races on
 * is_alive[]), dead sockets are closed and stay dead, --timeout adds the deadline detection the
 * reference lacks, --reassign least-loaded is offered beside the reference's first-alive rule,
 * keys and sizes have no 4096-per-chunk cap, and no key is logged.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <pthread.h>
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

#define MAX_WORKERS_LIMIT 256

typedef struct cluster {
    int n;
    int fds[MAX_WORKERS_LIMIT];
    int alive[MAX_WORKERS_LIMIT];
    int load[MAX_WORKERS_LIMIT];
    pthread_mutex_t wmutex[MAX_WORKERS_LIMIT]; /* w_socket_mutexes, server.c:23 */
    pthread_mutex_t state;                      /* guards alive[] and load[]          */
    int proto;
    double timeout_s;
    int retry_delay_us;
    int least_loaded;
} cluster;

typedef struct job {
    cluster *cl;
    int chunk;
    const int32_t *keys;
    size_t n;
    int32_t *result;
    int ok;
    int reassignments;
    double detect_ms; /* time from the start of a failed transaction to its detection */
    int served_by;
} job;

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

/* server.c:368-384 picks the first live worker; least-loaded picks the live worker with the
 * fewest transactions in flight (ties: lowest index). */
static int pick_worker(cluster *cl) {
    pthread_mutex_lock(&cl->state);
    int best = -1;
    for (int i = 0; i < cl->n; ++i) {
        if (!cl->alive[i]) continue;
        if (best < 0 || (cl->least_loaded && cl->load[i] < cl->load[best])) best = i;
        if (!cl->least_loaded) break;
    }
    pthread_mutex_unlock(&cl->state);
    return best;
}

static int is_alive(cluster *cl, int w) {
    pthread_mutex_lock(&cl->state);
    int a = cl->alive[w];
    pthread_mutex_unlock(&cl->state);
    return a;
}

static int transact(cluster *cl, int w, const int32_t *keys, size_t n, int32_t *out) {
    int fd = cl->fds[w];
    if (cl->proto == 0) {
        if (wire_v0_send_chunk(fd, keys, n)) return -1;
        return wire_v0_recv_sorted(fd, out, n);
    }
    if (wire_v1_send(fd, WIRE_SORT, 4, 0, keys, n)) return -1;
    wire_hdr h;
    if (wire_v1_recv_hdr(fd, &h)) return -1;
    if (h.type != WIRE_RESULT || h.count != n || h.elem_bytes != 4) {
        fprintf(stderr, "master: worker %d answered type %u status %d count %llu\n", w + 1, h.type,
                h.status, (unsigned long long)h.count);
        return -1;
    }
    return n ? wire_recv_all(fd, out, n * sizeof(int32_t)) : 0;
}

static void *worker_handler(void *arg) {
    job *jb = (job *)arg;
    cluster *cl = jb->cl;
    int cur = jb->chunk % cl->n;
    for (;;) {
        if (!is_alive(cl, cur)) {
            cur = pick_worker(cl);
            if (cur < 0) break;
        }
        pthread_mutex_lock(&cl->wmutex[cur]);
        if (!is_alive(cl, cur)) { /* died while we waited for its socket */
            pthread_mutex_unlock(&cl->wmutex[cur]);
            continue;
        }
        pthread_mutex_lock(&cl->state);
        cl->load[cur]++;
        pthread_mutex_unlock(&cl->state);
        double t0 = now_ms();
        int rc = transact(cl, cur, jb->keys, jb->n, jb->result);
        pthread_mutex_lock(&cl->state);
        cl->load[cur]--;
        if (rc) {
            cl->alive[cur] = 0;
            shutdown(cl->fds[cur], SHUT_RDWR);
        }
        pthread_mutex_unlock(&cl->state);
        pthread_mutex_unlock(&cl->wmutex[cur]);
        if (rc == 0) {
            jb->ok = 1;
            jb->served_by = cur;
            return NULL;
        }
        jb->detect_ms = now_ms() - t0;
        printf("Worker %d failed on chunk %d (%s after %.1f ms). Reassigning task...\n", cur + 1,
               jb->chunk + 1, errno == EAGAIN || errno == EWOULDBLOCK ? "timeout" : "disconnect",
               jb->detect_ms);
        fflush(stdout);
        int next = pick_worker(cl);
        if (next < 0) break;
        printf("Reassigning chunk %d to worker node %d\n", jb->chunk + 1, next + 1);
        fflush(stdout);
        jb->reassignments++;
        cur = next;
        usleep((useconds_t)cl->retry_delay_us); /* server.c:391 / 446 */
    }
    printf("No available worker nodes to handle chunk %d.\n", jb->chunk + 1);
    fflush(stdout);
    return NULL;
}

static char *read_file(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    size_t cap = 1 << 16, n = 0;
    char *b = (char *)malloc(cap + 1);
    for (;;) {
        if (!b) { fclose(f); return NULL; }
        size_t k = fread(b + n, 1, cap - n, f);
        n += k;
        if (n < cap) break;
        cap *= 2;
        char *nb = (char *)realloc(b, cap + 1);
        if (!nb) { free(b); fclose(f); return NULL; }
        b = nb;
    }
    fclose(f);
    b[n] = '\0';
    *len = n;
    return b;
}

/* %d tokens separated by whitespace; returns the count or -1 on a non-integer token (where
 * server.c:179 would spin forever). */
long master_parse_keys(const char *t, size_t len, int32_t **out) {
    size_t cap = len / 2 + 1, n = 0;
    int32_t *k = (int32_t *)malloc(cap * sizeof(int32_t));
    if (!k) return -1;
    size_t i = 0;
    while (i < len) {
        char c = t[i];
        if (c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\v' || c == '\f') { ++i; continue; }
        char *end = NULL;
        errno = 0;
        long long v = strtoll(t + i, &end, 10);
        if (end == t + i || (*end && !strchr(" \n\t\r\v\f", *end))) {
            free(k);
            return -1;
        }
        k[n++] = (int32_t)v;
        i = (size_t)(end - t);
    }
    *out = k;
    return (long)n;
}

/* output.txt: the GPU formatter (dsort_format_text_i32) or the host writer. */
static int write_output(dsort_ctx *ctx, int gpu, const char *path, const int32_t *k, size_t n) {
    if (!gpu) return dsort_write_text_i32(path, k, n);
    char *buf = (char *)malloc(12 * n + 1);
    size_t len = 0;
    int rc = buf ? dsort_format_text_i32(ctx, k, n, buf, 12 * n + 1, &len) : DSORT_ENOMEM;
    if (rc == 0) {
        FILE *f = fopen(path, "w");
        if (!f) {
            rc = DSORT_EINVAL;
        } else {
            if (fwrite(buf, 1, len, f) != len) rc = DSORT_EINVAL;
            if (fclose(f) != 0) rc = DSORT_EINVAL;
        }
    }
    free(buf);
    return rc;
}

static void usage(void) {
    fprintf(stderr, "usage: dsort_master [--workers N] [--proto v0|v1] [--device D] [--timeout SEC]\n"
                    "                    [--retry-delay-ms MS] [--reassign first|least-loaded]\n"
                    "                    [--codec gpu|cpu] [--output PATH] server.conf\n");
    exit(2);
}

int samplesort_master(int argc, char **argv, const char *argv0); /* ss_master.c */

int main(int argc, char **argv) {
    for (int i = 1; i + 1 < argc; ++i)
        if (!strcmp(argv[i], "--mode") && !strcmp(argv[i + 1], "samplesort"))
            return samplesort_master(argc - 1, argv + 1, argv[0]);
    static cluster cl;
    memset(&cl, 0, sizeof cl);
    cl.n = 4; /* MAX_WORKERS, server.c:11 */
    cl.retry_delay_us = 100000;
    int device = 0, codec_gpu = 1;
    const char *out_path = "output.txt", *conf_path = NULL;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--workers") && i + 1 < argc) cl.n = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--proto") && i + 1 < argc) {
            ++i;
            if (!strcmp(argv[i], "v0")) cl.proto = 0;
            else if (!strcmp(argv[i], "v1")) cl.proto = 1;
            else usage();
        } else if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--timeout") && i + 1 < argc) cl.timeout_s = atof(argv[++i]);
        else if (!strcmp(argv[i], "--retry-delay-ms") && i + 1 < argc) cl.retry_delay_us = atoi(argv[++i]) * 1000;
        else if (!strcmp(argv[i], "--reassign") && i + 1 < argc) {
            ++i;
            if (!strcmp(argv[i], "first")) cl.least_loaded = 0;
            else if (!strcmp(argv[i], "least-loaded")) cl.least_loaded = 1;
            else usage();
        } else if (!strcmp(argv[i], "--codec") && i + 1 < argc) {
            ++i;
            if (!strcmp(argv[i], "gpu")) codec_gpu = 1;
            else if (!strcmp(argv[i], "cpu")) codec_gpu = 0;
            else usage();
        } else if (!strcmp(argv[i], "--output") && i + 1 < argc) out_path = argv[++i];
        else if (argv[i][0] == '-') usage();
        else conf_path = argv[i];
    }
    if (!conf_path || cl.n < 1 || cl.n > MAX_WORKERS_LIMIT) usage();
    signal(SIGPIPE, SIG_IGN); /* server.c:116: failed sends must return, not kill the master */

    dsort_conf conf;
    if (dsort_conf_read(conf_path, 0, &conf)) return 1;
    printf("server port number is %d\n", conf.server_port);

    dsort_ctx *ctx = NULL;
    int rc = dsort_init(&ctx, device);
    if (rc) {
        fprintf(stderr, "master: dsort_init(device %d) failed (%d): the merge runs on a gfx950 GPU\n",
                device, rc);
        return 3;
    }

    int lfd = socket(AF_INET, SOCK_STREAM, 0);
    if (lfd < 0) { perror("Socket creation failed"); return 1; }
    int opt = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &opt, sizeof opt);
    struct sockaddr_in addr;
    memset(&addr, 0, sizeof addr);
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = INADDR_ANY;
    addr.sin_port = htons((uint16_t)conf.server_port);
    if (bind(lfd, (struct sockaddr *)&addr, sizeof addr) < 0) { perror("Binding failed"); return 1; }
    if (listen(lfd, cl.n) < 0) { perror("Listening failed"); return 1; }
    printf("Server is running and waiting for worker connections...\n");
    fflush(stdout);
    pthread_mutex_init(&cl.state, NULL);
    for (int i = 0; i < cl.n; ++i) {
        cl.fds[i] = accept(lfd, NULL, NULL);
        if (cl.fds[i] < 0) { perror("Connection acceptance failed"); return 1; }
        if (cl.proto == 1) wire_set_nodelay(cl.fds[i]);
        if (cl.timeout_s > 0) wire_set_recv_timeout(cl.fds[i], cl.timeout_s);
        cl.alive[i] = 1;
        pthread_mutex_init(&cl.wmutex[i], NULL);
        printf("Worker %d connected\n", i + 1);
        fflush(stdout);
    }

    char name[4096];
    for (;;) {
        printf("Enter the filename to sort (or 'exit' to quit): ");
        fflush(stdout);
        if (scanf("%4095s", name) != 1 || !strcmp(name, "exit")) {
            printf("Exiting server...\n");
            break;
        }
        double t0 = now_ms();
        size_t len = 0;
        char *text = read_file(name, &len);
        if (!text) { perror("Error opening file"); continue; }
        int32_t *keys = NULL;
        long nk;
        if (codec_gpu) {
            const size_t cap = len / 2 + 1;  /* at most one token per two bytes */
            size_t cnt = 0;
            keys = (int32_t *)malloc(cap * sizeof(int32_t));
            rc = keys ? dsort_parse_text_i32(ctx, text, len, keys, cap, &cnt) : DSORT_ENOMEM;
            if (rc && rc != DSORT_EINVAL) {
                fprintf(stderr, "master: GPU parse failed (%d): %s\n", rc, dsort_last_error(ctx));
                return 1;
            }
            nk = rc ? -1 : (long)cnt;
            if (rc) {
                free(keys);
                keys = NULL;
            }
        } else {
            nk = master_parse_keys(text, len, &keys);
        }
        free(text);
        if (nk < 0) {
            fprintf(stderr, "master: %s contains a non-integer token; file skipped\n", name);
            continue;
        }
        size_t n = (size_t)nk;
        if (cl.proto == 0) {
            int bad = 0;
            for (size_t i = 0; i < n && !bad; ++i) bad = keys[i] == WIRE_V0_END_MARKER;
            if (bad) {
                fprintf(stderr, "master: key -1 is the v0 end marker (client.c:113); use --proto v1. File skipped\n");
                free(keys);
                continue;
            }
        }
        double t_parse = now_ms();
        job *jobs = (job *)calloc((size_t)cl.n, sizeof(job));
        pthread_t *th = (pthread_t *)calloc((size_t)cl.n, sizeof(pthread_t));
        int32_t *result = (int32_t *)malloc((n ? n : 1) * sizeof(int32_t));
        const int32_t **runs = (const int32_t **)calloc((size_t)cl.n, sizeof(int32_t *));
        size_t *lens = (size_t *)calloc((size_t)cl.n, sizeof(size_t));
        if (!jobs || !th || !result || !runs || !lens) { fprintf(stderr, "master: out of memory\n"); return 1; }
        size_t off = 0;
        for (int i = 0; i < cl.n; ++i) {
            size_t sz = n / (size_t)cl.n + ((size_t)i < n % (size_t)cl.n ? 1 : 0);
            jobs[i] = (job){&cl, i, keys + off, sz, result + off, 0, 0, 0.0, -1};
            runs[i] = result + off;
            lens[i] = sz;
            off += sz;
            pthread_create(&th[i], NULL, worker_handler, &jobs[i]);
        }
        int all_ok = 1, reassign = 0;
        double detect = 0;
        for (int i = 0; i < cl.n; ++i) {
            pthread_join(th[i], NULL);
            all_ok &= jobs[i].ok;
            reassign += jobs[i].reassignments;
            if (jobs[i].detect_ms > detect) detect = jobs[i].detect_ms;
        }
        double t_sorted = now_ms();
        int alive = 0;
        for (int i = 0; i < cl.n; ++i) alive += is_alive(&cl, i);
        if (!all_ok) {
            printf("Sorting failed for file %s: no live worker left for some chunk\n", name);
        } else {
            int32_t *merged = (int32_t *)malloc((n ? n : 1) * sizeof(int32_t));
            rc = merged ? dsort_merge_i32(ctx, runs, lens, cl.n, merged) : DSORT_ENOMEM;
            double t_merged = now_ms();
            if (rc == 0) rc = write_output(ctx, codec_gpu, out_path, merged, n);
            double t_written = now_ms();
            if (rc) {
                fprintf(stderr, "master: merge/write failed (%d): %s\n", rc, dsort_last_error(ctx));
            } else {
                printf("Sorting completed for file %s. Output saved to %s\n", name, out_path);
                printf("dsort_master: file=%s keys=%zu workers=%d alive=%d reassignments=%d "
                       "detect_ms=%.3f parse_ms=%.3f sort_ms=%.3f merge_ms=%.3f write_ms=%.3f total_ms=%.3f\n",
                       name, n, cl.n, alive, reassign, detect, t_parse - t0, t_sorted - t_parse,
                       t_merged - t_sorted, t_written - t_merged, t_written - t0);
            }
            free(merged);
        }
        fflush(stdout);
        free(keys);
        free(result);
        free(jobs);
        free(th);
        free(runs);
        free(lens);
    }
    for (int i = 0; i < cl.n; ++i) {
        if (cl.proto == 1 && is_alive(&cl, i)) wire_v1_send(cl.fds[i], WIRE_BYE, 0, 0, NULL, 0);
        close(cl.fds[i]);
    }
    close(lfd);
    dsort_finalize(ctx);
    return 0;
}
