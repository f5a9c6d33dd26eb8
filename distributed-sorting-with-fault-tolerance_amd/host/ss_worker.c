/* ss_worker.c -- dsort_worker --mode samplesort: one GPU worker of the multi-GPU sample sort
 * (client.c's role, protocol in ss.h).
 *
 *   dsort_worker --mode samplesort --connect HOST:PORT [--device D] [--verbose]
 *
 * Per job: map the master's chunk replicas and pin them (dsort_host_register); stage this rank's
 * chunk in HBM (generated on the GPU and copied into the replica, or copied from it); build the
 * communicator of epoch 0; on GO run the sample sort of the chunk (dsort_sample_sort_dev_*: the
 * bucket exchange partitions the unsorted chunk, ships the buckets and sorts the received ones --
 * where client.c:117 calls merge_sort and server.c:414-415 gathers), report DONE.  A PLAN from the
 * master (a peer failed) aborts the communicator -- also from inside a running exchange, through
 * dsort_comm_abort on the reader thread -- and starts the recovery epoch: the chunks this worker
 * now owns come from the pinned replica and are appended to its keys, and the sample sort runs
 * again over the survivors. */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "dsort.h"
#include "ss.h"
#include "wire.h"

typedef struct wk {
    int fd;
    dsort_ctx *ctx;
    pthread_mutex_t send_mu;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int go, bye, closed, slice_req, stop;
    int plan_pending;
    int initing;         /* inside dsort_comm_init* (the heartbeat thread re-raises a lost abort) */
    ss_plan plan;
    uint32_t epoch;      /* epoch of the communicator in use */
    int world;           /* ranks of that epoch */
    int32_t relay_seq;   /* next relay request of this epoch */
    int32_t want_tag;    /* the relay response awaited (-1: none): the reader drops any other, e.g. a
                            late answer to a request abandoned at the deadline */
    int resp_ready;
    int32_t resp_tag;
    char *resp;
    size_t resp_len;
    uint32_t hb_ms;
    int64_t comm_timeout_ms; /* deadline of one relay exchange (the RCCL path's exchange deadline) */
} wk;

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

/* Sends one frame whose payload is up to two pieces (no copy). */
static int send_frame2(wk *w, uint16_t type, int32_t status, const void *a, size_t na, const void *b, size_t nb) {
    pthread_mutex_lock(&w->send_mu);
    wire_hdr h = {WIRE_MAGIC, WIRE_VERSION, type, 1, status, (uint64_t)(na + nb)};
    int rc = wire_send_all(w->fd, &h, sizeof h);
    if (!rc && na) rc = wire_send_all(w->fd, a, na);
    if (!rc && nb) rc = wire_send_all(w->fd, b, nb);
    pthread_mutex_unlock(&w->send_mu);
    return rc;
}
static int send_frame(wk *w, uint16_t type, const void *p, size_t bytes) {
    return send_frame2(w, type, 0, p, bytes, NULL, 0);
}

/* The only reader of the socket after start-up: demultiplexes the master's frames. */
static void *reader_main(void *arg) {
    wk *w = (wk *)arg;
    for (;;) {
        wire_hdr h;
        char *buf = NULL;
        int bad = wire_v1_recv_hdr(w->fd, &h);
        if (!bad && h.count) {
            buf = (char *)malloc(h.count);
            bad = !buf || wire_recv_all(w->fd, buf, h.count);
        }
        pthread_mutex_lock(&w->mu);
        if (bad) {
            w->closed = 1;
            dsort_comm_abort(w->ctx); /* the master is gone: abandon any exchange in flight */
            pthread_cond_broadcast(&w->cv);
            pthread_mutex_unlock(&w->mu);
            free(buf);
            return NULL;
        }
        switch (h.type) {
            case SS_GO: w->go = 1; break;
            case SS_BYE: w->bye = 1; break;
            case SS_GET_SLICE: w->slice_req = 1; break;
            case SS_PLAN:
                if (h.count == sizeof(ss_plan)) {
                    memcpy(&w->plan, buf, sizeof(ss_plan));
                    w->plan_pending = 1;
                    /* under w->mu: the main thread cannot have built the next epoch's
                     * communicator yet.  Inside a running exchange this only raises the abort
                     * flag; the exchange aborts the communicator itself (dsort.h). */
                    dsort_comm_abort(w->ctx);
                }
                break;
            case SS_RELAY_RESP:
                if (h.status != w->want_tag) break; /* abandoned or stale: dropped (buf freed below) */
                free(w->resp);
                w->resp = buf;
                buf = NULL;
                w->resp_len = h.count;
                w->resp_tag = h.status;
                w->resp_ready = 1;
                break;
            default:
                break;
        }
        pthread_cond_broadcast(&w->cv);
        pthread_mutex_unlock(&w->mu);
        free(buf);
    }
}

static void *heartbeat_main(void *arg) {
    wk *w = (wk *)arg;
    for (;;) {
        pthread_mutex_lock(&w->mu);
        struct timespec ts;
        clock_gettime(CLOCK_REALTIME, &ts);
        ts.tv_nsec += (long)w->hb_ms * 1000000L;
        ts.tv_sec += ts.tv_nsec / 1000000000L;
        ts.tv_nsec %= 1000000000L;
        while (!w->stop && !w->closed)
            if (pthread_cond_timedwait(&w->cv, &w->mu, &ts) == ETIMEDOUT) break;
        const int done = w->stop || w->closed;
        /* a PLAN for a newer epoch while the communicator of this one is being built: the
         * reader's abort may have come before dsort_comm_init took the communicator lock and been
         * lost; repeat it until the set-up returns (an init waiting for a dead peer never would) */
        /* (under w->mu, like the reader's abort: a late abort outside the lock could land after
         * the main thread moved on to the newer epoch and cancel that epoch's set-up; the call
         * only try-locks the communicator, so it never blocks here) */
        if (w->initing && w->plan_pending && w->plan.epoch > w->epoch) dsort_comm_abort(w->ctx);
        pthread_mutex_unlock(&w->mu);
        if (done || send_frame(w, SS_HB, NULL, 0)) return NULL;
    }
}

/* ---- relay transport: the sample sort's exchanges through the master -------------------- */
static int superseded(wk *w) { return w->closed || (w->plan_pending && w->plan.epoch > w->epoch); }

static int relay(wk *w, uint16_t type, const void *a, size_t na, const void *b, size_t nb, char **resp,
                 size_t *resp_len) {
    pthread_mutex_lock(&w->mu);
    if (superseded(w)) {
        pthread_mutex_unlock(&w->mu);
        return -1;
    }
    const int32_t tag = (int32_t)((w->epoch << 20) | (uint32_t)w->relay_seq++);
    w->resp_ready = 0;
    free(w->resp); /* (nothing else may be pending: the reader keeps only the awaited tag) */
    w->resp = NULL;
    w->want_tag = tag;
    pthread_mutex_unlock(&w->mu);
    if (send_frame2(w, type, tag, a, na, b, nb)) {
        pthread_mutex_lock(&w->mu);
        w->want_tag = -1;
        pthread_mutex_unlock(&w->mu);
        return -1;
    }
    pthread_mutex_lock(&w->mu);
    /* the sample sort's exchange deadline (DSORT_OPT_COMM_TIMEOUT_MS, from the start of the sort,
     * like the RCCL path's: it must cover the slowest rank's local part): a hung peer never posts
     * its part, and the master answers only when every live rank has.  The library says how much
     * of it is left (dsort_comm_deadline_ms); outside a sort, the option's full length. */
    int64_t left = -1;
    if (dsort_comm_deadline_ms(w->ctx, &left) != DSORT_OK || left < 0) left = w->comm_timeout_ms > 0 ? w->comm_timeout_ms : -1;
    struct timespec dl;
    clock_gettime(CLOCK_REALTIME, &dl);
    if (left >= 0) {
        dl.tv_sec += (time_t)(left / 1000);
        dl.tv_nsec += (long)(left % 1000) * 1000000L;
        dl.tv_sec += dl.tv_nsec / 1000000000L;
        dl.tv_nsec %= 1000000000L;
    }
    int timed_out = left == 0;
    while (!(w->resp_ready && w->resp_tag == tag) && !superseded(w) && !timed_out) {
        if (left >= 0) timed_out = pthread_cond_timedwait(&w->cv, &w->mu, &dl) == ETIMEDOUT;
        else pthread_cond_wait(&w->cv, &w->mu);
    }
    const int ok = w->resp_ready && w->resp_tag == tag;
    if (ok) {
        *resp = w->resp;
        *resp_len = w->resp_len;
        w->resp = NULL;
        w->resp_ready = 0;
    }
    w->want_tag = -1; /* a late answer to an abandoned request is dropped by the reader */
    pthread_mutex_unlock(&w->mu);
    return ok ? 0 : (timed_out ? DSORT_ETIMEOUT : -1);
}

static int relay_allgather(void *user, const void *send, void *recv, size_t bytes) {
    wk *w = (wk *)user;
    char *r = NULL;
    size_t rl = 0;
    const int rr = relay(w, SS_RELAY_AG, send, bytes, NULL, 0, &r, &rl);
    if (rr) return rr == DSORT_ETIMEOUT ? DSORT_ETIMEOUT : 1;
    const int bad = rl != bytes * (size_t)w->world;
    if (!bad) memcpy(recv, r, rl);
    free(r);
    return bad;
}

/* request: P send counts (uint64), then the pieces in destination order; response: P receive
 * counts, then the pieces in source order */
static int relay_alltoallv(void *user, const void *send, const size_t *sc, const size_t *sd, void *recv,
                           const size_t *rcnt, const size_t *rd) {
    wk *w = (wk *)user;
    const int P = w->world;
    uint64_t tot = 0;
    for (int d = 0; d < P; ++d) tot += sc[d];
    char *req = (char *)calloc(1, (size_t)P * 8 + tot);
    if (!req) return 1;
    uint64_t off = (uint64_t)P * 8;
    for (int d = 0; d < P; ++d) {
        const uint64_t c = sc[d];
        memcpy(req + (size_t)d * 8, &c, 8);
        if (c) memcpy(req + off, (const char *)send + sd[d], c);
        off += c;
    }
    char *r = NULL;
    size_t rl = 0;
    const int rc = relay(w, SS_RELAY_A2A, req, off, NULL, 0, &r, &rl);
    free(req);
    if (rc) return rc == DSORT_ETIMEOUT ? DSORT_ETIMEOUT : 1;
    int bad = rl < (size_t)P * 8;
    uint64_t pos = (uint64_t)P * 8;
    for (int s = 0; s < P && !bad; ++s) {
        uint64_t c;
        memcpy(&c, r + (size_t)s * 8, 8);
        if (c != rcnt[s] || pos + c > rl) {
            bad = 1;
            break;
        }
        if (c) memcpy((char *)recv + rd[s], r + pos, c);
        pos += c;
    }
    free(r);
    return bad;
}

/* ---- the sort ------------------------------------------------------------------------- */
static void chunk_range(uint64_t n, uint32_t world, uint32_t c, uint64_t *off, uint64_t *len) {
    const uint64_t q = n / world, r = n % world; /* server.c:185-216 */
    *len = q + (c < r ? 1 : 0);
    *off = (uint64_t)c * q + (c < r ? c : r);
}

#define CHECK(call)                                                                               \
    do {                                                                                          \
        int rc_ = (call);                                                                         \
        if (rc_) {                                                                                \
            fprintf(stderr, "worker: %s failed (%d): %s\n", #call, rc_, dsort_last_error(ctx));   \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

/* The communicator of `epoch`.  Returns COMM_SUPERSEDED (and builds nothing, or drops what it
 * built) when a PLAN for a newer epoch is pending, else the dsort_comm_init* code. */
#define COMM_SUPERSEDED 1
static int comm_up(wk *w, const ss_job *job, uint32_t epoch, int world, int rank, const char *uid,
                   dsort_transport *tx) {
    dsort_ctx *ctx = w->ctx;
    pthread_mutex_lock(&w->mu);
    if (w->plan_pending && w->plan.epoch > epoch) {
        pthread_mutex_unlock(&w->mu);
        return COMM_SUPERSEDED;
    }
    w->epoch = epoch; /* with initing, under one lock: the heartbeat's check sees both */
    w->world = world;
    w->relay_seq = 0;
    w->initing = 1;
    pthread_mutex_unlock(&w->mu);
    int rc = job->transport == 0 ? dsort_comm_init(ctx, world, rank, uid) : dsort_comm_init_transport(ctx, world, rank, tx);
    pthread_mutex_lock(&w->mu);
    w->initing = 0;
    const int newer = w->plan_pending && w->plan.epoch > epoch;
    pthread_mutex_unlock(&w->mu);
    if (newer) {
        dsort_comm_abort(ctx);
        rc = COMM_SUPERSEDED;
    }
    return rc;
}

int samplesort_worker(const char *host, int port, int device, int verbose) {
    (void)verbose;
    dsort_ctx *ctx = NULL;
    int rc = dsort_init(&ctx, device);
    if (rc) {
        fprintf(stderr, "worker: dsort_init(device %d) failed (%d): a gfx950 GPU is required\n", device, rc);
        return 3;
    }
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    struct sockaddr_in addr;
    memset(&addr, 0, sizeof addr);
    addr.sin_family = AF_INET;
    addr.sin_port = htons((uint16_t)port);
    if (fd < 0 || inet_pton(AF_INET, host, &addr.sin_addr) <= 0 ||
        connect(fd, (struct sockaddr *)&addr, sizeof addr) < 0) {
        perror("worker: connect");
        return 1;
    }
    wire_set_nodelay(fd);
    static wk w;
    memset(&w, 0, sizeof w);
    w.want_tag = -1;
    w.fd = fd;
    w.ctx = ctx;
    pthread_mutex_init(&w.send_mu, NULL);
    pthread_mutex_init(&w.mu, NULL);
    pthread_cond_init(&w.cv, NULL);
    ss_hello hello = {(int32_t)getpid(), device};
    if (send_frame(&w, SS_HELLO, &hello, sizeof hello)) return 1;
    wire_hdr h;
    ss_job job;
    if (wire_v1_recv_hdr(fd, &h) || h.type != SS_JOB || h.count != sizeof job || wire_recv_all(fd, &job, sizeof job)) {
        fprintf(stderr, "worker: no job from the master\n");
        return 1;
    }
    const double t_setup0 = now_ms();
    w.hb_ms = job.heartbeat_ms ? job.heartbeat_ms : 50;
    w.comm_timeout_ms = job.comm_timeout_ms;
    const size_t kb = job.key_bytes;
    const int i64 = kb == 8;
    /* the master's chunk replicas: shared memory, pinned here for DMA */
    const size_t shm_bytes = job.n_total > 0 ? job.n_total * kb : 1;
    int sfd = shm_open(job.shm_name, O_RDWR, 0600);
    char *rep = sfd < 0 ? MAP_FAILED : (char *)mmap(NULL, shm_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, sfd, 0);
    if (rep == MAP_FAILED) {
        perror("worker: chunk replicas (shm)");
        return 1;
    }
    close(sfd);
    CHECK(dsort_host_register(ctx, rep, shm_bytes));
    const uint64_t n0 = job.chunk_len;
    void *d_chunk = NULL;
    CHECK(dsort_dev_alloc(ctx, &d_chunk, (n0 ? n0 : 1) * kb));
    char *my_rep = rep + job.chunk_off * kb;
    if (job.source == 2) {
        CHECK(dsort_copy_h2d(ctx, d_chunk, my_rep, n0 * kb));
    } else if (n0) {
        if (job.source == 1) CHECK(dsort_gen_zipf_i64(ctx, (int64_t *)d_chunk, n0, job.seed, job.chunk_off, NULL));
        else if (i64) CHECK(dsort_gen_uniform_i64(ctx, (int64_t *)d_chunk, n0, job.seed, job.chunk_off, NULL));
        else CHECK(dsort_gen_uniform_i32(ctx, (int32_t *)d_chunk, n0, job.seed, job.chunk_off, NULL));
        CHECK(dsort_synchronize(ctx));
        CHECK(dsort_copy_d2h(ctx, my_rep, d_chunk, n0 * kb)); /* the master's replica of this chunk */
    }
    ss_ready ready = {job.rank, 0, n0, 0, 0, 0.0};
    if (n0) {
        if (i64) CHECK(dsort_fingerprint_i64(ctx, (const int64_t *)d_chunk, n0, &ready.fp_sum, &ready.fp_xor));
        else CHECK(dsort_fingerprint_i32(ctx, (const int32_t *)d_chunk, n0, &ready.fp_sum, &ready.fp_xor));
    }
    CHECK(dsort_set_option(ctx, DSORT_OPT_COMM_TIMEOUT_MS, job.comm_timeout_ms));
    CHECK(dsort_set_option(ctx, DSORT_OPT_KILL_IN_EXCHANGE, job.kill_in_exchange));
    dsort_transport tx = {&w, relay_allgather, relay_alltoallv};
    pthread_t rd_th, hb_th;
    pthread_create(&rd_th, NULL, reader_main, &w);
    pthread_create(&hb_th, NULL, heartbeat_main, &w);
    CHECK(comm_up(&w, &job, 0, (int)job.world, (int)job.rank, job.uid, &tx));
    ready.t_setup_ms = now_ms() - t_setup0;
    if (send_frame(&w, SS_READY, &ready, sizeof ready)) return 1;

    pthread_mutex_lock(&w.mu);
    while (!w.go && !w.bye && !w.closed && !w.plan_pending) pthread_cond_wait(&w.cv, &w.mu);
    const int start = w.go;
    pthread_mutex_unlock(&w.mu);
    int exit_code = 0;
    if (start) {
        /* the fault injection of config C5 strikes inside the first epoch's sort (after stage k of
         * the local part: the first partition level, before the exchange; or the second level /
         * tile sort of the received buckets) */
        CHECK(dsort_set_option(ctx, DSORT_OPT_KILL_AFTER_STAGE, job.kill_after_pass));
        if (job.hang_before_exchange) raise(SIGSTOP); /* fault injection: hung, not dead */
        void *d_run = d_chunk; /* the keys this worker owns (unsorted): its chunk, then inherited ones */
        uint64_t run_len = n0;
        uint32_t owned[SS_MAX_CHUNKS];
        uint32_t nowned = 1;
        owned[0] = job.rank;
        double t_rebuild = 0.0;
        for (;;) {
            /* one epoch's exchange over the current communicator */
            const double t_ex = now_ms();
            void *out = NULL;
            size_t nout = 0;
            rc = i64 ? dsort_sample_sort_dev_i64(ctx, (const int64_t *)d_run, run_len, (int64_t **)&out, &nout, NULL)
                     : dsort_sample_sort_dev_i32(ctx, (const int32_t *)d_run, run_len, (int32_t **)&out, &nout, NULL);
            if (!rc) rc = dsort_synchronize(ctx);
            dsort_set_option(ctx, DSORT_OPT_KILL_AFTER_STAGE, -1); /* (the first epoch only) */
            /* the local part of the sort: from the call to the start of the key exchange */
            dsort_stats sst;
            double t_sorted = 0.0;
            if (!rc && !dsort_get_stats(ctx, &sst)) t_sorted = sst.total_ms - sst.exchange_ms - sst.final_merge_ms;
            ss_done done;
            memset(&done, 0, sizeof done);
            done.epoch = w.epoch;
            done.rank = (uint32_t)-1;
            done.status = rc;
            done.run_keys = run_len;
            done.t_local_sort_ms = t_sorted;
            done.t_exchange_ms = now_ms() - t_ex; /* the whole sample sort call */
            done.t_rebuild_ms = t_rebuild;
            if (!rc) {
                if (nout) {
                    if (i64) {
                        CHECK(dsort_count_descents_i64(ctx, (const int64_t *)out, nout, &done.descents));
                        CHECK(dsort_fingerprint_i64(ctx, (const int64_t *)out, nout, &done.fp_sum, &done.fp_xor));
                        int64_t v;
                        CHECK(dsort_copy_d2h(ctx, &v, out, 8));
                        done.first = v;
                        CHECK(dsort_copy_d2h(ctx, &v, (char *)out + (nout - 1) * 8, 8));
                        done.last = v;
                    } else {
                        CHECK(dsort_count_descents_i32(ctx, (const int32_t *)out, nout, &done.descents));
                        CHECK(dsort_fingerprint_i32(ctx, (const int32_t *)out, nout, &done.fp_sum, &done.fp_xor));
                        int32_t v;
                        CHECK(dsort_copy_d2h(ctx, &v, out, 4));
                        done.first = v;
                        CHECK(dsort_copy_d2h(ctx, &v, (char *)out + (nout - 1) * 4, 4));
                        done.last = v;
                    }
                }
                done.n_out = nout;
            }
            if (send_frame(&w, SS_DONE, &done, sizeof done)) {
                exit_code = 1;
                break;
            }
            /* wait for the end of the job, a slice request or a recovery plan */
            ss_plan plan;
            int have_plan = 0;
            for (;;) {
                pthread_mutex_lock(&w.mu);
                while (!w.bye && !w.closed && !w.slice_req && !(w.plan_pending && w.plan.epoch > w.epoch))
                    pthread_cond_wait(&w.cv, &w.mu);
                const int bye = w.bye || w.closed, slice = w.slice_req;
                if (w.plan_pending && w.plan.epoch > w.epoch) {
                    plan = w.plan;
                    have_plan = 1;
                }
                w.slice_req = 0;
                pthread_mutex_unlock(&w.mu);
                if (slice && !rc) {
                    char *hbuf = (char *)malloc(nout * kb + 1);
                    if (!hbuf || dsort_copy_d2h(ctx, hbuf, out, nout * kb)) return 1;
                    send_frame(&w, SS_SLICE, hbuf, nout * kb);
                    free(hbuf);
                    continue;
                }
                if (bye || have_plan) break;
            }
            if (!have_plan) break;
            if (job.kill_in_recovery) raise(SIGKILL); /* fault injection: a second failure during recovery */
            /* recovery epoch: drop the communicator, append the chunks now owned to the keys (from
             * the master's pinned replicas; nothing is sorted here: the next sample sort partitions
             * them with the rest).  A PLAN for a newer epoch (another worker died meanwhile)
             * restarts from that plan: the chunks already added stay owned, the new ones are added. */
            const double t_rb = now_ms();
        rebuild:
            dsort_comm_abort(ctx);
            for (uint32_t i = 0; i < plan.nchunks; ++i) {
                const uint32_t c = plan.chunks[i];
                int have = 0;
                for (uint32_t j = 0; j < nowned; ++j) have |= owned[j] == c;
                if (have) continue;
                uint64_t off, len;
                chunk_range(job.n_total, job.world, c, &off, &len);
                void *d_both = NULL;
                CHECK(dsort_dev_alloc(ctx, &d_both, (run_len + len + 1) * kb));
                CHECK(dsort_copy_d2d(ctx, d_both, d_run, run_len * kb));
                CHECK(dsort_copy_h2d(ctx, (char *)d_both + run_len * kb, rep + off * kb, len * kb)); /* the replica */
                if (d_run != d_chunk) dsort_dev_free(ctx, d_run);
                d_run = d_both;
                run_len += len;
                owned[nowned++] = c;
            }
            rc = comm_up(&w, &job, plan.epoch, (int)plan.world, (int)plan.rank, plan.uid, &tx);
            if (rc == COMM_SUPERSEDED) {
                pthread_mutex_lock(&w.mu);
                plan = w.plan;
                pthread_mutex_unlock(&w.mu);
                goto rebuild;
            }
            t_rebuild = now_ms() - t_rb;
            if (rc) fprintf(stderr, "worker: communicator of epoch %u failed (%d): %s\n", plan.epoch, rc, dsort_last_error(ctx));
        }
        if (d_run != d_chunk) dsort_dev_free(ctx, d_run);
    }
    pthread_mutex_lock(&w.mu);
    w.stop = 1;
    pthread_cond_broadcast(&w.cv);
    pthread_mutex_unlock(&w.mu);
    pthread_join(hb_th, NULL);
    dsort_comm_destroy(ctx);
    shutdown(fd, SHUT_RDWR);
    pthread_join(rd_th, NULL);
    close(fd);
    dsort_dev_free(ctx, d_chunk);
    dsort_host_unregister(ctx, rep);
    munmap(rep, shm_bytes);
    dsort_finalize(ctx);
    return exit_code;
}
