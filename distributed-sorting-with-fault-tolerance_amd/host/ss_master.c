/* ss_master.c -- dsort_master --mode samplesort: the master of the multi-GPU sample sort
 * (server.c's role, protocol in ss.h).
 *
 *   dsort_master --mode samplesort --gpus N [--keys K] [--dtype i32|i64] [--dist uniform|zipf]
 *                [--input FILE] [--transport rccl|relay] [--devices LIST|share] [--worker PATH]
 *                [--kill-rank R [--kill-stage sort|exchange] [--kill-after-stage K]
 *                 [--kill-exchange-stage 1|2]] [--kill-in-recovery R2] [--reassign first-live|next-live]
 *                [--heartbeat-ms MS] [--timeout-ms MS] [--comm-timeout-ms MS] [--seed S]
 *                [--output FILE]
 *
 * 1. The chunk replicas (server.c:185-216's chunks[]): one shared-memory segment of all keys,
 *    filled by the workers from the GPU generator (synthetic input) or by the master from --input
 *    (text, "%d" tokens as server.c:177-182).  The workers map and pin it.
 * 2. Spawns N workers (dsort_worker --mode samplesort), one per GPU (--devices share: all on GPU
 *    0, relay transport); worker identity is accept order (server.c:148-157).
 * 3. Creates the RCCL unique id and ships it in every worker's JOB frame over the TCP control
 *    socket; waits for every READY, sends GO (the timed region starts).
 * 4. Supervises: a worker whose socket closes, whose process exits, or whose heartbeat is older
 *    than --timeout-ms (then killed) is dead.  Its chunks go to survivors by the reference's rule
 *    (first-live: the first live worker, server.c:368-384; next-live: the next one after it), and
 *    every survivor gets a PLAN for a new epoch: new world, new rank, new unique id, the chunks it
 *    owns.  The relay transport's all-gathers and all-to-alls are served here.
 * 5. When every live worker reported DONE for the current epoch: verification (no descents, the
 *    multiset fingerprint of the outputs equals the inputs', rank boundaries ordered), one JSON
 *    line on stdout, optional --output (the slices gathered in rank order, "%d\n" text as
 *    server.c:517-519), BYE. */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "dsort.h"
#include "ss.h"
#include "wire.h"

long master_parse_keys(const char *t, size_t len, int32_t **out); /* master.c */

typedef struct wstate {
    int fd;
    pid_t pid;
    int alive;
    double last_seen;
    int ready, done;
    double fail_at; /* DONE of the current epoch with a non-zero status: when it came */
    ss_ready rd;
    ss_done dn;
    /* relay request of the current epoch */
    int has_req;
    int32_t req_tag;
    uint16_t req_type;
    char *req;
    size_t req_len;
    int new_rank;
} wstate;

typedef struct mopt {
    int n;
    uint64_t keys;
    int key_bytes;
    int dist;  /* 0 uniform, 1 zipf */
    const char *input;
    int transport;  /* 0 rccl, 1 relay */
    int share;      /* all workers on GPU 0 */
    int devices[SS_MAX_WORKERS];
    const char *worker;
    int kill_rank, kill_after_pass, kill_exchange_stage, kill_in_recovery, hang_rank;
    int next_live;
    int hb_ms, timeout_ms;
    int64_t comm_timeout_ms;
    uint64_t seed;
    const char *output;
} mopt;

/* A DONE with an error status waits this long for a peer's death that would explain it (the
 * master sees a death within milliseconds: socket EOF, process exit) before the worker is fenced. */
#define SS_FAIL_GRACE_MS 1000.0
#define SS_SILENT_MIN_MS 500.0  /* a peer unheard for this long (or 20 heartbeats) counts as hung */

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

static int send_to(wstate *w, uint16_t type, int32_t status, const void *p, size_t bytes) {
    if (!w->alive) return -1;
    return wire_v1_send(w->fd, type, 1, status, p, bytes);
}

static void usage_ss(void) {
    fprintf(stderr,
            "usage: dsort_master --mode samplesort --gpus N [--keys K] [--dtype i32|i64] [--dist uniform|zipf]\n"
            "       [--input FILE] [--transport rccl|relay] [--devices 0,1,..|share] [--worker PATH]\n"
            "       [--kill-rank R [--kill-stage sort|exchange] [--kill-after-stage K] [--kill-exchange-stage 1|2]]\n"
            "       [--kill-in-recovery R2] [--hang-rank R3]\n"
            "       [--reassign first-live|next-live] [--heartbeat-ms MS] [--timeout-ms MS]\n"
            "       [--comm-timeout-ms MS] [--seed S] [--output FILE]\n");
    exit(2);
}

/* chunk owners after the deaths in `alive`: every chunk of a dead owner moves by the rule */
static void reassign(int n, const int *alive, int *owner, int next_live) {
    int first = -1;
    for (int i = 0; i < n; ++i)
        if (alive[i]) {
            first = i;
            break;
        }
    for (int c = 0; c < n; ++c) {
        const int o = owner[c];
        if (alive[o]) continue;
        int to = first;
        if (next_live) {
            for (int k = 1; k < n; ++k)
                if (alive[(o + k) % n]) {
                    to = (o + k) % n;
                    break;
                }
        }
        owner[c] = to;
    }
}

int samplesort_master(int argc, char **argv, const char *argv0) {
    mopt o;
    memset(&o, 0, sizeof o);
    o.n = 1;
    o.keys = 1u << 20;
    o.key_bytes = 4;
    o.kill_rank = -1;
    o.kill_after_pass = -1;
    o.kill_exchange_stage = -1;
    o.kill_in_recovery = -1;
    o.hang_rank = -1;
    o.hb_ms = 50;
    o.timeout_ms = 5000;
    o.seed = 0x5EED2026ull;
    int kill_stage_exchange = 0, have_devices = 0;
    for (int i = 0; i < argc; ++i) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : NULL;
#define NEXT() (v ? (++i, v) : (usage_ss(), ""))
        if (!strcmp(a, "--mode")) NEXT();
        else if (!strcmp(a, "--gpus")) o.n = atoi(NEXT());
        else if (!strcmp(a, "--keys")) o.keys = strtoull(NEXT(), NULL, 0);
        else if (!strcmp(a, "--dtype")) o.key_bytes = !strcmp(NEXT(), "i64") ? 8 : 4;
        else if (!strcmp(a, "--dist")) o.dist = !strcmp(NEXT(), "zipf");
        else if (!strcmp(a, "--input")) o.input = NEXT();
        else if (!strcmp(a, "--transport")) o.transport = !strcmp(NEXT(), "relay");
        else if (!strcmp(a, "--devices")) {
            const char *d = NEXT();
            if (!strcmp(d, "share")) o.share = 1;
            else {
                int k = 0;
                for (const char *p = d; *p && k < SS_MAX_WORKERS; ++k) {
                    o.devices[k] = atoi(p);
                    p = strchr(p, ',');
                    if (!p) break;
                    ++p;
                }
                have_devices = 1;
            }
        } else if (!strcmp(a, "--worker")) o.worker = NEXT();
        else if (!strcmp(a, "--kill-rank")) o.kill_rank = atoi(NEXT());
        else if (!strcmp(a, "--kill-stage")) kill_stage_exchange = !strcmp(NEXT(), "exchange");
        else if (!strcmp(a, "--kill-after-stage")) o.kill_after_pass = atoi(NEXT());
        else if (!strcmp(a, "--kill-in-recovery")) o.kill_in_recovery = atoi(NEXT());
        else if (!strcmp(a, "--hang-rank")) o.hang_rank = atoi(NEXT());
        else if (!strcmp(a, "--kill-exchange-stage")) o.kill_exchange_stage = atoi(NEXT());
        else if (!strcmp(a, "--reassign")) o.next_live = !strcmp(NEXT(), "next-live");
        else if (!strcmp(a, "--heartbeat-ms")) o.hb_ms = atoi(NEXT());
        else if (!strcmp(a, "--timeout-ms")) o.timeout_ms = atoi(NEXT());
        else if (!strcmp(a, "--comm-timeout-ms")) o.comm_timeout_ms = atoll(NEXT());
        else if (!strcmp(a, "--seed")) o.seed = strtoull(NEXT(), NULL, 0);
        else if (!strcmp(a, "--output")) o.output = NEXT();
        else usage_ss();
#undef NEXT
    }
    if (o.n < 1 || o.n > SS_MAX_WORKERS) usage_ss();
    if (o.dist == 1 && o.key_bytes != 8) {
        fprintf(stderr, "master: zipf keys are int64 (--dtype i64)\n");
        return 2;
    }
    if (o.kill_rank >= 0) {
        if (kill_stage_exchange && o.kill_exchange_stage < 0) o.kill_exchange_stage = 2;
        if (!kill_stage_exchange && o.kill_after_pass < 0) o.kill_after_pass = 0;
        if (kill_stage_exchange) o.kill_after_pass = -1;
        else o.kill_exchange_stage = -1;
    }
    if (o.hang_rank >= o.n) usage_ss();
    if (o.kill_rank >= o.n || o.kill_in_recovery >= o.n || (o.kill_in_recovery >= 0 && o.kill_in_recovery == o.kill_rank)) {
        fprintf(stderr, "master: --kill-rank / --kill-in-recovery must name two different workers of %d\n", o.n);
        return 2;
    }
    if (!have_devices)
        for (int i = 0; i < o.n; ++i) o.devices[i] = o.share ? 0 : i;
    if (o.share) o.transport = 1; /* RCCL needs one GPU per rank */
    signal(SIGPIPE, SIG_IGN);

    /* 1. the chunk replicas */
    int32_t *parsed = NULL;
    if (o.input) {
        FILE *f = fopen(o.input, "rb");
        if (!f) {
            perror("master: --input");
            return 1;
        }
        fseek(f, 0, SEEK_END);
        const long len = ftell(f);
        fseek(f, 0, SEEK_SET);
        char *text = (char *)malloc((size_t)len + 1);
        if (!text || fread(text, 1, (size_t)len, f) != (size_t)len) return 1;
        text[len] = 0;
        fclose(f);
        const long nk = master_parse_keys(text, (size_t)len, &parsed);
        free(text);
        if (nk < 0) {
            fprintf(stderr, "master: %s contains a non-integer token\n", o.input);
            return 1;
        }
        o.keys = (uint64_t)nk;
        o.key_bytes = 4;
    }
    if (o.kill_rank >= 0 && o.kill_after_pass >= 0) {
        /* a kill stage the victim's local sort never reaches would be a fault run without a fault */
        const uint64_t q = o.keys / (uint64_t)o.n, rm = o.keys % (uint64_t)o.n;
        const uint64_t len = q + ((uint64_t)o.kill_rank < rm ? 1 : 0);
        int stages = 0;
        if (dsort_sample_sort_stages(NULL, o.keys, o.n, o.kill_rank, o.key_bytes, &stages) ||
            o.kill_after_pass >= stages) {
            fprintf(stderr, "master: --kill-after-stage %d: the sort of worker %d (%llu keys) has %d stages "
                    "(kill points 0..%d)\n", o.kill_after_pass, o.kill_rank, (unsigned long long)len, stages,
                    stages - 1);
            free(parsed);
            return 2;
        }
    }
    const size_t kb = (size_t)o.key_bytes;
    const size_t shm_bytes = o.keys > 0 ? o.keys * kb : 1;
    char shm_name[64];
    static int shm_seq;
    snprintf(shm_name, sizeof shm_name, "/dsort-ss-%d-%d", (int)getpid(), shm_seq++);
    int sfd = shm_open(shm_name, O_RDWR | O_CREAT | O_EXCL, 0600);
    if (sfd < 0 || ftruncate(sfd, (off_t)shm_bytes)) {
        perror("master: shm");
        return 1;
    }
    char *rep = (char *)mmap(NULL, shm_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, sfd, 0);
    close(sfd);
    if (rep == MAP_FAILED) {
        perror("master: mmap");
        shm_unlink(shm_name);
        return 1;
    }
    if (parsed) {
        memcpy(rep, parsed, o.keys * kb);
        free(parsed);
    }

    /* 2. listen, spawn, accept */
    int lfd = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    struct sockaddr_in addr;
    memset(&addr, 0, sizeof addr);
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    addr.sin_port = 0;
    socklen_t al = sizeof addr;
    if (bind(lfd, (struct sockaddr *)&addr, sizeof addr) || listen(lfd, o.n) ||
        getsockname(lfd, (struct sockaddr *)&addr, &al)) {
        perror("master: listen");
        return 1;
    }
    const int port = ntohs(addr.sin_port);
    char wpath[4096];
    if (o.worker) snprintf(wpath, sizeof wpath, "%s", o.worker);
    else {
        snprintf(wpath, sizeof wpath, "%s", argv0);
        char *sl = strrchr(wpath, '/');
        if (sl) snprintf(sl + 1, sizeof wpath - (size_t)(sl + 1 - wpath), "dsort_worker");
        else snprintf(wpath, sizeof wpath, "dsort_worker");
    }
    static wstate W[SS_MAX_WORKERS];
    pid_t kids[SS_MAX_WORKERS];
    for (int r = 0; r < o.n; ++r) {
        char dev[16], conn[64];
        snprintf(dev, sizeof dev, "%d", o.devices[r]);
        snprintf(conn, sizeof conn, "127.0.0.1:%d", port);
        const pid_t p = fork();
        if (p == 0) {
            close(lfd);
            execl(wpath, wpath, "--mode", "samplesort", "--connect", conn, "--device", dev, (char *)NULL);
            perror("master: exec worker");
            _exit(127);
        }
        kids[r] = p;
    }
    const double t_start = now_ms();
    for (int r = 0; r < o.n; ++r) {
        struct pollfd pf = {lfd, POLLIN, 0};
        int ok = 0;
        while (now_ms() - t_start < 120000) {
            if (poll(&pf, 1, 100) > 0) {
                ok = 1;
                break;
            }
            int st;
            for (int k = 0; k < o.n; ++k)
                if (kids[k] > 0 && waitpid(kids[k], &st, WNOHANG) == kids[k]) {
                    fprintf(stderr, "master: worker process %d exited during start-up\n", (int)kids[k]);
                    kids[k] = -1;
                }
        }
        if (!ok) {
            fprintf(stderr, "master: only %d of %d workers connected\n", r, o.n);
            goto fail;
        }
        W[r].fd = accept(lfd, NULL, NULL);
        wire_set_nodelay(W[r].fd);
        W[r].alive = 1;
        W[r].last_seen = now_ms();
        wire_hdr h;
        ss_hello hello;
        if (wire_v1_recv_hdr(W[r].fd, &h) || h.type != SS_HELLO || h.count != sizeof hello ||
            wire_recv_all(W[r].fd, &hello, sizeof hello)) {
            fprintf(stderr, "master: bad hello\n");
            goto fail;
        }
        W[r].pid = hello.pid;
    }

    /* 3. jobs (the RCCL unique id goes over this TCP control socket, dsort.h) */
    {
        char uid[DSORT_UNIQUE_ID_BYTES];
        memset(uid, 0, sizeof uid);
        if (o.transport == 0 && dsort_comm_unique_id(uid)) {
            fprintf(stderr, "master: dsort_comm_unique_id failed\n");
            goto fail;
        }
        for (int r = 0; r < o.n; ++r) {
            ss_job j;
            memset(&j, 0, sizeof j);
            j.epoch = 0;
            j.world = (uint32_t)o.n;
            j.rank = (uint32_t)r;
            j.key_bytes = (uint32_t)kb;
            j.n_total = o.keys;
            const uint64_t q = o.keys / (uint64_t)o.n, rm = o.keys % (uint64_t)o.n;
            j.chunk_len = q + ((uint64_t)r < rm ? 1 : 0);
            j.chunk_off = (uint64_t)r * q + ((uint64_t)r < rm ? (uint64_t)r : rm);
            j.seed = o.seed;
            j.transport = (uint32_t)o.transport;
            j.source = o.input ? 2u : (uint32_t)o.dist;
            j.kill_after_pass = r == o.kill_rank ? o.kill_after_pass : -1;
            j.kill_in_exchange = r == o.kill_rank ? o.kill_exchange_stage : -1;
            j.kill_in_recovery = r == o.kill_in_recovery ? 1 : 0;
            j.hang_before_exchange = r == o.hang_rank ? 1 : 0;
            j.comm_timeout_ms = o.comm_timeout_ms;
            j.heartbeat_ms = (uint32_t)o.hb_ms;
            snprintf(j.shm_name, sizeof j.shm_name, "%s", shm_name);
            memcpy(j.uid, uid, sizeof j.uid);
            if (send_to(&W[r], SS_JOB, 0, &j, sizeof j)) goto fail;
        }
    }

    /* 4. supervise */
    {
        int owner[SS_MAX_CHUNKS], alive[SS_MAX_WORKERS], dead_list[SS_MAX_WORKERS], ndead = 0;
        for (int r = 0; r < o.n; ++r) {
            owner[r] = r;
            alive[r] = 1;
        }
        uint32_t epoch = 0;
        int go_sent = 0, finished = 0;
        double t_go = 0, t_fault = -1, t_plan = -1, t_end = 0;
        for (;;) {
            struct pollfd pf[SS_MAX_WORKERS];
            int idx[SS_MAX_WORKERS], np = 0;
            for (int r = 0; r < o.n; ++r)
                if (W[r].alive) {
                    pf[np].fd = W[r].fd;
                    pf[np].events = POLLIN;
                    pf[np].revents = 0;
                    idx[np++] = r;
                }
            if (np == 0) break;
            poll(pf, (nfds_t)np, 2);
            const double now = now_ms();
            int newly = 0;
            for (int k = 0; k < np; ++k) {
                if (!pf[k].revents) continue;
                wstate *w = &W[idx[k]];
                wire_hdr h;
                char *buf = NULL;
                int bad = wire_v1_recv_hdr(w->fd, &h);
                if (!bad && h.count) {
                    buf = (char *)malloc(h.count);
                    bad = !buf || wire_recv_all(w->fd, buf, h.count);
                }
                if (bad) { /* recv <= 0: a dead worker (server.c:421) */
                    free(buf);
                    w->alive = 0;
                    newly = 1;
                    continue;
                }
                w->last_seen = now;
                if (h.type == SS_READY && h.count == sizeof(ss_ready)) {
                    memcpy(&w->rd, buf, sizeof(ss_ready));
                    w->ready = 1;
                } else if (h.type == SS_DONE && h.count == sizeof(ss_done)) {
                    ss_done d;
                    memcpy(&d, buf, sizeof d);
                    if (d.epoch == epoch) {
                        w->dn = d;
                        w->done = 1;
                        if (d.status != 0 && w->fail_at <= 0) w->fail_at = now;
                        if (now - t_go > t_end) t_end = now - t_go;
                    }
                } else if ((h.type == SS_RELAY_AG || h.type == SS_RELAY_A2A) && (uint32_t)h.status >> 20 == epoch) {
                    free(w->req);
                    w->req = buf;
                    buf = NULL;
                    w->req_len = h.count;
                    w->req_tag = h.status;
                    w->req_type = h.type;
                    w->has_req = 1;
                }
                free(buf);
            }
            /* process exits and stale heartbeats (a hung worker is killed first: fencing) */
            for (int r = 0; r < o.n; ++r) {
                if (!W[r].alive) continue;
                int st;
                /* W[r].pid is the process that connected as rank r (accept order, not fork order) */
                if (waitpid(W[r].pid, &st, WNOHANG) == W[r].pid) {
                    fprintf(stderr, "master: worker %d (pid %d) exited (%s %d)\n", r + 1, (int)W[r].pid,
                            WIFSIGNALED(st) ? "signal" : "status", WIFSIGNALED(st) ? WTERMSIG(st) : WEXITSTATUS(st));
                    for (int k = 0; k < o.n; ++k)
                        if (kids[k] == W[r].pid) kids[k] = -1;
                    W[r].alive = 0;
                    newly = 1;
                } else if (go_sent && o.timeout_ms > 0 && now - W[r].last_seen > o.timeout_ms) {
                    kill(W[r].pid, SIGKILL);
                    W[r].alive = 0;
                    newly = 1;
                }
            }
            /* A failed exchange (DONE with DSORT_ECOMM / DSORT_ETIMEOUT) that no peer's death has
             * explained within the grace period.  A hung peer (stopped, or stuck so that even its
             * heartbeat thread is silent) makes every survivor's exchange time out: fence the
             * peers that have been silent for `silent` first and keep the reporters (they get the
             * next epoch's plan).  Only when every peer is heard from is the reporter itself the
             * suspect: fence it. */
            if (go_sent) {
                int due = 0;
                for (int r = 0; r < o.n; ++r)
                    if (W[r].alive && W[r].fail_at > 0 && now - W[r].fail_at > SS_FAIL_GRACE_MS) due = 1;
                if (due) {
                    const double silent = 20.0 * o.hb_ms > SS_SILENT_MIN_MS ? 20.0 * o.hb_ms : SS_SILENT_MIN_MS;
                    int fenced_silent = 0;
                    for (int r = 0; r < o.n; ++r)
                        if (W[r].alive && W[r].fail_at <= 0 && now - W[r].last_seen > silent) {
                            fprintf(stderr, "master: worker %d silent for %.0f ms while peers' exchanges failed; "
                                            "fenced\n", r + 1, now - W[r].last_seen);
                            kill(W[r].pid, SIGKILL);
                            W[r].alive = 0;
                            newly = fenced_silent = 1;
                        }
                    for (int r = 0; r < o.n && !fenced_silent; ++r)
                        if (W[r].alive && W[r].fail_at > 0 && now - W[r].fail_at > SS_FAIL_GRACE_MS) {
                            fprintf(stderr, "master: worker %d reported status %d for epoch %u; fenced\n", r + 1,
                                    W[r].dn.status, epoch);
                            kill(W[r].pid, SIGKILL);
                            W[r].alive = 0;
                            newly = 1;
                        }
                }
            }
            if (newly) {
                int any_new = 0;
                for (int r = 0; r < o.n; ++r)
                    if (alive[r] && !W[r].alive) {
                        alive[r] = 0;
                        dead_list[ndead++] = r;
                        any_new = 1;
                        close(W[r].fd);
                    }
                if (any_new) {
                    if (!go_sent) {
                        fprintf(stderr, "master: a worker died during start-up\n");
                        goto fail;
                    }
                    if (t_fault < 0) t_fault = now - t_go;
                    int live = 0;
                    for (int r = 0; r < o.n; ++r) live += alive[r];
                    if (live == 0) {
                        printf("No available worker nodes to handle the chunks.\n"); /* server.c:387-389 */
                        goto fail;
                    }
                    reassign(o.n, alive, owner, o.next_live);
                    ++epoch;
                    char uid[DSORT_UNIQUE_ID_BYTES];
                    memset(uid, 0, sizeof uid);
                    if (o.transport == 0 && dsort_comm_unique_id(uid)) goto fail;
                    int nr = 0;
                    for (int r = 0; r < o.n; ++r) {
                        if (!alive[r]) continue;
                        ss_plan p;
                        memset(&p, 0, sizeof p);
                        p.epoch = epoch;
                        p.world = (uint32_t)live;
                        p.rank = (uint32_t)nr;
                        W[r].new_rank = nr++;
                        for (int c = 0; c < o.n; ++c)
                            if (owner[c] == r) p.chunks[p.nchunks++] = (uint32_t)c;
                        memcpy(p.uid, uid, sizeof p.uid);
                        W[r].done = 0;
                        W[r].fail_at = 0;
                        W[r].has_req = 0;
                        send_to(&W[r], SS_PLAN, 0, &p, sizeof p);
                        printf("Reassigning: epoch %u, worker %d now rank %u of %d, chunks", epoch, r + 1, p.rank, live);
                        for (uint32_t c = 0; c < p.nchunks; ++c) printf(" %u", p.chunks[c] + 1);
                        printf("\n");
                    }
                    if (t_plan < 0) t_plan = now_ms() - t_go;
                    fflush(stdout);
                }
            }
            if (!go_sent) {
                int all = 1;
                for (int r = 0; r < o.n; ++r) all &= W[r].ready;
                if (all) {
                    t_go = now_ms();
                    for (int r = 0; r < o.n; ++r) {
                        W[r].last_seen = t_go;
                        W[r].new_rank = r;
                        send_to(&W[r], SS_GO, 0, NULL, 0);
                    }
                    go_sent = 1;
                }
                if (now_ms() - t_start > 300000) {
                    fprintf(stderr, "master: workers did not get ready\n");
                    goto fail;
                }
                continue;
            }
            /* relay: answer once every live rank of the epoch posted the same request */
            if (o.transport == 1) {
                int all = 1, tag = -1;
                uint16_t type = 0;
                for (int r = 0; r < o.n && all; ++r) {
                    if (!alive[r]) continue;
                    if (!W[r].has_req) all = 0;
                    else if (tag < 0) {
                        tag = W[r].req_tag;
                        type = W[r].req_type;
                    } else if (W[r].req_tag != tag || W[r].req_type != type) all = 0;
                }
                if (all && tag >= 0) {
                    int order[SS_MAX_WORKERS], P = 0;
                    for (int r = 0; r < o.n; ++r)
                        if (alive[r]) order[W[r].new_rank] = r, ++P;
                    if (type == SS_RELAY_AG) {
                        size_t tot = 0;
                        for (int q = 0; q < P; ++q) tot += W[order[q]].req_len;
                        char *resp = (char *)malloc(tot + 1);
                        size_t off = 0;
                        for (int q = 0; q < P; ++q) {
                            memcpy(resp + off, W[order[q]].req, W[order[q]].req_len);
                            off += W[order[q]].req_len;
                        }
                        for (int q = 0; q < P; ++q) send_to(&W[order[q]], SS_RELAY_RESP, tag, resp, tot);
                        free(resp);
                    } else {
                        for (int d = 0; d < P; ++d) {
                            size_t tot = (size_t)P * 8;
                            for (int s = 0; s < P; ++s) {
                                uint64_t c;
                                memcpy(&c, W[order[s]].req + (size_t)d * 8, 8);
                                tot += c;
                            }
                            char *resp = (char *)malloc(tot + 1);
                            size_t off = (size_t)P * 8;
                            for (int s = 0; s < P; ++s) {
                                const char *rq = W[order[s]].req;
                                uint64_t c, pos = (uint64_t)P * 8;
                                memcpy(&c, rq + (size_t)d * 8, 8);
                                for (int e = 0; e < d; ++e) {
                                    uint64_t ce;
                                    memcpy(&ce, rq + (size_t)e * 8, 8);
                                    pos += ce;
                                }
                                memcpy(resp + (size_t)s * 8, &c, 8);
                                if (c) memcpy(resp + off, rq + pos, c);
                                off += c;
                            }
                            send_to(&W[order[d]], SS_RELAY_RESP, tag, resp, tot);
                            free(resp);
                        }
                    }
                    for (int r = 0; r < o.n; ++r)
                        if (alive[r]) W[r].has_req = 0;
                }
            }
            if (now_ms() - t_go > 900000) {
                fprintf(stderr, "master: the sort did not finish within 900 s\n");
                goto fail;
            }
            int all_done = 1;
            for (int r = 0; r < o.n; ++r)
                if (alive[r]) all_done &= W[r].done && W[r].dn.status == 0;
            if (all_done) {
                finished = 1;
                break;
            }
        }
        if (!finished) goto fail;

        /* 5. verification and report */
        int order[SS_MAX_WORKERS], P = 0;
        for (int r = 0; r < o.n; ++r)
            if (alive[r]) order[W[r].new_rank] = r, ++P;
        const uint64_t M = ~0ull;
        uint64_t fin_s = 0, fin_x = 0, fout_s = 0, fout_x = 0, nsum = 0, desc = 0;
        for (int r = 0; r < o.n; ++r) {
            fin_s += W[r].rd.fp_sum;
            fin_x ^= W[r].rd.fp_xor;
        }
        int bounds_ok = 1, have_prev = 0;
        int64_t prev_last = 0;
        double t_rebuild = 0, t_local = 0;
        for (int q = 0; q < P; ++q) {
            const ss_done *d = &W[order[q]].dn;
            fout_s += d->fp_sum;
            fout_x ^= d->fp_xor;
            nsum += d->n_out;
            desc += d->descents;
            if (d->t_rebuild_ms > t_rebuild) t_rebuild = d->t_rebuild_ms;
            if (d->t_local_sort_ms > t_local) t_local = d->t_local_sort_ms;
            if (d->n_out) {
                if (have_prev && prev_last > d->first) bounds_ok = 0;
                prev_last = d->last;
                have_prev = 1;
            }
        }
        const int ok = desc == 0 && nsum == o.keys && (fin_s & M) == (fout_s & M) && fin_x == fout_x && bounds_ok;
        int out_ok = 1;
        if (o.output) {
            char *all = (char *)malloc(o.keys * kb + 1);
            size_t off = 0;
            for (int q = 0; q < P && all; ++q) {
                wstate *w = &W[order[q]];
                wire_hdr h;
                if (send_to(w, SS_GET_SLICE, 0, NULL, 0)) out_ok = 0;
                for (;;) { /* skip heartbeats */
                    if (wire_v1_recv_hdr(w->fd, &h)) {
                        out_ok = 0;
                        break;
                    }
                    if (h.type == SS_SLICE) break;
                    char tmp[256];
                    for (uint64_t left = h.count; left;) {
                        const size_t m = left < sizeof tmp ? (size_t)left : sizeof tmp;
                        if (wire_recv_all(w->fd, tmp, m)) break;
                        left -= m;
                    }
                }
                if (!out_ok || off + h.count > o.keys * kb || wire_recv_all(w->fd, all + off, h.count)) {
                    out_ok = 0;
                    break;
                }
                off += h.count;
            }
            if (out_ok && off == o.keys * kb) {
                if (kb == 4) out_ok = dsort_write_text_i32(o.output, (const int32_t *)all, o.keys) == 0;
                else {
                    FILE *f = fopen(o.output, "wb");
                    out_ok = f && fwrite(all, 1, off, f) == off;
                    if (f) fclose(f);
                }
            } else {
                out_ok = 0;
            }
            free(all);
        }
        printf("{\"ss_result\": true, \"ok\": %s, \"world\": %d, \"survivors\": %d, \"n\": %llu, \"key_bytes\": %d, "
               "\"transport\": \"%s\", \"epochs\": %u, \"dead\": [",
               ok && out_ok ? "true" : "false", o.n, P, (unsigned long long)o.keys, (int)kb,
               o.transport ? "relay" : "rccl", epoch + 1);
        for (int i = 0; i < ndead; ++i) printf("%s%d", i ? ", " : "", dead_list[i]);
        printf("], \"owners\": [");
        for (int c = 0; c < o.n; ++c) printf("%s%d", c ? ", " : "", owner[c]);
        printf("], \"slices\": [");
        for (int q = 0; q < P; ++q) printf("%s%llu", q ? ", " : "", (unsigned long long)W[order[q]].dn.n_out);
        printf("], \"t_end_ms\": %.3f, \"t_local_sort_ms\": %.3f, \"t_fault_seen_ms\": %.3f, "
               "\"t_survivors_notified_ms\": %.3f, \"t_rebuild_ms\": %.3f, \"output_written\": %s}\n",
               t_end, t_local, t_fault, t_plan, t_rebuild, o.output ? (out_ok ? "true" : "false") : "null");
        fflush(stdout);
        for (int r = 0; r < o.n; ++r) send_to(&W[r], SS_BYE, 0, NULL, 0);
        for (int r = 0; r < o.n; ++r) {
            if (kids[r] <= 0) continue;
            int st;
            for (int t = 0; t < 3000 && waitpid(kids[r], &st, WNOHANG) == 0; ++t) usleep(10000);
            if (kill(kids[r], 0) == 0) {
                kill(kids[r], SIGKILL);
                waitpid(kids[r], &st, 0);
            }
        }
        munmap(rep, shm_bytes);
        shm_unlink(shm_name);
        close(lfd);
        return ok && out_ok ? 0 : 1;
    }
fail:
    for (int r = 0; r < o.n; ++r)
        if (kids[r] > 0) {
            kill(kids[r], SIGKILL);
            int st;
            waitpid(kids[r], &st, 0);
        }
    munmap(rep, shm_bytes);
    shm_unlink(shm_name);
    close(lfd);
    printf("{\"ss_result\": true, \"ok\": false}\n");
    return 1;
}
