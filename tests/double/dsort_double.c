/* dsort_double.c -- TEST DOUBLE of the libdsort C ABI for the CPU-only plumbing tests.
 *
 * NOT PRODUCT CODE.  It implements just the entry points the C master/worker call
 * (init/finalize/last_error/sort/merge/write_text) on the CPU by delegating to the oracle, so
 * tests/test_plumbing.py can exercise the wire protocol, the reference interop and the fault
 * tolerance paths in a container without a GPU.  The real libdsort.so (HIP, gfx950) is used by
 * the same tests on the GPU box (tests marked gpu); it never falls back to this file.
 * Built by the tests into tests/double/build/libdsort.so and selected with LD_LIBRARY_PATH.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/dsort.h"
#include "../../oracle/oracle.h"

struct dsort_ctx {
    int device;
};

int dsort_init(dsort_ctx **ctx, int device) {
    *ctx = (dsort_ctx *)calloc(1, sizeof(dsort_ctx));
    if (!*ctx) return DSORT_ENOMEM;
    (*ctx)->device = device;
    return getenv("DSORT_DOUBLE_NO_GPU") ? DSORT_ENODEV : DSORT_OK;
}

int dsort_finalize(dsort_ctx *ctx) {
    free(ctx);
    return DSORT_OK;
}

const char *dsort_last_error(const dsort_ctx *ctx) {
    (void)ctx;
    return "test double";
}

int dsort_sort_i32(dsort_ctx *ctx, int32_t *k, size_t n) {
    (void)ctx;
    return oracle_merge_sort_i32(k, n) ? DSORT_ENOMEM : DSORT_OK;
}

int dsort_sort_i64(dsort_ctx *ctx, int64_t *k, size_t n) {
    (void)ctx;
    return oracle_merge_sort_i64(k, n) ? DSORT_ENOMEM : DSORT_OK;
}

int dsort_merge_i32(dsort_ctx *ctx, const int32_t *const runs[], const size_t lens[], int k, int32_t *out) {
    (void)ctx;
    oracle_merge_runs_i32(k, runs, lens, out);
    return DSORT_OK;
}

int dsort_write_text_i32(const char *path, const int32_t *keys, size_t n) {
    FILE *f = fopen(path, "w");
    if (!f) return DSORT_EINVAL;
    char *buf = (char *)malloc(12 * n + 1);
    long len = buf ? oracle_format_i32(keys, n, buf, 12 * n + 1) : -1;
    int ok = len >= 0 && fwrite(buf, 1, (size_t)len, f) == (size_t)len;
    free(buf);
    return (fclose(f) == 0 && ok) ? DSORT_OK : DSORT_EINVAL;
}

/* CPU stand-ins of the GPU text codec (host-buffer forms), for the master's plumbing tests. */
int dsort_parse_text_i32(dsort_ctx *ctx, const char *text, size_t len, int32_t *keys, size_t cap,
                         size_t *n_out) {
    (void)ctx;
    long n = oracle_parse_i32(text, len, keys, cap);
    if (n < 0) return DSORT_EINVAL;
    *n_out = (size_t)n;
    return DSORT_OK;
}

int dsort_format_text_i32(dsort_ctx *ctx, const int32_t *keys, size_t n, char *text, size_t cap,
                          size_t *len_out) {
    (void)ctx;
    long len = oracle_format_i32(keys, n, text, cap);
    if (len < 0) return DSORT_EINVAL;
    *len_out = (size_t)len;
    return DSORT_OK;
}

/* ---- the subset the C sample sort (host/ss_master.c, host/ss_worker.c) calls ----------------
 * "Device" memory is host memory here.  The sample sort follows the library's rules (regular
 * samples at (j+1)n/(s+1), splitters at the P-quantiles of the (value, rank, index) order, cuts
 * by the composite rule, source-order merge) through the caller's transport, so the C master's
 * supervision, relay and recovery run on CPU exactly as on the GPU box. */
#include <signal.h>

static int g_kill_after_pass = -1, g_kill_in_exchange = -1;
static int g_nranks = 1, g_rank = 0, g_has_tx = 0, g_abort = 0;
static dsort_transport g_tx;
static void *g_out = NULL;

int dsort_set_option(dsort_ctx *ctx, int option, int64_t v) {
    (void)ctx;
    if (option == DSORT_OPT_KILL_AFTER_STAGE) g_kill_after_pass = (int)v;
    else if (option == DSORT_OPT_KILL_IN_EXCHANGE) g_kill_in_exchange = (int)v;
    else if (option < 1 || option > 12) return DSORT_EINVAL;
    return DSORT_OK;
}
int dsort_get_option(const dsort_ctx *ctx, int option, int64_t *v) {
    (void)ctx;
    *v = option == DSORT_OPT_KILL_AFTER_STAGE ? g_kill_after_pass : option == DSORT_OPT_KILL_IN_EXCHANGE ? g_kill_in_exchange : 0;
    return DSORT_OK;
}
int dsort_synchronize(dsort_ctx *ctx) { (void)ctx; return DSORT_OK; }
int dsort_get_stats(const dsort_ctx *ctx, dsort_stats *out) {
    (void)ctx;
    if (!out) return DSORT_EINVAL;
    memset(out, 0, sizeof *out); /* (no device timings on the CPU) */
    return DSORT_OK;
}
int dsort_dev_alloc(dsort_ctx *ctx, void **p, size_t bytes) { (void)ctx; *p = malloc(bytes ? bytes : 1); return *p ? DSORT_OK : DSORT_ENOMEM; }
int dsort_dev_free(dsort_ctx *ctx, void *p) { (void)ctx; free(p); return DSORT_OK; }
int dsort_copy_h2d(dsort_ctx *ctx, void *d, const void *h, size_t b) { (void)ctx; if (b) memmove(d, h, b); return DSORT_OK; }
int dsort_copy_d2h(dsort_ctx *ctx, void *h, const void *d, size_t b) { (void)ctx; if (b) memmove(h, d, b); return DSORT_OK; }
int dsort_copy_d2d(dsort_ctx *ctx, void *d, const void *s, size_t b) { (void)ctx; if (b) memmove(d, s, b); return DSORT_OK; }
int dsort_host_register(dsort_ctx *ctx, void *h, size_t b) { (void)ctx; (void)h; (void)b; return DSORT_OK; }
int dsort_host_unregister(dsort_ctx *ctx, void *h) { (void)ctx; (void)h; return DSORT_OK; }
int dsort_gen_uniform_i32(dsort_ctx *ctx, int32_t *d, size_t n, uint64_t seed, uint64_t first, void *s) {
    (void)ctx; (void)s; oracle_gen_uniform_i32(seed, first, n, d); return DSORT_OK;
}
int dsort_gen_uniform_i64(dsort_ctx *ctx, int64_t *d, size_t n, uint64_t seed, uint64_t first, void *s) {
    (void)ctx; (void)s; oracle_gen_uniform_i64(seed, first, n, d); return DSORT_OK;
}
int dsort_gen_zipf_i64(dsort_ctx *ctx, int64_t *d, size_t n, uint64_t seed, uint64_t first, void *s) {
    (void)ctx; (void)d; (void)n; (void)seed; (void)first; (void)s; return DSORT_EINVAL;
}
int dsort_fingerprint_i32(dsort_ctx *ctx, const int32_t *d, size_t n, uint64_t *s, uint64_t *x) { (void)ctx; oracle_fingerprint_i32(d, n, s, x); return DSORT_OK; }
int dsort_fingerprint_i64(dsort_ctx *ctx, const int64_t *d, size_t n, uint64_t *s, uint64_t *x) { (void)ctx; oracle_fingerprint_i64(d, n, s, x); return DSORT_OK; }
#define DESC(T, NAME) int NAME(dsort_ctx *ctx, const T *d, size_t n, uint64_t *c) { (void)ctx; uint64_t k = 0; for (size_t i = 1; i < n; ++i) k += d[i - 1] > d[i]; *c = k; return DSORT_OK; }
DESC(int32_t, dsort_count_descents_i32)
DESC(int64_t, dsort_count_descents_i64)
int dsort_comm_unique_id(char id[DSORT_UNIQUE_ID_BYTES]) { memset(id, 7, DSORT_UNIQUE_ID_BYTES); return DSORT_OK; }
int dsort_comm_init(dsort_ctx *ctx, int nranks, int rank, const char id[DSORT_UNIQUE_ID_BYTES]) {
    (void)ctx; (void)nranks; (void)rank; (void)id; return DSORT_ECOMM; /* no RCCL in the double */
}
int dsort_comm_init_transport(dsort_ctx *ctx, int nranks, int rank, const dsort_transport *t) {
    (void)ctx; g_nranks = nranks; g_rank = rank; g_tx = *t; g_has_tx = 1; g_abort = 0; return DSORT_OK;
}
int dsort_comm_abort(dsort_ctx *ctx) { (void)ctx; g_has_tx = 0; return DSORT_OK; }
int dsort_comm_deadline_ms(const dsort_ctx *ctx, int64_t *ms) { (void)ctx; if (!ms) return DSORT_EINVAL; *ms = -1; return DSORT_OK; }
int dsort_comm_destroy(dsort_ctx *ctx) { (void)ctx; g_has_tx = 0; return DSORT_OK; }

/* The double's sort has the library's three bucketed-sort kill points (dsort.h,
 * DSORT_OPT_KILL_AFTER_STAGE), as three real stages: 0 the lower half sorted, 1 the upper half
 * sorted, 2 the halves merged.  A stage never reached is an error, as in the library. */
int dsort_sort_stages(const dsort_ctx *ctx, size_t n, int key_bytes, int *stages) {
    (void)ctx;
    if (!stages || (key_bytes != 4 && key_bytes != 8)) return DSORT_EINVAL;
    *stages = n < 2 ? 0 : 3;
    return DSORT_OK;
}
int dsort_sample_sort_stages(const dsort_ctx *ctx, size_t n_total, int nranks, int rank, int key_bytes, int *stages) {
    if (nranks < 1 || rank < 0 || rank >= nranks) return DSORT_EINVAL;
    return dsort_sort_stages(ctx, n_total / nranks + ((size_t)rank < n_total % nranks), key_bytes, stages);
}
#define DOUBLE_SORT(T, SFX)                                                                          \
    int dsort_sort_dev_copy_##SFX(dsort_ctx *ctx, const T *in, T *out, size_t n, void *s) {            \
        (void)ctx; (void)s;                                                                          \
        if (n && in != out) memmove(out, in, n * sizeof(T));                                        \
        if (n < 2) return g_kill_after_pass >= 0 ? DSORT_ESTAGE : DSORT_OK;                          \
        const size_t h = n / 2;                                                                      \
        if (oracle_merge_sort_##SFX(out, h)) return DSORT_ENOMEM;                                    \
        if (g_kill_after_pass == 0) raise(SIGKILL);                                                  \
        if (oracle_merge_sort_##SFX(out + h, n - h)) return DSORT_ENOMEM;                            \
        if (g_kill_after_pass == 1) raise(SIGKILL);                                                  \
        T *tmp = (T *)malloc(n * sizeof(T));                                                         \
        if (!tmp) return DSORT_ENOMEM;                                                               \
        const T *runs[2] = {out, out + h};                                                           \
        const size_t lens[2] = {h, n - h};                                                           \
        oracle_merge_runs_##SFX(2, runs, lens, tmp);                                                 \
        memcpy(out, tmp, n * sizeof(T));                                                             \
        free(tmp);                                                                                   \
        if (g_kill_after_pass == 2) raise(SIGKILL);                                                  \
        return g_kill_after_pass >= 0 ? DSORT_ESTAGE : DSORT_OK;                                     \
    }                                                                                                \
    int dsort_merge_dev_##SFX(dsort_ctx *ctx, const T *in, const size_t lens[], int k, T *out, void *s) { \
        (void)ctx; (void)s;                                                                          \
        const T **runs = (const T **)malloc(sizeof(T *) * (k ? k : 1));                              \
        size_t off = 0;                                                                              \
        for (int j = 0; j < k; ++j) { runs[j] = in + off; off += lens[j]; }                          \
        oracle_merge_runs_##SFX(k, (const T *const *)runs, lens, out);                               \
        free(runs);                                                                                  \
        return DSORT_OK;                                                                             \
    }                                                                                                \
    typedef struct { T v; int32_t r; uint64_t i; } samp_##SFX;                                       \
    static int cmp_##SFX(const void *a, const void *b) {                                             \
        const samp_##SFX *x = (const samp_##SFX *)a, *y = (const samp_##SFX *)b;                     \
        if (x->v != y->v) return x->v < y->v ? -1 : 1;                                               \
        if (x->r != y->r) return x->r < y->r ? -1 : 1;                                               \
        return x->i < y->i ? -1 : (x->i > y->i);                                                     \
    }                                                                                                \
    int dsort_sample_merge_dev_##SFX(dsort_ctx *ctx, const T *run, size_t n, T **d_out, size_t *n_out, void *st) { \
        (void)ctx; (void)st;                                                                         \
        if (!g_has_tx) return DSORT_ECOMM;                                                           \
        const int P = g_nranks, me = g_rank, S = 512;                                                \
        const size_t rec = (size_t)S * sizeof(T) + 8;                                                \
        char *mine = (char *)malloc(rec), *all = (char *)malloc(rec * P);                            \
        for (int j = 0; j < S; ++j) {                                                                \
            uint64_t p = n ? (uint64_t)(j + 1) * n / (S + 1) : 0;                                    \
            if (n && p >= n) p = n - 1;                                                              \
            T v = n ? run[p] : (T)(sizeof(T) == 4 ? INT32_MAX : INT64_MAX);                          \
            memcpy(mine + (size_t)j * sizeof(T), &v, sizeof(T));                                     \
        }                                                                                            \
        uint64_t nl = n;                                                                             \
        memcpy(mine + (size_t)S * sizeof(T), &nl, 8);                                                \
        if (g_tx.allgather(g_tx.user, mine, all, rec)) { free(mine); free(all); return DSORT_ECOMM; } \
        if (g_kill_in_exchange == 1) raise(SIGKILL);                                                 \
        samp_##SFX *sm = (samp_##SFX *)malloc(sizeof(samp_##SFX) * (size_t)P * S);                   \
        for (int r = 0; r < P; ++r) {                                                                \
            uint64_t nr;                                                                             \
            memcpy(&nr, all + (size_t)r * rec + (size_t)S * sizeof(T), 8);                           \
            for (int j = 0; j < S; ++j) {                                                            \
                uint64_t p = nr ? (uint64_t)(j + 1) * nr / (S + 1) : 0;                              \
                if (nr && p >= nr) p = nr - 1;                                                       \
                memcpy(&sm[(size_t)r * S + j].v, all + (size_t)r * rec + (size_t)j * sizeof(T), sizeof(T)); \
                sm[(size_t)r * S + j].r = r;                                                         \
                sm[(size_t)r * S + j].i = p;                                                         \
            }                                                                                        \
        }                                                                                            \
        qsort(sm, (size_t)P * S, sizeof(samp_##SFX), cmp_##SFX);                                     \
        uint64_t *cuts = (uint64_t *)calloc(P + 1, 8);                                               \
        cuts[P] = n;                                                                                 \
        for (int q = 1; q < P; ++q) {                                                                \
            const samp_##SFX sp = sm[(size_t)q * P * S / P];                                         \
            uint64_t lo = 0, hi = n;                                                                 \
            if (sp.r == me) lo = sp.i < n ? sp.i : n;                                                \
            else {                                                                                   \
                const int upper = me < sp.r;                                                         \
                while (lo < hi) {                                                                    \
                    const uint64_t mid = (lo + hi) / 2;                                              \
                    if (upper ? run[mid] <= sp.v : run[mid] < sp.v) lo = mid + 1; else hi = mid;     \
                }                                                                                    \
            }                                                                                        \
            cuts[q] = lo;                                                                            \
        }                                                                                            \
        uint64_t *cnt = (uint64_t *)malloc(8 * P), *mat = (uint64_t *)malloc(8 * (size_t)P * P);     \
        for (int r = 0; r < P; ++r) cnt[r] = cuts[r + 1] - cuts[r];                                  \
        if (g_tx.allgather(g_tx.user, cnt, mat, 8 * (size_t)P)) return DSORT_ECOMM;                  \
        if (g_kill_in_exchange == 2) raise(SIGKILL);                                                 \
        size_t *sc = (size_t *)malloc(sizeof(size_t) * P * 4), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P; \
        size_t *lens = (size_t *)malloc(sizeof(size_t) * P);                                         \
        size_t tot = 0;                                                                              \
        for (int r = 0; r < P; ++r) {                                                                \
            sc[r] = cnt[r] * sizeof(T); sd[r] = cuts[r] * sizeof(T);                                 \
            lens[r] = mat[(size_t)r * P + me]; rc[r] = lens[r] * sizeof(T); rd[r] = tot * sizeof(T); tot += lens[r]; \
        }                                                                                            \
        T *recv = (T *)malloc(sizeof(T) * (tot ? tot : 1));                                          \
        if (g_tx.alltoallv(g_tx.user, run, sc, sd, recv, rc, rd)) return DSORT_ECOMM;                \
        free(g_out);                                                                                 \
        g_out = malloc(sizeof(T) * (tot ? tot : 1));                                                 \
        dsort_merge_dev_##SFX(ctx, recv, lens, P, (T *)g_out, NULL);                                 \
        *d_out = (T *)g_out;                                                                         \
        *n_out = tot;                                                                                \
        free(mine); free(all); free(sm); free(cuts); free(cnt); free(mat); free(sc); free(lens); free(recv); \
        return DSORT_OK;                                                                             \
    }                                                                                                \
    /* the whole sample sort: the double's local sort (its kill stages), then the exchange */      \
    int dsort_sample_sort_dev_##SFX(dsort_ctx *ctx, const T *in, size_t n, T **d_out, size_t *n_out, void *st) { \
        T *tmp = (T *)malloc(sizeof(T) * (n ? n : 1));                                               \
        if (!tmp) return DSORT_ENOMEM;                                                               \
        int rc = dsort_sort_dev_copy_##SFX(ctx, in, tmp, n, st);                                     \
        if (!rc) rc = dsort_sample_merge_dev_##SFX(ctx, tmp, n, d_out, n_out, st);                   \
        free(tmp);                                                                                   \
        return rc;                                                                                   \
    }
#include <limits.h>
DOUBLE_SORT(int32_t, i32)
DOUBLE_SORT(int64_t, i64)
