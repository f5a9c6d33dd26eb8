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
