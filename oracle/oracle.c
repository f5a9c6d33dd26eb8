/*
 * oracle.c -- CPU restatement of the reference sort path.  TEST INFRASTRUCTURE ONLY
 * (see oracle.h).  Clean-room: written from the behaviour documented in SURVEY.md §3/§8 and
 * the reference files cited per function; no reference source is copied.
 */
#include "oracle.h"

#include <limits.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- merge sort ----------- */
/* client.c:166-173: sort [lo, hi] inclusive, split at lo + (hi-lo)/2, recurse left, recurse
 * right, then merge.  client.c:140-164: both halves are copied to fresh heap buffers and
 * merged back with `<=` (left wins ties).  We keep the per-node allocation so the CPU
 * baseline times the reference's algorithm, not a tuned one. */
#define DEFINE_MERGE_SORT(T, NAME)                                                         \
    static int NAME##_merge(T *a, size_t lo, size_t mid, size_t hi) {                      \
        size_t nl = mid - lo + 1, nr = hi - mid;                                           \
        T *l = (T *)malloc(nl * sizeof(T));                                                \
        T *r = (T *)malloc(nr * sizeof(T));                                                \
        if (!l || !r) { free(l); free(r); return -1; }                                     \
        memcpy(l, a + lo, nl * sizeof(T));                                                 \
        memcpy(r, a + mid + 1, nr * sizeof(T));                                            \
        size_t i = 0, j = 0, o = lo;                                                       \
        while (i < nl && j < nr) a[o++] = (l[i] <= r[j]) ? l[i++] : r[j++];                \
        while (i < nl) a[o++] = l[i++];                                                    \
        while (j < nr) a[o++] = r[j++];                                                    \
        free(l);                                                                           \
        free(r);                                                                           \
        return 0;                                                                          \
    }                                                                                      \
    static int NAME##_rec(T *a, size_t lo, size_t hi) {                                    \
        if (lo >= hi) return 0;                                                            \
        size_t mid = lo + (hi - lo) / 2;                                                   \
        if (NAME##_rec(a, lo, mid) || NAME##_rec(a, mid + 1, hi)) return -1;               \
        return NAME##_merge(a, lo, mid, hi);                                               \
    }                                                                                      \
    int NAME(T *data, size_t n) { return n < 2 ? 0 : NAME##_rec(data, 0, n - 1); }

DEFINE_MERGE_SORT(int32_t, oracle_merge_sort_i32)
DEFINE_MERGE_SORT(int64_t, oracle_merge_sort_i64)

/* ---------------------------------------------------------------- k-way merge ---------- */
/* server.c:500-515: for every output slot scan all runs, keep the head that is strictly
 * below the running minimum (initialised to INT_MAX), ties -> lowest index; if no head
 * qualified (all remaining heads == INT_MAX) nothing is written and no cursor moves. */
void oracle_merge_chunks_i32(int k, const int32_t *const runs[], const size_t lens[],
                             int32_t *out) {
    size_t total = 0;
    for (int j = 0; j < k; ++j) total += lens[j];
    size_t *cur = (size_t *)calloc((size_t)(k > 0 ? k : 1), sizeof(size_t));
    if (!cur) return;
    for (size_t i = 0; i < total; ++i) {
        int32_t best = INT_MAX;
        int who = -1;
        for (int j = 0; j < k; ++j)
            if (cur[j] < lens[j] && runs[j][cur[j]] < best) { best = runs[j][cur[j]]; who = j; }
        if (who >= 0) { out[i] = best; cur[who]++; }
    }
    free(cur);
}

#define DEFINE_MERGE_RUNS(T, NAME)                                                         \
    void NAME(int k, const T *const runs[], const size_t lens[], T *out) {                 \
        size_t total = 0;                                                                  \
        for (int j = 0; j < k; ++j) total += lens[j];                                      \
        size_t *cur = (size_t *)calloc((size_t)(k > 0 ? k : 1), sizeof(size_t));           \
        if (!cur) return;                                                                  \
        for (size_t i = 0; i < total; ++i) {                                               \
            int who = -1;                                                                  \
            for (int j = 0; j < k; ++j)                                                    \
                if (cur[j] < lens[j] && (who < 0 || runs[j][cur[j]] < runs[who][cur[who]])) \
                    who = j;                                                               \
            out[i] = runs[who][cur[who]++];                                                \
        }                                                                                  \
        free(cur);                                                                         \
    }

DEFINE_MERGE_RUNS(int32_t, oracle_merge_runs_i32)
DEFINE_MERGE_RUNS(int64_t, oracle_merge_runs_i64)

/* ---------------------------------------------------------------- partition ------------ */
void oracle_partition(size_t n, int w, size_t *sizes, size_t *offsets) {
    size_t base = n / (size_t)w, extra = n % (size_t)w, off = 0;
    for (int i = 0; i < w; ++i) {
        sizes[i] = base + ((size_t)i < extra ? 1 : 0);
        offsets[i] = off;
        off += sizes[i];
    }
}

int oracle_reference_sort_i32(const int32_t *keys, size_t n, int workers, int32_t *out) {
    if (workers < 1) return -1;
    size_t *sz = (size_t *)malloc(sizeof(size_t) * (size_t)workers);
    size_t *of = (size_t *)malloc(sizeof(size_t) * (size_t)workers);
    int32_t **chunks = (int32_t **)calloc((size_t)workers, sizeof(int32_t *));
    int rc = 0;
    if (!sz || !of || !chunks) { rc = -1; goto done; }
    oracle_partition(n, workers, sz, of);
    for (int i = 0; i < workers; ++i) {
        chunks[i] = (int32_t *)malloc((sz[i] ? sz[i] : 1) * sizeof(int32_t));
        if (!chunks[i]) { rc = -1; goto done; }
        memcpy(chunks[i], keys + of[i], sz[i] * sizeof(int32_t));
        if (oracle_merge_sort_i32(chunks[i], sz[i])) { rc = -1; goto done; }
    }
    oracle_merge_chunks_i32(workers, (const int32_t *const *)chunks, sz, out);
done:
    if (chunks)
        for (int i = 0; i < workers; ++i) free(chunks[i]);
    free(chunks);
    free(sz);
    free(of);
    return rc;
}

/* ---------------------------------------------------------------- text codec ----------- */
long oracle_parse_i32(const char *text, size_t len, int32_t *out, size_t cap) {
    size_t i = 0, count = 0;
    while (i < len) {
        char c = text[i];
        if (c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\v' || c == '\f') { ++i; continue; }
        int neg = 0;
        if (c == '-' || c == '+') { neg = (c == '-'); ++i; }
        if (i >= len || text[i] < '0' || text[i] > '9') return -1;
        long long v = 0;
        while (i < len && text[i] >= '0' && text[i] <= '9') {
            v = v * 10 + (text[i] - '0');
            if (v > 4294967296LL) v = 4294967296LL; /* saturate; %d overflow is UB anyway */
            ++i;
        }
        if (i < len && !(text[i] == ' ' || text[i] == '\n' || text[i] == '\t' || text[i] == '\r' ||
                         text[i] == '\v' || text[i] == '\f'))
            return -1;
        if (count < cap) out[count] = (int32_t)(neg ? -v : v);
        ++count;
    }
    return (long)count;
}

long oracle_format_i32(const int32_t *keys, size_t n, char *buf, size_t cap) {
    size_t o = 0;
    char tmp[16];
    for (size_t i = 0; i < n; ++i) {
        int64_t v = keys[i];
        int neg = v < 0;
        uint64_t u = neg ? (uint64_t)(-v) : (uint64_t)v;
        int t = 0;
        do { tmp[t++] = (char)('0' + (u % 10)); u /= 10; } while (u);
        if (o + (size_t)t + (size_t)neg + 1 > cap) return -1;
        if (neg) buf[o++] = '-';
        while (t) buf[o++] = tmp[--t];
        buf[o++] = '\n';
    }
    return (long)o;
}

/* ---------------------------------------------------------------- generators ----------- */
uint64_t oracle_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

void oracle_gen_uniform_i32(uint64_t seed, uint64_t first, size_t n, int32_t *out) {
    for (size_t i = 0; i < n; ++i) out[i] = (int32_t)(uint32_t)(oracle_splitmix64(seed + first + i) >> 32);
}

void oracle_gen_uniform_i64(uint64_t seed, uint64_t first, size_t n, int64_t *out) {
    for (size_t i = 0; i < n; ++i) out[i] = (int64_t)oracle_splitmix64(seed + first + i);
}

void oracle_fingerprint_i32(const int32_t *keys, size_t n, uint64_t *sum, uint64_t *xr) {
    uint64_t s = 0, x = 0;
    for (size_t i = 0; i < n; ++i) {
        uint64_t k = (uint64_t)(uint32_t)keys[i];
        s += oracle_splitmix64(k);
        x ^= oracle_splitmix64(k ^ 0xD1B54A32D192ED03ULL);
    }
    *sum = s;
    *xr = x;
}

void oracle_fingerprint_i64(const int64_t *keys, size_t n, uint64_t *sum, uint64_t *xr) {
    uint64_t s = 0, x = 0;
    for (size_t i = 0; i < n; ++i) {
        uint64_t k = (uint64_t)keys[i];
        s += oracle_splitmix64(k);
        x ^= oracle_splitmix64(k ^ 0xD1B54A32D192ED03ULL);
    }
    *sum = s;
    *xr = x;
}
