/*
 * oracle.h -- CPU restatement of the reference sort path.  TEST INFRASTRUCTURE ONLY.
 *
 * This header and oracle.c are the CHECKER for the MI355X sort path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so.
 * The product library (libdsort.so) never links, calls or falls back to this code.
 *
 * Each function restates (does not copy) an algorithm of the reference repo
 * khimansusinha/Distributed-sorting-with-fault-tolerance; the file:line it follows is
 * given per function.  Parity is PINNED: tests/test_oracle.py checks these functions
 * against the reference's own input.txt/output.txt pair and against golden vectors
 * produced by the reference compiled from source (oracle/_ref, tests/golden/make_golden.py).
 */
#ifndef DSORT_ORACLE_H
#define DSORT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Top-down recursive merge sort of data[0..n), ascending, stable, one scratch allocation
 * per merge node (the reference allocates both halves per merge).
 * Follows merge_sort/merge, client.c:140-173 (mid = left + (right-left)/2, ties: left half
 * first because the comparison is `<=`, client.c:152).  Returns 0, or -1 on malloc failure
 * (the reference does not check malloc, client.c:144-145). */
int oracle_merge_sort_i32(int32_t *data, size_t n);
int oracle_merge_sort_i64(int64_t *data, size_t n);

/* k-way merge by a linear argmin scan over the run heads, exactly as merge_chunks,
 * server.c:481-524 (strict `<` against a running minimum initialised to INT_MAX, ties go to
 * the lowest run index).  Reproduces the reference quirk: when every remaining head equals
 * INT_MAX no run is chosen and out[i] is left untouched (server.c:501-515).  `out` must hold
 * sum(lens) entries; the caller pre-fills it (the reference leaves it uninitialised). */
void oracle_merge_chunks_i32(int k, const int32_t *const runs[], const size_t lens[],
                             int32_t *out);

/* Full-range k-way merge (no INT_MAX quirk): same argmin rule with an explicit
 * "have a candidate" flag.  This is the semantics the build defines outside the reference's
 * domain (SURVEY.md §8a "result semantics"). */
void oracle_merge_runs_i32(int k, const int32_t *const runs[], const size_t lens[], int32_t *out);
void oracle_merge_runs_i64(int k, const int64_t *const runs[], const size_t lens[], int64_t *out);

/* Equal contiguous partition of n keys over w workers: chunk i holds n/w + (i < n%w) keys,
 * in file order (server.c:185-216).  sizes[] and offsets[] receive w entries. */
void oracle_partition(size_t n, int w, size_t *sizes, size_t *offsets);

/* The reference end to end, in process: partition over `workers` chunks, merge-sort each
 * chunk, then merge_chunks (server.c:177-268 + client.c:117).  `keys` is sorted in place
 * using `out` (n entries) as the merge destination; result is left in `out`. */
int oracle_reference_sort_i32(const int32_t *keys, size_t n, int workers, int32_t *out);

/* Text codec of the reference: input = whitespace separated %d tokens (server.c:179,213);
 * output = one "%d\n" per key (server.c:518).
 * oracle_parse_i32: returns the number of keys parsed into out (at most cap), or -1 if a
 * token is not an integer (the reference spins forever there).
 * oracle_format_i32: writes the output.txt bytes into buf (cap bytes); returns the length,
 * or -1 if buf is too small.  12 bytes per key always suffice. */
long oracle_parse_i32(const char *text, size_t len, int32_t *out, size_t cap);
long oracle_format_i32(const int32_t *keys, size_t n, char *buf, size_t cap);

/* Synthetic inputs shared with the GPU generator:
 * key i = f(splitmix64(seed + i)); uniform i32 = high 32 bits; uniform i64 = all 64 bits;
 * Zipf i64 = rank from an inverse-CDF table over 2^24 ranks (s = 1.2), key = rank * golden. */
uint64_t oracle_splitmix64(uint64_t x);
void oracle_gen_uniform_i32(uint64_t seed, uint64_t first, size_t n, int32_t *out);
void oracle_gen_uniform_i64(uint64_t seed, uint64_t first, size_t n, int64_t *out);

/* Order-independent multiset fingerprint used for the size-independent parity checks at full
 * sizes: sum over keys of splitmix64(key) (mod 2^64) and xor of splitmix64(key ^ C). */
void oracle_fingerprint_i32(const int32_t *keys, size_t n, uint64_t *sum, uint64_t *xr);
void oracle_fingerprint_i64(const int64_t *keys, size_t n, uint64_t *sum, uint64_t *xr);

#ifdef __cplusplus
}
#endif
#endif
