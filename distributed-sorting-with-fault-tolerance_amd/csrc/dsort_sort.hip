// dsort_sort.hip -- the worker sort and the master merge on MI355X (gfx950).
//
// Replaces merge_sort()/merge() (reference client.c:140-173) and the merge loop of
// merge_chunks() (reference server.c:481-515).  Same result: the input multiset in ascending
// signed order; ties resolved like the reference (left run first), which for keys-only data
// is unobservable but keeps the merge deterministic.
//
// Structure:
//   1. block_sort_kernel   one workgroup sorts one TILE of keys: coalesced 16-B loads, a Batcher
//                          odd-even network over the K keys each lane holds in registers, then
//                          log2(TILE/K) merge-path levels through LDS; coalesced 16-B stores.
//                          Algorithmic traffic: read + write of every key (2*w bytes/key).
//   2. merge passes        ceil(log2(#tiles)) passes.  partition2_kernel finds, for every
//                          output tile, the merge-path split of the two input runs (a binary
//                          search per tile diagonal); merge2_kernel stages the two input windows
//                          of its tile in LDS and each lane merges K outputs.  Traffic per pass:
//                          2*w bytes/key.
//   The k-way master merge (dsort_merge_*) runs the same pass kernels over a pairwise tree of
//   arbitrary-length runs.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <climits>
#include <vector>

#include "dsort_internal.h"

namespace dsort {

template <typename T> __host__ __device__ constexpr T key_max();
template <> __host__ __device__ constexpr int32_t key_max<int32_t>() { return INT32_MAX; }
template <> __host__ __device__ constexpr int64_t key_max<int64_t>() { return INT64_MAX; }

// 16-byte vector of keys, the unit of every global load/store of a full tile.
template <typename T> struct Vec16;
template <> struct Vec16<int32_t> { using type = int4; static constexpr int N = 4; };
template <> struct Vec16<int64_t> { using type = longlong2; static constexpr int N = 2; };

template <typename T>
__device__ __forceinline__ void cex(T &a, T &b) {
    const T lo = a < b ? a : b;
    const T hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// Batcher odd-even merge sort network over K (power of two) register-resident keys; fully
// unrolled so every index is a compile-time constant (no scratch).
template <typename T, int K>
__device__ __forceinline__ void sort_regs(T (&v)[K]) {
#pragma unroll
    for (int p = 1; p < K; p <<= 1) {
#pragma unroll
        for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
            for (int j = k % p; j + k < K; j += 2 * k) {
#pragma unroll
                for (int i = 0; i < k; ++i) {
                    if (i + j + k < K && (i + j) / (2 * p) == (i + j + k) / (2 * p))
                        cex(v[i + j], v[i + j + k]);
                }
            }
        }
    }
}

// Merge-path split on LDS: number of A keys among the first `diag` outputs of merge(A, B),
// A-first on ties (the reference's `<=`, client.c:152).
template <typename T>
__device__ __forceinline__ int lds_merge_path(const T *A, int na, const T *B, int nb, int diag) {
    int lo = diag > nb ? diag - nb : 0;
    int hi = diag < na ? diag : na;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (A[mid] <= B[diag - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// The same search over global memory with 64-bit positions.
template <typename T>
__device__ __forceinline__ uint64_t glb_merge_path(const T *__restrict__ A, uint64_t na,
                                                   const T *__restrict__ B, uint64_t nb,
                                                   uint64_t diag) {
    uint64_t lo = diag > nb ? diag - nb : 0;
    uint64_t hi = diag < na ? diag : na;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (A[mid] <= B[diag - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Serial merge of K outputs starting at (a, b); exhausted inputs read as key_max and the
// `b >= nb` test keeps a real key_max in A ahead of an exhausted B.
template <typename T, int K>
__device__ __forceinline__ void serial_merge(const T *A, int na, const T *B, int nb, int a, int b,
                                             T (&out)[K]) {
    T av = a < na ? A[a] : key_max<T>();
    T bv = b < nb ? B[b] : key_max<T>();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const bool take_a = (b >= nb) || (a < na && av <= bv);
        out[k] = take_a ? av : bv;
        if (take_a) {
            ++a;
            av = a < na ? A[a] : key_max<T>();
        } else {
            ++b;
            bv = b < nb ? B[b] : key_max<T>();
        }
    }
}

// ---------------------------------------------------------------------------------------
// 1. Tile sort.
// ---------------------------------------------------------------------------------------
template <typename T, int THREADS, int K>
__global__ void __launch_bounds__(THREADS) block_sort_kernel(const T *__restrict__ in,
                                                             T *__restrict__ out, uint64_t n) {
    constexpr int TILE = THREADS * K;
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::N;
    __shared__ __attribute__((aligned(16))) T s[TILE];

    const int t = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    const uint64_t rem = n - base;
    const int valid = rem < (uint64_t)TILE ? (int)rem : TILE;

    T v[K];
    if (valid == TILE) {
        const V *src = reinterpret_cast<const V *>(in + base);
#pragma unroll
        for (int i = 0; i < K / VN; ++i) {
            const V x = src[i * THREADS + t];
            const T *px = reinterpret_cast<const T *>(&x);
#pragma unroll
            for (int j = 0; j < VN; ++j) v[i * VN + j] = px[j];
        }
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int e = i * THREADS + t;
            v[i] = e < valid ? in[base + e] : key_max<T>();
        }
    }

    sort_regs<T, K>(v);
#pragma unroll
    for (int i = 0; i < K; ++i) s[t * K + i] = v[i];
    __syncthreads();

    const int pos = t * K;
#pragma unroll 1
    for (int r = K; r < TILE; r <<= 1) {
        const int pb = pos & ~(2 * r - 1);
        const int diag = pos - pb;
        const T *A = s + pb;
        const T *B = A + r;
        const int a = lds_merge_path(A, r, B, r, diag);
        serial_merge<T, K>(A, r, B, r, a, diag - a, v);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < K; ++i) s[pos + i] = v[i];
        __syncthreads();
    }

    if (valid == TILE) {
        V *dst = reinterpret_cast<V *>(out + base);
        const V *sv = reinterpret_cast<const V *>(s);
#pragma unroll
        for (int i = 0; i < K / VN; ++i) dst[i * THREADS + t] = sv[i * THREADS + t];
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int e = i * THREADS + t;
            if (e < valid) out[base + e] = s[e];
        }
    }
}

// ---------------------------------------------------------------------------------------
// 2a. Partition: one thread per output tile computes the merge-path splits at the tile's
//     first and last diagonal.  REGULAR: runs of length R back to back (pass p of the sort);
//     otherwise pairs come from a table (user runs of arbitrary length).
// ---------------------------------------------------------------------------------------
template <typename T, bool REGULAR>
__global__ void __launch_bounds__(256) partition2_kernel(const T *__restrict__ in, uint64_t n,
                                                         uint64_t R, int tile,
                                                         const Pair *__restrict__ pairs,
                                                         int npairs, Bucket2 *__restrict__ out,
                                                         uint64_t nbuckets) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nbuckets) return;
    uint64_t a0, na, nb, rel;
    if (REGULAR) {
        const uint64_t start = j * (uint64_t)tile;
        const uint64_t gstart = start - start % (2 * R);
        a0 = gstart;
        na = n - gstart < R ? n - gstart : R;
        const uint64_t b0 = gstart + na;
        nb = n > b0 ? (n - b0 < R ? n - b0 : R) : 0;
        rel = start - gstart;
    } else {
        int lo = 0, hi = npairs - 1;  // last pair with first_bucket <= j
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pairs[mid].first_bucket <= j) lo = mid;
            else hi = mid - 1;
        }
        const Pair p = pairs[lo];
        a0 = p.a_off;
        na = p.a_len;
        nb = p.b_len;
        rel = (j - p.first_bucket) * (uint64_t)tile;
    }
    const uint64_t b0 = a0 + na;
    const uint64_t total = na + nb;
    const uint64_t end = rel + tile < total ? rel + tile : total;
    const uint64_t as = glb_merge_path(in + a0, na, in + b0, nb, rel);
    const uint64_t ae = end == total ? na : glb_merge_path(in + a0, na, in + b0, nb, end);
    Bucket2 b;
    b.out_off = a0 + rel;
    b.a_start = a0 + as;
    b.b_start = b0 + (rel - as);
    b.a_len = (uint32_t)(ae - as);
    b.b_len = (uint32_t)((end - ae) - (rel - as));
    out[j] = b;
}

// ---------------------------------------------------------------------------------------
// 2b. Merge one output tile: stage both input windows in LDS, merge-path per lane, K outputs
//     per lane, coalesced stores through LDS.
// ---------------------------------------------------------------------------------------
template <typename T, int THREADS, int K>
__global__ void __launch_bounds__(THREADS) merge2_kernel(const T *__restrict__ in,
                                                         T *__restrict__ out,
                                                         const Bucket2 *__restrict__ buckets) {
    constexpr int TILE = THREADS * K;
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::N;
    __shared__ __attribute__((aligned(16))) T s[TILE];

    const int t = threadIdx.x;
    const Bucket2 bk = buckets[blockIdx.x];
    const int na = (int)bk.a_len;
    const int nb = (int)bk.b_len;
    const int total = na + nb;

#pragma unroll
    for (int i = 0; i < K; ++i) {
        const int e = i * THREADS + t;
        if (e < total) s[e] = e < na ? in[bk.a_start + e] : in[bk.b_start + (e - na)];
    }
    __syncthreads();

    T v[K];
    const int pos = t * K;
    if (pos < total) {
        const int a = lds_merge_path(s, na, s + na, nb, pos);
        serial_merge<T, K>(s, na, s + na, nb, a, pos - a, v);
    }
    __syncthreads();
    if (pos < total) {
#pragma unroll
        for (int i = 0; i < K; ++i) s[pos + i] = v[i];
    }
    __syncthreads();

    if (total == TILE && (bk.out_off % VN) == 0) {
        V *dst = reinterpret_cast<V *>(out + bk.out_off);
        const V *sv = reinterpret_cast<const V *>(s);
#pragma unroll
        for (int i = 0; i < K / VN; ++i) dst[i * THREADS + t] = sv[i * THREADS + t];
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int e = i * THREADS + t;
            if (e < total) out[bk.out_off + e] = s[e];
        }
    }
}

// ---------------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------------
static inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

static int merge_passes_for(uint64_t runs) {
    int p = 0;
    while ((1ull << p) < runs) ++p;
    return p;
}

template <typename T>
int sort_device(dsort_ctx *ctx, const T *d_in, T *d_keys, size_t n, hipStream_t s, bool timed) {
    constexpr int THREADS = Geom<T>::THREADS, K = Geom<T>::K, TILE = Geom<T>::TILE;
    ctx->stats = dsort_stats{};
    ctx->stats.keys_in = n;
    ctx->stats.keys_out = n;
    ctx->stats.tile_keys = TILE;
    ctx->ev_mask = 0;
    ctx->kev_used = 0;
    ctx->last_stream = s;
    if (n < 2) {
        if (n == 1 && d_in != d_keys)
            DSORT_HIP(ctx, hipMemcpyAsync(d_keys, d_in, sizeof(T), hipMemcpyDeviceToDevice, s));
        return DSORT_OK;
    }
    const uint64_t tiles = ceil_div(n, TILE);
    const int passes = merge_passes_for(tiles);
    ctx->stats.merge_passes = passes;
    T *scratch = nullptr;
    if (passes > 0) {
        int rc = ensure(ctx, &ctx->scratch, &ctx->scratch_bytes, n * sizeof(T), "sort scratch");
        if (rc) return rc;
        rc = ensure(ctx, &ctx->buckets, &ctx->buckets_bytes, tiles * sizeof(Bucket2), "buckets");
        if (rc) return rc;
        scratch = static_cast<T *>(ctx->scratch);
    }
    // Ping-pong so that the last pass lands in d_keys.  The tile sort reads d_in (which may
    // alias d_keys: every workgroup reads its whole tile before writing it).
    T *bufs[2] = {d_keys, scratch};
    int cur = (passes % 2 == 0) ? 0 : 1;
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[0], s));
        ctx->ev_mask |= 1u;
    }
    hipLaunchKernelGGL((block_sort_kernel<T, THREADS, K>), dim3((unsigned)tiles), dim3(THREADS), 0,
                       s, d_in, bufs[cur], (uint64_t)n);
    DSORT_HIP(ctx, hipGetLastError());
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[1], s));
        ctx->ev_mask |= 2u;
    }
    Bucket2 *bk = static_cast<Bucket2 *>(ctx->buckets);
    ctx->kev_used = 0;
    for (int p = 0; p < passes; ++p) {
        const uint64_t R = (uint64_t)TILE << p;
        hipLaunchKernelGGL((partition2_kernel<T, true>), dim3((unsigned)ceil_div(tiles, 256)),
                           dim3(256), 0, s, bufs[cur], (uint64_t)n, R, TILE, nullptr, 0, bk,
                           tiles);
        DSORT_HIP(ctx, hipGetLastError());
        const bool kt = timed && ctx->ev_ok && ctx->kev_used + 2 <= dsort_ctx::kMaxKev;
        if (kt) DSORT_HIP(ctx, hipEventRecord(ctx->kev[ctx->kev_used], s));
        hipLaunchKernelGGL((merge2_kernel<T, THREADS, K>), dim3((unsigned)tiles), dim3(THREADS),
                           0, s, bufs[cur], bufs[cur ^ 1], bk);
        DSORT_HIP(ctx, hipGetLastError());
        if (kt) {
            DSORT_HIP(ctx, hipEventRecord(ctx->kev[ctx->kev_used + 1], s));
            ctx->kev_used += 2;
        }
        cur ^= 1;
    }
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[2], s));
        ctx->ev_mask |= 4u;
    }
    return DSORT_OK;
}

// k-way merge of back-to-back runs as a pairwise tree of 2-way passes.  Level l merges runs
// (2i, 2i+1); an odd last run is carried through as a pair with an empty partner.  Ties keep
// the lower run first at every level, so the result matches the reference's lowest-index-wins
// argmin scan (server.c:504).
template <typename T>
int merge_device(dsort_ctx *ctx, const T *d_in, const size_t *lens, int k, T *d_out,
                 hipStream_t s) {
    constexpr int THREADS = Geom<T>::THREADS, K = Geom<T>::K, TILE = Geom<T>::TILE;
    ctx->stats = dsort_stats{};
    ctx->last_stream = s;
    uint64_t n = 0;
    std::vector<uint64_t> rl;
    for (int j = 0; j < k; ++j) {
        n += lens[j];
        rl.push_back(lens[j]);
    }
    ctx->stats.keys_in = ctx->stats.keys_out = n;
    ctx->stats.tile_keys = TILE;
    if (n == 0) return DSORT_OK;
    if (k == 1) {
        DSORT_HIP(ctx, hipMemcpyAsync(d_out, d_in, n * sizeof(T), hipMemcpyDeviceToDevice, s));
        return DSORT_OK;
    }
    int levels = merge_passes_for((uint64_t)k);
    ctx->stats.merge_passes = levels;
    int rc = DSORT_OK;
    if (levels > 1) {
        rc = ensure(ctx, &ctx->scratch, &ctx->scratch_bytes, n * sizeof(T), "merge scratch");
        if (rc) return rc;
    }
    // level l reads src, writes dst; the final level writes d_out.
    const T *src = d_in;
    T *scr = static_cast<T *>(ctx->scratch);
    // choose the first destination so that the last level writes d_out
    T *dsts[2] = {d_out, scr};
    int which = (levels % 2 == 1) ? 0 : 1;
    std::vector<Pair> pairs;
    for (int l = 0; l < levels; ++l) {
        pairs.clear();
        uint64_t off = 0, nbk = 0;
        std::vector<uint64_t> next;
        for (size_t i = 0; i < rl.size(); i += 2) {
            Pair p;
            p.a_off = off;
            p.a_len = rl[i];
            p.b_len = i + 1 < rl.size() ? rl[i + 1] : 0;
            p.first_bucket = nbk;
            const uint64_t tot = p.a_len + p.b_len;
            nbk += ceil_div(tot, TILE);
            off += tot;
            next.push_back(tot);
            if (tot) pairs.push_back(p);
        }
        rl.swap(next);
        rc = ensure(ctx, &ctx->pairs, &ctx->pairs_bytes, pairs.size() * sizeof(Pair), "pairs");
        if (rc) return rc;
        rc = ensure(ctx, &ctx->buckets, &ctx->buckets_bytes, nbk * sizeof(Bucket2), "buckets");
        if (rc) return rc;
        DSORT_HIP(ctx, hipMemcpyAsync(ctx->pairs, pairs.data(), pairs.size() * sizeof(Pair),
                                      hipMemcpyHostToDevice, s));
        T *dst = dsts[which];
        Bucket2 *bk = static_cast<Bucket2 *>(ctx->buckets);
        hipLaunchKernelGGL((partition2_kernel<T, false>), dim3((unsigned)ceil_div(nbk, 256)),
                           dim3(256), 0, s, src, n, (uint64_t)0, TILE,
                           static_cast<const Pair *>(ctx->pairs), (int)pairs.size(), bk, nbk);
        DSORT_HIP(ctx, hipGetLastError());
        hipLaunchKernelGGL((merge2_kernel<T, THREADS, K>), dim3((unsigned)nbk), dim3(THREADS), 0,
                           s, src, dst, bk);
        DSORT_HIP(ctx, hipGetLastError());
        // the pair table is re-filled next level: keep the copy ordered behind this level
        DSORT_HIP(ctx, hipStreamSynchronize(s));
        src = dst;
        which ^= 1;
    }
    return DSORT_OK;
}

template int sort_device<int32_t>(dsort_ctx *, const int32_t *, int32_t *, size_t, hipStream_t,
                                  bool);
template int sort_device<int64_t>(dsort_ctx *, const int64_t *, int64_t *, size_t, hipStream_t,
                                  bool);
template int merge_device<int32_t>(dsort_ctx *, const int32_t *, const size_t *, int, int32_t *,
                                   hipStream_t);
template int merge_device<int64_t>(dsort_ctx *, const int64_t *, const size_t *, int, int64_t *,
                                   hipStream_t);

}  // namespace dsort
