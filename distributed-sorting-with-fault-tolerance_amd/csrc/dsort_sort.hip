// dsort_sort.hip -- the worker sort and the master merge on MI355X (gfx950).
//
// Replaces merge_sort()/merge() (reference client.c:140-173) and the merge loop of
// merge_chunks() (reference server.c:481-515).  Same result: the input multiset in ascending
// signed order; equal keys from different runs are emitted lower run first, like the reference's
// `<=` (client.c:152) and lowest-index-wins argmin (server.c:504) -- unobservable for keys-only
// data, but it makes every split point below unique.
//
// Structure:
//   1. block_sort_kernel   one workgroup sorts one TILE of keys: 16-B coalesced loads, a Batcher
//                          odd-even network over the K keys each lane holds in registers, then
//                          log2(TILE/K) merge levels through LDS, 16-B coalesced stores.
//   2. k-way merge passes  each pass merges groups of F runs (F up to 64), so the sort needs
//                          ceil(log_F(#tiles)) passes instead of log2(#tiles):
//        partk_kernel      one wave per output tile finds the exact split of the tile's first
//                          output rank over the F runs: bisection over the KEY range with
//                          64/F candidate keys per step (lanes = runs x candidates), each lane a
//                          binary search in its run narrowed by the previous step, then ties
//                          at the split key are handed out in run order;
//        mergek_kernel     stages the F input windows of its tile in LDS and merges them in
//                          log2(F) pairwise levels.
//   Every LDS merge level uses merge path to place each lane's K outputs, then a bitonic merge of
//   the two K-key windows in registers (no dependent LDS-load chain per output key).
//   Algorithmic HBM traffic: 2*w bytes per key for the tile sort and for every pass.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <vector>

#include "dsort_internal.h"

namespace dsort {

template <typename T> __host__ __device__ constexpr T key_max();
template <> __host__ __device__ constexpr int32_t key_max<int32_t>() { return INT32_MAX; }
template <> __host__ __device__ constexpr int64_t key_max<int64_t>() { return INT64_MAX; }
template <typename T> __host__ __device__ constexpr T key_min();
template <> __host__ __device__ constexpr int32_t key_min<int32_t>() { return INT32_MIN; }
template <> __host__ __device__ constexpr int64_t key_min<int64_t>() { return INT64_MIN; }
template <typename T> struct Unsigned;
template <> struct Unsigned<int32_t> { using type = uint32_t; };
template <> struct Unsigned<int64_t> { using type = uint64_t; };

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

// LDS layout: key position p lives at word p + p/32 (one pad word per 32).  Merge levels make
// lane t touch positions ~K/2*t + i (windows) and K*t + i (outputs); unpadded, those strides
// fold onto a few of the 32 banks (up to 16-way conflicts); the pad rotates every 32-key row
// by one bank.
__device__ __forceinline__ int swz(int p) { return p + (p >> 5); }
__host__ __device__ constexpr int padded(int n) { return n + n / 32; }

// Merge-path split on LDS: number of A keys among the first `diag` outputs of merge(A, B),
// A first on ties.  A = s[A0 .. A0+na), B = s[B0 .. B0+nb) in key positions.
template <typename T>
__device__ __forceinline__ int lds_merge_path(const T *s, int A0, int na, int B0, int nb, int diag) {
    int lo = diag > nb ? diag - nb : 0;
    int hi = diag < na ? diag : na;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[swz(A0 + mid)] <= s[swz(B0 + diag - 1 - mid)]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// The K smallest keys of A[a..na) u B[b..nb): the two ascending K-windows form the bitonic
// sequence x ++ reverse(y); its lower half-cleaner min(x[i], y[K-1-i]) holds exactly the K
// smallest keys (as a bitonic sequence), which log2(K) compare-exchange stages sort.
template <typename T, int K>
__device__ __forceinline__ void kmerge(const T *s, int A0, int na, int B0, int nb, int a, int b,
                                       T (&m)[K]) {
    T x[K], y[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = (a + i < na) ? s[swz(A0 + a + i)] : key_max<T>();
#pragma unroll
    for (int i = 0; i < K; ++i) y[i] = (b + i < nb) ? s[swz(B0 + b + i)] : key_max<T>();
#pragma unroll
    for (int i = 0; i < K; ++i) m[i] = x[i] < y[K - 1 - i] ? x[i] : y[K - 1 - i];
#pragma unroll
    for (int s = K / 2; s >= 1; s >>= 1) {
#pragma unroll
        for (int i = 0; i < K; ++i)
            if ((i & s) == 0) cex(m[i], m[i + s]);
    }
}

// Coalesced store of the first `valid` keys of a padded LDS tile: full tiles leave as 16-byte
// vectors (lane t writes vectors t, t+THREADS, ...), assembled from conflict-free 4-byte reads.
template <typename T, int THREADS, int K>
__device__ __forceinline__ void store_tile(const T *s, T *out, int valid) {
    constexpr int TILE = THREADS * K;
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::N;
    const int t = threadIdx.x;
    if (valid == TILE && (reinterpret_cast<uintptr_t>(out) % 16) == 0) {
        V *dst = reinterpret_cast<V *>(out);
#pragma unroll
        for (int i = 0; i < K / VN; ++i) {
            const int q = i * THREADS + t;
            V x;
            T *px = reinterpret_cast<T *>(&x);
#pragma unroll
            for (int j = 0; j < VN; ++j) px[j] = s[swz(q * VN + j)];
            dst[q] = x;
        }
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int e = i * THREADS + t;
            if (e < valid) out[e] = s[swz(e)];
        }
    }
}

// ---------------------------------------------------------------------------------------
// 1. Tile sort.
// ---------------------------------------------------------------------------------------
template <typename T, int THREADS, int K>
__global__ void __launch_bounds__(THREADS) block_sort_kernel(const T *in, T *out, uint64_t n) {
    // `in` may alias `out` (in-place sort): every workgroup reads its whole tile first.
    constexpr int TILE = THREADS * K;
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::N;
    __shared__ __attribute__((aligned(16))) T s[padded(TILE)];

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
    const int pos = t * K;
#pragma unroll
    for (int i = 0; i < K; ++i) s[swz(pos + i)] = v[i];
    __syncthreads();

#pragma unroll 1
    for (int r = K; r < TILE; r <<= 1) {
        const int pb = pos & ~(2 * r - 1);
        const int diag = pos - pb;
        const int a = lds_merge_path(s, pb, r, pb + r, r, diag);
        kmerge<T, K>(s, pb, r, pb + r, r, a, diag - a, v);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < K; ++i) s[swz(pos + i)] = v[i];
        __syncthreads();
    }
    store_tile<T, THREADS, K>(s, out + base, valid);
}

// ---------------------------------------------------------------------------------------
// Tile / group geometry of a k-way pass.
// ---------------------------------------------------------------------------------------
struct TileInfo {
    uint64_t base;    // group start
    uint64_t gtotal;  // keys in the group
    uint64_t d0, d1;  // the tile's output ranks [d0, d1) within the group
};

template <bool REG>
__device__ __forceinline__ const GroupK *tile_info(const PassDesc &pd, uint64_t j, int tile,
                                                   TileInfo &ti) {
    const GroupK *g = nullptr;
    if (REG) {
        const uint64_t gsize = (uint64_t)pd.F * pd.R;
        const uint64_t start = j * (uint64_t)tile;
        ti.base = start - start % gsize;
        ti.gtotal = pd.n - ti.base < gsize ? pd.n - ti.base : gsize;
        ti.d0 = start - ti.base;
    } else {
        int lo = 0, hi = pd.ngroups - 1;  // last group with first_tile <= j
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pd.groups[mid].first_tile <= j) lo = mid;
            else hi = mid - 1;
        }
        g = pd.groups + lo;
        ti.base = g->base;
        ti.gtotal = g->total;
        ti.d0 = (j - g->first_tile) * (uint64_t)tile;
    }
    ti.d1 = ti.d0 + tile < ti.gtotal ? ti.d0 + tile : ti.gtotal;
    return g;
}

template <bool REG>
__device__ __forceinline__ void run_range(const PassDesc &pd, const TileInfo &ti, const GroupK *g,
                                          int i, uint64_t &start, uint64_t &len) {
    if (REG) {
        uint64_t o = (uint64_t)i * pd.R, e = o + pd.R;
        o = o < ti.gtotal ? o : ti.gtotal;
        e = e < ti.gtotal ? e : ti.gtotal;
        start = ti.base + o;
        len = e - o;
    } else if (i < (int)g->nruns) {
        start = ti.base + g->roff[i];
        len = g->roff[i + 1] - g->roff[i];
    } else {
        start = ti.base + g->total;
        len = 0;
    }
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T w = __shfl_xor(v, o);
        v = w < v ? w : v;
    }
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

// Candidate key c of C strictly inside [lo, hi): lo + floor((hi-lo) * (c+1) / (C+1)), computed
// without overflow in the unsigned type of T.
template <typename T>
__device__ __forceinline__ T candidate(T lo, T hi, int c, int C) {
    using U = typename Unsigned<T>::type;
    const U range = (U)hi - (U)lo;
    const U q = range / (U)(C + 1), r = range % (U)(C + 1);
    return (T)((U)lo + q * (U)(c + 1) + (r * (U)(c + 1)) / (U)(C + 1));
}

// ---------------------------------------------------------------------------------------
// 2a. Exact split of output rank d0 of every tile over the F runs of its group.
//     Writes splits[j*F + i] = number of keys of run i before rank d0 (relative to the run).
// ---------------------------------------------------------------------------------------
template <typename T, bool REG>
__global__ void __launch_bounds__(256) partk_kernel(const T *__restrict__ in, PassDesc pd, int tile,
                                                    uint32_t *__restrict__ splits,
                                                    uint64_t ntiles) {
    const int lane = threadIdx.x & 63;
    const uint64_t j = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= ntiles) return;  // wave-uniform
    TileInfo ti;
    const GroupK *g = tile_info<REG>(pd, j, tile, ti);
    const int F = pd.F;
    const int C = 64 / F;
    const int i = lane & (F - 1);
    const int c = lane / F;
    uint64_t rs, rl;
    run_range<REG>(pd, ti, g, i, rs, rl);
    const T *A = in + rs;
    uint32_t *outp = splits + j * (uint64_t)F;
    const uint64_t d = ti.d0;
    if (d == 0) {
        if (c == 0) outp[i] = 0;
        return;
    }
    T lo = wave_min(rl ? A[0] : key_max<T>());
    T hi = wave_max(rl ? A[rl - 1] : key_min<T>());
    // invariant: ilo = #keys < lo, ihi = #keys <= hi in run i; sum(ilo) < d <= sum(ihi)
    uint64_t ilo = 0, ihi = rl;
    while (lo < hi) {
        const T cand = candidate(lo, hi, c, C);
        uint64_t u = ilo, h = ihi;
        while (u < h) {
            const uint64_t m = (u + h) >> 1;
            if (A[m] <= cand) u = m + 1;
            else h = m;
        }
        uint64_t tot = u;
        for (int o = 1; o < F; o <<= 1) tot += __shfl_xor(tot, o);
        const unsigned long long mask = __ballot(tot >= d);
        const int cs = mask ? (int)((__ffsll((long long)mask) - 1) / F) : C;  // first cand with U >= d
        const uint64_t ub_cs = __shfl(u, (cs < C ? cs : 0) * F + i);
        const uint64_t ub_pr = __shfl(u, (cs > 0 ? cs - 1 : 0) * F + i);
        const T lo0 = lo, hi0 = hi;
        if (cs < C) {
            hi = candidate(lo0, hi0, cs, C);
            ihi = ub_cs;
        }
        if (cs > 0) {
            lo = candidate(lo0, hi0, cs - 1, C) + 1;
            ilo = ub_pr;
        }
    }
    // lo == hi == the key at rank d: ilo = #keys < key, ihi = #keys <= key.  The d - sum(ilo)
    // remaining slots go to the equal keys in run order (lower runs first).
    uint64_t below = ilo;
    for (int o = 1; o < F; o <<= 1) below += __shfl_xor(below, o);
    const uint64_t cnt = ihi - ilo;
    uint64_t incl = cnt;  // inclusive scan of cnt over the F lanes of this candidate group
    for (int o = 1; o < F; o <<= 1) {
        const uint64_t v = __shfl_up(incl, o);
        if (i >= o) incl += v;
    }
    const uint64_t excl = incl - cnt;
    const uint64_t need = d - below;
    const uint64_t take = need > excl ? (need - excl < cnt ? need - excl : cnt) : 0;
    if (c == 0) outp[i] = (uint32_t)(ilo + take);
}

// ---------------------------------------------------------------------------------------
// 2b. Merge one output tile of a k-way pass: stage the F input windows in LDS, then log2(F)
//     pairwise merge levels (double-buffered LDS), then coalesced stores.
// ---------------------------------------------------------------------------------------
template <typename T, int THREADS, int K, int LOGF, bool REG>
__global__ void __launch_bounds__(THREADS) mergek_kernel(const T *__restrict__ in,
                                                         T *__restrict__ out, PassDesc pd,
                                                         const uint32_t *__restrict__ splits) {
    constexpr int TILE = THREADS * K;
    constexpr int F = 1 << LOGF;
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::N;
    __shared__ __attribute__((aligned(16))) T buf[2 * padded(TILE)];
    __shared__ int soff[F + 1];
    __shared__ uint64_t sstart[F];

    const int t = threadIdx.x;
    const uint64_t j = blockIdx.x;
    TileInfo ti;
    const GroupK *g = tile_info<REG>(pd, j, TILE, ti);
    if (t < 64) {
        const int i = t & (F - 1);
        uint64_t rs, rl;
        run_range<REG>(pd, ti, g, i, rs, rl);
        const uint32_t s0 = splits[j * F + i];
        const uint32_t s1 = ti.d1 == ti.gtotal ? (uint32_t)rl : splits[(j + 1) * F + i];
        const int len = (int)(s1 - s0);
        int incl = len;
        for (int o = 1; o < F; o <<= 1) {
            const int v = __shfl_up(incl, o);
            if (i >= o) incl += v;
        }
        if (t < F) {
            soff[i + 1] = incl;
            sstart[i] = rs + s0;
            if (i == 0) soff[0] = 0;
        }
    }
    __syncthreads();
    const int total = soff[F];

    T *src = buf, *dst = buf + padded(TILE);
    {
        int seg = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int e = k * THREADS + t;
            if (e < total) {
                while (e >= soff[seg + 1]) ++seg;
                src[swz(e)] = in[sstart[seg] + (uint64_t)(e - soff[seg])];
            }
        }
    }
    __syncthreads();

#pragma unroll 1
    for (int l = 0; l < LOGF; ++l) {
        int pos = t * K;
        const int end = pos + K < total ? pos + K : total;
        const int npairs = F >> (l + 1);
        while (pos < end) {
            int lo = 0, hi = npairs - 1;  // first pair whose end lies beyond pos
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (soff[(2 * mid + 2) << l] > pos) hi = mid;
                else lo = mid + 1;
            }
            const int ps = soff[(2 * lo) << l];
            const int pm = soff[(2 * lo + 1) << l];
            const int pe = soff[(2 * lo + 2) << l];
            const int na = pm - ps, nb = pe - pm, diag = pos - ps;
            const int a = lds_merge_path(src, ps, na, pm, nb, diag);
            T m[K];
            kmerge<T, K>(src, ps, na, pm, nb, a, diag - a, m);
            const int cnt = (end < pe ? end : pe) - pos;
            if (cnt == K) {
#pragma unroll
                for (int q = 0; q < K; ++q) dst[swz(pos + q)] = m[q];
            } else {
#pragma unroll
                for (int q = 0; q < K; ++q)
                    if (q < cnt) dst[swz(pos + q)] = m[q];
            }
            pos += cnt;
        }
        __syncthreads();
        T *tmp = src;
        src = dst;
        dst = tmp;
    }

    store_tile<T, THREADS, K>(src, out + ti.base + ti.d0, total);
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------
static inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

static int ceil_log2(uint64_t x) {
    int p = 0;
    while ((1ull << p) < x) ++p;
    return p;
}

// Largest F (log2) a pass may use; DSORT_MAX_LOGF overrides it for experiments.
static int max_logf() {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("DSORT_MAX_LOGF");
        int x = e ? atoi(e) : 5;
        v = x < 1 ? 1 : (x > kMaxLogF ? kMaxLogF : x);
    }
    return v;
}

// log2(F) of each pass: as few passes as the cap allows, the bits spread evenly over them.
static std::vector<int> plan_passes(uint64_t runs) {
    std::vector<int> out;
    const int bits = ceil_log2(runs);
    if (bits == 0) return out;
    const int cap = max_logf();
    const int P = (bits + cap - 1) / cap;
    for (int p = 0; p < P; ++p) out.push_back(bits / P + (p < bits % P ? 1 : 0));
    return out;
}

template <typename T, int THREADS, int K, bool REG>
static int launch_pass(dsort_ctx *ctx, const T *src, T *dst, const PassDesc &pd, int logf,
                       uint64_t ntiles, hipStream_t s, bool timed) {
    constexpr int TILE = THREADS * K;
    int rc = ensure(ctx, &ctx->splits, &ctx->splits_bytes,
                    (size_t)(ntiles + 1) * (size_t)(1 << logf) * sizeof(uint32_t), "split vectors");
    if (rc) return rc;
    uint32_t *sp = static_cast<uint32_t *>(ctx->splits);
    hipLaunchKernelGGL((partk_kernel<T, REG>), dim3((unsigned)ceil_div(ntiles, 4)), dim3(256), 0, s,
                       src, pd, TILE, sp, ntiles);
    DSORT_HIP(ctx, hipGetLastError());
    const bool kt = timed && ctx->ev_ok && ctx->kev_used + 2 <= dsort_ctx::kMaxKev;
    if (kt) DSORT_HIP(ctx, hipEventRecord(ctx->kev[ctx->kev_used], s));
    const dim3 grid((unsigned)ntiles), block(THREADS);
    switch (logf) {
        case 1: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 1, REG>), grid, block, 0, s, src, dst, pd, sp); break;
        case 2: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 2, REG>), grid, block, 0, s, src, dst, pd, sp); break;
        case 3: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 3, REG>), grid, block, 0, s, src, dst, pd, sp); break;
        case 4: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 4, REG>), grid, block, 0, s, src, dst, pd, sp); break;
        case 5: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 5, REG>), grid, block, 0, s, src, dst, pd, sp); break;
        case 6: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 6, REG>), grid, block, 0, s, src, dst, pd, sp); break;
        default: return set_err(ctx, DSORT_EINVAL, "bad pass fan-in");
    }
    DSORT_HIP(ctx, hipGetLastError());
    if (kt) {
        DSORT_HIP(ctx, hipEventRecord(ctx->kev[ctx->kev_used + 1], s));
        ctx->kev_used += 2;
    }
    return DSORT_OK;
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
    const std::vector<int> plan = plan_passes(tiles);
    const int passes = (int)plan.size();
    ctx->stats.merge_passes = passes;
    T *scratch = nullptr;
    if (passes > 0) {
        int rc = ensure(ctx, &ctx->scratch, &ctx->scratch_bytes, n * sizeof(T), "sort scratch");
        if (rc) return rc;
        scratch = static_cast<T *>(ctx->scratch);
    }
    // Ping-pong so that the last pass lands in d_keys.  The tile sort reads d_in (which may
    // alias d_keys).
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
    uint64_t R = TILE;
    for (int p = 0; p < passes; ++p) {
        PassDesc pd{(uint64_t)n, R, 1 << plan[p], 0, nullptr};
        int rc = launch_pass<T, THREADS, K, true>(ctx, bufs[cur], bufs[cur ^ 1], pd, plan[p], tiles, s,
                                                  timed);
        if (rc) return rc;
        R <<= plan[p];
        cur ^= 1;
    }
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[2], s));
        ctx->ev_mask |= 4u;
    }
    return DSORT_OK;
}

// k-way merge of back-to-back runs of arbitrary lengths (the master merge, server.c:481-515,
// and the multi-GPU receive merge).  Up to kMaxF runs merge in one pass; more runs merge in
// levels of kMaxF-run groups.  Lower runs win ties at every level.
template <typename T>
int merge_device(dsort_ctx *ctx, const T *d_in, const size_t *lens, int k, T *d_out,
                 hipStream_t s) {
    constexpr int THREADS = Geom<T>::THREADS, K = Geom<T>::K, TILE = Geom<T>::TILE;
    ctx->stats = dsort_stats{};
    ctx->last_stream = s;
    ctx->kev_used = 0;
    uint64_t n = 0;
    std::vector<uint64_t> rl(lens, lens + k);
    for (int j = 0; j < k; ++j) n += lens[j];
    ctx->stats.keys_in = ctx->stats.keys_out = n;
    ctx->stats.tile_keys = TILE;
    if (n == 0) return DSORT_OK;
    if (k == 1) {
        DSORT_HIP(ctx, hipMemcpyAsync(d_out, d_in, n * sizeof(T), hipMemcpyDeviceToDevice, s));
        return DSORT_OK;
    }
    // levels: each merges groups of up to kMaxF consecutive runs
    int levels = 0;
    for (uint64_t r = (uint64_t)k; r > 1; r = ceil_div(r, kMaxF)) ++levels;
    ctx->stats.merge_passes = levels;
    int rc;
    if (levels > 1) {
        rc = ensure(ctx, &ctx->scratch2, &ctx->scratch2_bytes, n * sizeof(T), "merge scratch");
        if (rc) return rc;
    }
    T *dsts[2] = {d_out, static_cast<T *>(ctx->scratch2)};
    int which = (levels % 2 == 1) ? 0 : 1;
    const T *src = d_in;
    if (!ctx->groups_ev && hipEventCreateWithFlags(&ctx->groups_ev, hipEventDisableTiming) != hipSuccess)
        return set_err(ctx, DSORT_EHIP, "hipEventCreate");
    for (int l = 0; l < levels; ++l) {
        const int nr = (int)rl.size();
        const int per = nr < kMaxF ? nr : kMaxF;
        const int logf = ceil_log2((uint64_t)per) < 1 ? 1 : ceil_log2((uint64_t)per);
        const int ng = (nr + kMaxF - 1) / kMaxF;
        const size_t gbytes = (size_t)ng * sizeof(GroupK);
        if (ctx->groups_ev_pending) DSORT_HIP(ctx, hipEventSynchronize(ctx->groups_ev));
        ctx->groups_ev_pending = false;
        if (ctx->groups_host_bytes < gbytes) {
            if (ctx->groups_host) (void)hipHostFree(ctx->groups_host);
            ctx->groups_host = nullptr;
            ctx->groups_host_bytes = 0;
            DSORT_HIP(ctx, hipHostMalloc(&ctx->groups_host, gbytes, hipHostMallocDefault));
            ctx->groups_host_bytes = gbytes;
        }
        rc = ensure(ctx, &ctx->groups, &ctx->groups_bytes, gbytes, "group table");
        if (rc) return rc;
        GroupK *gh = static_cast<GroupK *>(ctx->groups_host);
        std::vector<uint64_t> next;
        uint64_t base = 0, tiles = 0;
        for (int gi = 0; gi < ng; ++gi) {
            GroupK &gk = gh[gi];
            gk.base = base;
            gk.first_tile = tiles;
            gk.nruns = 0;
            gk.pad = 0;
            uint64_t tot = 0;
            gk.roff[0] = 0;
            for (int r = gi * kMaxF; r < nr && r < (gi + 1) * kMaxF; ++r) {
                tot += rl[r];
                gk.roff[++gk.nruns] = tot;
            }
            for (int r = (int)gk.nruns + 1; r <= kMaxF; ++r) gk.roff[r] = tot;
            gk.total = tot;
            tiles += ceil_div(tot, TILE);
            base += tot;
            next.push_back(tot);
        }
        DSORT_HIP(ctx, hipMemcpyAsync(ctx->groups, gh, gbytes, hipMemcpyHostToDevice, s));
        DSORT_HIP(ctx, hipEventRecord(ctx->groups_ev, s));
        ctx->groups_ev_pending = true;
        PassDesc pd{n, 0, 1 << logf, ng, static_cast<const GroupK *>(ctx->groups)};
        T *dst = dsts[which];
        rc = launch_pass<T, THREADS, K, false>(ctx, src, dst, pd, logf, tiles, s, false);
        if (rc) return rc;
        rl.swap(next);
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
