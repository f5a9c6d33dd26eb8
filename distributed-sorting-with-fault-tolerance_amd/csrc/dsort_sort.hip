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
#include <cstring>
#include <csignal>
#include <string>
#include <type_traits>
#include <vector>

#include "dsort_bucket.h"
#include "dsort_internal.h"
#include "dsort_part.h"

#ifndef DSORT_MERGEK_MINW
#define DSORT_MERGEK_MINW 6  // waves per SIMD the merge kernel is compiled for (3 workgroups / CU)
#endif

namespace dsort {

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

// LDS layout.  Keys are grouped in 16-byte chunks (4 int32 / 2 int64) and every 8th chunk slot
// is left empty: chunk c lives at slot c + c/8.  A lane writing its K keys (chunks
// K/KPC*t ...) then lands in a distinct 16-byte slot of its ds_write_b128 lane group, every
// chunk stays 16-byte contiguous (windows and outputs move as ds_read_b128 / ds_write_b128),
// and the address of a key costs three VALU ops.
template <typename T> struct Chunk;
template <> struct Chunk<int32_t> { using V = int4; static constexpr int KPC = 4, SH = 2; };
template <> struct Chunk<int64_t> { using V = longlong2; static constexpr int KPC = 2, SH = 1; };

__device__ __forceinline__ int cslot(int c) { return c + (c >> 3); }
template <typename T>
__device__ __forceinline__ int kpos(int p) {  // LDS word (key) index of key position p
    constexpr int SH = Chunk<T>::SH;
    return p + ((p >> (SH + 3)) << SH);
}
// LDS keys to allocate for a tile of n keys (n a multiple of 8 chunks): the pad slots plus the
// window over-read (up to 2 chunks past the end).
template <typename T> __host__ __device__ constexpr int lds_keys(int n) {
    return n + n / 8 + 4 * Chunk<T>::KPC;
}

// Merge-path split on LDS: number of A keys among the first `diag` outputs of merge(A, B),
// A first on ties.  A = positions [A0, A0+na), B = [B0, B0+nb).
template <typename T>
__device__ __forceinline__ int lds_merge_path(const T *s, int A0, int na, int B0, int nb, int diag) {
    int lo = diag > nb ? diag - nb : 0;
    int hi = diag < na ? diag : na;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[kpos<T>(A0 + mid)] <= s[kpos<T>(B0 + diag - 1 - mid)]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// K keys from position `start` (keys at offset >= lim read as key_max): the K/KPC+1 chunks that
// cover the window are read as 16-byte LDS vectors, then shifted by start % KPC in registers.
template <typename T, int K>
__device__ __forceinline__ void load_window(const T *s, int start, int lim, T (&x)[K]) {
    using V = typename Chunk<T>::V;
    constexpr int KPC = Chunk<T>::KPC, SH = Chunk<T>::SH, NCH = K / KPC + 1;
    const V *sv = reinterpret_cast<const V *>(s);
    const int c0 = start >> SH, off = start & (KPC - 1);
    T w[NCH * KPC];
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
        const V v = sv[cslot(c0 + j)];
        const T *pv = reinterpret_cast<const T *>(&v);
#pragma unroll
        for (int q = 0; q < KPC; ++q) w[j * KPC + q] = pv[q];
    }
    // The shift is a bitwise blend on purpose: written as `(off & 1) ? w[i+1] : w[i]` hipcc
    // folds it into w[i + off], a dynamically indexed array, i.e. scratch memory.
    using U = typename Unsigned<T>::type;
    const U m1 = (U)0 - (U)(off & 1);
    if (KPC == 4) {
        const U m2 = (U)0 - (U)((off >> 1) & 1);
        T u[NCH * KPC - 1];
#pragma unroll
        for (int i = 0; i < NCH * KPC - 1; ++i) u[i] = (T)(((U)w[i] & ~m1) | ((U)w[i + 1] & m1));
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = (T)(((U)u[i] & ~m2) | ((U)u[i + 2] & m2));
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = (T)(((U)w[i] & ~m1) | ((U)w[i + 1] & m1));
    }
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = i < lim ? x[i] : key_max<T>();
}

// The K smallest keys of A[a..na) u B[b..nb): the two ascending K-windows form the bitonic
// sequence x ++ reverse(y); its lower half-cleaner min(x[i], y[K-1-i]) holds exactly the K
// smallest keys (as a bitonic sequence), which log2(K) compare-exchange stages sort.
template <typename T, int K>
__device__ __forceinline__ void kmerge(const T *s, int A0, int na, int B0, int nb, int a, int b,
                                       T (&m)[K]) {
    T x[K], y[K];
    load_window<T, K>(s, A0 + a, na - a, x);
    load_window<T, K>(s, B0 + b, nb - b, y);
#pragma unroll
    for (int i = 0; i < K; ++i) m[i] = x[i] < y[K - 1 - i] ? x[i] : y[K - 1 - i];
#pragma unroll
    for (int st = K / 2; st >= 1; st >>= 1) {
#pragma unroll
        for (int i = 0; i < K; ++i)
            if ((i & st) == 0) cex(m[i], m[i + st]);
    }
}

// K keys of one lane to positions [pos, pos+K), pos a multiple of K: whole chunks.
template <typename T, int K>
__device__ __forceinline__ void store_lane(T *s, int pos, const T (&v)[K]) {
    using V = typename Chunk<T>::V;
    constexpr int KPC = Chunk<T>::KPC, SH = Chunk<T>::SH;
    V *sv = reinterpret_cast<V *>(s);
#pragma unroll
    for (int j = 0; j < K / KPC; ++j) {
        V x;
        T *px = reinterpret_cast<T *>(&x);
#pragma unroll
        for (int q = 0; q < KPC; ++q) px[q] = v[j * KPC + q];
        sv[cslot((pos >> SH) + j)] = x;
    }
}

// Coalesced store of the first `valid` keys of an LDS tile: full tiles leave as 16-byte vectors
// (lane t moves chunks t, t+THREADS, ...: one ds_read_b128 and one global_store_dwordx4 each).
template <typename T, int THREADS, int K>
__device__ __forceinline__ void store_tile(const T *s, T *out, int valid) {
    constexpr int TILE = THREADS * K;
    using V = typename Chunk<T>::V;
    constexpr int KPC = Chunk<T>::KPC;
    const int t = threadIdx.x;
    if (valid == TILE && (reinterpret_cast<uintptr_t>(out) % 16) == 0) {
        V *dst = reinterpret_cast<V *>(out);
        const V *sv = reinterpret_cast<const V *>(s);
#pragma unroll
        for (int i = 0; i < K / KPC; ++i) {
            const int q = i * THREADS + t;
            dst[q] = sv[cslot(q)];
        }
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int e = i * THREADS + t;
            if (e < valid) out[e] = s[kpos<T>(e)];
        }
    }
}

// ---------------------------------------------------------------------------------------
// 1. Tile sort.
// ---------------------------------------------------------------------------------------
// tiles: NULL = tile j is keys [j * TILE, (j + 1) * TILE) of n; else tile j = tiles[j] (the
// bucketed sort's tiles, which never cross a bucket; bk::TileRef), j < *ntiles.
template <typename T, int THREADS, int K>
__global__ void __launch_bounds__(THREADS) block_sort_kernel(const T *in, T *out, uint64_t n,
                                                             const uint4 *tiles,
                                                             const uint32_t *ntiles) {
    // `in` may alias `out` (in-place sort): every workgroup reads its whole tile first.
    constexpr int TILE = THREADS * K;
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::N;
    __shared__ __attribute__((aligned(16))) T s[lds_keys<T>(TILE)];

    const int t = threadIdx.x;
    uint64_t base;
    int valid;
    if (tiles) {
        if (blockIdx.x >= *ntiles) return;  // the grid is an upper bound
        const uint4 r = tiles[blockIdx.x];
        base = (uint64_t)r.x | ((uint64_t)r.y << 32);
        valid = (int)r.z;
    } else {
        base = (uint64_t)blockIdx.x * TILE;
        const uint64_t rem = n - base;
        valid = rem < (uint64_t)TILE ? (int)rem : TILE;
    }

    T v[K];
    if (valid == TILE && (reinterpret_cast<uintptr_t>(in + base) & 15) == 0) {
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
    store_lane<T, K>(s, pos, v);
    __syncthreads();

#pragma unroll 1
    for (int r = K; r < TILE; r <<= 1) {
        const int pb = pos & ~(2 * r - 1);
        const int diag = pos - pb;
        const int a = lds_merge_path(s, pb, r, pb + r, r, diag);
        kmerge<T, K>(s, pb, r, pb + r, r, a, diag - a, v);
        __syncthreads();
        store_lane<T, K>(s, pos, v);
        __syncthreads();
    }
    store_tile<T, THREADS, K>(s, out + base, valid);
}

// ---------------------------------------------------------------------------------------
// 2b. Merge one output tile of a k-way pass.  The F input windows are staged in LDS, each padded
//     with key_max up to a multiple of K (the last one up to TILE), so every pair boundary of
//     every level is K-aligned: each lane's K outputs come from one pair, and a level is
//     merge path + bitonic window merge in registers, barrier, in-place store, barrier (one
//     TILE-key LDS buffer: 4 workgroups per CU).  Only the first `total` (real) keys leave.
// ---------------------------------------------------------------------------------------
template <typename T, int THREADS, int K, int LOGF, bool REG>
__global__ void __launch_bounds__(THREADS, DSORT_MERGEK_MINW) mergek_kernel(const T *__restrict__ in,
                                                         T *__restrict__ out, PassDesc pd, int tnom,
                                                         const uint32_t *__restrict__ splits) {
    constexpr int TILE = THREADS * K;
    constexpr int F = 1 << LOGF;
    __shared__ __attribute__((aligned(16))) T s[lds_keys<T>(TILE)];
    __shared__ int soff[F + 1];  // padded segment offsets, soff[F] = TILE
    __shared__ int slen[F];
    __shared__ uint64_t sstart[F];
    __shared__ uint64_t s_out;
    __shared__ int s_total;
    __shared__ uint64_t ubase[THREADS];  // per K-key unit: first source key, real keys in it
    __shared__ int uvalid[THREADS];

    const int t = threadIdx.x;
    const uint64_t j = blockIdx.x;
    TileInfo ti;
    const GroupK *g = tile_info<REG>(pd, j, tnom, ti);
    if (t < 64) {
        const int i = t & (F - 1);
        uint64_t rs, rl;
        run_range<REG>(pd, ti, g, i, rs, rl);
        const uint32_t s0 = splits[j * F + i];
        const uint32_t s1 = ti.jr + 1 == ti.ntg ? (uint32_t)rl : splits[(j + 1) * F + i];
        const int len = (int)(s1 - s0);
        const int plen = (len + K - 1) & ~(K - 1);
        int incl = plen, real = len;
        uint64_t before = s0;  // output offset of the tile = keys of the group below its cut
        for (int o = 1; o < F; o <<= 1) {
            const int v = __shfl_up(incl, o);
            if (i >= o) incl += v;
            real += __shfl_xor(real, o);
            before += __shfl_xor(before, o);
        }
        if (t < F) {
            soff[i + 1] = i == F - 1 ? TILE : incl;
            slen[i] = len;
            sstart[i] = rs + s0;
            if (i == 0) {
                soff[0] = 0;
                s_out = ti.base + before;
                s_total = real;
            }
        }
    }
    __syncthreads();
    const int total = s_total;

    // Staging.  Every K-key unit of the padded tile lies in one segment: thread t resolves unit t
    // (its source address and how many of its K slots hold real keys) once; then all K loads of
    // every thread are issued back to back, lane-consecutive (coalesced), with no branches.
    {
        const int pos = t * K;
        int lo = 0, hi = F - 1;  // last segment starting at or before pos
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (soff[mid] <= pos) lo = mid;
            else hi = mid - 1;
        }
        const int r = pos - soff[lo];
        int valid = slen[lo] - r;
        valid = valid < 0 ? 0 : (valid > K ? K : valid);
        ubase[t] = valid > 0 ? sstart[lo] + (uint64_t)r : ti.base;  // ti.base: a key that exists
        uvalid[t] = valid;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int e = k * THREADS + t;
        const int u = e / K, q = e & (K - 1);
        const bool real_key = q < uvalid[u];
        const T v = in[ubase[u] + (uint64_t)(real_key ? q : 0)];
        s[kpos<T>(e)] = real_key ? v : key_max<T>();
    }
    __syncthreads();

    const int pos = t * K;
#pragma unroll 1
    for (int l = 0; l < LOGF; ++l) {
        const int npairs = F >> (l + 1);
        int lo = 0, hi = npairs - 1;  // the pair holding pos
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (soff[(2 * mid + 2) << l] > pos) hi = mid;
            else lo = mid + 1;
        }
        const int ps = soff[(2 * lo) << l];
        const int pm = soff[(2 * lo + 1) << l];
        const int pe = soff[(2 * lo + 2) << l];
        const int na = pm - ps, nb = pe - pm, diag = pos - ps;
        const int a = lds_merge_path(s, ps, na, pm, nb, diag);
        T m[K];
        kmerge<T, K>(s, ps, na, pm, nb, a, diag - a, m);
        __syncthreads();
        store_lane<T, K>(s, pos, m);
        __syncthreads();
    }

    store_tile<T, THREADS, K>(s, out + s_out, total);
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------
static inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// Merge tiles: nominal size TILE - 2*slack - F*(K-1), so a cut off by at most `slack` on either
// side, with every staged run padded to a multiple of K, still fits the TILE-key LDS buffer.
template <typename T> static constexpr int slack_of() { return Geom<T>::TILE / 32; }
template <typename T> static int tnom_of(int logf) {
    return Geom<T>::TILE - 2 * slack_of<T>() - (1 << logf) * (Geom<T>::K - 1);
}

static int ceil_log2(uint64_t x) {
    int p = 0;
    while ((1ull << p) < x) ++p;
    return p;
}

int max_logf(const dsort_ctx *ctx, int type_default, int type_cap) {
    const int64_t o = ctx->opt.max_logf;
    const int x = o < 0 ? type_default : (int)o;
    return x < 1 ? 1 : (x > type_cap ? type_cap : x);
}

// log2(F) of each pass: as few passes as the cap allows, the bits spread evenly over them.
static std::vector<int> plan_passes(const dsort_ctx *ctx, uint64_t runs) {
    std::vector<int> out;
    const int bits = ceil_log2(runs);
    if (bits == 0) return out;
    const int cap = max_logf(ctx, 5, kMaxLogF);
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
                       src, pd, tnom_of<T>(logf), slack_of<T>(), sp, ntiles);
    DSORT_HIP(ctx, hipGetLastError());
    const bool kt = timed && ctx->ev_ok && ctx->kev_used + 2 <= dsort_ctx::kMaxKev;
    if (kt) DSORT_HIP(ctx, hipEventRecord(ctx->kev[ctx->kev_used], s));
    const dim3 grid((unsigned)ntiles), block(THREADS);
    switch (logf) {
        case 1: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 1, REG>), grid, block, 0, s, src, dst, pd, tnom_of<T>(logf), sp); break;
        case 2: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 2, REG>), grid, block, 0, s, src, dst, pd, tnom_of<T>(logf), sp); break;
        case 3: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 3, REG>), grid, block, 0, s, src, dst, pd, tnom_of<T>(logf), sp); break;
        case 4: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 4, REG>), grid, block, 0, s, src, dst, pd, tnom_of<T>(logf), sp); break;
        case 5: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 5, REG>), grid, block, 0, s, src, dst, pd, tnom_of<T>(logf), sp); break;
        case 6: hipLaunchKernelGGL((mergek_kernel<T, THREADS, K, 6, REG>), grid, block, 0, s, src, dst, pd, tnom_of<T>(logf), sp); break;
        default: return set_err(ctx, DSORT_EINVAL, "bad pass fan-in");
    }
    DSORT_HIP(ctx, hipGetLastError());
    if (kt) {
        DSORT_HIP(ctx, hipEventRecord(ctx->kev[ctx->kev_used + 1], s));
        ctx->kev_used += 2;
    }
    return DSORT_OK;
}

void fault_point(dsort_ctx *ctx, hipStream_t s, int pass_done) {
    if (ctx->nested == 0 && ctx->opt.kill_after_pass >= 0 && ctx->opt.kill_after_pass == pass_done) {
        (void)hipStreamSynchronize(s);
        raise(SIGKILL);
    }
}

// ---- bucketed int64 sort (dsort_bucket.h) --------------------------------------------------
// As the int32 one (dsort_wave.hip): B ~ n / 2^21 buckets by (key, index) splitters, one
// partition pass, then the tile sort (4096-key tiles) and the k-way passes inside every bucket
// (groups of <= 2^max_logf runs): 2 merge passes at 2^30 keys instead of 4.  The 32*B samples
// are sorted on the host (16-byte (key, index) pairs).  DSORT_OPT_BUCKETS as for int32; a nested
// sort never buckets.
static int bucket_count_i64(const dsort_ctx *ctx, uint64_t n) {
    if (ctx->nested) return 0;
    const int64_t forced = ctx->opt.buckets;
    if (forced == 0) return 0;
    uint64_t B = forced > 0 ? (uint64_t)forced : (n >> 21);
    if (forced < 0 && n < (1ull << 25)) return 0;
    if (n >= (1ull << 32)) return 0;
    if (B > (uint64_t)bk::BK_MAXB) B = bk::BK_MAXB;
    return B >= 2 ? (int)B : 0;
}

static int bucket_sort_i64(dsort_ctx *ctx, const int64_t *d_in, int64_t *d_keys, size_t n,
                           hipStream_t s, bool timed, int B) {
    using namespace bk;
    using T = int64_t;
    using C = Comp<T>::C;
    constexpr int THREADS = Geom<T>::THREADS, K = Geom<T>::K, TILE = Geom<T>::TILE;
    constexpr uint64_t ALIGN = 16 / sizeof(T);
    const int BP = 1 << ceil_log2((uint64_t)B);
    const int subs = bucket_wg_subs<T>(n);
    const uint64_t G = ceil_div(n, (uint64_t)subs * BK_T * Geo<T>::KPT);
    const uint64_t nchunk = ceil_div(G, BK_CHUNK);
    const uint32_t S = (uint32_t)B * BK_OS;
    const uint64_t tmax = ceil_div(n, TILE) + 2 * (uint64_t)B;
    ctx->stats = dsort_stats{};
    ctx->stats.keys_in = ctx->stats.keys_out = n;
    ctx->stats.tile_keys = TILE;
    ctx->ev_mask = 0;
    ctx->kev_used = 0;
    ctx->last_stream = s;
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    const size_t o_smp = take((size_t)S * sizeof(C)), o_spl = take((size_t)BP * sizeof(C)),
                 o_cnt = take((size_t)G * B * 4), o_part = take((size_t)nchunk * B * 8),
                 o_offs = take((size_t)G * B * 8), o_bst = take((size_t)(B + 1) * 8),
                 o_tt = take((size_t)tmax * sizeof(TileRef)), o_nt = take(4);
    int rc = ensure(ctx, &ctx->bucket, &ctx->bucket_bytes, off, "bucket partition");
    if (rc) return rc;
    char *a = static_cast<char *>(ctx->bucket);
    C *smp = reinterpret_cast<C *>(a + o_smp);
    C *spl = reinterpret_cast<C *>(a + o_spl);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(a + o_cnt);
    uint64_t *part = reinterpret_cast<uint64_t *>(a + o_part);
    uint64_t *offs = reinterpret_cast<uint64_t *>(a + o_offs);
    uint64_t *bst = reinterpret_cast<uint64_t *>(a + o_bst);
    TileRef *tt = reinterpret_cast<TileRef *>(a + o_tt);
    uint32_t *ntl = reinterpret_cast<uint32_t *>(a + o_nt);
    rc = ensure(ctx, &ctx->scratch, &ctx->scratch_bytes, n * sizeof(T), "sort scratch");
    if (rc) return rc;
    T *scratch = static_cast<T *>(ctx->scratch);
    const size_t hbytes = (size_t)BK_MAXB * BK_OS * sizeof(C) + (size_t)(BK_MAXB + 1) * 8;
    if (ctx->bucket_host_bytes < hbytes) {
        if (ctx->bucket_host) (void)hipHostFree(ctx->bucket_host);
        ctx->bucket_host = nullptr;
        ctx->bucket_host_bytes = 0;
        DSORT_HIP(ctx, hipHostMalloc(&ctx->bucket_host, hbytes, hipHostMallocDefault));
        ctx->bucket_host_bytes = hbytes;
    }
    if (!ctx->bucket_ev && hipEventCreateWithFlags(&ctx->bucket_ev, hipEventDisableTiming) != hipSuccess)
        return set_err(ctx, DSORT_EHIP, "hipEventCreate");
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[0], s));
        ctx->ev_mask |= 1u;
    }
    // 1. splitters: samples to the host, sorted in (key, index) order, every BK_OS-th back
    C *hs = static_cast<C *>(ctx->bucket_host);
    hipLaunchKernelGGL(bucket_sample_kernel<T>, dim3(ceil_div(S, 256)), dim3(256), 0, s, d_in, (uint64_t)n, smp, S);
    DSORT_HIP(ctx, hipGetLastError());
    DSORT_HIP(ctx, hipMemcpyAsync(hs, smp, (size_t)S * sizeof(C), hipMemcpyDeviceToHost, s));
    DSORT_HIP(ctx, hipStreamSynchronize(s));
    std::sort(hs, hs + S, [](const C &x, const C &y) { return Comp<T>::lt(x, y); });
    for (int b = 0; b < BP; ++b) hs[b] = b < B - 1 ? hs[(size_t)(b + 1) * BK_OS - 1] : Comp<T>::inf();
    DSORT_HIP(ctx, hipMemcpyAsync(spl, hs, (size_t)BP * sizeof(C), hipMemcpyHostToDevice, s));
    // 2. histograms, their scan, bucket starts to the host
    hipLaunchKernelGGL(bucket_hist_kernel<T>, dim3((unsigned)G), dim3(BK_T), 0, s, d_in, (uint64_t)n, spl, B, BP, subs, cnt);
    hipLaunchKernelGGL(bucket_colsum_kernel, dim3((unsigned)nchunk), dim3(BK_MAXB), 0, s, cnt, (uint32_t)G, B, part);
    hipLaunchKernelGGL(bucket_scan_kernel, dim3(1), dim3(BK_MAXB), 0, s, part, (uint32_t)nchunk, B,
                       (uint32_t)TILE, (uint32_t)ALIGN, bst, tt, ntl);
    hipLaunchKernelGGL(bucket_offsets_kernel, dim3((unsigned)nchunk), dim3(BK_MAXB), 0, s, cnt, part, bst, (uint32_t)G, B, offs);
    DSORT_HIP(ctx, hipGetLastError());
    uint64_t *hb = reinterpret_cast<uint64_t *>(hs + BK_MAXB * BK_OS);
    DSORT_HIP(ctx, hipMemcpyAsync(hb, bst, (size_t)(B + 1) * 8, hipMemcpyDeviceToHost, s));
    DSORT_HIP(ctx, hipEventRecord(ctx->bucket_ev, s));
    DSORT_HIP(ctx, hipEventSynchronize(ctx->bucket_ev));
    if (hb[B] != n) return set_err(ctx, DSORT_EHIP, "bucket partition lost keys");
    // pass plan: the tile sort's runs of every bucket; the largest bucket's run count sets the
    // levels, spread over the fewest passes of <= max_logf levels (as the int32 driver)
    std::vector<std::vector<uint64_t>> runs(B);
    uint64_t maxruns = 1;
    for (int b = 0; b < B; ++b) {
        const uint64_t len = hb[b + 1] - hb[b], h = bucket_head(hb[b], len, ALIGN);
        if (h) runs[b].push_back(h);
        for (uint64_t o = h; o < len; o += TILE) runs[b].push_back(len - o < (uint64_t)TILE ? len - o : TILE);
        maxruns = runs[b].size() > maxruns ? runs[b].size() : maxruns;
    }
    const std::vector<int> pbits = plan_passes(ctx, maxruns);
    const int passes = (int)pbits.size();
    ctx->stats.merge_passes = passes;
    T *bufs[2] = {d_keys, scratch};
    int cur = (passes % 2 == 0) ? 0 : 1;
    T *part_out = (bufs[cur] == d_in) ? bufs[cur ^ 1] : bufs[cur];
    hipLaunchKernelGGL(bucket_scatter_kernel<T>, dim3((unsigned)G), dim3(BK_T), 0, s, d_in, (uint64_t)n, spl, B, BP, subs, offs, part_out);
    DSORT_HIP(ctx, hipGetLastError());
    // 3. tile sort inside the buckets
    hipLaunchKernelGGL((block_sort_kernel<T, THREADS, K>), dim3((unsigned)tmax), dim3(THREADS), 0, s,
                       part_out, bufs[cur], (uint64_t)n, reinterpret_cast<const uint4 *>(tt), ntl);
    DSORT_HIP(ctx, hipGetLastError());
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[1], s));
        ctx->ev_mask |= 2u;
    }
    // 4. group tables of every pass (one staging buffer, one copy), then the passes.  Per-bucket
    // fan-in as in the int32 driver: the passes after the first keep the global fan-in, the first
    // resolves only the levels the bucket still needs; one launch per kernel fan-in of a pass.
    struct PassPlan { int logf; uint64_t ngroups, ntiles; size_t group_off, tile_off; int pass; };
    std::vector<PassPlan> plan;  // one entry per launch
    std::vector<GroupK> groups;
    std::vector<uint32_t> tgroup;
    std::vector<int> tail(passes + 1, 0);
    for (int p = passes - 1; p >= 0; --p) tail[p] = tail[p + 1] + pbits[p];
    std::vector<int> blev(B);
    for (int b = 0; b < B; ++b) blev[b] = ceil_log2((uint64_t)runs[b].size());
    for (int p = 0; p < passes; ++p) {
        std::vector<GroupK> pg;
        std::vector<int> pk;
        uint64_t base = 0;
        for (int b = 0; b < B; ++b) {
            const int need = blev[b] - tail[p + 1];
            const int fb = need < 0 ? 0 : (need < pbits[p] ? need : pbits[p]);
            blev[b] -= fb;
            const size_t MAXF = (size_t)1 << fb;
            std::vector<uint64_t> next;
            const size_t nr = runs[b].size();
            for (size_t r0 = 0; r0 < nr; r0 += MAXF) {
                GroupK gk{};
                gk.base = base;
                uint64_t tot = 0;
                for (size_t r = r0; r < nr && r < r0 + MAXF; ++r) {
                    tot += runs[b][r];
                    gk.roff[++gk.nruns] = tot;
                }
                for (int r = (int)gk.nruns + 1; r <= kMaxF; ++r) gk.roff[r] = tot;
                gk.total = tot;
                base += tot;
                next.push_back(tot);
                pg.push_back(gk);
                const int kl = ceil_log2((uint64_t)gk.nruns);
                pk.push_back(kl < 1 ? 1 : kl);
            }
            runs[b].swap(next);
        }
        int lmin = 99, lmax = 1;
        for (size_t g = 0; g < pg.size(); ++g)
            if (pk[g] >= 2) { lmin = pk[g] < lmin ? pk[g] : lmin; lmax = pk[g] > lmax ? pk[g] : lmax; }
        if (lmin == 99) lmin = lmax = 1;
        for (size_t g = 0; g < pg.size(); ++g) pk[g] = pk[g] < lmin ? lmin : pk[g];
        for (int l = lmin; l <= lmax; ++l) {
            PassPlan pp{l, 0, 0, groups.size(), tgroup.size(), p};
            const uint64_t tn = (uint64_t)tnom_of<T>(l);
            uint64_t tiles = 0;
            for (size_t g = 0; g < pg.size(); ++g) {
                if (pk[g] != l) continue;
                GroupK gk = pg[g];
                gk.first_tile = tiles;
                const uint64_t gt = ceil_div(gk.total, tn);
                for (uint64_t k = 0; k < gt; ++k) tgroup.push_back((uint32_t)(groups.size() - pp.group_off));
                tiles += gt;
                groups.push_back(gk);
            }
            pp.ngroups = groups.size() - pp.group_off;
            pp.ntiles = tiles;
            if (pp.ngroups) plan.push_back(pp);
        }
    }
    if (passes > 0) {
        const size_t gbytes = groups.size() * sizeof(GroupK), tbytes = tgroup.size() * sizeof(uint32_t);
        const size_t tb_off = (gbytes + 255) & ~(size_t)255;
        if (ctx->groups_ev_pending) DSORT_HIP(ctx, hipEventSynchronize(ctx->groups_ev));
        ctx->groups_ev_pending = false;
        if (ctx->groups_host_bytes < tb_off + tbytes) {
            if (ctx->groups_host) (void)hipHostFree(ctx->groups_host);
            ctx->groups_host = nullptr;
            ctx->groups_host_bytes = 0;
            DSORT_HIP(ctx, hipHostMalloc(&ctx->groups_host, tb_off + tbytes, hipHostMallocDefault));
            ctx->groups_host_bytes = tb_off + tbytes;
        }
        rc = ensure(ctx, &ctx->groups, &ctx->groups_bytes, tb_off + tbytes, "group table");
        if (rc) return rc;
        std::memcpy(ctx->groups_host, groups.data(), gbytes);
        std::memcpy(static_cast<char *>(ctx->groups_host) + tb_off, tgroup.data(), tbytes);
        DSORT_HIP(ctx, hipMemcpyAsync(ctx->groups, ctx->groups_host, tb_off + tbytes, hipMemcpyHostToDevice, s));
        if (!ctx->groups_ev && hipEventCreateWithFlags(&ctx->groups_ev, hipEventDisableTiming) != hipSuccess)
            return set_err(ctx, DSORT_EHIP, "hipEventCreate");
        DSORT_HIP(ctx, hipEventRecord(ctx->groups_ev, s));
        ctx->groups_ev_pending = true;
        const GroupK *dg = static_cast<const GroupK *>(ctx->groups);
        const uint32_t *dt = reinterpret_cast<const uint32_t *>(static_cast<const char *>(ctx->groups) + tb_off);
        for (size_t q = 0; q < plan.size(); ++q) {
            PassDesc pd{(uint64_t)n, 0, 1 << plan[q].logf, (int)plan[q].ngroups, dg + plan[q].group_off};
            pd.tile_group = dt + plan[q].tile_off;
            rc = launch_pass<T, THREADS, K, false>(ctx, bufs[cur], bufs[cur ^ 1], pd, plan[q].logf,
                                                   plan[q].ntiles, s, timed);
            if (rc) return rc;
            if (q + 1 == plan.size() || plan[q + 1].pass != plan[q].pass) {  // pass complete
                cur ^= 1;
                fault_point(ctx, s, plan[q].pass);
            }
        }
    }
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[2], s));
        ctx->ev_mask |= 4u;
    }
    return DSORT_OK;
}

template <typename T>
int sort_device(dsort_ctx *ctx, const T *d_in, T *d_keys, size_t n, hipStream_t s, bool timed) {
    if constexpr (std::is_same<T, int32_t>::value) {
        return wave_sort_i32(ctx, d_in, d_keys, n, s, timed);
    } else {
    if (const int B = bucket_count_i64(ctx, n)) return bucket_sort_i64(ctx, d_in, d_keys, n, s, timed, B);
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
    const std::vector<int> plan = plan_passes(ctx, tiles);
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
                       s, d_in, bufs[cur], (uint64_t)n, nullptr, nullptr);
    DSORT_HIP(ctx, hipGetLastError());
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[1], s));
        ctx->ev_mask |= 2u;
    }
    uint64_t R = TILE;
    for (int p = 0; p < passes; ++p) {
        PassDesc pd{(uint64_t)n, R, 1 << plan[p], 0, nullptr};
        const uint64_t gsize = R << plan[p];
        const uint64_t ngroups = ceil_div(n, gsize);
        const uint64_t tn = (uint64_t)tnom_of<T>(plan[p]);
        const uint64_t tpg = ceil_div(gsize, tn);
        const uint64_t mtiles = (ngroups - 1) * tpg + ceil_div(n - (ngroups - 1) * gsize, tn);
        int rc = launch_pass<T, THREADS, K, true>(ctx, bufs[cur], bufs[cur ^ 1], pd, plan[p], mtiles, s,
                                                  timed);
        if (rc) return rc;
        R <<= plan[p];
        cur ^= 1;
        fault_point(ctx, s, p);
    }
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[2], s));
        ctx->ev_mask |= 4u;
    }
    return DSORT_OK;
    }
}

// k-way merge of back-to-back runs of arbitrary lengths (the master merge, server.c:481-515,
// and the multi-GPU receive merge).  Up to kMaxF runs merge in one pass; more runs merge in
// levels of kMaxF-run groups.  Lower runs win ties at every level.
template <typename T>
int merge_device(dsort_ctx *ctx, const T *d_in, const size_t *lens, int k, T *d_out,
                 hipStream_t s, bool keep_stats) {
    if constexpr (std::is_same<T, int32_t>::value) {
        return wave_merge_i32(ctx, d_in, lens, k, d_out, s, keep_stats);
    } else {
    constexpr int THREADS = Geom<T>::THREADS, K = Geom<T>::K, TILE = Geom<T>::TILE;
    if (!keep_stats) {
        ctx->stats = dsort_stats{};
        ctx->kev_used = 0;
    }
    ctx->last_stream = s;
    uint64_t n = 0;
    std::vector<uint64_t> rl(lens, lens + k);
    for (int j = 0; j < k; ++j) n += lens[j];
    if (!keep_stats) {
        ctx->stats.keys_in = ctx->stats.keys_out = n;
        ctx->stats.tile_keys = TILE;
    }
    if (n == 0) return DSORT_OK;
    if (k == 1) {
        DSORT_HIP(ctx, hipMemcpyAsync(d_out, d_in, n * sizeof(T), hipMemcpyDeviceToDevice, s));
        return DSORT_OK;
    }
    // levels: each merges groups of up to kMaxF consecutive runs
    int levels = 0;
    for (uint64_t r = (uint64_t)k; r > 1; r = ceil_div(r, kMaxF)) ++levels;
    if (!keep_stats) ctx->stats.merge_passes = levels;
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
            tiles += ceil_div(tot, (uint64_t)tnom_of<T>(logf));
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
}

template int sort_device<int32_t>(dsort_ctx *, const int32_t *, int32_t *, size_t, hipStream_t,
                                  bool);
template int sort_device<int64_t>(dsort_ctx *, const int64_t *, int64_t *, size_t, hipStream_t,
                                  bool);
template int merge_device<int32_t>(dsort_ctx *, const int32_t *, const size_t *, int, int32_t *,
                                   hipStream_t, bool);
template int merge_device<int64_t>(dsort_ctx *, const int64_t *, const size_t *, int, int64_t *,
                                   hipStream_t, bool);

}  // namespace dsort
