// dsort_sub.h -- the second partition level of the bucketed sort (namespace dsort::sb; included
// by dsort_wave.hip).
//
// The first level (dsort_bucket.h) cuts the keys into B <= 1024 buckets of about 2^20 keys.  In
// round 1 every bucket was then tile-sorted and merged in two k-way passes (64..128 tiles per
// bucket), and those passes were half of the sort's time.  Here every bucket is cut once more,
// into `nsub` sub-buckets of about TILE / 8 keys by splitters from a sample of the bucket, and
// consecutive sub-buckets are packed into tiles of at most TILE keys.  A tile then holds exactly
// the keys of its output range, so the tile sort finishes the sort: no merge pass at all.  A
// sub-bucket that alone exceeds a tile (not expected from the sampling; possible for adversarial
// inputs) is tile-sorted in pieces and merged afterwards (merge records, host side).
//
// Order: keys are compared as composites (key, position in the first level's output) and the
// splitters are sampled composites, so equal keys spread over sub-buckets like any other
// (DESIGN.md §3.2).
//
// Kernels:
//   sb_sample_kernel    per bucket: ns = nsub * os keys at regular positions
//   (the samples of all buckets sorted by (key, position) in one nested int64 sort of
//   composites -- int64 keys first sort the keys and rank them, sb_rank_kernel -- bucket b's
//   samples keep their range [soff, soff + ns) since the buckets are ordered)
//   sb_splitter_kernel  per bucket: nsub - 1 splitters (key, position) + the slot table
//   sb_hist_kernel      per chunk (<= SB_CH keys of one bucket): keys per sub-bucket
//   sb_scan_kernel      per bucket: sub-bucket starts, per-chunk offsets, tile packing
//   sb_scatter_kernel   per chunk: keys grouped by sub-bucket in LDS, written to their places
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dsort_bucket.h"

namespace dsort {
namespace sb {

constexpr int SB_T = 256;              // threads of the per-chunk kernels
constexpr int SB_MAXS = 1024;          // sub-buckets per bucket at most
constexpr int SB_SLOTB = 10;           // slot table: 1024 key slots per bucket
constexpr int SB_SLOTS = 1 << SB_SLOTB;
#ifndef DSORT_SUB_TOTALS
#define DSORT_SUB_TOTALS 1  // local path: sb_local_kernel adds up the sub-bucket totals (global atomics)
#endif
constexpr int SB_ST = 4;               // sub-tiles per chunk
template <typename T> constexpr int SB_KPT = sizeof(T) == 4 ? 16 : 8;  // keys per thread per sub-tile
template <typename T> constexpr int SB_SUB = SB_T * SB_KPT<T>;   // keys of a sub-tile
template <typename T> constexpr int SB_CH = SB_ST * SB_SUB<T>;   // keys of a chunk

struct BInfo {       // one first-level bucket (host-built)
    uint64_t start;  // first key of its output range (one piece: also its first key in the source)
    uint64_t soff;   // first sample
    uint32_t len;    // keys
    uint32_t nsub;   // sub-buckets, 1..SB_MAXS
    uint32_t ns;     // samples (0 when nsub == 1)
    uint32_t c0, c1; // chunks [c0, c1)
    uint32_t single; // sample single keys (the retry after the local partition: its chunks are
                     // partitioned, so adjacent keys lie in one old sub-bucket)
    uint32_t multi;  // the bucket's keys lie in several source pieces (the multi-GPU path: one per
                     // sending rank), found through its chunks (Chunk.boff); else at start..
};

struct Chunk {
    uint64_t start;  // first key in the source
    uint32_t len;
    uint32_t b;
    uint32_t boff;   // keys of its bucket in the chunks before it
    uint32_t pad;
};

// Source position of key p (0 <= p < len) of bucket b in the order of its chunks: b.start + p for a
// one-piece bucket; a bucket of several pieces finds its chunk (binary search over boff).
__device__ __forceinline__ uint64_t bucket_src_pos(const BInfo &b, const Chunk *ch, uint64_t p) {
    if (!b.multi) return b.start + p;
    uint32_t lo = b.c0, hi = b.c1 - 1;  // the last chunk with boff <= p
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (ch[mid].boff <= p) lo = mid;
        else hi = mid - 1;
    }
    return ch[lo].start + (p - ch[lo].boff);
}

// Chunk c: from the table, or (ch == NULL: the first level, one segment) SB_CH<T>-key pieces of
// segment 0 in order.
template <typename T>
__device__ __forceinline__ Chunk chunk_of(const Chunk *ch, const BInfo *bi, uint32_t c) {
    if (ch) return ch[c];
    const uint64_t o = (uint64_t)c * SB_CH<T>, len = bi[0].len;
    return Chunk{bi[0].start + o, (uint32_t)(len - o < (uint64_t)SB_CH<T> ? len - o : (uint64_t)SB_CH<T>), 0u,
                 (uint32_t)o, 0u};
}

template <typename T> struct KeyU;
template <> struct KeyU<int32_t> { using U = uint32_t; };
template <> struct KeyU<int64_t> { using U = uint64_t; };

template <typename T>
struct SlotFn {      // slot(key) = (clamp(key, klo, ..) - klo) >> sh, capped at SB_SLOTS - 1
    T klo;
    uint32_t sh;
    uint32_t pad;
};

template <typename T>
__host__ __device__ __forceinline__ uint32_t slot_of(T key, T klo, uint32_t sh) {
    using U = typename KeyU<T>::U;
    const U d = key < klo ? (U)0 : (U)((U)key - (U)klo);
    const U s = d >> sh;
    return s > (U)(SB_SLOTS - 1) ? (uint32_t)(SB_SLOTS - 1) : (uint32_t)s;
}

// A splitter: key and position (8 bytes for int32 keys, 16 for int64: one LDS read).
template <typename T> struct Spl;
template <> struct __attribute__((aligned(8))) Spl<int32_t> {
    int32_t k;
    uint32_t p;
};
template <> struct __attribute__((aligned(16))) Spl<int64_t> {
    int64_t k;
    uint32_t p, pad;
};

// splitter s lies below key `key` at position `pos`
template <typename T>
__device__ __forceinline__ bool below(const Spl<T> &s, T key, uint32_t pos) {
    return s.k < key || (s.k == key && s.p <= pos);
}

// sub-bucket of (key, pos): the number of splitters below it.  Splitters outside the key's
// slot are below it iff their slot is lower (slot_of is monotone), so only the slot's own
// splitters are searched -- usually none or one.
// The part after the reads: r = the key's slot entry, a and b = the slot's first two splitters.
// One-key slots (bit 15 of the entry: three or more splitters, all of one key K -- a duplicate
// run of a skewed bucket, int64 Zipf): a key other than K lies below or above all of them, with no
// search.  A copy of K positioned before the first of them or from the last one on goes to the
// outer sub-bucket the (key, position) order gives it, so those stay as full as sampled; the
// copies in between may go to any sub-bucket between the first and the last K splitter (each holds
// only K), and a hash of the position spreads them evenly -- instead of a divergent binary search
// (C4: second level 3.0 -> 2.3 ms).  (In proportion to the position, the first level's rule, the
// sub-buckets came out uneven -- a bucket at the edge of a heavy key's run holds that key's copies
// from one end of the input only -- and one overflowed a tile in most sorts.)  Only this function
// places keys on the local path; the scatter path's two passes both call it.
constexpr uint32_t SB_ONEKEY = 0x8000u;
template <typename T>
__device__ __forceinline__ int sub_pick(const Spl<T> *spl, uint32_t r, const Spl<T> &a, const Spl<T> &b, T key,
                                        uint32_t pos) {
    int lo = (int)(r & 0x7FFF);
    const int hi = (int)(r >> 16);
    if (r & SB_ONEKEY) {
        if (key != a.k) return key < a.k ? lo : hi;
        if (pos < a.p) return lo;
        const Spl<T> z = spl[hi - 1];
        if (pos >= z.p) return hi;
        // (any sub-bucket in [lo + 1, hi - 1] holds only K: spread the copies by a hash of the
        // position, which balances them whatever their positions are)
        const float f = (float)((pos * 2654435761u) >> 8) * 0x1p-24f;
        const int jj = (int)(f * (float)(hi - lo - 1));
        return lo + 1 + (jj < hi - lo - 2 ? jj : hi - lo - 2);
    }
    const int j = lo + (lo < hi && below<T>(a, key, pos) ? 1 + (lo + 1 < hi && below<T>(b, key, pos)) : 0);
    if (j < lo + 2 || j >= hi) return j;
    lo = j;
    int h = hi;
    while (lo < h) {
        const int mid = (lo + h) >> 1;
        if (below<T>(spl[mid], key, pos)) lo = mid + 1;
        else h = mid;
    }
    return lo;
}
template <typename T>
__device__ __forceinline__ int sub_of(const Spl<T> *spl, const uint32_t *rng, T klo, uint32_t sh, T key,
                                      uint32_t pos) {
    // the slot's first two splitters, read only by the lanes whose slot holds them (a slot holds
    // none in about 60 % of the keys' cases at 2^30 uniform: fewer lanes in every random LDS read,
    // fewer bank conflicts), then the rare crowded slot
    const uint32_t r = rng[slot_of<T>(key, klo, sh)];
    const int lo = (int)(r & 0x7FFF), hi = (int)(r >> 16);
    Spl<T> a{}, b{};
    if (lo < hi) a = spl[lo];
    if (lo + 1 < hi) b = spl[lo + 1];
    return sub_pick<T>(spl, r, a, b, key, pos);
}

// Samples are taken in runs of SB_RUN consecutive keys (one 64-byte line, mostly, instead of one
// line per sample: the sampling kernel went from 81 us to 31 us per sort at 2^30 int32), run r of the
// bucket's ns / SB_RUN runs centred at ((2r + 1) len) / (2 nr).  The first level's output holds a
// bucket's keys in the order its workgroups met them, so a run samples as well as isolated keys do
// on unstructured input, and on sorted input the bucket is sorted and every run lies at its
// quantile.  Sample g (global index, bucket b's samples at [soff, soff + ns)) is written as the
// key (smp) and, for int32, as the composite key * 2^32 + g (cmp), whose sort orders the samples
// by (key, position).  A bucket whose ns is not a multiple of SB_RUN (DSORT_OPT_SUB_OVERSAMPLE
// not a multiple of 8) samples single keys.  Runs of 8 keys (round 4, at 8 samples per
// sub-bucket): the kernel fetches a line per run, half the lines of runs of 4 (-0.05 ms per sort
// at 2^30 int32; no over-tile sub-bucket in 24 sorts).
#ifndef DSORT_SB_RUN
#define DSORT_SB_RUN 8
#endif
constexpr uint32_t SB_RUN = DSORT_SB_RUN;
constexpr uint32_t SB_SMP_CH = 1024;  // chunks of a several-piece bucket staged in LDS for its sampling
__host__ __device__ __forceinline__ uint32_t sample_run(const BInfo &b) { return b.single || b.ns % SB_RUN ? 1u : SB_RUN; }
// (positions relative to the bucket: bucket_src_pos maps them to the source)
__host__ __device__ __forceinline__ uint64_t sample_run_pos(const BInfo &b, uint32_t run, uint64_t r) {
    const uint64_t nr = b.ns / run;
    const uint64_t p = ((2 * r + 1) * b.len) / (2 * nr);
    return p + run > b.len ? b.len - run : p;
}
__host__ __device__ __forceinline__ uint64_t sample_pos(const BInfo &b, uint64_t k) {
    const uint32_t run = sample_run(b);
    return sample_run_pos(b, run, k / run) + k % run;
}
template <typename T>
__global__ void __launch_bounds__(SB_T) sb_sample_kernel(const T *__restrict__ src, const BInfo *__restrict__ bi,
                                                         const Chunk *__restrict__ ch, T *__restrict__ smp,
                                                         int64_t *__restrict__ cmp) {
    const BInfo b = bi[blockIdx.x];
    auto put = [&](uint64_t k, T key) {
        const uint64_t g = b.soff + k;
        smp[g] = key;
        if constexpr (sizeof(T) == 4) cmp[g] = (int64_t)((uint64_t)(int64_t)key << 32 | (uint32_t)g);
    };
    if (sample_run(b) == SB_RUN && !b.multi) {
#pragma unroll 2  // (independent gathers in flight)
        for (uint32_t r = threadIdx.x; r < b.ns / SB_RUN; r += SB_T) {
            const T *p = src + b.start + sample_run_pos(b, SB_RUN, r);
            T key[SB_RUN];
#pragma unroll
            for (uint32_t i = 0; i < SB_RUN; ++i) key[i] = p[i];
#pragma unroll
            for (uint32_t i = 0; i < SB_RUN; ++i) put((uint64_t)r * SB_RUN + i, key[i]);
        }
    } else if (b.multi && b.c1 - b.c0 <= SB_SMP_CH) {
        // a bucket of several pieces: its chunks' offsets in LDS, a run's chunk found there (a run
        // crossing a chunk end takes its keys one by one)
        __shared__ uint32_t cbo[SB_SMP_CH + 1];
        __shared__ uint64_t cst[SB_SMP_CH];
        const uint32_t nc = b.c1 - b.c0;
        for (uint32_t c = threadIdx.x; c < nc; c += SB_T) {
            const Chunk x = ch[b.c0 + c];
            cbo[c] = x.boff;
            cst[c] = x.start;
        }
        if (threadIdx.x == 0) cbo[nc] = b.len;
        __syncthreads();
        const uint32_t run = sample_run(b);
        for (uint32_t r = threadIdx.x; r < b.ns / run; r += SB_T) {
            const uint32_t p = (uint32_t)sample_run_pos(b, run, r);
            uint32_t lo = 0, hi = nc - 1;  // the last chunk with boff <= p
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (cbo[mid] <= p) lo = mid;
                else hi = mid - 1;
            }
            if (p + run <= cbo[lo + 1]) {
                const T *q = src + cst[lo] + (p - cbo[lo]);
                for (uint32_t i = 0; i < run; ++i) put((uint64_t)r * run + i, q[i]);
            } else {
                for (uint32_t i = 0; i < run; ++i) put((uint64_t)r * run + i, src[bucket_src_pos(b, ch, p + i)]);
            }
        }
    } else {
        // (a run of a bucket of many pieces may cross a chunk: every key mapped on its own)
        for (uint32_t k = threadIdx.x; k < b.ns; k += SB_T) put(k, src[bucket_src_pos(b, ch, sample_pos(b, k))]);
    }
}

template <typename T>
__device__ __forceinline__ uint32_t lower_bound_k(const T *a, uint32_t n, T k) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
template <typename T>
__device__ __forceinline__ uint32_t upper_bound_k(const T *a, uint32_t n, T k) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (!(k < a[mid])) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// int64 keys do not fit a composite with the sample index: once the keys are sorted (srt), the
// composite of sample g is (index of the first sample equal to its key in srt) * 2^32 + g, whose
// sort orders the samples by (key, position) as well.
__global__ void __launch_bounds__(SB_T) sb_rank_kernel(const int64_t *__restrict__ smp, const int64_t *__restrict__ srt,
                                                       const BInfo *__restrict__ bi, int64_t *__restrict__ cmp) {
    const BInfo b = bi[blockIdx.x];
    for (uint32_t k = threadIdx.x; k < b.ns; k += SB_T) {
        const uint64_t g = b.soff + k;
        const uint64_t lo = b.soff + lower_bound_k<int64_t>(srt + b.soff, b.ns, smp[g]);
        cmp[g] = (int64_t)(lo << 32 | (uint32_t)g);
    }
}

// Splitter j of bucket b (j < nsub - 1) = the sample of rank (j + 1) * os - 1 in (key, position)
// order: its key and position.  Keys are compared as (key, position in the first level's
// output), so duplicates split over sub-buckets exactly like distinct keys (sizes depend on the
// sample positions only).  Then the slot table: rng[s] = (splitters with slot < s) |
// (splitters with slot <= s) << 16.
template <typename T>
__global__ void __launch_bounds__(SB_MAXS) sb_splitter_kernel(const int64_t *__restrict__ cmp, const T *__restrict__ smp,
                                                              const BInfo *__restrict__ bi, const Chunk *__restrict__ ch,
                                                              int os, int SS,
                                                              Spl<T> *__restrict__ spl, uint32_t *__restrict__ rng,
                                                              SlotFn<T> *__restrict__ sfn, uint32_t *__restrict__ stot) {
    using U = typename KeyU<T>::U;
    __shared__ uint32_t sslot[SB_MAXS];
    __shared__ T skey[SB_MAXS];
    const BInfo b = bi[blockIdx.x];
    const int tid = threadIdx.x;
    if (stot)  // (the bucket's sub-bucket totals, which sb_local_kernel adds up)
        for (int j = tid; j < SS; j += SB_MAXS) stot[(uint64_t)blockIdx.x * SS + j] = 0;
    const int nspl = (int)b.nsub - 1;
    T klo = 0;
    uint32_t sh = 0;
    if (nspl > 0) {
        const int64_t *cm = cmp + b.soff;
        klo = smp[(uint32_t)cm[0]];
        const U span = (U)((U)smp[(uint32_t)cm[b.ns - 1]] - (U)klo);
        while (sh < 8 * sizeof(T) && (span >> sh) >= (U)SB_SLOTS) ++sh;
        if (tid < nspl) {
            const uint32_t g = (uint32_t)cm[(uint32_t)(tid + 1) * (uint32_t)os - 1];
            const T K = smp[g];
            Spl<T> sp{};
            sp.k = K;
            sp.p = (uint32_t)bucket_src_pos(b, ch, sample_pos(b, g - b.soff));
            spl[(uint64_t)blockIdx.x * SS + tid] = sp;
            sslot[tid] = slot_of<T>(K, klo, sh);
            skey[tid] = K;
        }
    }
    __syncthreads();
    for (int s = tid; s < SB_SLOTS; s += SB_MAXS) {
        uint32_t lo = 0, hi = (uint32_t)(nspl > 0 ? nspl : 0);
        while (lo < hi) {  // first splitter with slot >= s
            const uint32_t mid = (lo + hi) >> 1;
            if (sslot[mid] < (uint32_t)s) lo = mid + 1;
            else hi = mid;
        }
        uint32_t lo2 = lo, hi2 = (uint32_t)(nspl > 0 ? nspl : 0);
        while (lo2 < hi2) {  // first splitter with slot > s
            const uint32_t mid = (lo2 + hi2) >> 1;
            if (sslot[mid] <= (uint32_t)s) lo2 = mid + 1;
            else hi2 = mid;
        }
        const bool one = lo2 >= lo + 3 && skey[lo] == skey[lo2 - 1];
        rng[(uint64_t)blockIdx.x * SB_SLOTS + s] = lo | (one ? SB_ONEKEY : 0u) | (lo2 << 16);
    }
    if (tid == 0) sfn[blockIdx.x] = SlotFn<T>{klo, sh, 0};
}

template <typename T>
__device__ __forceinline__ void load_sub_tables(const BInfo &b, uint32_t bid, int SS, const Spl<T> *spl_g,
                                                const uint32_t *rng_g, Spl<T> *spl, uint32_t *rng) {
    const int nspl = (int)b.nsub - 1;
    for (int j = threadIdx.x; j < nspl; j += blockDim.x) spl[j] = spl_g[(uint64_t)bid * SS + j];
    for (int s = threadIdx.x; s < SB_SLOTS; s += blockDim.x) rng[s] = rng_g[(uint64_t)bid * SB_SLOTS + s];
}

// counts[c * SS + j] = keys of chunk c in sub-bucket j of its bucket
template <typename T>
__global__ void __launch_bounds__(SB_T) sb_hist_kernel(const T *__restrict__ src, const Chunk *__restrict__ ch,
                                                       const BInfo *__restrict__ bi, int SS,
                                                       const Spl<T> *__restrict__ spl_g,
                                                       const uint32_t *__restrict__ rng_g,
                                                       const SlotFn<T> *__restrict__ sfn,
                                                       uint32_t *__restrict__ counts) {
    __shared__ Spl<T> spl[SB_MAXS + 1];  // + 1: sub_of reads two entries
    __shared__ uint32_t rng[SB_SLOTS];
    __shared__ uint32_t hist[SB_MAXS];
    const Chunk c = chunk_of<T>(ch, bi, blockIdx.x);
    const BInfo b = bi[c.b];
    uint32_t *out = counts + (uint64_t)blockIdx.x * SS;
    if (b.nsub == 1) {
        if (threadIdx.x == 0) out[0] = c.len;
        return;
    }
    load_sub_tables<T>(b, c.b, SS, spl_g, rng_g, spl, rng);
    for (int j = threadIdx.x; j < (int)b.nsub; j += SB_T) hist[j] = 0;
    const SlotFn<T> f = sfn[c.b];
    __syncthreads();
    constexpr int UN = 8;
#pragma unroll 1
    for (uint32_t i0 = 0; i0 < c.len; i0 += UN * SB_T) {
        T key[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const uint32_t i = i0 + threadIdx.x + u * SB_T;
            key[u] = i < c.len ? src[c.start + i] : T(0);
        }
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const uint32_t i = i0 + threadIdx.x + u * SB_T;
            if (i < c.len)
                atomicAdd(&hist[sub_of<T>(spl, rng, f.klo, f.sh, key[u], (uint32_t)(c.start + i))], 1u);
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < (int)b.nsub; j += SB_T) out[j] = hist[j];
}

// exclusive scan over a SB_MAXS-thread workgroup (one value per thread); `all` = total
__device__ __forceinline__ uint32_t scan_excl_1024(uint32_t v, uint32_t *wsum, uint32_t &all) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t incl = wave_incl_sum(v);
    __syncthreads();
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t off = 0;
    all = 0;
    for (int i = 0; i < SB_MAXS / 64; ++i) {
        const uint32_t x = wsum[i];
        off += i < w ? x : 0;
        all += x;
    }
    return off + incl - v;
}

// Packing of sub-buckets into tiles (host mirror: sub_tile_runs in dsort_wave.hip).  A tile
// starting at position p may hold TILE - off(p) keys, off(p) = (p + mis) mod ALIGN (the tile
// sort loads 16-byte-aligned vectors from p - off(p)).  Tiles are greedy: a tile starting with
// sub-bucket i takes i, i+1, .. while they fit.  A sub-bucket that alone exceeds its tile's room
// becomes pieces: TILE - off(p) keys, then TILE-key pieces, merged afterwards (merge record).
// LOCAL: such a sub-bucket is cut by chunks instead -- tiles [tile0, tile0 + nt) each gather the
// sub-bucket's pieces of a run of consecutive chunks -- and those tiles' outputs are merged
// afterwards (the host reads their sizes from the tile records).
struct Ovf {
    uint64_t start;
    uint64_t len;
    uint32_t tile0, nt;  // LOCAL: the tiles the sub-bucket was cut into
};

// A tile of the local-partition path: sub-buckets [j0, j1) of bucket b, `valid` keys, output
// position `base`; the tile sort gathers one piece per chunk of the bucket.
struct GTile {
    uint64_t base;         // output position
    uint64_t src;          // first key of the bucket's first chunk (chunk c0 + k at src + k * SB_LCH)
    uint32_t valid, b, j0, j1;
    uint32_t c0, nch;      // the bucket's chunks [c0, c0 + nch)
    uint32_t nsub, flags;  // the bucket's sub-buckets; bit 0: gathered key by key (no vector room);
                           // bits 8-31: a split tile's start inside its first chunk's piece
};

// What the gathering tile sort needs (block_sort_w_kernel<T, true>): its tiles, the chunk and
// bucket tables and the chunks' prefix tables (pref[c * (SS + 1) + j]).
struct Gather {
    const GTile *tiles;
    const Chunk *ch;
    const BInfo *bi;
    const uint32_t *pref;
    const uint2 *pieces;  // tile j's pieces [lo, hi) (global key indices) at pieces[j * PS ..], one per chunk
    uint32_t PS;          // piece-table stride: the most chunks of a bucket
    int SS;
    const void *spl;  // the splitters (Spl<T>, SS per bucket): equal neighbours = a duplicate run
    const void *bspl; // the first level's splitters (bk::Comp<T>::C, B - 1): a bucket's key bounds
    int B;
    uint32_t tcap;    // tiles the tile and piece tables hold (>= 1): a tile's reads may go out before its
                      // index is checked against the count on the device
};

// LOCAL: the chunk histograms are the prefix tables of sb_local_kernel (pref[c][j+1] -
// pref[c][j]); tiles are GTiles and a tile has no alignment constraint (room = tile); a sub-bucket
// above a tile is cut by chunks into several tiles (split_tiles) and recorded in ovf: the host
// merges those tiles' outputs after the tile sort (rare: a sampling outlier).
// SCATTER: counts[c][j]; the per-chunk offsets of the scatter are written too; tiles are
// TileRefs.
// LOCAL: a tile's room is tile - cpad * (the bucket's chunks): the gathering tile sort reads every
// piece as the 16-byte vectors covering it, up to cpad extra slots per piece (gather_tile).
// LOCAL: every tile's piece table (PS entries per tile, tiles below tcap) -- here when `pieces` is
// given (many buckets: the workgroups fill the chip), else by sb_pieces_kernel afterwards (few large
// buckets, e.g. 128 of 4M keys: a workgroup per bucket would walk ~280 tiles of ~280 pieces); the
// gathering tile sort reads it together with the tile record, one round trip before its key loads
// instead of two.  Tile records past trec (the record array's size) are not written: the host sees
// *ntiles > trec and takes the scatter path.
//
// Split of sub-bucket j (LOCAL, above a tile): greedy over the bucket's chunks, a tile taking
// consecutive chunks' pieces while its keys plus cpad per piece fit `full`.  A piece larger than a
// tile's room (a chunk holds more keys than an int32 tile: 15360 vs 8192) is cut: the tiles that
// start inside it take `full - cpad` keys of it each.  Calls f(ca, aoff, cb, valid) per tile in
// order -- chunks [ca, cb), the first one's piece from offset aoff (GTile.flags >> 8); a one-chunk
// tile takes `valid` keys from there -- and returns the tile count.
template <typename F>
__device__ __forceinline__ uint32_t split_tiles(const uint32_t *counts, int SS, uint32_t c0, uint32_t c1, int j,
                                                uint32_t full, uint32_t cpad, F &&f) {
    uint32_t nt = 0, ca = c0, aoff = 0, v = 0, np = 0;
    for (uint32_t c = c0; c < c1; ++c) {
        const uint32_t *pc = counts + (uint64_t)c * (SS + 1);
        const uint32_t piece = pc[j + 1] - pc[j];
        uint32_t off = 0;
        while (off < piece) {
            const uint32_t r = piece - off, used = v + cpad * (np + 1);
            const uint32_t cap = full > used ? full - used : 0;
            if (r <= cap) {  // the rest of the piece fits the open tile
                v += r;
                ++np;
                break;
            }
            if (np == 0) {  // an empty tile: a cut of this piece alone
                f(c, off, c + 1, cap);
                ++nt;
                off += cap;
                ca = c;
                aoff = off;
                continue;
            }
            f(ca, aoff, c, v);  // the open tile ends before this chunk
            ++nt;
            ca = c;
            aoff = off;
            v = 0;
            np = 0;
        }
        if (piece == 0 && np == 0 && v == 0) {  // (an empty piece at the open tile's start)
            ca = c + 1;
            aoff = 0;
        }
    }
    if (np) {
        f(ca, aoff, c1, v);
        ++nt;
    }
    return nt;
}
// The piece of a gathered tile in chunk c (global key indices): [pref[c][j0], pref[c][j1]) of the
// chunk, from offset flags >> 8 in the tile's first chunk; a one-chunk tile takes `valid` keys.
__device__ __forceinline__ uint2 tile_piece(const uint32_t *counts, int SS, uint32_t base, uint32_t c, uint32_t c0,
                                            uint32_t nch, uint32_t j0, uint32_t j1, uint32_t valid, uint32_t flags) {
    const uint32_t *pc = counts + (uint64_t)c * (SS + 1);
    const uint32_t lo = base + pc[j0] + (c == c0 ? flags >> 8 : 0u);
    return make_uint2(lo, nch == 1 ? lo + valid : base + pc[j1]);
}

#ifdef DSORT_STAMPS
// Diagnostic build only: per-workgroup phase cycles of sb_local_kernel (or, with DSORT_SCAN_STAMPS,
// of sb_scan_kernel<true> in rows 0..B-1), read back by dsort_debug_sbstamps().
__device__ unsigned long long g_sbstamps[(1u << 18) * 8];
#endif
template <bool LOCAL>
__global__ void __launch_bounds__(SB_MAXS, 8) sb_scan_kernel(const BInfo *__restrict__ bi, int SS,
                                                          const uint32_t *__restrict__ counts,
                                                          uint32_t *__restrict__ offs, int tile, int align,
                                                          uint32_t mis, uint32_t cpad, void *__restrict__ tiles,
                                                          uint32_t *__restrict__ ntiles, Ovf *__restrict__ ovf,
                                                          uint32_t *__restrict__ novf, uint32_t trec,
                                                          const Chunk *__restrict__ ch, uint2 *__restrict__ pieces,
                                                          uint32_t PS, uint32_t tcap, const uint32_t *__restrict__ stot) {
    __shared__ uint32_t wsum[SB_MAXS / 64];
    __shared__ uint32_t ss[SB_MAXS + 1];   // sub-bucket starts (positions)
    __shared__ uint16_t nxt[SB_MAXS];      // first sub-bucket after the tile starting at i
    __shared__ uint16_t chain[SB_MAXS];    // sub-buckets that start a tile
    __shared__ uint16_t tix[SB_MAXS];      // LOCAL: tile of chain entry i, relative to tbase (0xFFFF: none)
    __shared__ uint32_t nchain, tbase;
#ifdef DSORT_SCAN_STAMPS
    uint64_t sc_acc[8] = {}, sc_t0 = __builtin_amdgcn_s_memtime();
#define SCST(k)                                            \
    do {                                                   \
        const uint64_t t1_ = __builtin_amdgcn_s_memtime(); \
        sc_acc[k] += t1_ - sc_t0;                          \
        sc_t0 = t1_;                                       \
    } while (0)
#else
#define SCST(k) \
    do {        \
    } while (0)
#endif
    const BInfo b = bi[blockIdx.x];
    const int j = threadIdx.x;
    const int ns = (int)b.nsub;
    const int full = tile;  // LOCAL: a lone sub-bucket above the padded room still makes a tile up to
                            // `full` keys, gathered key by key (GTile.flags bit 0)
    if (LOCAL) tile -= (int)(cpad * (b.c1 - b.c0));
    auto cnt = [&](uint32_t c) -> uint32_t {
        if constexpr (LOCAL) {
            const uint32_t *pc = counts + (uint64_t)c * (SS + 1);
            return pc[j + 1] - pc[j];
        } else {
            return counts[(uint64_t)c * SS + j];
        }
    };
    uint32_t tot = 0;
    if (LOCAL && stot) {  // (the totals sb_local_kernel added up)
        if (j < ns) tot = stot[(uint64_t)blockIdx.x * SS + j];
    } else if constexpr (LOCAL) {
        // sub-bucket j's total = A_j - A_{j-1}, A_j = the sum over the chunks of pref[c][j + 1]
        // (pref[c][0] = 0): one load per chunk instead of two
        uint32_t a = 0;
        if (j < ns) {
#ifndef DSORT_SCAN_SUM_U
#define DSORT_SCAN_SUM_U 16
#endif
#pragma unroll DSORT_SCAN_SUM_U  // (independent loads in flight: the loop is latency-bound)
            for (uint32_t c = b.c0; c < b.c1; ++c) a += counts[(uint64_t)c * (SS + 1) + j + 1];
            ss[j + 1] = a;
        }
        __syncthreads();
        if (j < ns) tot = a - (j ? ss[j] : 0u);
    } else if (j < ns) {
#pragma unroll 8
        for (uint32_t c = b.c0; c < b.c1; ++c) tot += cnt(c);
    }
    uint32_t all;
    const uint32_t ex = scan_excl_1024(tot, wsum, all);
    SCST(0);
    const uint32_t st = (uint32_t)b.start + ex;
    if (j < ns) {
        if constexpr (!LOCAL) {
            uint32_t run = st;
            for (uint32_t c = b.c0; c < b.c1; ++c) {
                offs[(uint64_t)c * SS + j] = run;
                run += cnt(c);
            }
        }
        ss[j] = st;
    }
    if (j == 0) ss[ns] = (uint32_t)b.start + b.len;
    __syncthreads();
    SCST(1);
    if (j < ns) {
        const uint32_t p = ss[j];
        const uint32_t room = (uint32_t)tile - ((p + mis) & (uint32_t)(align - 1));
        // last e in (j, ns] with ss[e] - p <= room
        int lo = j + 1, hi = ns;  // answer in [j, ns]; ss[j] - p = 0 <= room
        int e = j;
        while (lo <= hi) {
            const int mid = (lo + hi) >> 1;
            if (ss[mid] - p <= room) {
                e = mid;
                lo = mid + 1;
            } else {
                hi = mid - 1;
            }
        }
        nxt[j] = (uint16_t)(e > j ? e : j + 1);  // e == j: sub-bucket j alone is too large
    }
    __syncthreads();
    SCST(2);
#ifndef DSORT_SCAN_CHAIN_WAVE
#define DSORT_SCAN_CHAIN_WAVE 1
#endif
    if (DSORT_SCAN_CHAIN_WAVE && j < 64) {
        // the chain 0, nxt[0], nxt[nxt[0]], ... walked by wave 0 through a 64-entry window of nxt
        // held one entry per lane: a step is a lane read (readlane) instead of an LDS round trip
        // (one thread walking ~130 steps through LDS was a quarter of the kernel).  i, base, k and
        // the window's member mask m are wave-uniform.
        const int lane = j;
        int i = 0, base = 0;
        uint32_t k = 0;
        uint32_t v = lane < ns ? nxt[lane] : 0u;
        uint64_t m = 0;
        const auto flush = [&]() {
            if ((m >> lane) & 1ull) chain[k + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)(base + lane);
            k += (uint32_t)__popcll(m);
        };
        while (i < ns) {
            if (i >= base + 64) {
                flush();
                base = i & ~63;
                v = base + lane < ns ? nxt[base + lane] : 0u;
                m = 0;
            }
            m |= 1ull << (i - base);
            i = __builtin_amdgcn_readlane((int)v, i - base);
        }
        flush();
        if (lane == 0) nchain = k;
    }
    if (!DSORT_SCAN_CHAIN_WAVE && j == 0) {
        int k = 0;
        for (int i = 0; i < ns; i = nxt[i]) chain[k++] = (uint16_t)i;
        nchain = (uint32_t)k;
    }
    __syncthreads();
    SCST(3);
    const int nc = (int)nchain;
    uint32_t nt = 0, i0 = 0, i1 = 0, room = 0;
    bool over = false;
    if (j < nc) {
        i0 = chain[j];
        i1 = nxt[i0];
        const uint32_t p = ss[i0], len = ss[i1] - p;
        room = (uint32_t)tile - ((p + mis) & (uint32_t)(align - 1));
        over = len > (LOCAL ? (uint32_t)full : room);
        if (LOCAL && over)  // (i1 == i0 + 1: a lone sub-bucket) cut by chunks
            nt = split_tiles(counts, SS, b.c0, b.c1, (int)i0, (uint32_t)full, cpad,
                             [](uint32_t, uint32_t, uint32_t, uint32_t) {});
        else
            nt = len == 0 ? 0 : over ? 1 + (len - room + tile - 1) / tile : 1;
    }
    uint32_t tall;
    const uint32_t tex = scan_excl_1024(nt, wsum, tall);
    if (j == 0) tbase = tall ? atomicAdd(ntiles, tall) : 0;
    __syncthreads();
    SCST(4);
    if (LOCAL && j < nc) tix[j] = nt && !over ? (uint16_t)tex : (uint16_t)0xFFFF;
    if (j < nc && nt) {
        const uint32_t p = ss[i0], len = ss[i1] - p;
        uint32_t k = tbase + tex;
        if constexpr (LOCAL) {
            GTile *gt = static_cast<GTile *>(tiles);
            if (!over) {
                if (k < trec)
                    gt[k] = GTile{p, b.start, len, blockIdx.x, i0, i1, b.c0, b.c1 - b.c0, b.nsub, len > room ? 1u : 0u};
            } else {
                // the split tiles (this thread alone: a rare path); sb_pieces_kernel writes their
                // piece tables like any tile's
                uint32_t q = p;
                split_tiles(counts, SS, b.c0, b.c1, (int)i0, (uint32_t)full, cpad,
                            [&](uint32_t ca, uint32_t aoff, uint32_t cb, uint32_t v) {
                                if (k < trec)
                                    gt[k] = GTile{q, b.start, v, blockIdx.x, i0, i1, ca, cb - ca, b.nsub, aoff << 8};
                                for (uint32_t c = ca; pieces && c < cb && k < tcap; ++c)
                                    pieces[(uint64_t)k * PS + (c - ca)] =
                                        tile_piece(counts, SS, (uint32_t)ch[c].start, c, ca, cb - ca, i0, i1, v, aoff << 8);
                                q += v;
                                ++k;
                            });
                ovf[atomicAdd(novf, 1u)] = Ovf{p, len, tbase + tex, nt};
            }
        } else {
            bk::TileRef *tt = static_cast<bk::TileRef *>(tiles);
            if (!over) {
                tt[k] = bk::TileRef{p, len, 0};
            } else {
                tt[k++] = bk::TileRef{p, room, 0};
                for (uint32_t q = room; q < len; q += (uint32_t)tile)
                    tt[k++] = bk::TileRef{(uint64_t)p + q, len - q < (uint32_t)tile ? len - q : (uint32_t)tile, 0};
                ovf[atomicAdd(novf, 1u)] = Ovf{p, len, 0u, 0u};
            }
        }
    }
#ifndef DSORT_SCAN_PIECES
#define DSORT_SCAN_PIECES 1
#endif
    if (LOCAL && pieces && DSORT_SCAN_PIECES) {
        // The piece tables: entry (tile t, chunk c) = chunk c's start + pref[c][bnd[t]], + pref[c][bnd[t + 1]]
        // with bnd = the chain, then ns.  A group of chunks' prefix values at the tile bounds goes to
        // LDS first: the loads run along a chunk's prefix row and the table stores along a tile's
        // chunks, both coalesced.  (A wave per tile walking its chunks, or the (tile, chunk) entries
        // spread over the workgroup, loaded each chunk's row at two words per entry: a 64-byte line
        // per lane and load, 9100 entries per 2^20-key bucket -- the texture unit's line rate, 36 %
        // of the kernel, in both forms.)
        constexpr uint32_t PVW = 8192, PVC = 256, U = 8;
        __shared__ uint32_t pv[PVW];   // [chunk of the group][bound]
        __shared__ uint32_t pbs[PVC];  // the group's chunk starts
        const uint32_t nch = b.c1 - b.c0, nb = (uint32_t)nc + 1;
        uint32_t cg = PVW / nb;
        cg = cg < PVC ? cg : PVC;
        for (uint32_t g0 = 0; g0 < nch; g0 += cg) {
            const uint32_t gn = nch - g0 < cg ? nch - g0 : cg, items = gn * nb;
            __syncthreads();  // (tix; the previous group's reads of pv)
            for (uint32_t i0 = j; i0 < items; i0 += U * SB_MAXS) {
                uint32_t v[U];
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t i = i0 + u * SB_MAXS;
                    v[u] = 0;
                    if (i < items) {
                        const uint32_t c = i / nb, q = i - c * nb;
                        const uint32_t bnd = q < (uint32_t)nc ? (uint32_t)chain[q] : (uint32_t)ns;
                        v[u] = counts[(uint64_t)(b.c0 + g0 + c) * (SS + 1) + bnd];
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < U; ++u)
                    if (i0 + u * SB_MAXS < items) pv[i0 + u * SB_MAXS] = v[u];
            }
            for (uint32_t c = j; c < gn; c += SB_MAXS) pbs[c] = (uint32_t)ch[b.c0 + g0 + c].start;
            __syncthreads();
            for (uint32_t i = j; i < (uint32_t)nc * gn; i += SB_MAXS) {
                const uint32_t t = i / gn, c = i - t * gn;
                const uint32_t k = tbase + tix[t];
                if (tix[t] == 0xFFFF || k >= tcap) continue;  // (the host sees ntiles > tcap and fails the sort)
                const uint32_t bs = pbs[c];
                pieces[(uint64_t)k * PS + g0 + c] = make_uint2(bs + pv[c * nb + t], bs + pv[c * nb + t + 1]);
            }
        }
    }
    if (LOCAL && pieces && !DSORT_SCAN_PIECES) {
        __syncthreads();
        // the piece tables: a wave per tile, a lane per chunk (no division per entry)
        const uint32_t nch = b.c1 - b.c0, lane = threadIdx.x & 63;
        for (uint32_t t = threadIdx.x >> 6; t < (uint32_t)nc; t += blockDim.x >> 6) {
            if (tix[t] == 0xFFFF) continue;
            const uint32_t k = tbase + tix[t];
            if (k >= tcap) continue;  // (the host sees ntiles > tcap and fails the sort)
            const uint32_t a0 = chain[t], a1 = nxt[a0];
            for (uint32_t c = lane; c < nch; c += 64) {
                const uint32_t *pc = counts + (uint64_t)(b.c0 + c) * (SS + 1);
                const uint32_t base = (uint32_t)ch[b.c0 + c].start;
                pieces[(uint64_t)k * PS + c] = make_uint2(base + pc[a0], base + pc[a1]);
            }
        }
    }
    SCST(6);
#ifdef DSORT_SCAN_STAMPS
    if (threadIdx.x == 0 && LOCAL && blockIdx.x < (1u << 18))
        for (int k = 0; k < 8; ++k) g_sbstamps[blockIdx.x * 8 + k] = sc_acc[k];
#endif
#undef SCST
}

// The piece table of every gathered tile (LOCAL path): a wave per tile, a lane per chunk -- the
// tile's chunks [c0, c0 + nch), its sub-buckets [j0, j1): chunk c's piece is [pref[c][j0],
// pref[c][j1]) of the chunk.  (Inside sb_scan_kernel this was one workgroup per bucket walking all
// its tiles: 270 us for 128 buckets of 4M keys, where every tile has ~280 pieces.)
__global__ void __launch_bounds__(256) sb_pieces_kernel(const GTile *__restrict__ tiles,
                                                        const uint32_t *__restrict__ ntiles,
                                                        const Chunk *__restrict__ ch,
                                                        const uint32_t *__restrict__ counts, int SS,
                                                        uint2 *__restrict__ pieces, uint32_t PS, uint32_t tcap) {
    const uint32_t k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (k >= *ntiles || k >= tcap) return;  // (wave-uniform; the host fails a sort past tcap)
    const GTile t = tiles[k];
    for (uint32_t c = lane; c < t.nch; c += 64)
        pieces[(uint64_t)k * PS + c] = tile_piece(counts, SS, (uint32_t)ch[t.c0 + c].start, t.c0 + c, t.c0, t.nch, t.j0,
                                                  t.j1, t.valid, t.flags);
}

// Local partition (the default second level).  Chunk c (<= SB_LCH keys of one bucket) is loaded
// whole, partitioned by sub-bucket in LDS and written back in place with coalesced stores;
// pref[c][j] = keys of the chunk in sub-buckets below j (j = 0..nsub).  A tile (sub-buckets
// [j0, j1) of a bucket) is then one contiguous piece of every chunk of the bucket,
// [pref[c][j0], pref[c][j1]), gathered by the tile sort (about 1 KiB per piece) -- no
// element-granular scatter to HBM.
// Workgroup -> chunk: every XCD takes a contiguous block of chunks, i.e. of buckets, so the
// workgroups that write pieces of the same sub-buckets share an L2 (a bijection on [0, G)).
__device__ __forceinline__ uint32_t sb_chunk_order(uint32_t bid, uint32_t G) {
    constexpr uint32_t NX = 8;
    const uint32_t q = G / NX, r = G % NX, x = bid % NX, i = bid / NX;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// int32: 1024 threads of 15 keys, 8 waves per SIMD at two workgroups per CU: twice the waves of
// round 2's 512 threads of 31 keys to hide the lookups' LDS round trips (2.33 -> 2.02 ms at 2^30).
// int64 (round 6): 1024 threads of 6 keys, lookups in pairs (DSORT_SB_G64) -- round 5 measured this
// geometry with 8-key batches, which spilled 22 VGPRs at 8 waves per SIMD (C4 +0.9 ms,
// profiles/r5_ab_c4_local_1024x6.log); in pairs nothing spills, and since the first level's one-key
// hash (dsort_bucket.h bucket_onekey) C4's buckets hold hardly any duplicate run: C4 second level
// 2.21 -> 1.82 ms, uniform int64 3.78 -> 3.48 ms (profiles/r6_ab_local_partition_i64_1024x6.log;
// 512 x 13 with 8-key batches before)
#ifndef DSORT_SB_LT32
#define DSORT_SB_LT32 1024
#endif
#ifndef DSORT_SB_KPT32
#define DSORT_SB_KPT32 15
#endif
#ifndef DSORT_SB_G32
#define DSORT_SB_G32 1  // int32 keys per batch of the classify (G below)
#endif
#ifndef DSORT_SB_LT64
#define DSORT_SB_LT64 1024
#endif
#ifndef DSORT_SB_KPT64
#define DSORT_SB_KPT64 6
#endif
template <typename T> constexpr int SB_LT = sizeof(T) == 4 ? DSORT_SB_LT32 : DSORT_SB_LT64;
// keys per thread: the chunk (int32 60 KiB, int64 48 KiB) + tables fit two workgroups per CU
template <typename T> constexpr int SB_LKPT = sizeof(T) == 4 ? DSORT_SB_KPT32 : DSORT_SB_KPT64;

template <typename T> constexpr int SB_LCH = SB_LT<T> * SB_LKPT<T>;

template <typename T>
__global__ void __launch_bounds__(SB_LT<T>, SB_LT<T> / 128) sb_local_kernel(T *__restrict__ buf, const Chunk *__restrict__ ch,
                                                         const BInfo *__restrict__ bi, int SS,
                                                         const Spl<T> *__restrict__ spl_g,
                                                         const uint32_t *__restrict__ rng_g,
                                                         const SlotFn<T> *__restrict__ sfn,
                                                         uint32_t *__restrict__ pref, const uint32_t *__restrict__ hotp,
                                                         uint32_t *__restrict__ stot) {
    constexpr int LT = SB_LT<T>, KPT = SB_LKPT<T>, CHL = SB_LCH<T>, PER = SB_MAXS / LT;
    static_assert(SB_MAXS % LT == 0, "sub-buckets per thread");
    __shared__ Spl<T> spl[SB_MAXS + 1];
    __shared__ uint32_t rng[SB_SLOTS];
    __shared__ uint32_t hist[SB_MAXS];   // chunk histogram, then the LDS starts
    __shared__ uint32_t wsum[LT / 64];
    __shared__ T lk[CHL];
#ifdef DSORT_STAMPS
    uint64_t st_acc[6] = {}, st_t0 = __builtin_amdgcn_s_memtime();
#define SBST(k)                                            \
    do {                                                   \
        const uint64_t t1_ = __builtin_amdgcn_s_memtime(); \
        st_acc[k] = t1_ - st_t0;                           \
        st_t0 = t1_;                                       \
    } while (0)
#else
#define SBST(k) \
    do {        \
    } while (0)
#endif
    // (every XCD takes a contiguous block of chunks, i.e. of buckets: a bucket's tables and the
    // lines its neighbouring chunks share stay in one L2; measured neutral to -0.05 ms)
    const uint32_t cid = sb_chunk_order(blockIdx.x, gridDim.x);
    const Chunk c = ch[cid];
    const BInfo b = bi[c.b];
    uint32_t *pc = pref + (uint64_t)cid * (SS + 1);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int ns = (int)b.nsub;
    if (ns == 1) {
        if (tid == 0) {
            pc[0] = 0;
            pc[1] = c.len;
            if (stot) atomicAdd(&stot[(uint64_t)c.b * SS], c.len);
        }
        return;
    }
    // (Slots shifted to the 128-byte line below the chunk start, so that every wave's loads and
    // stores cover whole lines, measured 2.00 -> 2.10 ms: the PMC traffic of this kernel is 1.23x
    // its algorithmic bytes, but the split lines are not what bounds it.)
    const uint32_t m = 0;
    T *src = buf + c.start;
    T key[KPT];
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
        const uint32_t s = tid + k * LT;
        key[k] = s - m < c.len ? src[s] : T(0);  // (s < m wraps)
    }
    load_sub_tables<T>(b, c.b, SS, spl_g, rng_g, spl, rng);
#pragma unroll
    for (int q = 0; q < PER; ++q) hist[PER * tid + q] = 0;
    const SlotFn<T> f = sfn[c.b];
    // sorted or reversed input (the first level's bk::BkMap.hot): a wave's consecutive keys share
    // a sub-bucket, counted with one atomic (bk::bucket_bump); 2^30 sorted int32 sub level 4.3 -> 2.1 ms
    const bool hotf = hotp != nullptr && *hotp != 0;
    __syncthreads();
    SBST(0);
    uint32_t pk[KPT];  // sub-bucket | rank << 10
    // In groups of G keys: the slot-table reads, then the splitter reads, then the atomics, so a
    // key's LDS round trips do not wait for the previous key's.  A key past the chunk adds 0.
    // (int32: 31 keys and their ranks are already live; batching spills and measured slower)
#ifndef DSORT_SB_G64
#define DSORT_SB_G64 2
#endif
    constexpr int G = sizeof(T) == 4 ? DSORT_SB_G32 : DSORT_SB_G64;
    // a whole chunk: only the first and last slot rows can fall outside it
    const bool whole = c.len == (uint32_t)CHL;
    if constexpr (G == 1) {
        if (hotf) {
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint32_t s = tid + k * LT;
                const bool act = s - m < c.len;
                const int j = act ? sub_of<T>(spl, rng, f.klo, f.sh, key[k], (uint32_t)(c.start + s - m)) : 0;
                pk[k] = (uint32_t)j | bk::bucket_bump<true>(hist, j, act) << 10;
            }
        } else if (whole) {  // (no per-key branch in the middle rows)
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint32_t s = tid + k * LT;
                if ((k > 0 && k + 1 < KPT) || s - m < c.len) {  // (rows 1..KPT-2 lie inside)
                    const int j = sub_of<T>(spl, rng, f.klo, f.sh, key[k], (uint32_t)(c.start + s - m));
                    pk[k] = (uint32_t)j | atomicAdd(&hist[j], 1u) << 10;
                }
            }
        } else
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            const uint32_t s = tid + k * LT;
            if (s - m < c.len) {
                const int j = sub_of<T>(spl, rng, f.klo, f.sh, key[k], (uint32_t)(c.start + s - m));
                pk[k] = (uint32_t)j | atomicAdd(&hist[j], 1u) << 10;
            }
        }
    } else {
#pragma unroll
    for (int g0 = 0; g0 < KPT; g0 += G) {
        uint32_t r[G];
        Spl<T> sa[G], sb[G];
#pragma unroll
        for (int u = 0; u < G; ++u)
            if (g0 + u < KPT) r[u] = rng[slot_of<T>(key[g0 + u], f.klo, f.sh)];
#pragma unroll
        for (int u = 0; u < G; ++u)
            if (g0 + u < KPT) {
                const uint32_t lo = r[u] & 0x7FFF, hi = r[u] >> 16;
                sa[u] = Spl<T>{};
                sb[u] = Spl<T>{};
                if (lo < hi) sa[u] = spl[lo];
                if (lo + 1 < hi) sb[u] = spl[lo + 1];
            }
#pragma unroll
        for (int u = 0; u < G; ++u)
            if (g0 + u < KPT) {
                const uint32_t s = tid + (g0 + u) * LT, i = s - m;
                const int j = sub_pick<T>(spl, r[u], sa[u], sb[u], key[g0 + u], (uint32_t)(c.start + i));
                // (a key past the chunk adds 0 to a lane-spread counter, not all to one)
                if (hotf) pk[g0 + u] = (uint32_t)j | bk::bucket_bump<true>(hist, j, i < c.len) << 10;
                else pk[g0 + u] = (uint32_t)j | atomicAdd(&hist[i < c.len ? j : lane], i < c.len ? 1u : 0u) << 10;
            }
    }
    }
    __syncthreads();
    SBST(1);
    uint32_t h[PER], sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        h[q] = hist[PER * tid + q];
        sum += h[q];
    }
    uint32_t incl = wave_incl_sum(sum);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    SBST(2);
    uint32_t ex = incl - sum;
#pragma unroll
    for (int i = 0; i < LT / 64; ++i) ex += i < w ? wsum[i] : 0u;
    if (tid == 0) pc[ns] = c.len;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int j = PER * tid + q;
        hist[j] = ex;
        if (j < ns) pc[j] = ex;
        // the bucket's sub-bucket totals for sb_scan_kernel (summing every chunk's prefix row
        // there read the whole table again: 190 MB at 2^30 int32, 60 % of that kernel)
        if (stot && j < ns && h[q]) atomicAdd(&stot[(uint64_t)c.b * SS + j], h[q]);
        ex += h[q];
    }
    __syncthreads();
    SBST(3);
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
        const uint32_t s = tid + k * LT;
        if (s - m < c.len) lk[hist[pk[k] & 1023] + (pk[k] >> 10)] = key[k];
    }
    __syncthreads();
    SBST(4);
    // write-back in wave blocks aligned to 64 keys of the buffer: every wave store covers whole
    // lines.  (At the chunk's own offsets a store straddled a line at each end; the L2 filled such
    // lines from HBM before merging the halves: the kernel moved 10.5 GB for 8.6 GB of keys, now
    // 8.75 GB, 2.00 -> 1.92 ms at 2^30 int32.)
    {
        const uint32_t mw = (uint32_t)((reinterpret_cast<uintptr_t>(src) / sizeof(T)) & 63u);
#pragma unroll
        for (int k = 0; k <= KPT; ++k) {
            const uint32_t s = tid + k * LT - mw;  // (wraps below 0)
            if (s < c.len) src[s] = lk[s];
        }
    }
#ifdef DSORT_STAMPS
    SBST(5);
    if (tid == 0 && blockIdx.x < (1u << 18))
        for (int k = 0; k < 6; ++k) g_sbstamps[blockIdx.x * 8 + k] = st_acc[k];
#endif
#undef SBST
}


// Per sub-tile (SB_SUB keys): sub-bucket and slot of every key (LDS atomic), scan, keys grouped
// by sub-bucket in LDS, then consecutive threads write consecutive keys of a sub-bucket to
// consecutive addresses.  Thread t owns sub-buckets 4t .. 4t+3 (their running global offsets).
template <typename T>
__global__ void __launch_bounds__(SB_T) sb_scatter_kernel(const T *__restrict__ src, T *__restrict__ dst,
                                                          const Chunk *__restrict__ ch, uint32_t G,
                                                          const BInfo *__restrict__ bi, int SS,
                                                          const Spl<T> *__restrict__ spl_g,
                                                          const uint32_t *__restrict__ rng_g,
                                                          const SlotFn<T> *__restrict__ sfn,
                                                          const uint32_t *__restrict__ offs) {
    constexpr int KPT = SB_KPT<T>, SUB = SB_SUB<T>;
    static_assert(SB_MAXS == 4 * SB_T, "4 sub-buckets per thread");
    __shared__ Spl<T> spl[SB_MAXS + 1];  // + 1: sub_of reads two entries
    __shared__ uint32_t rng[SB_SLOTS];
    __shared__ uint32_t hist[SB_MAXS];   // sub-tile histogram, then the sub-tile's LDS starts
    __shared__ uint32_t dl[SB_MAXS];     // global offset - LDS start, per sub-bucket
    __shared__ uint32_t wsum[SB_T / 64];
    __shared__ T lk[SUB];
    __shared__ uint16_t lj[SUB];
    const uint32_t cid = sb_chunk_order(blockIdx.x, G);
    const Chunk c = chunk_of<T>(ch, bi, cid);
    const BInfo b = bi[c.b];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (b.nsub == 1) {  // one sub-bucket: a plain copy
        const uint32_t o = offs[(uint64_t)cid * SS];
        for (uint32_t i = tid; i < c.len; i += SB_T) dst[o + i] = src[c.start + i];
        return;
    }
    load_sub_tables<T>(b, c.b, SS, spl_g, rng_g, spl, rng);
    const SlotFn<T> f = sfn[c.b];
    const int ns = (int)b.nsub;
    uint32_t gof[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int j = 4 * tid + q;
        gof[q] = j < ns ? offs[(uint64_t)cid * SS + j] : 0u;
        hist[j] = 0;
    }
#pragma unroll 1
    for (uint32_t s0 = 0; s0 < c.len; s0 += SUB) {
        const uint32_t cnt = c.len - s0 < (uint32_t)SUB ? c.len - s0 : (uint32_t)SUB;
        T key[KPT];
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            const uint32_t i = tid + k * SB_T;
            key[k] = i < cnt ? src[c.start + s0 + i] : T(0);
        }
        __syncthreads();  // tables loaded / previous sub-tile written and its histogram cleared
        int jj[KPT];
        uint32_t slot[KPT];
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            const uint32_t i = tid + k * SB_T;
            jj[k] = -1;
            if (i < cnt) {
                jj[k] = sub_of<T>(spl, rng, f.klo, f.sh, key[k], (uint32_t)(c.start + s0 + i));
                slot[k] = atomicAdd(&hist[jj[k]], 1u);
            }
        }
        __syncthreads();
        uint32_t h[4], sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            h[q] = hist[4 * tid + q];
            sum += h[q];
        }
        uint32_t incl = wave_incl_sum(sum);
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t ex = incl - sum;
#pragma unroll
        for (int i = 0; i < SB_T / 64; ++i) ex += i < w ? wsum[i] : 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            hist[4 * tid + q] = ex;
            dl[4 * tid + q] = gof[q] - ex;
            gof[q] += h[q];
            ex += h[q];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            if (jj[k] >= 0) {
                const uint32_t lp = hist[jj[k]] + slot[k];
                lk[lp] = key[k];
                lj[lp] = (uint16_t)jj[k];
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            const uint32_t p = tid + k * SB_T;
            if (p < cnt) dst[dl[lj[p]] + p] = lk[p];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) hist[4 * tid + q] = 0;
    }
}

}  // namespace sb
}  // namespace dsort
