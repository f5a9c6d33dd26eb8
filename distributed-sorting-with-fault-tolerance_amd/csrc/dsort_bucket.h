// dsort_bucket.h -- the sample-splitter partition pass in front of the sorts (namespace
// dsort::bk; included by dsort_wave.hip for int32 and dsort_sort.hip for int64, whose drivers run
// their own tile sort and k-way passes inside the buckets).
//
// The multi-GPU design cuts the keys into key ranges with sample-sort splitters and sorts every
// range on its own GPU.  The same idea inside one GPU's HBM: B buckets (about
// 2^21 keys each) by splitters taken from a regular sample, in (key, input index) order so that
// duplicates are spread over buckets like any other key; one partition pass writes every bucket
// contiguously; then the tile sort and the k-way merge passes run inside every bucket.  A
// partition pass resolves log2(B) bits of the order in about one read + one write of the keys
// (plus a read for the histogram), where a merge pass resolves log2(F) = 4: at 2^30 keys the
// 16 bits of merging above the 16384-key tiles become 9 bits of partition + 7 bits of merging,
// 2 merge passes instead of 4.
//
// Kernels (all keyed by the composite c = key * 2^32 + input index, unique per key):
//   bucket_sample_kernel   s regular samples -> composites (sorted by the int64 sort)
//   bucket_splitter_kernel splitter b = sample (b+1)*s/B - 1; padded with +inf to BP
//   bucket_hist_kernel     per 65536-key workgroup: keys per bucket (LDS atomics)
//   bucket_colsum_kernel   per 64 workgroups: column sums        } exclusive scan of the
//   bucket_scan_kernel     one workgroup: chunk prefixes, bucket   } histograms in (bucket,
//                          starts, tile table of the tile sort     }  workgroup) order
//   bucket_offsets_kernel  per-workgroup bucket offsets          }
//   bucket_scatter_kernel  per 16384-key sub-tile: keys grouped by bucket in LDS, then written
//                          to their buckets (consecutive lanes on consecutive keys of a bucket)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsort {
namespace bk {

constexpr int BK_T = 1024;               // threads of the partition kernels
constexpr int BK_MAXB = 1024;            // buckets at most (<= threads, one bucket per thread)
constexpr int BK_OS = 32;                // samples per bucket
constexpr int BK_CHUNK = 64;             // workgroups per column-sum chunk

// Scatter sub-tile per key width: KPT keys per thread, SUB = BK_T * KPT keys staged in LDS
// (int32: 56 KiB next to the 64 KiB line carry of the line scatter; 12 and 13 measured slower).
template <typename T> struct Geo;
template <> struct Geo<int32_t> { static constexpr int KPT = 14; };
template <> struct Geo<int64_t> { static constexpr int KPT = 8; };

struct TileRef {
    uint64_t base;   // first key of the tile
    uint32_t valid;  // keys in the tile (<= the tile size)
    uint32_t pad;
};

// The composite order (key, input index): unique per key, so duplicates spread over buckets.
// int32: packed in one int64 (key * 2^32 + index); int64: a (key, index) pair.
struct Pair {
    int64_t k;
    uint32_t i, pad;
};
template <typename T> struct Comp;
template <> struct Comp<int32_t> {
    using C = int64_t;
    __host__ __device__ static C make(int32_t key, uint64_t idx) {
        return (int64_t)((uint64_t)(int64_t)key << 32 | (uint32_t)idx);
    }
    __host__ __device__ static bool lt(C a, C b) { return a < b; }
    __host__ __device__ static C inf() { return INT64_MAX; }
    // composite (key of the slot start, index 0) of sign-flipped key prefix `u`
    __host__ __device__ static C slot_start(uint64_t ubias) {
        return (int64_t)(((uint64_t)((uint32_t)ubias ^ 0x80000000u)) << 32);
    }
    __host__ __device__ static uint32_t slot_of(int32_t key, int bits) {
        return ((uint32_t)key ^ 0x80000000u) >> (32 - bits);
    }
    __host__ __device__ static int32_t key_of(C c) { return (int32_t)(c >> 32); }
    __host__ __device__ static uint32_t idx_of(C c) { return (uint32_t)c; }
    using U = uint32_t;
    __host__ __device__ static U flip(int32_t key) { return (uint32_t)key ^ 0x80000000u; }
    static constexpr int KB = 32;  // key bits
    static constexpr bool ADAPT = false;  // fixed top-bit slots, no one-key slots (see BkMap)
};
template <> struct Comp<int64_t> {
    using C = Pair;
    __host__ __device__ static C make(int64_t key, uint64_t idx) { return Pair{key, (uint32_t)idx, 0}; }
    __host__ __device__ static bool lt(const C &a, const C &b) {
        return a.k < b.k || (a.k == b.k && a.i < b.i);
    }
    __host__ __device__ static C inf() { return Pair{INT64_MAX, 0xFFFFFFFFu, 0}; }
    __host__ __device__ static C slot_start(uint64_t ubias) {
        return Pair{(int64_t)(ubias ^ 0x8000000000000000ull), 0, 0};
    }
    __host__ __device__ static uint32_t slot_of(int64_t key, int bits) {
        return (uint32_t)(((uint64_t)key ^ 0x8000000000000000ull) >> (64 - bits));
    }
    __host__ __device__ static int64_t key_of(const C &c) { return c.k; }
    __host__ __device__ static uint32_t idx_of(const C &c) { return c.i; }
    using U = uint64_t;
    __host__ __device__ static U flip(int64_t key) { return (uint64_t)key ^ 0x8000000000000000ull; }
    static constexpr int KB = 64;
    static constexpr bool ADAPT = true;
};

// bucket of composite c: the number of splitters below c (spl holds BP entries, +inf padded)
template <typename T>
__device__ __forceinline__ int bucket_of(const typename Comp<T>::C *spl, int BP,
                                         const typename Comp<T>::C &c) {
    int lo = 0;
    for (int st = BP >> 1; st >= 1; st >>= 1) lo += Comp<T>::lt(spl[lo + st - 1], c) ? st : 0;
    return lo;
}

// Radix-assisted lookup: rng[slot(key)] packs the number of splitters whose key lies below the
// slot (bits 0-14), a "one-key slot" flag (bit 15) and the number below the next slot (bits
// 16-31).  Only splitters inside the key's slot need a comparison -- usually none or one --
// instead of a log2(B)-step search with bank conflicts on every step.
//
// The slot of a key is a monotone function of its sign-flipped value u above the first
// splitter's, d = max(u - ulo, 0) (BkMap, chosen once per sort by bucket_slotmap_kernel):
//   linear (mode 0): d >> sh, sh the smallest shift that maps the last splitter into the table:
//                    uniform keys put ~B/SLOTS splitters in every slot;
//   log    (mode 1): d itself below 2^M, else (bit length, the M bits after the leading one):
//                    skewed keys (Zipf's small heavy integers) get a slot per heavy key and the
//                    sparse tail shares wide slots.  Under the linear map they all fall in one
//                    slot and every key binary-searches hundreds of splitters.
// int32 keeps the fixed map (the top SLOTB bits, ulo = 0) and no one-key slots: its histogram
// runs at the HBM rate and the extra lookup work measured +0.5 ms there at 2^30 uniform keys.
constexpr int BK_SLOTB = 11;
constexpr int BK_SLOTS = 1 << BK_SLOTB;

struct BkMap {
    uint64_t ulo;   // flipped key of the first splitter
    uint32_t sh;    // linear shift
    uint32_t mode;  // 0 linear, 1 log
    uint64_t invn;  // 2^48 / n: index -> 16-bit fraction of the input
};
// log mode: mantissa bits M, the largest with (KB - M + 1) * 2^M slots in the table
template <typename T, int SB>
__host__ __device__ constexpr int log_m() {
    int m = 0;
    while (m < 16 && (Comp<T>::KB - (m + 1) + 1) * (1 << (m + 1)) <= (1 << SB)) ++m;
    return m;
}

template <typename T, int SB, int MODE>
__host__ __device__ __forceinline__ uint32_t slot_mode(const BkMap &m, T key) {
    using U = typename Comp<T>::U;
    constexpr uint32_t NS = 1u << SB;
    constexpr int M = log_m<T, SB>();
    if (!Comp<T>::ADAPT) return Comp<T>::slot_of(key, SB);
    const U u = Comp<T>::flip(key);
    const U d = u < (U)m.ulo ? (U)0 : (U)(u - (U)m.ulo);
    if (MODE == 0) {
        const U q = d >> m.sh;
        return q > (U)(NS - 1) ? NS - 1 : (uint32_t)q;
    }
    if (d < ((U)1 << M)) return (uint32_t)d;
    const int e = (int)(sizeof(U) * 8) - (sizeof(U) == 8 ? __builtin_clzll((uint64_t)d) : __builtin_clz((uint32_t)d));
    return (uint32_t)(e - M) << M | ((uint32_t)(d >> (e - 1 - M)) & ((1u << M) - 1));
}
template <typename T, int SB = BK_SLOTB>
__host__ __device__ __forceinline__ uint32_t slot_at(const BkMap &m, T key) {
    return m.mode == 0 ? slot_mode<T, SB, 0>(m, key) : slot_mode<T, SB, 1>(m, key);
}
// the slots of K keys, the (workgroup-uniform) mode branch taken once
template <typename T, int K>
__device__ __forceinline__ void slots_at(const BkMap &m, const T (&key)[K], uint32_t (&sl)[K]) {
    if (!Comp<T>::ADAPT || m.mode == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) sl[k] = slot_mode<T, BK_SLOTB, 0>(m, key[k]);
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) sl[k] = slot_mode<T, BK_SLOTB, 1>(m, key[k]);
    }
}

// the smallest flipped key of slot i (i >= 1), or false when no key maps there or beyond
template <typename T, int SB = BK_SLOTB>
__host__ __device__ __forceinline__ bool slot_first(const BkMap &m, uint32_t i, uint64_t &u0) {
    using U = typename Comp<T>::U;
    constexpr int M = log_m<T, SB>();
    constexpr int KB = Comp<T>::KB;
    U d;
    if (m.mode == 0) {
        if (m.sh + SB > KB && (i >> (KB - m.sh)) != 0) return false;
        d = (U)i << m.sh;
    } else if (i < (1u << M)) {
        d = (U)i;
    } else {
        const int e = (int)(i >> M) + M;
        if (e > KB) return false;
        d = (U)((1u << M) | (i & ((1u << M) - 1))) << (e - 1 - M);
    }
    const U umax = (U)~(U)0;
    if (d > (U)(umax - (U)m.ulo)) return false;
    u0 = (uint64_t)(U)((U)m.ulo + d);
    return true;
}

template <typename T, int SB = BK_SLOTB>
__device__ __forceinline__ void build_slots(const typename Comp<T>::C *spl, int BP, const BkMap &m,
                                            uint32_t *rng) {
    using CT = Comp<T>;
    constexpr int NS = 1 << SB;
    for (int i = threadIdx.x; i < NS; i += blockDim.x) {
        uint32_t cnt[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            // splitters whose key lies below the start of slot i + e (slot 0 starts at -inf)
            uint64_t u0 = 0;
            if (i + e == 0) {
                cnt[e] = 0;
            } else {
                const typename CT::C c = i + e < NS && slot_first<T, SB>(m, (uint32_t)(i + e), u0)
                                             ? CT::slot_start(u0) : CT::inf();
                cnt[e] = (uint32_t)bucket_of<T>(spl, BP, c);
            }
        }
        // a slot whose (>= 2) splitters all hold one key K: see bucket_fast
        const bool one = CT::ADAPT && cnt[1] >= cnt[0] + 2 && CT::key_of(spl[cnt[0]]) == CT::key_of(spl[cnt[1] - 1]);
        rng[i] = cnt[0] | (uint32_t)one << 15 | (cnt[1] << 16);
    }
}

// Bucket of (key, index).  In a one-key slot the copies of K may go to any bucket from the
// first of K's splitters to the one after the last (every one of those buckets holds keys <= K
// before it and >= K after it, and the buckets strictly inside hold only K).  The two outer
// buckets take exactly the copies the composite order gives them (index <= the first run
// splitter's, > the last one's), so they stay as full as a sample bucket should; the copies in
// between are split over the inner buckets by index range, in proportion -- two splitter reads
// and a division instead of a search over K's run (and a sub-tile's copies, adjacent in the
// input, land together in one or two buckets).
// Histogram and scatter use the same map and table, so they agree key for key.  (Which copy of
// K lands where does not matter to a keys-only sort.)
template <typename T>
__device__ __forceinline__ int bucket_fast(const typename Comp<T>::C *spl, const uint32_t *rng, uint32_t slot,
                                           T key, const typename Comp<T>::C &c) {
    const uint32_t r = rng[slot];
    int lo = (int)(r & 0x7FFF), hi = (int)(r >> 16);
    if (Comp<T>::ADAPT && (r & 0x8000)) {
        const typename Comp<T>::C a = spl[lo], z = spl[hi - 1];
        const T K = Comp<T>::key_of(a);
        const uint32_t i = Comp<T>::idx_of(c), ia = Comp<T>::idx_of(a), iz = Comp<T>::idx_of(z);
        if (key != K || i <= ia) return key <= K ? lo : hi;
        if (i > iz) return hi;
        // hi - lo - 1 inner buckets over the indices (ia, iz] (the hardware reciprocal: the same
        // instruction in the histogram and the scatter; IEEE division measured 0.25 ms slower)
        const float q = (float)(i - ia - 1) * ((float)(hi - lo - 1) * __builtin_amdgcn_rcpf((float)(iz - ia)));
        const int j = (int)q;
        return lo + 1 + (j < hi - lo - 2 ? j : hi - lo - 2);
    }
    while (lo < hi) {  // lower bound among the splitters of the slot
        const int mid = (lo + hi) >> 1;
        if (Comp<T>::lt(spl[mid], c)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// The slot map of a sort: linear unless the log map leaves fewer distinct splitter keys in its
// most crowded slot (one workgroup; out = BkMap).
template <typename T>
__global__ void __launch_bounds__(BK_MAXB) bucket_slotmap_kernel(const typename Comp<T>::C *__restrict__ spl,
                                                                  int B, uint64_t n, BkMap *__restrict__ out) {
    using CT = Comp<T>;
    using U = typename CT::U;
    __shared__ uint32_t cnt[2][BK_SLOTS];
    __shared__ uint32_t crowd[2];
    const int j = threadIdx.x, nsp = B - 1;
    for (int i = j; i < 2 * BK_SLOTS; i += blockDim.x) cnt[i / BK_SLOTS][i % BK_SLOTS] = 0;
    if (j < 2) crowd[j] = 0;
    const uint64_t invn = ((uint64_t)1 << 48) / (n > 0 ? n : 1);
    BkMap mm[2] = {{0, (uint32_t)(CT::KB - BK_SLOTB), 0, invn}, {0, 0, 1, invn}};
    if (!CT::ADAPT) {
        if (j == 0) *out = mm[0];
        return;
    }
    if (nsp >= 1) {
        const U lo = CT::flip(CT::key_of(spl[0])), hi = CT::flip(CT::key_of(spl[nsp - 1]));
        const U r = hi - lo;
        const int bits = r == 0 ? 0 : (int)(sizeof(U) * 8) - (sizeof(U) == 8 ? __builtin_clzll((uint64_t)r)
                                                                               : __builtin_clz((uint32_t)r));
        mm[0] = BkMap{(uint64_t)lo, (uint32_t)(bits > BK_SLOTB ? bits - BK_SLOTB : 0), 0, invn};
        mm[1] = BkMap{(uint64_t)lo, 0, 1, invn};
    }
    __syncthreads();
    // count the distinct splitter keys of every slot under both maps
    if (j < nsp && (j == 0 || CT::key_of(spl[j]) != CT::key_of(spl[j - 1]))) {
        const T k = CT::key_of(spl[j]);
        atomicAdd(&cnt[0][slot_at<T>(mm[0], k)], 1u);
        atomicAdd(&cnt[1][slot_at<T>(mm[1], k)], 1u);
    }
    __syncthreads();
    for (int i = j; i < 2 * BK_SLOTS; i += blockDim.x) atomicMax(&crowd[i / BK_SLOTS], cnt[i / BK_SLOTS][i % BK_SLOTS]);
    __syncthreads();
    if (j == 0) *out = crowd[1] < crowd[0] ? mm[1] : mm[0];
}

template <typename T>
__global__ void __launch_bounds__(256) bucket_sample_kernel(const T *__restrict__ in, uint64_t n,
                                                            typename Comp<T>::C *__restrict__ smp,
                                                            uint32_t s) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= s) return;
    const uint64_t pos = ((2 * (uint64_t)k + 1) * n) / (2 * (uint64_t)s);
    smp[k] = Comp<T>::make(in[pos], pos);
}

// splitter b = sample (b+1)*os - 1 of the sorted samples (os samples per bucket), b < B-1;
// +inf up to BP
template <typename T>
__global__ void __launch_bounds__(BK_MAXB) bucket_splitter_kernel(const typename Comp<T>::C *__restrict__ smp,
                                                                 int B, int BP, int os,
                                                                 typename Comp<T>::C *__restrict__ spl) {
    const int b = threadIdx.x;
    if (b < BP) spl[b] = b < B - 1 ? smp[(uint64_t)(b + 1) * os - 1] : Comp<T>::inf();
}

// int64 keys: the (key, index) pairs are sorted on the GPU in two int64 sorts -- the sampled keys
// (keys -> srt), then composites (index of the first equal key in srt) * 2^32 + sample index,
// whose order is the pair order -- and splitter b is the pair of composite (b+1)*os - 1.
__device__ __forceinline__ uint64_t sample_pos(uint64_t k, uint64_t n, uint32_t s) {
    return ((2 * k + 1) * n) / (2 * (uint64_t)s);
}
__global__ void __launch_bounds__(256) pair_sample_keys_kernel(const int64_t *__restrict__ in, uint64_t n,
                                                               int64_t *__restrict__ keys, uint32_t s) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k < s) keys[k] = in[sample_pos(k, n, s)];
}
__global__ void __launch_bounds__(256) pair_rank_kernel(const int64_t *__restrict__ keys,
                                                        const int64_t *__restrict__ srt, uint32_t s,
                                                        int64_t *__restrict__ cmp) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= s) return;
    const int64_t x = keys[k];
    uint32_t lo = 0, hi = s;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (srt[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    cmp[k] = (int64_t)((uint64_t)lo << 32 | k);
}
__global__ void __launch_bounds__(BK_MAXB) pair_splitter_kernel(const int64_t *__restrict__ cmp,
                                                                const int64_t *__restrict__ keys, uint64_t n,
                                                                uint32_t s, int B, int BP, int os,
                                                                Pair *__restrict__ spl) {
    const int b = threadIdx.x;
    if (b >= BP) return;
    if (b < B - 1) {
        const uint32_t g = (uint32_t)cmp[(uint64_t)(b + 1) * os - 1];
        spl[b] = Pair{keys[g], (uint32_t)sample_pos(g, n, s), 0};
    } else {
        spl[b] = Comp<int64_t>::inf();
    }
}

template <typename T>
__device__ __forceinline__ void load_splitters(const typename Comp<T>::C *spl_g, int BP,
                                               typename Comp<T>::C *spl) {
    for (int b = threadIdx.x; b < BP; b += BK_T) spl[b] = spl_g[b];
}

// Keys per partition workgroup: `subs` sub-tiles of BK_T * KPT keys, 4..16 so that a large
// input gets >= ~2048 workgroups with long per-bucket runs and a small one still fills the chip.
// The scatter holds one workgroup per CU (its LDS), so it runs in rounds of BK_CUS workgroups:
// among subs values up to that cap the one with the fewest sub-tiles per CU over all rounds wins
// (2^30 int32: 14 sub-tiles, 21 rounds = 294 sub-tiles per CU, instead of 16 with 18.3 rounds =
// 19 x 16 = 304).
constexpr uint64_t BK_CUS = 256;  // MI355X compute units
template <typename T>
__host__ __forceinline__ int bucket_wg_subs(uint64_t n) {
    const uint64_t sub = (uint64_t)BK_T * Geo<T>::KPT;
    const uint64_t v = n / (2048 * sub);
    const int cap = v < 4 ? 4 : (v > 16 ? 16 : (int)v);
    if (cap > 4) {
        const uint64_t nsub = (n + sub - 1) / sub;
        int best = cap;
        uint64_t bcost = ~0ull;
        for (int s = cap; s >= (cap + 1) / 2; --s) {
            const uint64_t rounds = ((nsub + s - 1) / s + BK_CUS - 1) / BK_CUS;
            if (rounds * s < bcost) {
                bcost = rounds * s;
                best = s;
            }
        }
        return best;
    }
    return cap;
}

// counts[g * B + b] = keys of workgroup g's subs sub-tiles in bucket b.  (The same slot table as
// the scatter's: the one-key slots must agree.)
template <typename T>
__global__ void __launch_bounds__(BK_T) bucket_hist_kernel(const T *__restrict__ in, uint64_t n,
                                                           const typename Comp<T>::C *__restrict__ spl_g,
                                                           const BkMap *__restrict__ map, int B, int BP,
                                                           int subs, uint32_t *__restrict__ counts) {
    using CT = Comp<T>;
    constexpr int KPT = Geo<T>::KPT, SUB = BK_T * KPT;
    __shared__ typename CT::C spl[BK_MAXB];
    __shared__ uint32_t rng[BK_SLOTS];
    const BkMap m = *map;
    __shared__ uint32_t hist[BK_MAXB];
    load_splitters<T>(spl_g, BP, spl);
    for (int b = threadIdx.x; b < B; b += BK_T) hist[b] = 0;
    __syncthreads();
    build_slots<T>(spl, BP, m, rng);
    __syncthreads();
    const uint64_t g0 = (uint64_t)blockIdx.x * subs * SUB;
#pragma unroll 1
    for (int sub = 0; sub < subs; ++sub) {
        const uint64_t b0 = g0 + (uint64_t)sub * SUB + threadIdx.x;
        T key[KPT];
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            const uint64_t i = b0 + (uint64_t)k * BK_T;
            key[k] = i < n ? in[i] : T(0);
        }
        // (the mode branch outside the key loop: a slot array would cost the second workgroup)
        if (!CT::ADAPT || m.mode == 0) {
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint64_t i = b0 + (uint64_t)k * BK_T;
                const uint32_t sl = slot_mode<T, BK_SLOTB, 0>(m, key[k]);
                if (i < n) atomicAdd(&hist[bucket_fast<T>(spl, rng, sl, key[k], CT::make(key[k], i))], 1u);
            }
        } else {
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint64_t i = b0 + (uint64_t)k * BK_T;
                const uint32_t sl = slot_mode<T, BK_SLOTB, 1>(m, key[k]);
                if (i < n) atomicAdd(&hist[bucket_fast<T>(spl, rng, sl, key[k], CT::make(key[k], i))], 1u);
            }
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < B; b += BK_T) counts[(uint64_t)blockIdx.x * B + b] = hist[b];
}

// part[c * B + b] = sum of counts[g * B + b] over the BK_CHUNK workgroups g of chunk c
static __global__ void __launch_bounds__(BK_MAXB) bucket_colsum_kernel(const uint32_t *__restrict__ counts,
                                                               uint32_t G, int B,
                                                               uint64_t *__restrict__ part) {
    const int b = threadIdx.x;
    if (b >= B) return;
    const uint32_t g0 = blockIdx.x * BK_CHUNK;
    const uint32_t g1 = g0 + BK_CHUNK < G ? g0 + BK_CHUNK : G;
    uint64_t sum = 0;
    for (uint32_t g = g0; g < g1; ++g) sum += counts[(uint64_t)g * B + b];
    part[(uint64_t)blockIdx.x * B + b] = sum;
}

// Tiles of a bucket [sk, sk + len) for a tile sort of TILE-key tiles with 16-byte loads of
// ALIGN keys: a head tile up to the next ALIGN-key boundary (0..ALIGN-1 keys), then TILE-key
// tiles from there.  The host plans the merge passes with the same rule.
__host__ __device__ __forceinline__ uint64_t bucket_head(uint64_t sk, uint64_t len, uint64_t align) {
    const uint64_t h = (align - (sk & (align - 1))) & (align - 1);
    return h < len ? h : len;
}
__host__ __device__ __forceinline__ uint64_t bucket_tiles(uint64_t sk, uint64_t len, uint64_t tile,
                                                          uint64_t align) {
    const uint64_t h = bucket_head(sk, len, align);
    return (h ? 1 : 0) + (len - h + tile - 1) / tile;
}

// exclusive scan of one value per thread over a BK_MAXB-thread workgroup; `all` = total
__device__ __forceinline__ uint64_t scan_excl_u64(uint64_t v, uint64_t *wsum, uint64_t &all) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    __syncthreads();
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint64_t off = 0;
    all = 0;
    for (int i = 0; i < BK_MAXB / 64; ++i) {
        if (i < w) off += wsum[i];
        all += wsum[i];
    }
    return off + incl - v;
}

// One workgroup: part -> exclusive prefix over chunks (in place); bucket starts bstart[0..B];
// the tile table of the tile sort (every bucket cut into tiles, bucket_tiles) and its size.
static __global__ void __launch_bounds__(BK_MAXB) bucket_scan_kernel(uint64_t *__restrict__ part,
                                                             uint32_t nchunk, int B, uint32_t tile,
                                                             uint32_t align,
                                                             uint64_t *__restrict__ bstart,
                                                             TileRef *__restrict__ tt,
                                                             uint32_t *__restrict__ ntiles) {
    __shared__ uint64_t wsum[BK_MAXB / 64];
    const int b = threadIdx.x;
    uint64_t tot = 0;
    if (b < B) {
        for (uint32_t c = 0; c < nchunk; ++c) {
            const uint64_t v = part[(uint64_t)c * B + b];
            part[(uint64_t)c * B + b] = tot;
            tot += v;
        }
    }
    uint64_t allk, allt;
    const uint64_t sk = scan_excl_u64(tot, wsum, allk);
    const uint64_t nt = b < B ? bucket_tiles(sk, tot, tile, align) : 0;
    const uint64_t st = scan_excl_u64(nt, wsum, allt);
    if (b < B) {
        bstart[b] = sk;
        const uint64_t h = bucket_head(sk, tot, align);
        uint64_t k = st;
        if (h) tt[k++] = TileRef{sk, (uint32_t)h, 0};
        for (uint64_t base = sk + h; base < sk + tot; base += tile) {
            const uint64_t rem = sk + tot - base;
            tt[k++] = TileRef{base, (uint32_t)(rem < (uint64_t)tile ? rem : tile), 0};
        }
    }
    if (b == 0) {
        bstart[B] = allk;
        *ntiles = (uint32_t)allt;
    }
}

// offs[g * B + b] = global position of workgroup g's first key of bucket b
template <typename O>
__global__ void __launch_bounds__(BK_MAXB) bucket_offsets_kernel(const uint32_t *__restrict__ counts,
                                                                const uint64_t *__restrict__ part,
                                                                const uint64_t *__restrict__ bstart,
                                                                uint32_t G, int B,
                                                                O *__restrict__ offs) {
    const int b = threadIdx.x;
    if (b >= B) return;
    const uint32_t g0 = blockIdx.x * BK_CHUNK;
    const uint32_t g1 = g0 + BK_CHUNK < G ? g0 + BK_CHUNK : G;
    uint64_t run = bstart[b] + part[(uint64_t)blockIdx.x * B + b];
    for (uint32_t g = g0; g < g1; ++g) {
        offs[(uint64_t)g * B + b] = (O)run;
        run += counts[(uint64_t)g * B + b];
    }
}

// Per sub-tile (BK_T * KPT keys): every key takes a slot of its bucket (atomic on the sub-tile
// histogram), which gives both its global position (the bucket's next position in this
// workgroup's range + slot) and its LDS position in the sub-tile laid out bucket by bucket
// (scan + slot).  Key and global position go to LDS there; then consecutive threads write
// consecutive LDS entries, i.e. consecutive keys of a bucket to consecutive addresses.  The order
// of keys inside a bucket is not kept (the bucket is sorted afterwards; the keys carry no
// payload).  The next sub-tile's keys are loaded while the current one is placed.
template <typename T>
__global__ void __launch_bounds__(BK_T) bucket_scatter_kernel(const T *__restrict__ in, uint64_t n,
                                                              const typename Comp<T>::C *__restrict__ spl_g,
                                                              const BkMap *__restrict__ map, int B, int BP, int subs,
                                                              const uint64_t *__restrict__ offs,
                                                              T *__restrict__ out, T *__restrict__ out2) {
    using CT = Comp<T>;
    constexpr int KPT = Geo<T>::KPT, SUB = BK_T * KPT;
    __shared__ typename CT::C spl[BK_MAXB];
    __shared__ uint8_t bpure[BK_MAXB];  // bucket between two splitters of one key: written to out2
    __shared__ uint32_t rng[BK_SLOTS];
    __shared__ uint2 sgo[BK_MAXB];       // (sub-tile scan, next global position) per bucket; n < 2^32
    __shared__ uint32_t hist[BK_MAXB];   // sub-tile histogram
    __shared__ uint32_t wsum[BK_T / 64];
    __shared__ T lk[SUB];                // the sub-tile grouped by bucket
    __shared__ uint32_t lg[SUB];         // global position of every LDS entry
    for (int b = threadIdx.x; b < B; b += BK_T) sgo[b] = make_uint2(0u, (uint32_t)offs[(uint64_t)blockIdx.x * B + b]);
    load_splitters<T>(spl_g, BP, spl);
    const BkMap m = *map;
    __syncthreads();
    build_slots<T>(spl, BP, m, rng);
    for (int b = threadIdx.x; b < B; b += BK_T)
        bpure[b] = out2 && b > 0 && b + 1 < B && CT::key_of(spl[b - 1]) == CT::key_of(spl[b]);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t g0 = (uint64_t)blockIdx.x * subs * SUB;
    T nxt[KPT];
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
        const uint64_t i = g0 + threadIdx.x + (uint64_t)k * BK_T;
        nxt[k] = i < n ? in[i] : T(0);
    }
#pragma unroll 1
    for (int sub = 0; sub < subs; ++sub) {
        const uint64_t s0 = g0 + (uint64_t)sub * SUB;
        if (s0 >= n) break;  // workgroup-uniform
        for (int b = threadIdx.x; b < B; b += BK_T) hist[b] = 0;
        __syncthreads();
        T key[KPT];
        int bk[KPT];
        uint32_t slot[KPT];
#pragma unroll
        for (int k = 0; k < KPT; ++k) key[k] = nxt[k];
        uint32_t sl[KPT];
        slots_at<T, KPT>(m, key, sl);
        if (sub + 1 < subs) {
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint64_t i = s0 + SUB + threadIdx.x + (uint64_t)k * BK_T;
                nxt[k] = i < n ? in[i] : T(0);
            }
        }
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            const uint64_t i = s0 + threadIdx.x + (uint64_t)k * BK_T;
            bk[k] = -1;
            if (i < n) {
                bk[k] = bucket_fast<T>(spl, rng, sl[k], key[k], CT::make(key[k], i));
                slot[k] = atomicAdd(&hist[bk[k]], 1u);
            }
        }
        __syncthreads();
        // exclusive scan of the sub-tile histogram (one bucket per thread)
        const uint32_t hv = threadIdx.x < (unsigned)B ? hist[threadIdx.x] : 0;
        uint32_t incl = hv;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t woff = 0;
        for (int i = 0; i < w; ++i) woff += wsum[i];
        if (threadIdx.x < (unsigned)B) sgo[threadIdx.x].x = woff + incl - hv;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            if (bk[k] >= 0) {
                const uint2 so = sgo[bk[k]];
                lk[so.x + slot[k]] = key[k];
                // (bit 31: a pure bucket, to out2; out2 is only given when n < 2^31)
                lg[so.x + slot[k]] = (so.y + slot[k]) | (uint32_t)bpure[bk[k]] << 31;
            }
        }
        __syncthreads();
        const uint32_t cnt = s0 + SUB <= n ? SUB : (uint32_t)(n - s0);
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            const uint32_t p = threadIdx.x + k * BK_T;
            if (p < cnt) {
                const uint32_t gp = lg[p];
                (gp >> 31 ? out2 : out)[gp & 0x7FFFFFFFu] = lk[p];
            }
        }
        // advance every bucket's global position by this sub-tile's keys (sgo.x is not read
        // again before the next scan, which follows two barriers)
        if (threadIdx.x < (unsigned)B) sgo[threadIdx.x].y += hv;
    }
}


// Inclusive sum over a wave (DPP row shifts, then the row broadcasts of lane 15 and 31).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// The int32 scatter with whole-line writes.  Every bucket of a workgroup's range is a stream of
// aligned 64-byte lines (16 keys): a sub-tile writes only the whole lines of each bucket (the
// bucket's carried keys + its new keys) and carries the rest (< 16 keys per bucket) in LDS to the
// next sub-tile, so HBM sees whole-line writes only (a per-sub-tile scatter writes each bucket's
// ~14 keys as a piece of a line the neighbouring sub-tiles complete: partial-line writes).  Only
// the first and last line of each bucket in the workgroup's range can be partial; the first is
// padded at the front with "phantom" entries up to the line boundary (never written).
// Per sub-tile, five barriers (round 2 had nine):
//   classify + rank (slot table, splitters, one LDS atomic per key)      | A
//   owner b: its count, whole lines and carry; one wave scan (DPP)       | B
//   owner b: its LDS start (into the dense count array), line-map entries for its lines | C
//   keys to LDS grouped by bucket                                        | D
//   line phase: 4 lanes per line, 16-byte stores                         | E
//   carry phase: owner b copies its stream's tail into its carry slot.
// (Measured and dropped, round 3: a thread per line entry with 4-byte stores, and 16-byte aligned
// stream regions with 16-byte LDS reads, which need 3 pad entries per bucket and so a 12-key
// sub-tile per thread: 3.6 ms vs 3.0 ms at 2^30.)
constexpr int BK_LK = 16;                                       // int32 keys per 64-byte line
constexpr int BK_LSUB = BK_T * Geo<int32_t>::KPT;               // keys per sub-tile
constexpr int BK_MAPN = (BK_LSUB + 30 * BK_MAXB) / BK_LK;       // lines per sub-tile, at most
static __global__ void __launch_bounds__(BK_T) bucket_scatter_lines_kernel(const int32_t *__restrict__ in, uint64_t n,
                                                                    const int64_t *__restrict__ spl_g,
                                                                    const BkMap *__restrict__ map, int B, int BP, int subs,
                                                                    const uint64_t *__restrict__ offs,
                                                                    int32_t *__restrict__ out,
                                                                    int32_t *__restrict__ out2) {
    using CT = Comp<int32_t>;
    constexpr int KPT = Geo<int32_t>::KPT, SUB = BK_LSUB;
    static_assert(SUB < (1 << 16), "packed scan fields");
    // (a non-last sub-tile writes <= (SUB + 15 B) / 16 lines, the last <= (SUB + 30 B) / 16)
    __shared__ int64_t spl[BK_MAXB];
    __shared__ uint32_t rng[BK_SLOTS];
    __shared__ uint32_t hist[BK_MAXB];               // sub-tile histogram, then the LDS starts
    __shared__ uint2 st[BK_MAXB];                    // per bucket: LDS start | first line << 16, vc|ph|pure|L
    __shared__ uint32_t sgb[BK_MAXB];                // per bucket: global index of stream entry 0
    __shared__ uint16_t lmap[BK_MAPN];               // line -> bucket
    __shared__ uint32_t wsum[BK_T / 64];
    __shared__ int32_t lk[SUB];                      // the sub-tile's new keys grouped by bucket
    __shared__ int32_t carry[BK_MAXB * BK_LK];       // per bucket: stream entries not yet written (< 16)
    const int tb = threadIdx.x, lane = tb & 63, w = tb >> 6;
    const uint32_t g = blockIdx.x;
    const bool owner = tb < B;  // thread b owns bucket b's line stream
    // owner state: vc = stream entries held in carry (phantoms included), ph = phantoms still in
    // front (the stream's first line not written yet), gb = global index of stream entry 0 (mod 2^32)
    uint32_t vc = 0, ph = 0, gb = 0, pure = 0;
    if (owner) {
        const uint32_t o = (uint32_t)offs[(uint64_t)g * B + tb];
        pure = out2 && tb > 0 && tb + 1 < B && CT::key_of(spl_g[tb - 1]) == CT::key_of(spl_g[tb]);
        ph = (uint32_t)(((uintptr_t)((pure ? out2 : out) + o) >> 2) & (BK_LK - 1));
        vc = ph;
        gb = o - ph;
        hist[tb] = 0;
    }
    load_splitters<int32_t>(spl_g, BP, spl);
    const BkMap m = *map;
    __syncthreads();
    build_slots<int32_t>(spl, BP, m, rng);
    __syncthreads();
    const uint64_t g0 = (uint64_t)g * subs * SUB;
    int32_t nxt[KPT];
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
        const uint64_t i = g0 + tb + (uint64_t)k * BK_T;
        nxt[k] = i < n ? in[i] : 0;
    }
#pragma unroll 1
    for (int sub = 0; sub < subs; ++sub) {
        const uint64_t s0 = g0 + (uint64_t)sub * SUB;
        if (s0 >= n) break;  // workgroup-uniform
        const bool last = sub + 1 == subs || s0 + SUB >= n;
        int32_t key[KPT];
        uint32_t pk[KPT];  // rank | bucket << 16; ~0 past the input
#pragma unroll
        for (int k = 0; k < KPT; ++k) key[k] = nxt[k];
        uint32_t sl[KPT];
        slots_at<int32_t, KPT>(m, key, sl);
        if (!last) {
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint64_t i = s0 + SUB + tb + (uint64_t)k * BK_T;
                nxt[k] = i < n ? in[i] : 0;
            }
        }
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            const uint64_t i = s0 + tb + (uint64_t)k * BK_T;
            pk[k] = ~0u;
            if (i < n) {
                const int b = bucket_fast<int32_t>(spl, rng, sl[k], key[k], CT::make(key[k], i));
                pk[k] = atomicAdd(&hist[b], 1u) | (uint32_t)b << 16;
            }
        }
        __syncthreads();  // A
        // owner: new keys, whole lines to write, entries carried to the next sub-tile
        const uint32_t hv = owner ? hist[tb] : 0;
        const uint32_t L = vc + hv;  // stream entries not yet written
        const uint32_t nl = !owner ? 0 : last ? (L > ph ? (L + BK_LK - 1) / BK_LK : 0) : L / BK_LK;
        const uint32_t pv = hv | nl << 16;
        const uint32_t incl = wave_incl_sum(pv);
        if (lane == 63) wsum[w] = incl;
        __syncthreads();  // B
        uint32_t woff = 0, all = 0;
#pragma unroll
        for (int i = 0; i < BK_T / 64; ++i) {
            const uint32_t v = wsum[i];
            woff += i < w ? v : 0;
            all += v;
        }
        const uint32_t ex = woff + incl - pv;
        const uint32_t lks = ex & 0xFFFF, p0 = ex >> 16, C = all >> 16;
        if (owner) {
            st[tb] = make_uint2(lks | p0 << 16, vc | ph << 5 | pure << 10 | L << 11);
            sgb[tb] = gb;
            hist[tb] = lks;  // the placement's LDS starts (a dense array: fewer bank conflicts)
            for (uint32_t i = 0; i < nl; ++i) lmap[p0 + i] = (uint16_t)tb;
        }
        __syncthreads();  // C
#pragma unroll
        for (int k = 0; k < KPT; ++k)
            if (pk[k] != ~0u) lk[hist[pk[k] >> 16] + (pk[k] & 0xFFFF)] = key[k];
        __syncthreads();  // D
        if (owner) hist[tb] = 0;  // (the next sub-tile's atomics follow barrier E)
        // whole lines: 4 lanes per line, 4 keys (16 bytes) per lane
        for (uint32_t it = tb; it < 4 * C; it += BK_T) {
            const uint32_t j = it >> 2, q = it & 3;
            const uint32_t b = lmap[j];
            const uint2 sb = st[b];
            const uint32_t cv = sb.y & 31, cp = (sb.y >> 5) & 31, cL = sb.y >> 11, lb = sb.x & 0xFFFF;
            const uint32_t e0 = (j - (sb.x >> 16)) * BK_LK + 4 * q;
            int32_t v[4];
            bool ok[4];
            bool full = true;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t e = e0 + t;
                ok[t] = e >= cp && e < cL;
                full = full && ok[t];
                v[t] = e < cv ? carry[b * BK_LK + e] : lk[lb + e - cv];
            }
            const uint32_t gi = sgb[b] + e0;  // mod 2^32
            int32_t *tgt = (sb.y >> 10) & 1 ? out2 : out;
            if (full) {
                *reinterpret_cast<int4 *>(tgt + gi) = make_int4(v[0], v[1], v[2], v[3]);
            } else {
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (ok[t]) tgt[(uint32_t)(gi + t)] = v[t];
            }
        }
        if (last) break;
        __syncthreads();  // E
        // carry the tail of every stream: entries [16 nl, L) -> carry[0, L - 16 nl) (the entries
        // below vc of a stream that wrote no line are there already)
        if (owner) {
            const uint32_t nv = L - nl * BK_LK;
            for (uint32_t e2 = nl ? 0 : vc; e2 < nv; ++e2) carry[tb * BK_LK + e2] = lk[lks + nl * BK_LK + e2 - vc];
            if (nl) ph = 0;
            gb += nl * BK_LK;
            vc = nv;
        }
    }
}

}  // namespace bk
}  // namespace dsort
