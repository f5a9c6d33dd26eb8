// dsort_bucket.h -- the first partition level of the bucketed sort (namespace dsort::bk; included
// by dsort_wave.hip, whose driver runs the second level (dsort_sub.h) and the tile sort inside
// the buckets).
//
// The multi-GPU design cuts the keys into key ranges with sample-sort splitters and sorts every
// range on its own GPU.  The same idea inside one GPU's HBM: B buckets (about
// 2^20 keys each) by splitters taken from a regular sample, in (key, input index) order so that
// duplicates are spread over buckets like any other key; one partition pass writes every bucket
// contiguously.  A partition pass resolves log2(B) bits of the order in about one read + one
// write of the keys (plus a read for the histogram).
//
// Kernels (all keyed by the composite c = (key, input index), unique per key):
//   bucket_sample_kernel / pair_*   s regular samples -> composites (sorted by the int64 sort)
//   bucket_splitter_kernel          splitter b = sample (b+1)*s/B - 1; padded with +inf to BP
//   bucket_slotmap_kernel           the lookups' slot map (int64: linear or log, one-key slots)
//   bucket_hist_kernel              per workgroup range: keys per bucket (LDS atomics)
//   bucket_colsum_kernel            per 64 workgroups: column sums        } exclusive scan of the
//   bucket_scan_kernel              one workgroup: chunk prefixes, bucket } histograms in (bucket,
//                                   starts, tile table of the tile sort   }  workgroup) order
//   bucket_offsets_kernel           per-workgroup bucket offsets          }
//   bucket_scatter_lines_kernel     per sub-tile: keys grouped by bucket in LDS, every bucket of
//                                   the workgroup's range written as whole 64-byte lines
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dsort_internal.h"

namespace dsort {
namespace bk {

constexpr int BK_T = 1024;               // threads of the partition kernels
constexpr int BK_MAXB = 1024;            // buckets at most (<= threads, one bucket per thread)
constexpr int BK_OS = 32;                // samples per bucket
#ifndef DSORT_BK_CHUNK
#define DSORT_BK_CHUNK 16
#endif
// workgroups per column-sum chunk.  (Round 6: 64 -> 16 with the chunk prefixes scanned by
// bucket_colscan_kernel: at 2^30 keys, 4681 histogram rows made 74 column-sum workgroups of 64
// serial-ish loads per thread, and the one-workgroup scan walked 74 chunk rows per column --
// column sums + scan + offsets took 68 us of a 7.6 ms sort.)
constexpr int BK_CHUNK = DSORT_BK_CHUNK;
constexpr int BK_CSEG = 16;              // segments of the chunk rows per column (bucket_colscan_kernel)

// Scatter sub-tile per key width: KPT keys per thread, SUB = BK_T * KPT keys staged in LDS
// (int32: 64 KiB next to the 64 KiB line carry of the line scatter).
template <typename T> struct Geo;
template <> struct Geo<int32_t> { static constexpr int KPT = 16; };  // (14: +0.09 ms; 12, 13 slower still)
// int64: 48 KiB next to the 64 KiB carry (8 keys with the splitters read from global memory on
// the lookups: C4 scatter 6.47 -> 7.09 ms)
#ifndef DSORT_BK_KPT64
#define DSORT_BK_KPT64 6
#endif
template <> struct Geo<int64_t> { static constexpr int KPT = DSORT_BK_KPT64; };
// Bucket ids (int64, skewed keys): the histogram stores every key's bucket (2 bytes) and the
// scatter reads it instead of repeating the lookup, when the lookup is the expensive one -- the log
// slot map or one-key slots (BkMap.ids, set by bucket_slotmap_kernel): at 2^30 Zipf (C4) scatter
// 6.52 -> 5.2-5.3 ms for histogram 2.08 -> 2.33 ms.  Uniform int64 keys (the linear map, no repeated
// splitter) keep the lookup: there the scatter gained nothing and the histogram's writes cost
// 1.50 -> 2.08 ms.  int32's packed lookup costs less than the 2 bytes per key would
// (DSORT_BK_IDS32 builds it for comparison: histogram 0.77 -> 1.23 ms, scatter 2.67 -> 3.25 ms at
// 2^30, profiles/r4_ab_bucket_ids_int32.log).
// Round 6: three 10-bit buckets per word (DSORT_BK_IDS3, int64: KPT = 6 keys in two words, B <=
// 1024) -- 1.33 bytes per key instead of 2: C4's id traffic 4.2 -> 2.8 GB, and the scatter still only
// unpacks.  (One byte per key, the bucket above its slot's first, took it to 2.1 GB, but the scatter's
// slot computation and table read cost more than the bytes saved: C4 11.84 -> 11.89 ms,
// profiles/r6_ab_ids8_dropped.log.)
#ifndef DSORT_BK_IDS3
#define DSORT_BK_IDS3 1
#endif
// Non-temporal stores (round 6) for the histogram's bucket ids and the int32 scatter's whole lines:
// written once and read by a later kernel after gigabytes of other traffic, they gain nothing from
// the caches.  2^30 int32 7.52 -> 7.46 ms of device time (4 of 4 interleaved runs), C4 10.81 ->
// 10.75 ms (profiles/r6_ab_nontemporal_lines_ids.log); the int64 scatter's lines measured neutral to
// worse, and the fill of the pure buckets +0.25 ms (profiles/r6_ab_fill_nontemporal_dropped.log);
// the sorted-runs instance (HT) keeps cached stores: its long streams of one bucket lost 0.05 ms
// (sorted and reversed input, profiles/r6_ab_nt_other_inputs.log).
#ifndef DSORT_IDS_NT
#define DSORT_IDS_NT 1
#endif
#ifndef DSORT_LINES_NT
#define DSORT_LINES_NT 1  // (bit 0: int32, bit 1: int64)
#endif
typedef int bk_v4i __attribute__((ext_vector_type(4)));
typedef long long bk_v2l __attribute__((ext_vector_type(2)));
template <typename T> struct BkIds {
#ifdef DSORT_BK_IDS32
    static constexpr bool ON = true;
#else
    static constexpr bool ON = sizeof(T) == 8;
#endif
    static constexpr int PER_WORD = DSORT_BK_IDS3 && sizeof(T) == 8 ? 3 : 2;  // buckets per 32-bit word
    static constexpr int BITS = PER_WORD == 3 ? 10 : 16;
    static constexpr uint32_t MASK = (1u << BITS) - 1;
};
static_assert(BK_MAXB <= 1024, "10-bit bucket ids");
// Ids of a sub-tile (SUB keys from key s): thread-major pairs (PER_WORD 2) -- thread t's KPT / 2 words
// at s / 2 + KPT t / 2 --, or (PER_WORD 3) word w of thread t at (s / SUB) (KPT / 3) BK_T + w BK_T + t:
// every access of a wave is 64 consecutive words.

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
    static constexpr bool ADAPT = false;  // fixed top-bit slots (see BkMap)
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
// int32 keeps the fixed map (the top SLOTB bits, ulo = 0), one-key slots included: its histogram
// runs at the HBM rate and the extra lookup work measured +0.5 ms there at 2^30 uniform keys.
constexpr int BK_SLOTB = 11;
constexpr int BK_SLOTS = 1 << BK_SLOTB;

struct BkMap {
    uint64_t ulo;   // flipped key of the first splitter
    uint32_t sh;    // linear shift
    uint32_t mode;  // 0 linear, 1 log
    uint64_t invn;  // 2^48 / n: index -> 16-bit fraction of the input
    uint32_t ids;   // int64: the histogram stores the buckets for the scatter (BkIds)
    uint32_t hot;   // runs of one bucket in the input (sorted, reversed, few keys): a wave's keys
                    // that share its first key's bucket count with one atomic (bucket_bump)
    uint32_t one;   // int32: neighbouring splitters share a key, so one-key slots may exist; the
                    // histogram's usual loop leaves their check out (2^30 uniform: 0.85 -> 0.78 ms)
    uint32_t ad;    // int32 (round 5): the adaptive map (ulo, sh, mode as int64's) instead of the fixed
                    // top-11-bit slots, when those crowd many splitters of several keys into one slot
                    // (many small keys: the reference's input.txt holds only 1..100).  The host reads
                    // it back and launches the kernels' adaptive instances (first_level)
    // int32 on the fixed map (round 6): ONE refined slot -- the most crowded slot of splitters of
    // several keys, when neither adaptive map thins it (keys of [1, 100] mixed half and half with
    // uniform ones: every map puts the small keys in one slot) -- gets a second table of BK_R2
    // sub-slots, linear over its splitters' key range (BkRefine); its keys look their bucket up
    // there instead of searching the slot's splitters.  r2s = the slot + 1 (0: none).
    uint32_t r2s;
    uint32_t r2lo;  // flipped key one below the refined slot's first splitter's (or the slot's start)
    uint32_t r2sh;  // sub-slot = (flipped key - r2lo) >> r2sh, clamped to [0, BK_R2)
};
// The refined slot's table follows the map (bucket_slotmap_kernel writes both): entry i = the
// splitters below sub-slot i (bits 0-13), "key implied" (bit 14: the sub-slot holds one key value),
// one-key flag (bit 15: its >= 2 splitters hold one key K), the splitters below sub-slot i + 1 (bits
// 16-31).  Sub-slot 0 reaches down to the slot's start, the last up to its end.  256 entries: the
// scatter keeps them in LDS (1 KiB is what its LDS has left) -- from global memory, the classify of a
// 2^30-key sort of [1, 100] keys mixed with uniform ones waited 20 K cycles per batch of 4 keys.
constexpr int BK_R2 = 256;
constexpr int BK_R2_BITS = 8;
constexpr uint32_t BK_R2_IMPLIED = 0x4000u;
constexpr size_t BK_MAP_BYTES = 64 + 4 * BK_R2;
static_assert(sizeof(BkMap) <= 64, "the refined table sits 64 bytes into the map");
__host__ __device__ __forceinline__ const uint32_t *bk_tab2(const BkMap *m) {
    return reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(m) + 64);
}
// the packed (scatter) entry of the refined slot: two or more splitters, count field all ones
constexpr uint32_t BK_PACKED_R2 = 0xFFFFFu;
// the non-packed (histogram) entry's flag of the refined slot
constexpr uint32_t BK_R2_FLAG = 0x4000u;

// The splitters say whether a wave's consecutive keys will mostly share a bucket: the input is
// sorted or reversed when the splitters' input indices run (nearly) monotone with their order, and
// has few distinct keys when a quarter of the neighbouring splitters share a key.  Then 64 lanes
// incrementing one LDS counter serialise (2^30 sorted int32: histogram 3.7 ms, scatter 5.4 ms, 5x and
// 2x uniform input), and the first level aggregates them; uniform input keeps its plain atomics.
template <typename T>
__device__ __forceinline__ uint32_t bucket_runs_hint(uint32_t nasc, uint32_t ndup, int nsp) {
    if (nsp < 16) return 0;
    const uint32_t pairs = (uint32_t)(nsp - 1);
    (void)ndup;  // (few distinct keys or Zipf: a wave holds several such runs -- not aggregated)
    return (8 * nasc >= 7 * pairs || 8 * nasc <= pairs) ? 1u : 0u;
}
// Count (rank) of bucket b for the active lanes of a wave: the lanes in the first active lane's
// bucket with one atomic, the others one each.  RANK: returns the key's rank in its bucket.
template <bool RANK>
__device__ __forceinline__ uint32_t bucket_bump(uint32_t *hist, int b, bool act) {
    const uint64_t am = __ballot(act);
    if (!am) return 0u;
    const int lane = (int)(threadIdx.x & 63), first = (int)__ffsll((long long)am) - 1;
    const int b0 = __shfl(b, first);
    const uint64_t same = __ballot(act && b == b0);
    uint32_t pos = 0, base = 0;
    if (act && b != b0) pos = atomicAdd(&hist[b], 1u);
    if (lane == first) base = atomicAdd(&hist[b0], (uint32_t)__popcll(same));
    if (RANK) {
        base = (uint32_t)__shfl((int)base, first);
        if (act && b == b0) pos = base + (uint32_t)__popcll(same & ((1ull << lane) - 1));
    }
    return pos;
}
// log mode: mantissa bits M, the largest with (KB - M + 1) * 2^M slots in the table
template <typename T, int SB>
__host__ __device__ constexpr int log_m() {
    int m = 0;
    while (m < 16 && (Comp<T>::KB - (m + 1) + 1) * (1 << (m + 1)) <= (1 << SB)) ++m;
    return m;
}

// ADP: the map of the sort is adaptive (int64 always; int32 when BkMap.ad, see bucket_slotmap_kernel)
template <typename T, int SB, int MODE, bool ADP = Comp<T>::ADAPT>
__host__ __device__ __forceinline__ uint32_t slot_mode(const BkMap &m, T key) {
    using U = typename Comp<T>::U;
    constexpr uint32_t NS = 1u << SB;
    constexpr int M = log_m<T, SB>();
    if (!ADP) return Comp<T>::slot_of(key, SB);
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
template <typename T, int SB = BK_SLOTB, bool ADP = Comp<T>::ADAPT>
__host__ __device__ __forceinline__ uint32_t slot_at(const BkMap &m, T key) {
    return m.mode == 0 ? slot_mode<T, SB, 0, ADP>(m, key) : slot_mode<T, SB, 1, ADP>(m, key);
}
// the slots of K keys, the (workgroup-uniform) mode branch taken once
template <typename T, int K, bool ADP = Comp<T>::ADAPT>
__device__ __forceinline__ void slots_at(const BkMap &m, const T (&key)[K], uint32_t (&sl)[K]) {
    if (!ADP || m.mode == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) sl[k] = slot_mode<T, BK_SLOTB, 0, ADP>(m, key[k]);
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) sl[k] = slot_mode<T, BK_SLOTB, 1, ADP>(m, key[k]);
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

// PACK (int32 on the fixed map only): the packed entry of bucket_fast's first branch (the scatter's table)
template <typename T, bool PACK, int SB = BK_SLOTB, bool ADP = Comp<T>::ADAPT>
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
        if constexpr (!ADP && PACK) {
            // int32: lo (bits 0-9), splitters in the slot (bits 10-11: 0, 1, 2 = two or more) and
            // bits 20..1 of the flipped key of the slot's one splitter, or the number of splitters
            // of a crowded slot (bits 12-31): see bucket_fast
            // (3: a one-key slot of that many splitters)
            const uint32_t in = cnt[1] - cnt[0];
            const uint32_t kb = in == 1 ? ((uint32_t)CT::key_of(spl[cnt[0]]) ^ 0x80000000u) << 11 >> 12 : in;
            const bool one = in >= 2 && CT::key_of(spl[cnt[0]]) == CT::key_of(spl[cnt[1] - 1]);
            rng[i] = m.r2s == (uint32_t)i + 1 ? cnt[0] | 2u << 10 | BK_PACKED_R2 << 12
                                              : cnt[0] | (one ? 3u : in > 2 ? 2u : in) << 10 | kb << 12;
        } else {
            // a slot whose (>= 2) splitters all hold one key K: see bucket_fast
            const bool one = cnt[1] >= cnt[0] + 2 && CT::key_of(spl[cnt[0]]) == CT::key_of(spl[cnt[1] - 1]);
            const bool r2 = !ADP && m.r2s == (uint32_t)i + 1;
            rng[i] = cnt[0] | (r2 ? BK_R2_FLAG : (uint32_t)one << 15) | (cnt[1] << 16);
        }
    }
}

// Bucket of (key, index).  In a one-key slot the copies of K may go to any bucket from the
// first of K's splitters to the one after the last (every one of those buckets holds keys <= K
// before it and >= K after it, and the buckets strictly inside hold only K).  Since round 6
// (bucket_onekey, DSORT_ONEKEY_HASH) they all go to the inner buckets, by a hash of the index.
// (Before: the two outer buckets took exactly the copies the composite order gives them (index <=
// the first run splitter's, > the last one's) and the copies in between were split over the inner
// buckets by index range, in proportion -- onekey_ab, kept for DSORT_ONEKEY_HASH=0.)
// Histogram and scatter use the same map and table, so they agree key for key.  (Which copy of
// K lands where does not matter to a keys-only sort.)
// int32: the slot entry carries the slot's first splitter's key down to bit 1 (the slot is the
// top 11 bits), so a key in a slot of at most one splitter needs no splitter read -- the usual
// case: uniform keys put one splitter in every other slot, about 2^22 values apart.  A key equal
// to that splitter in bits 31..1 compares its composite; a slot of two or more splitters searches
// them (their number is in the entry).  (Round 2 read the splitter for every key of a slot
// that had one: half of the keys, a dependent 8-byte LDS read on the way to the rank atomic.)
template <typename T>
__device__ __forceinline__ int onekey_ab(const typename Comp<T>::C &a, const typename Comp<T>::C &z, int lo, int hi,
                                         T key, const typename Comp<T>::C &c) {
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
__device__ __forceinline__ int refine_inner(int lo, int hi, uint32_t idx);
// Round 6 (DSORT_ONEKEY_HASH): the copies of K all go to the buckets strictly between K's first
// and last splitter, spread by a hash of the index (as in the refined slot, refine_pick) -- one read
// of K instead of two splitter reads (the int64 lookups are bound by LDS bandwidth, and C4 puts ~58 %
// of its keys in one-key slots), no run of neighbouring copies piling onto one bucket's counter, and
// the outer buckets hold only keys below / above K, so every copy of K lands in a pure bucket that
// the second level skips.  2^30 keys: C4 (int64 Zipf) 11.7 -> 11.2 ms, 16 distinct int32 keys 7.9 ->
// 5.2 ms, int32 keys of [1, 100] 6.1 -> 4.1 ms, uniform unchanged (profiles/r6_ab_onekey_hash_*.log).
// (Bit 0: int64, bit 1: int32.)
#ifndef DSORT_ONEKEY_HASH
#define DSORT_ONEKEY_HASH 3
#endif
template <typename T>
__device__ __forceinline__ int bucket_onekey(const typename Comp<T>::C *spl, int lo, int hi, T key,
                                             const typename Comp<T>::C &c) {
    if constexpr ((DSORT_ONEKEY_HASH >> (sizeof(T) == 8 ? 0 : 1)) & 1) {
        const T K = Comp<T>::key_of(spl[lo]);
        if (key != K) return key < K ? lo : hi;
        return refine_inner(lo, hi, Comp<T>::idx_of(c));
    }
    return onekey_ab<T>(spl[lo], spl[hi - 1], lo, hi, key, c);
}
// The refined slot (BkMap.r2s, int32 on the fixed map): the key's sub-slot entry, then
//  - a one-key sub-slot (its splitters all hold K): a key other than K lies below or above all of
//    them; the copies of K go to the buckets strictly between K's first and last splitter (each
//    holds only K, so any of them keeps the order), spread by a hash of the index.  (The first
//    level's one-key slots split K's copies by index range instead, which needs K's first and last
//    splitter -- two more reads -- and piles a workgroup's copies onto one counter.)  When the
//    sub-slot is one key value (key implied), no splitter is read at all;
//  - else a search among the sub-slot's splitters (none to a few)
// -- instead of a search over the whole slot's (e.g. ~500 splitters of 100 small keys, from global
// memory in the scatter).  Histogram and scatter pick alike, key for key.
__device__ __forceinline__ uint32_t refine_sub(uint32_t r2lo, uint32_t r2sh, int32_t key) {
    const uint32_t u = (uint32_t)key ^ 0x80000000u;
    const uint32_t d = (u < r2lo ? 0u : u - r2lo) >> r2sh;
    return d < (uint32_t)BK_R2 ? d : (uint32_t)BK_R2 - 1;
}
// the inner bucket of a copy of K at composite index idx (hi - lo >= 2)
__device__ __forceinline__ int refine_inner(int lo, int hi, uint32_t idx) {
    return lo + 1 + (int)__umulhi(idx * 2654435761u, (uint32_t)(hi - lo - 1));
}
// e: the sub-slot entry; kk: the key of the sub-slot's first splitter when not implied (one-key)
template <typename T>
__device__ __forceinline__ int refine_pick(const typename Comp<T>::C *spl, uint32_t e, T key,
                                           const typename Comp<T>::C &c) {
    int lo = (int)(e & 0x3FFF), hi = (int)(e >> 16);
    if (e & 0x8000) {
        if (!(e & BK_R2_IMPLIED)) {
            const T K = Comp<T>::key_of(spl[lo]);
            if (key != K) return key < K ? lo : hi;
        }
        return refine_inner(lo, hi, Comp<T>::idx_of(c));
    }
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (Comp<T>::lt(spl[mid], c)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ bool packed_refined(uint32_t r) { return ((r >> 10) & 3) == 2 && (r >> 12) == BK_PACKED_R2; }
// A slow key's splitters as a slot entry (lo | one-key << 15 | hi << 16), from its packed entry
__device__ __forceinline__ uint32_t packed_range(uint32_t r) {
    const uint32_t lo = r & 1023, in = (r >> 10) & 3, sb = r >> 12;
    return lo | (in == 3 ? 0x8000u : 0u) | (lo + (in == 1 ? 1u : sb)) << 16;
}

// The packed int32 entry (bucket_fast's first branch) split in two, for a classify that keeps
// several keys' table reads in flight: the fast result and whether the key needs the slow path
// (a slot of two or more splitters, or a key equal to the slot's splitter in bits 31..1).
__device__ __forceinline__ int packed_fast(uint32_t r, int32_t key, bool &slow) {
    const int lo = (int)(r & 1023);
    const uint32_t in = (r >> 10) & 3, sb = r >> 12;
    const uint32_t kb = ((uint32_t)key ^ 0x80000000u) << 11 >> 12;
    slow = in > 1 || (in == 1 && kb == sb);
    return lo + (int)(in == 1 && kb > sb);
}
__device__ __forceinline__ int packed_slow(const int64_t *spl, uint32_t r, int32_t key, int64_t c) {
    int lo = (int)(r & 1023);
    const uint32_t in = (r >> 10) & 3, sb = r >> 12;  // (the refined slot is the caller's: packed_refined)
    int hi = lo + (in == 1 ? 1 : (int)sb);
    if (in == 3) return bucket_onekey<int32_t>(spl, lo, hi, key, c);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (spl[mid] < c) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// int32 (round 4): one-key slots as well -- 16 distinct keys spread over the range put 64
// splitters of one key in a slot, and every key searched them (2^30: histogram 4.96 ms, scatter
// 9.0 ms).  The packed entry marks them with splitter count field 3.
// ONE = false: the caller knows the table has no one-key slot (BkMap.one).
// tab2 / m: the refined slot's table and the map (int32 on the fixed map; see BkMap.r2s)
template <typename T, bool PACK, bool ONE = true, bool ADP = Comp<T>::ADAPT>
__device__ __forceinline__ int bucket_fast(const typename Comp<T>::C *spl, const uint32_t *rng, uint32_t slot,
                                           T key, const typename Comp<T>::C &c, const uint32_t *tab2 = nullptr,
                                           const BkMap *m = nullptr) {
    const uint32_t r = rng[slot];
    if constexpr (!ADP && PACK) {
        // branch-free on the usual path; the rare keys that search take one wave-uniform branch
        // (per-key early returns doubled the histogram's branches and cost it 0.2 ms at 2^30)
        int lo = (int)(r & 1023);
        const uint32_t in = (r >> 10) & 3, sb = r >> 12;
        const uint32_t kb = ((uint32_t)key ^ 0x80000000u) << 11 >> 12;
        const int j = lo + (int)(in == 1 && kb > sb);
        const bool slow = in > 1 || (in == 1 && kb == sb);
        if (__builtin_expect(__ballot(slow) == 0, 1)) return j;
        if (!slow) return j;
        if (tab2 && sb == BK_PACKED_R2 && in == 2)
            return refine_pick<T>(spl, tab2[refine_sub(m->r2lo, m->r2sh, (int32_t)key)], key, c);
        int hi = lo + (in == 1 ? 1 : (int)sb);  // (the splitters searched: those of the slot)
        if (in == 3) return bucket_onekey<T>(spl, lo, hi, key, c);
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (Comp<T>::lt(spl[mid], c)) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    if constexpr (!ADP) {
        if (ONE && tab2 && (r & BK_R2_FLAG))
            return refine_pick<T>(spl, tab2[refine_sub(m->r2lo, m->r2sh, (int32_t)key)], key, c);
    }
    int lo = (int)(r & 0x3FFF), hi = (int)(r >> 16);
    if (ONE && (r & 0x8000)) return bucket_onekey<T>(spl, lo, hi, key, c);
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
    __shared__ uint32_t dup;  // two adjacent splitters of one key: one-key slots
    __shared__ uint32_t nasc, ndup;  // neighbouring splitters with ascending input index / one key
    if (j == 0) dup = nasc = ndup = 0;
    __syncthreads();
    if (j + 1 < nsp) {
        if (CT::idx_of(spl[j]) < CT::idx_of(spl[j + 1])) atomicAdd(&nasc, 1u);
        if (CT::key_of(spl[j]) == CT::key_of(spl[j + 1])) atomicAdd(&ndup, 1u);
    }
    const uint64_t invn = ((uint64_t)1 << 48) / (n > 0 ? n : 1);
    BkMap mm[2] = {{0, (uint32_t)(CT::KB - BK_SLOTB), 0, invn, 0, 0}, {0, 0, 1, invn, 0, 0}};
    if constexpr (!CT::ADAPT) {
        // int32: the fixed map (the packed lookup) unless it puts more than AD_MIX splitters of
        // several keys into one slot -- every key there binary-searches them, from global memory in
        // the scatter (2^30 keys of 1..100: 19.8 ms).  Then the adaptive map of int64 (linear over
        // the splitters' range, or log) with one-key slots, if its most crowded such slot is smaller.
        // The cost of a map: its largest slot of splitters of at least two keys (a slot of one key is
        // a one-key slot: no search).
        constexpr uint32_t AD_MIX = 8;
        __shared__ uint32_t tot[3][BK_SLOTS], dst[3][BK_SLOTS];
        __shared__ uint32_t cost[3];
        for (int i = j; i < 3 * BK_SLOTS; i += blockDim.x) tot[i / BK_SLOTS][i % BK_SLOTS] = dst[i / BK_SLOTS][i % BK_SLOTS] = 0;
        if (j < 3) cost[j] = 0;
        BkMap am[3] = {mm[0], mm[0], mm[1]};  // fixed, adaptive linear, adaptive log
        if (nsp >= 1) {
            const uint32_t lo = CT::flip(CT::key_of(spl[0])), hi = CT::flip(CT::key_of(spl[nsp - 1]));
            const uint32_t r = hi - lo;
            const int bits = r == 0 ? 0 : 32 - __builtin_clz(r);
            am[1] = BkMap{(uint64_t)lo, (uint32_t)(bits > BK_SLOTB ? bits - BK_SLOTB : 0), 0, invn, 0, 0};
            am[2] = BkMap{(uint64_t)lo, 0, 1, invn, 0, 0};
        }
        __syncthreads();
        if (j < nsp) {
            const T k = CT::key_of(spl[j]);
            const bool first = j == 0 || CT::key_of(spl[j - 1]) != k;
            const uint32_t sl[3] = {slot_mode<T, BK_SLOTB, 0, false>(am[0], k), slot_mode<T, BK_SLOTB, 0, true>(am[1], k),
                                    slot_mode<T, BK_SLOTB, 1, true>(am[2], k)};
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                atomicAdd(&tot[q][sl[q]], 1u);
                if (first) atomicAdd(&dst[q][sl[q]], 1u);
            }
        }
        __syncthreads();
        for (int i = j; i < 3 * BK_SLOTS; i += blockDim.x)
            if (dst[i / BK_SLOTS][i % BK_SLOTS] >= 2) atomicMax(&cost[i / BK_SLOTS], tot[i / BK_SLOTS][i % BK_SLOTS]);
        __syncthreads();
        // the fixed map kept although its most crowded slot of several keys holds more than AD_MIX
        // splitters: that slot (the lowest of the most crowded) is refined (BkMap.r2s)
        // -- unless an adaptive map thins every slot to AD_MIX (e.g. all keys in [1, 100]): the choice
        // is the lower of the adaptive maps' cost and the fixed map's cost without the refined slot
        __shared__ uint32_t r2slot, cost2;
        __shared__ BkMap rm;
        if (j == 0) {
            r2slot = ~0u;
            cost2 = 0;
        }
        __syncthreads();
        const int qa = cost[2] < cost[1] ? 2 : 1;  // the better adaptive map
        if (cost[0] > AD_MIX && cost[qa] > AD_MIX)
            for (int i = j; i < BK_SLOTS; i += blockDim.x)
                if (dst[0][i] >= 2 && tot[0][i] == cost[0]) atomicMin(&r2slot, (uint32_t)i);
        __syncthreads();
        if (r2slot != ~0u)
            for (int i = j; i < BK_SLOTS; i += blockDim.x)
                if ((uint32_t)i != r2slot && dst[0][i] >= 2) atomicMax(&cost2, tot[0][i]);
        __syncthreads();
        const bool refine = r2slot != ~0u && cost2 <= cost[qa];
        const bool fixed = cost[0] <= AD_MIX || refine;
        if (j == 0) {
            if (!refine) r2slot = ~0u;
            BkMap r = fixed ? am[0] : am[qa];
            r.ad = r.ulo != 0 || r.mode != 0 || r.sh != (uint32_t)(CT::KB - BK_SLOTB) ? 1u : 0u;
            r.ids = BkIds<T>::ON ? 1u : 0u;  // (int32 with DSORT_BK_IDS32: always)
            r.hot = bucket_runs_hint<T>(nasc, ndup, nsp);
            r.one = r.ad ? 1u : (ndup != 0);
            r.r2s = r.r2lo = r.r2sh = 0;
            if (r2slot != ~0u) {
                // the slot's splitters [a, z): sub-slots linear over their key range
                uint32_t a = 0, z = 0;
                for (int k = 0; k < nsp; ++k) {
                    const uint32_t sk = slot_mode<T, BK_SLOTB, 0, false>(am[0], CT::key_of(spl[k]));
                    a += sk < r2slot;
                    z += sk <= r2slot;
                }
                // (sub-slot 0 below the first splitter's key when the slot starts lower: then sub-slot
                // 1 is that key, and with r2sh = 0 every inner sub-slot is one key value)
                uint64_t us0 = 0;
                (void)slot_first<T, BK_SLOTB>(am[0], r2slot, us0);
                // (the top 1/32 of the slot's splitters left out of the range: a stray splitter far
                // above the crowd -- a uniform key in the small keys' slot -- would widen every
                // sub-slot; keys above the range take the last sub-slot, which searches)
                const uint32_t k0 = CT::flip(CT::key_of(spl[a])), hi = CT::flip(CT::key_of(spl[z - 1 - (z - a) / 32]));
                const uint32_t lo = r2slot > 0 && k0 > (uint32_t)us0 ? k0 - 1 : k0;
                const uint32_t rr = hi - lo;
                const int bits = rr == 0 ? 0 : 32 - __builtin_clz(rr);
                r.r2s = r2slot + 1;
                r.r2lo = lo;
                r.r2sh = (uint32_t)(bits > BK_R2_BITS ? bits - BK_R2_BITS : 0);
                r.one = 1;  // (the histogram's loop with the one-key and refined checks)
                static_assert(BK_R2 == 1 << BK_R2_BITS, "sub-slots");
            }
            rm = r;
            *out = r;
        }
        __syncthreads();
        if (rm.r2s) {
            // sub-slot i: the splitters below its start (sub-slot 0 from the slot's start, a sub-slot
            // past the slot's end empty at its end), one-key flag as in a slot entry
            uint32_t *tab = const_cast<uint32_t *>(bk_tab2(out));
            const uint32_t s2 = rm.r2s - 1;
            uint64_t us = 0, ue = 0;
            const bool has_next = s2 + 1 < (uint32_t)BK_SLOTS && slot_first<T, BK_SLOTB>(am[0], s2 + 1, ue);
            (void)slot_first<T, BK_SLOTB>(am[0], s2, us);  // (the fixed map: slot s2's first flipped key)
            const int BPl = 1 << (32 - __builtin_clz((uint32_t)(nsp > 0 ? nsp : 1)));  // (a power of two >= nsp)
            auto below = [&](uint64_t u) -> uint32_t {  // splitters with composite < (flipped key u, index 0)
                const typename CT::C cc = CT::slot_start(u);
                uint32_t lo = 0, hi = (uint32_t)nsp;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (CT::lt(spl[mid], cc)) lo = mid + 1;
                    else hi = mid;
                }
                return lo;
            };
            (void)BPl;
            const uint32_t c_lo = s2 == 0 ? 0u : below(us), c_hi = has_next ? below(ue) : (uint32_t)nsp;
            for (int i = j; i < BK_R2; i += blockDim.x) {
                uint32_t c0 = c_lo, c1 = c_hi;
                if (i > 0) {
                    const uint64_t u = (uint64_t)rm.r2lo + ((uint64_t)i << rm.r2sh);
                    c0 = has_next && u >= ue ? c_hi : (u > 0xFFFFFFFFull ? c_hi : below(u));
                }
                if (i + 1 < BK_R2) {
                    const uint64_t u = (uint64_t)rm.r2lo + ((uint64_t)(i + 1) << rm.r2sh);
                    c1 = has_next && u >= ue ? c_hi : (u > 0xFFFFFFFFull ? c_hi : below(u));
                }
                c0 = c0 < c_lo ? c_lo : c0;
                const bool one = c1 >= c0 + 2 && CT::key_of(spl[c0]) == CT::key_of(spl[c1 - 1]);
                // (one key value: sub-slots 1 .. BK_R2 - 2 of a unit-width table; the outer ones take
                // every key below / above)
                const bool implied = rm.r2sh == 0 && i > 0 && i + 1 < BK_R2;
                tab[i] = c0 | (implied ? BK_R2_IMPLIED : 0u) | (uint32_t)one << 15 | c1 << 16;
            }
        }
        return;
    }
    if (nsp >= 1) {
        const U lo = CT::flip(CT::key_of(spl[0])), hi = CT::flip(CT::key_of(spl[nsp - 1]));
        const U r = hi - lo;
        const int bits = r == 0 ? 0 : (int)(sizeof(U) * 8) - (sizeof(U) == 8 ? __builtin_clzll((uint64_t)r)
                                                                               : __builtin_clz((uint32_t)r));
        mm[0] = BkMap{(uint64_t)lo, (uint32_t)(bits > BK_SLOTB ? bits - BK_SLOTB : 0), 0, invn, 0, 0};
        mm[1] = BkMap{(uint64_t)lo, 0, 1, invn, 0, 0};
    }
    __syncthreads();
    // count the distinct splitter keys of every slot under both maps
    if (j > 0 && j < nsp && CT::key_of(spl[j]) == CT::key_of(spl[j - 1])) dup = 1;
    if (j < nsp && (j == 0 || CT::key_of(spl[j]) != CT::key_of(spl[j - 1]))) {
        const T k = CT::key_of(spl[j]);
        atomicAdd(&cnt[0][slot_at<T>(mm[0], k)], 1u);
        atomicAdd(&cnt[1][slot_at<T>(mm[1], k)], 1u);
    }
    __syncthreads();
    for (int i = j; i < 2 * BK_SLOTS; i += blockDim.x) atomicMax(&crowd[i / BK_SLOTS], cnt[i / BK_SLOTS][i % BK_SLOTS]);
    __syncthreads();
    if (j == 0) {
        BkMap r = crowd[1] < crowd[0] ? mm[1] : mm[0];
        r.ids = BkIds<T>::ON && (r.mode == 1 || dup) ? 1u : 0u;
        r.hot = bucket_runs_hint<T>(nasc, ndup, nsp);
        r.one = 1;
        *out = r;
    }
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

// A sub-tile's keys of one thread: in[i0 + k BK_T], k < KPT.  UNGUARDED: a whole sub-tile (the
// usual case, workgroup-uniform) loads without bounds checks -- with them every load sat in a
// branch of its own (an exec-mask save, a conditional jump), and the scatter's loads were not
// issued together (int32 scatter 2.59 -> 2.49 ms, int64 Zipf 4.53 -> 4.45 ms).  The histogram keeps
// the checks: unguarded, its int64 instance took 2.21 -> 3.09 ms at 2^30 Zipf (int32: no change).
#ifndef DSORT_NOGUARD
#define DSORT_NOGUARD 1
#endif
template <typename T, int KPT, bool UNGUARDED = true>
__device__ __forceinline__ void load_sub(const T *__restrict__ in, uint64_t i0, uint64_t n, uint64_t sub_end,
                                         T (&x)[KPT]) {
    if (UNGUARDED && DSORT_NOGUARD && sub_end <= n) {
#pragma unroll
        for (int k = 0; k < KPT; ++k) x[k] = in[i0 + (uint64_t)k * BK_T];
    } else {
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
            const uint64_t i = i0 + (uint64_t)k * BK_T;
            x[k] = i < n ? in[i] : T(0);
        }
    }
}

// spl holds BK_MAXB + 1 entries: the BP splitters (+inf padded), +inf up to the end (the int32
// lookup of the last slot searches up to BK_MAXB)
template <typename T>
__device__ __forceinline__ void load_splitters(const typename Comp<T>::C *spl_g, int BP,
                                               typename Comp<T>::C *spl) {
    for (int b = threadIdx.x; b <= BK_MAXB; b += BK_T) spl[b] = b < BP ? spl_g[b] : Comp<T>::inf();
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
// the scatter's: the one-key slots must agree.)  ioff: the composite index of in[0] (the multi-GPU
// path: this rank's first key in the global order; 0 on one GPU).  AD (int32): the instance of the
// adaptive map (BkMap.ad; the host launches the one the slot map chose).
template <typename T, bool AD = false>
__global__ void __launch_bounds__(BK_T, 2) bucket_hist_kernel(const T *__restrict__ in, uint64_t n,
                                                              const typename Comp<T>::C *__restrict__ spl_g,
                                                              const BkMap *__restrict__ map, int B, int BP,
                                                              int subs, uint32_t *__restrict__ counts,
                                                              uint64_t ioff, uint32_t *__restrict__ ids) {
    using CT = Comp<T>;
    constexpr bool ADP = CT::ADAPT || AD;
    constexpr int KPT = Geo<T>::KPT, SUB = BK_T * KPT;
    static_assert(!BkIds<T>::ON || KPT % BkIds<T>::PER_WORD == 0, "bucket ids: whole words per thread");
    __shared__ typename CT::C spl[BK_MAXB + 1];
    __shared__ uint32_t rng[BK_SLOTS];
    const BkMap m = *map;
    if (!ADP && m.ad) return;  // (int32: the adaptive map's instance counts this sort, first_level)
    __shared__ uint32_t hist[BK_MAXB];
    __shared__ uint32_t tab2[ADP ? 1 : BK_R2];  // (the refined slot's table, BkMap.r2s)
    load_splitters<T>(spl_g, BP, spl);
    for (int b = threadIdx.x; b < B; b += BK_T) hist[b] = 0;
    if (!ADP && m.r2s)
        for (int i = threadIdx.x; i < BK_R2; i += BK_T) tab2[i] = bk_tab2(map)[i];
    __syncthreads();
    build_slots<T, false, BK_SLOTB, ADP>(spl, BP, m, rng);  // (the packed table measured 0.78 -> 0.93 ms here)
    __syncthreads();
    const uint64_t g0 = (uint64_t)blockIdx.x * subs * SUB;
    // the next sub-tile's keys are loaded while the current one is counted (two workgroups per CU
    // alone left the loads' latency exposed: 0.79 ms for 4.3 GB)
    T nxt[KPT];
    load_sub<T, KPT, false>(in, g0 + threadIdx.x, n, g0 + SUB, nxt);
#pragma unroll 1
    for (int sub = 0; sub < subs; ++sub) {
        const uint64_t b0 = g0 + (uint64_t)sub * SUB + threadIdx.x;
        T key[KPT];
#pragma unroll
        for (int k = 0; k < KPT; ++k) key[k] = nxt[k];
        if (sub + 1 < subs) load_sub<T, KPT, false>(in, b0 + SUB, n, b0 - threadIdx.x + 2 * SUB, nxt);
        // the buckets of the thread's keys, BkIds::PER_WORD per word (bucket ids)
        constexpr int PW = BkIds<T>::PER_WORD;
        static_assert(!BkIds<T>::ON || KPT % PW == 0, "bucket ids: whole words per thread");
        uint32_t idw[KPT / PW > 0 ? KPT / PW : 1] = {};
        const auto idput = [&](int k, int b) { idw[k / PW] |= (uint32_t)b << (BkIds<T>::BITS * (k % PW)); };
        // (the mode branch outside the key loop: a slot array would cost the second workgroup)
        if (m.hot) {  // (runs of one bucket: aggregated increments, bucket_runs_hint)
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint64_t i = b0 + (uint64_t)k * BK_T;
                const uint32_t sl = m.mode == 0 ? slot_mode<T, BK_SLOTB, 0, ADP>(m, key[k]) : slot_mode<T, BK_SLOTB, 1, ADP>(m, key[k]);
                const int b = bucket_fast<T, false, true, ADP>(spl, rng, sl, key[k], CT::make(key[k], i + ioff), tab2, &m);
                bucket_bump<false>(hist, b, i < n);
                if (i < n) idput(k, b);
            }
        } else if (ADP ? m.mode == 0 : !m.one) {
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint64_t i = b0 + (uint64_t)k * BK_T;
                const uint32_t sl = slot_mode<T, BK_SLOTB, 0, ADP>(m, key[k]);
                if (i < n) {
                    const int b = bucket_fast<T, false, ADP, ADP>(spl, rng, sl, key[k], CT::make(key[k], i + ioff));
                    atomicAdd(&hist[b], 1u);
                    idput(k, b);
                }
            }
        } else {  // (int64 log map; int32 with one-key slots -- its slot_mode ignores the mode)
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint64_t i = b0 + (uint64_t)k * BK_T;
                const uint32_t sl = slot_mode<T, BK_SLOTB, 1, ADP>(m, key[k]);
                if (i < n) {
                    const int b = bucket_fast<T, false, true, ADP>(spl, rng, sl, key[k], CT::make(key[k], i + ioff), tab2, &m);
                    atomicAdd(&hist[b], 1u);
                    idput(k, b);
                }
            }
        }
        // thread-major: the KPT ids of thread t of a sub-tile at words (sub-tile start + KPT t) / 2,
        // i.e. a thread stores (and the scatter's thread loads) KPT / 2 consecutive words -- one
        // 2-byte access per key measured slower than the lookup it replaces (int32)
        if (BkIds<T>::ON && m.ids) {
            if constexpr (PW == 3) {
                uint32_t *dst = ids + (b0 - threadIdx.x) / SUB * (KPT / 3) * BK_T + threadIdx.x;
#pragma unroll
                for (int w = 0; w < KPT / 3; ++w) {
#if DSORT_IDS_NT
                    __builtin_nontemporal_store(idw[w], dst + w * BK_T);
#else
                    dst[w * BK_T] = idw[w];
#endif
                }
            } else {
                uint32_t *dst = ids + (b0 - threadIdx.x) / 2 + (uint64_t)threadIdx.x * (KPT / 2);
#pragma unroll
                for (int w = 0; w < KPT / 2; ++w) dst[w] = idw[w];
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
#pragma unroll 8
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

// Columns [64 blk, 64 blk + 64) of part (nchunk rows of chunk sums): every column's exclusive
// prefix over the chunks, in place, and its total tot[b].  Thread (column c, segment q) sums its
// segment's rows (loads in flight together), the 16 segment sums are scanned in LDS, then the
// segment's rows are rewritten as prefixes.
static __global__ void __launch_bounds__(BK_MAXB) bucket_colscan_kernel(uint64_t *__restrict__ part, uint32_t nchunk,
                                                                       int B, uint64_t *__restrict__ tot) {
    __shared__ uint64_t seg[BK_CSEG][64];
    const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int b = (int)blockIdx.x * 64 + c;
    const uint32_t per = (nchunk + BK_CSEG - 1) / BK_CSEG;
    const uint32_t r0 = (uint32_t)q * per, r1 = r0 + per < nchunk ? r0 + per : nchunk;
    constexpr uint32_t U = 8;
    uint64_t sum = 0;
    if (b < B)
        for (uint32_t r = r0; r < r1; r += U) {
            uint64_t v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) v[u] = r + u < r1 ? part[(uint64_t)(r + u) * B + b] : 0;
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) sum += v[u];
        }
    seg[q][c] = sum;
    __syncthreads();
    uint64_t run = 0;
    for (int i = 0; i < q; ++i) run += seg[i][c];
    if (b < B) {
        if (q == BK_CSEG - 1) tot[b] = run + sum;
        for (uint32_t r = r0; r < r1; r += U) {
            uint64_t v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) v[u] = r + u < r1 ? part[(uint64_t)(r + u) * B + b] : 0;
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                if (r + u < r1) part[(uint64_t)(r + u) * B + b] = run;
                run += v[u];
            }
        }
    }
}

// One workgroup: part -> exclusive prefix over chunks (in place); bucket starts bstart[0..B];
// the tile table of the tile sort (every bucket cut into tiles, bucket_tiles) and its size.
// ctot (not null): the column totals of bucket_colscan_kernel, which has scanned part already.
// cspl (not null, the bucket exchange, round 6): the compacted starts cstart[0..B] too -- the
// starts with every pure bucket (between two splitters of one key, whose keys the scatter drops)
// of size 0: the scatter's layout of `part`, so the keys a rank ships are contiguous per peer and
// a pure bucket ships none.
template <typename T>
__global__ void __launch_bounds__(BK_MAXB) bucket_scan_kernel(uint64_t *__restrict__ part,
                                                             uint32_t nchunk, int B, uint32_t tile,
                                                             uint32_t align,
                                                             uint64_t *__restrict__ bstart,
                                                             TileRef *__restrict__ tt,
                                                             uint32_t *__restrict__ ntiles,
                                                             const uint64_t *__restrict__ ctot,
                                                             const typename Comp<T>::C *__restrict__ cspl,
                                                             uint64_t *__restrict__ cstart) {
    __shared__ uint64_t wsum[BK_MAXB / 64];
    const int b = threadIdx.x;
    uint64_t tot = 0;
    if (ctot) {
        if (b < B) tot = ctot[b];
    } else if (b < B) {
        // column b's chunk sums -> exclusive prefixes, 8 loads in flight at a time (a serial chain
        // of dependent round trips took 92 us per sort at 2^30)
        constexpr uint32_t U = 8;
        for (uint32_t c0 = 0; c0 < nchunk; c0 += U) {
            uint64_t v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) v[u] = c0 + u < nchunk ? part[(uint64_t)(c0 + u) * B + b] : 0;
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                if (c0 + u < nchunk) part[(uint64_t)(c0 + u) * B + b] = tot;
                tot += v[u];
            }
        }
    }
    uint64_t allk, allt;
    const uint64_t sk = scan_excl_u64(tot, wsum, allk);
    // (tile == 0: no tile table -- the second partition level makes its own tiles)
    const uint64_t nt = b < B && tile ? bucket_tiles(sk, tot, tile, align) : 0;
    const uint64_t st = scan_excl_u64(nt, wsum, allt);
    if (b < B) bstart[b] = sk;
    if (b < B && tile) {
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
    if (cspl) {  // (workgroup-uniform)
        const bool pure = b > 0 && b + 1 < B && Comp<T>::key_of(cspl[b - 1]) == Comp<T>::key_of(cspl[b]);
        uint64_t allc;
        const uint64_t sc = scan_excl_u64(b < B && !pure ? tot : 0, wsum, allc);
        if (b < B) cstart[b] = sc;
        if (b == 0) cstart[B] = allc;
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
#pragma unroll 8
    for (uint32_t g = g0; g < g1; ++g) {
        offs[(uint64_t)g * B + b] = (O)run;
        run += counts[(uint64_t)g * B + b];
    }
}


// The scatter with whole-line writes (both key widths).  Every bucket of a workgroup's range is a stream of
// aligned 64-byte lines (16 int32 / 8 int64 keys): a sub-tile writes only the whole lines of each bucket (the
// bucket's carried keys + its new keys) and carries the rest (< 16 keys per bucket) in LDS to the
// next sub-tile, so HBM sees whole-line writes only (a per-sub-tile scatter writes each bucket's
// ~14 keys as a piece of a line the neighbouring sub-tiles complete: partial-line writes, 34 % of
// the int64 scatter's write requests in round 2).  Only
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
// Line geometry per key width: LK keys per 64-byte line, SUB keys per sub-tile, map entries.
template <typename T> struct LineGeo {
    static constexpr int LK = 64 / (int)sizeof(T);                  // keys per 64-byte line
    static constexpr int KPL = 16 / (int)sizeof(T);                 // keys per 16-byte lane store
    static constexpr int SUB = BK_T * Geo<T>::KPT;                  // keys per sub-tile
    static constexpr int MAPN = (SUB + 2 * (LK - 1) * BK_MAXB) / LK; // lines per sub-tile, at most
};
#ifdef DSORT_STAMPS
// Diagnostic build only: per-workgroup phase cycles of the line scatter (wave 0's view), read back
// by dsort_debug_bkstamps() (scripts/dev/bkstamps.py).
__device__ unsigned long long g_bkstamps[8192 * 16];
#define BKST(k)                                            \
    do {                                                   \
        const uint64_t t1_ = __builtin_amdgcn_s_memtime(); \
        bk_acc[k] += t1_ - bk_t0;                          \
        bk_t0 = t1_;                                       \
    } while (0)
#else
#define BKST(k) \
    do {        \
    } while (0)
#endif
// IDS: the variant that reads the histogram's buckets (BkIds).  The host launches both variants for
// int64 (it does not know the map's choice); the one that does not match m.ids returns at once
// (one kernel with a run-time branch: uniform int64 scatter 5.29 -> 5.84 ms).
// HT: the instance for input with runs of one bucket (BkMap.hot: sorted, reversed), which enters a
// long line stream in the line map with the owner's whole wave.
template <typename T, bool IDS, bool AD = false, bool HT = false>
__global__ void __launch_bounds__(BK_T) bucket_scatter_lines_kernel(const T *__restrict__ in, uint64_t n,
                                                                    const typename Comp<T>::C *__restrict__ spl_g,
                                                                    const BkMap *__restrict__ map, int B, int BP, int subs,
                                                                    const uint32_t *__restrict__ offs,
                                                                    T *__restrict__ out, T *__restrict__ out2,
                                                                    uint64_t ioff, const uint32_t *__restrict__ ids) {
    using CT = Comp<T>;
    constexpr bool ADP = CT::ADAPT || AD;  // (AD: int32's adaptive-map instance, BkMap.ad)
    static_assert(!IDS || BkIds<T>::ON, "bucket ids of this key width");
    using G = LineGeo<T>;
    using V = typename std::conditional<sizeof(T) == 4, int4, longlong2>::type;
    constexpr int KPT = Geo<T>::KPT, SUB = G::SUB, LK = G::LK, KPL = G::KPL;
    static_assert(SUB + LK < (1 << 16) && LK <= 16, "packed fields");
    // (a non-last sub-tile writes <= (SUB + (LK-1) B) / LK lines, the last <= (SUB + 2 (LK-1) B) / LK)
    // int32: the splitters are staged in lk for the slot table only (the packed lookup reads them
    // from global memory on its rare slow path), which leaves lk room for 16 keys per thread
    constexpr bool SPL_LK = !CT::ADAPT;
    __shared__ typename CT::C spl_own[SPL_LK || IDS ? 1 : BK_MAXB + 1];
    __shared__ uint32_t rng[IDS ? 1 : BK_SLOTS];
    __shared__ uint32_t hist[BK_MAXB];               // sub-tile histogram, then the LDS starts
    __shared__ uint2 st[BK_MAXB];                    // per bucket: LDS start | first line << 16, vc|ph|pure|L
    __shared__ uint32_t sgb[BK_MAXB];                // per bucket: global index of stream entry 0
    __shared__ uint16_t lmap[G::MAPN];               // line -> bucket
    __shared__ uint32_t wsum[BK_T / 64];
    __shared__ T lk[SUB];                            // the sub-tile's new keys grouped by bucket
    __shared__ T carry[BK_MAXB * LK];                // per bucket: stream entries not yet written (< LK)
    static_assert(!SPL_LK || sizeof(lk) >= (BK_MAXB + 1) * sizeof(typename CT::C), "splitters staged in lk");
    // carry entry e of bucket b at b LK + (e ^ ((b >> 1) & (LK - 1))): the owners' copy (lane b
    // writes entry e2 of its bucket) and the line phase's reads hit distinct banks instead of the
    // two (int32) that the LK-word row stride leaves them (scatter 2.72 -> 2.62 ms at 2^30 int32)
    const auto cswz = [](uint32_t b, uint32_t e) { return e ^ ((b >> 1) & (uint32_t)(LK - 1)); };
    typename CT::C *spl = SPL_LK ? reinterpret_cast<typename CT::C *>(lk) : spl_own;
    const typename CT::C *spl_look = SPL_LK ? spl_g : spl;  // (global: only BP entries, searched within a slot)
    const int tb = threadIdx.x, lane = tb & 63, w = tb >> 6;
    const uint32_t g = blockIdx.x;
    const bool owner = tb < B;  // thread b owns bucket b's line stream
    // owner state: vc = stream entries held in carry (phantoms included), ph = phantoms still in
    // front (the stream's first line not written yet), gb = global index of stream entry 0 (mod 2^32)
    uint32_t vc = 0, ph = 0, gb = 0, pure = 0;
    if (owner) {
        const uint32_t o = offs[(uint64_t)g * B + tb];
        pure = out2 && tb > 0 && tb + 1 < B && CT::key_of(spl_g[tb - 1]) == CT::key_of(spl_g[tb]);
        ph = (uint32_t)(((uintptr_t)((pure ? out2 : out) + o) / sizeof(T)) & (LK - 1));
        vc = ph;
        gb = o - ph;
        hist[tb] = 0;
    }
    // Pure buckets (one key) with out2: their keys are dropped here -- not ranked, placed or written
    // -- and the host fills their output ranges with their key (bucket_sort: fill_segments_kernel),
    // write-only.  (Through the line streams they cost the scatter as much LDS work as any key: C4
    // has 47 % of its keys in pure buckets.)  pmask: bit b = bucket b is pure, one ballot per wave.
#ifndef DSORT_DROP_PURE
#define DSORT_DROP_PURE 1
#endif
    __shared__ uint32_t pmask[BK_MAXB / 32];
    {
        const uint64_t pb = __ballot(DSORT_DROP_PURE && pure != 0);
        if (lane == 0 && 2 * w + 1 < BK_MAXB / 32) {
            pmask[2 * w] = (uint32_t)pb;
            pmask[2 * w + 1] = (uint32_t)(pb >> 32);
        }
    }
    const BkMap m = *map;
    // (the refined slot's table, BkMap.r2s: in the LDS the scatter has left)
    __shared__ uint32_t tab2s[ADP || IDS ? 1 : BK_R2];
    const uint32_t *tab2 = ADP || IDS ? nullptr : tab2s;
#ifndef DSORT_IDS_ONLY
    if (BkIds<T>::ON && (m.ids != 0) != IDS) return;  // (workgroup-uniform: the other variant's sort)
#endif
    if (!IDS) {
        load_splitters<T>(spl_g, BP, spl);
        if (!ADP && m.r2s)
            for (int i = tb; i < BK_R2; i += BK_T) tab2s[i] = bk_tab2(map)[i];
        __syncthreads();
        build_slots<T, true, BK_SLOTB, ADP>(spl, BP, m, rng);
    }
    __syncthreads();
    bool anyp = false;  // (workgroup-uniform)
#pragma unroll
    for (int i = 0; i < BK_MAXB / 32; ++i) anyp = anyp || pmask[i] != 0u;
    const auto dropped = [&](int b) { return anyp && ((pmask[b >> 5] >> (b & 31)) & 1u) != 0u; };
    const uint64_t g0 = (uint64_t)g * subs * SUB;
#ifdef DSORT_STAMPS
    uint64_t bk_acc[8] = {}, bk_t0 = __builtin_amdgcn_s_memtime();
#endif
    T nxt[KPT];
    constexpr int PW = BkIds<T>::PER_WORD;
    uint32_t nid[IDS ? KPT / PW : 1];  // (the histogram's bucket ids, PW per word)
    // the ids of the sub-tile from key s
    const auto load_ids = [&](uint64_t s) {
        if constexpr (IDS && PW == 3) {
            const uint32_t *src = ids + s / SUB * (KPT / 3) * BK_T + tb;
#pragma unroll
            for (int w = 0; w < KPT / 3; ++w) nid[w] = src[w * BK_T];
        } else if constexpr (IDS) {
#pragma unroll
            for (int w = 0; w < KPT / 2; ++w) nid[w] = ids[s / 2 + (uint64_t)tb * (KPT / 2) + w];
        }
    };
    load_sub<T, KPT>(in, g0 + tb, n, g0 + SUB, nxt);
    if constexpr (IDS) {
        if (g0 < n) load_ids(g0);
    }
#pragma unroll 1
    for (int sub = 0; sub < subs; ++sub) {
        const uint64_t s0 = g0 + (uint64_t)sub * SUB;
        if (s0 >= n) break;  // workgroup-uniform
        const bool last = sub + 1 == subs || s0 + SUB >= n;
        T key[KPT];
        uint32_t pk[KPT];  // rank | bucket << 16; ~0 past the input
        uint32_t sl[KPT];  // (the lookup's slots, or the stored buckets)
#pragma unroll
        for (int k = 0; k < KPT; ++k) key[k] = nxt[k];
        if constexpr (IDS) {
#pragma unroll
            for (int k = 0; k < KPT; ++k) sl[k] = (nid[k / PW] >> (BkIds<T>::BITS * (k % PW))) & BkIds<T>::MASK;
        } else {
            slots_at<T, KPT, ADP>(m, key, sl);
        }
        if (!last) {
            load_sub<T, KPT>(in, s0 + SUB + tb, n, s0 + 2 * SUB, nxt);
            if constexpr (IDS) load_ids(s0 + SUB);
        }
        BKST(6);  // (the sub-tile's keys in, their slots)
#ifndef DSORT_HOT_SCATTER
#define DSORT_HOT_SCATTER 1
#endif
#ifndef DSORT_SCATTER_CB
#define DSORT_SCATTER_CB 4  // keys per batch of the whole-sub-tile classify (int32, fixed map)
#endif

        if (DSORT_HOT_SCATTER && m.hot) {  // (runs of one bucket: aggregated ranks, bucket_runs_hint)
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint64_t i = s0 + tb + (uint64_t)k * BK_T;
                const bool act = i < n;
                const int b = IDS ? (int)sl[k] : bucket_fast<T, true, true, ADP>(spl_look, rng, sl[k], key[k], CT::make(key[k], i + ioff), tab2, &m);
                const bool a = act && !dropped(b);
                const uint32_t r = bucket_bump<true>(hist, b, a);
                pk[k] = a ? r | (uint32_t)b << 16 : ~0u;
            }
        } else {
          bool batched = false;
          if constexpr (!ADP && !IDS && DSORT_SCATTER_CB > 0) {
           if (s0 + SUB <= n) {
            batched = true;
            // (int32 on the fixed map, a whole sub-tile: no per-key bounds.)  The table reads of CB
            // keys are issued together, then their rank atomics: one LDS round trip per batch and
            // kind instead of two per key (the per-key form waited for each read and each atomic
            // before the next key's, with the key's bounds check as a branch around it).  The rare
            // slow keys of a batch (crowded slot, equal to the slot's splitter) take one
            // wave-uniform branch.
            constexpr int CB = DSORT_SCATTER_CB > 0 ? DSORT_SCATTER_CB : 1;
#pragma unroll
            for (int k0 = 0; k0 < KPT; k0 += CB) {
                uint32_t r[CB];
                int b[CB];
                bool sw[CB], any = false;
#pragma unroll
                for (int g = 0; g < CB; ++g) r[g] = rng[sl[k0 + g]];
#pragma unroll
                for (int g = 0; g < CB; ++g) {
                    b[g] = packed_fast(r[g], (int32_t)key[k0 + g], sw[g]);
                    any = any || sw[g];
                }
                if (__builtin_expect(__ballot(any) != 0, 0)) {
#pragma unroll
                    for (int g = 0; g < CB; ++g)
                        if (sw[g]) {
                            const int64_t cg = (int64_t)CT::make(key[k0 + g], s0 + tb + (uint64_t)(k0 + g) * BK_T + ioff);
                            // (the refined slot, BkMap.r2s: its sub-slot entry from LDS -- a one-key sub-slot of
                            // one key value resolves without a splitter read)
                            b[g] = m.r2s && packed_refined(r[g])
                                       ? refine_pick<int32_t>(reinterpret_cast<const int64_t *>(spl_look),
                                                              tab2[refine_sub(m.r2lo, m.r2sh, (int32_t)key[k0 + g])],
                                                              (int32_t)key[k0 + g], cg)
                                       : packed_slow(reinterpret_cast<const int64_t *>(spl_look), r[g], (int32_t)key[k0 + g], cg);
                        }
                }
                if (anyp) {
#pragma unroll
                    for (int g = 0; g < CB; ++g)
                        pk[k0 + g] = dropped(b[g]) ? ~0u : atomicAdd(&hist[b[g]], 1u) | (uint32_t)b[g] << 16;
                } else {
#pragma unroll
                    for (int g = 0; g < CB; ++g) pk[k0 + g] = atomicAdd(&hist[b[g]], 1u) | (uint32_t)b[g] << 16;
                }
            }
           }
          }
          if (!batched) {
#pragma unroll
            for (int k = 0; k < KPT; ++k) {
                const uint64_t i = s0 + tb + (uint64_t)k * BK_T;
                pk[k] = ~0u;
                if (i < n) {
                    const int b = IDS ? (int)sl[k] : bucket_fast<T, true, true, ADP>(spl_look, rng, sl[k], key[k], CT::make(key[k], i + ioff), tab2, &m);
                    if (!dropped(b)) pk[k] = atomicAdd(&hist[b], 1u) | (uint32_t)b << 16;
                }
            }
          }
        }
        BKST(7);  // (classify + rank)
        __syncthreads();  // A
        BKST(0);
        // owner: new keys, whole lines to write, entries carried to the next sub-tile
        const uint32_t hv = owner ? hist[tb] : 0;
        const uint32_t L = vc + hv;  // stream entries not yet written
        const uint32_t nl = !owner ? 0 : last ? (L > ph ? (L + LK - 1) / LK : 0) : L / LK;
        const uint32_t pv = hv | nl << 16;
        const uint32_t incl = wave_incl_sum(pv);
        if (lane == 63) wsum[w] = incl;
        __syncthreads();  // B
        BKST(1);
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
            if (!HT || nl <= 8)
                for (uint32_t i = 0; i < nl; ++i) lmap[p0 + i] = (uint16_t)tb;
        }
        if constexpr (HT) {
            // sorted or reversed input puts a sub-tile's keys in one or two buckets, up to SUB / LK
            // lines of one stream: its owner's whole wave enters them in the line map (the owner
            // thread alone: 2^30 sorted int32 scatter 3.3 ms; in every instance, the code cost the
            // uniform scatter 0.22 ms -- profiles/r5_ab_lmap_wave.log)
            uint64_t big = __ballot(nl > 8);
            while (big) {
                const int l = __ffsll((long long)big) - 1;
                big &= big - 1;
                const uint32_t bp0 = __shfl(p0, l), bnl = __shfl(nl, l);
                for (uint32_t i = (uint32_t)lane; i < bnl; i += 64) lmap[bp0 + i] = (uint16_t)(64 * w + l);
            }
        }
        __syncthreads();  // C
        BKST(2);
#pragma unroll
        for (int k = 0; k < KPT; ++k)
            if (pk[k] != ~0u) lk[hist[pk[k] >> 16] + (pk[k] & 0xFFFF)] = key[k];
        __syncthreads();  // D
        BKST(3);
        if (owner) hist[tb] = 0;  // (the next sub-tile's atomics follow barrier E)
        // whole lines: 4 lanes per line, 16 bytes per lane
        for (uint32_t it = tb; it < 4 * C; it += BK_T) {
            const uint32_t j = it >> 2, q = it & 3;
            const uint32_t b = lmap[j];
            const uint2 sb = st[b];
            const uint32_t cv = sb.y & 31, cp = (sb.y >> 5) & 31, cL = sb.y >> 11, lb = sb.x & 0xFFFF;
            const uint32_t e0 = (j - (sb.x >> 16)) * LK + KPL * q;
            T v[KPL];
            bool ok[KPL];
            bool full = true;
#pragma unroll
            for (int t = 0; t < KPL; ++t) {
                const uint32_t e = e0 + t;
                ok[t] = e >= cp && e < cL;
                full = full && ok[t];
                v[t] = e < cv ? carry[b * LK + cswz(b, e)] : lk[lb + e - cv];
            }
            const uint32_t gi = sgb[b] + e0;  // mod 2^32
            T *tgt = (sb.y >> 10) & 1 ? out2 : out;
            if (full) {
                if constexpr (((DSORT_LINES_NT >> (sizeof(T) == 8 ? 1 : 0)) & 1) && !HT) {
                    using NV = typename std::conditional<sizeof(T) == 4, bk_v4i, bk_v2l>::type;
                    NV vv;
                    __builtin_memcpy(&vv, v, sizeof(NV));
                    __builtin_nontemporal_store(vv, reinterpret_cast<NV *>(tgt + gi));
                } else {
                    V vv;
                    __builtin_memcpy(&vv, v, sizeof(V));
                    *reinterpret_cast<V *>(tgt + gi) = vv;
                }
            } else {
#pragma unroll
                for (int t = 0; t < KPL; ++t)
                    if (ok[t]) tgt[(uint32_t)(gi + t)] = v[t];
            }
        }
        if (last) break;
        __syncthreads();  // E
        BKST(4);
        // carry the tail of every stream: entries [LK nl, L) -> carry[0, L - LK nl) (the entries
        // below vc of a stream that wrote no line are there already)
        if (owner) {
            const uint32_t nv = L - nl * LK;
            for (uint32_t e2 = nl ? 0 : vc; e2 < nv; ++e2) carry[tb * LK + cswz((uint32_t)tb, e2)] = lk[lks + nl * LK + e2 - vc];
            if (nl) ph = 0;
            gb += nl * LK;
            vc = nv;
        }
        BKST(5);
    }
#ifdef DSORT_STAMPS
    BKST(4);
    if (tb == 0 && g < 8192)
        for (int k = 0; k < 8; ++k) g_bkstamps[g * 16 + k] = bk_acc[k];
#endif
}
#undef BKST

}  // namespace bk
}  // namespace dsort
