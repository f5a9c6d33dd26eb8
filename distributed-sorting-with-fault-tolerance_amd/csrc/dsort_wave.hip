// dsort_wave.hip -- the sort and the k-way merge on wave-wide register bitonic networks (gfx950),
// for 32-bit and 64-bit keys.
//
// Replaces merge_sort()/merge() (reference client.c:140-173) and the merge loop of
// merge_chunks() (server.c:481-515).  Result: the input multiset in ascending signed order.
// Machine mapping:
//
//   * A wave holds 1024 keys, 16 per lane.  Every merge step of the sort is a bitonic network
//     executed in registers: compare-exchanges between registers of one lane, cross-lane ones
//     through DPP (quad_perm, row_ror, row_shl/shr, row_mirror) -- for int32 with v_med3_i32 and a
//     per-lane +-inf constant (one instruction gives the min to the lower lane and the max to the
//     upper), for int64 a 64-bit compare and a select by lane side -- and the two row-crossing
//     bits by v_permlane16/32_swap transpositions.  No per-lane merge-path search and no
//     data-dependent LDS addressing: LDS is only read and written with consecutive lanes on
//     consecutive words.
//   * block_sort_w_kernel: one workgroup (WAVES waves) sorts a TILE of WAVES * 1024 keys: each
//     wave sorts its 1024 keys in registers (Batcher network per lane, then bitonic merges of
//     32..1024), then log2(WAVES) LDS levels merge runs of 1024 -> TILE.
//   * mergew_kernel: one workgroup merges one output tile of a k-way pass: the F input windows
//     (cut by partk_kernel, dsort_part.h) are staged back to back in LDS and merged in log2(F)
//     pairwise levels.
//   * An LDS level cuts every pair of runs into windows of 1024 outputs.  The B run of a pair is
//     kept descending in LDS (every level writes the groups that become B runs reversed), so
//     after one 64-ary merge-path search for the window start (64 probes per step, ballot) the
//     window is min(A[a0 + e], B[b0 + 1023 - e]) -- two ascending LDS reads and a min per key,
//     a bitonic sequence -- sorted by the 10-stage half-cleaner network.  Windows are held in
//     registers across a barrier, so the level merges in place in one LDS buffer.
//   Key types: int32 tiles of 8 waves (8192 keys, 32 KiB LDS, four workgroups per CU; 16 waves and
//   16384 keys for buckets above 2M keys), merge tiles of 16 waves; int64 tiles of 8 waves (8192
//   keys, 64 KiB).
//
// Algorithmic HBM traffic: 2 * sizeof(key) bytes per key for the tile sort and for every pass.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>
#include <climits>
#include <ctime>
#include <sched.h>
#include <unistd.h>
#include <csignal>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "dsort_bucket.h"
#include "dsort_internal.h"

#include <rocprofiler-sdk-roctx/roctx.h>
#include "dsort_part.h"
#include "dsort_sub.h"

namespace dsort {
namespace wv {

constexpr int R = 16;              // keys per lane
constexpr int WK = 64 * R;         // keys per wave: one bitonic window
constexpr int kWaveMaxLogF = 5;    // fan-in cap of one merge pass
constexpr int kWaveMaxF = 1 << kWaveMaxLogF;

// Per key type: waves of the tile sort and of the merge tile, and the occupancy they are
// compiled for (waves per SIMD).
template <typename T> struct WG;
// int32 tile sort: 8192-key tiles of 512 threads, four workgroups per CU (40 KiB of LDS each):
// while one workgroup gathers its tile another sorts (16384-key tiles, two per CU: bin sort 2.47
// -> 2.05 ms at 2^30; round 4).
#ifndef DSORT_I32_WAVES
#define DSORT_I32_WAVES 8
#endif
template <> struct WG<int32_t> {
    static constexpr int WAVES = DSORT_I32_WAVES, MWAVES = 16, OCC = 8, MAXLOGF = 5;
};
template <> struct WG<int64_t> {
    // F = 32 would need 32 run heads of 64-bit keys per lane next to the window: it spills, so
    // int64 passes stop at F = 16.
    static constexpr int WAVES = 8, MWAVES = 8, OCC = 4, MAXLOGF = 4;
};
template <typename T> constexpr int TILE_OF = WK * WG<T>::WAVES;
// The tile sort's kernels also come with W waves (W = 16: 16384-key int32 tiles, for buckets above
// 2M keys, whose sub-buckets would come too close to an 8192-key tile; sub_sort picks).
template <int W> constexpr int TILE_W = WK * W;
template <typename T> constexpr int MTILE_OF = WK * WG<T>::MWAVES;
template <typename T> constexpr int MSLACK_OF = MTILE_OF<T> / 32;      // cut tolerance of partk
template <typename T> constexpr int MTNOM_OF = MTILE_OF<T> - 2 * MSLACK_OF<T>;
template <typename T> constexpr int KPC = 16 / (int)sizeof(T);         // keys per 16-byte chunk
template <typename T> constexpr int LKPC = sizeof(T) == 4 ? 2 : 1;

// DPP controls (gfx9 encoding)
constexpr int QP_1032 = 0xB1;      // lane ^ 1
constexpr int QP_2301 = 0x4E;      // lane ^ 2
constexpr int QP_3210 = 0x1B;      // lane ^ 3
constexpr int ROW_ROR8 = 0x128;    // lane ^ 8
constexpr int ROW_MIRROR = 0x140;  // lane ^ 15
constexpr int ROW_HMIRROR = 0x141; // lane ^ 7

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Workgroup -> work item such that XCD x (workgroups bid with bid % 8 == x, the hardware's
// round-robin) takes the contiguous block of items x * (G / 8) + ... : a bijection on [0, G).
__device__ __forceinline__ uint32_t xcd_block(uint32_t bid, uint32_t G) {
    constexpr uint32_t NX = 8;
    const uint32_t q = G / NX, r = G % NX, x = bid % NX, i = bid / NX;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

#ifdef DSORT_STAMPS
// Diagnostic build only: per-workgroup phase timestamps of mergew (s_memtime), read back by
// dsort_debug_stamps().  Stamp k of workgroup b at g_stamps[b * 32 + k] (wave 0, lane 0) and the
// wave-15 view at +16.
constexpr int kStampTiles = 1 << 17;
__device__ unsigned long long g_stamps[kStampTiles * 32];
#define STAMP(k)                                                                              \
    do {                                                                                      \
        if ((threadIdx.x & 63) == 0 && (threadIdx.x >> 6) % 15 == 0 && blockIdx.x < kStampTiles) \
            g_stamps[blockIdx.x * 32 + (threadIdx.x >> 6 ? 16 : 0) + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define RSTAMP(slot)                                                                          \
    do {                                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < kStampTiles)                                     \
            g_stamps[blockIdx.x * 32 + (slot)] = __builtin_amdgcn_s_memrealtime();            \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#define RSTAMP(slot) \
    do {             \
    } while (0)
#endif

// ------------------------------------------------------------------------------------------
// Key-type primitives.  `side` values are per-lane +-inf of the key type: -inf on lanes that
// keep the min of a cross-lane compare-exchange, +inf on lanes that keep the max.
// ------------------------------------------------------------------------------------------
// median of three: with c = -inf it is min(a, b), with c = +inf max(a, b)
__device__ __forceinline__ int med3(int a, int b, int c) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ int sel_side(int x, int p, int c) { return med3(x, p, c); }
// int64 has no med3: the partner p is taken when it is below x on a min lane, above on a max
// lane (either when equal)
__device__ __forceinline__ int64_t sel_side(int64_t x, int64_t p, int64_t c) {
    return ((c < 0) == (p < x)) ? p : x;
}

template <int CTRL>
__device__ __forceinline__ int dpp(int x) {
    return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ void split64(int64_t v, int &lo, int &hi) {
    lo = (int)v;
    hi = (int)(v >> 32);
}
__device__ __forceinline__ int64_t join64(int lo, int hi) {
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int CTRL>
__device__ __forceinline__ int64_t dpp(int64_t x) {
    int lo, hi;
    split64(x, lo, hi);
    return join64(dpp<CTRL>(lo), dpp<CTRL>(hi));
}

// partner of lane ^ 4 within a row: banks 0,2 read the lane 4 above (row_shl:4), banks 1,3 the
// lane 4 below (row_shr:4)
__device__ __forceinline__ int xor4_partner(int x) {
    int y;
    asm volatile(
        "s_nop 1\n\t"
        "v_mov_b32_dpp %0, %1 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
        "v_mov_b32_dpp %0, %1 row_shr:4 row_mask:0xf bank_mask:0xa"
        : "=&v"(y)
        : "v"(x));
    return y;
}

// compare-exchange with lane ^ 4: lanes in banks 0,2 (bit 2 clear) keep the min, banks 1,3 the
// max; for int32 the DPP source of each half is the other half (row_shl:4 / row_shr:4) and the
// min/max is fused into the DPP instruction
__device__ __forceinline__ int cex_xor4(int x, int) {
    int y;
    asm volatile(
        "s_nop 1\n\t"
        "v_min_i32_dpp %0, %1, %1 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
        "v_max_i32_dpp %0, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xa"
        : "=&v"(y)
        : "v"(x));
    return y;
}
__device__ __forceinline__ int64_t cex_xor4(int64_t x, int64_t c2) {
    int lo, hi;
    split64(x, lo, hi);
    return sel_side(x, join64(xor4_partner(lo), xor4_partner(hi)), c2);
}

template <typename T>
__device__ __forceinline__ void cex(T &a, T &b) {
    const T lo = a < b ? a : b;
    const T hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// +inf on lanes whose bit b is set (they keep the max of a compare-exchange), -inf elsewhere
template <typename T>
__device__ __forceinline__ T lane_side(int b) { return ((lane_id() >> b) & 1) ? key_max<T>() : key_min<T>(); }

__device__ __forceinline__ void swap32(int &a, int &b) {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)a, (unsigned)b, false, false);
    a = (int)r[0];
    b = (int)r[1];
}
__device__ __forceinline__ void swap16(int &a, int &b) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)a, (unsigned)b, false, false);
    a = (int)r[0];
    b = (int)r[1];
}
__device__ __forceinline__ void swap32(int64_t &a, int64_t &b) {
    int al, ah, bl, bh;
    split64(a, al, ah);
    split64(b, bl, bh);
    swap32(al, bl);
    swap32(ah, bh);
    a = join64(al, ah);
    b = join64(bl, bh);
}
__device__ __forceinline__ void swap16(int64_t &a, int64_t &b) {
    int al, ah, bl, bh;
    split64(a, al, ah);
    split64(b, bl, bh);
    swap16(al, bl);
    swap16(ah, bh);
    a = join64(al, ah);
    b = join64(bl, bh);
}

// ------------------------------------------------------------------------------------------
// Half-cleaner network on a reg-major window: x[i] at lane t is element e = 64 i + t of a
// bitonic sequence of 1024 keys; afterwards the sequence is ascending, element
// out_elem(i, t) in x[i] at lane t (bits 5 and 4 are moved between lanes and registers by the
// permlane transpositions).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ constexpr int out_hi(int i) {
    return ((i >> 3) & 1) << 9 | ((i >> 2) & 1) << 8 | (i & 1) << 5 | ((i >> 1) & 1) << 4;
}
__device__ __forceinline__ int out_lo(int t) {
    return ((t >> 4) & 1) << 7 | ((t >> 5) & 1) << 6 | (t & 15);
}

template <typename T>
__device__ __forceinline__ void merge_net(T (&x)[R], T c0, T c1, T c2, T c3) {
#pragma unroll
    for (int b = 3; b >= 0; --b) {  // element bits 9..6 = register bits 3..0
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (!(i & (1 << b))) cex(x[i], x[i | (1 << b)]);
    }
#pragma unroll
    for (int k = 0; k < R; k += 2) {  // element bit 5: lane bit 5 <-> register bit 0
        swap32(x[k], x[k + 1]);
        cex(x[k], x[k + 1]);
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {  // element bit 4: lane bit 4 <-> register bit 1
        if (k & 2) continue;
        swap16(x[k], x[k + 2]);
        cex(x[k], x[k + 2]);
    }
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = sel_side(x[i], dpp<ROW_ROR8>(x[i]), c3);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = cex_xor4(x[i], c2);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = sel_side(x[i], dpp<QP_2301>(x[i]), c1);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = sel_side(x[i], dpp<QP_1032>(x[i]), c0);
}

// ------------------------------------------------------------------------------------------
// Sort of one wave's 1024 keys in registers, lane-major: x[i] at lane t is element 16 t + i.
// ------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void sort16(T (&v)[R]) {  // Batcher odd-even merge sort, 63 cex
#pragma unroll
    for (int p = 1; p < R; p <<= 1) {
#pragma unroll
        for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
            for (int j = k % p; j + k < R; j += 2 * k) {
#pragma unroll
                for (int i = 0; i < k; ++i) {
                    if (i + j + k < R && (i + j) / (2 * p) == (i + j + k) / (2 * p))
                        cex(v[i + j], v[i + j + k]);
                }
            }
        }
    }
}

// Batcher odd-even merge sort of K keys in registers (K a power of two).
template <int K, typename T>
__device__ __forceinline__ void sort_net(T (&v)[K]) {
#pragma unroll
    for (int p = 1; p < K; p <<= 1) {
#pragma unroll
        for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
            for (int j = k % p; j + k < K; j += 2 * k) {
#pragma unroll
                for (int i = 0; i < k; ++i) {
                    if (i + j + k < K && (i + j) / (2 * p) == (i + j + k) / (2 * p)) cex(v[i + j], v[i + j + k]);
                }
            }
        }
    }
}

// Half-cleaner on element bit b of a lane-major wave (b <= 8).
template <int B, typename T>
__device__ __forceinline__ void hc_lane_major(T (&x)[R], const T (&c)[6]) {
    if constexpr (B <= 3) {
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (!(i & (1 << B))) cex(x[i], x[i | (1 << B)]);
    } else if constexpr (B == 4) {
#pragma unroll
        for (int i = 0; i < R; ++i) x[i] = sel_side(x[i], dpp<QP_1032>(x[i]), c[0]);
    } else if constexpr (B == 5) {
#pragma unroll
        for (int i = 0; i < R; ++i) x[i] = sel_side(x[i], dpp<QP_2301>(x[i]), c[1]);
    } else if constexpr (B == 6) {
#pragma unroll
        for (int i = 0; i < R; ++i) x[i] = cex_xor4(x[i], c[2]);
    } else if constexpr (B == 7) {
#pragma unroll
        for (int i = 0; i < R; ++i) x[i] = sel_side(x[i], dpp<ROW_ROR8>(x[i]), c[3]);
    } else {  // B == 8: lane bit 4, through a permlane16 transposition with register bit 0
        static_assert(B == 8, "half-cleaner bit out of range");
#pragma unroll
        for (int k = 0; k < R; k += 2) {
            swap16(x[k], x[k + 1]);
            cex(x[k], x[k + 1]);
            swap16(x[k], x[k + 1]);
        }
    }
}

// Partner of the mirror stage of a merge of 2^M keys: lane t ^ (2^(M-4) - 1).
template <int M, typename T>
__device__ __forceinline__ T mirror_partner(T v) {
    if constexpr (M == 5) return dpp<QP_1032>(v);
    else if constexpr (M == 6) return dpp<QP_3210>(v);
    else if constexpr (M == 7) return dpp<ROW_HMIRROR>(v);
    else if constexpr (M == 8) return dpp<ROW_MIRROR>(v);
    else if constexpr (M == 9) return __shfl_xor(v, 31);
    else return __shfl_xor(v, 63);
}

template <int B, int M, typename T>
__device__ __forceinline__ void hc_down(T (&x)[R], const T (&c)[6]) {
    hc_lane_major<B>(x, c);
    if constexpr (B > 0) hc_down<B - 1, M>(x, c);
}

// Merge of sorted (ascending) blocks of 2^(M-1) keys into blocks of 2^M: the first stage
// compares element e with its mirror e ^ (2^M - 1), then half-cleaners on bits M-2 .. 0.
template <int M, typename T>
__device__ __forceinline__ void merge_lane_major(T (&x)[R], const T (&c)[6]) {
    T y[R];
#pragma unroll
    for (int i = 0; i < R; ++i) y[i] = sel_side(x[i], mirror_partner<M>(x[R - 1 - i]), c[M - 5]);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = y[i];
    hc_down<M - 2, M>(x, c);
}

template <typename T>
__device__ __forceinline__ void sort_wave(T (&x)[R], const T (&c)[6]) {
    sort16(x);
    merge_lane_major<5>(x, c);
    merge_lane_major<6>(x, c);
    merge_lane_major<7>(x, c);
    merge_lane_major<8>(x, c);
    merge_lane_major<9>(x, c);
    merge_lane_major<10>(x, c);
}

// ------------------------------------------------------------------------------------------
// LDS levels
// ------------------------------------------------------------------------------------------
// ---- Windows over a pair whose B run is stored DESCENDING in LDS -------------------------
// Pair = A ascending at s[pa, pa+na) followed by B descending (B[k] at s[pbe - k], pbe = pa + na
// + nb - 1).  For a window starting at output d0 with merge-path split (a0, b0 = d0 - a0), the
// 1024 smallest keys of A[a0..] u B[b0..] are min(A[a0 + e], B[b0 + 1023 - e]), e < 1024, and in
// that order they form a bitonic sequence.  Both operands are ascending LDS ranges
// (s[pa + a0 + e] and s[pbe - b0 - 1023 + e]); when at least 1024 outputs remain from d0 a read
// past either run lands on the other run's larger keys of the same pair and never wins the min
// (DESIGN.md §3.1), so a full window needs one split search, 32 reads and 16 min.

// Number of A keys among the first d outputs of merge(A, B) (one 64-ary search, wave-uniform).
template <typename T>
__device__ __forceinline__ int coop_split_desc(const T *s, int pa, int na, int pbe, int nb, int d) {
    int lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    const int lane = lane_id();
#pragma unroll 1
    while (lo < hi) {
        const int len = hi - lo;
        const int st = ((len + 63) >> 6) | 1;
        const int off = (int)__umul24((unsigned)lane, (unsigned)st);
        const int ia = pa + lo + off;                  // <= TILE + WK - 1 (slack slots)
        int ib = pbe - d + 1 + lo + off;               // B[d - 1 - lo - off]
        ib = ib > pbe ? pbe : ib;                      // probes past the bracket: in bounds
        const bool q = (off >= len) | (s[ia] > s[ib]);
        const unsigned long long m = __ballot(q);
        const int j = m ? (int)__ffsll((long long)m) - 1 : 64;
        const int nhi = lo + j * st < hi ? lo + j * st : hi;
        lo = __builtin_amdgcn_readfirstlane(j ? lo + (j - 1) * st + 1 : lo);
        hi = __builtin_amdgcn_readfirstlane(nhi);
    }
    return lo;
}

// Full window: x[i] at lane t = min(s[ia0 + e], s[ib0 + e]), e = 64 i + t.
template <typename T>
__device__ __forceinline__ void load_min(const T *s, int ia0, int ib0, T (&x)[R]) {
    const int t = lane_id();
    const T *sa = s + ia0 + t;
    const T *sb = s + ib0 + t;
#pragma unroll
    for (int hlf = 0; hlf < 2; ++hlf) {
        T vb[R / 2];
#pragma unroll
        for (int k = 0; k < R / 2; ++k) {
            const int i = hlf * (R / 2) + k;
            x[i] = sa[64 * i];
            vb[k] = sb[64 * i];
        }
#pragma unroll
        for (int k = 0; k < R / 2; ++k) {
            const int i = hlf * (R / 2) + k;
            x[i] = x[i] < vb[k] ? x[i] : vb[k];
        }
    }
}

// Pair of fewer than 1024 keys (one window, d0 = 0): A[e] for e < na, B[1023 - e] for
// e >= 1024 - nb, +inf elsewhere.
template <typename T>
__device__ __forceinline__ void load_min_short(const T *s, int pa, int na, int pbe, int nb,
                                               T (&x)[R]) {
    const int t = lane_id();
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int e = 64 * i + t;
        int ib = pbe - 1023 + e;
        ib = ib < 0 ? 0 : ib;
        const T va = e < na ? s[pa + e] : key_max<T>();
        const T vb = e >= WK - nb ? s[ib] : key_max<T>();
        x[i] = va < vb ? va : vb;
    }
}

// A window of a pair with B descending: outputs [d0 + skip, d0 + skip + cnt) of the pair's merge
// are kept (skip > 0 only for the last window of a pair, shifted back to end at the pair's end).
struct WinD {
    int pa, na, nb, d0, skip, cnt, desc;
};

template <typename T>
__device__ __forceinline__ void merge_window_desc(const T *s, const WinD &w, T (&x)[R], T c0,
                                                  T c1, T c2, T c3) {
    const int pbe = w.pa + w.na + w.nb - 1;
    if (w.na + w.nb >= WK) {
        const int a0 = coop_split_desc(s, w.pa, w.na, pbe, w.nb, w.d0);
        load_min(s, w.pa + a0, pbe - (w.d0 - a0) - (WK - 1), x);
    } else {
        load_min_short(s, w.pa, w.na, pbe, w.nb, x);
    }
    merge_net(x, c0, c1, c2, c3);
}

// Stores the kept outputs of a window: pair output position d lands at dst[ob + d] (ascending
// group) or dst[ob + len - 1 - d] (descending group; LDS only: the last level is ascending).
template <bool DESC, typename T>
__device__ __forceinline__ void store_window_desc(T *dst, const WinD &w, int ob, int lo,
                                                  const T (&x)[R]) {
    const bool part = w.skip != 0 || w.cnt != WK;
    if (!DESC || !w.desc) {
        T *p = dst + ob + w.d0 + lo;
        if (!part) {
#pragma unroll
            for (int i = 0; i < R; ++i) p[out_hi(i)] = x[i];
        } else {
#pragma unroll
            for (int i = 0; i < R; ++i)
                if ((unsigned)(out_hi(i) + lo - w.skip) < (unsigned)w.cnt) p[out_hi(i)] = x[i];
        }
    } else {
        T *p = dst + ob + (w.na + w.nb - 1 - w.d0) - lo;
        if (!part) {
#pragma unroll
            for (int i = 0; i < R; ++i) p[-out_hi(i)] = x[i];
        } else {
#pragma unroll
            for (int i = 0; i < R; ++i)
                if ((unsigned)(out_hi(i) + lo - w.skip) < (unsigned)w.cnt) p[-out_hi(i)] = x[i];
        }
    }
}

// 16-byte vector of keys
template <typename T> struct V16;
template <> struct V16<int32_t> {
    using type = int4;
    __device__ static void get(const int4 &v, int32_t *o) { o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w; }
    __device__ static int4 make(const int32_t *o) { return make_int4(o[0], o[1], o[2], o[3]); }
};
template <> struct V16<int64_t> {
    using type = longlong2;
    __device__ static void get(const longlong2 &v, int64_t *o) { o[0] = v.x; o[1] = v.y; }
    __device__ static longlong2 make(const int64_t *o) { return make_longlong2(o[0], o[1]); }
};

// ------------------------------------------------------------------------------------------
// Bin sort of a tile.  After the two partition levels a tile covers a narrow key range that its
// keys fill about evenly (they are a contiguous run of sampled sub-buckets), so binning them by
// (key - min) over the tile's range into TILE/2 bins leaves about 2 keys per bin: a counting pass
// into LDS (counts, then cursors) groups the keys by bin, and 16-key window networks (one window
// per thread, in registers) sort inside the bins: a sort at offset 0 and a merge of the sorted
// halves at offset 8, a second merge at offset 0 only when a bin of more than 9 keys left a
// descent.  About 45 compare-exchange operations per key instead of the ~180 of the bitonic tile
// sort.  Details and the fallback: bin_sort_tile.

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const T y = __shfl_xor(v, o);
        v = y < v ? y : v;
    }
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const T y = __shfl_xor(v, o);
        v = y > v ? y : v;
    }
    return v;
}

// Bins per tile: two keys per bin on average.  The counters (16-bit, two per word) and the tile
// fill exactly 80 KiB of LDS for int32 (64 + 16), so two workgroups share a CU.
template <int W> constexpr int BIN_NB = TILE_W<W> / 2;

// Per-wave scratch of the bin sort; it lives at the start of the tile array s, which is free
// until the keys are placed (step 4).
template <typename T, int W>
struct BinSm {
    T mn[W], mx[W];
    uint32_t wsum[W];
    uint32_t flag[W];
};

// __syncthreads_or with the caller's scratch (one word per wave): HIP's own reserves 256 bytes of
// LDS of its own, which would leave the int32 bin sort 256 bytes short of two workgroups per CU.
template <int WAVES>
__device__ __forceinline__ bool block_or(bool p, uint32_t *flag) {
    const bool any = __ballot(p) != 0;
    if ((threadIdx.x & 63) == 0) flag[threadIdx.x >> 6] = any;
    __syncthreads();
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < WAVES; ++i) r |= flag[i];
    return r != 0;
}

// Bin of key offset `off` (key - min): the top 32 bits of the offset times a 32-bit reciprocal
// of the range, so all NB bins are used (monotone in the key, < NB).
template <typename T>
struct BinMap {
    using U = typename sb::KeyU<T>::U;
    uint32_t pre;    // offsets are shifted right by pre first (int64 ranges above 2^32)
    uint32_t scale;  // <= NB * 2^32 / ((range >> pre) + 1), capped at 2^32 - 1
    __device__ __forceinline__ uint32_t operator()(U off) const {
        return __umulhi((uint32_t)(off >> pre), scale);
    }
};

// The keys of one register slot into the bins.  HOT: the lanes whose bin is the first active
// lane's add with one atomic (a duplicate run puts a whole wave into one bin).  SCATTER: the
// atomic returns the bin's cursor and the key goes to s there; else it only counts.
// Physical LDS slot of tile position p in the bin sort.  A window of 16 keys (one thread's) is
// sizeof(T) 16-byte chunks; unswizzled, the lanes of one ds_read_b128 / ds_write_b128 group read
// windows 64 (int32) or 128 (int64) bytes apart, i.e. the same banks 4 or 8 times over.  The
// chunks of a window are XOR-rotated by the window's index above its bank row, so those lanes hit
// distinct banks; the rotation stays inside the window (a bijection on [0, TILE)).
template <typename T>
__device__ __forceinline__ uint32_t bsw(uint32_t p) {
    constexpr int CW = (int)sizeof(T);          // chunks per window: 4 (int32), 8 (int64)
    constexpr int LK = sizeof(T) == 4 ? 2 : 1;  // log2 keys per chunk
    constexpr int A = sizeof(T) == 4 ? 6 : 5;   // log2 keys per bank row of windows (256 B) + 4
    return p ^ (((p >> A) & (CW - 1)) << LK);
}

// Counting (SCATTER = false) or placing (the atomic returns the bin's cursor and the key goes to
// s there) of one key.  hot (a duplicate run): the lanes whose bin is the first active lane's add
// with one aggregated atomic.  (The batched int64 plain path is bin_count / bin_place.)
template <bool SCATTER, typename T>
__device__ __forceinline__ void bin_put(T xv, T mn, const BinMap<T> &bm, uint32_t *hw, T *s, int lane,
                                            bool hot) {
    using U = typename sb::KeyU<T>::U;
    const bool act = xv != key_max<T>();
    const uint32_t b = bm((U)xv - (U)mn);
    const uint32_t inc = (b & 1) ? 0x10000u : 1u;
    if (!hot) {  // (the plain path one key at a time: int32)
        if (act) {
            if constexpr (SCATTER) {
                const uint32_t old = atomicAdd(&hw[b >> 1], inc);
                s[bsw<T>((b & 1) ? old >> 16 : old & 0xFFFFu)] = xv;
            } else {
                atomicAdd(&hw[b >> 1], inc);
            }
        }
        return;
    }
    const uint64_t am = __ballot(act);
    if (!am) return;
    const int first = (int)__ffsll((long long)am) - 1;
    const uint32_t b0 = (uint32_t)__shfl((int)b, first);
    const uint64_t same = __ballot(act && b == b0);
    const uint32_t inc0 = ((b0 & 1) ? 0x10000u : 1u) * (uint32_t)__popcll(same);
    if constexpr (SCATTER) {
        uint32_t pos = 0;
        if (act && b != b0) {
            const uint32_t old = atomicAdd(&hw[b >> 1], inc);
            pos = (b & 1) ? old >> 16 : old & 0xFFFFu;
        }
        uint32_t old0 = 0;
        if (lane == first) old0 = atomicAdd(&hw[b0 >> 1], inc0);
        old0 = (uint32_t)__shfl((int)old0, first);
        if (act && b == b0)
            pos = ((b0 & 1) ? old0 >> 16 : old0 & 0xFFFFu) + (uint32_t)__popcll(same & ((1ull << lane) - 1));
        if (act) s[bsw<T>(pos)] = xv;
    } else {
        if (act && b != b0) atomicAdd(&hw[b >> 1], inc);
        if (lane == first) atomicAdd(&hw[b0 >> 1], inc0);
    }
}

// Batched plain path (int64): bin, counter word and half of every key, with no branch in the
// atomics -- a key that is not binned (key_max, the padding) adds 0 to the lane's own counter
// word (spread: a whole padding wave on one word would serialise) and is not stored -- and all
// of a thread's atomics issued (in batches of 8) before any result is used.  That pays at the
// int64 tile's 4 waves per SIMD (bin sort 8.46 -> 8.18 ms at 2^30 Zipf); at int32's 8 waves per
// SIMD the other waves already hide the latency and one key at a time is faster (3.26 vs 3.61 ms).
template <typename T> constexpr bool BIN_BATCH = sizeof(T) == 8;
template <typename T>
struct BinAt {
    uint32_t word, sh, inc;
    __device__ __forceinline__ BinAt(T xv, T mn, const BinMap<T> &bm) {
        using U = typename sb::KeyU<T>::U;
        const bool act = xv != key_max<T>();
        const uint32_t b = bm((U)xv - (U)mn);
        word = act ? b >> 1 : (uint32_t)(threadIdx.x & 63);
        sh = (b & 1) << 4;
        inc = act ? 1u << sh : 0u;
    }
};
template <typename T>
__device__ __forceinline__ void bin_count(const T (&x)[R], T mn, const BinMap<T> &bm, uint32_t *cw) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const BinAt<T> a(x[i], mn, bm);
        atomicAdd(&cw[a.word], a.inc);
    }
}
template <typename T>
__device__ __forceinline__ void bin_place(const T (&x)[R], T mn, const BinMap<T> &bm, uint32_t *cw, T *s) {
    constexpr int G = 8;  // atomics in flight per thread (more spill at 64 registers)
#pragma unroll
    for (int g = 0; g < R; g += G) {
        uint32_t old[G];
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const BinAt<T> a(x[g + i], mn, bm);
            old[i] = atomicAdd(&cw[a.word], a.inc);
        }
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const BinAt<T> a(x[g + i], mn, bm);
            if (a.inc) s[bsw<T>((old[i] >> a.sh) & 0xFFFFu)] = x[g + i];
        }
    }
}

// Batcher's odd-even merge of two sorted halves of K keys (the last stage of sort_net<K>).
template <int K, typename T>
__device__ __forceinline__ void merge_halves(T (&v)[K]) {
    constexpr int P = K / 2;
#pragma unroll
    for (int k = P; k >= 1; k >>= 1) {
#pragma unroll
        for (int j = k % P; j + k < K; j += 2 * k) {
#pragma unroll
            for (int i = 0; i < k; ++i)
                if (i + j + k < K) cex(v[i + j], v[i + j + k]);
        }
    }
}

// One window pass over s[0, P) (P <= TILE): thread t sorts (MERGE: merges the sorted halves of)
// the 16 keys at 16 t + OFF.  Windows of one pass are disjoint, so each is read and written in
// place.  The slots from P up to 24 past it (or the tile's end) hold key_max (bin_sort_tile), so a
// window reaching past P needs no masking: key_max sorts to its end.  A window is always moved as
// 16-byte vectors.  (Guarding the vector path with `ws + 16 <= M` let the compiler fold it into
// the scalar path: 16 ds_read2_b32 per window at a 64-byte lane stride, 16-way bank conflicts.)
// The last window at offset 8 would reach past the tile; its second half is empty, so the merge
// is a no-op and it is skipped.
template <int OFF, bool MERGE, int TILE, typename T>
__device__ __forceinline__ void window_pass(T *s, int P, int tid) {
    using V = typename V16<T>::type;
    constexpr int N = KPC<T>;
    const int ws = 16 * tid + OFF;
    if (ws >= P || ws + 16 > TILE) return;
    T v[16];
    V *p[16 / N];  // the window's 16-byte chunks (their physical slots: bsw)
#pragma unroll
    for (int q = 0; q < 16 / N; ++q) p[q] = reinterpret_cast<V *>(s + bsw<T>((uint32_t)(ws + N * q)));
#pragma unroll
    for (int q = 0; q < 16 / N; ++q) V16<T>::get(*p[q], v + N * q);
    if constexpr (MERGE) merge_halves<16>(v);
    else sort_net<16>(v);
#pragma unroll
    for (int q = 0; q < 16 / N; ++q) *p[q] = V16<T>::make(v + N * q);
}

// The tile sort's output as non-temporal stores (round 6, int32: bit 0; int64 bit 1): 2^30 int32
// 7.56 -> 7.50 ms of device time over 3 of 3 interleaved runs; 2^30 uniform int64 16.43 -> 16.21 ms
// (3 of 3), C4 neutral; the local partition's in-place write-back the same way measured neutral
// (profiles/r6_ab_nontemporal_tile_out.log, r6_ab_nontemporal_i64.log).
#ifndef DSORT_TILE_OUT_NT
#define DSORT_TILE_OUT_NT 3
#endif
// Bin sort of one tile held in x (slots past `valid` are key_max) into out[0, valid).
//   1. range [mn, mx] of the keys below key_max (they and the padding are not binned: the output
//      ends with valid - M of them, M = the binned keys);
//   2. NB = TILE / 2 bins over the range, counted by LDS atomics on 16-bit counters (a duplicate
//      run -- HOT -- with aggregated atomics);
//   3. bin starts: thread t scans its own NB / THREADS consecutive bins (one 16-byte word), then
//      the threads' totals;
//   4. keys to their bins (the starts are cursors now);
//   5. 16-key windows: sorted at 16 t, their halves merged at 16 t + 8.  That sorts every bin of
//      at most 9 keys (a bin crossing 16 t + 8 lies inside [16 t, 16 t + 16)); a descent left at
//      a boundary 16 t + 8 means a bigger bin: one more merge at 16 t sorts bins of <= 16 keys
//      (the three passes are an odd-even transposition of 8-key blocks).  A tile still unsorted
//      returns false (out untouched) and the caller runs the bitonic sort.
// About 30 operations per key on the window networks, against ~180 for the bitonic tile sort.
// cw holds the counters (NB / 2 words); the caller has passed a barrier since its last use.
template <typename T, int W>
__device__ __forceinline__ bool bin_sort_tile(const T (&x)[R], int valid, T *s, uint32_t *cw, T *out,
                                              bool hot_hint, bool known, T klo, T khi, const int tid) {
    using U = typename sb::KeyU<T>::U;
    constexpr int WAVES = W, THREADS = 64 * WAVES, NB = BIN_NB<W>, TL = TILE_W<W>;
    constexpr int BPT = NB / THREADS;
    static_assert(BPT == 8, "one 16-byte word of counters per thread");
    BinSm<T, W> &sm = *reinterpret_cast<BinSm<T, W> *>(s);
    const int lane = tid & 63, w = tid >> 6;
    // 1. range: the caller's bounds, or a reduction over the keys (which waits for all of them)
    T mn = klo, mx = khi;
    uint4 *c4 = reinterpret_cast<uint4 *>(cw) + tid;  // this thread's bins [8 tid, 8 tid + 8) (zeroed)
    if (!known) {
        mn = key_max<T>();
        mx = key_min<T>();
#pragma unroll
        for (int i = 0; i < R; ++i) {
            mn = x[i] < mn ? x[i] : mn;
            const T xm = x[i] == key_max<T>() ? key_min<T>() : x[i];
            mx = xm > mx ? xm : mx;
        }
        mn = wave_min(mn);
        mx = wave_max(mx);
        if (lane == 0) {
            sm.mn[w] = mn;
            sm.mx[w] = mx;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < WAVES; ++i) {
            mn = sm.mn[i] < mn ? sm.mn[i] : mn;
            mx = sm.mx[i] > mx ? sm.mx[i] : mx;
        }
    }
    STAMP(2);
    if (mx < mn || (mn == key_max<T>())) {  // every key is key_max
        for (int i = tid; i < valid; i += THREADS) out[i] = key_max<T>();
        return true;
    }
    // The tile's LDS slots are shifted by sh = out's misalignment within a 16-byte chunk, so LDS
    // chunk q (slots N q .. N q + N - 1) is output chunk q of out - sh, a 16-byte aligned address:
    // step 6 moves whole chunks (ds_read_b128 -> 16-byte stores).  Slots [0, sh) hold key_min.
    // A tile within 3 keys of TILE keeps sh = 0 (its shifted slots would not fit) and writes keys.
    constexpr int N = KPC<T>;
    const int sh0 = (int)((reinterpret_cast<uintptr_t>(out) / sizeof(T)) & (N - 1));
    const int sh = valid + sh0 <= TL ? sh0 : 0;
    const U range = (U)mx - (U)mn;
    BinMap<T> bm;
    bm.pre = 0;
    while ((range >> bm.pre) > (U)0xFFFFFFFFu) ++bm.pre;
    {
        // NB * 2^32 / (range' + 1) through a float reciprocal, shaded down by 2^-20 (more than its
        // error) so that the largest offset still maps below NB
        const float den = (float)(uint32_t)(range >> bm.pre) + 1.0f;
        const float f = (float)NB * 4294967296.0f * (1.0f - 0x1p-20f) * __builtin_amdgcn_rcpf(den);
        bm.scale = f >= 4294967040.0f ? 0xFFFFFFFFu : (uint32_t)f;
    }
    // a duplicate run (8 or more of a wave's first keys in one bin): aggregated atomics, decided
    // per wave (no barrier: the other keys may still be on their way)
    const bool act0 = x[0] != key_max<T>();
    const uint32_t bx = bm((U)x[0] - (U)mn);
    const uint32_t bf = (uint32_t)__builtin_amdgcn_readfirstlane((int)bx);
    const bool hot = hot_hint || __popcll(__ballot(act0 && bx == bf)) >= 8;
    // 2. counting
    if (!hot && !BIN_BATCH<T>) {  // (wave-uniform: the plain loop carries no aggregation code)
#pragma unroll
        for (int i = 0; i < R; ++i) bin_put<false>(x[i], mn, bm, cw, s, lane, false);
    } else if (hot || !BIN_BATCH<T>) {
#pragma unroll
        for (int i = 0; i < R; ++i) bin_put<false>(x[i], mn, bm, cw, s, lane, hot);
    } else {
        bin_count(x, mn, bm, cw);
    }
    __syncthreads();
    STAMP(3);
    // 3. starts
    uint4 cv = *c4;
    uint32_t wd[4] = {cv.x, cv.y, cv.z, cv.w};
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) tot += (wd[k] & 0xFFFFu) + (wd[k] >> 16);
    uint32_t incl = wave_incl_sum(tot);
    if (lane == 63) sm.wsum[w] = incl;
    __syncthreads();
    uint32_t run = incl - tot + (uint32_t)sh, M = 0;
#pragma unroll
    for (int i = 0; i < WAVES; ++i) {
        const uint32_t v = sm.wsum[i];
        run += i < w ? v : 0;
        M += v;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t c0 = wd[k] & 0xFFFFu, c1 = wd[k] >> 16;
        wd[k] = run | (run + c0) << 16;
        run += c0 + c1;
    }
    *c4 = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    __syncthreads();  // (also: sm, in s, is dead from here)
    STAMP(4);
    // Binned keys go to slots [sh, P); key_min below, key_max from P to the end of the output
    // (E) and at least 24 slots past P (the windows reaching past P read them: no masking).
    const int P = (int)M + sh, E = valid + sh;
    {
        const int F0 = E > P + 24 ? E : P + 24, F = F0 < TL ? F0 : TL;
        if (tid < sh) s[bsw<T>((uint32_t)tid)] = key_min<T>();
        for (int p = P + tid; p < F; p += THREADS) s[bsw<T>((uint32_t)p)] = key_max<T>();
    }
    // 4. keys to their places
    // (mn through an opaque copy: the bins are recomputed here, not kept in registers across
    // the scan, where they would spill)
    asm volatile("" : "+v"(mn));
    if (!hot && !BIN_BATCH<T>) {
#pragma unroll
        for (int i = 0; i < R; ++i) bin_put<true>(x[i], mn, bm, cw, s, lane, false);
    } else if (hot || !BIN_BATCH<T>) {
#pragma unroll
        for (int i = 0; i < R; ++i) bin_put<true>(x[i], mn, bm, cw, s, lane, hot);
    } else {
        bin_place(x, mn, bm, cw, s);
    }
    __syncthreads();
    STAMP(5);
    // 5. window passes; a descent can only be left at a boundary of the last pass's windows
    window_pass<0, false, TL>(s, P, tid);
    __syncthreads();
    STAMP(6);
    window_pass<8, true, TL>(s, P, tid);
    __syncthreads();
    STAMP(7);
    const int e8 = 16 * tid + 8;
    if (block_or<WAVES>(e8 < P && s[bsw<T>(e8 - 1)] > s[bsw<T>(e8)], cw)) {  // (cw is dead from step 5)
        window_pass<0, true, TL>(s, P, tid);
        __syncthreads();
        const int e16 = 16 * tid + 16;
        if (block_or<WAVES>(e16 < P && s[bsw<T>(e16 - 1)] > s[bsw<T>(e16)], cw + WAVES)) return false;
    }
    // 6. out: slots [sh, E) -- the binned keys in order, then key_max.  Chunk q of out - sh is
    // LDS chunk q; indices start at the 128-byte line below out - sh, so every wave's stores cover
    // whole lines (tiles start anywhere, and lines shared by two waves' stores came out as partial
    // writes, 14 % of the written bytes).  Round 2 moved one key per lane and instruction.
    STAMP(8);
    if (sh == sh0) {
        using V = typename V16<T>::type;
        T *ob = out - sh;  // 16-byte aligned
        const int m8 = (int)((reinterpret_cast<uintptr_t>(ob) / 16) & 7);
        const int nq = (E + N - 1) / N;
        for (int q = tid - m8; q < nq; q += THREADS) {
            if (q < 0) continue;
            const int p0 = N * q;
            const V v = *reinterpret_cast<const V *>(s + bsw<T>((uint32_t)p0));
            if (p0 >= sh && p0 + N <= E) {
                if constexpr ((DSORT_TILE_OUT_NT >> (sizeof(T) == 8 ? 1 : 0)) & 1) {
                    using NV = typename std::conditional<sizeof(T) == 4, bk::bk_v4i, bk::bk_v2l>::type;
                    NV nv;
                    __builtin_memcpy(&nv, &v, sizeof(NV));
                    __builtin_nontemporal_store(nv, reinterpret_cast<NV *>(ob + p0));
                } else {
                    *reinterpret_cast<V *>(ob + p0) = v;
                }
            } else {
                T k[N];
                V16<T>::get(v, k);
#pragma unroll
                for (int e = 0; e < N; ++e)
                    if (p0 + e >= sh && p0 + e < E) ob[p0 + e] = k[e];
            }
        }
    } else {
        constexpr int LK = 128 / (int)sizeof(T);
        const int m = (int)((reinterpret_cast<uintptr_t>(out) / sizeof(T)) & (LK - 1));
        for (int i = tid - m; i < valid; i += THREADS)
            if (i >= 0) out[i] = s[bsw<T>((uint32_t)i)];
    }
    STAMP(9);
    return true;
}

// ------------------------------------------------------------------------------------------
// 1. Tile sort.
// ------------------------------------------------------------------------------------------
// tiles: NULL = tile j is keys [j * TILE, (j + 1) * TILE) of n; else tile j = tiles[j] (the
// bucketed sort's tiles, which never cross a bucket), j < *ntiles.
// Pieces of a gathered tile at most (= chunks of a bucket on the local-partition path).
template <typename T> constexpr int kMaxPieces = WK * (int)sizeof(T) / 8 - 2;
static_assert(64 + 3 * kMaxPieces<int32_t> + 1 <= TILE_OF<int32_t> && 64 + 3 * kMaxPieces<int64_t> + 1 <= 2 * TILE_OF<int64_t>,
              "the piece table of a gathered tile fits in the tile's LDS");

// The tile of a GTile (local-partition path, dsort_sub.h): one piece per chunk of its bucket.
// Keys move as aligned 16-byte vectors (N keys): piece k is read as the vectors that cover it,
// its neighbours' keys in its first and last vector masked to key_max.  The piece table (vector
// offsets in the tile, piece bounds) goes to LDS; lane t of wave w loads the tile's vector slots
// w * WK / N + 64 i + t straight into x[N i .. N i + N) (the order before the sort does not
// matter), walking the pieces upwards as i grows: consecutive lanes read consecutive vectors of a
// piece, and all R / N loads of a lane are in flight together.  The masked keys take up to
// 2 (N - 1) slots per piece beyond `valid`: the tile packing leaves that room (sb_scan_kernel).
// (Round 2 moved one key per lane and load, walking the pieces key by key: 4x the loads and the
// address arithmetic of int32.)  `in` is 16-byte aligned (the context's scratch).
// The piece-table entries of thread t (pieces 2t, 2t + 1 of tile jt), loaded before the tile record
// is waited for.
__device__ __forceinline__ void gather_pieces(const sb::Gather &ga, uint32_t jt, uint2 (&pe)[2],
                                              const int tid = threadIdx.x) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {  // (up to the stride: the reads do not wait for the record)
        const uint32_t k = 2 * tid + q;
        pe[q] = k < ga.PS ? ga.pieces[(uint64_t)jt * ga.PS + k] : make_uint2(0u, 0u);
    }
}
// ptab: 3 kMaxPieces + 1 words of LDS for the piece table, then (DSORT_GATHER_VPC) TILE / N 16-bit
// piece indices of the vector slots; wsum: one word per wave.
#ifndef DSORT_GATHER_VPC
#define DSORT_GATHER_VPC 1
#endif
template <typename T, int W>
__device__ __forceinline__ void gather_tile(const sb::Gather &ga, const uint2 (&pe)[2], const sb::GTile &gt,
                                            const T *in, uint32_t *ptab, uint32_t *wsum, T (&x)[R],
                                            const int tid = threadIdx.x) {
    constexpr int WAVES = W, THREADS = 64 * WAVES, N = KPC<T>, KP = kMaxPieces<T>;
    using V = typename V16<T>::type;
    static_assert(2 * THREADS >= KP + 1, "two pieces per thread");
    uint32_t *voff = ptab, *plo = ptab + KP + 1, *phi = plo + KP;  // vector offsets, piece bounds
    // (the piece table, written by sb_scan_kernel, is read with the tile record: one round trip
    // before the key loads)
    const int np = (int)gt.nch;
    const int lane = tid & 63, w = tid >> 6;
    // (flags bit 0: a lone sub-bucket above the vector room, gathered key by key; nv = keys)
    const bool keyw = (gt.flags & 1) != 0;
    uint32_t nv[2], lo[2], hi[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int k = 2 * tid + q;
        nv[q] = lo[q] = hi[q] = 0;
        if (k < np) {
            lo[q] = pe[q].x;
            hi[q] = pe[q].y;
            nv[q] = lo[q] < hi[q] ? (keyw ? hi[q] - lo[q] : (hi[q] + N - 1) / N - lo[q] / N) : 0;
        }
    }
    const uint32_t sum = nv[0] + nv[1];
    uint32_t incl = wave_incl_sum(sum);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t ex = incl - sum, tot = 0;
    for (int i = 0; i < WAVES; ++i) {
        const uint32_t v = wsum[i];
        ex += i < w ? v : 0;
        tot += v;
    }
    // DSORT_GATHER_VPC (round 6): with small pieces (under 20 vectors on average: a C3 rank's tiles
    // gather 273 pieces of ~60 int32 keys) the piece of every vector slot (16-bit, behind the piece
    // table), written by the piece's thread -- a lane's loads then look their piece up with one read
    // each, independently, where the walk up the pieces (a binary search for the first, then a step
    // per piece boundary crossed, each an LDS round trip the next load's address waited for) chained
    // up to ~25 round trips in front of the last load.  C3 rank: tile sort 1.51 -> 1.38 ms; with the
    // one-GPU sort's ~30-vector pieces the fill cost more than the walk (+0.04 ms), so those walk
    // (profiles/r6_ab_gather_vpc.log).  Workgroup-uniform.
    const bool vp = DSORT_GATHER_VPC && !keyw && tot < 20u * (uint32_t)np;
    uint16_t *vpc = reinterpret_cast<uint16_t *>(phi + KP);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int k = 2 * tid + q;
        if (k < np) {
            voff[k] = ex;
            plo[k] = lo[q];
            phi[k] = hi[q];
            if (vp)
                for (uint32_t v = ex; v < ex + nv[q]; ++v) vpc[v] = (uint16_t)k;
        }
        ex += nv[q];
    }
    if (tid == 0) voff[np] = tot;
    __syncthreads();
    if (keyw) {
        // slot e = w WK + 64 i + t of key offsets; piece of the first: the last k with voff[k] <= e
        const uint32_t e0 = (uint32_t)(w * WK + lane);
        int a = 0, b = np;
        while (b - a > 1) {
            const int mid = (a + b) >> 1;
            if (voff[mid] <= e0) a = mid;
            else b = mid;
        }
        int k = a;
        uint32_t pend = voff[k + 1], pbase = plo[k] - voff[k];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const uint32_t e = e0 + 64 * i;
            x[i] = key_max<T>();
            if (e < tot) {
                while (e >= pend) {
                    ++k;
                    pend = voff[k + 1];
                    pbase = plo[k] - voff[k];
                }
                x[i] = in[pbase + e];
            }
        }
        return;
    }
    const uint32_t e0 = (uint32_t)(w * (WK / N) + lane);
    if (vp) {
        uint32_t keep = 0;  // bit N i + j: key j of vector i belongs to the tile
#pragma unroll
        for (int i = 0; i < R / N; ++i) {
            const uint32_t e = e0 + 64 * i;
            if (e < tot) {
                const uint32_t k = vpc[e], pl = plo[k], ph = phi[k];
                const uint32_t g = (pl / N - voff[k] + e) * N;  // first key of the vector
                V16<T>::get(*reinterpret_cast<const V *>(in + g), x + N * i);
#pragma unroll
                for (int j = 0; j < N; ++j) keep |= (uint32_t)(g + j >= pl && g + j < ph) << (N * i + j);
            }
        }
#pragma unroll
        for (int i = 0; i < R; ++i) x[i] = (keep >> i) & 1 ? x[i] : key_max<T>();
        return;
    }
    // piece of vector slot e0: the last k with voff[k] <= e0
    int a = 0, b = np;
    while (b - a > 1) {
        const int mid = (a + b) >> 1;
        if (voff[mid] <= e0) a = mid;
        else b = mid;
    }
    int k = a;
    uint32_t vend = voff[k + 1], pl = plo[k], ph = phi[k], vb = pl / N - voff[k];
    uint32_t keep = 0;  // bit N i + j: key j of vector i belongs to the tile
    // all loads first, the masks applied once they are in flight (a select right after its load
    // would wait for that load before the next one issues)
#pragma unroll
    for (int i = 0; i < R / N; ++i) {
        const uint32_t e = e0 + 64 * i;
        if (e < tot) {
            while (e >= vend) {
                ++k;
                vend = voff[k + 1];
                pl = plo[k];
                ph = phi[k];
                vb = pl / N - voff[k];
            }
            const uint32_t g = (vb + e) * N;  // first key of the vector
            V16<T>::get(*reinterpret_cast<const V *>(in + g), x + N * i);
#pragma unroll
            for (int j = 0; j < N; ++j) keep |= (uint32_t)(g + j >= pl && g + j < ph) << (N * i + j);
        }
    }
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = (keep >> i) & 1 ? x[i] : key_max<T>();
}

// Tile j's keys into x (any order; slots past `valid` are key_max).  Returns false when j is
// past the tile count (the grid is an upper bound).
template <typename T, bool GATHER, int W>
__device__ __forceinline__ bool load_tile(const T *in, uint64_t n, const uint4 *tiles, const uint32_t *ntiles,
                                          const sb::Gather &ga, uint32_t j, uint32_t *poff, uint32_t *wsum,
                                          T (&x)[R], uint64_t &base, int &valid, const int tid = threadIdx.x) {
    constexpr int TILE = TILE_W<W>, N = KPC<T>;
    using V = typename V16<T>::type;
    const int t = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
    if constexpr (GATHER) {
        if (j >= *ntiles) return false;
        const sb::GTile gt = ga.tiles[j];
        base = gt.base;
        valid = (int)gt.valid;
        uint2 pe[2];
        gather_pieces(ga, j, pe, tid);
        gather_tile<T, W>(ga, pe, gt, in, poff, wsum, x, tid);
        return true;
    } else if (tiles) {
        if (j >= *ntiles) return false;
        const uint4 r = tiles[j];  // TileRef: base (2 words), valid
        base = (uint64_t)r.x | ((uint64_t)r.y << 32);
        valid = (int)r.z;
    } else {
        base = (uint64_t)j * TILE;
        if (base >= n) return false;
        const uint64_t rem = n - base;
        valid = rem < (uint64_t)TILE ? (int)rem : TILE;
    }
    // off = keys between the 16-byte boundary below the tile and its first key
    const int off = (int)((reinterpret_cast<uintptr_t>(in + base) / sizeof(T)) & (N - 1));
    if (off + valid <= TILE) {
        // 16-byte vectors from the boundary; entries outside [off, off + valid) become +inf.  A
        // vector is loaded only when it holds a key of the tile (an aligned 16-byte block never
        // crosses a page); the keys of a neighbouring tile it also holds are dropped.
        const V *src = reinterpret_cast<const V *>(in + base - off) + w * (WK / N);
        const int lim = off + valid;
#pragma unroll
        for (int q = 0; q < R / N; ++q) {
            const int e0 = w * WK + N * (q * 64 + t);
            T vals[N];
#pragma unroll
            for (int jj = 0; jj < N; ++jj) vals[jj] = key_max<T>();
            if (e0 < lim) V16<T>::get(src[q * 64 + t], vals);
#pragma unroll
            for (int jj = 0; jj < N; ++jj)
                x[N * q + jj] = (e0 + jj >= off && e0 + jj < lim) ? vals[jj] : key_max<T>();
        }
    } else {
#pragma unroll
        for (int q = 0; q < R / N; ++q) {
#pragma unroll
            for (int jj = 0; jj < N; ++jj) {
                const int e = w * WK + N * (q * 64 + t) + jj;
                x[N * q + jj] = e < valid ? in[base + e] : key_max<T>();
            }
        }
    }
    return true;
}

// The bin sort of every tile (bin_sort_tile); a tile it declines is appended to fb (*nfb) for
// the bitonic kernel.  Separate from the bitonic kernel so that each keeps its own registers.
template <typename T, bool GATHER, int W>
__global__ void __launch_bounds__(64 * W, WG<T>::OCC) bin_sort_kernel(const T *in, T *out, uint64_t n,
                                                                     const uint4 *tiles, const uint32_t *ntiles,
                                                                     sb::Gather ga, uint32_t *fb, uint32_t *nfb,
                                                                     uint32_t toff) {
    constexpr int TILE = TILE_W<W>;
    static_assert(128 + 3 * kMaxPieces<T> + 1 + (TILE / KPC<T> + 1) / 2 <= TILE * (int)sizeof(T) / 4,
                  "the piece table and the vector slots' pieces fit in the tile");
    __shared__ __attribute__((aligned(16))) T s[TILE];
    __shared__ __attribute__((aligned(16))) uint32_t cw[BIN_NB<W> / 2];
    // the counters are zeroed before the gather's barriers; the piece table of a gathered tile and
    // its scan words live in the tile array (free until the keys are placed), past BinSm
    reinterpret_cast<uint4 *>(cw)[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
    uint32_t *s32 = reinterpret_cast<uint32_t *>(s);
    T x[R];
    uint64_t base;
    int valid;
    STAMP(0);
    bool hint = false, known = false;
    T klo = T(0), khi = T(0);
    uint32_t j;
    if constexpr (GATHER) {
        // Gathered tiles: each XCD takes a contiguous block of tiles (workgroups are dealt
        // round-robin over the 8 XCDs).  Consecutive tiles of a bucket end and start inside the
        // same 128-byte lines of every chunk: run on one XCD at about the same time, such a line
        // comes from HBM once and from that XCD's L2 the second time.
        j = toff + xcd_block(blockIdx.x, gridDim.x);  // (toff: tiles [toff, toff + grid) of a split launch)
        // the tile record and its piece table are read together with the tile count, not after it
        // (an index past the count reads an entry inside the tables, and returns below)
        const uint32_t jr = j < ga.tcap ? j : ga.tcap - 1;
        uint2 pe[2];
        gather_pieces(ga, jr, pe);
        const sb::GTile gt = ga.tiles[jr];
        if (j >= *ntiles) return;
        base = gt.base;
        valid = (int)gt.valid;
        if (valid == 0) return;
        // The tile's key range from the splitters around it (read with the prefix tables, before
        // the keys): sub-buckets [j0, j1) of bucket b hold keys in [spl[j0 - 1], spl[j1 - 1]], a
        // bucket's bounds are the first level's splitters b - 1 and b.  Known bounds let the
        // counting start on the first keys that arrive, with no reduction and no barrier between
        // the loads and the counting; only the first tile of bucket 0 and the last of bucket B - 1
        // reduce over their keys.
        const sb::Spl<T> *sp = static_cast<const sb::Spl<T> *>(ga.spl) + (uint64_t)gt.b * ga.SS;
        const auto *bs = static_cast<const typename bk::Comp<T>::C *>(ga.bspl);
        const bool lk = gt.j0 > 0 || gt.b > 0, hk = gt.j1 < gt.nsub || (int)gt.b + 1 < ga.B;
        known = lk && hk;
        // int32 (DSORT_LATE_BOUNDS): the bounds and the duplicate hint are read after the key loads
        // are issued -- read here, their round trip sat between the tile record and the key loads
        // (one of the gather's four dependent round trips); int64 needs them first (one-key tiles)
#ifndef DSORT_LATE_BOUNDS
#define DSORT_LATE_BOUNDS 1
#endif
        constexpr bool late = DSORT_LATE_BOUNDS && sizeof(T) == 4;
        const int jl = gt.j0 > 0 ? (int)gt.j0 - 1 : 0, jh = (int)gt.j1 - 1;  // splitters around the tile
        const int nspl = (int)gt.nsub - 1;
        const int jj = jl + lane_id();
        if (late) {
            gather_tile<T, W>(ga, pe, gt, in, s32 + 128, s32 + 96, x, threadIdx.x);
            if (known) {
                klo = gt.j0 > 0 ? sp[gt.j0 - 1].k : bk::Comp<T>::key_of(bs[gt.b - 1]);
                khi = gt.j1 < gt.nsub ? sp[gt.j1 - 1].k : bk::Comp<T>::key_of(bs[gt.b]);
            }
            if (jj < jh && jj + 1 < nspl) hint = sp[jj].k == sp[jj + 1].k;
            hint = __ballot(hint) != 0;
        }
        if (!late && known) {
            klo = gt.j0 > 0 ? sp[gt.j0 - 1].k : bk::Comp<T>::key_of(bs[gt.b - 1]);
            khi = gt.j1 < gt.nsub ? sp[gt.j1 - 1].k : bk::Comp<T>::key_of(bs[gt.b]);
#ifndef DSORT_ONEKEY_TILES
#define DSORT_ONEKEY_TILES 1
#endif
            if (DSORT_ONEKEY_TILES && sizeof(T) == 8 && klo == khi) {
                // Bounds of one key: every key of the tile is that key (the sub-buckets of a heavy
                // duplicate, int64 Zipf's keys with thousands of copies) -- the tile is written as
                // its key, without reading it.  (The first level does the same for pure buckets.)
                // C4 tile sort 2.94 -> 1.79 ms.  int64 only: the branch makes the gather wait for the
                // bounds' loads, +0.04 ms on the 2^30 int32 tile sort, where such tiles are rare.)
                T *o = out + base;
                for (int i = (int)threadIdx.x; i < valid; i += (int)blockDim.x) o[i] = klo;
                return;
            }
        }
        if (!late) {
            // a duplicate run inside a gathered tile shows as two equal neighbouring splitters
            if (jj < jh && jj + 1 < nspl) hint = sp[jj].k == sp[jj + 1].k;
            hint = __ballot(hint) != 0;
            gather_tile<T, W>(ga, pe, gt, in, s32 + 128, s32 + 96, x, threadIdx.x);
        }
    } else {
        j = toff + blockIdx.x;
        if (!load_tile<T, false, W>(in, n, tiles, ntiles, ga, j, nullptr, nullptr, x, base, valid)) return;
        if (valid == 0) return;
    }
    STAMP(1);
    if (!bin_sort_tile<T, W>(x, valid, s, cw, out + base, hint, known, klo, khi, threadIdx.x) && threadIdx.x == 0)
        fb[atomicAdd(nfb, 1u)] = j;
}

// The bitonic tile sort of the bin sort's declined tiles fb[i], i < *nfb, each workgroup taking
// i = blockIdx.x, blockIdx.x + gridDim.x, ... (the count stays on the device: the host never
// waits for the bin sort, and with no declined tile every workgroup exits at once).
template <typename T, bool GATHER, int W>
__global__ void __launch_bounds__(64 * W, WG<T>::OCC) block_sort_w_kernel(
    const T *in, T *out, uint64_t n, const uint4 *tiles, const uint32_t *ntiles, sb::Gather ga,
    const uint32_t *fb, const uint32_t *nfb) {
    constexpr int TILE = TILE_W<W>, N = KPC<T>;
    using V = typename V16<T>::type;
    // `in` may alias `out`: every workgroup reads its tile before it writes it
    __shared__ __attribute__((aligned(16))) T s[TILE + WK];  // + slack read by load_window
    const int t = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const T c[6] = {lane_side<T>(0), lane_side<T>(1), lane_side<T>(2), lane_side<T>(3), lane_side<T>(4),
                    lane_side<T>(5)};
    const uint32_t nj = *nfb;
#pragma unroll 1
    for (uint32_t i = blockIdx.x; i < nj; i += gridDim.x) {
    if (i != blockIdx.x) __syncthreads();  // the previous tile's last reads of s are done
    T x[R];
    uint64_t base;
    int valid;
    const uint32_t j = fb[i];
    // (the piece table of a gathered tile sits in the runs' space: a barrier before they are written)
    if (!load_tile<T, GATHER, W>(in, n, tiles, ntiles, ga, j, reinterpret_cast<uint32_t *>(s) + 64,
                              reinterpret_cast<uint32_t *>(s), x, base, valid))
        return;
    if (GATHER) __syncthreads();
    sort_wave(x, c);
    // lane-major run of the wave -> LDS; odd waves' runs (the B runs of the first level) are
    // stored descending
    {
        if (w & 1) {
            V *dst = reinterpret_cast<V *>(s + w * WK + WK - R * (t + 1));
#pragma unroll
            for (int q = 0; q < R / N; ++q) {
                T rv[N];
#pragma unroll
                for (int j = 0; j < N; ++j) rv[j] = x[R - 1 - (N * q + j)];
                dst[q] = V16<T>::make(rv);
            }
        } else {
            V *dst = reinterpret_cast<V *>(s + w * WK + t * R);
#pragma unroll
            for (int q = 0; q < R / N; ++q) dst[q] = V16<T>::make(x + N * q);
        }
    }
    __syncthreads();
    const int lo = out_lo(t);
#pragma unroll 1
    for (int r = WK; r < TILE; r <<= 1) {
        const int wpp = (2 * r) / WK;  // windows per pair
        const int j = w / wpp, o = w % wpp;
        const int ps = j * 2 * r;
        const bool last = 2 * r == TILE;
        WinD win{ps, r, r, o * WK, 0, WK, !last && (j & 1)};
        merge_window_desc(s, win, x, c[0], c[1], c[2], c[3]);
        __syncthreads();
        if (last) {
            const int lim = valid - o * WK;
            win.cnt = lim < WK ? lim : WK;
            if (lim > 0) store_window_desc<false>(out + base, win, ps, lo, x);
        } else {
            store_window_desc<true>(s, win, ps, lo, x);
            __syncthreads();
        }
    }
    }
}

// ------------------------------------------------------------------------------------------
// 2. Merge of one output tile of a k-way pass (cuts from partk_kernel).
// ------------------------------------------------------------------------------------------
template <typename T, int LOGF, bool REG>
__global__ void __launch_bounds__(64 * WG<T>::MWAVES, WG<T>::OCC) mergew_kernel(
    const T *__restrict__ in, T *__restrict__ out, PassDesc pd, int tnom, const uint32_t *__restrict__ splits) {
    constexpr int WAVES = WG<T>::MWAVES, THREADS = 64 * WAVES, TILE = MTILE_OF<T>;
    constexpr int N = KPC<T>, LN = LKPC<T>;
    using V = typename V16<T>::type;
    constexpr int F = 1 << LOGF;
    constexpr int MAXWIN = (WAVES + F / 2 + WAVES - 1) / WAVES;
    static_assert(WAVES * MAXWIN <= 64, "window table: one lane per window");
    __shared__ __attribute__((aligned(16))) T s[TILE + WK];  // + slack read by load_window
    __shared__ int soff[F + 1];          // tile position of segment i (soff[F] = keys of the tile)
    // Staging works on 16-byte-aligned chunks of N keys of each segment (absolute alignment):
    __shared__ int cpre[F + 1];          // chunks before segment i (cpre[F] = chunks of the tile)
    __shared__ int4 sinfo[F];            // cpre[i], soff[i], keys, first chunk - first key
    __shared__ int64_t sa0[F];           // global index of the segment's first aligned chunk
    __shared__ uint64_t s_out;
    __shared__ int4 wtab_a[LOGF][WAVES * MAXWIN];  // per level and window: pa, na, nb, d0
    __shared__ int4 wtab_b[LOGF][WAVES * MAXWIN];  // skip, cnt (0 = no window), desc, -
    const int t = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const uint64_t j = blockIdx.x;
    STAMP(0);
    RSTAMP(13);
    TileInfo ti;
    const GroupK *g = tile_info<REG>(pd, j, tnom, ti);
    if (threadIdx.x < 64) {
        const int i = t & (F - 1);
        uint64_t rs, rl;
        run_range<REG>(pd, ti, g, i, rs, rl);
        const uint32_t s0 = splits[j * F + i];
        const uint32_t s1 = ti.jr + 1 == ti.ntg ? (uint32_t)rl : splits[(j + 1) * F + i];
        const int len = (int)(s1 - s0);
        int incl = len;
        uint64_t before = s0;  // output offset of the tile = keys of the group below its cut
        for (int o = 1; o < F; o <<= 1) {
            const int v = __shfl_up(incl, o);
            if (i >= o) incl += v;
            before += __shfl_xor(before, o);
        }
        // aligned chunks of segment i (absolute 16-B alignment of &in[g])
        const int mis = (int)((reinterpret_cast<uintptr_t>(in) / sizeof(T)) & (N - 1));
        const int64_t gs = (int64_t)(rs + s0);
        const int64_t a0 = ((gs + mis) & ~(int64_t)(N - 1)) - mis;
        const int nc = len ? (int)((gs + len + mis + N - 1) >> LN) - (int)((gs + mis) >> LN) : 0;
        int cinc = nc;
        for (int o = 1; o < F; o <<= 1) {
            const int v = __shfl_up(cinc, o);
            if (i >= o) cinc += v;
        }
        if (t < F) {
            soff[i + 1] = incl;
            sa0[i] = a0;
            sinfo[i] = make_int4(cinc - nc, incl - len, len, (int)(a0 - gs));
            cpre[i + 1] = cinc;
            if (i == 0) cpre[0] = 0;
            if (i == 0) {
                soff[0] = 0;
                s_out = ti.base + before;
            }
        }
    }
    __syncthreads();
    STAMP(1);
    const int nchunks = __builtin_amdgcn_readfirstlane(cpre[F]);
    if (nchunks == 0) return;  // empty tile (workgroup-uniform)
    STAMP(2);
    RSTAMP(14);
    // Staging: chunk q (N keys, 16-B aligned in global memory) is loaded by thread q % THREADS
    // with one dwordx4 (consecutive lanes on consecutive chunks of a segment: 1 KiB per wave
    // instruction); the keys of a chunk that lie outside its segment are dropped.  An aligned
    // 16-B block holding a key of the array never crosses a page, so edge chunks are safe; lanes
    // past the last chunk load the last chunk again and drop it.
    {
        constexpr int NK = (TILE / N + kWaveMaxF + THREADS - 1) / THREADS;  // chunks per thread
        V v[NK];
        int ebase[NK], lo4[NK], hi4[NK], dirk[NK], qc[NK], sg[NK];
        // All chunk addresses are computed branch-free and side by side (the searches of the NK
        // chunks interleave), so the NK loads leave together.
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int q = threadIdx.x + k * THREADS;
            qc[k] = q < nchunks ? q : nchunks - 1;
            sg[k] = 0;  // last segment whose chunks start at or before qc (a non-empty one)
        }
#pragma unroll
        for (int st = F / 2; st >= 1; st >>= 1) {
#pragma unroll
            for (int k = 0; k < NK; ++k) sg[k] += cpre[sg[k] + st] <= qc[k] ? st : 0;
        }
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int4 si = sinfo[sg[k]];
            const int c = N * (qc[k] - si.x);
            const int off = si.w + c;  // key offset of the chunk in its segment
            // odd segments (B runs of level 0) are staged descending
            const bool odd = sg[k] & 1;
            dirk[k] = odd ? -1 : 1;
            ebase[k] = odd ? si.y + si.z - 1 - off : si.y + off;
            lo4[k] = -off;  // valid jj: -off <= jj < len - off
            hi4[k] = threadIdx.x + k * THREADS < nchunks ? si.z - off : 0;
            v[k] = *reinterpret_cast<const V *>(in + sa0[sg[k]] + c);
        }
        // Window table of every level, built from the segment offsets alone (they do not depend on
        // the keys): level l merges pairs of 2^l-segment groups; pair p is cut into ceil(len / 1024)
        // windows; window k of the level goes to wave k % WAVES (k < WAVES * MAXWIN).  Wave l
        // builds the table of level l while its staging loads are in flight.
        for (int l = w; l < LOGF; l += WAVES) {
            const int npairs = F >> (l + 1);
            int ps = 0, pm = 0, pe = 0, nw = 0;
            if (t < npairs) {
                ps = soff[t << (l + 1)];
                pm = soff[((2 * t + 1) << l)];
                pe = soff[(t + 1) << (l + 1)];
                nw = (pe - ps + WK - 1) / WK;
            }
            int incl = nw;
            for (int o = 1; o < 16; o <<= 1) {
                const int vv = __shfl_up(incl, o);
                if (t >= o) incl += vv;
            }
            // lane k (< WAVES * MAXWIN) describes window k: its pair is the number of pairs whose
            // windows all come before k
            int p = 0;
            for (int q = 0; q < npairs; ++q) p += __builtin_amdgcn_readlane(incl, q) <= t ? 1 : 0;
            const int pp = p < npairs ? p : 0;
            const int fps = __shfl(ps, pp), fpm = __shfl(pm, pp), fpe = __shfl(pe, pp);
            const int first = __shfl(incl - nw, pp);
            if (t < WAVES * MAXWIN) {
                int4 a = make_int4(0, 0, 0, 0), b = make_int4(0, 0, 0, 0);  // cnt 0: no window
                if (p < npairs) {
                    const int len = fpe - fps;
                    const int dn = (t - first) * WK;  // nominal start of the window
                    const int rem = len - dn;
                    // the last window of a pair of >= 1024 keys is shifted to end at the pair's end
                    const int d0 = rem < WK && len >= WK ? len - WK : dn;
                    a = make_int4(fps, fpm - fps, fpe - fpm, d0);
                    // groups that become the B run of the next level are stored descending
                    b = make_int4(dn - d0, rem < WK ? rem : WK, (l + 1 < LOGF) && (p & 1), 0);
                }
                wtab_a[l][t] = a;
                wtab_b[l][t] = b;
            }
        }
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            T vals[N];
            V16<T>::get(v[k], vals);
#pragma unroll
            for (int jj = 0; jj < N; ++jj)
                if (jj >= lo4[k] && jj < hi4[k]) s[ebase[k] + dirk[k] * jj] = vals[jj];
        }
    }
    STAMP(3);
    __syncthreads();
    STAMP(4);
    RSTAMP(15);

    const T c0 = lane_side<T>(0), c1 = lane_side<T>(1), c2 = lane_side<T>(2), c3 = lane_side<T>(3);
    const int lo = out_lo(t);
    const uint64_t so = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(s_out >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)s_out);
    T *outp = out + so;
#pragma unroll 1
    for (int l = 0; l < LOGF; ++l) {
        const bool last = l + 1 == LOGF;
        WinD win[MAXWIN];
#pragma unroll
        for (int h = 0; h < MAXWIN; ++h) {
            const int4 a = wtab_a[l][w + h * WAVES];
            const int4 b = wtab_b[l][w + h * WAVES];
            win[h].pa = __builtin_amdgcn_readfirstlane(a.x);
            win[h].na = __builtin_amdgcn_readfirstlane(a.y);
            win[h].nb = __builtin_amdgcn_readfirstlane(a.z);
            win[h].d0 = __builtin_amdgcn_readfirstlane(a.w);
            win[h].skip = __builtin_amdgcn_readfirstlane(b.x);
            win[h].cnt = __builtin_amdgcn_readfirstlane(b.y);
            win[h].desc = __builtin_amdgcn_readfirstlane(b.z);
        }
        T x[MAXWIN][R];
#pragma unroll
        for (int h = 0; h < MAXWIN; ++h)
            if (win[h].cnt > 0) merge_window_desc(s, win[h], x[h], c0, c1, c2, c3);
        STAMP(5 + 2 * l);
        __syncthreads();
#pragma unroll
        for (int h = 0; h < MAXWIN; ++h) {
            if (win[h].cnt > 0) {
                if (last) store_window_desc<false>(outp, win[h], win[h].pa, lo, x[h]);
                else store_window_desc<true>(s, win[h], win[h].pa, lo, x[h]);
            }
        }
        if (!last) __syncthreads();
        STAMP(6 + 2 * l);
        if (last) RSTAMP(29);
    }
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
static inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
static int ceil_log2(uint64_t x) {
    int p = 0;
    while ((1ull << p) < x) ++p;
    return p;
}
// log2(F) of each pass: as few passes as the cap allows (default F <= 16), the bits spread
// evenly over them.
template <typename T>
static std::vector<int> plan_passes(const dsort_opts &opt, uint64_t runs) {
    std::vector<int> out;
    const int bits = ceil_log2(runs);
    if (bits == 0) return out;
    const int cap = max_logf(opt, 4, WG<T>::MAXLOGF);
    const int P = (bits + cap - 1) / cap;
    for (int p = 0; p < P; ++p) out.push_back(bits / P + (p < bits % P ? 1 : 0));
    return out;
}

// Stage event i of a timed sort (dsort_internal.h: ctx->ev): 7 / 8 around the tile sort kernel
// (dsort_stats.tile_sort_kernel_ms, partition_ms), 9 / 10 the first-level histogram, 11 / 12 the
// first-level scatter, 13 / 14 the second-level partition.
// Every stage boundary of the outermost sort also opens / closes a roctx range on the host thread
// (rocprofv3 --marker-trace shows when each stage was enqueued; the device times are the events'):
// dsort:histogram, dsort:scatter, dsort:second-level, dsort:tile-sort.
static void stage_range(const dsort_ctx *ctx, int i) {
    if (ctx->nested) return;
    switch (i) {
        case 9: roctxRangePushA("dsort:histogram"); break;
        case 11: roctxRangePushA("dsort:scatter"); break;
        case 13: roctxRangePushA("dsort:second-level"); break;
        case 7: roctxRangePushA("dsort:tile-sort"); break;
        case 10: case 12: case 14: case 8: roctxRangePop(); break;
        default: break;
    }
}
static int stage_event(dsort_ctx *ctx, hipStream_t s, bool timed, int i) {
    if (timed) stage_range(ctx, i);
    if (!timed || !ctx->ev_ok) return DSORT_OK;
    if (i == 1 || i == 7 || i == 8 || i == 13 || i == 14) i += ctx->ev_off;
    DSORT_HIP(ctx, hipEventRecord(ctx->ev[i], s));
    ctx->ev_mask |= 1u << i;
    return DSORT_OK;
}
static int tile_sort_event(dsort_ctx *ctx, hipStream_t s, bool timed, int which) {
    return stage_event(ctx, s, timed, 7 + which);
}

// The tile sort of `grid` tiles (an upper bound when the count lives on the device): the bin
// sort first, then the bitonic sort of the tiles it declined.  Events 7 / 8 around both.
constexpr uint32_t kFallbackWgs = 512;  // two workgroups per CU
// In parts: tile_sort_begin (the fallback list for up to `cap` tiles, the bin sort of tiles
// [0, grid)), tile_sort_more (tiles [toff, toff + grid)), tile_sort_end (the bitonic kernel over the
// declined tiles of `tiles_total`).  The local path launches the first part before the host knows
// the tile count (tile_sort_early).
template <typename T, bool GATHER, int W>
static int tile_sort_begin(dsort_ctx *ctx, const T *in, T *out, uint64_t n, const uint4 *tiles, const uint32_t *ntiles,
                           const sb::Gather &ga, uint32_t grid, uint32_t cap, hipStream_t s) {
    int rc = ensure(ctx, &ctx->tfb, &ctx->tfb_bytes, ((size_t)cap + 1) * 4, "tile fallback list");
    if (rc) return rc;
    uint32_t *fb = static_cast<uint32_t *>(ctx->tfb), *nfb = fb + cap;
    DSORT_HIP(ctx, hipMemsetAsync(nfb, 0, 4, s));
    if (grid)
        hipLaunchKernelGGL((bin_sort_kernel<T, GATHER, W>), dim3(grid), dim3(64 * W), 0, s, in, out, n, tiles, ntiles, ga, fb,
                           nfb, 0u);
    DSORT_HIP(ctx, hipGetLastError());
    return DSORT_OK;
}
template <typename T, bool GATHER, int W>
static int tile_sort_more(dsort_ctx *ctx, const T *in, T *out, uint64_t n, const uint4 *tiles, const uint32_t *ntiles,
                          const sb::Gather &ga, uint32_t toff, uint32_t grid, uint32_t cap, hipStream_t s) {
    uint32_t *fb = static_cast<uint32_t *>(ctx->tfb), *nfb = fb + cap;
    if (grid)
        hipLaunchKernelGGL((bin_sort_kernel<T, GATHER, W>), dim3(grid), dim3(64 * W), 0, s, in, out, n, tiles, ntiles, ga, fb,
                           nfb, toff);
    DSORT_HIP(ctx, hipGetLastError());
    return DSORT_OK;
}
template <typename T, bool GATHER, int W>
static int tile_sort_end(dsort_ctx *ctx, const T *in, T *out, uint64_t n, const uint4 *tiles, const uint32_t *ntiles,
                         const sb::Gather &ga, uint32_t tiles_total, uint32_t cap, hipStream_t s) {
    const uint32_t *fb = static_cast<const uint32_t *>(ctx->tfb), *nfb = fb + cap;
    // the declined tiles: a grid of at most one round of workgroups over the chip walks the
    // list, whose length stays on the device (round 2 read it back: the host waited for the
    // bin sort, and the GPU idled about 70 us per sort until the next work arrived)
    const uint32_t fgrid = tiles_total < kFallbackWgs ? tiles_total : kFallbackWgs;
    if (fgrid)
        hipLaunchKernelGGL((block_sort_w_kernel<T, GATHER, W>), dim3(fgrid), dim3(64 * W), 0, s, in, out, n, tiles, ntiles,
                           ga, fb, nfb);
    DSORT_HIP(ctx, hipGetLastError());
    return DSORT_OK;
}
template <typename T, bool GATHER, int W>
static int tile_sort_w(dsort_ctx *ctx, const T *in, T *out, uint64_t n, const uint4 *tiles, const uint32_t *ntiles,
                       const sb::Gather &ga, uint32_t grid, hipStream_t s) {
    int rc = tile_sort_begin<T, GATHER, W>(ctx, in, out, n, tiles, ntiles, ga, grid, grid, s);
    if (rc) return rc;
    return tile_sort_end<T, GATHER, W>(ctx, in, out, n, tiles, ntiles, ga, grid, grid, s);
}
// f(std::integral_constant<int, W>) with the wave count W of a tile size (TILE_OF<T>, or int32's 16384)
template <typename T, typename F>
static int with_tile_waves(dsort_ctx *ctx, int tile, F &&f) {
    if (tile == TILE_OF<T>) return f(std::integral_constant<int, WG<T>::WAVES>{});
    if constexpr (sizeof(T) == 4)
        if (tile == TILE_W<16>) return f(std::integral_constant<int, 16>{});
    return set_err(ctx, DSORT_EINVAL, "tile sort: no kernel for this tile size");
}
// tile: the tile size in keys (TILE_OF<T>, or 16384 for int32's large buckets: sub_sort)
template <typename T, bool GATHER>
static int tile_sort(dsort_ctx *ctx, const T *in, T *out, uint64_t n, const uint4 *tiles, const uint32_t *ntiles,
                     const sb::Gather &ga, uint32_t grid, hipStream_t s, bool timed, int tile = TILE_OF<T>) {
    int rc = tile_sort_event(ctx, s, timed, 0);
    if (rc) return rc;
    // (The library's own small sorts, the splitter samples, take the same path: nothing is read
    // back, and a tile of a bucket's 2048 samples costs the bin sort a quarter of what the bitonic
    // sort spends on the whole padded tile.)
    if (grid) {
        rc = with_tile_waves<T>(ctx, tile, [&](auto w) {
            return tile_sort_w<T, GATHER, decltype(w)::value>(ctx, in, out, n, tiles, ntiles, ga, grid, s);
        });
        if (rc) return rc;
    }
    return tile_sort_event(ctx, s, timed, 1);
}

template <typename T, bool REG>
static int launch_pass_w(dsort_ctx *ctx, const T *src, T *dst, const PassDesc &pd, int logf,
                         uint64_t ntiles, hipStream_t s, bool timed) {
    int rc = ensure(ctx, &ctx->splits, &ctx->splits_bytes,
                    (size_t)(ntiles + 1) * (size_t)(1 << logf) * sizeof(uint32_t), "split vectors");
    if (rc) return rc;
    uint32_t *sp = static_cast<uint32_t *>(ctx->splits);
    constexpr int TN = MTNOM_OF<T>;
    hipLaunchKernelGGL((partk_kernel<T, REG>), dim3((unsigned)ceil_div(ntiles, 4)), dim3(256), 0, s, src, pd,
                       TN, MSLACK_OF<T>, sp, ntiles);
    DSORT_HIP(ctx, hipGetLastError());
    const bool kt = timed && ctx->ev_ok && ctx->kev_used + 2 <= dsort_ctx::kMaxKev;
    if (kt) DSORT_HIP(ctx, hipEventRecord(ctx->kev[ctx->kev_used], s));
    const dim3 grid((unsigned)ntiles), block(64 * WG<T>::MWAVES);
    switch (logf) {
        case 1: hipLaunchKernelGGL((mergew_kernel<T, 1, REG>), grid, block, 0, s, src, dst, pd, TN, sp); break;
        case 2: hipLaunchKernelGGL((mergew_kernel<T, 2, REG>), grid, block, 0, s, src, dst, pd, TN, sp); break;
        case 3: hipLaunchKernelGGL((mergew_kernel<T, 3, REG>), grid, block, 0, s, src, dst, pd, TN, sp); break;
        case 4: hipLaunchKernelGGL((mergew_kernel<T, 4, REG>), grid, block, 0, s, src, dst, pd, TN, sp); break;
        case 5:
            if constexpr (WG<T>::MAXLOGF >= 5) {
                hipLaunchKernelGGL((mergew_kernel<T, 5, REG>), grid, block, 0, s, src, dst, pd, TN, sp);
                break;
            }
            return set_err(ctx, DSORT_EINVAL, "bad pass fan-in");
        default: return set_err(ctx, DSORT_EINVAL, "bad pass fan-in");
    }
    DSORT_HIP(ctx, hipGetLastError());
    if (kt) {
        DSORT_HIP(ctx, hipEventRecord(ctx->kev[ctx->kev_used + 1], s));
        ctx->kev_used += 2;
    }
    return DSORT_OK;
}

// ---- bucketed sort (dsort_bucket.h) ------------------------------------------------------
// Buckets of about 2^20 keys: at most 1024, and none below 2^25 keys (DSORT_OPT_BUCKETS = 0
// turns the partition off, B forces B buckets, DSORT_OPT_BUCKET_KEYS sets the nominal bucket
// size).  Without the second level (DSORT_OPT_SUB_KEYS = 0) every bucket is tile-sorted and
// merged with a per-bucket fan-in (int32 at 2^30 keys: 1024 buckets of about 128 8K-key tiles).
// A nested sort (the splitter samples) never buckets.
static int bucket_count(const dsort_opts &opt, uint64_t n) {
    const int64_t forced = opt.buckets;
    if (forced == 0) return 0;
    const uint64_t tk = opt.bucket_keys > 0 ? (uint64_t)opt.bucket_keys : (1ull << 20);
    uint64_t B = forced > 0 ? (uint64_t)forced : ceil_div(n, tk);
    if (forced < 0 && n < (1ull << 25)) return 0;
    if (n >= (1ull << 32)) return 0;  // 32-bit bucket positions in the scatter
    if (B > (uint64_t)bk::BK_MAXB) B = bk::BK_MAXB;
    return B >= 2 ? (int)B : 0;
}
static int bucket_count(const dsort_ctx *ctx, uint64_t n) { return ctx->nested ? 0 : bucket_count(ctx->opt, n); }

// Samples per bucket for the int32 splitters (sorted on the GPU): the relative spread of the
// bucket sizes is about 1/sqrt(os) (DSORT_OPT_BUCKET_OVERSAMPLE).
static int bucket_os(const dsort_ctx *ctx) {
    const int64_t v = ctx->opt.bucket_os;
    return v < 1 ? 1 : (v > 4096 ? 4096 : (int)v);
}

// Group tables of the merge passes inside buckets: pass p merges groups of up to 2^bits
// consecutive runs of one bucket; a bucket with a single run left is carried as a 1-run group.
struct BucketPass {
    int logf;
    uint64_t ngroups, ntiles;
    size_t group_off, tile_off;  // in the group / tile_group staging
};

template <typename T>
static int wave_merge(dsort_ctx *ctx, const T *d_in, const size_t *lens, int k, T *d_out, hipStream_t s,
                      bool keep_stats);

// ---- second partition level (dsort_sub.h) -------------------------------------------------
// Nominal keys per sub-bucket: TILE / 8 unless DSORT_OPT_SUB_KEYS says otherwise (0 = off).
#ifndef DSORT_SUB_NOM_16THS
#define DSORT_SUB_NOM_16THS 3
#endif
constexpr uint64_t SUB_NOM_16THS = DSORT_SUB_NOM_16THS;  // nominal sub-bucket: 3/16 of a tile
template <typename T>
static uint64_t sub_keys(const dsort_opts &opt) {
    const int64_t v = opt.sub_keys;
    return v < 0 ? (uint64_t)TILE_OF<T> * SUB_NOM_16THS / 16 : (uint64_t)v;
}
template <typename T>
static uint64_t sub_keys(const dsort_ctx *ctx) { return sub_keys<T>(ctx->opt); }

// Runs of an oversized sub-bucket as the packer cut it (sb_scan_kernel): the room of the first
// tile, then whole tiles.
static std::vector<size_t> sub_tile_runs(uint64_t p, uint64_t len, uint64_t tile, uint64_t align, uint64_t mis) {
    std::vector<size_t> r;
    const uint64_t room = tile - ((p + mis) & (align - 1));
    r.push_back(room);
    for (uint64_t q = room; q < len; q += tile) r.push_back(len - q < tile ? len - q : tile);
    return r;
}

// Sub-buckets of every bucket (src = the first level's output), packed into tiles and
// tile-sorted in d_keys.  Called from bucket_sort once the bucket starts hb[0..B] are on the
// host (the first level's scatter is still running).
//
// Two ways to form the tiles (DSORT_OPT_SUB_GATHER): local (default) -- every chunk of a bucket
// is partitioned by sub-bucket in place (sb_local_kernel) and the tile sort gathers a tile's
// piece of every chunk; scatter -- histograms, then every key is scattered to its sub-bucket in
// d_keys (sb_scatter_kernel) and the tile sort reads contiguous tiles.  Local needs no oversized
// sub-bucket and at most kMaxPieces chunks per bucket; otherwise the scatter path runs (on the
// locally partitioned keys, if the local pass already ran: still the same buckets).
// The context's side stream and its two events (created on first use).
static int side_stream(dsort_ctx *ctx) {
    if (!ctx->side && hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking) != hipSuccess)
        return set_err(ctx, DSORT_EHIP, "hipStreamCreate");
    if (!ctx->side_ev && hipEventCreateWithFlags(&ctx->side_ev, hipEventDisableTiming) != hipSuccess)
        return set_err(ctx, DSORT_EHIP, "hipEventCreate");
    if (!ctx->ready_ev && hipEventCreateWithFlags(&ctx->ready_ev, hipEventDisableTiming) != hipSuccess)
        return set_err(ctx, DSORT_EHIP, "hipEventCreate");
    return DSORT_OK;
}

// The local path's sub-buckets above a tile (sb_scan_kernel<true>: each cut by chunks into the
// tiles [tile0, tile0 + nt), sorted by the tile sort into consecutive output ranges): every one's
// runs merged by the k-way pass kernels into tmp, then copied back.  Sets merge_passes to the
// deepest such merge and sub_split_subbuckets to their number.
template <typename T>
static int merge_split_subbuckets(dsort_ctx *ctx, const sb::Ovf *d_ovf, uint32_t novf, const sb::GTile *d_tiles,
                                  T *d_keys, hipStream_t s) {
    using namespace sb;
    std::vector<Ovf> ov(novf);
    DSORT_HIP(ctx, hipMemcpyAsync(ov.data(), d_ovf, novf * sizeof(Ovf), hipMemcpyDeviceToHost, s));
    if (int rc_ = sync_stream(ctx, s, "sort stream")) return rc_;
    // the merge output goes to a buffer of its own (the sort's source may still hold keys: the bucket
    // exchange's later waves), then back
    uint64_t mx = 0;
    for (const Ovf &o : ov) mx = o.len > mx ? o.len : mx;
    if (int rc_ = ensure(ctx, &ctx->stmp, &ctx->stmp_bytes, mx * sizeof(T) + 16, "split sub-bucket merge")) return rc_;
    T *tmp = static_cast<T *>(ctx->stmp);
    int lv = 0;
    for (const Ovf &o : ov) {
        std::vector<GTile> gt(o.nt);
        DSORT_HIP(ctx, hipMemcpyAsync(gt.data(), d_tiles + o.tile0, o.nt * sizeof(GTile), hipMemcpyDeviceToHost, s));
        if (int rc_ = sync_stream(ctx, s, "sort stream")) return rc_;
        std::vector<size_t> runs(o.nt);
        uint64_t tot = 0;
        for (uint32_t i = 0; i < o.nt; ++i) {
            runs[i] = gt[i].valid;
            tot += gt[i].valid;
        }
        if (tot != o.len || (o.nt && gt[0].base != o.start))
            return set_err(ctx, DSORT_EHIP, "split sub-bucket: tile records do not cover it");
        int rc = wave_merge<T>(ctx, d_keys + o.start, runs.data(), (int)runs.size(), tmp, s, true);
        if (rc) return rc;
        DSORT_HIP(ctx, hipMemcpyAsync(d_keys + o.start, tmp, o.len * sizeof(T), hipMemcpyDeviceToDevice, s));
        int l = 0;
        for (uint64_t r = runs.size(); r > 1; r = ceil_div(r, (uint64_t)1 << WG<T>::MAXLOGF)) ++l;
        lv = l > lv ? l : lv;
    }
    ctx->stats.merge_passes = lv;
    ctx->stats.sub_split_subbuckets = (int)novf;
    return DSORT_OK;
}

// Where the second level's buckets lie in its source (sub_sort): nullptr -- bucket b is
// src[hb[b], hb[b+1]), the first level's own output; or a PieceMap -- bucket b is the
// concatenation of pieces p[first[b] .. first[b+1]) (the multi-GPU path: one piece per sending
// rank in the receive buffer), and pure buckets are written as their one key.
struct SrcPiece {
    uint64_t src, len;
};
template <typename T>
struct PieceMap {
    std::vector<SrcPiece> p;
    std::vector<uint32_t> first;  // B + 1
    std::vector<T> pure_key;      // B: the key of a pure bucket
};
// Fill of output ranges with one key (pure buckets of the multi-GPU path): segment blockIdx.y.
template <typename T>
struct FillSeg {
    uint64_t dst, len;
    T key;
};
// 16-byte stores from the segment's first 16-byte boundary (the keys before it and the ones after
// the last whole vector by the first threads of block 0), FILL_U stores in flight per thread.  (One
// key per lane and store: 4 GB of C4's pure buckets at 3 TB/s.)
constexpr int FILL_U = 8;
template <typename T>
__global__ void __launch_bounds__(256) fill_segments_kernel(T *out, const FillSeg<T> *segs) {
    using V = typename std::conditional<sizeof(T) == 4, int4, longlong2>::type;
    constexpr int N = 16 / (int)sizeof(T);
    const FillSeg<T> f = segs[blockIdx.y];
    T *p = out + f.dst;
    const uint64_t h = ((16 - ((uintptr_t)p & 15)) & 15) / sizeof(T);
    const uint64_t head = h < f.len ? h : f.len;
    const uint64_t nv = (f.len - head) / N, t0 = head + nv * N;
    if (blockIdx.x == 0 && threadIdx.x < head) p[threadIdx.x] = f.key;
    if (blockIdx.x == 0 && threadIdx.x < f.len - t0) p[t0 + threadIdx.x] = f.key;
    V v;
    T *vk = reinterpret_cast<T *>(&v);
#pragma unroll
    for (int j = 0; j < N; ++j) vk[j] = f.key;
    V *q = reinterpret_cast<V *>(p + head);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * FILL_U + threadIdx.x; i < nv; i += (uint64_t)gridDim.x * 256 * FILL_U) {
#pragma unroll
        for (int u = 0; u < FILL_U; ++u)
            if (i + (uint64_t)u * 256 < nv) q[i + (uint64_t)u * 256] = v;
    }
}

template <typename T>
static int sub_sort(dsort_ctx *ctx, T *src, T *d_keys, uint64_t n, const uint64_t *hb, int B, uint64_t m_in,
                    hipStream_t s, bool timed, bool local, const uint8_t *pure, bool pure_done, const void *bspl,
                    bool retry = false, const PieceMap<T> *pm = nullptr, const T *fill_keys = nullptr) {
    using namespace sb;
    // The tile: int32 buckets above 2M keys take 16384-key tiles -- their sub-buckets (at most
    // SB_MAXS per bucket) would average above a quarter of an 8192-key tile, and sampled 8 per
    // sub-bucket many would overflow it (a 2^29-key rank of C3 has 4M-key buckets: 115 ms of split
    // merges per sort on 8192-key tiles).  The nominal sub-bucket (DSORT_OPT_SUB_KEYS unset): 3/16 of
    // an 8192-key tile, an eighth of a 16384-key one.
    uint64_t maxlen = 0;
    for (int b = 0; b < B; ++b)
        if (!pure[b]) maxlen = std::max<uint64_t>(maxlen, hb[b + 1] - hb[b]);
    const int TILE = sizeof(T) == 4 && maxlen > (uint64_t)SB_MAXS * TILE_OF<T> / 4 ? TILE_W<16> : TILE_OF<T>;
    const uint64_t m = ctx->opt.sub_keys < 0 && TILE != TILE_OF<T> ? (uint64_t)TILE / 8 : m_in;
    ctx->stats.tile_keys = TILE;
    constexpr uint64_t ALIGN = KPC<T>;
    const bool asked_local = local;
    const uint64_t LCH = SB_LCH<T>;
    // chunks of bucket b at chunk size ch
    auto bucket_chunks = [&](int b, uint64_t ch) -> uint64_t {
        if (pure[b]) return 0;
        if (!pm) return ceil_div(hb[b + 1] - hb[b], ch);
        uint64_t c = 0;
        for (uint32_t q = pm->first[b]; q < pm->first[b + 1]; ++q) c += ceil_div(pm->p[q].len, ch);
        return c;
    };
    for (int b = 0; b < B && local; ++b)
        if (bucket_chunks(b, LCH) > (uint64_t)kMaxPieces<T>) local = false;
    if (reinterpret_cast<uintptr_t>(src) % 16) local = false;  // (the gather reads aligned 16-byte vectors)
    if (asked_local && !local) ctx->stats.sub_scatter_fallback = 1;
    const uint64_t CH = local ? SB_LCH<T> : SB_CH<T>;
    // samples per sub-bucket; a bucket's samples (<= SB_MAXS * 8) fit one int64 tile
    constexpr int kMaxOs = TILE_OF<int64_t> / SB_MAXS;
    // (nominal sub-buckets above an eighth of a tile -- the default 3/16 -- sample at the maximum
    // rate: at 4 samples 10 of 16 sorts of 2^30 int32 met a sub-bucket above a tile, each costing
    // 0.1-0.7 ms of split merge)
    int os = ctx->opt.sub_os > 0 ? (ctx->opt.sub_os < kMaxOs ? (int)ctx->opt.sub_os : kMaxOs)
                                 : (m > (uint64_t)TILE / 8 ? kMaxOs : 4);
    // buckets so large that even SB_MAXS sub-buckets average above the nominal size (and above an
    // eighth of a tile): sample at the maximum rate, so the size spread (about 1/sqrt(os)) keeps
    // every sub-bucket below a tile
    // (at a quarter tile and os = 4, about one sort in 30 of two 3.3M-key buckets met a sub-bucket
    // above a tile and took the scatter path)
    if (ctx->opt.sub_os <= 0)
        for (int b = 0; b < B; ++b)
            if (!pure[b] && hb[b + 1] - hb[b] > (uint64_t)SB_MAXS * std::max<uint64_t>(m, TILE / 8)) os = kMaxOs;
    // bucket and chunk tables
    std::vector<BInfo> bi((size_t)B);
    uint64_t nsmp = 0, nch = 0, nsubs = 0;
    int SS = 1;
    // local path: the piece tables' stride (most chunks of a bucket) and a bound on the tiles -- a
    // greedy packing's consecutive tiles hold more than a tile's room together, so a bucket of len
    // keys takes at most 2 len / room + 1 tiles
    uint32_t PS = 1;
    uint64_t tcap = 0;
    for (int b = 0; b < B; ++b) {
        const uint64_t len = pure[b] ? 0 : hb[b + 1] - hb[b];  // (a pure bucket: no chunks, no tiles)
        uint64_t ns = len <= (uint64_t)TILE ? 1 : ceil_div(len, m);
        ns = ns > (uint64_t)SB_MAXS ? SB_MAXS : ns;
        const uint64_t nc = bucket_chunks(b, CH);
        if (local && len) {
            PS = nc > PS ? (uint32_t)nc : PS;
            // (+ 8: the split tiles of a rare sub-bucket above a tile -- sub-buckets split by chunks
            // add up to one tile each beyond the bound; nominal sub-buckets above half a tile
            // (DSORT_OPT_SUB_KEYS) make that every one of them.  Beyond the tables the sort takes
            // the scatter path.)
            const uint64_t room = (uint64_t)TILE - 2 * (ALIGN - 1) * nc;
            tcap += 2 * len / room + 1 + 8 + (2 * m > room ? ns : 0);
        }
        bi[b] = BInfo{hb[b], nsmp, (uint32_t)len, (uint32_t)ns, ns > 1 ? (uint32_t)(ns * os) : 0u, (uint32_t)nch,
                      (uint32_t)(nch + nc), retry ? 1u : 0u, pm ? 1u : 0u};
        nsmp += bi[b].ns;
        nch += nc;
        nsubs += ns;
        SS = (int)ns > SS ? (int)ns : SS;
    }
    SS = (SS + 63) & ~63;
    if (ctx->opt.test_tile_cap > 0) tcap = std::min<uint64_t>(tcap, (uint64_t)ctx->opt.test_tile_cap);
    // local path, int32: the sub-bucket totals added up by sb_local_kernel's atomics (sb_scan 126 -> 91 us,
    // sb_local +10 us at 2^30); int64 sums the prefix rows in sb_scan (C4: the atomics cost sb_local
    // about as much as they saved, profiles/r5_ab_sub_scan.log)
    constexpr bool SUB_TOTALS = DSORT_SUB_TOTALS && sizeof(T) == 4;
    // tiles, bound (sb_scan_kernel); the local path's split tiles: tcap
    const uint64_t tmax = std::max<uint64_t>(nsubs + ceil_div(n, TILE) + (uint64_t)B, local ? tcap : 0);
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    const size_t o_bi = take(B * sizeof(BInfo)), o_ch = take(nch * sizeof(Chunk)), o_smp = take(nsmp * sizeof(T)),
                 o_cmp = take(nsmp * 8), o_srt = take(sizeof(T) == 8 ? nsmp * 8 : 0),
                 o_spl = take((size_t)B * SS * sizeof(Spl<T>)),
                 o_rng = take((size_t)B * SB_SLOTS * 4), o_sfn = take(B * sizeof(SlotFn<T>)),
                 o_cnt = take(nch * (SS + 1) * 4), o_offs = take(local ? 0 : nch * SS * 4),
                 o_tt = take(tmax * sizeof(GTile)),
                 o_ovf = take(nsubs * sizeof(Ovf)), o_num = take(8), o_stl = take(B * sizeof(bk::TileRef) + 16),
                 o_pcs = take(local ? tcap * PS * sizeof(uint2) : 0),
                 o_fill = take(pm || fill_keys ? B * sizeof(FillSeg<T>) : 0),
                 o_tot = take(local && SUB_TOTALS ? (size_t)B * SS * 4 : 0);
    int rc = ensure(ctx, &ctx->sub, &ctx->sub_bytes, off, "sub-bucket partition");
    if (rc) return rc;
    char *a = static_cast<char *>(ctx->sub);
    BInfo *dbi = reinterpret_cast<BInfo *>(a + o_bi);
    Chunk *dch = reinterpret_cast<Chunk *>(a + o_ch);
    T *smp = reinterpret_cast<T *>(a + o_smp);
    int64_t *cmp = reinterpret_cast<int64_t *>(a + o_cmp), *srt = reinterpret_cast<int64_t *>(a + o_srt);
    Spl<T> *spl = reinterpret_cast<Spl<T> *>(a + o_spl);
    uint32_t *rng = reinterpret_cast<uint32_t *>(a + o_rng);
    SlotFn<T> *sfn = reinterpret_cast<SlotFn<T> *>(a + o_sfn);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(a + o_cnt), *offs = reinterpret_cast<uint32_t *>(a + o_offs);
    void *tt = a + o_tt;  // GTile (local) or TileRef (scatter)
    Ovf *ovf = reinterpret_cast<Ovf *>(a + o_ovf);
    uint32_t *num = reinterpret_cast<uint32_t *>(a + o_num);  // tiles, merge records
    bk::TileRef *stl = reinterpret_cast<bk::TileRef *>(a + o_stl);  // sample tiles, then their count
    uint2 *pcs = reinterpret_cast<uint2 *>(a + o_pcs);                // local path: piece tables
    uint32_t *stot = local && SUB_TOTALS ? reinterpret_cast<uint32_t *>(a + o_tot) : nullptr;  // sub-bucket totals
    // pinned staging: the two tables, the sample tiles + count, then the two counters read back
    const size_t h_ch = (B * sizeof(BInfo) + 15) & ~(size_t)15, h_stl = h_ch + nch * sizeof(Chunk);
    const size_t h_num = h_stl + B * sizeof(bk::TileRef) + 16;
    const size_t h_fill = h_num + 16;
    const size_t hbytes = h_fill + (pm || fill_keys ? B * sizeof(FillSeg<T>) : 0);
    if (!ctx->sub_ev && hipEventCreateWithFlags(&ctx->sub_ev, hipEventDisableTiming) != hipSuccess)
        return set_err(ctx, DSORT_EHIP, "hipEventCreate");
    if (int rc_ = sync_event(ctx, ctx->sub_ev, "tile count")) return rc_;  // the previous call's read-back is done with the staging
    if (ctx->sub_host_bytes < hbytes) {  // (after that wait: the previous call's uploads are done with it)
        release_host(ctx, ctx->sub_host);
        ctx->sub_host = nullptr;
        ctx->sub_host_bytes = 0;
        DSORT_HIP(ctx, hipHostMalloc(&ctx->sub_host, hbytes, hipHostMallocDefault));
        ctx->sub_host_bytes = hbytes;
    }
    char *h = static_cast<char *>(ctx->sub_host);
    std::memcpy(h, bi.data(), B * sizeof(BInfo));
    Chunk *hc = reinterpret_cast<Chunk *>(h + h_ch);
    for (int b = 0; b < B; ++b) {
        if (!bi[b].len) continue;
        if (!pm) {
            for (uint64_t o = 0; o < bi[b].len; o += CH)
                *hc++ = Chunk{bi[b].start + o, (uint32_t)(bi[b].len - o < CH ? bi[b].len - o : CH), (uint32_t)b,
                              (uint32_t)o, 0u};
            continue;
        }
        uint64_t boff = 0;  // the bucket's pieces in order, each cut into chunks
        for (uint32_t q = pm->first[b]; q < pm->first[b + 1]; ++q) {
            const SrcPiece &pc = pm->p[q];
            for (uint64_t o = 0; o < pc.len; o += CH, boff += CH)
                *hc++ = Chunk{pc.src + o, (uint32_t)(pc.len - o < CH ? pc.len - o : CH), (uint32_t)b, (uint32_t)boff, 0u};
            boff -= ceil_div(pc.len, CH) * CH - pc.len;  // (the last chunk of a piece may be short)
        }
    }
    // pure buckets of a piece map, or whose keys the first-level scatter dropped (fill_keys): their
    // one key written over their output range
    FillSeg<T> *hf = reinterpret_cast<FillSeg<T> *>(h + h_fill);
    uint32_t nfill = 0;
    uint64_t maxfill = 0;
    for (int b = 0; (pm || fill_keys) && b < B; ++b)
        if (pure[b] && hb[b + 1] > hb[b]) {
            hf[nfill++] = FillSeg<T>{hb[b], hb[b + 1] - hb[b], pm ? pm->pure_key[b] : fill_keys[b]};
            maxfill = std::max(maxfill, hb[b + 1] - hb[b]);
        }
    bk::TileRef *hst = reinterpret_cast<bk::TileRef *>(h + h_stl);
    uint32_t nst = 0;
    for (int b = 0; b < B; ++b)
        if (bi[b].ns) hst[nst++] = bk::TileRef{bi[b].soff, bi[b].ns, 0};
    *reinterpret_cast<uint32_t *>(hst + B) = nst;
    // The tables go up on a side stream, so the copies run while the first-level scatter (queued
    // on s before this point) is still running; s waits for them before the first kernel that
    // reads them.  (On s they queued behind the scatter: about 60 us of idle GPU per sort at 2^30.)
    // Nothing still reads the arena: the host got here after waiting for the histogram of this
    // sort, which follows every kernel of the previous sort on s.
    if ((rc = side_stream(ctx))) return rc;
    DSORT_HIP(ctx, hipMemcpyAsync(dbi, h, B * sizeof(BInfo), hipMemcpyHostToDevice, ctx->side));
    if (nch) DSORT_HIP(ctx, hipMemcpyAsync(dch, h + h_ch, nch * sizeof(Chunk), hipMemcpyHostToDevice, ctx->side));
    DSORT_HIP(ctx, hipMemcpyAsync(stl, hst, B * sizeof(bk::TileRef) + 16, hipMemcpyHostToDevice, ctx->side));
    DSORT_HIP(ctx, hipMemsetAsync(num, 0, 8, ctx->side));
    if (nfill)
        DSORT_HIP(ctx, hipMemcpyAsync(a + o_fill, hf, nfill * sizeof(FillSeg<T>), hipMemcpyHostToDevice, ctx->side));
    DSORT_HIP(ctx, hipEventRecord(ctx->side_ev, ctx->side));
    DSORT_HIP(ctx, hipStreamWaitEvent(s, ctx->side_ev, 0));
    uint64_t npure = 0;
    for (int b = 0; b < B; ++b) npure += pure[b] ? hb[b + 1] - hb[b] : 0;
    ctx->stats.tile_sort_keys = n - npure;
    // pure buckets (one key) to the output as they lie, runs of them in one copy (unless the
    // scatter wrote them there); a piece map's pure buckets are filled with their key
    if (nfill) {
        const unsigned gx = (unsigned)std::min<uint64_t>(ceil_div(maxfill, 256 * FILL_U * (16 / sizeof(T))), 1024);
        hipLaunchKernelGGL(fill_segments_kernel<T>, dim3(gx, nfill), dim3(256), 0, s, d_keys,
                           reinterpret_cast<const FillSeg<T> *>(a + o_fill));
        DSORT_HIP(ctx, hipGetLastError());
    }
    for (int b = 0; b < B && !pure_done && !pm;) {
        if (!pure[b]) {
            ++b;
            continue;
        }
        int e = b;
        while (e < B && pure[e]) ++e;
        if (hb[e] > hb[b])
            DSORT_HIP(ctx, hipMemcpyAsync(d_keys + hb[b], src + hb[b], (hb[e] - hb[b]) * sizeof(T),
                                          hipMemcpyDeviceToDevice, s));
        b = e;
    }
    // 1. splitters of every bucket from a regular sample.  A bucket's samples fit one int64 tile,
    // so the tile sort alone sorts them, one workgroup per bucket.
    if (nsmp) {
        hipLaunchKernelGGL(sb_sample_kernel<T>, dim3((unsigned)B), dim3(SB_T), 0, s, src, dbi, dch, smp, cmp);
        DSORT_HIP(ctx, hipGetLastError());
        const uint4 *stl4 = reinterpret_cast<const uint4 *>(stl);
        const uint32_t *pnst = reinterpret_cast<const uint32_t *>(stl + B);
        if constexpr (sizeof(T) == 8) {  // int64: sort the keys, rank them, then the composites
            rc = tile_sort<int64_t, false>(ctx, smp, srt, nsmp, stl4, pnst, sb::Gather{}, nst, s, false);
            if (rc) return rc;
            hipLaunchKernelGGL(sb_rank_kernel, dim3((unsigned)B), dim3(SB_T), 0, s, smp, srt, dbi, cmp);
        }
        rc = tile_sort<int64_t, false>(ctx, cmp, cmp, nsmp, stl4, pnst, sb::Gather{}, nst, s, false);
        if (rc) return rc;
        hipLaunchKernelGGL(sb_splitter_kernel<T>, dim3((unsigned)B), dim3(SB_MAXS), 0, s, cmp, smp, dbi, dch, os, SS, spl,
                           rng, sfn, stot);
        DSORT_HIP(ctx, hipGetLastError());
    } else if (stot) {
        DSORT_HIP(ctx, hipMemsetAsync(stot, 0, (size_t)B * SS * 4, s));
    }
    const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(d_keys) / sizeof(T)) & (ALIGN - 1));
    uint32_t *hn = reinterpret_cast<uint32_t *>(h + h_num);
    if (local) {
        // 2. every chunk partitioned in place (cnt = the prefix tables), sub-bucket starts, tiles
        if (nch) {
            if ((rc = stage_event(ctx, s, timed, 13))) return rc;
            hipLaunchKernelGGL(sb_local_kernel<T>, dim3((unsigned)nch), dim3(SB_LT<T>), 0, s, src, dch, dbi, SS, spl, rng,
                               sfn, cnt, ctx->bk_hot, stot);
            DSORT_HIP(ctx, hipGetLastError());
            if ((rc = stage_event(ctx, s, timed, 14))) return rc;
        }
        // (the piece tables inside the scan with many buckets; with few, a kernel of their own)
#ifndef DSORT_PIECES_SCAN_MINB
#define DSORT_PIECES_SCAN_MINB 256
#endif
        const bool pieces_in_scan = B >= DSORT_PIECES_SCAN_MINB;
        hipLaunchKernelGGL(sb_scan_kernel<true>, dim3((unsigned)B), dim3(SB_MAXS), 0, s, dbi, SS, cnt, nullptr, TILE, 1,
                           0u, (uint32_t)(2 * (ALIGN - 1)), tt, num, ovf, num + 1, (uint32_t)tmax,
                           static_cast<const Chunk *>(dch), pieces_in_scan ? pcs : nullptr, PS, (uint32_t)tcap, stot);
        DSORT_HIP(ctx, hipGetLastError());
        const Gather ga{static_cast<const GTile *>(tt), dch, dbi, cnt, pcs, PS, SS, spl, bspl, B,
                        (uint32_t)std::max<uint64_t>(tcap, 1)};
        // (few buckets, round 6: the piece tables' kernel goes out before the tile count is read
        // back, on a grid for the tile tables' capacity -- its workgroups past the count return at
        // once -- so the early tile sort can follow it and the host's wait for the count runs under
        // both: a C3 rank's two waves each idled the GPU ~40 us between the scan and the tile sort)
#ifndef DSORT_PIECES_EARLY
#define DSORT_PIECES_EARLY 1
#endif
        const bool pieces_early = DSORT_PIECES_EARLY && !pieces_in_scan && pcs && tcap > 0;
        if (pieces_early) {
            hipLaunchKernelGGL(sb_pieces_kernel, dim3((unsigned)ceil_div(tcap, 4)), dim3(256), 0, s,
                               static_cast<const GTile *>(tt), num, static_cast<const Chunk *>(dch), cnt, SS, pcs, PS,
                               (uint32_t)tcap);
            DSORT_HIP(ctx, hipGetLastError());
        }
        DSORT_HIP(ctx, hipMemcpyAsync(hn, num, 8, hipMemcpyDeviceToHost, s));
        DSORT_HIP(ctx, hipEventRecord(ctx->sub_ev, s));
        // The tile sort of the first `early` tiles goes out behind the count's read-back, before the
        // host waits for it: every tile holds at most TILE keys, so there are at least (keys in
        // tiles) / TILE of them.  The rest follow the count (at 2^30 int32 ~15 % of the tiles), and
        // the wait -- the read-back, then the launch -- runs under the first part instead of idling
        // the GPU (about 35 us per sort).  (With the piece tables made by the scan, or by their own
        // kernel on a grid for the tables' capacity, pieces_early.  Not under a stage-1 kill point, which must see
        // the second level finished and nothing after it.)
#ifndef DSORT_TILE_EARLY
#define DSORT_TILE_EARLY 1
#endif
        const uint64_t ebound = (n - npure) / (uint64_t)TILE;
        const uint32_t early = DSORT_TILE_EARLY && (pieces_in_scan || pieces_early) && ctx->opt.kill_after_pass != 1
                                   ? (uint32_t)std::min<uint64_t>(ebound, tcap)
                                   : 0u;
        if (early) {
            if ((rc = tile_sort_event(ctx, s, timed, 0))) return rc;
            rc = with_tile_waves<T>(ctx, TILE, [&](auto w) {
                return tile_sort_begin<T, true, decltype(w)::value>(ctx, src, d_keys, n, nullptr, num, ga, early,
                                                                    (uint32_t)tcap, s);
            });
            if (rc) return rc;
        }
        // (the tile count sizes the grid: a grid at its bound, 9x the tiles at 2^30 int32, cost
        // more in empty workgroups than this wait -- measured 10.6 vs 10.1 ms)
        if (int rc_ = sync_event(ctx, ctx->sub_ev, "tile count")) return rc_;
        const uint32_t ntiles = hn[0], novf = hn[1];
        // Beyond the tile tables (only when many sub-buckets were split): the scatter path over the
        // partitioned chunks -- its sample takes single keys, since a run of adjacent keys now lies
        // in one sub-bucket of this attempt.
        if (ntiles > tmax || ntiles > tcap) {
            // (the early tile sort still reads the tables the scatter path's side-stream uploads
            // overwrite: it finishes first -- its output is rewritten by that path)
            if (early)
                if (int rc_ = sync_stream(ctx, s, "early tile sort")) return rc_;
            ctx->stats.sub_scatter_fallback = 1;
            // (fill_keys passed on: the retry fills the dropped pure buckets itself instead of relying
            // on this attempt's queued fill -- ADVICE r5)
            return sub_sort<T>(ctx, src, d_keys, n, hb, B, m, s, timed, false, pure, pure_done, bspl, true, pm,
                               fill_keys);
        }
        // every tile's piece table
        if (ntiles && !pieces_in_scan && !pieces_early) {
            hipLaunchKernelGGL(sb_pieces_kernel, dim3((unsigned)ceil_div(ntiles, 4)), dim3(256), 0, s,
                               static_cast<const GTile *>(tt), num, static_cast<const Chunk *>(dch), cnt, SS, pcs, PS,
                               (uint32_t)tcap);
            DSORT_HIP(ctx, hipGetLastError());
        }
        fault_point(ctx, s, 1);  // second-level partition done
        ctx->stats.merge_passes = 0;
        // 3. tile sort: gathered from the chunks into d_keys
        if (early) {  // (ntiles >= early)
            rc = with_tile_waves<T>(ctx, TILE, [&](auto w) {
                constexpr int W = decltype(w)::value;
                int r = tile_sort_more<T, true, W>(ctx, src, d_keys, n, nullptr, num, ga, early,
                                                   ntiles > early ? ntiles - early : 0u, (uint32_t)tcap, s);
                return r ? r : tile_sort_end<T, true, W>(ctx, src, d_keys, n, nullptr, num, ga, ntiles, (uint32_t)tcap, s);
            });
            if (rc) return rc;
            if ((rc = tile_sort_event(ctx, s, timed, 1))) return rc;
        } else if (ntiles) {
            rc = tile_sort<T, true>(ctx, src, d_keys, n, nullptr, num, ga, ntiles, s, timed, TILE);
            if (rc) return rc;
        }
        if ((rc = stage_event(ctx, s, timed, 1))) return rc;
        fault_point(ctx, s, 2);  // tile sort done (a split sub-bucket's merge follows)
        // sub-buckets above a tile (a sampling outlier): their split tiles' outputs merged (src,
        // read by the tile sort, is free scratch now)
        if (novf) {
            rc = merge_split_subbuckets<T>(ctx, ovf, novf, static_cast<const GTile *>(tt), d_keys, s);
            if (rc) return rc;
        }
        if (timed && ctx->ev_ok) {
            DSORT_HIP(ctx, hipEventRecord(ctx->ev[ctx->ev_done], s));
            ctx->ev_mask |= 1u << ctx->ev_done;
        }
        return DSORT_OK;
    }
    // 2. histograms, sub-bucket starts, tiles
    if (nch) {
        if ((rc = stage_event(ctx, s, timed, 13))) return rc;
        hipLaunchKernelGGL(sb_hist_kernel<T>, dim3((unsigned)nch), dim3(SB_T), 0, s, src, dch, dbi, SS, spl, rng,
                           sfn, cnt);
        DSORT_HIP(ctx, hipGetLastError());
    }
    hipLaunchKernelGGL(sb_scan_kernel<false>, dim3((unsigned)B), dim3(SB_MAXS), 0, s, dbi, SS, cnt, offs, TILE,
                       (int)ALIGN, mis, 0u, tt, num, ovf, num + 1, (uint32_t)tmax, nullptr, nullptr, 0u, 0u, nullptr);
    DSORT_HIP(ctx, hipGetLastError());
    DSORT_HIP(ctx, hipMemcpyAsync(hn, num, 8, hipMemcpyDeviceToHost, s));
    DSORT_HIP(ctx, hipEventRecord(ctx->sub_ev, s));
    // 3. scatter into d_keys (the host reads the tile count meanwhile), tile sort in place
    if (nch) {
        hipLaunchKernelGGL(sb_scatter_kernel<T>, dim3((unsigned)nch), dim3(SB_T), 0, s, src, d_keys, dch,
                           (uint32_t)nch, dbi, SS, spl, rng, sfn, offs);
        DSORT_HIP(ctx, hipGetLastError());
        if ((rc = stage_event(ctx, s, timed, 14))) return rc;
    }
    if (int rc_ = sync_event(ctx, ctx->sub_ev, "tile count")) return rc_;
    const uint32_t ntiles = hn[0], novf = hn[1];
    if (ntiles > tmax || novf > nsubs) return set_err(ctx, DSORT_EHIP, "sub-bucket packing overflow");
    fault_point(ctx, s, 1);  // second-level partition done
    ctx->stats.merge_passes = 0;
    if (ntiles) {
        rc = tile_sort<T, false>(ctx, d_keys, d_keys, n, static_cast<const uint4 *>(tt), num, Gather{}, ntiles, s,
                                 timed, TILE);
        if (rc) return rc;
    }
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[1], s));
        ctx->ev_mask |= 2u;
    }
    fault_point(ctx, s, 2);  // tile sort done (the oversized sub-buckets' merges follow)
    // 4. oversized sub-buckets: their tile-sorted pieces merged into a buffer of their own, then
    //    copied back.  (Not into src: in the bucket exchange src is the partition buffer, which
    //    still holds this rank's later waves' buckets and, over RCCL, buckets the comm stream is
    //    still sending -- as merge_split_subbuckets does on the local path.)
    if (novf) {
        std::vector<Ovf> ov(novf);
        DSORT_HIP(ctx, hipMemcpyAsync(ov.data(), ovf, novf * sizeof(Ovf), hipMemcpyDeviceToHost, s));
        if (int rc_ = sync_stream(ctx, s, "sort stream")) return rc_;
        uint64_t mx = 0;
        for (const Ovf &o : ov) mx = o.len > mx ? o.len : mx;
        if (int rc_ = ensure(ctx, &ctx->stmp, &ctx->stmp_bytes, mx * sizeof(T) + 16, "oversized sub-bucket merge"))
            return rc_;
        // (the merge output keeps the sub-bucket's misalignment inside a 16-byte chunk)
        T *tmp = static_cast<T *>(ctx->stmp);
        int lv = 0;
        for (const Ovf &o : ov) {
            const std::vector<size_t> runs = sub_tile_runs(o.start, o.len, TILE, ALIGN, mis);
            T *to = tmp + ((o.start + mis) & (ALIGN - 1));
            rc = wave_merge<T>(ctx, d_keys + o.start, runs.data(), (int)runs.size(), to, s, true);
            if (rc) return rc;
            DSORT_HIP(ctx, hipMemcpyAsync(d_keys + o.start, to, o.len * sizeof(T), hipMemcpyDeviceToDevice, s));
            int l = 0;
            for (uint64_t r = runs.size(); r > 1; r = ceil_div(r, (uint64_t)1 << WG<T>::MAXLOGF)) ++l;
            lv = l > lv ? l : lv;
        }
        ctx->stats.merge_passes = lv;
        ctx->stats.sub_split_subbuckets = (int)novf;
    }
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[ctx->ev_done], s));
        ctx->ev_mask |= 1u << ctx->ev_done;
    }
    return DSORT_OK;
}

// The first level's device arena (ctx->bucket): the splitter samples (their layout is the
// caller's: smp_bytes), splitters, per-workgroup counts, chunk sums, offsets, bucket starts, the
// tile table of the merge path, the slot map.
template <typename T>
struct BkLayout {
    using C = typename bk::Comp<T>::C;
    int B, BP, subs;
    uint64_t G, nchunk, tmax;
    char *smp;
    C *spl;
    uint32_t *cnt, *offs, *ntl;
    uint64_t *part, *bst;
    uint64_t *cst;  // the bucket exchange's compacted starts (pure buckets of size 0, bucket_scan_kernel)
    bk::TileRef *tt;
    bk::BkMap *map;
    uint32_t *ids;  // every key's bucket (bk::BkIds: 2 or 3 per word), else null
};
template <typename T>
static int bk_layout(dsort_ctx *ctx, uint64_t n, int B, size_t smp_bytes, BkLayout<T> &L) {
    using namespace bk;
    using C = typename Comp<T>::C;
    L.B = B;
    L.BP = 1 << ceil_log2((uint64_t)B);
    L.subs = bucket_wg_subs<T>(n);
    L.G = ceil_div(n ? n : 1, (uint64_t)L.subs * BK_T * Geo<T>::KPT);
    L.nchunk = ceil_div(L.G, BK_CHUNK);
    L.tmax = ceil_div(n, TILE_OF<T>) + 2 * (uint64_t)B;  // + a head and a tail per bucket
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    const size_t o_smp = take(smp_bytes), o_spl = take((size_t)L.BP * sizeof(C)), o_cnt = take((size_t)L.G * B * 4),
                 o_part = take((size_t)L.nchunk * B * 8 + (size_t)BK_MAXB * 8), o_offs = take((size_t)L.G * B * 4),
                 o_bst = take((size_t)(B + 1) * 8), o_cst = take((size_t)(B + 1) * 8), o_tt = take((size_t)L.tmax * sizeof(TileRef)), o_nt = take(4),
                 o_map = take(BK_MAP_BYTES), o_ids = take(BkIds<T>::ON ? (size_t)L.G * L.subs * BK_T * Geo<T>::KPT * 4 / BkIds<T>::PER_WORD : 0);
    int rc = ensure(ctx, &ctx->bucket, &ctx->bucket_bytes, off, "bucket partition");
    if (rc) return rc;
    char *a = static_cast<char *>(ctx->bucket);
    L.smp = a + o_smp;
    L.spl = reinterpret_cast<C *>(a + o_spl);
    L.cnt = reinterpret_cast<uint32_t *>(a + o_cnt);
    L.part = reinterpret_cast<uint64_t *>(a + o_part);
    L.offs = reinterpret_cast<uint32_t *>(a + o_offs);  // (positions mod 2^32: the scatter's index width)
    L.bst = reinterpret_cast<uint64_t *>(a + o_bst);
    L.cst = reinterpret_cast<uint64_t *>(a + o_cst);
    L.tt = reinterpret_cast<TileRef *>(a + o_tt);
    L.ntl = reinterpret_cast<uint32_t *>(a + o_nt);
    L.map = reinterpret_cast<BkMap *>(a + o_map);
    L.ids = BkIds<T>::ON ? reinterpret_cast<uint32_t *>(a + o_ids) : nullptr;
    // starts, then the splitters, then the slot map (int32 reads its choice back)
    const size_t hbytes = (size_t)(BK_MAXB + 1) * 8 + (size_t)BK_MAXB * 16 + sizeof(BkMap);
    if (ctx->bucket_host_bytes < hbytes) {
        release_host(ctx, ctx->bucket_host);
        ctx->bucket_host = nullptr;
        ctx->bucket_host_bytes = 0;
        DSORT_HIP(ctx, hipHostMalloc(&ctx->bucket_host, hbytes, hipHostMallocDefault));
        ctx->bucket_host_bytes = hbytes;
    }
    if (!ctx->bucket_ev && hipEventCreateWithFlags(&ctx->bucket_ev, hipEventDisableTiming) != hipSuccess)
        return set_err(ctx, DSORT_EHIP, "hipEventCreate");
    return DSORT_OK;
}

// The first level once the splitters are in L.spl: slot map, histograms, their scan, the scatter of
// d_in into part_out (pure buckets into `direct` when not null).  On return the host holds the
// bucket starts hb[0..B] and the splitters hspl[0..B-2] (it waits for them while the scatter runs).
// ioff = the composite index of d_in[0].  `tile` != 0: also the merge path's tile table.
// compact (the bucket exchange): the keys of pure buckets are dropped and part_out holds the others
// at the compacted starts (bucket_scan_kernel); hb stays the real starts.
template <typename T>
static int first_level(dsort_ctx *ctx, const T *d_in, uint64_t n, uint64_t ioff, T *part_out, T *direct,
                       const BkLayout<T> &L, uint32_t tile, hipStream_t s, bool timed, uint64_t *&hb,
                       typename bk::Comp<T>::C *&hspl, bool compact = false) {
    using namespace bk;
    using C = typename Comp<T>::C;
    const int B = L.B, BP = L.BP;
    int rc;
    hb = static_cast<uint64_t *>(ctx->bucket_host);
    hspl = reinterpret_cast<C *>(hb + BK_MAXB + 1);
    hipLaunchKernelGGL(bucket_slotmap_kernel<T>, dim3(1), dim3(BK_MAXB), 0, s, L.spl, B, n, L.map);
    ctx->bk_hot = &L.map->hot;
    // int32: which map did the splitters choose -- the fixed one (packed lookup) or the adaptive
    // one (many small keys)?  Its kernels are separate instances, so the host reads the choice back
    // (launching both scatter instances and letting the other return at once would cost a grid of
    // empty workgroups, about 40 us)
    // int64 (round 5): likewise which scatter variant -- with or without the histogram's bucket ids
    // (launching both and letting the other return cost its grid of ~11 K workgroups, 48 us at C4)
#ifndef DSORT_IDS_READBACK
#define DSORT_IDS_READBACK 1
#endif
    constexpr bool RB = !Comp<T>::ADAPT || (BkIds<T>::ON && DSORT_IDS_READBACK);
    bool ad = false, ids = false;
    BkMap *hm = reinterpret_cast<BkMap *>(reinterpret_cast<char *>(hb) + (size_t)(BK_MAXB + 1) * 8 + (size_t)BK_MAXB * 16);
    if constexpr (RB) {
        DSORT_HIP(ctx, hipMemcpyAsync(hm, L.map, sizeof(BkMap), hipMemcpyDeviceToHost, s));
        DSORT_HIP(ctx, hipEventRecord(ctx->bucket_ev, s));
    }
    if ((rc = stage_event(ctx, s, timed, 9))) return rc;
    // (int32: the fixed map's histogram goes first -- it returns at once when the map is adaptive
    // -- so the GPU is busy while the host reads the map's choice; only the adaptive case launches
    // a second instance behind it)
    hipLaunchKernelGGL((bucket_hist_kernel<T, false>), dim3((unsigned)L.G), dim3(BK_T), 0, s, d_in, n, L.spl, L.map, B,
                       BP, L.subs, L.cnt, ioff, L.ids);
    if constexpr (RB) {
        if (int rc_ = sync_event(ctx, ctx->bucket_ev, "slot map")) return rc_;
        ad = !Comp<T>::ADAPT && hm->ad != 0;
        ids = BkIds<T>::ON && hm->ids != 0;
    }
    if constexpr (!Comp<T>::ADAPT) {
        if (ad)
            hipLaunchKernelGGL((bucket_hist_kernel<T, true>), dim3((unsigned)L.G), dim3(BK_T), 0, s, d_in, n, L.spl,
                               L.map, B, BP, L.subs, L.cnt, ioff, L.ids);
    }
    if ((rc = stage_event(ctx, s, timed, 10))) return rc;
    hipLaunchKernelGGL(bucket_colsum_kernel, dim3((unsigned)L.nchunk), dim3(BK_MAXB), 0, s, L.cnt, (uint32_t)L.G, B,
                       L.part);
    // (the column totals after the chunk sums: part's slack)
    uint64_t *ctot = L.part + (size_t)L.nchunk * B;
    hipLaunchKernelGGL(bucket_colscan_kernel, dim3((unsigned)ceil_div((uint64_t)B, 64)), dim3(BK_MAXB), 0, s, L.part,
                       (uint32_t)L.nchunk, B, ctot);
    hipLaunchKernelGGL(bucket_scan_kernel<T>, dim3(1), dim3(BK_MAXB), 0, s, L.part, (uint32_t)L.nchunk, B, tile,
                       (uint32_t)KPC<T>, L.bst, L.tt, L.ntl, (const uint64_t *)ctot, compact ? L.spl : nullptr, L.cst);
    hipLaunchKernelGGL(bucket_offsets_kernel<uint32_t>, dim3((unsigned)L.nchunk), dim3(BK_MAXB), 0, s, L.cnt, L.part,
                       compact ? L.cst : L.bst, (uint32_t)L.G, B, L.offs);
    if (compact) direct = part_out;  // (a pure bucket's keys are dropped by the scatter: nothing goes there)
    DSORT_HIP(ctx, hipGetLastError());
    // bucket starts to the host (the second level is planned from the bucket sizes); the host
    // waits for them while the scatter runs.  (The copies run on the side stream once the offsets
    // are written, so the scatter does not queue behind them: ~10 us of idle GPU per sort.)
    if ((rc = side_stream(ctx))) return rc;
    DSORT_HIP(ctx, hipEventRecord(ctx->ready_ev, s));
    DSORT_HIP(ctx, hipStreamWaitEvent(ctx->side, ctx->ready_ev, 0));
    DSORT_HIP(ctx, hipMemcpyAsync(hb, L.bst, (size_t)(B + 1) * 8, hipMemcpyDeviceToHost, ctx->side));
    if (B > 1) DSORT_HIP(ctx, hipMemcpyAsync(hspl, L.spl, (size_t)(B - 1) * sizeof(C), hipMemcpyDeviceToHost, ctx->side));
    if constexpr (!RB)  // (int64: the map only for the statistics)
        DSORT_HIP(ctx, hipMemcpyAsync(hm, L.map, sizeof(BkMap), hipMemcpyDeviceToHost, ctx->side));
    DSORT_HIP(ctx, hipEventRecord(ctx->bucket_ev, ctx->side));
    if ((rc = stage_event(ctx, s, timed, 11))) return rc;
#ifdef DSORT_IDS_ONLY
    if constexpr (!BkIds<T>::ON)
#endif
    {
        if constexpr (!Comp<T>::ADAPT) {
            if (ad)
                hipLaunchKernelGGL((bucket_scatter_lines_kernel<T, false, true>), dim3((unsigned)L.G), dim3(BK_T), 0, s,
                                   d_in, n, L.spl, L.map, B, BP, L.subs, L.offs, part_out, direct, ioff, L.ids);
        }
        if (!ad && !(RB && ids)) {
            if (!Comp<T>::ADAPT && RB && hm->hot)  // (int32 read the map back: runs of one bucket)
                hipLaunchKernelGGL((bucket_scatter_lines_kernel<T, false, false, true>), dim3((unsigned)L.G), dim3(BK_T), 0,
                                   s, d_in, n, L.spl, L.map, B, BP, L.subs, L.offs, part_out, direct, ioff, L.ids);
            else
                hipLaunchKernelGGL((bucket_scatter_lines_kernel<T, false, false>), dim3((unsigned)L.G), dim3(BK_T), 0, s,
                                   d_in, n, L.spl, L.map, B, BP, L.subs, L.offs, part_out, direct, ioff, L.ids);
        }
    }
    if constexpr (BkIds<T>::ON)  // (without the read-back: the variant the slot map did not choose returns at once)
        if (!RB || ids)
            hipLaunchKernelGGL((bucket_scatter_lines_kernel<T, true>), dim3((unsigned)L.G), dim3(BK_T), 0, s, d_in, n,
                               L.spl, L.map, B, BP, L.subs, L.offs, part_out, direct, ioff, L.ids);
    DSORT_HIP(ctx, hipGetLastError());
    if ((rc = stage_event(ctx, s, timed, 12))) return rc;
    fault_point(ctx, s, 0);  // first-level partition done
    if (int rc_ = sync_event(ctx, ctx->bucket_ev, "bucket starts")) return rc_;
    if (hb[B] != n) return set_err(ctx, DSORT_EHIP, "bucket partition lost keys");
    ctx->stats.first_level_map = !Comp<T>::ADAPT && !ad ? (RB && hm->r2s ? 3 : 0) : hm->mode == 0 ? 1 : 2;
    return DSORT_OK;
}

// The stats and events of a bucketed sort start after its nested splitter sort.
static int bucketed_stats_start(dsort_ctx *ctx, uint64_t n, int tile, hipStream_t s, bool timed) {
    ctx->bk_hot = nullptr;  // (set by this sort's first level, if it runs one)
    ctx->stats = fresh_stats();
    ctx->stats.keys_in = ctx->stats.keys_out = n;
    ctx->stats.tile_sort_keys = n;
    ctx->stats.tile_keys = tile;
    ctx->ev_mask = 0;
    ctx->kev_used = 0;
    ctx->last_stream = s;
    return stage_event(ctx, s, timed, 0);
}

template <typename T>
static int bucket_sort(dsort_ctx *ctx, const T *d_in, T *d_keys, size_t n, hipStream_t s, bool timed, int B) {
    using namespace bk;
    using C = typename Comp<T>::C;
    constexpr int TILE = TILE_OF<T>;
    constexpr uint64_t ALIGN = KPC<T>;
    const int os = bucket_os(ctx);
    const uint32_t S = (uint32_t)B * (uint32_t)os;
    // samples: int32 composites; int64 keys, sorted keys and composites (3 x 8 bytes)
    BkLayout<T> L;
    int rc = bk_layout<T>(ctx, n, B, (size_t)S * (sizeof(T) == 8 ? 24 : sizeof(C)), L);
    if (rc) return rc;
    const int BP = L.BP;
    C *smp = reinterpret_cast<C *>(L.smp);
    C *spl = L.spl;
    TileRef *tt = L.tt;
    uint32_t *ntl = L.ntl;
    const uint64_t tmax = L.tmax;
    // (+ 16 bytes: the gathering tile sort reads the 16-byte vector that holds the last key)
    rc = ensure(ctx, &ctx->scratch, &ctx->scratch_bytes, n * sizeof(T) + 16, "sort scratch");
    if (rc) return rc;
    T *scratch = static_cast<T *>(ctx->scratch);
    // 1. splitters from a regular sample in (key, input index) order, sorted on the GPU (the
    // sample sorts never bucket and never fire the fault injection)
    int64_t *pk = reinterpret_cast<int64_t *>(smp), *psrt = pk + S, *pcmp = pk + 2 * (size_t)S;
    ++ctx->nested;
    if constexpr (std::is_same<T, int32_t>::value) {
        // int32 composites are int64 (key * 2^32 + index): one int64 sort
        hipLaunchKernelGGL(bucket_sample_kernel<T>, dim3(ceil_div(S, 256)), dim3(256), 0, s, d_in, (uint64_t)n, smp, S);
        rc = hipGetLastError() == hipSuccess ? sort_device<int64_t>(ctx, smp, smp, S, s, false)
                                             : set_err(ctx, DSORT_EHIP, "bucket_sample_kernel launch");
    } else {
        // int64: the keys, then the composites (pair_rank_kernel)
        hipLaunchKernelGGL(pair_sample_keys_kernel, dim3(ceil_div(S, 256)), dim3(256), 0, s, d_in, (uint64_t)n, pk, S);
        rc = sort_device<int64_t>(ctx, pk, psrt, S, s, false);
        if (!rc) {
            hipLaunchKernelGGL(pair_rank_kernel, dim3(ceil_div(S, 256)), dim3(256), 0, s, pk, psrt, S, pcmp);
            rc = sort_device<int64_t>(ctx, pcmp, pcmp, S, s, false);
        }
    }
    --ctx->nested;
    if (rc) return rc;
    // (the nested sort reset the statistics and events; this sort's start from here)
    if ((rc = bucketed_stats_start(ctx, n, TILE, s, timed))) return rc;
    if constexpr (std::is_same<T, int32_t>::value) {
        hipLaunchKernelGGL(bucket_splitter_kernel<int32_t>, dim3(1), dim3(BK_MAXB), 0, s, smp, B, BP, os, spl);
    } else {
        hipLaunchKernelGGL(pair_splitter_kernel, dim3(1), dim3(BK_MAXB), 0, s, pcmp, pk, (uint64_t)n, S, B, BP, os,
                           spl);
    }
    // 2. the first level.  The scatter always writes the scratch buffer (never the input: the
    // context owns it); the tile sort then writes whichever buffer makes the last pass land in
    // d_keys.  Pure buckets (one key, see below) go straight to d_keys, in their final places, when
    // the second level runs (it skips them) and d_keys is not the input the scatter still reads.
    T *part_out = scratch;
    T *direct = sub_keys<T>(ctx) && (const void *)d_in != (const void *)d_keys && n < (1ull << 31) ? d_keys : nullptr;
    uint64_t *hb;
    C *hspl;
    rc = first_level<T>(ctx, d_in, n, 0, part_out, direct, L, sub_keys<T>(ctx) ? 0u : (uint32_t)TILE, s, timed, hb,
                        hspl);
    if (rc) return rc;
    if (const uint64_t m = sub_keys<T>(ctx)) {
        // A bucket between two splitters of the same key holds only that key: it is sorted as it
        // lies (a heavy duplicate -- Zipf's top keys fill whole buckets).  The second level skips
        // it and copies it to the output.
        std::vector<uint8_t> pure((size_t)B, 0);
        for (int b = 1; b + 1 < B; ++b) pure[b] = Comp<T>::key_of(hspl[b - 1]) == Comp<T>::key_of(hspl[b]);
        // (the scatter dropped the pure buckets' keys when it had `direct`: the second level fills
        // their output ranges with their key, dsort_bucket.h)
        std::vector<T> fk;
        if (direct && DSORT_DROP_PURE) {
            fk.assign((size_t)B, T(0));
            for (int b = 1; b + 1 < B; ++b)
                if (pure[b]) fk[b] = Comp<T>::key_of(hspl[b]);
        }
        return sub_sort<T>(ctx, part_out, d_keys, n, hb, B, m, s, timed, ctx->opt.sub_gather != 0, pure.data(),
                           direct != nullptr, spl, false, nullptr, fk.empty() ? nullptr : fk.data());
    }
    // pass plan: the runs of every bucket; the largest bucket's run count R sets the merge
    // levels L = ceil(log2 R), split into the fewest passes of <= max_logf levels (larger passes
    // first).
    std::vector<std::vector<uint64_t>> runs(B);
    uint64_t maxruns = 1;
    for (int b = 0; b < B; ++b) {
        // the tile sort's runs of bucket b (bucket_tiles: a head up to 16-byte alignment, then
        // TILE-key tiles)
        const uint64_t len = hb[b + 1] - hb[b], h = bucket_head(hb[b], len, ALIGN);
        if (h) runs[b].push_back(h);
        for (uint64_t o = h; o < len; o += TILE) runs[b].push_back(len - o < (uint64_t)TILE ? len - o : TILE);
        maxruns = runs[b].size() > maxruns ? runs[b].size() : maxruns;
    }
    const std::vector<int> pbits = plan_passes<T>(ctx->opt, maxruns);
    const int passes = (int)pbits.size();
    ctx->stats.merge_passes = passes;
    T *bufs[2] = {d_keys, scratch};
    int cur = (passes % 2 == 0) ? 0 : 1;  // tile sort output; the passes end in d_keys
    // 3. tile sort inside the buckets
    rc = tile_sort<T, false>(ctx, part_out, bufs[cur], n, reinterpret_cast<const uint4 *>(tt), ntl, sb::Gather{},
                             (uint32_t)tmax, s, timed);
    if (rc) return rc;
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[1], s));
        ctx->ev_mask |= 2u;
    }
    fault_point(ctx, s, 1);  // tile sort done
    // 4. group tables of every pass (one staging buffer, one copy).  Every bucket gets its own
    // fan-in per pass: the passes after the first keep the global plan's fan-in and the first
    // takes only the levels the bucket still needs (a bucket of <= 64 runs merges F = 8 twice
    // instead of F = 16 then F = 8).  A pass is then one launch per kernel fan-in among its
    // groups.
    std::vector<BucketPass> plan;  // one entry per launch
    std::vector<int> plan_pass;    // the pass of every launch
    std::vector<GroupK> groups;
    std::vector<uint32_t> tgroup;
    std::vector<int> tail(passes + 1, 0);  // tail[p] = levels of the global plan from pass p on
    for (int p = passes - 1; p >= 0; --p) tail[p] = tail[p + 1] + pbits[p];
    std::vector<int> blev(B);
    for (int b = 0; b < B; ++b) blev[b] = ceil_log2((uint64_t)runs[b].size());
    constexpr uint64_t MTN = MTNOM_OF<T>;
    for (int p = 0; p < passes; ++p) {
        std::vector<GroupK> pg;       // this pass's groups (base = global key position)
        std::vector<int> pk;          // kernel log2 fan-in of every group
        uint64_t base = 0;
        for (int b = 0; b < B; ++b) {
            const int need = blev[b] - tail[p + 1];  // levels this pass must resolve
            const int fb = need < 0 ? 0 : (need < pbits[p] ? need : pbits[p]);
            blev[b] -= fb;
            const size_t MAXF = (size_t)1 << fb;
            std::vector<uint64_t> next;
            const size_t nr = runs[b].size();
            for (size_t r0 = 0; r0 < nr; r0 += MAXF) {
                GroupK gk{};
                gk.base = base;
                gk.roff[0] = 0;
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
        // launch classes: the fan-ins of the groups that merge >= 3 runs; groups of 1-2 runs ride
        // with the smallest class (or form the only one)
        int lmin = 99, lmax = 1;
        for (size_t g = 0; g < pg.size(); ++g)
            if (pk[g] >= 2) { lmin = pk[g] < lmin ? pk[g] : lmin; lmax = pk[g] > lmax ? pk[g] : lmax; }
        if (lmin == 99) lmin = lmax = 1;
        for (size_t g = 0; g < pg.size(); ++g) pk[g] = pk[g] < lmin ? lmin : pk[g];
        for (int l = lmin; l <= lmax; ++l) {
            BucketPass bp{l, 0, 0, groups.size(), tgroup.size()};
            uint64_t tiles = 0;
            for (size_t g = 0; g < pg.size(); ++g) {
                if (pk[g] != l) continue;
                GroupK gk = pg[g];
                gk.first_tile = tiles;
                const uint64_t gt = ceil_div(gk.total, MTN);
                for (uint64_t k = 0; k < gt; ++k) tgroup.push_back((uint32_t)(groups.size() - bp.group_off));
                tiles += gt;
                groups.push_back(gk);
            }
            bp.ngroups = groups.size() - bp.group_off;
            bp.ntiles = tiles;
            if (bp.ngroups) {
                plan.push_back(bp);
                plan_pass.push_back(p);
            }
        }
    }
    if (passes > 0) {
        const size_t gbytes = groups.size() * sizeof(GroupK), tbytes = tgroup.size() * sizeof(uint32_t);
        const size_t tb_off = (gbytes + 255) & ~(size_t)255;
        if (ctx->groups_ev_pending) { if (int rc_ = sync_event(ctx, ctx->groups_ev, "group table")) return rc_; }
        ctx->groups_ev_pending = false;
        if (ctx->groups_host_bytes < tb_off + tbytes) {
            release_host(ctx, ctx->groups_host);
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
            rc = launch_pass_w<T, false>(ctx, bufs[cur], bufs[cur ^ 1], pd, plan[q].logf, plan[q].ntiles, s, timed);
            if (rc) return rc;
            if (q + 1 == plan.size() || plan_pass[q + 1] != plan_pass[q]) {  // pass complete
                cur ^= 1;
                fault_point(ctx, s, 2 + plan_pass[q]);
            }
        }
    }
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[2], s));
        ctx->ev_mask |= 4u;
    }
    return DSORT_OK;
}

// ---- bucket exchange (dsort_internal.h; the multi-GPU sample sort) ------------
// Samples of the bucket exchange: record k < s_r at position ((2k + 1) n) / (2 s_r) with its global
// index (ioff + position), the rest of the s_max records +inf (they sort last and are never picked).
template <typename T>
__global__ void __launch_bounds__(256) bx_sample_kernel(const T *__restrict__ in, uint64_t n, uint64_t ioff,
                                                        uint32_t s_r, uint32_t s_max, BxSample *__restrict__ out) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= s_max) return;
    if (k < s_r) {
        const uint64_t pos = ((2 * (uint64_t)k + 1) * n) / (2 * (uint64_t)s_r);
        out[k] = BxSample{(int64_t)in[pos], ioff + pos};
    } else {
        out[k] = BxSample{INT64_MAX, ~0ull};
    }
}
// The records as sort keys: int32 -> the composite key * 2^32 + (global index mod 2^32) (padding:
// INT64_MAX); int64 -> the keys (their composites follow the rank kernel, as in bucket_sort).
template <typename T>
__global__ void __launch_bounds__(256) bx_compose_kernel(const BxSample *__restrict__ all, uint32_t S,
                                                         int64_t *__restrict__ out) {
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= S) return;
    const BxSample r = all[g];
    if constexpr (sizeof(T) == 4)
        out[g] = r.i == ~0ull ? INT64_MAX : (int64_t)((uint64_t)(int64_t)(int32_t)r.k << 32 | (uint32_t)r.i);
    else
        out[g] = r.k;
}
// Global splitter b (b < Btot - 1): the sample of rank ((b + 1) S_real) / Btot - 1 in (key, global
// index) order; +inf up to BP.
template <typename T>
__global__ void __launch_bounds__(bk::BK_MAXB) bx_splitter_kernel(const int64_t *__restrict__ srt,
                                                                 const int64_t *__restrict__ keys,
                                                                 const BxSample *__restrict__ all, uint64_t S_real,
                                                                 int Btot, int BP, typename bk::Comp<T>::C *__restrict__ spl) {
    const int b = threadIdx.x;
    if (b >= BP) return;
    if (b >= Btot - 1) {
        spl[b] = bk::Comp<T>::inf();
        return;
    }
    uint64_t pos = ((uint64_t)(b + 1) * S_real) / (uint64_t)Btot;
    pos = pos ? pos - 1 : 0;
    if constexpr (sizeof(T) == 4) {
        spl[b] = srt[pos];
    } else {
        const uint32_t g = (uint32_t)srt[pos];  // composite rank * 2^32 + record index
        spl[b] = bk::Pair{keys[g], (uint32_t)all[g].i, 0};
    }
}

// The bucket arena of a bucket exchange: the first level of n_local keys into Btot buckets, with
// room for every rank's samples as int64 keys, sorted keys and composites.
template <typename T>
static int bx_layout(dsort_ctx *ctx, const BxPlan &pl, BkLayout<T> &L) {
    const size_t S = (size_t)pl.P * pl.s_max;
    return bk_layout<T>(ctx, pl.n_local, pl.Btot, S * 24, L);
}

}  // namespace wv

bool bx_make_plan(const dsort_opts &opt, int P, int me, const uint64_t *n_of, int key_bytes, BxPlan &pl) {
    pl.P = P;
    pl.me = me;
    pl.n_of.assign(n_of, n_of + P);
    pl.ioff.assign(P + 1, 0);
    for (int r = 0; r < P; ++r) pl.ioff[r + 1] = pl.ioff[r] + n_of[r];
    pl.n_total = pl.ioff[P];
    pl.n_local = n_of[me];
    // (the one-GPU sort's switches: no partition, or no second level -> the sort-then-merge path)
    if (opt.buckets == 0 || opt.sub_keys == 0 || P < 1) return false;
    if (pl.n_total < (uint64_t)P << 22) return false;                 // small: sort locally, then merge
    if (key_bytes == 4 && pl.n_total > (1ull << 32)) return false;    // composite indices are 32-bit
    const uint64_t bk = opt.bucket_keys > 0 ? (uint64_t)opt.bucket_keys : (1ull << 20);
    // (DSORT_OPT_BUCKETS = B forces about B global buckets: B / P per rank)
    uint64_t bl = opt.buckets > 0 ? (uint64_t)opt.buckets / (uint64_t)P : (pl.n_total / P + bk - 1) / bk;
    const uint64_t cap = (uint64_t)bk::BK_MAXB / (uint64_t)P;
    bl = bl > cap ? cap : bl;
    bl = bl < 1 ? 1 : bl;
    pl.Bl = (int)bl;
    pl.Btot = P * pl.Bl;
    if (pl.Btot < 2) return false;
    // samples: bucket_os per global bucket, shared out in proportion to the ranks' keys
    const uint64_t os = opt.bucket_os < 1 ? 1 : (opt.bucket_os > 4096 ? 4096 : (uint64_t)opt.bucket_os);
    const uint64_t S = (uint64_t)pl.Btot * os;
    pl.s_of.assign(P, 0);
    uint32_t mx = 1;
    for (int r = 0; r < P; ++r) {
        uint64_t sr = pl.n_total ? (S * n_of[r] + pl.n_total - 1) / pl.n_total : 0;
        sr = sr > n_of[r] ? n_of[r] : sr;
        pl.s_of[r] = (uint32_t)sr;
        mx = (uint32_t)sr > mx ? (uint32_t)sr : mx;
    }
    pl.s_max = mx;
    // the others' pieces behind this rank's partitioned keys: its expected share plus a margin (a
    // larger receive takes a separate buffer and copies this rank's own buckets there)
    pl.recv_room = P == 1 ? 0 : pl.n_total / P + pl.n_total / (4 * (uint64_t)P) + (1u << 16);
    return true;
}

template <typename T>
int bx_sample(dsort_ctx *ctx, const T *d_in, const BxPlan &pl, BxSample *d_smp, hipStream_t s) {
    hipLaunchKernelGGL(wv::bx_sample_kernel<T>, dim3(wv::ceil_div(pl.s_max, 256)), dim3(256), 0, s, d_in, pl.n_local,
                       pl.ioff[pl.me], pl.s_of[pl.me], pl.s_max, d_smp);
    DSORT_HIP(ctx, hipGetLastError());
    return DSORT_OK;
}

#ifndef DSORT_BX_DROP_PURE
#define DSORT_BX_DROP_PURE 1
#endif
template <typename T>
int bx_partition(dsort_ctx *ctx, const T *d_in, const BxPlan &pl, const BxSample *d_all, hipStream_t s, bool timed,
                 const uint64_t **hb_out, T **part, std::vector<uint8_t> &pure) {
    using namespace wv;
    using C = typename bk::Comp<T>::C;
    ctx->stages_done = 0;
    BkLayout<T> L;
    int rc = bx_layout<T>(ctx, pl, L);
    if (rc) return rc;
    const uint32_t S = (uint32_t)((size_t)pl.P * pl.s_max);
    uint64_t S_real = 0;
    for (int r = 0; r < pl.P; ++r) S_real += pl.s_of[r];
    int64_t *pk = reinterpret_cast<int64_t *>(L.smp), *psrt = pk + S, *pcmp = pk + 2 * (size_t)S;
    // the global splitters, identical on every rank (the same records, the same sorts)
    ++ctx->nested;
    hipLaunchKernelGGL(bx_compose_kernel<T>, dim3(ceil_div(S, 256)), dim3(256), 0, s, d_all, S, pk);
    rc = hipGetLastError() == hipSuccess ? DSORT_OK : set_err(ctx, DSORT_EHIP, "bx_compose_kernel launch");
    if (!rc) {
        if constexpr (sizeof(T) == 4) {
            rc = sort_device<int64_t>(ctx, pk, psrt, S, s, false);
        } else {
            rc = sort_device<int64_t>(ctx, pk, psrt, S, s, false);
            if (!rc) {
                hipLaunchKernelGGL(bk::pair_rank_kernel, dim3(ceil_div(S, 256)), dim3(256), 0, s, pk, psrt, S, pcmp);
                rc = sort_device<int64_t>(ctx, pcmp, pcmp, S, s, false);
            }
        }
    }
    --ctx->nested;
    if (rc) return rc;
    if ((rc = bucketed_stats_start(ctx, pl.n_local, TILE_OF<T>, s, timed))) return rc;
    hipLaunchKernelGGL(bx_splitter_kernel<T>, dim3(1), dim3(bk::BK_MAXB), 0, s, sizeof(T) == 4 ? psrt : pcmp, pk, d_all,
                       S_real, pl.Btot, L.BP, L.spl);
    DSORT_HIP(ctx, hipGetLastError());
    rc = ensure(ctx, &ctx->scratch, &ctx->scratch_bytes, (pl.n_local + pl.recv_room) * sizeof(T) + 16, "sort scratch");
    if (rc) return rc;
    T *scratch = static_cast<T *>(ctx->scratch);
    uint64_t *hb;
    C *hspl;
    if (pl.n_local) {
        rc = first_level<T>(ctx, d_in, pl.n_local, pl.ioff[pl.me], scratch, nullptr, L, 0u, s, timed, hb, hspl,
                            DSORT_BX_DROP_PURE != 0);
        if (rc) return rc;
    } else {
        // no keys here: empty buckets (the splitters still go to the host for the second level)
        hb = static_cast<uint64_t *>(ctx->bucket_host);
        hspl = reinterpret_cast<C *>(hb + bk::BK_MAXB + 1);
        for (int b = 0; b <= pl.Btot; ++b) hb[b] = 0;
        DSORT_HIP(ctx, hipMemcpyAsync(hspl, L.spl, (size_t)(pl.Btot - 1) * sizeof(C), hipMemcpyDeviceToHost, s));
        if (int rc_ = sync_stream(ctx, s, "sort stream")) return rc_;
        fault_point(ctx, s, 0);
    }
    if ((rc = stage_event(ctx, s, timed, 2))) return rc;  // the local part done: the exchange starts
    // (the scatter's rule, bucket_scatter_lines_kernel / bucket_scan_kernel: the same splitters on
    // every rank, which derive every rank's compacted starts from its bucket starts)
    pure.assign((size_t)pl.Btot, 0);
    for (int g = 1; DSORT_BX_DROP_PURE && g + 1 < pl.Btot; ++g)
        pure[(size_t)g] = bk::Comp<T>::key_of(hspl[g - 1]) == bk::Comp<T>::key_of(hspl[g]) ? 1 : 0;
    *hb_out = hb;
    *part = scratch;
    return DSORT_OK;
}

template <typename T>
int bx_local_sort(dsort_ctx *ctx, T *recv, T *out, const BxPlan &pl, const uint64_t *hb_all, const uint64_t *hc_all,
                  const uint64_t *base, int j_lo, int j_hi, uint64_t out_off, int w, int W, hipStream_t s, bool timed,
                  uint64_t *n_out) {
    using namespace wv;
    using C = typename bk::Comp<T>::C;
    const int P = pl.P, me = pl.me, Bt = pl.Btot, Bl = j_hi - j_lo;  // (Bl: this wave's buckets)
    const uint64_t g0 = (uint64_t)me * pl.Bl + (uint64_t)j_lo;
    // this wave's buckets: one piece per source, in source order
    PieceMap<T> pm;
    pm.first.assign(Bl + 1, 0);
    pm.pure_key.assign(Bl, T(0));
    std::vector<uint64_t> hbo(Bl + 1, 0);
    std::vector<uint8_t> pure(Bl, 0);
    const C *hspl = reinterpret_cast<const C *>(static_cast<const uint64_t *>(ctx->bucket_host) + bk::BK_MAXB + 1);
    for (int j = 0; j < Bl; ++j) {
        const uint64_t g = g0 + (uint64_t)j;
        pm.first[j] = (uint32_t)pm.p.size();
        uint64_t tot = 0;
        for (int r = 0; r < P; ++r) {
            const uint64_t *h = hb_all + (size_t)r * (Bt + 1), *hc = hc_all + (size_t)r * (Bt + 1);
            const uint64_t len = hc[g + 1] - hc[g];  // (0 for a pure bucket whose keys stayed home)
            if (len) pm.p.push_back(SrcPiece{base[r] + (hc[g] - hc[g0]), len});
            tot += h[g + 1] - h[g];
        }
        hbo[j + 1] = hbo[j] + tot;
        // a global bucket between two splitters of one key holds only that key
        if (g >= 1 && g + 2 <= (uint64_t)Bt && bk::Comp<T>::key_of(hspl[g - 1]) == bk::Comp<T>::key_of(hspl[g])) {
            pure[j] = 1;
            pm.pure_key[j] = bk::Comp<T>::key_of(hspl[g]);
        }
    }
    pm.first[Bl] = (uint32_t)pm.p.size();
    const uint64_t nrecv = hbo[Bl];
    *n_out = nrecv;
    const bool last = w + 1 == W;
    // the statistics of the waves add up
    const dsort_stats before = ctx->stats;
    if (w == 0) ctx->stats.tile_sort_keys = 0;
    int rc = DSORT_OK;
    if (nrecv) {
        BkLayout<T> L;
        if ((rc = bx_layout<T>(ctx, pl, L))) return rc;  // (the arena as bx_partition left it: the splitters)
        // a second wave's tables go to the other second-level arena: the first wave's kernels may
        // still read theirs when this wave's tables are uploaded
        if (w & 1) {
            std::swap(ctx->sub, ctx->sub_alt);
            std::swap(ctx->sub_bytes, ctx->sub_alt_bytes);
        }
        const int saved_done = ctx->ev_done, saved_off = ctx->ev_off;
        ctx->ev_off = last ? 0 : 15;
        ctx->ev_done = last ? 4 : 16;
        rc = sub_sort<T>(ctx, recv, out + out_off, nrecv, hbo.data(), Bl, sub_keys<T>(ctx), s, timed,
                         ctx->opt.sub_gather != 0, pure.data(), false, L.spl + g0, false, &pm);
        ctx->ev_done = saved_done;
        ctx->ev_off = saved_off;
        if (w & 1) {
            std::swap(ctx->sub, ctx->sub_alt);
            std::swap(ctx->sub_bytes, ctx->sub_alt_bytes);
        }
        if (rc) return rc;
        if (w > 0) {
            ctx->stats.tile_sort_keys += before.tile_sort_keys;
            ctx->stats.merge_passes = std::max(ctx->stats.merge_passes, before.merge_passes);
            ctx->stats.sub_split_subbuckets += before.sub_split_subbuckets;
            ctx->stats.sub_scatter_fallback |= before.sub_scatter_fallback;
        }
    } else {
        if (w == 0) {
            fault_point(ctx, s, 1);
            fault_point(ctx, s, 2);
        }
        if (last && timed && ctx->ev_ok) {
            DSORT_HIP(ctx, hipEventRecord(ctx->ev[4], s));
            ctx->ev_mask |= 16u;
        }
    }
    if (!last) return DSORT_OK;
    if (ctx->opt.kill_after_pass >= 0)  // (a kill stage this sort never reached)
        return set_err(ctx, DSORT_ESTAGE, "DSORT_OPT_KILL_AFTER_STAGE = " + std::to_string(ctx->opt.kill_after_pass) +
                                              ": the bucket exchange has " + std::to_string(ctx->stages_done) +
                                              " stages (kill points 0.." + std::to_string(ctx->stages_done - 1) + ")");
    return DSORT_OK;
}

template int bx_sample<int32_t>(dsort_ctx *, const int32_t *, const BxPlan &, BxSample *, hipStream_t);
template int bx_sample<int64_t>(dsort_ctx *, const int64_t *, const BxPlan &, BxSample *, hipStream_t);
template int bx_partition<int32_t>(dsort_ctx *, const int32_t *, const BxPlan &, const BxSample *, hipStream_t, bool,
                                   const uint64_t **, int32_t **, std::vector<uint8_t> &);
template int bx_partition<int64_t>(dsort_ctx *, const int64_t *, const BxPlan &, const BxSample *, hipStream_t, bool,
                                   const uint64_t **, int64_t **, std::vector<uint8_t> &);
template int bx_local_sort<int32_t>(dsort_ctx *, int32_t *, int32_t *, const BxPlan &, const uint64_t *,
                                    const uint64_t *, const uint64_t *, int, int, uint64_t, int, int, hipStream_t, bool,
                                    uint64_t *);
template int bx_local_sort<int64_t>(dsort_ctx *, int64_t *, int64_t *, const BxPlan &, const uint64_t *,
                                    const uint64_t *, const uint64_t *, int, int, uint64_t, int, int, hipStream_t, bool,
                                    uint64_t *);

namespace wv {

template <typename T>
static int wave_sort(dsort_ctx *ctx, const T *d_in, T *d_keys, size_t n, hipStream_t s, bool timed) {
    constexpr int TILE = TILE_OF<T>;
    ctx->stats = fresh_stats();
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
    if (const int B = bucket_count(ctx, n)) return bucket_sort<T>(ctx, d_in, d_keys, n, s, timed, B);
    const uint64_t tiles = ceil_div(n, TILE);
    const std::vector<int> plan = plan_passes<T>(ctx->opt, tiles);
    const int passes = (int)plan.size();
    ctx->stats.merge_passes = passes;
    T *scratch = nullptr;
    if (passes > 0) {
        // a nested sort (splitter samples) runs while the scratch holds the partitioned keys
        void **sb = ctx->nested ? &ctx->scratch2 : &ctx->scratch;
        size_t *sbb = ctx->nested ? &ctx->scratch2_bytes : &ctx->scratch_bytes;
        int rc = ensure(ctx, sb, sbb, n * sizeof(T), "sort scratch");
        if (rc) return rc;
        scratch = static_cast<T *>(*sb);
    }
    // ping-pong so that the last pass lands in d_keys; the tile sort reads d_in (which may alias
    // d_keys)
    T *bufs[2] = {d_keys, scratch};
    int cur = (passes % 2 == 0) ? 0 : 1;
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[0], s));
        ctx->ev_mask |= 1u;
    }
    int rc = tile_sort<T, false>(ctx, d_in, bufs[cur], n, nullptr, nullptr, sb::Gather{}, (uint32_t)tiles, s, timed);
    if (rc) return rc;
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[1], s));
        ctx->ev_mask |= 2u;
    }
    fault_point(ctx, s, 0);  // tile sort done
    constexpr uint64_t MTN = MTNOM_OF<T>;
    uint64_t Rr = TILE;
    for (int p = 0; p < passes; ++p) {
        PassDesc pd{(uint64_t)n, Rr, 1 << plan[p], 0, nullptr};
        const uint64_t gsize = Rr << plan[p];
        const uint64_t ngroups = ceil_div(n, gsize);
        const uint64_t tpg = ceil_div(gsize, MTN);
        const uint64_t mtiles = (ngroups - 1) * tpg + ceil_div(n - (ngroups - 1) * gsize, MTN);
        int rc = launch_pass_w<T, true>(ctx, bufs[cur], bufs[cur ^ 1], pd, plan[p], mtiles, s, timed);
        if (rc) return rc;
        Rr <<= plan[p];
        cur ^= 1;
        fault_point(ctx, s, 1 + p);  // merge pass p done
    }
    if (timed && ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[2], s));
        ctx->ev_mask |= 4u;
    }
    return DSORT_OK;
}

// k-way merge of back-to-back runs of arbitrary lengths (the master merge, server.c:481-515, and
// the multi-GPU receive merge).  Up to 32 runs (int64: 16) merge in one pass; more runs merge in
// levels of such groups.  Lower runs win ties at every level.
template <typename T>
static int wave_merge(dsort_ctx *ctx, const T *d_in, const size_t *lens, int k, T *d_out, hipStream_t s,
                      bool keep_stats) {
    constexpr int MAXF = 1 << WG<T>::MAXLOGF;
    if (!keep_stats) {
        ctx->stats = fresh_stats();
        ctx->kev_used = 0;
    }
    ctx->last_stream = s;
    uint64_t n = 0;
    std::vector<uint64_t> rl(lens, lens + k);
    for (int j = 0; j < k; ++j) n += lens[j];
    if (!keep_stats) {
        ctx->stats.keys_in = ctx->stats.keys_out = n;
        ctx->stats.tile_sort_keys = n;
        ctx->stats.tile_keys = TILE_OF<T>;
    }
    if (n == 0) return DSORT_OK;
    if (k == 1) {
        DSORT_HIP(ctx, hipMemcpyAsync(d_out, d_in, n * sizeof(T), hipMemcpyDeviceToDevice, s));
        return DSORT_OK;
    }
    int levels = 0;
    for (uint64_t r = (uint64_t)k; r > 1; r = ceil_div(r, MAXF)) ++levels;
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
    constexpr uint64_t MTN = MTNOM_OF<T>;
    for (int l = 0; l < levels; ++l) {
        const int nr = (int)rl.size();
        const int per = nr < MAXF ? nr : MAXF;
        const int logf = ceil_log2((uint64_t)per) < 1 ? 1 : ceil_log2((uint64_t)per);
        const int ng = (nr + MAXF - 1) / MAXF;
        const size_t gbytes = (size_t)ng * sizeof(GroupK);
        if (ctx->groups_ev_pending) { if (int rc_ = sync_event(ctx, ctx->groups_ev, "group table")) return rc_; }
        ctx->groups_ev_pending = false;
        if (ctx->groups_host_bytes < gbytes) {
            release_host(ctx, ctx->groups_host);
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
            for (int r = gi * MAXF; r < nr && r < (gi + 1) * MAXF; ++r) {
                tot += rl[r];
                gk.roff[++gk.nruns] = tot;
            }
            for (int r = (int)gk.nruns + 1; r <= kMaxF; ++r) gk.roff[r] = tot;
            gk.total = tot;
            tiles += ceil_div(tot, MTN);
            base += tot;
            next.push_back(tot);
        }
        DSORT_HIP(ctx, hipMemcpyAsync(ctx->groups, gh, gbytes, hipMemcpyHostToDevice, s));
        DSORT_HIP(ctx, hipEventRecord(ctx->groups_ev, s));
        ctx->groups_ev_pending = true;
        PassDesc pd{n, 0, 1 << logf, ng, static_cast<const GroupK *>(ctx->groups)};
        T *dst = dsts[which];
        // a top-level merge times its merge kernels (dsort_stats.merge_kernel_ms)
        rc = launch_pass_w<T, false>(ctx, src, dst, pd, logf, tiles, s, !keep_stats);
        if (rc) return rc;
        rl.swap(next);
        src = dst;
        which ^= 1;
    }
    return DSORT_OK;
}

}  // namespace wv

#ifdef DSORT_STAMPS
extern "C" int dsort_debug_stamps(void *host, size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(wv::g_stamps), bytes) == hipSuccess ? 0 : -1;
}
extern "C" int dsort_debug_bkstamps(void *host, size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(bk::g_bkstamps), bytes) == hipSuccess ? 0 : -1;
}
extern "C" int dsort_debug_sbstamps(void *host, size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(sb::g_sbstamps), bytes) == hipSuccess ? 0 : -1;
}
#endif

// ------------------------------------------------------------------------------------------
// Entry points of the worker sort and the master merge (dsort_internal.h).
// Replace merge_sort()/merge() (reference client.c:140-173) and the merge loop of merge_chunks()
// (server.c:481-515).  Same result: the input multiset in ascending signed order; equal keys
// from different runs are emitted lower run first, like the reference's `<=` (client.c:152) and
// lowest-index-wins argmin (server.c:504) -- unobservable for keys-only data.
// ------------------------------------------------------------------------------------------
static double mono_ms() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}
void PollPause::operator()() {
    const double t = mono_ms();
    if (t0 < 0) t0 = t;
    if (t - t0 < POLL_SPIN_MS) sched_yield();
    else usleep(20);
}
// (The waits outside an exchange poll the same way, without the abort and deadline checks:
// measured the same as hipEventSynchronize on the one-GPU sort.)
static int poll_done(dsort_ctx *ctx, hipError_t (*query)(void *), void *h, const char *what, bool comm) {
    PollPause pause;
    for (;;) {
        const hipError_t q = query(h);
        if (q == hipSuccess) return DSORT_OK;
        if (q != hipErrorNotReady) return hip_err(ctx, q, what);
        if (comm && ctx->abort_req.load())
            return set_err(ctx, DSORT_ECOMM, std::string(what) + ": aborted by dsort_comm_abort (keys in flight)");
        if (comm && ctx->poll_deadline > 0 && mono_ms() > ctx->poll_deadline)
            return set_err(ctx, DSORT_ETIMEOUT, std::string(what) + ": no progress before the deadline (keys in flight)");
        pause();
    }
}
int sync_event(dsort_ctx *ctx, hipEvent_t e, const char *what) {
    return poll_done(ctx, [](void *h) { return hipEventQuery(static_cast<hipEvent_t>(h)); }, e, what, ctx->poll_waits);
}
int sync_stream(dsort_ctx *ctx, hipStream_t s, const char *what) {
    return poll_done(ctx, [](void *h) { return hipStreamQuery(static_cast<hipStream_t>(h)); }, s, what,
                     ctx->poll_waits);
}

int max_logf(const dsort_opts &opt, int type_default, int type_cap) {
    const int64_t o = opt.max_logf;
    const int x = o < 0 ? type_default : (int)o;
    return x < 1 ? 1 : (x > type_cap ? type_cap : x);
}

void fault_point(dsort_ctx *ctx, hipStream_t s, int stage) {
    if (ctx->nested) return;
    if (ctx->opt.kill_after_pass == stage) {
        (void)hipStreamSynchronize(s);  // the stage has finished on the GPU: the worker dies after it
        raise(SIGKILL);
    }
    if (stage + 1 > ctx->stages_done) ctx->stages_done = stage + 1;
}

int sort_stages(const dsort_opts &opt, uint64_t n, int key_bytes) {
    if (n < 2) return 0;
    const bool w8 = key_bytes == 8;
    if (wv::bucket_count(opt, n)) {
        const uint64_t m = w8 ? wv::sub_keys<int64_t>(opt) : wv::sub_keys<int32_t>(opt);
        return m ? 3 : 2;
    }
    const uint64_t tile = w8 ? wv::TILE_OF<int64_t> : wv::TILE_OF<int32_t>;
    const uint64_t tiles = wv::ceil_div(n, tile);
    const size_t passes = w8 ? wv::plan_passes<int64_t>(opt, tiles).size() : wv::plan_passes<int32_t>(opt, tiles).size();
    return 1 + (int)passes;
}

// A top-level call first waits (on the device) for the context's previous call when that ran on
// another stream, and marks its own end: the calls share the context's arenas and return while
// their last kernels still run.
static int order_begin(dsort_ctx *ctx, hipStream_t s) {
    if (ctx->nested) return DSORT_OK;
    if (ctx->done_pending && ctx->done_stream != s) DSORT_HIP(ctx, hipStreamWaitEvent(s, ctx->done_ev, 0));
    return DSORT_OK;
}
static int order_end(dsort_ctx *ctx, hipStream_t s) {
    if (ctx->nested) return DSORT_OK;
    if (!ctx->done_ev && hipEventCreateWithFlags(&ctx->done_ev, hipEventDisableTiming) != hipSuccess)
        return set_err(ctx, DSORT_EHIP, "hipEventCreate");
    DSORT_HIP(ctx, hipEventRecord(ctx->done_ev, s));
    ctx->done_stream = s;
    ctx->done_pending = true;
    return DSORT_OK;
}

template <typename T>
int sort_device(dsort_ctx *ctx, const T *d_in, T *d_keys, size_t n, hipStream_t s, bool timed) {
    const bool top = ctx->nested == 0;
    if (top) ctx->stages_done = 0;
    int rc = order_begin(ctx, s);
    if (!rc) rc = wv::wave_sort<T>(ctx, d_in, d_keys, n, s, timed);
    if (!rc) rc = order_end(ctx, s);
    if (rc || !top || ctx->opt.kill_after_pass < 0) return rc;
    // the kill stage was never reached: a fault-injection run that would silently not fail
    return set_err(ctx, DSORT_ESTAGE,
                   "DSORT_OPT_KILL_AFTER_STAGE = " + std::to_string(ctx->opt.kill_after_pass) + ": this sort of " +
                       std::to_string(n) + " keys has " + std::to_string(ctx->stages_done) +
                       " stages (kill points 0.." + std::to_string(ctx->stages_done - 1) + ")");
}

// k-way merge of back-to-back runs of arbitrary lengths (the master merge, server.c:481-515,
// and the multi-GPU receive merge); lower runs win ties at every level.
template <typename T>
int merge_device(dsort_ctx *ctx, const T *d_in, const size_t *lens, int k, T *d_out, hipStream_t s,
                 bool keep_stats) {
    int rc = order_begin(ctx, s);
    if (!rc) rc = wv::wave_merge<T>(ctx, d_in, lens, k, d_out, s, keep_stats);
    if (!rc) rc = order_end(ctx, s);
    return rc;
}

template int sort_device<int32_t>(dsort_ctx *, const int32_t *, int32_t *, size_t, hipStream_t, bool);
template int sort_device<int64_t>(dsort_ctx *, const int64_t *, int64_t *, size_t, hipStream_t, bool);
template int merge_device<int32_t>(dsort_ctx *, const int32_t *, const size_t *, int, int32_t *, hipStream_t,
                                   bool);
template int merge_device<int64_t>(dsort_ctx *, const int64_t *, const size_t *, int, int64_t *, hipStream_t,
                                   bool);

}  // namespace dsort
