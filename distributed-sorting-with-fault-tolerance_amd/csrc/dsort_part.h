// dsort_part.h -- device code shared by the sort kernels of both key widths: key limits, the
// group/tile geometry of a k-way merge pass and the cut search of every output tile boundary
// (partk_kernel).  Included by dsort_sort.hip (legacy LDS merge-path kernels, int64) and
// dsort_wave.hip (wave-register bitonic kernels, int32).  gfx950 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>

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

// ---------------------------------------------------------------------------------------
// Tile / group geometry of a k-way pass.  A group's output is cut into tiles of NOMINAL size
// tnom = TILE - 2*slack; the actual cut of boundary jr lies within +-slack of jr*tnom, so every
// tile holds at most TILE keys.
// ---------------------------------------------------------------------------------------
struct TileInfo {
    uint64_t base;    // group start
    uint64_t gtotal;  // keys in the group
    uint64_t jr;      // tile index within the group
    uint64_t ntg;     // tiles in the group
};

template <bool REG>
__device__ __forceinline__ const GroupK *tile_info(const PassDesc &pd, uint64_t j, int tnom,
                                                   TileInfo &ti) {
    const GroupK *g = nullptr;
    if (REG) {
        const uint64_t gsize = (uint64_t)pd.F * pd.R;
        const uint64_t tpg = (gsize + tnom - 1) / tnom;
        const uint64_t gi = j / tpg;
        ti.base = gi * gsize;
        ti.gtotal = pd.n - ti.base < gsize ? pd.n - ti.base : gsize;
        ti.jr = j - gi * tpg;
    } else {
        int lo = 0, hi = pd.ngroups - 1;  // last group with first_tile <= j
        if (pd.tile_group) {
            lo = (int)pd.tile_group[j];  // one load instead of a dependent binary search
        } else {
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (pd.groups[mid].first_tile <= j) lo = mid;
                else hi = mid - 1;
            }
        }
        g = pd.groups + lo;
        ti.base = g->base;
        ti.gtotal = g->total;
        ti.jr = j - g->first_tile;
    }
    ti.ntg = (ti.gtotal + tnom - 1) / tnom;
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

// lo + round(frac * (hi - lo)) clamped to [lo, hi - 1]; frac in [0, 1].  Doubles carry the
// estimate only: the result is always a valid key strictly below hi.
template <typename T>
__device__ __forceinline__ T key_at(T lo, T hi, double frac) {
    using U = typename Unsigned<T>::type;
    const U range = (U)hi - (U)lo;  // > 0
    frac = frac < 0.0 ? 0.0 : (frac > 1.0 ? 1.0 : frac);
    double off = frac * (double)range;
    U o = off >= (double)range ? range - 1 : (U)off;
    if (o >= range) o = range - 1;
    return (T)((U)lo + o);
}

// 16-byte vector of keys (int4 / longlong2)
template <typename T> struct Vec16Part;
template <> struct Vec16Part<int32_t> { using type = int4; };
template <> struct Vec16Part<int64_t> { using type = longlong2; };

// #keys <= v in A[u, h) for a short window (at most 4 16-byte chunks of keys): every chunk
// that overlaps the window is loaded at once (one memory round trip instead of a dependent
// binary search); `end` bounds the array so a chunk never reads past it.
template <typename T>
__device__ __forceinline__ uint64_t count_le_window(const T *A, uint64_t u, uint64_t h, T v,
                                                    const T *end) {
    using V = typename Vec16Part<T>::type;
    constexpr int N = 16 / (int)sizeof(T);
    const T *p0 = A + u;
    const T *ph = A + h;
    const T *pa = reinterpret_cast<const T *>(reinterpret_cast<uintptr_t>(p0) & ~(uintptr_t)15);
    T x[5][N];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const T *q = pa + k * N;
        if (q < ph && q + N <= end) {
            const V w = *reinterpret_cast<const V *>(q);
            const T *pw = reinterpret_cast<const T *>(&w);
#pragma unroll
            for (int j = 0; j < N; ++j) x[k][j] = pw[j];
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) x[k][j] = (q + j < ph && q + j < end) ? q[j] : key_max<T>();
        }
    }
    uint64_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const T *e = pa + k * N + j;
            cnt += (e >= p0 && e < ph && x[k][j] <= v) ? 1 : 0;
        }
    }
    return u + cnt;
}

// #keys <= v in A[u, h), knowing A[u..h) lies within [klo, khi]: interpolation probes while the
// window is large, then one vector count of the last <= 4 chunks.  Each probe is one dependent
// load.
template <typename T>
__device__ __forceinline__ uint64_t upper_bound_interp(const T *A, uint64_t u, uint64_t h, T v,
                                                       T klo, T khi, const T *end) {
    using U = typename Unsigned<T>::type;
    constexpr uint64_t WIN = 64 / sizeof(T) - 16 / sizeof(T);  // fits 4 chunks at any alignment
#pragma unroll 1
    for (int it = 0; it < 6 && h - u > WIN; ++it) {
        if (v < klo) return u;
        if (v >= khi) return h;
        const double frac = (double)((U)v - (U)klo) / ((double)((U)khi - (U)klo) + 1.0);
        uint64_t m = u + (uint64_t)(frac * (double)(h - u));
        m = m < u ? u : (m >= h ? h - 1 : m);
        const T x = A[m];
        if (x <= v) {
            u = m + 1;
            klo = x;
        } else {
            h = m;
            khi = x;
        }
    }
#pragma unroll 1
    while (h - u > WIN) {
        const uint64_t m = (u + h) >> 1;
        if (A[m] <= v) u = m + 1;
        else h = m;
    }
    return u < h ? count_le_window(A, u, h, v, end) : u;
}

// ---------------------------------------------------------------------------------------
// 2a. Cut of every tile boundary: for nominal rank d = jr*tnom find a VALID cut (all keys below
//     a threshold in (key, run, position) order) whose rank lies in [d - slack, d + slack].
//     One wave per tile; lane (c, i) evaluates candidate key c on run i (C = 64/F candidates
//     per step).  Candidates bracket the interpolated key of rank d; a step that does not at
//     least halve the bracket is followed by a plain C-section step.  A bracket collapsed to a
//     single key (a heavy duplicate) is cut exactly at d, equal keys taken in run order.
//     Writes splits[j*F + i] = keys of run i below the cut (relative to the run start).
// ---------------------------------------------------------------------------------------
template <typename T, bool REG>
__global__ void __launch_bounds__(256) partk_kernel(const T *__restrict__ in, PassDesc pd, int tnom,
                                                    int slack, uint32_t *__restrict__ splits,
                                                    uint64_t ntiles) {
    const int lane = threadIdx.x & 63;
    const uint64_t j = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= ntiles) return;  // wave-uniform
    TileInfo ti;
    const GroupK *g = tile_info<REG>(pd, j, tnom, ti);
    const int F = pd.F;
    const int C = 64 / F;
    const int i = lane & (F - 1);
    const int c = lane / F;
    uint64_t rs, rl;
    run_range<REG>(pd, ti, g, i, rs, rl);
    const T *A = in + rs;
    uint32_t *outp = splits + j * (uint64_t)F;
    const uint64_t d = ti.jr * (uint64_t)tnom;
    if (d == 0) {
        if (c == 0) outp[i] = 0;
        return;
    }
    T lo = wave_min(rl ? A[0] : key_max<T>());
    T hi = wave_max(rl ? A[rl - 1] : key_min<T>());
    // bracket: ilo = #keys < lo, ihi = #keys <= hi in run i; nlo = sum(ilo) <= d <= sum(ihi) = nhi
    uint64_t ilo = 0, ihi = rl;
    uint64_t nlo = 0, nhi = ti.gtotal;
    // candidate selection: 0 = interpolation in key space (uniform-like keys), 1 = interpolation
    // in the data (keys read from the run with the widest index bracket at the target's relative
    // rank: any distribution, e.g. sparse heavy-duplicate Zipf keys), 2 = evenly spaced keys of
    // that run (guaranteed progress).  A step that does not halve the bracket escalates.
    int mode = 0;
    uint64_t cut_i = 0;
    bool done = false;
#pragma unroll 1
    for (int it = 0; it < 4096 && !done; ++it) {
        if (nhi - nlo <= (uint64_t)slack) {  // cut just below lo: rank nlo in [d - slack, d]
            cut_i = ilo;
            done = true;
            break;
        }
        if (lo == hi) break;  // a single key left: exact tie split below
        T cand;
        const double n = (double)(nhi - nlo);
        const double spread = fmax((double)slack * 0.5, 3.0 * sqrt(n));
        const double r = C == 1 ? 0.0 : -spread + 2.0 * spread * (double)c / (double)(C - 1);
        if (mode == 0) {
            cand = key_at(lo, hi, ((double)d + r - (double)nlo) / n);
        } else {
            // the run with the widest bracket (ties: lowest run); its lane of candidate c reads
            const uint64_t packed = wave_max(((ihi - ilo) << 6) | (uint64_t)(63 - i));
            const int rr = 63 - (int)(packed & 63);
            double frac = mode == 1 ? ((double)d + r - (double)nlo) / n : (double)(c + 1) / (double)(C + 1);
            frac = frac < 0.0 ? 0.0 : (frac > 1.0 ? 1.0 : frac);
            T mine = key_max<T>();
            if (i == rr) {
                const uint64_t range = ihi - ilo;  // > 0: the bracket holds more than slack keys
                uint64_t pos = ilo + (uint64_t)(frac * (double)range);
                pos = pos >= ihi ? ihi - 1 : pos;
                mine = A[pos];
            }
            cand = __shfl(mine, c * F + rr);
            // keep candidates in [lo, hi - 1] (non-decreasing in c): a candidate hi - 1 counts
            // the keys below the block of the largest key, so a target inside a run of duplicates
            // of hi collapses the bracket to that key on the next step
            cand = cand < hi ? cand : (T)(hi - 1);
        }
        const uint64_t u = upper_bound_interp(A, ilo, ihi, cand, lo, hi, in + pd.n);
        uint64_t tot = u;
        for (int o = 1; o < F; o <<= 1) tot += __shfl_xor(tot, o);
        // a candidate whose cut already lands within the slack ends the search
        const bool ok = tot + (uint64_t)slack >= d && tot <= d + (uint64_t)slack;
        const unsigned long long okm = __ballot(ok);
        if (okm) {
            const int cg = (int)((__ffsll((long long)okm) - 1) / F);
            cut_i = __shfl(u, cg * F + i);
            done = true;
            break;
        }
        const unsigned long long mask = __ballot(tot >= d);
        const int cs = mask ? (int)((__ffsll((long long)mask) - 1) / F) : C;  // first cand with U >= d
        const uint64_t ub_cs = __shfl(u, (cs < C ? cs : 0) * F + i);
        const uint64_t ub_pr = __shfl(u, (cs > 0 ? cs - 1 : 0) * F + i);
        const uint64_t tot_cs = __shfl(tot, (cs < C ? cs : 0) * F);
        const uint64_t tot_pr = __shfl(tot, (cs > 0 ? cs - 1 : 0) * F);
        const T cand_cs = __shfl(cand, (cs < C ? cs : 0) * F);
        const T cand_pr = __shfl(cand, (cs > 0 ? cs - 1 : 0) * F);
        const uint64_t before = nhi - nlo;
        if (cs < C) {
            hi = cand_cs;
            ihi = ub_cs;
            nhi = tot_cs;
        }
        if (cs > 0) {
            lo = cand_pr + 1;
            ilo = ub_pr;
            nlo = tot_pr;
        }
        if (mode != 0) {
            // tighten the key bracket to the keys actually inside the index bracket (keeps
            // ilo = #keys < lo and ihi = #keys <= hi); one key left -> lo == hi
            lo = wave_min(ilo < ihi ? A[ilo] : key_max<T>());
            hi = wave_max(ilo < ihi ? A[ihi - 1] : key_min<T>());
        }
        const bool halved = (nhi - nlo) * 2 <= before;
        mode = halved ? (mode == 2 ? 1 : mode) : (mode == 0 ? 1 : 2);
    }
    if (!done) {
        // lo == hi: ilo = #keys < key, ihi = #keys <= key; take d - sum(ilo) equal keys in run order
        const uint64_t cnt = ihi - ilo;
        uint64_t incl = cnt;
        for (int o = 1; o < F; o <<= 1) {
            const uint64_t v = __shfl_up(incl, o);
            if (i >= o) incl += v;
        }
        const uint64_t excl = incl - cnt;
        const uint64_t need = d - nlo;
        const uint64_t take = need > excl ? (need - excl < cnt ? need - excl : cnt) : 0;
        cut_i = ilo + take;
    }
    if (c == 0) outp[i] = (uint32_t)cut_i;
}

}  // namespace dsort
