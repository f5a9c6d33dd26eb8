// LDS merge-level microbenchmark (dev tool): merges a 16384-key LDS tile from sorted runs of 1024
// to one run of 16384 (4 levels) with
//   V0  the bitonic window levels of dsort_wave.hip (merge_net, 15 VALU ops per key per level)
//   V1  a serial merge per lane: merge-path binary search for the lane's 16 outputs, then 16
//       compare/select steps, B runs kept descending in LDS so reads past a run end are harmless
// and checks the tiles against the host sort.  Usage: lvl_bench [log2 tiles]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

constexpr int R = 16, WK = 1024, WAVES = 16, THREADS = 1024, TILE = 16384;
constexpr int KMAX = INT32_MAX, KMIN = INT32_MIN;
constexpr int QP_1032 = 0xB1, QP_2301 = 0x4E, ROW_ROR8 = 0x128;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int med3(int a, int b, int c) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
template <int CTRL> __device__ __forceinline__ int dpp(int x) { return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, false); }
__device__ __forceinline__ int cex_xor4(int x) {
    int y;
    asm volatile("s_nop 1\n\tv_min_i32_dpp %0, %1, %1 row_shl:4 row_mask:0xf bank_mask:0x5\n\tv_max_i32_dpp %0, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xa" : "=&v"(y) : "v"(x));
    return y;
}
__device__ __forceinline__ void cex(int &a, int &b) { const int lo = a < b ? a : b, hi = a < b ? b : a; a = lo; b = hi; }
__device__ __forceinline__ int lane_side(int b) { return ((lane_id() >> b) & 1) ? KMAX : KMIN; }
__device__ __forceinline__ void swap32(int &a, int &b) { const auto r = __builtin_amdgcn_permlane32_swap((unsigned)a, (unsigned)b, false, false); a = (int)r[0]; b = (int)r[1]; }
__device__ __forceinline__ void swap16(int &a, int &b) { const auto r = __builtin_amdgcn_permlane16_swap((unsigned)a, (unsigned)b, false, false); a = (int)r[0]; b = (int)r[1]; }
__device__ __forceinline__ constexpr int out_hi(int i) { return ((i >> 3) & 1) << 9 | ((i >> 2) & 1) << 8 | (i & 1) << 5 | ((i >> 1) & 1) << 4; }
__device__ __forceinline__ int out_lo(int t) { return ((t >> 4) & 1) << 7 | ((t >> 5) & 1) << 6 | (t & 15); }

__device__ __forceinline__ void merge_net(int (&x)[R], int c0, int c1, int c3) {
#pragma unroll
    for (int b = 3; b >= 0; --b)
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (!(i & (1 << b))) cex(x[i], x[i | (1 << b)]);
#pragma unroll
    for (int k = 0; k < R; k += 2) { swap32(x[k], x[k + 1]); cex(x[k], x[k + 1]); }
#pragma unroll
    for (int k = 0; k < R; ++k) { if (k & 2) continue; swap16(x[k], x[k + 2]); cex(x[k], x[k + 2]); }
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = med3(x[i], dpp<ROW_ROR8>(x[i]), c3);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = cex_xor4(x[i]);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = med3(x[i], dpp<QP_2301>(x[i]), c1);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = med3(x[i], dpp<QP_1032>(x[i]), c0);
}

__device__ __forceinline__ int coop_split_desc(const int *s, int pa, int na, int pbe, int nb, int d) {
    int lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    const int lane = lane_id();
#pragma unroll 1
    while (lo < hi) {
        const int len = hi - lo;
        const int st = ((len + 63) >> 6) | 1;
        const int off = (int)__umul24((unsigned)lane, (unsigned)st);
        const int ia = pa + lo + off;
        int ib = pbe - d + 1 + lo + off;
        ib = ib > pbe ? pbe : ib;
        const bool q = (off >= len) | (s[ia] > s[ib]);
        const unsigned long long m = __ballot(q);
        const int j = m ? (int)__ffsll((long long)m) - 1 : 64;
        const int nhi = lo + j * st < hi ? lo + j * st : hi;
        lo = __builtin_amdgcn_readfirstlane(j ? lo + (j - 1) * st + 1 : lo);
        hi = __builtin_amdgcn_readfirstlane(nhi);
    }
    return lo;
}

__device__ __forceinline__ void load_min(const int *s, int ia0, int ib0, int (&x)[R]) {
    const int t = lane_id();
    const int *sa = s + ia0 + t, *sb = s + ib0 + t;
#pragma unroll
    for (int i = 0; i < R; ++i) { const int a = sa[64 * i], b = sb[64 * i]; x[i] = a < b ? a : b; }
}

// ---------------------------------------------------------------- V0: bitonic windows
__global__ void __launch_bounds__(THREADS, 8) lv_bitonic(const int *in, int *out) {
    __shared__ __attribute__((aligned(16))) int s[TILE + WK];
    const int t = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t base = (size_t)blockIdx.x * TILE;
    // input: runs of 1024 sorted, odd runs stored descending already (host layout)
    {
        const int4 *src = reinterpret_cast<const int4 *>(in + base);
        int4 *dst = reinterpret_cast<int4 *>(s);
#pragma unroll
        for (int q = 0; q < TILE / 4 / THREADS; ++q) dst[q * THREADS + threadIdx.x] = src[q * THREADS + threadIdx.x];
    }
    __syncthreads();
    const int c0 = lane_side(0), c1 = lane_side(1), c3 = lane_side(3);
    const int lo = out_lo(t);
    int x[R];
#pragma unroll 1
    for (int r = WK; r < TILE; r <<= 1) {
        const int wpp = (2 * r) / WK, j = w / wpp, o = w % wpp, ps = j * 2 * r;
        const bool last = 2 * r == TILE, desc = !last && (j & 1);
        const int pbe = ps + 2 * r - 1, d0 = o * WK;
        const int a0 = coop_split_desc(s, ps, r, pbe, r, d0);
        load_min(s, ps + a0, pbe - (d0 - a0) - (WK - 1), x);
        merge_net(x, c0, c1, c3);
        __syncthreads();
        if (last) {
            int *p = out + base + ps + d0 + lo;
#pragma unroll
            for (int i = 0; i < R; ++i) p[out_hi(i)] = x[i];
        } else if (!desc) {
            int *p = s + ps + d0 + lo;
#pragma unroll
            for (int i = 0; i < R; ++i) p[out_hi(i)] = x[i];
            __syncthreads();
        } else {
            int *p = s + ps + (2 * r - 1 - d0) - lo;
#pragma unroll
            for (int i = 0; i < R; ++i) p[-out_hi(i)] = x[i];
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------- V1: serial merge per lane
// Lane (global thread) g produces outputs [16 g, 16 g + 16) of the tile.  Pair layout: A
// ascending at s[pa, pa + na), B descending after it (B[k] at s[pbe - k]); a read of A past its
// end returns B's largest keys and a read of B past its end A's largest keys, so no bounds checks
// are needed while the lane stays inside its pair (16 | pair length here).
template <int PADL>
__device__ __forceinline__ int px(int k) { return PADL ? k + (k >> PADL) : k; }

template <int PADL>
__device__ __forceinline__ void serial16(const int *s, int pa, int na, int pbe, int nb, int d, int (&o)[16]) {
    // merge path: a = number of A keys among the first d outputs (A wins ties)
    int lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        // A[mid] <= B[d - 1 - mid] -> more A
        if (s[px<PADL>(pa + mid)] <= s[px<PADL>(pbe - (d - 1 - mid))]) lo = mid + 1;
        else hi = mid;
    }
    int ia = pa + lo, ib = pbe - (d - lo);  // next A / B positions (B descends)
    int va = s[px<PADL>(ia)], vb = s[px<PADL>(ib)];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const bool p = va <= vb;
        o[j] = p ? va : vb;
        ia += p ? 1 : 0;
        ib -= p ? 0 : 1;
        const int v = s[px<PADL>(p ? ia : ib)];
        va = p ? v : va;
        vb = p ? vb : v;
    }
}

template <int PADL>
__global__ void __launch_bounds__(THREADS, 8) lv_serial(const int *in, int *out) {
    constexpr int SZ = PADL ? TILE + (TILE >> PADL) + 64 : TILE + 64;
    __shared__ __attribute__((aligned(16))) int s[SZ];
    const int g = threadIdx.x;
    const size_t base = (size_t)blockIdx.x * TILE;
    for (int q = g; q < TILE; q += THREADS) s[px<PADL>(q)] = in[base + q];
    __syncthreads();
    int o[16];
#pragma unroll 1
    for (int r = WK; r < TILE; r <<= 1) {
        const int o0 = 16 * g, j = o0 / (2 * r), d = o0 % (2 * r), ps = j * 2 * r;
        const bool last = 2 * r == TILE, desc = !last && (j & 1);
        serial16<PADL>(s, ps, r, ps + 2 * r - 1, r, d, o);
        __syncthreads();
        if (last) {
            int4 *p = reinterpret_cast<int4 *>(out + base + o0);
#pragma unroll
            for (int q = 0; q < 4; ++q) p[q] = make_int4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) s[px<PADL>(desc ? ps + 2 * r - 1 - (d + k) : ps + d + k)] = o[k];
            __syncthreads();
        }
    }
}

int main(int argc, char **argv) {
    const int lt = argc > 1 ? atoi(argv[1]) : 16;
    const size_t tiles = (size_t)1 << lt, n = tiles * TILE;
    std::vector<int> h(n), ref(n);
    std::mt19937_64 rng(7);
    for (size_t i = 0; i < n; ++i) h[i] = (int)(rng() >> 32);
    // a few tiles with heavy duplicates
    for (size_t i = 0; i < 4 * (size_t)TILE && i < n; ++i) h[i] = (int)(rng() % 5) - 2;
    for (size_t i = 4 * (size_t)TILE; i < 6 * (size_t)TILE && i < n; ++i) h[i] = (i & 1) ? INT32_MAX : INT32_MIN;
    for (size_t r0 = 0; r0 < n; r0 += WK) {
        std::sort(h.begin() + r0, h.begin() + r0 + WK);
        if ((r0 / WK) & 1) std::reverse(h.begin() + r0, h.begin() + r0 + WK);
    }
    for (size_t t0 = 0; t0 < n; t0 += TILE) {
        std::copy(h.begin() + t0, h.begin() + t0 + TILE, ref.begin() + t0);
        std::sort(ref.begin() + t0, ref.begin() + t0 + TILE);
    }
    int *din, *dout;
    (void)hipMalloc(&din, n * 4);
    (void)hipMalloc(&dout, n * 4);
    (void)hipMemcpy(din, h.data(), n * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<int> got(n);
    auto bench = [&](const char *name, void (*k)(const int *, int *)) {
        (void)hipMemset(dout, 0, n * 4);
        hipLaunchKernelGGL(k, dim3((unsigned)tiles), dim3(THREADS), 0, 0, din, dout);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(got.data(), dout, n * 4, hipMemcpyDeviceToHost);
        const bool ok = got == ref;
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(k, dim3((unsigned)tiles), dim3(THREADS), 0, 0, din, dout);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            best = std::min(best, ms);
        }
        printf("%-28s %s  %.3f ms for %zu keys (4 levels)  %.1f GB/s\n", name, ok ? "OK " : "BAD", best, n,
               2.0 * 4 * n / (best * 1e-3) / 1e9);
    };
    bench("bitonic windows", lv_bitonic);
    bench("serial, no pad", lv_serial<0>);
    bench("serial, pad 1/32", lv_serial<5>);
    bench("serial, pad 1/16", lv_serial<4>);
    return 0;
}
