// Throughput of the register networks alone (no LDS, no barriers): every wave runs the
// 1024-key half-cleaner network (merge_net) or the full wave sort (sort_wave) ITERS times.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../distributed-sorting-with-fault-tolerance_amd/csrc/dsort_wave.hip"

using namespace dsort::wv;

// Experiment: the four lane-bit-0..3 stages of merge_net with the partner fetched by ds_swizzle
// (LDS crossbar, no VALU) instead of a DPP move: 1 VALU (v_med3) per register instead of 2.
template <int XOR>
__device__ __forceinline__ int swz(int x) {
    return __builtin_amdgcn_ds_swizzle(x, (XOR << 10) | 0x1F);
}
__device__ __forceinline__ void merge_net_swz(int (&x)[R], int c0, int c1, int c2, int c3) {
#pragma unroll
    for (int b = 3; b >= 0; --b) {
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (!(i & (1 << b))) cex(x[i], x[i | (1 << b)]);
    }
#pragma unroll
    for (int k = 0; k < R; k += 2) {
        swap32(x[k], x[k + 1]);
        cex(x[k], x[k + 1]);
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
        if (k & 2) continue;
        swap16(x[k], x[k + 2]);
        cex(x[k], x[k + 2]);
    }
    int y[R];
#pragma unroll
    for (int i = 0; i < R; ++i) y[i] = swz<8>(x[i]);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = med3(x[i], y[i], c3);
#pragma unroll
    for (int i = 0; i < R; ++i) y[i] = swz<4>(x[i]);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = med3(x[i], y[i], c2);
#pragma unroll
    for (int i = 0; i < R; ++i) y[i] = swz<2>(x[i]);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = med3(x[i], y[i], c1);
#pragma unroll
    for (int i = 0; i < R; ++i) y[i] = swz<1>(x[i]);
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = med3(x[i], y[i], c0);
}

template <int MODE>
__global__ void __launch_bounds__(1024, 8) netbench(int *out, int iters, int seed) {
    int x[R];
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = (t * 2654435761u + i * 40503u + seed) ^ (blockIdx.x << 7);
    const int c[6] = {lane_side(0), lane_side(1), lane_side(2), lane_side(3), lane_side(4), lane_side(5)};
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) merge_net(x, c[0], c[1], c[2], c[3]);
        else if (MODE == 2) merge_net_swz(x, c[0], c[1], c[2], c[3]);
        else sort_wave(x, c);
        x[it & 15] ^= it;  // keep the loop honest
    }
    int acc = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) acc ^= x[i];
    out[blockIdx.x * 1024 + t] = acc;
}

int main() {
    int *d;
    const int blocks = 256 * 2 * 4;
    (void)hipMalloc(&d, blocks * 1024 * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int mode = 0; mode < 3; ++mode) {
        const int iters = mode == 1 ? 8 : 64;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a);
            if (mode == 0) netbench<0><<<blocks, 1024>>>(d, iters, rep);
            else if (mode == 2) netbench<2><<<blocks, 1024>>>(d, iters, rep);
            else netbench<1><<<blocks, 1024>>>(d, iters, rep);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            const double keys = (double)blocks * 16 * 1024 * iters;
            printf("%s: %.3f ms, %.2f ns per 1024-key network per SIMD-slot, %.1f Gkey-nets/s\n",
                   mode == 0 ? "merge_net" : (mode == 2 ? "merge_net_swz" : "sort_wave"), ms, ms * 1e6 / (blocks * 16.0 * iters / 1024.0),
                   keys / ms / 1e6);
        }
    }
    return 0;
}
