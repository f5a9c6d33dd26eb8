// Per-instruction VALU throughput on gfx950: 16 independent registers per lane, 8 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int med3(int a, int b, int c) {
    int r;
    asm volatile("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <int MODE>
__global__ void __launch_bounds__(1024, 8) opbench(int *out, int iters) {
    int x[16];
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = t * 77 + i * 1231 + blockIdx.x;
    const int c = (t & 1) ? 0x7fffffff : (int)0x80000000;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (MODE == 0) {  // plain min (1 op)
                x[i] = x[i] < x[(i + 1) & 15] ? x[i] : x[(i + 1) & 15];
                x[i] ^= it;
            } else if (MODE == 1) {  // dpp mov + xor
                x[i] = __builtin_amdgcn_mov_dpp(x[i], 0xB1, 0xF, 0xF, false) ^ it;
            } else if (MODE == 2) {  // med3 + xor
                x[i] = med3(x[i], x[(i + 3) & 15], c) ^ it;
            } else if (MODE == 3) {  // permlane32 swap pairs + xor
                if (i & 1) continue;
                auto r = __builtin_amdgcn_permlane32_swap((unsigned)x[i], (unsigned)x[i + 1], false, false);
                x[i] = (int)r[0] ^ it;
                x[i + 1] = (int)r[1] ^ it;
            } else if (MODE == 4) {  // xor only (baseline)
                x[i] = (x[i] ^ it) + 1;
            }
        }
    }
    int acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= x[i];
    out[blockIdx.x * 1024 + t] = acc;
}

int main() {
    int *d;
    const int blocks = 256 * 2 * 4;
    (void)hipMalloc(&d, blocks * 1024 * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const char *names[] = {"min+xor (2 ops)", "dpp+xor (2 ops)", "med3+xor (2 ops)", "permlane32swap+2xor (2 ops/key)", "xor+add (2 ops)"};
    const int iters = 256;
    for (int mode = 0; mode < 5; ++mode) {
        float best = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a);
            switch (mode) {
                case 0: opbench<0><<<blocks, 1024>>>(d, iters); break;
                case 1: opbench<1><<<blocks, 1024>>>(d, iters); break;
                case 2: opbench<2><<<blocks, 1024>>>(d, iters); break;
                case 3: opbench<3><<<blocks, 1024>>>(d, iters); break;
                case 4: opbench<4><<<blocks, 1024>>>(d, iters); break;
            }
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        // wave-instructions per SIMD: blocks*16 waves / 1024 SIMDs * iters * 32 instr
        const double winst = (double)blocks * 16 / 1024 * iters * 32;
        printf("%-34s %.3f ms  -> %.2f ns per wave-instruction per SIMD (%.2f cyc @2.4GHz)\n", names[mode], best,
               best * 1e6 / winst, best * 1e6 / winst * 2.4);
    }
    return 0;
}
