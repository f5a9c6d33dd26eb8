// Bin-index formulations on gfx950 (dev micro-benchmark): v_mul_hi_u32 against a float
// multiply with conversions.  16 independent registers per lane, 8 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(1024, 8) opbench(unsigned *out, int iters, unsigned scale, float fs) {
    unsigned x[16];
    const unsigned t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = t * 77u + i * 1231u + blockIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (MODE == 0) {  // xor + add (baseline, 2 ops)
                x[i] = (x[i] ^ (unsigned)it) + 1u;
            } else if (MODE == 1) {  // mul_hi + xor (2 ops)
                x[i] = __umulhi(x[i], scale) ^ (unsigned)it;
            } else if (MODE == 2) {  // cvt + mul + cvt + xor (4 ops)
                x[i] = (unsigned)((float)x[i] * fs) ^ (unsigned)it;
            } else if (MODE == 3) {  // mul_lo + xor (2 ops)
                x[i] = (x[i] * scale) ^ (unsigned)it;
            } else if (MODE == 4) {  // mul_u32_u24 + xor (2 ops)
                x[i] = __umul24(x[i], scale) ^ (unsigned)it;
            }
        }
    }
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= x[i];
    out[blockIdx.x * 1024 + t] = acc;
}

int main() {
    unsigned *d;
    const int blocks = 256 * 2 * 4;
    (void)hipMalloc(&d, blocks * 1024 * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const char *names[] = {"xor+add (2 ops)", "mul_hi+xor (2 ops)", "cvt+mul_f32+cvt+xor (4 ops)", "mul_lo+xor (2 ops)",
                           "mul_u24+xor (2 ops)"};
    const int nops[] = {2, 2, 4, 2, 2};
    const int iters = 256;
    for (int mode = 0; mode < 5; ++mode) {
        float best = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a);
            switch (mode) {
                case 0: opbench<0><<<blocks, 1024>>>(d, iters, 12345u, 0.001f); break;
                case 1: opbench<1><<<blocks, 1024>>>(d, iters, 12345u, 0.001f); break;
                case 2: opbench<2><<<blocks, 1024>>>(d, iters, 12345u, 0.001f); break;
                case 3: opbench<3><<<blocks, 1024>>>(d, iters, 12345u, 0.001f); break;
                case 4: opbench<4><<<blocks, 1024>>>(d, iters, 12345u, 0.001f); break;
            }
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        // wave-instructions per SIMD: blocks*16 waves / 1024 SIMDs * iters * 16 keys * ops
        const double winst = (double)blocks * 16 / 1024 * iters * 16 * nops[mode];
        printf("%-30s %.3f ms  -> %.2f cyc per wave-instruction per SIMD @2.4GHz\n", names[mode], best,
               best * 1e6 / winst * 2.4);
    }
    return 0;
}
