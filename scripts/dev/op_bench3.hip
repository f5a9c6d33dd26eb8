// VALU issue rates, part 2 (dev tool): which ops run at the full SIMD-32 rate (2 cycles per
// wave64 instruction) and which at half rate, with and without DPP, and the cost of
// compare + select formulations of a compare-exchange.  8 waves/SIMD, 16 independent registers.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(1024, 8) opb(int *out, int iters) {
    int x[16];
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = t * 77 + i * 1231 + blockIdx.x;
    const int y = t * 3 + 1;
    long long z[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = ((long long)x[i] << 32) | (unsigned)x[i + 8];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if constexpr (MODE == 0) asm volatile("v_mov_b32 %0, %1" : "=v"(x[i]) : "v"(x[(i + 1) & 15]));
            else if constexpr (MODE == 1) asm volatile("v_add_u32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]) : "v"(y));
            else if constexpr (MODE == 2) asm volatile("v_cmp_gt_i32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(y) : "vcc");
            else if constexpr (MODE == 3) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(y));
            else if constexpr (MODE == 4) asm volatile("v_cmp_gt_i32 vcc, %0, %1" : : "v"(x[i]), "v"(y) : "vcc");
            else if constexpr (MODE == 5) asm volatile("v_cmp_gt_i32_e64 %0, %1, %2" : "=s"(z[i & 7]) : "v"(x[i]), "v"(y));
            else if constexpr (MODE == 6) asm volatile("v_cndmask_b32_dpp %0, %0, %0, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
            else if constexpr (MODE == 7) asm volatile("v_sub_co_u32_dpp %0, vcc, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]) : "v"(y) : "vcc");
            else if constexpr (MODE == 8) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
            else if constexpr (MODE == 9) asm volatile("v_max_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
            else if constexpr (MODE == 10) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(x[(i + 5) & 15]));
            else if constexpr (MODE == 11) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(x[i]));
            else if constexpr (MODE == 12) { if (i >= 8) continue; asm volatile("v_cmp_lt_i64 vcc, %0, %1" : : "v"(z[i]), "v"(z[(i + 1) & 7]) : "vcc"); }
            else if constexpr (MODE == 13) asm volatile("v_mov_b32_dpp %0, %0 row_shl:4 row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
            else if constexpr (MODE == 14) asm volatile("v_mov_b32_dpp %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
            else if constexpr (MODE == 15) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(x[(i + 5) & 15]));
            else if constexpr (MODE == 16) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\ts_nop 0\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(y) : "vcc");
            else if constexpr (MODE == 17) asm volatile("v_subrev_co_u32 %0, vcc, %0, %1" : "+v"(x[i]) : "v"(y) : "vcc");
            else if constexpr (MODE == 18) asm volatile("v_xad_u32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(y));
            else if constexpr (MODE == 19) asm volatile("v_max3_i32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(y));
        }
    }
    int acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= x[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= (int)z[i];
    out[blockIdx.x * 1024 + t] = acc;
}

template <int M>
static float run(int *d, int blocks, int iters) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        opb<M><<<blocks, 1024>>>(d, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    return best;
}

int main() {
    int *d;
    const int blocks = 256 * 2 * 4;
    (void)hipMalloc(&d, blocks * 1024 * 4);
    const int iters = 512;
    const char *names[] = {"v_mov_b32", "v_add_u32_dpp", "v_cmp_gt_i32 vcc + v_cndmask (pair)", "v_cndmask_b32 vcc",
                           "v_cmp_gt_i32 vcc", "v_cmp_gt_i32_e64 sgpr", "v_cndmask_b32_dpp", "v_sub_co_u32_dpp vcc",
                           "v_sub_u32", "v_max_u32", "v_bfi_b32", "v_lshlrev_b32", "v_cmp_lt_i64 vcc",
                           "v_mov_b32_dpp row_shl:4", "v_mov_b32_dpp row_ror:8", "v_perm_b32",
                           "cmp_u32 + nop + cndmask (triple)", "v_subrev_co_u32", "v_xad_u32", "v_max3_i32"};
    float ms[20];
    ms[0] = run<0>(d, blocks, iters);
    ms[1] = run<1>(d, blocks, iters);
    ms[2] = run<2>(d, blocks, iters);
    ms[3] = run<3>(d, blocks, iters);
    ms[4] = run<4>(d, blocks, iters);
    ms[5] = run<5>(d, blocks, iters);
    ms[6] = run<6>(d, blocks, iters);
    ms[7] = run<7>(d, blocks, iters);
    ms[8] = run<8>(d, blocks, iters);
    ms[9] = run<9>(d, blocks, iters);
    ms[10] = run<10>(d, blocks, iters);
    ms[11] = run<11>(d, blocks, iters);
    ms[12] = run<12>(d, blocks, iters);
    ms[13] = run<13>(d, blocks, iters);
    ms[14] = run<14>(d, blocks, iters);
    ms[15] = run<15>(d, blocks, iters);
    ms[16] = run<16>(d, blocks, iters);
    ms[17] = run<17>(d, blocks, iters);
    ms[18] = run<18>(d, blocks, iters);
    ms[19] = run<19>(d, blocks, iters);
    for (int m = 0; m < 20; ++m) {
        const double per = (m == 12) ? 8 : 16;  // instruction groups per iteration
        const double winst = (double)blocks * 16 / 1024 * iters * per;
        printf("%-40s %.3f ms  %.2f cyc/group/SIMD @2.4GHz\n", names[m], ms[m], ms[m] * 1e6 / winst * 2.4);
    }
    return 0;
}
