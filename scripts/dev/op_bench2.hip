// VALU issue rate per instruction kind on gfx950 (dev tool): 16 independent registers per lane,
// 8 waves/SIMD, one inline-asm instruction per register per iteration.  Prints cycles per
// wave64 instruction per SIMD at 2.4 GHz (the chip may clock lower under load: compare rows).
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP1(ins) asm volatile(ins " %0, %0, %1" : "+v"(x[i]) : "v"(y))
#define OP2(ins) asm volatile(ins " %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(c))

template <int MODE>
__global__ void __launch_bounds__(1024, 8) opb(int *out, int iters) {
    int x[16];
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = t * 77 + i * 1231 + blockIdx.x;
    const int y = t * 3 + 1, c = (t & 1) ? 0x7f7fffff : 0;
    long long z[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = ((long long)x[i] << 32) | x[i + 8];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if constexpr (MODE == 0) OP1("v_min_i32");
            else if constexpr (MODE == 1) OP1("v_min_f32");
            else if constexpr (MODE == 2) OP2("v_med3_i32");
            else if constexpr (MODE == 3) OP2("v_med3_f32");
            else if constexpr (MODE == 4) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
            else if constexpr (MODE == 5) asm volatile("v_min_f32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]) : "v"(y));
            else if constexpr (MODE == 6) asm volatile("v_min_i32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]) : "v"(y));
            else if constexpr (MODE == 7) OP1("v_pk_min_i16");
            else if constexpr (MODE == 8) OP2("v_min3_i32");
            else if constexpr (MODE == 9) OP1("v_xor_b32");
            else if constexpr (MODE == 10) OP1("v_add_u32");
            else if constexpr (MODE == 11) { if (i & 1) continue; auto r = __builtin_amdgcn_permlane32_swap((unsigned)x[i], (unsigned)x[i + 1], false, false); x[i] = (int)r[0]; x[i + 1] = (int)r[1]; }
            else if constexpr (MODE == 12) { if (i >= 8) continue; asm volatile("v_cmp_lt_i64 vcc, %0, %1\n\tv_cndmask_b32 %2, %2, %3, vcc" : : "v"(z[i]), "v"(z[(i + 1) & 7]), "v"(x[i]), "v"(x[i + 8])); }
            else if constexpr (MODE == 13) OP1("v_max_f32");
            else if constexpr (MODE == 14) OP2("v_cndmask_b32");  // placeholder shape (vcc form below)
            else if constexpr (MODE == 15) { if (i >= 8) continue; asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(z[i]) : "v"(z[(i + 3) & 7])); }
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
    const char *names[] = {"v_min_i32", "v_min_f32", "v_med3_i32", "v_med3_f32", "v_mov_b32_dpp",
                           "v_min_f32_dpp", "v_min_i32_dpp", "v_pk_min_i16", "v_min3_i32", "v_xor_b32",
                           "v_add_u32", "v_permlane32_swap (per reg pair)", "v_cmp_lt_i64+cndmask (per pair)",
                           "v_max_f32", "v_cndmask(vop3 s)", "v_pk_add_f32"};
    float ms[16];
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
    ms[14] = 0;
    ms[15] = run<15>(d, blocks, iters);
    for (int m = 0; m < 16; ++m) {
        if (m == 14) continue;
        const double per = (m == 11 || m == 12 || m == 15) ? 8 : 16;  // instructions (pairs) per iteration
        const double winst = (double)blocks * 16 / 1024 * iters * per;
        printf("%-34s %.3f ms  %.2f cyc/wave-instr/SIMD @2.4GHz\n", names[m], ms[m], ms[m] * 1e6 / winst * 2.4);
    }
    return 0;
}
