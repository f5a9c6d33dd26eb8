// Probe of the cross-lane primitives the wave bitonic network relies on (gfx950):
// prints, for each primitive, which source lane every destination lane received.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL, int RM, int BM>
__device__ int dpp(int old, int x) { return __builtin_amdgcn_update_dpp(old, x, CTRL, RM, BM, false); }

__global__ void probe(int *out) {
    const int t = threadIdx.x;
    int x = t, y = 1000 + t;
    int k = 0;
    out[64 * k++ + t] = dpp<0x104, 0xF, 0xF>(-1, x);          // row_shl:4
    out[64 * k++ + t] = dpp<0x114, 0xF, 0xF>(-1, x);          // row_shr:4
    out[64 * k++ + t] = dpp<0x128, 0xF, 0xF>(-1, x);          // row_ror:8
    out[64 * k++ + t] = dpp<0x140, 0xF, 0xF>(-1, x);          // row_mirror
    out[64 * k++ + t] = dpp<0x141, 0xF, 0xF>(-1, x);          // row_half_mirror
    out[64 * k++ + t] = dpp<0xB1, 0xF, 0xF>(-1, x);           // quad_perm [1,0,3,2]
    out[64 * k++ + t] = dpp<0x1B, 0xF, 0xF>(-1, x);           // quad_perm [3,2,1,0]
    out[64 * k++ + t] = dpp<0x4E, 0xF, 0xF>(-1, x);           // quad_perm [2,3,0,1]
    {   // xor 4 by two bank-masked shifts
        int p = dpp<0x104, 0xF, 0x5>(-1, x);
        p = dpp<0x114, 0xF, 0xA>(p, x);
        out[64 * k++ + t] = p;
    }
    {
        auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
        out[64 * k++ + t] = r[0];
        out[64 * k++ + t] = r[1];
    }
    {
        auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
        out[64 * k++ + t] = r[0];
        out[64 * k++ + t] = r[1];
    }
    {
        int m;
        int c = (t & 1) ? 0x7fffffff : (int)0x80000000;
        int p = dpp<0xB1, 0xF, 0xF>(-1, 63 - t);
        int v = 63 - t;
        asm volatile("v_med3_i32 %0, %1, %2, %3" : "=v"(m) : "v"(v), "v"(p), "v"(c));
        out[64 * k++ + t] = m;
    }
}

int main() {
    int *d, h[64 * 16];
    hipMalloc(&d, sizeof(h));
    hipMemset(d, 0xff, sizeof(h));
    probe<<<1, 64>>>(d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char *names[] = {"row_shl4", "row_shr4", "row_ror8", "row_mirror", "row_half_mirror",
                           "qp_1032", "qp_3210", "qp_2301", "xor4_banks", "pl16_r0", "pl16_r1",
                           "pl32_r0", "pl32_r1", "med3_xor1"};
    for (int k = 0; k < 14; ++k) {
        printf("%-16s", names[k]);
        for (int t = 0; t < 64; ++t) printf(" %d", h[64 * k + t]);
        printf("\n");
    }
    return 0;
}
