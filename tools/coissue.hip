// Does a MFMA-bound wave and a VALU-bound wave on the SAME SIMD overlap?  One 512-thread workgroup per
// CU (8 waves, two per SIMD: wave w and w + 4 share SIMD w % 4 -- checked with HW_ID), waves 0-3 run
// role A, waves 4-7 role B.  Roles: 0 idle, 1 MFMA (8 independent fp4 32x32x64 accumulators), 2 VALU
// (8 independent chains of v_xor_b32), 3 VALU slow class (v_bfi_b32).  Each wave times its loop with
// s_memtime; the host prints mean cycles per role.  Diagnostic only (config-5 co-residence):
//   hipcc --offload-arch=gfx950 -O3 -o tools/coissue tools/coissue.hip && tools/coissue
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kIters = 4096;

__global__ __launch_bounds__(512, 1) void k_coissue(int role_a, int role_b, unsigned long long *cyc, uint32_t *simd,
                                                     float *sink) {
    __shared__ uint32_t pad[24 * 1024];  // 96 KB: one workgroup per CU
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int role = wave < 4 ? role_a : role_b;
    if (threadIdx.x == 0) pad[0] = 1;
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const unsigned long long t0 = __builtin_readcyclecounter();
    float s = 0.f;
    if (role == 1) {
        v16f acc[8];
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[a][v] = 0.f;
        v8i fa, fb;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            fa[e] = lane + e;
            fb[e] = lane * 3 + e;
        }
        for (int i = 0; i < kIters / 8; ++i)
#pragma unroll
            for (int a = 0; a < 8; ++a)
                acc[a] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa, fb, acc[a], 4, 4, 0, 0x7F7F7F7F, 0,
                                                                         0x7F7F7F7F);
#pragma unroll
        for (int a = 0; a < 8; ++a) s += acc[a][0];
    } else if (role == 2 || role == 3) {
        uint32_t x[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) x[c] = lane + c;
        const uint32_t y = lane * 7;
        if (role == 2) {
            for (int i = 0; i < kIters; ++i)
#pragma unroll
                for (int c = 0; c < 8; ++c) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
        } else {
            for (int i = 0; i < kIters; ++i)
#pragma unroll
                for (int c = 0; c < 8; ++c) asm volatile("v_bfi_b32 %0, %0, %1, %0" : "+v"(x[c]) : "v"(y));
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) s += (float)x[c];
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) {
        const int g = blockIdx.x * 8 + wave;
        cyc[g] = t1 - t0;
        simd[g] = (hw >> 4) & 3;
    }
    sink[blockIdx.x * 512 + threadIdx.x] = s + (float)pad[(lane * 37) & 1023];
}

int main() {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned long long *d_c;
    uint32_t *d_s;
    float *d_f;
    (void)hipMalloc(&d_c, cus * 8 * 8);
    (void)hipMalloc(&d_s, cus * 8 * 4);
    (void)hipMalloc(&d_f, cus * 512 * 4);
    const char *names[] = {"idle", "mfma", "valu_xor", "valu_bfi"};
    const int cases[][2] = {{1, 0}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 2}, {1, 1}};
    for (auto &c : cases) {
        for (int rep = 0; rep < 2; ++rep)
            hipLaunchKernelGGL(k_coissue, dim3(cus), dim3(512), 0, 0, c[0], c[1], d_c, d_s, d_f);
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> cy(cus * 8);
        std::vector<uint32_t> sm(cus * 8);
        (void)hipMemcpy(cy.data(), d_c, cus * 8 * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(sm.data(), d_s, cus * 8 * 4, hipMemcpyDeviceToHost);
        double a = 0, b = 0;
        int same = 0;
        for (int g = 0; g < cus; ++g) {
            for (int w = 0; w < 4; ++w) {
                a += cy[g * 8 + w];
                b += cy[g * 8 + 4 + w];
                same += sm[g * 8 + w] == sm[g * 8 + 4 + w];
            }
        }
        a /= 4.0 * cus;
        b /= 4.0 * cus;
        printf("{\"A\": \"%s\", \"B\": \"%s\", \"A_cycles\": %.0f, \"B_cycles\": %.0f, \"A_per_op\": %.2f, "
               "\"B_per_op\": %.2f, \"pairs_on_same_simd\": %.3f}\n",
               names[c[0]], names[c[1]], a, b, a / (c[0] == 1 ? kIters : 8.0 * kIters),
               b / (c[1] == 1 ? kIters : 8.0 * kIters), same / (4.0 * cus));
    }
    return 0;
}
