// How many VALU / MFMA instructions of different waves can one SIMD run at once?  One 1024-thread
// workgroup per CU (16 waves, four per SIMD: waves w, w + 4, w + 8, w + 12 share SIMD w % 4 -- checked
// with HW_ID); the four wave quartets run roles A, B, C, D.  Roles: 0 idle, 1 MFMA (8 independent fp4
// 32x32x64 accumulators), 2 v_xor_b32, 3 v_bfi_b32, 4 v_bcnt_u32_b32, 5 v_cndmask_b32 (VCC), 6
// v_mul_i32_i24, 7 v_add_u32 with an SGPR operand, 8 v_lshlrev_b32, 9 v_cmp_gt_u32 (VOPC), 10 v_mov_b32
// DPP, 11 v_pk_add_u16 -- 8 independent chains of each.  (The MFMA role spills at this workgroup size:
// its rows say nothing; tools/mfma_rate.hip measures the MFMA.)
// Each wave times its loop with s_memtime; the host prints the mean cycles per instruction of each
// quartet.  rocprofv3 --pmc over it calibrates SQ_ACTIVE_INST_VALU / SQ_ACTIVE_INST_VALU2.
// Diagnostic only:
//   hipcc --offload-arch=gfx950 -O3 -o tools/coissue tools/coissue.hip && tools/coissue
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kIters = 4096;

template <int OP>
__device__ __forceinline__ void valu_loop(uint32_t (&x)[8], uint32_t y, uint32_t s) {
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if constexpr (OP == 2) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if constexpr (OP == 3) asm volatile("v_bfi_b32 %0, %0, %1, %0" : "+v"(x[c]) : "v"(y));
            if constexpr (OP == 4) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
            if constexpr (OP == 5) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[c]) : "v"(y));
            if constexpr (OP == 6) asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if constexpr (OP == 7) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x[c]) : "s"(s));
            if constexpr (OP == 8) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x[c]) : "v"(y));
            if constexpr (OP == 9) asm volatile("v_cmp_gt_u32 vcc, %0, %1" ::"v"(x[c]), "v"(y) : "vcc");
            if constexpr (OP == 10) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[c]));
            if constexpr (OP == 11) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x[c]) : "v"(y));
        }
    }
}

__global__ __launch_bounds__(1024, 1) void k_coissue(int4 roles, unsigned long long *cyc, uint32_t *simd, float *sink,
                                                      uint32_t s) {
    __shared__ uint32_t pad[24 * 1024];  // 96 KB: one workgroup per CU
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = wave >> 2;
    const int role = q == 0 ? roles.x : q == 1 ? roles.y : q == 2 ? roles.z : roles.w;
    if (threadIdx.x == 0) pad[0] = 1;
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("v_cmp_ne_u32 vcc, 0, %0" ::"v"(lane & 1) : "vcc");
    const unsigned long long t0 = __builtin_readcyclecounter();
    float out = 0.f;
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
        for (int a = 0; a < 8; ++a) out += acc[a][0];
    } else if (role >= 2) {
        uint32_t x[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) x[c] = lane + c;
        const uint32_t y = lane * 7;
        switch (role) {
            case 2: valu_loop<2>(x, y, s); break;
            case 3: valu_loop<3>(x, y, s); break;
            case 4: valu_loop<4>(x, y, s); break;
            case 5: valu_loop<5>(x, y, s); break;
            case 6: valu_loop<6>(x, y, s); break;
            case 7: valu_loop<7>(x, y, s); break;
            case 8: valu_loop<8>(x, y, s); break;
            case 9: valu_loop<9>(x, y, s); break;
            case 10: valu_loop<10>(x, y, s); break;
            default: valu_loop<11>(x, y, s); break;
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) out += (float)x[c];
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) {
        const int g = blockIdx.x * 16 + wave;
        cyc[g] = t1 - t0;
        simd[g] = (hw >> 4) & 3;
    }
    sink[blockIdx.x * 1024 + threadIdx.x] = out + (float)pad[(lane * 37) & 1023];
}

int main() {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned long long *d_c;
    uint32_t *d_s;
    float *d_f;
    (void)hipMalloc(&d_c, cus * 16 * 8);
    (void)hipMalloc(&d_s, cus * 16 * 4);
    (void)hipMalloc(&d_f, cus * 1024 * 4);
    const char *names[] = {"idle", "mfma", "xor", "bfi", "bcnt", "cndmask", "mul24", "add_sgpr", "lshl", "cmp", "dpp",
                           "pk_add"};
    // (A, B, C, D) per case: single waves, pairs, quartets of one op, mixes
    const int cases[][4] = {{2, 0, 0, 0}, {3, 0, 0, 0}, {4, 0, 0, 0}, {5, 0, 0, 0}, {6, 0, 0, 0}, {7, 0, 0, 0},
                            {8, 0, 0, 0}, {2, 2, 0, 0}, {3, 3, 0, 0}, {4, 4, 0, 0}, {5, 5, 0, 0}, {2, 3, 0, 0},
                            {2, 4, 0, 0}, {2, 5, 0, 0}, {2, 2, 2, 2}, {3, 3, 3, 3}, {4, 4, 4, 4}, {5, 5, 5, 5},
                            {6, 6, 6, 6}, {7, 7, 7, 7}, {8, 8, 8, 8}, {2, 2, 4, 4}, {2, 2, 5, 5}, {1, 0, 0, 0},
                            {1, 2, 0, 0}, {1, 3, 0, 0}, {1, 2, 2, 2}, {1, 3, 3, 3}, {1, 1, 0, 0}, {9, 9, 9, 9},
                            {10, 10, 10, 10}, {11, 11, 11, 11}, {2, 2, 9, 9}};
    for (auto &c : cases) {
        const int4 roles = make_int4(c[0], c[1], c[2], c[3]);
        for (int rep = 0; rep < 2; ++rep)
            hipLaunchKernelGGL(k_coissue, dim3(cus), dim3(1024), 0, 0, roles, d_c, d_s, d_f, 5u);
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> cy(cus * 16);
        std::vector<uint32_t> sm(cus * 16);
        (void)hipMemcpy(cy.data(), d_c, cus * 16 * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(sm.data(), d_s, cus * 16 * 4, hipMemcpyDeviceToHost);
        double per[4] = {0, 0, 0, 0};
        int same = 0;
        for (int g = 0; g < cus; ++g)
            for (int w = 0; w < 16; ++w) {
                per[w >> 2] += cy[g * 16 + w];
                same += sm[g * 16 + w] == (uint32_t)(w & 3);
            }
        printf("{\"roles\": [\"%s\", \"%s\", \"%s\", \"%s\"], \"cycles_per_inst\": [", names[c[0]], names[c[1]],
               names[c[2]], names[c[3]]);
        for (int r = 0; r < 4; ++r) {
            const double ops = c[r] == 1 ? kIters : c[r] ? 8.0 * kIters : 0.0;
            printf("%s%.2f", r ? ", " : "", ops ? per[r] / (4.0 * cus) / ops : 0.0);
        }
        printf("], \"waves_on_expected_simd\": %.3f}\n", same / (16.0 * cus));
    }
    return 0;
}
