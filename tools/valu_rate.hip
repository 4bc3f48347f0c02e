// VALU throughput per SIMD on gfx950 for the instruction classes of the draw kernels
// (diagnostic; the roofline of the draw kernels is their VALU issue rate).
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip && tools/valu_rate
// Each kernel runs 8 independent chains of N instructions per lane, with 1, 2, 4 or 8 waves per
// SIMD (256, 512, 1024, 2048 workgroups of 256 threads on 256 CUs: the dispatcher spreads a
// workgroup's 4 waves over the CU's 4 SIMDs), so issue -- not latency -- bounds it once a SIMD holds
// enough waves.  Prints cycles per wave-instruction per SIMD at the reported peak clock: 2 = one
// wave64 VALU every 2 cycles (SIMD-32 at full rate), 4 = every 4 cycles.  Packed ops (v_pk_*) do two
// 16- or 32-bit operations per lane per instruction: their rows say whether that doubles the work
// per issue slot (same cycles as the scalar form) or not.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;  // x 8 chains x 8 unrolled ops

#define CHAINS(OP)                                                                      \
    for (int i = 0; i < kIters; ++i) {                                                  \
        _Pragma("unroll") for (int c = 0; c < 8; ++c) { OP(v[c]); }                     \
    }

#define KERNEL_U32(NAME, OP)                                                            \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t s) {            \
        uint32_t v[8];                                                                  \
        for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c;                             \
        CHAINS(OP)                                                                      \
        uint32_t r = 0;                                                                 \
        for (int c = 0; c < 8; ++c) r ^= v[c];                                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                 \
    }

#define OPADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "s"(s))
#define OPBCNT(x) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "s"(s))
#define OPCND(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(x) : "v"(s))
#define OPMUL(x) asm volatile("v_mul_i32_i24_sdwa %0, sext(%0), %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0" : "+v"(x) : "v"(s))
#define OPMAD24(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(s))
#define OPPKADD16(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(s))
// encodings: _e32 = the 32-bit VOP1 / VOP2 form (VGPR second source; cndmask reads VCC), _e64 = the
// 64-bit VOP3 form of the same operation
#define OPADD32(x) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(x) : "v"(s))
#define OPADD64(x) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(s))
#define OPAND32(x) asm volatile("v_and_b32_e32 %0, %0, %1" : "+v"(x) : "v"(s))
#define OPAND64(x) asm volatile("v_and_b32_e64 %0, %0, %1" : "+v"(x) : "v"(s))
#define OPXOR32(x) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(x) : "v"(s))
#define OPLSH32(x) asm volatile("v_lshlrev_b32_e32 %0, 1, %0" : "+v"(x))
#define OPCND32(x) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(s))
#define OPMOV32(x) asm volatile("v_mov_b32_e32 %0, %1" : "+v"(x) : "v"(s))
#define OPNOT32(x) asm volatile("v_not_b32_e32 %0, %0" : "+v"(x))
#define OPBFE(x) asm volatile("v_bfe_u32 %0, %0, 3, 9" : "+v"(x))
#define OPADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(s))
#define OPBITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x1e" : "+v"(x) : "v"(s))
#define OPDPP(x) asm volatile("v_add_u32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(s))
#define OPMUL24E32(x) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(x) : "v"(s))
#define OPANDC(x) asm volatile("v_and_b32_e32 %0, 0x7fffffff, %0" : "+v"(x))
#define OPANDI(x) asm volatile("v_and_b32_e32 %0, 63, %0" : "+v"(x))
#define OPANDS(x) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(x) : "s"(s))
#define OPLSHV(x) asm volatile("v_lshlrev_b32_e32 %0, %1, %0" : "+v"(x) : "v"(s))
#define OPADDI(x) asm volatile("v_add_u32_e32 %0, 5, %0" : "+v"(x))
#define OPBCNTV(x) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "v"(s))
#define OP_k_or32(x) asm volatile("v_or_b32_e32 %0, %0, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_or32, OP_k_or32)
#define OP_k_sub32(x) asm volatile("v_sub_u32_e32 %0, %0, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_sub32, OP_k_sub32)
#define OP_k_max32(x) asm volatile("v_max_u32_e32 %0, %0, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_max32, OP_k_max32)
#define OP_k_min32(x) asm volatile("v_min_u32_e32 %0, %0, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_min32, OP_k_min32)
#define OP_k_lshr32(x) asm volatile("v_lshrrev_b32_e32 %0, %1, %0" : "+v"(x) : "v"(s))
KERNEL_U32(k_lshr32, OP_k_lshr32)
#define OP_k_lshlor(x) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_lshlor, OP_k_lshlor)
#define OP_k_andor(x) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_andor, OP_k_andor)
#define OP_k_bfi(x) asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_bfi, OP_k_bfi)
#define OP_k_alignbit(x) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(s))
KERNEL_U32(k_alignbit, OP_k_alignbit)
#define OP_k_perm(x) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_perm, OP_k_perm)
#define OP_k_mulhi(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_mulhi, OP_k_mulhi)
#define OP_k_mullo(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_mullo, OP_k_mullo)
#define OP_k_cmpvcc(x) asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1\n v_mov_b32_e32 %0, %0" : "+v"(x) : "v"(s) : "vcc")
KERNEL_U32(k_cmpvcc, OP_k_cmpvcc)
#define OP_k_movdpp(x) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(s))
KERNEL_U32(k_movdpp, OP_k_movdpp)
#define OP_k_cndvcc(x) asm volatile("v_cmp_gt_u32_e32 vcc, %1, %0\n v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(s) : "vcc")
KERNEL_U32(k_cndvcc, OP_k_cndvcc)
#define OP_k_cndsg(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(x) : "v"(s) : "s40", "s41")
KERNEL_U32(k_cndsg, OP_k_cndsg)
#define OP_k_cmpsg(x) asm volatile("v_cmp_gt_u32_e64 s[40:41], %0, %1\n v_mov_b32_e32 %0, %0" : "+v"(x) : "v"(s) : "s40", "s41")
KERNEL_U32(k_cmpsg, OP_k_cmpsg)
#define OP_k_sadu(x) asm volatile("v_max3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_sadu, OP_k_sadu)
#define OP_k_pkadd16v(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(s))
KERNEL_U32(k_pkadd16v, OP_k_pkadd16v)
#define OP_k_addco(x) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(x) : "v"(s) : "vcc")
KERNEL_U32(k_addco, OP_k_addco)
KERNEL_U32(k_andc, OPANDC)
KERNEL_U32(k_andi, OPANDI)
KERNEL_U32(k_ands, OPANDS)
KERNEL_U32(k_lshv, OPLSHV)
KERNEL_U32(k_addi, OPADDI)
KERNEL_U32(k_bcntv, OPBCNTV)
KERNEL_U32(k_add32, OPADD32)

// Mixed streams: chain c runs FULL when c % PERIOD < NFULL, else HALF; the cycles per instruction against
// the weighted mean of the pure rates say whether the two classes add up or overlap.
#define MIXK(NAME, FULLOP, HALFOP, PERIOD, NFULL)                                       \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t s) {            \
        uint32_t v[8];                                                                  \
        for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c;                             \
        for (int i = 0; i < kIters; ++i) {                                              \
            _Pragma("unroll") for (int c = 0; c < 8; ++c) {                             \
                if (c % PERIOD < NFULL) { FULLOP(v[c]); } else { HALFOP(v[c]); }        \
            }                                                                           \
        }                                                                               \
        uint32_t r = 0;                                                                 \
        for (int c = 0; c < 8; ++c) r ^= v[c];                                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                 \
    }
MIXK(k_mix_add_bcnt_11, OPADD32, OPBCNTV, 2, 1)
MIXK(k_mix_add_bcnt_31, OPADD32, OPBCNTV, 4, 3)
MIXK(k_mix_add_bcnt_13, OPADD32, OPBCNTV, 4, 1)
MIXK(k_mix_and_lshl_11, OPAND32, OPLSHV, 2, 1)
MIXK(k_mix_add_mulhi_11, OPADD32, OP_k_mulhi, 2, 1)
MIXK(k_mix_xor_bitop3_11, OPXOR32, OPBITOP3, 2, 1)
KERNEL_U32(k_add64, OPADD64)
KERNEL_U32(k_and32, OPAND32)
KERNEL_U32(k_and64, OPAND64)
KERNEL_U32(k_xor32, OPXOR32)
KERNEL_U32(k_lsh32, OPLSH32)
KERNEL_U32(k_cnd32, OPCND32)
KERNEL_U32(k_mov32, OPMOV32)
KERNEL_U32(k_not32, OPNOT32)
KERNEL_U32(k_bfe, OPBFE)
KERNEL_U32(k_add3, OPADD3)
KERNEL_U32(k_bitop3, OPBITOP3)
KERNEL_U32(k_dpp, OPDPP)
KERNEL_U32(k_mul24e32, OPMUL24E32)
KERNEL_U32(k_add, OPADD)
KERNEL_U32(k_bcnt, OPBCNT)
KERNEL_U32(k_cndmask, OPCND)
KERNEL_U32(k_mul24sdwa, OPMUL)
KERNEL_U32(k_mad24, OPMAD24)
KERNEL_U32(k_pk_add_u16, OPPKADD16)

__global__ __launch_bounds__(256) void k_fma(float *out, float s) {
    float v[8];
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c;
#define OPFMA(x) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(s))
    CHAINS(OPFMA)
    float r = 0;
    for (int c = 0; c < 8; ++c) r += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ __launch_bounds__(256) void k_mul_f32(float *out, float s) {
    float v[8];
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c;
#define OPMULF(x) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(s))
    CHAINS(OPMULF)
    float r = 0;
    for (int c = 0; c < 8; ++c) r += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
// packed f32: one instruction = two f32 operations per lane (64-bit register pairs)
__global__ __launch_bounds__(256) void k_pk_mul_f32(float *out, float s) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 v[8];
    const f2 ss = {s, s};
    for (int c = 0; c < 8; ++c) v[c] = f2{(float)threadIdx.x + c, (float)c};
#define OPPKMUL(x) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x) : "v"(ss))
    CHAINS(OPPKMUL)
    float r = 0;
    for (int c = 0; c < 8; ++c) r += v[c].x + v[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ __launch_bounds__(256) void k_pk_fma_f32(float *out, float s) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 v[8];
    const f2 ss = {s, s};
    for (int c = 0; c < 8; ++c) v[c] = f2{(float)threadIdx.x + c, (float)c};
#define OPPKFMA(x) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(ss))
    CHAINS(OPPKFMA)
    float r = 0;
    for (int c = 0; c < 8; ++c) r += v[c].x + v[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <typename K, typename T>
void run(const char *name, K kern, T *d, T arg, int waves_per_simd, int ops_per_inst) {
    const int threads = 256, blocks = 256 * waves_per_simd;  // 256 CUs x 4 SIMDs
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, arg);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, arg);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    int clk_khz = 0;
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    const double waves = (double)blocks * threads / 64 * 5;
    const double insts = waves * kIters * 8;          // wave-instructions
    const double simds = 256.0 * 4;
    const double sec = ms * 1e-3;
    const double cyc = sec * clk_khz * 1e3 * simds / insts;
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ops_per_lane_per_inst\": %d, \"ms\": %.4f, "
           "\"cycles_per_wave_inst_per_simd_at_peak_clock\": %.3f, \"peak_clock_MHz\": %.0f, "
           "\"wave_inst_per_s_per_simd\": %.4g, \"wave_inst_per_s_chip\": %.4g}\n",
           name, waves_per_simd, ops_per_inst, ms, cyc, clk_khz / 1e3, insts / sec / simds, insts / sec);
}

int main(int argc, char **argv) {
    (void)argv;
    uint32_t *d;
    float *f;
    hipMalloc(&d, 2048 * 256 * 4);
    hipMalloc(&f, 2048 * 256 * 4);
    const bool encodings = argc > 1;  // `valu_rate enc`: the encoding comparison only (4 and 8 waves)
    if (encodings) {
        for (int w : {4, 8}) {
            run("mix add:bcnt 1:1", k_mix_add_bcnt_11, d, 3u, w, 1);
            run("mix add:bcnt 3:1", k_mix_add_bcnt_31, d, 3u, w, 1);
            run("mix add:bcnt 1:3", k_mix_add_bcnt_13, d, 3u, w, 1);
            run("mix and:lshlrev 1:1", k_mix_and_lshl_11, d, 3u, w, 1);
            run("mix add:mul_hi 1:1", k_mix_add_mulhi_11, d, 3u, w, 1);
            run("mix xor:bitop3 1:1", k_mix_xor_bitop3_11, d, 3u, w, 1);
            run("v_or_b32_e32", k_or32, d, 3u, w, 1);
            run("v_sub_u32_e32", k_sub32, d, 3u, w, 1);
            run("v_max_u32_e32", k_max32, d, 3u, w, 1);
            run("v_min_u32_e32", k_min32, d, 3u, w, 1);
            run("v_lshrrev_b32_e32 vgpr", k_lshr32, d, 3u, w, 1);
            run("v_lshl_or_b32", k_lshlor, d, 3u, w, 1);
            run("v_and_or_b32", k_andor, d, 3u, w, 1);
            run("v_bfi_b32", k_bfi, d, 3u, w, 1);
            run("v_alignbit_b32", k_alignbit, d, 3u, w, 1);
            run("v_perm_b32", k_perm, d, 3u, w, 1);
            run("v_mul_hi_u32", k_mulhi, d, 3u, w, 1);
            run("v_mul_lo_u32", k_mullo, d, 3u, w, 1);
            run("v_cmp_gt_u32_e32 (vcc)", k_cmpvcc, d, 3u, w, 1);
            run("v_mov_b32_dpp row_shr:1", k_movdpp, d, 3u, w, 1);
            run("v_cndmask_b32_e32 after vcc write", k_cndvcc, d, 3u, w, 1);
            run("v_cndmask_b32_e64 sgpr cond", k_cndsg, d, 3u, w, 1);
            run("v_cmp_gt_u32_e64 -> sgpr", k_cmpsg, d, 3u, w, 1);
            run("v_max3_u32", k_sadu, d, 3u, w, 1);
            run("v_pk_add_u16 vgpr", k_pkadd16v, d, 3u, w, 1);
            run("v_add_co_u32_e32", k_addco, d, 3u, w, 1);
            run("v_and_b32 literal", k_andc, d, 3u, w, 1);
            run("v_and_b32 inline const", k_andi, d, 3u, w, 1);
            run("v_and_b32 sgpr", k_ands, d, 3u, w, 1);
            run("v_lshlrev_b32 vgpr amount", k_lshv, d, 3u, w, 1);
            run("v_add_u32 inline const", k_addi, d, 3u, w, 1);
            run("v_bcnt_u32_b32 vgpr", k_bcntv, d, 3u, w, 1);
            run("v_add_u32_e32", k_add32, d, 3u, w, 1);
            run("v_add_u32_e64", k_add64, d, 3u, w, 1);
            run("v_and_b32_e32", k_and32, d, 3u, w, 1);
            run("v_and_b32_e64", k_and64, d, 3u, w, 1);
            run("v_xor_b32_e32", k_xor32, d, 3u, w, 1);
            run("v_lshlrev_b32_e32", k_lsh32, d, 3u, w, 1);
            run("v_cndmask_b32_e32", k_cnd32, d, 3u, w, 1);
            run("v_mov_b32_e32", k_mov32, d, 3u, w, 1);
            run("v_not_b32_e32", k_not32, d, 3u, w, 1);
            run("v_mul_u32_u24_e32", k_mul24e32, d, 3u, w, 1);
            run("v_bfe_u32", k_bfe, d, 3u, w, 1);
            run("v_add3_u32", k_add3, d, 3u, w, 1);
            run("v_bitop3_b32", k_bitop3, d, 3u, w, 1);
            run("v_add_u32_dpp", k_dpp, d, 3u, w, 1);
            run("v_mul_f32", k_mul_f32, f, 1.0001f, w, 1);
            run("v_fma_f32", k_fma, f, 1.0001f, w, 1);
        }
        hipFree(d);
        hipFree(f);
        return 0;
    }
    for (int w : {1, 2, 4, 8}) {
        run("v_add_u32", k_add, d, 3u, w, 1);
        run("v_bcnt", k_bcnt, d, 3u, w, 1);
        run("v_cndmask", k_cndmask, d, 3u, w, 1);
        run("v_mul24_sdwa", k_mul24sdwa, d, 3u, w, 1);
        run("v_mad_u32_u24", k_mad24, d, 3u, w, 1);
        run("v_pk_add_u16", k_pk_add_u16, d, 3u, w, 2);
        run("v_fma_f32", k_fma, f, 1.0001f, w, 1);
        run("v_mul_f32", k_mul_f32, f, 1.0001f, w, 1);
        run("v_pk_mul_f32", k_pk_mul_f32, f, 1.0001f, w, 2);
        run("v_pk_fma_f32", k_pk_fma_f32, f, 1.0001f, w, 2);
    }
    hipFree(d);
    hipFree(f);
    return 0;
}
