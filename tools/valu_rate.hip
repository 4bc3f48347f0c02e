// VALU throughput per SIMD on gfx950 for the instruction classes of the draw kernels
// (diagnostic; the roofline of draw_lane_kernel is its VALU issue rate).
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip && tools/valu_rate
// Each kernel runs 8 independent chains of N instructions per lane, 8 waves per SIMD (2048
// workgroups of 256 threads on 256 CUs), so issue -- not latency -- bounds it.  Prints cycles per
// wave-instruction per SIMD: 2 = one wave64 VALU every 2 cycles (SIMD-32), 4 = every 4 cycles.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;  // x 8 chains x 8 unrolled ops

#define CHAINS(OP)                                                                      \
    for (int i = 0; i < kIters; ++i) {                                                  \
        _Pragma("unroll") for (int c = 0; c < 8; ++c) { OP(v[c]); }                     \
    }

__global__ __launch_bounds__(256) void k_add(uint32_t *out, uint32_t s) {
    uint32_t v[8];
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c;
#define OPADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "s"(s))
    CHAINS(OPADD)
    uint32_t r = 0;
    for (int c = 0; c < 8; ++c) r ^= v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ __launch_bounds__(256) void k_bcnt(uint32_t *out, uint32_t s) {
    uint32_t v[8];
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c;
#define OPBCNT(x) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "s"(s))
    CHAINS(OPBCNT)
    uint32_t r = 0;
    for (int c = 0; c < 8; ++c) r ^= v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ __launch_bounds__(256) void k_cndmask(uint32_t *out, uint32_t s) {
    uint32_t v[8];
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c;
#define OPCND(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(x) : "v"(s))
    CHAINS(OPCND)
    uint32_t r = 0;
    for (int c = 0; c < 8; ++c) r ^= v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ __launch_bounds__(256) void k_mul24sdwa(uint32_t *out, uint32_t s) {
    uint32_t v[8];
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c;
#define OPMUL(x) asm volatile("v_mul_i32_i24_sdwa %0, sext(%0), %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0" : "+v"(x) : "v"(s))
    CHAINS(OPMUL)
    uint32_t r = 0;
    for (int c = 0; c < 8; ++c) r ^= v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ __launch_bounds__(256) void k_fma(float *out, float s) {
    float v[8];
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c;
#define OPFMA(x) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(s))
    CHAINS(OPFMA)
    float r = 0;
    for (int c = 0; c < 8; ++c) r += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <typename K, typename T>
void run(const char *name, K kern, T *d, T arg) {
    const int blocks = 2048, threads = 256;
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
    // cycles per wave-instruction per SIMD at the reported peak clock (and the clock it implies at 2 / 4)
    const double cyc = sec * clk_khz * 1e3 * simds / insts;
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"cycles_per_wave_inst_per_simd_at_peak_clock\": %.3f, "
           "\"peak_clock_MHz\": %.0f, \"wave_inst_per_s_per_simd\": %.4g, \"wave_inst_per_s_chip\": %.4g}\n",
           name, ms, cyc, clk_khz / 1e3, insts / sec / simds, insts / sec);
}

int main() {
    uint32_t *d;
    float *f;
    hipMalloc(&d, 2048 * 256 * 4);
    hipMalloc(&f, 2048 * 256 * 4);
    run("v_add_u32", k_add, d, 3u);
    run("v_bcnt", k_bcnt, d, 3u);
    run("v_cndmask", k_cndmask, d, 3u);
    run("v_mul24_sdwa", k_mul24sdwa, d, 3u);
    run("v_fma_f32", k_fma, f, 1.0001f);
    hipFree(d);
    hipFree(f);
    return 0;
}
