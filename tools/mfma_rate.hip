// Achievable rate of v_mfma_scale_f32_32x32x64_f8f6f4 (fp4 operands) on gfx950 with the shape of
// pair_fp4_tile_kernel: one 256-thread workgroup per CU (one wave per SIMD), NA x 4 independent 32x32
// accumulators per wave (NA = 4: the tile kernel's 256 AGPRs; NA = 2: 128, no register pressure),
// 4 NA MFMAs per "block".  Variants add, per block, the work the
// tile kernel does besides MFMAs: 48 independent VALU (fragment expansion), one s_barrier, 8 LDS
// reads.  Diagnostic only:
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_rate tools/mfma_rate.hip && tools/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kBlocks = 2048;

template <int NA, int VALU, bool BARRIER, bool LDS>
__global__ __launch_bounds__(256, 1) void k_mfma(float *out, int seed) {
    __shared__ uint32_t sm[4096];
    v16f acc[NA][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.0f;
    v8i fa[NA], fb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            if (q < NA) fa[q][e] = seed * (q + 1) + e + (int)threadIdx.x;
            fb[q][e] = seed * (q + 3) - e;
        }
    for (int t = threadIdx.x; t < 4096; t += 256) sm[t] = t * seed;
    __syncthreads();
    uint32_t x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = threadIdx.x + c;
    uint32_t r = 0;
    for (int blk = 0; blk < kBlocks; ++blk) {
        if constexpr (BARRIER) __builtin_amdgcn_s_barrier();
        if constexpr (LDS) {
#pragma unroll
            for (int q = 0; q < 8; ++q) r += sm[(threadIdx.x + 64 * q + blk) & 4095];
        }
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                acc[a][b] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[a], fb[b], acc[a][b], 4, 4, 0,
                                                                            0x7F7F7F7F, 0, 0x7F7F7F7F);
                if constexpr (VALU > 0) {
#pragma unroll
                    for (int u = 0; u < VALU / (4 * NA); ++u)
                        asm volatile("v_bfi_b32 %0, %0, %1, %0" : "+v"(x[(a * 4 + b + u) & 7]) : "v"(r));
                }
            }
    }
    float s = 0.0f;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) s += acc[a][b][v];
#pragma unroll
    for (int c = 0; c < 8; ++c) r ^= x[c];
    out[blockIdx.x * 256 + threadIdx.x] = s + (float)r;
}

template <typename K>
void run(const char *name, K kern, float *d, int na) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, d, 3);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, d, 3);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double flops = 256.0 * 4 * kBlocks * 4 * na * (2.0 * 32 * 32 * 64);
    const double pf = flops / (ms * 1e-3) / 1e15;
    printf("{\"variant\": \"%s\", \"accumulators\": %d, \"ms\": %.4f, \"PFLOPs\": %.3f, \"frac_of_10.066PF\": %.3f, \"cycles_per_mfma_at_2400MHz\": %.2f}\n",
           name, 4 * na, ms, pf, pf / 10.066, ms * 1e-3 * 2.4e9 / (kBlocks * 4.0 * na));
}

int main() {
    float *d;
    (void)hipMalloc(&d, 256 * 256 * 4);
    run("mfma only", k_mfma<2, 0, false, false>, d, 2);
    run("+24 valu", k_mfma<2, 24, false, false>, d, 2);
    run("+barrier", k_mfma<2, 0, true, false>, d, 2);
    run("+8 lds", k_mfma<2, 0, false, true>, d, 2);
    run("+24 valu +barrier +8 lds", k_mfma<2, 24, true, true>, d, 2);
    run("mfma only", k_mfma<4, 0, false, false>, d, 4);
    run("+48 valu", k_mfma<4, 48, false, false>, d, 4);
    return 0;
}
