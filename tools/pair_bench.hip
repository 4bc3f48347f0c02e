// Microbenchmark of X^T X variants on int8 MFMA (development tool, not part of the product).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/pair_bench tools/pair_bench.hip
// Run:   tools/pair_bench [n] [panels]
// Variants (template MODE): 0 full kernel, 1 no expansion (no VALU / LDS writes), 2 no
// expansion and no barrier, 3 MFMA + LDS reads only from a fixed stage, 4 MFMA only.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            printf("%s: %s\n", #x, hipGetErrorString(e));                                      \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int kPairBlock = 256;
constexpr int kFragBytes = 64 * 16;
constexpr int kPairStage = 2 * 2 * 8 * kFragBytes;

__device__ __forceinline__ v4i expand16(uint32_t bits) {
    v4i r;
    r[0] = (int)(((bits & 0xFu) * 0x00204081u) & 0x01010101u);
    r[1] = (int)((((bits >> 4) & 0xFu) * 0x00204081u) & 0x01010101u);
    r[2] = (int)((((bits >> 8) & 0xFu) * 0x00204081u) & 0x01010101u);
    r[3] = (int)((((bits >> 12) & 0xFu) * 0x00204081u) & 0x01010101u);
    return r;
}

// shift-and expansion: fragment (ks, h) dword q = bits {4h+q + 8j} (j = 0..3) of 32-bit half ks
__device__ __forceinline__ v4i frag_sa(uint64_t w, int ks, int h) {
    const uint32_t x = (uint32_t)(w >> (32 * ks));
    v4i r;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = (int)((x >> (4 * h + q)) & 0x01010101u);
    return r;
}
#ifndef EXPANDV
#define EXPANDV 1
#endif
__device__ __forceinline__ v4i frag_of(uint64_t w, int ks, int h) {
#if EXPANDV
    return frag_sa(w, ks, h);
#else
    return expand16((uint32_t)(w >> (32 * ks + 16 * h)) & 0xFFFFu);
#endif
}

template <int MODE>
__global__ __launch_bounds__(256) void pair_k(const uint64_t *__restrict__ xt, uint64_t nblk, int n, int npad,
                                             int nbt, int nsplit, int64_t *__restrict__ pairs) {
    extern __shared__ __attribute__((aligned(16))) unsigned char pair_lds[];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int item = blockIdx.x;
    const int tri = item / nsplit, split = item - tri * nsplit;
    int bi = 0, rem = tri;
    while (rem >= nbt - bi) {
        rem -= nbt - bi;
        ++bi;
    }
    const int bj = bi + rem;
    const int I0 = bi * kPairBlock, J0 = bj * kPairBlock;
    const uint64_t per = (nblk + nsplit - 1) / nsplit;
    const uint64_t kb0 = (uint64_t)split * per, kb1 = min(nblk, kb0 + per);
    v16i acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[a][b][v] = 0;
    const int sub = t >> 5, r32 = t & 31;
    const int wr = wave >> 1, wc = wave & 1;
    auto expand_to = [&](unsigned char *st, uint64_t wa, uint64_t wb) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int off = ((ks * 8 + sub) * 64 + r32 + 32 * h) * 16;
                *reinterpret_cast<v4i *>(st + off) = frag_of(wa, ks, h);
                *reinterpret_cast<v4i *>(st + 16 * kFragBytes + off) = frag_of(wb, ks, h);
            }
    };
    uint64_t na = 0, nb = 0;
    if (kb0 < kb1) {
        expand_to(pair_lds + (size_t)(kb0 & 1) * kPairStage, xt[kb0 * (uint64_t)npad + I0 + t],
                  xt[kb0 * (uint64_t)npad + J0 + t]);
        expand_to(pair_lds + (size_t)((kb0 + 1) & 1) * kPairStage, xt[kb0 * (uint64_t)npad + I0 + t],
                  xt[kb0 * (uint64_t)npad + J0 + t]);
        if (kb0 + 1 < kb1) {
            na = xt[(kb0 + 1) * (uint64_t)npad + I0 + t];
            nb = xt[(kb0 + 1) * (uint64_t)npad + J0 + t];
        }
    }
    __syncthreads();
    v4i fa[2][4], fb[2][4];
    if (MODE == 4) {
        const unsigned char *st = pair_lds;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                fa[ks][x] = *reinterpret_cast<const v4i *>(st + ((ks * 8 + wr * 4 + x) * 64 + lane) * 16);
                fb[ks][x] = *reinterpret_cast<const v4i *>(st + 16 * kFragBytes + ((ks * 8 + wc * 4 + x) * 64 + lane) * 16);
            }
    }
    for (uint64_t kb = kb0; kb < kb1; ++kb) {
        const unsigned char *st = pair_lds + (size_t)((MODE == 3 ? 0 : kb) & 1) * kPairStage;
        if (MODE != 4) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    fa[ks][x] = *reinterpret_cast<const v4i *>(st + ((ks * 8 + wr * 4 + x) * 64 + lane) * 16);
                    fb[ks][x] = *reinterpret_cast<const v4i *>(st + 16 * kFragBytes + ((ks * 8 + wc * 4 + x) * 64 + lane) * 16);
                }
        }
        if (MODE == 0) {
            expand_to(pair_lds + (size_t)((kb + 1) & 1) * kPairStage, na, nb);
            const uint64_t nk = min(kb + 2, kb1 - 1);
            na = xt[nk * (uint64_t)npad + I0 + t];
            nb = xt[nk * (uint64_t)npad + J0 + t];
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[ks][a], fb[ks][b], acc[a][b], 0, 0, 0);
        if (MODE == 0) {
            __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            }
        }
        if (MODE <= 1) __syncthreads();
    }
    const int rbase = I0 + 128 * wr + 4 * (lane >> 5);
    const int cbase = J0 + 128 * wc + (lane & 31);
    int64_t local = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) local += acc[a][b][v];
    if (rbase < n && cbase < n)
        atomicAdd(reinterpret_cast<unsigned long long *>(pairs + (uint64_t)rbase * n + cbase),
                  (unsigned long long)local);
}

template <int MODE>
float run(const uint64_t *xt, uint64_t nblk, int n, int npad, int64_t *pairs, int cus, int reps) {
    const int nbt = npad / kPairBlock, ntri = nbt * (nbt + 1) / 2;
    int nsplit = std::max(1, cus / ntri);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 2; ++w)
        hipLaunchKernelGGL(pair_k<MODE>, dim3(ntri * nsplit), dim3(256), 2 * kPairStage, nullptr, xt, nblk, n, npad,
                           nbt, nsplit, pairs);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(pair_k<MODE>, dim3(ntri * nsplit), dim3(256), 2 * kPairStage, nullptr, xt, nblk, n, npad,
                           nbt, nsplit, pairs);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

// 8 waves (2 per SIMD): wave (wr = w>>2, wc = w&3) owns rows I0+128wr.. x cols J0+64wc.. (4 x 2 tiles)
template <int MODE>
__global__ __launch_bounds__(512) void pair_k8(const uint64_t *__restrict__ xt, uint64_t nblk, int n, int npad,
                                              int nbt, int nsplit, int64_t *__restrict__ pairs) {
    extern __shared__ __attribute__((aligned(16))) unsigned char pair_lds[];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int item = blockIdx.x;
    const int tri = item / nsplit, split = item - tri * nsplit;
    int bi = 0, rem = tri;
    while (rem >= nbt - bi) {
        rem -= nbt - bi;
        ++bi;
    }
    const int bj = bi + rem;
    const int I0 = bi * kPairBlock, J0 = bj * kPairBlock;
    const uint64_t per = (nblk + nsplit - 1) / nsplit;
    const uint64_t kb0 = (uint64_t)split * per, kb1 = min(nblk, kb0 + per);
    v16i acc[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[a][b][v] = 0;
    // thread t < 256 expands A row I0+t, t >= 256 expands B col J0+t-256
    const int tt = t & 255, isb = t >> 8;
    const int sub = tt >> 5, r32 = tt & 31;
    const int wr = wave >> 2, wc = wave & 3;
    const int base = isb ? J0 : I0;
    auto expand_to = [&](unsigned char *st, uint64_t w) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int off = isb * 16 * kFragBytes + ((ks * 8 + sub) * 64 + r32 + 32 * h) * 16;
                *reinterpret_cast<v4i *>(st + off) = frag_of(w, ks, h);
            }
    };
    uint64_t nw = 0;
    if (kb0 < kb1) {
        expand_to(pair_lds + (size_t)(kb0 & 1) * kPairStage, xt[kb0 * (uint64_t)npad + base + tt]);
        nw = xt[min(kb0 + 1, kb1 - 1) * (uint64_t)npad + base + tt];
    }
    __syncthreads();
    for (uint64_t kb = kb0; kb < kb1; ++kb) {
        const unsigned char *st = pair_lds + (size_t)(kb & 1) * kPairStage;
        v4i fa[2][4], fb[2][2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int x = 0; x < 4; ++x)
                fa[ks][x] = *reinterpret_cast<const v4i *>(st + ((ks * 8 + wr * 4 + x) * 64 + lane) * 16);
#pragma unroll
            for (int x = 0; x < 2; ++x)
                fb[ks][x] = *reinterpret_cast<const v4i *>(st + 16 * kFragBytes + ((ks * 8 + wc * 2 + x) * 64 + lane) * 16);
        }
        if (MODE == 0) {
            expand_to(pair_lds + (size_t)((kb + 1) & 1) * kPairStage, nw);
            nw = xt[min(kb + 2, kb1 - 1) * (uint64_t)npad + base + tt];
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[ks][a], fb[ks][b], acc[a][b], 0, 0, 0);
        __syncthreads();
    }
    const int rbase = I0 + 128 * wr + 4 * (lane >> 5);
    const int cbase = J0 + 64 * wc + (lane & 31);
    int64_t local = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) local += acc[a][b][v];
    if (rbase < n && cbase < n)
        atomicAdd(reinterpret_cast<unsigned long long *>(pairs + (uint64_t)rbase * n + cbase),
                  (unsigned long long)local);
}

template <int MODE>
float run8(const uint64_t *xt, uint64_t nblk, int n, int npad, int64_t *pairs, int cus, int reps) {
    const int nbt = npad / kPairBlock, ntri = nbt * (nbt + 1) / 2;
    int nsplit = std::max(1, cus / ntri);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 2; ++w)
        hipLaunchKernelGGL(pair_k8<MODE>, dim3(ntri * nsplit), dim3(512), 2 * kPairStage, nullptr, xt, nblk, n, npad,
                           nbt, nsplit, pairs);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(pair_k8<MODE>, dim3(ntri * nsplit), dim3(512), 2 * kPairStage, nullptr, xt, nblk, n, npad,
                           nbt, nsplit, pairs);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

// no LDS, no barrier: every wave loads and expands its own A rows / B columns into registers
__global__ __launch_bounds__(256) void pair_kw(const uint64_t *__restrict__ xt, uint64_t nblk, int n, int npad,
                                              int nbt, int nsplit, int64_t *__restrict__ pairs) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int item = blockIdx.x;
    const int tri = item / nsplit, split = item - tri * nsplit;
    int bi = 0, rem = tri;
    while (rem >= nbt - bi) {
        rem -= nbt - bi;
        ++bi;
    }
    const int bj = bi + rem;
    const int wr = wave >> 1, wc = wave & 1;
    const int I0 = bi * kPairBlock + 128 * wr, J0 = bj * kPairBlock + 128 * wc;
    const uint64_t per = (nblk + nsplit - 1) / nsplit;
    const uint64_t kb0 = (uint64_t)split * per, kb1 = min(nblk, kb0 + per);
    v16i acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[a][b][v] = 0;
    const int r32 = lane & 31, h = lane >> 5;
    uint64_t wa[4], wb[4], na[4], nb[4];
    if (kb0 < kb1) {
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            wa[x] = xt[kb0 * (uint64_t)npad + I0 + 32 * x + r32];
            wb[x] = xt[kb0 * (uint64_t)npad + J0 + 32 * x + r32];
        }
    }
    for (uint64_t kb = kb0; kb < kb1; ++kb) {
        const uint64_t nk = min(kb + 1, kb1 - 1);
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            na[x] = xt[nk * (uint64_t)npad + I0 + 32 * x + r32];
            nb[x] = xt[nk * (uint64_t)npad + J0 + 32 * x + r32];
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            v4i fa[4], fb[4];
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                fa[x] = frag_of(wa[x], ks, h);
                fb[x] = frag_of(wb[x], ks, h);
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a], fb[b], acc[a][b], 0, 0, 0);
        }
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            wa[x] = na[x];
            wb[x] = nb[x];
        }
    }
    int64_t local = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) local += acc[a][b][v];
    const int rbase = I0 + 4 * h, cbase = J0 + r32;
    if (rbase < n && cbase < n)
        atomicAdd(reinterpret_cast<unsigned long long *>(pairs + (uint64_t)rbase * n + cbase),
                  (unsigned long long)local);
}

float runw(const uint64_t *xt, uint64_t nblk, int n, int npad, int64_t *pairs, int cus, int reps) {
    const int nbt = npad / kPairBlock, ntri = nbt * (nbt + 1) / 2;
    int nsplit = std::max(1, cus / ntri);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 2; ++w)
        hipLaunchKernelGGL(pair_kw, dim3(ntri * nsplit), dim3(256), 0, nullptr, xt, nblk, n, npad, nbt, nsplit, pairs);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(pair_kw, dim3(ntri * nsplit), dim3(256), 0, nullptr, xt, nblk, n, npad, nbt, nsplit, pairs);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

// 8 waves, packed words through LDS (4 KB per stage), each wave expands its own fragments
__global__ __launch_bounds__(512) void pair_kp(const uint64_t *__restrict__ xt, uint64_t nblk, int n, int npad,
                                              int nbt, int nsplit, int64_t *__restrict__ pairs) {
    __shared__ uint64_t wl[2][512];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int item = blockIdx.x;
    const int tri = item / nsplit, split = item - tri * nsplit;
    int bi = 0, rem = tri;
    while (rem >= nbt - bi) {
        rem -= nbt - bi;
        ++bi;
    }
    const int bj = bi + rem;
    const int I0 = bi * kPairBlock, J0 = bj * kPairBlock;
    const uint64_t per = (nblk + nsplit - 1) / nsplit;
    const uint64_t kb0 = (uint64_t)split * per, kb1 = min(nblk, kb0 + per);
    v16i acc[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[a][b][v] = 0;
    const int wr = wave >> 2, wc = wave & 3;
    const int r32 = lane & 31, h = lane >> 5;
    const int src = (t < 256) ? I0 + t : J0 + t - 256;
    uint64_t nw = 0;
    if (kb0 < kb1) {
        wl[kb0 & 1][t] = xt[kb0 * (uint64_t)npad + src];
        nw = xt[min(kb0 + 1, kb1 - 1) * (uint64_t)npad + src];
    }
    __syncthreads();
    for (uint64_t kb = kb0; kb < kb1; ++kb) {
        const uint64_t *w = wl[kb & 1];
        uint64_t wa[4], wb[2];
#pragma unroll
        for (int x = 0; x < 4; ++x) wa[x] = w[128 * wr + 32 * x + r32];
#pragma unroll
        for (int x = 0; x < 2; ++x) wb[x] = w[256 + 64 * wc + 32 * x + r32];
        wl[(kb + 1) & 1][t] = nw;
        nw = xt[min(kb + 2, kb1 - 1) * (uint64_t)npad + src];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            v4i fa[4], fb[2];
#pragma unroll
            for (int x = 0; x < 4; ++x) fa[x] = frag_of(wa[x], ks, h);
#pragma unroll
            for (int x = 0; x < 2; ++x) fb[x] = frag_of(wb[x], ks, h);
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a], fb[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }
    int64_t local = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) local += acc[a][b][v];
    const int rbase = I0 + 128 * wr + 4 * h, cbase = J0 + 64 * wc + r32;
    if (rbase < n && cbase < n)
        atomicAdd(reinterpret_cast<unsigned long long *>(pairs + (uint64_t)rbase * n + cbase),
                  (unsigned long long)local);
}

float runp(const uint64_t *xt, uint64_t nblk, int n, int npad, int64_t *pairs, int cus, int reps) {
    const int nbt = npad / kPairBlock, ntri = nbt * (nbt + 1) / 2;
    int nsplit = std::max(1, cus / ntri);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 2; ++w)
        hipLaunchKernelGGL(pair_kp, dim3(ntri * nsplit), dim3(512), 0, nullptr, xt, nblk, n, npad, nbt, nsplit, pairs);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(pair_kp, dim3(ntri * nsplit), dim3(512), 0, nullptr, xt, nblk, n, npad, nbt, nsplit, pairs);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1727;
    const uint64_t S = argc > 2 ? strtoull(argv[2], nullptr, 10) : 1000000;
    const int npad = ((n + 255) / 256) * 256;
    const uint64_t nblk = (S + 63) / 64;
    std::vector<uint64_t> h(nblk * npad);
    uint64_t x = 88172645463325252ull;
    for (auto &v : h) {  // ~6% density
        uint64_t m = 0;
        for (int j = 0; j < 4; ++j) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            m |= x;
        }
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v = m & x & (x >> 3);
    }
    uint64_t *d;
    int64_t *p;
    CK(hipMalloc(&d, h.size() * 8));
    CK(hipMalloc(&p, (size_t)n * n * 8));
    CK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const double ops = (double)S * n * (n + 1);
    const float t0 = run<0>(d, nblk, n, npad, p, cus, 5);
    const float t1 = run<1>(d, nblk, n, npad, p, cus, 5);
    const float t2 = run<2>(d, nblk, n, npad, p, cus, 5);
    const float t3 = run<3>(d, nblk, n, npad, p, cus, 5);
    const float t4 = run<4>(d, nblk, n, npad, p, cus, 5);
    const float u0 = run8<0>(d, nblk, n, npad, p, cus, 5);
    const float u1 = run8<1>(d, nblk, n, npad, p, cus, 5);
    const float w0 = runw(d, nblk, n, npad, p, cus, 5);
    const float p0 = runp(d, nblk, n, npad, p, cus, 5);
    printf("8-wave packed-LDS: %.3f ms (%.0f TOPs)\n", p0, ops / p0 / 1e9);
    printf("per-wave regs: %.3f ms (%.0f TOPs)\n", w0, ops / w0 / 1e9);
    printf("8-wave: full %.3f ms (%.0f TOPs)  no-expand %.3f\n", u0, ops / u0 / 1e9, u1);
    printf("n=%d S=%llu  full %.3f ms (%.0f TOPs)  no-expand %.3f  no-barrier %.3f  fixed-stage %.3f  mfma-only %.3f\n",
           n, (unsigned long long)S, t0, ops / t0 / 1e9, t1, t2, t3, t4);
    return 0;
}
