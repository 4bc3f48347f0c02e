// csa_legacy.hip -- MI355X (gfx950) kernels + C ABI for the LEGACY Monte Carlo path.
//
// Replaces the reference's hot loop (analysis.py:162-191 -> analysis.py:141-159 ->
// legacy.py:178-200) with four kernels:
//   draw_kernel          one panel per 64-lane wavefront; the feature bitmasks live in
//                        LDS, every per-panel counter lives in registers (lane f = feature
//                        f, lane w = bitset word w); Philox4x32-10 keyed by
//                        (seed, panel, attempt, step).               legacy.py:47-200
//   xt_count_kernel      64x64 bit-matrix transpose of the packed panels + per-person
//                        popcounts (Counter.update, analysis.py:179,187).  HBM-bound.
//   pair_mfma_kernel     X^T X on v_mfma_i32_32x32x32_i8, panels as the K dimension,
//                        upper-triangular 128x128 tiles, split-K, int64 atomics
//                        (PairHistogram.add_portfolio_of_panels_to_histogram, analysis.py:90-95).
//   unique_kernel        open-addressing table of panel indices keyed by a 128-bit panel
//                        hash, exact full-bitmask compare (found_panels, analysis.py:171,186).
// The C ABI is declared in include/csa_legacy.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/csa_legacy.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(CSA_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));          \
    } while (0)

constexpr int kWave = 64;
constexpr int kDrawThreads = 256;
constexpr uint32_t kDefaultMaxAttempts = 100000;

// ------------------------------------------------------------------------------------------
// Philox4x32-10 (Random123 constants).  Stream contract: oracle/philox.py.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3,
                                              uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// position (0..63) of the rr-th (1-based) set bit of m; requires 1 <= rr <= popcount(m)
__device__ __forceinline__ int select_bit(uint64_t m, int rr) {
    int pos = 0;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const int c = __popcll(m & ((1ull << s) - 1));
        if (rr > c) {
            rr -= c;
            m >>= s;
            pos += s;
        }
    }
    return pos;
}

__device__ __forceinline__ uint64_t fmix_a(uint64_t z) {  // splitmix64 finaliser
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t fmix_b(uint64_t z) {  // murmur3 fmix64
    z ^= z >> 33;
    z *= 0xFF51AFD7ED558CCDull;
    z ^= z >> 33;
    z *= 0xC4CEB9FE1A85EC53ull;
    return z ^ (z >> 33);
}

// ------------------------------------------------------------------------------------------
// Draw kernel
// ------------------------------------------------------------------------------------------
struct DrawArgs {
    const uint64_t *featmask;  // F x Ws, Ws = W | 1 (odd stride: conflict-free lane-f reads)
    const int32_t *fmin, *fmax, *sel0, *rem0;
    const uint64_t *present0;  // W
    int32_t n, F, W, Ws, k;
    uint32_t max_attempts, attempt_base;
    int32_t single;            // 1: exactly one attempt, no min-quota check, write final state
    uint64_t seed, panel_begin, n_panels;
    uint64_t *panels;          // n_panels x W
    uint64_t *hashes;          // 2 x n_panels or null
    uint32_t *attempts;        // n_panels or null
    int32_t *picks;            // n_panels x k or null
    uint32_t *status;          // 4 words
    int32_t *sel_out, *rem_out;
    uint64_t *present_out;
};

enum : int { kAccept = 0, kFail = 1, kReject = 2, kNoCandidate = 3 };

__device__ __forceinline__ void raise_status(uint32_t *status, uint32_t code, uint64_t panel) {
    if (atomicCAS(&status[0], 0u, code) == 0u) {
        status[1] = (uint32_t)panel;
        status[2] = (uint32_t)(panel >> 32);
    }
}

// One attempt of find_random_sample_legacy (legacy.py:178-200) + check_min_cats
// (legacy.py:160-168) for one wavefront.  All branch conditions are wave-uniform.
template <int WPL>
__device__ int draw_attempt(const DrawArgs &A, const uint64_t *__restrict__ fm, uint64_t idx,
                            uint64_t panel, uint32_t attempt, int lane, bool fvalid, int fmin,
                            int fmax, int &sel, int &rem, uint64_t (&rmn)[WPL], uint64_t (&pk)[WPL]) {
    const int W = A.W, Ws = A.Ws, k = A.k;
    const uint32_t key0 = (uint32_t)A.seed, key1 = (uint32_t)(A.seed >> 32);
    const uint32_t pan0 = (uint32_t)panel, pan1 = (uint32_t)(panel >> 32);
    sel = fvalid ? A.sel0[lane] : 0;
    rem = fvalid ? A.rem0[lane] : 0;
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
        const int w = lane * WPL + j;
        rmn[j] = w < W ? A.present0[w] : 0ull;
        pk[j] = 0ull;
    }
    // Philox blocks for this attempt: lane j holds block (base + j) = steps 4(base+j) .. +3
    uint32_t blk_base = 0;
    uint32_t x0 = (uint32_t)lane, x1 = attempt, x2 = pan0, x3 = pan1;
    philox4x32_10(x0, x1, x2, x3, key0, key1);
    int32_t *picks = A.picks ? A.picks + idx * (uint64_t)k : nullptr;

    for (int step = 0; step < k; ++step) {
        const uint32_t blk = (uint32_t)step >> 2;
        if (blk >= blk_base + kWave) {  // k > 256: next 64 blocks
            blk_base += kWave;
            x0 = blk_base + lane;
            x1 = attempt;
            x2 = pan0;
            x3 = pan1;
            philox4x32_10(x0, x1, x2, x3, key0, key1);
        }
        // --- find_max_ratio_cat (legacy.py:124-157) --------------------------------
        const int need = fmin - sel;
        if (__ballot(fvalid && sel < fmin && rem < need)) return kFail;  // legacy.py:132-137
        const bool cand = fvalid && rem != 0 && fmax != 0 && need > -100 * rem;  // 140-141,125
        int bn = need, bd = rem, bi = cand ? lane : kWave;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {  // argmax, strict '>' => lowest index wins ties
            const int on = __shfl_xor(bn, m), od = __shfl_xor(bd, m), oi = __shfl_xor(bi, m);
            const int l = on * bd, r = bn * od;
            const bool take = oi < kWave && (bi == kWave || l > r || (l == r && oi < bi));
            if (take) {
                bn = on;
                bd = od;
                bi = oi;
            }
        }
        const int fs = __builtin_amdgcn_readfirstlane(bi);
        bool any_present = false;
#pragma unroll
        for (int j = 0; j < WPL; ++j) any_present |= rmn[j] != 0ull;
        const bool nonempty = __ballot(any_present) != 0ull;
        int p = -1;
        if (fs == kWave) {
            if (nonempty) return kNoCandidate;  // KeyError at legacy.py:188
        } else {
            // --- randint(1, remaining) (legacy.py:149), Philox verification mode ----------
            const uint32_t sw = (uint32_t)step & 3u;
            const uint32_t xv = sw == 0 ? x0 : (sw == 1 ? x1 : (sw == 2 ? x2 : x3));
            const uint32_t u = __builtin_amdgcn_readlane(xv, (int)(blk - blk_base));
            const uint32_t remf = (uint32_t)__builtin_amdgcn_readlane(rem, fs);
            const int r = 1 + (int)(((uint64_t)u * remf) >> 32);
            // --- r-th remaining holder of f* in agent order (legacy.py:186-197) ------------
            uint64_t m[WPL];
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < WPL; ++j) {
                const int w = lane * WPL + j;
                m[j] = w < W ? (rmn[j] & fm[fs * Ws + w]) : 0ull;
                cnt += __popcll(m[j]);
            }
            int incl = cnt;
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const int t = __shfl_up(incl, d);
                if (lane >= d) incl += t;
            }
            const uint64_t hit = __ballot(incl >= r);
            if (hit) {
                const int L = __ffsll((unsigned long long)hit) - 1;
                int pl = 0;
                if (lane == L) {
                    int rr = r - (incl - cnt);
#pragma unroll
                    for (int j = 0; j < WPL; ++j) {
                        const int c = __popcll(m[j]);
                        if (rr >= 1 && rr <= c) pl = (lane * WPL + j) * 64 + select_bit(m[j], rr);
                        rr -= c;
                    }
                }
                p = __builtin_amdgcn_readlane(pl, L);
                // --- delete_person / really_delete_person (legacy.py:103-120, 67-75) -------
                const int wi = p >> 6, bp = p & 63;
                const uint64_t fw = fvalid ? fm[lane * Ws + wi] : 0ull;
                const int has = (int)((fw >> bp) & 1ull);
                sel += has;
                rem -= has;
                if (lane == wi / WPL) {
#pragma unroll
                    for (int j = 0; j < WPL; ++j)
                        if (j == wi % WPL) {
                            rmn[j] &= ~(1ull << bp);
                            pk[j] |= 1ull << bp;
                        }
                }
                // --- delete_all_in_cat for every full feature of the pick (legacy.py:47-62,
                //     115-119), bulk form: D = remaining & OR(featmask[full]) --------------
                uint64_t full = __ballot(has && sel == fmax);
                if (full) {
                    uint64_t D[WPL];
#pragma unroll
                    for (int j = 0; j < WPL; ++j) D[j] = 0ull;
                    while (full) {
                        const int f = __ffsll((unsigned long long)full) - 1;
                        full &= full - 1;
#pragma unroll
                        for (int j = 0; j < WPL; ++j) {
                            const int w = lane * WPL + j;
                            if (w < W) D[j] |= fm[f * Ws + w];
                        }
                    }
                    int dec = 0;
#pragma unroll
                    for (int j = 0; j < WPL; ++j) {
                        D[j] &= rmn[j];
                        rmn[j] &= ~D[j];
                        uint64_t nz = __ballot(D[j] != 0ull);
                        while (nz) {
                            const int l = __ffsll((unsigned long long)nz) - 1;
                            nz &= nz - 1;
                            const int w = l * WPL + j;
                            const uint64_t dw = readlane64(D[j], l);
                            if (fvalid) dec += __popcll(dw & fm[lane * Ws + w]);
                        }
                    }
                    rem -= dec;
                }
                // remaining == 0 and selected < min raised inside the deletes (legacy.py:55,73)
                if (__ballot(fvalid && rem == 0 && sel < fmin)) {
                    if (picks && lane == 0) picks[step] = p;
                    return kFail;
                }
            }
        }
        if (picks && lane == 0) picks[step] = p;
        if (step < k - 1) {  // legacy.py:198-199
            bool any = false;
#pragma unroll
            for (int j = 0; j < WPL; ++j) any |= rmn[j] != 0ull;
            if (!__ballot(any)) return kFail;
        }
    }
    if (__ballot(fvalid && sel < fmin)) return kReject;  // check_min_cats, analysis.py:155-159
    return kAccept;
}

template <int WPL>
__global__ __launch_bounds__(kDrawThreads) void draw_kernel(DrawArgs A) {
    extern __shared__ uint64_t lds_fm[];
    const int nfm = A.F * A.Ws;
    for (int i = threadIdx.x; i < nfm; i += blockDim.x) lds_fm[i] = A.featmask[i];
    __syncthreads();

    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / kWave);
    const bool fvalid = lane < A.F;
    const int fmin = fvalid ? A.fmin[lane] : 0;
    const int fmax = fvalid ? A.fmax[lane] : 0;
    const uint32_t max_att = A.single ? 1u : A.max_attempts;

    for (uint64_t i = wave; i < A.n_panels; i += nwaves) {
        if (__hip_atomic_load(&A.status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
        const uint64_t panel = A.panel_begin + i;
        int sel = 0, rem = 0;
        uint64_t rmn[WPL], pk[WPL];
        int rc = kFail;
        uint32_t a = 0;
        for (; a < max_att; ++a) {
            rc = draw_attempt<WPL>(A, lds_fm, i, panel, A.attempt_base + a, lane, fvalid, fmin, fmax,
                                   sel, rem, rmn, pk);
            if (rc == kAccept || rc == kNoCandidate || (A.single && rc == kReject)) break;
        }
        if (A.single) {  // find_random_sample_legacy: report one attempt + its final state
            if (lane == 0) A.status[3] = (uint32_t)rc;
            if (rc == kNoCandidate && lane == 0) raise_status(A.status, CSA_E_NO_CANDIDATE, panel);
            if (A.sel_out && fvalid) {
                A.sel_out[lane] = sel;
                A.rem_out[lane] = rem;
            }
#pragma unroll
            for (int j = 0; j < WPL; ++j) {
                const int w = lane * WPL + j;
                if (w < A.W) {
                    if (A.present_out) A.present_out[w] = rmn[j];
                    A.panels[i * A.W + w] = pk[j];
                }
            }
            continue;
        }
        if (rc != kAccept) {
            if (lane == 0)
                raise_status(A.status, rc == kNoCandidate ? CSA_E_NO_CANDIDATE : CSA_E_ATTEMPT_LIMIT, panel);
            return;
        }
        uint64_t h1 = 0, h2 = 0;
#pragma unroll
        for (int j = 0; j < WPL; ++j) {
            const uint64_t w = (uint64_t)(lane * WPL + j);
            if (w < (uint64_t)A.W) {
                A.panels[i * A.W + w] = pk[j];
                h1 += fmix_a(pk[j] ^ (w * 0x9E3779B97F4A7C15ull));
                h2 += fmix_b(pk[j] + (w + 1) * 0xD6E8FEB86659FD93ull);
            }
        }
        if (A.hashes) {
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) {
                h1 += (uint64_t)__shfl_xor((long long)h1, m);
                h2 += (uint64_t)__shfl_xor((long long)h2, m);
            }
            if (lane == 0) {
                A.hashes[2 * i] = h1;
                A.hashes[2 * i + 1] = h2;
            }
        }
        if (A.attempts && lane == 0) A.attempts[i] = a + 1;
    }
}

// ------------------------------------------------------------------------------------------
// Bit transpose + per-person counts
// ------------------------------------------------------------------------------------------
constexpr int kXtThreads = 256;
constexpr int kXtBlocksPerGroup = 16;  // 1024 panels per workgroup

// 64x64 bit-matrix transpose across a wavefront: lane i holds row i (bit j = column j);
// afterwards lane j holds column j (bit i = row i).
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t x, int lane) {
    const uint64_t masks[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                               0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
    for (int t = 0; t < 6; ++t) {
        const int s = 32 >> t;
        const uint64_t M = masks[t];
        const uint64_t y = (uint64_t)__shfl_xor((long long)x, s);
        if (lane & s)
            x = (x & ~M) | ((y & ~M) >> s);
        else
            x = (x & M) | ((y & M) << s);
    }
    return x;
}

__global__ __launch_bounds__(kXtThreads) void xt_count_kernel(const uint64_t *__restrict__ panels,
                                                              uint64_t S, int n, int W, int npad,
                                                              uint64_t *__restrict__ xt,
                                                              int64_t *__restrict__ counts) {
    extern __shared__ uint64_t smem[];
    const int Wp = W | 1;
    uint64_t *tile = smem;                                   // 64 x Wp
    uint32_t *cnt = reinterpret_cast<uint32_t *>(smem + 64 * Wp);  // n
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    for (int p = threadIdx.x; p < n; p += blockDim.x) cnt[p] = 0;
    const uint64_t nblk = (S + 63) / 64;
    const uint64_t b0 = (uint64_t)blockIdx.x * kXtBlocksPerGroup;
    const uint64_t b1 = min(nblk, b0 + kXtBlocksPerGroup);
    const int ncol = npad / 64;
    for (uint64_t b = b0; b < b1; ++b) {
        __syncthreads();
        const uint64_t row0 = b * 64;
        const int rows = (int)min<uint64_t>(64, S - row0);
        const uint64_t *src = panels + row0 * (uint64_t)W;
        for (int t = threadIdx.x; t < 64 * W; t += blockDim.x) {
            const int r = t / W, c = t - r * W;
            tile[r * Wp + c] = r < rows ? src[t] : 0ull;
        }
        __syncthreads();
        for (int w = wv; w < ncol; w += nwv) {
            uint64_t x = w < W ? tile[lane * Wp + w] : 0ull;
            x = wave_transpose64(x, lane);
            const int p = 64 * w + lane;
            if (xt) xt[b * (uint64_t)npad + p] = x;
            if (p < n) cnt[p] += (uint32_t)__popcll(x);
        }
    }
    __syncthreads();
    for (int p = threadIdx.x; p < n; p += blockDim.x)
        if (cnt[p]) atomicAdd(reinterpret_cast<unsigned long long *>(counts + p), (unsigned long long)cnt[p]);
}

// ------------------------------------------------------------------------------------------
// Pair counts: X^T X on int8 MFMA
// ------------------------------------------------------------------------------------------
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kPairTile = 128;  // per wavefront: 4 x 4 MFMA tiles of 32 x 32
constexpr int kPairThreads = 256;

// 16 bits -> 16 bytes of 0/1 (byte q*4+e = bit 4q+e)
__device__ __forceinline__ v4i expand16(uint32_t bits) {
    v4i r;
    r[0] = (int)(((bits & 0xFu) * 0x00204081u) & 0x01010101u);
    r[1] = (int)((((bits >> 4) & 0xFu) * 0x00204081u) & 0x01010101u);
    r[2] = (int)((((bits >> 8) & 0xFu) * 0x00204081u) & 0x01010101u);
    r[3] = (int)((((bits >> 12) & 0xFu) * 0x00204081u) & 0x01010101u);
    return r;
}

__global__ __launch_bounds__(kPairThreads) void pair_mfma_kernel(const uint64_t *__restrict__ xt,
                                                                 uint64_t nblk, int n, int npad,
                                                                 int ntile, int nsplit,
                                                                 int64_t *__restrict__ pairs) {
    const int lane = threadIdx.x & 63;
    const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6));
    const int ntri = ntile * (ntile + 1) / 2;
    if (item >= ntri * nsplit) return;
    const int tri = item / nsplit, split = item - tri * nsplit;
    // tri -> (ti, tj) with ti <= tj, row-major over the upper triangle
    int ti = 0, rem = tri;
    while (rem >= ntile - ti) {
        rem -= ntile - ti;
        ++ti;
    }
    const int tj = ti + rem;
    const int I0 = ti * kPairTile, J0 = tj * kPairTile;
    const uint64_t per = (nblk + nsplit - 1) / nsplit;
    const uint64_t kb0 = (uint64_t)split * per, kb1 = min(nblk, kb0 + per);

    v16i acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[a][b][v] = 0;

    const int r32 = lane & 31;
    const int hsh = 16 * (lane >> 5);
    uint64_t wa[4], wb[4], na[4], nb[4];
    if (kb0 < kb1) {
        const uint64_t *row = xt + kb0 * (uint64_t)npad;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            wa[t] = row[I0 + 32 * t + r32];
            wb[t] = row[J0 + 32 * t + r32];
        }
    }
    for (uint64_t kb = kb0; kb < kb1; ++kb) {
        if (kb + 1 < kb1) {  // prefetch the next panel block
            const uint64_t *row = xt + (kb + 1) * (uint64_t)npad;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                na[t] = row[I0 + 32 * t + r32];
                nb[t] = row[J0 + 32 * t + r32];
            }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int sh = 32 * ks + hsh;
            v4i fa[4], fb[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                fa[t] = expand16((uint32_t)(wa[t] >> sh) & 0xFFFFu);
                fb[t] = expand16((uint32_t)(wb[t] >> sh) & 0xFFFFu);
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a], fb[b], acc[a][b], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            wa[t] = na[t];
            wb[t] = nb[t];
        }
    }
    // C/D layout (gfx950, dtype-independent): col = lane & 31, row = (v&3) + 8*(v>>2) + 4*(lane>>5)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int row = I0 + 32 * a + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
                const int col = J0 + 32 * b + r32;
                const int val = acc[a][b][v];
                if (val != 0 && row < n && col < n)
                    atomicAdd(reinterpret_cast<unsigned long long *>(pairs + (uint64_t)row * n + col),
                              (unsigned long long)(long long)val);
            }
}

// ------------------------------------------------------------------------------------------
// Distinct panels
// ------------------------------------------------------------------------------------------
// owner filter: only hashes with h1 % world == rank are inserted (multi-GPU partition)
__global__ void unique_kernel(const uint64_t *__restrict__ hashes, const uint64_t *__restrict__ panels,
                              uint64_t S, int W, unsigned long long *__restrict__ table,
                              uint64_t mask, unsigned long long *__restrict__ unique, uint32_t world,
                              uint32_t rank) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool inserted = false;
    if (i < S && (world <= 1 || hashes[2 * i] % world == rank)) {
        const uint64_t h1 = hashes[2 * i], h2 = hashes[2 * i + 1];
        uint64_t slot = (h1 ^ (h2 >> 29)) & mask;
        for (uint64_t probe = 0; probe <= mask; ++probe) {
            const unsigned long long v = atomicCAS(table + slot, 0ull, (unsigned long long)(i + 1));
            if (v == 0ull) {
                inserted = true;
                break;
            }
            const uint64_t j = v - 1;
            if (hashes[2 * j] == h1 && hashes[2 * j + 1] == h2) {
                bool same = true;
                if (panels)
                    for (int w = 0; w < W && same; ++w) same = panels[i * W + w] == panels[j * W + w];
                if (same) break;
            }
            slot = (slot + 1) & mask;
        }
    }
    const uint64_t b = __ballot(inserted);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(unique, (unsigned long long)__popcll(b));
}

}  // namespace

// ==========================================================================================
// Host side
// ==========================================================================================
struct csa_instance {
    int32_t n = 0, C = 0, F = 0, W = 0, Ws = 0;
    int device = 0;
    std::vector<int32_t> pf, fmin, fmax, fcat, pool;
    std::vector<uint64_t> featmask;  // F x Ws
    uint64_t *d_featmask = nullptr;
    int32_t *d_fmin = nullptr, *d_fmax = nullptr, *d_sel0 = nullptr, *d_rem0 = nullptr;
    uint64_t *d_present0 = nullptr;
    int32_t max_abs = 0;  // max |fmin| / |sel0| bound for the cross-multiplication range check
};

namespace {

template <typename T>
int dalloc(T **p, size_t count) {
    HIPCHK(hipMalloc(reinterpret_cast<void **>(p), std::max<size_t>(count, 1) * sizeof(T)));
    return CSA_OK;
}

int wpl_for(int W) { return W <= 64 ? 1 : (W <= 128 ? 2 : (W <= 256 ? 4 : 0)); }

struct ScopedDevice {
    int prev = -1;
    explicit ScopedDevice(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~ScopedDevice() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int check_k(const csa_instance *I, int32_t k) {
    if (k < 0) return fail(CSA_E_INVALID, "k must be >= 0 (got %d)", k);
    // need*den must stay inside int32 (need = fmin - sel, |need| <= max_abs + k, den <= n)
    const int64_t bound = (int64_t)(I->max_abs + k + 1) * (I->n + 1) * 100;
    if (bound >= (int64_t)1 << 31)
        return fail(CSA_E_UNSUPPORTED, "k=%d with n=%d exceeds the int32 ratio range", k, I->n);
    return CSA_OK;
}

int launch_draw(const csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                uint32_t max_attempts, uint32_t attempt_base, int single, uint64_t *d_panels,
                uint64_t *d_hashes, uint32_t *d_attempts, int32_t *d_picks, uint32_t *d_status,
                int32_t *d_sel_out, int32_t *d_rem_out, uint64_t *d_present_out, hipStream_t stream) {
    int rc = check_k(I, k);
    if (rc) return rc;
    if (!d_panels || !d_status) return fail(CSA_E_INVALID, "d_panels and d_status are required");
    if (n_panels == 0) return CSA_OK;
    const int wpl = wpl_for(I->W);
    if (I->F > kWave || wpl == 0)
        return fail(CSA_E_UNSUPPORTED, "draw kernel supports F <= 64 and n <= 16384 (F=%d n=%d)", I->F, I->n);
    DrawArgs A;
    A.featmask = I->d_featmask;
    A.fmin = I->d_fmin;
    A.fmax = I->d_fmax;
    A.sel0 = I->d_sel0;
    A.rem0 = I->d_rem0;
    A.present0 = I->d_present0;
    A.n = I->n;
    A.F = I->F;
    A.W = I->W;
    A.Ws = I->Ws;
    A.k = k;
    A.max_attempts = max_attempts ? max_attempts : kDefaultMaxAttempts;
    A.attempt_base = attempt_base;
    A.single = single;
    A.seed = seed;
    A.panel_begin = panel_begin;
    A.n_panels = n_panels;
    A.panels = d_panels;
    A.hashes = d_hashes;
    A.attempts = d_attempts;
    A.picks = d_picks;
    A.status = d_status;
    A.sel_out = d_sel_out;
    A.rem_out = d_rem_out;
    A.present_out = d_present_out;
    const size_t lds = (size_t)I->F * I->Ws * sizeof(uint64_t);
    if (lds > 160 * 1024) return fail(CSA_E_UNSUPPORTED, "feature bitmasks need %zu B of LDS", lds);
    const void *fn = wpl == 1 ? (const void *)draw_kernel<1>
                              : (wpl == 2 ? (const void *)draw_kernel<2> : (const void *)draw_kernel<4>);
    int per_cu = 0, cus = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kDrawThreads, lds));
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, I->device));
    const uint64_t waves_per_block = kDrawThreads / kWave;
    const uint64_t want = (n_panels + waves_per_block - 1) / waves_per_block;
    const uint64_t cap = (uint64_t)std::max(per_cu, 1) * (uint64_t)std::max(cus, 1);
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min(want, cap));
    if (wpl == 1)
        hipLaunchKernelGGL(draw_kernel<1>, dim3(grid), dim3(kDrawThreads), lds, stream, A);
    else if (wpl == 2)
        hipLaunchKernelGGL(draw_kernel<2>, dim3(grid), dim3(kDrawThreads), lds, stream, A);
    else
        hipLaunchKernelGGL(draw_kernel<4>, dim3(grid), dim3(kDrawThreads), lds, stream, A);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int read_status(const uint32_t *d_status, hipStream_t stream, uint32_t *h) {
    HIPCHK(hipMemcpyAsync(h, d_status, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    return CSA_OK;
}

uint64_t pow2_at_least(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

template <typename T>
struct DevBuf {
    T *p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

extern "C" {

int csa_version(void) { return 1; }

const char *csa_last_error(void) { return g_err.c_str(); }

int csa_device_count(int32_t *out) {
    if (!out) return fail(CSA_E_INVALID, "null out");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *out = 0;
        return fail(CSA_E_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *out = c;
    return CSA_OK;
}

int csa_instance_create(int32_t n, int32_t C, int32_t F, const int32_t *person_feat, const int32_t *fmin,
                        const int32_t *fmax, const int32_t *feat_cat, csa_instance **out) {
    if (!out) return fail(CSA_E_INVALID, "null out");
    *out = nullptr;
    if (n < 0 || C <= 0 || F <= 0 || (n > 0 && !person_feat) || !fmin || !fmax || !feat_cat)
        return fail(CSA_E_INVALID, "invalid instance arguments (n=%d C=%d F=%d)", n, C, F);
    csa_instance *I = new csa_instance();
    I->n = n;
    I->C = C;
    I->F = F;
    I->W = (n + 63) / 64;
    I->Ws = I->W | 1;
    I->pf.assign(person_feat, person_feat + (size_t)n * C);
    I->fmin.assign(fmin, fmin + F);
    I->fmax.assign(fmax, fmax + F);
    I->fcat.assign(feat_cat, feat_cat + F);
    I->pool.assign(F, 0);
    I->featmask.assign((size_t)F * I->Ws, 0ull);
    for (int f = 1; f < F; ++f)
        if (feat_cat[f] < feat_cat[f - 1]) {
            delete I;
            return fail(CSA_E_INVALID, "features must be category-major (feat_cat non-decreasing)");
        }
    for (int f = 0; f < F; ++f) {
        I->max_abs = std::max(I->max_abs, std::abs(fmin[f]));
        if (feat_cat[f] < 0 || feat_cat[f] >= C) {
            delete I;
            return fail(CSA_E_INVALID, "feature %d has category %d outside [0,%d)", f, feat_cat[f], C);
        }
    }
    for (int p = 0; p < n; ++p)
        for (int c = 0; c < C; ++c) {
            const int g = person_feat[(size_t)p * C + c];
            if (g < 0 || g >= F || feat_cat[g] != c) {
                delete I;
                return fail(CSA_E_INVALID, "agent %d category %d has feature %d of another category", p, c, g);
            }
            I->featmask[(size_t)g * I->Ws + (p >> 6)] |= 1ull << (p & 63);
            I->pool[g] += 1;
        }
    if (hipGetDevice(&I->device) != hipSuccess) {
        delete I;
        return fail(CSA_E_HIP, "no HIP device available");
    }
    std::vector<int32_t> zeros(F, 0);
    std::vector<uint64_t> present(I->W, 0ull);
    for (int p = 0; p < n; ++p) present[p >> 6] |= 1ull << (p & 63);
    int rc = CSA_OK;
    if ((rc = dalloc(&I->d_featmask, I->featmask.size())) || (rc = dalloc(&I->d_fmin, F)) ||
        (rc = dalloc(&I->d_fmax, F)) || (rc = dalloc(&I->d_sel0, F)) || (rc = dalloc(&I->d_rem0, F)) ||
        (rc = dalloc(&I->d_present0, I->W))) {
        csa_instance_destroy(I);
        return rc;
    }
    hipError_t e = hipSuccess;
    e = e ? e : hipMemcpy(I->d_featmask, I->featmask.data(), I->featmask.size() * 8, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(I->d_fmin, fmin, F * 4, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(I->d_fmax, fmax, F * 4, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(I->d_sel0, zeros.data(), F * 4, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(I->d_rem0, I->pool.data(), F * 4, hipMemcpyHostToDevice);
    if (I->W) e = e ? e : hipMemcpy(I->d_present0, present.data(), I->W * 8, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        csa_instance_destroy(I);
        return fail(CSA_E_HIP, "instance upload: %s", hipGetErrorString(e));
    }
    *out = I;
    return CSA_OK;
}

void csa_instance_destroy(csa_instance *I) {
    if (!I) return;
    ScopedDevice sd(I->device);
    if (I->d_featmask) (void)hipFree(I->d_featmask);
    if (I->d_fmin) (void)hipFree(I->d_fmin);
    if (I->d_fmax) (void)hipFree(I->d_fmax);
    if (I->d_sel0) (void)hipFree(I->d_sel0);
    if (I->d_rem0) (void)hipFree(I->d_rem0);
    if (I->d_present0) (void)hipFree(I->d_present0);
    delete I;
}

int csa_instance_info(const csa_instance *I, int32_t *n, int32_t *C, int32_t *F, int32_t *W) {
    if (!I) return fail(CSA_E_INVALID, "null instance");
    if (n) *n = I->n;
    if (C) *C = I->C;
    if (F) *F = I->F;
    if (W) *W = I->W;
    return CSA_OK;
}

int csa_instance_set_state(csa_instance *I, const int32_t *sel, const int32_t *rem, const uint64_t *present) {
    if (!I) return fail(CSA_E_INVALID, "null instance");
    ScopedDevice sd(I->device);
    std::vector<int32_t> zeros(I->F, 0);
    std::vector<uint64_t> all(I->W, 0ull);
    for (int p = 0; p < I->n; ++p) all[p >> 6] |= 1ull << (p & 63);
    int32_t mx = 0;
    for (int f = 0; f < I->F; ++f) mx = std::max(mx, std::abs(I->fmin[f]));
    if (sel)
        for (int f = 0; f < I->F; ++f) mx = std::max(mx, std::abs(sel[f]));
    I->max_abs = mx;
    if (present)
        for (int w = 0; w < I->W; ++w)
            if (present[w] & ~all[w]) return fail(CSA_E_INVALID, "present mask has bits beyond n");
    HIPCHK(hipMemcpy(I->d_sel0, sel ? sel : zeros.data(), I->F * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(I->d_rem0, rem ? rem : I->pool.data(), I->F * 4, hipMemcpyHostToDevice));
    if (I->W) HIPCHK(hipMemcpy(I->d_present0, present ? present : all.data(), I->W * 8, hipMemcpyHostToDevice));
    return CSA_OK;
}

int csa_status_decode(const uint32_t *h) {
    if (!h) return fail(CSA_E_INVALID, "null status");
    const uint64_t panel = (uint64_t)h[1] | ((uint64_t)h[2] << 32);
    switch (h[0]) {
        case 0:
            return CSA_OK;
        case CSA_E_NO_CANDIDATE:
            return fail(CSA_E_NO_CANDIDATE,
                        "panel %llu: no feature is a candidate while agents remain (reference: KeyError at legacy.py:188)",
                        (unsigned long long)panel);
        case CSA_E_ATTEMPT_LIMIT:
            return fail(CSA_E_ATTEMPT_LIMIT, "panel %llu: attempt limit reached without an accepted panel",
                        (unsigned long long)panel);
        default:
            return fail((int)h[0], "device status %u at panel %llu", h[0], (unsigned long long)panel);
    }
}

int csa_draw_async(const csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                   uint32_t max_attempts, uint64_t *d_panels, uint64_t *d_hashes, uint32_t *d_attempts,
                   int32_t *d_picks, uint32_t *d_status, void *stream) {
    if (!I) return fail(CSA_E_INVALID, "null instance");
    return launch_draw(I, k, seed, panel_begin, n_panels, max_attempts, 0, 0, d_panels, d_hashes, d_attempts,
                       d_picks, d_status, nullptr, nullptr, nullptr, (hipStream_t)stream);
}

int32_t csa_xt_pad(int32_t n) { return ((n + kPairTile - 1) / kPairTile) * kPairTile; }

int csa_transpose_count_async(const uint64_t *d_panels, uint64_t n_panels, int32_t n, uint64_t *d_xt,
                              int64_t *d_counts, void *stream) {
    if (n <= 0 || !d_panels || !d_counts) return fail(CSA_E_INVALID, "transpose: bad arguments");
    if (n_panels == 0) return CSA_OK;
    const int W = (n + 63) / 64, Wp = W | 1;
    const size_t lds = (size_t)64 * Wp * 8 + (size_t)n * 4;
    if (lds > 160 * 1024) return fail(CSA_E_UNSUPPORTED, "transpose needs %zu B of LDS", lds);
    const uint64_t nblk = (n_panels + 63) / 64;
    const unsigned grid = (unsigned)((nblk + kXtBlocksPerGroup - 1) / kXtBlocksPerGroup);
    hipLaunchKernelGGL(xt_count_kernel, dim3(grid), dim3(kXtThreads), lds, (hipStream_t)stream, d_panels,
                       n_panels, n, W, csa_xt_pad(n), d_xt, d_counts);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_pair_counts_async(const uint64_t *d_xt, uint64_t n_blocks, int32_t n, int64_t *d_pairs, void *stream) {
    if (n <= 0 || !d_xt || !d_pairs) return fail(CSA_E_INVALID, "pairs: bad arguments");
    if (n_blocks == 0) return CSA_OK;
    if (n_blocks * 64 >= (1ull << 31)) return fail(CSA_E_UNSUPPORTED, "pairs: > 2^31 panels per call");
    const int npad = csa_xt_pad(n), ntile = npad / kPairTile;
    const int ntri = ntile * (ntile + 1) / 2;
    // enough (tile, split) work items to fill 256 CUs x 4 SIMDs twice, >= 8 panel blocks each
    int nsplit = std::max(1, (2048 + ntri - 1) / ntri);
    nsplit = (int)std::min<uint64_t>((uint64_t)nsplit, std::max<uint64_t>(1, n_blocks / 8));
    const int waves = ntri * nsplit, wpb = kPairThreads / 64;
    hipLaunchKernelGGL(pair_mfma_kernel, dim3((waves + wpb - 1) / wpb), dim3(kPairThreads), 0,
                       (hipStream_t)stream, d_xt, n_blocks, n, npad, ntile, nsplit, d_pairs);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_unique_async(const uint64_t *d_hashes, const uint64_t *d_panels, uint64_t n_panels, int32_t W,
                     uint64_t *d_table, uint64_t table_slots, uint64_t *d_unique, void *stream) {
    if (!d_hashes || !d_table || !d_unique || W <= 0) return fail(CSA_E_INVALID, "unique: bad arguments");
    if (table_slots < 2 * n_panels || (table_slots & (table_slots - 1)))
        return fail(CSA_E_INVALID, "unique: table_slots must be a power of two >= 2*n_panels");
    if (n_panels == 0) return CSA_OK;
    HIPCHK(hipMemsetAsync(d_table, 0, table_slots * 8, (hipStream_t)stream));
    const unsigned grid = (unsigned)((n_panels + 255) / 256);
    hipLaunchKernelGGL(unique_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_hashes, d_panels,
                       n_panels, W, reinterpret_cast<unsigned long long *>(d_table), table_slots - 1,
                       reinterpret_cast<unsigned long long *>(d_unique), 1u, 0u);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_unique_hashes_async(const uint64_t *d_hashes, uint64_t n_hashes, uint32_t world, uint32_t rank,
                            uint64_t *d_table, uint64_t table_slots, uint64_t *d_unique, void *stream) {
    if (!d_hashes || !d_table || !d_unique || world == 0 || rank >= world)
        return fail(CSA_E_INVALID, "unique_hashes: bad arguments");
    if (table_slots < 2 * n_hashes || (table_slots & (table_slots - 1)))
        return fail(CSA_E_INVALID, "unique_hashes: table_slots must be a power of two >= 2*n_hashes");
    if (n_hashes == 0) return CSA_OK;
    HIPCHK(hipMemsetAsync(d_table, 0, table_slots * 8, (hipStream_t)stream));
    const unsigned grid = (unsigned)((n_hashes + 255) / 256);
    hipLaunchKernelGGL(unique_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_hashes, nullptr,
                       n_hashes, 1, reinterpret_cast<unsigned long long *>(d_table), table_slots - 1,
                       reinterpret_cast<unsigned long long *>(d_unique), world, rank);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_legacy_sample(csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                      uint32_t flags, uint32_t max_attempts, uint64_t *panels_out, int64_t *person_counts,
                      int64_t *pair_counts, uint64_t *unique_out, uint32_t *attempts_out) {
    if (!I) return fail(CSA_E_INVALID, "null instance");
    if ((flags & CSA_WANT_PANELS) && !panels_out) return fail(CSA_E_INVALID, "panels_out is NULL");
    if ((flags & CSA_WANT_COUNTS) && !person_counts) return fail(CSA_E_INVALID, "person_counts is NULL");
    if ((flags & CSA_WANT_PAIRS) && !pair_counts) return fail(CSA_E_INVALID, "pair_counts is NULL");
    if ((flags & CSA_WANT_UNIQUE) && !unique_out) return fail(CSA_E_INVALID, "unique_out is NULL");
    // analysis.py:174-176
    for (int c = 0; c < I->C; ++c) {
        int64_t smin = 0, smax = 0;
        for (int f = 0; f < I->F; ++f)
            if (I->fcat[f] == c) {
                smin += I->fmin[f];
                smax += I->fmax[f];
            }
        if (smin > k || smax < k)
            return fail(CSA_E_BAD_QUOTAS, "category %d: sum(min)=%lld, sum(max)=%lld, k=%d", c, (long long)smin,
                        (long long)smax, k);
    }
    ScopedDevice sd(I->device);
    const int n = I->n, W = I->W;
    const int npad = csa_xt_pad(std::max(n, 1));
    const uint64_t nblk = (n_panels + 63) / 64;
    hipStream_t st = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct StreamGuard {
        hipStream_t s;
        ~StreamGuard() { (void)hipStreamDestroy(s); }
    } sg{st};
    DevBuf<uint64_t> panels, hashes, xt, table, uniq;
    DevBuf<int64_t> counts, pairs;
    DevBuf<uint32_t> attempts, status;
    int rc;
    const bool want_unique = flags & CSA_WANT_UNIQUE, want_pairs = flags & CSA_WANT_PAIRS;
    const bool want_counts = flags & CSA_WANT_COUNTS;
    const uint64_t slots = pow2_at_least(std::max<uint64_t>(2 * n_panels, 64));
    if ((rc = dalloc(&panels.p, n_panels * W)) || (rc = dalloc(&status.p, 4))) return rc;
    if (want_unique && ((rc = dalloc(&hashes.p, 2 * n_panels)) || (rc = dalloc(&table.p, slots)) ||
                        (rc = dalloc(&uniq.p, 1))))
        return rc;
    if (attempts_out && (rc = dalloc(&attempts.p, n_panels))) return rc;
    if ((want_counts || want_pairs) && (rc = dalloc(&counts.p, n))) return rc;
    if (want_pairs && ((rc = dalloc(&xt.p, nblk * npad)) || (rc = dalloc(&pairs.p, (size_t)n * n)))) return rc;
    HIPCHK(hipMemsetAsync(status.p, 0, 16, st));
    if (counts.p) HIPCHK(hipMemsetAsync(counts.p, 0, (size_t)n * 8, st));
    if (pairs.p) HIPCHK(hipMemsetAsync(pairs.p, 0, (size_t)n * n * 8, st));
    if (uniq.p) HIPCHK(hipMemsetAsync(uniq.p, 0, 8, st));
    if ((rc = launch_draw(I, k, seed, panel_begin, n_panels, max_attempts, 0, 0, panels.p, hashes.p, attempts.p,
                          nullptr, status.p, nullptr, nullptr, nullptr, st)))
        return rc;
    uint32_t hs[4];
    if ((rc = read_status(status.p, st, hs))) return rc;
    if ((rc = csa_status_decode(hs))) return rc;
    if (counts.p && (rc = csa_transpose_count_async(panels.p, n_panels, n, xt.p, counts.p, st))) return rc;
    if (pairs.p && (rc = csa_pair_counts_async(xt.p, nblk, n, pairs.p, st))) return rc;
    if (want_unique && (rc = csa_unique_async(hashes.p, panels.p, n_panels, W, table.p, slots, uniq.p, st)))
        return rc;
    if (flags & CSA_WANT_PANELS)
        HIPCHK(hipMemcpyAsync(panels_out, panels.p, n_panels * W * 8, hipMemcpyDeviceToHost, st));
    if (want_counts) HIPCHK(hipMemcpyAsync(person_counts, counts.p, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    if (want_pairs) HIPCHK(hipMemcpyAsync(pair_counts, pairs.p, (size_t)n * n * 8, hipMemcpyDeviceToHost, st));
    if (want_unique) HIPCHK(hipMemcpyAsync(unique_out, uniq.p, 8, hipMemcpyDeviceToHost, st));
    if (attempts_out) HIPCHK(hipMemcpyAsync(attempts_out, attempts.p, n_panels * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return CSA_OK;
}

int csa_legacy_find(csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                    uint32_t max_attempts, int32_t *picks_out, uint32_t *attempts_out) {
    if (!I || !picks_out) return fail(CSA_E_INVALID, "null instance or picks_out");
    ScopedDevice sd(I->device);
    DevBuf<uint64_t> panels;
    DevBuf<int32_t> picks;
    DevBuf<uint32_t> attempts, status;
    int rc;
    if ((rc = dalloc(&panels.p, n_panels * I->W)) || (rc = dalloc(&picks.p, n_panels * (uint64_t)k)) ||
        (rc = dalloc(&status.p, 4)))
        return rc;
    if (attempts_out && (rc = dalloc(&attempts.p, n_panels))) return rc;
    HIPCHK(hipMemset(status.p, 0, 16));
    if ((rc = launch_draw(I, k, seed, panel_begin, n_panels, max_attempts, 0, 0, panels.p, nullptr, attempts.p,
                          picks.p, status.p, nullptr, nullptr, nullptr, nullptr)))
        return rc;
    uint32_t hs[4];
    if ((rc = read_status(status.p, nullptr, hs))) return rc;
    if ((rc = csa_status_decode(hs))) return rc;
    HIPCHK(hipMemcpy(picks_out, picks.p, n_panels * (uint64_t)k * 4, hipMemcpyDeviceToHost));
    if (attempts_out) HIPCHK(hipMemcpy(attempts_out, attempts.p, n_panels * 4, hipMemcpyDeviceToHost));
    return CSA_OK;
}

int csa_legacy_attempt(csa_instance *I, int32_t k, uint64_t seed, uint64_t panel, uint32_t attempt,
                       int32_t *picks_out, int32_t *n_picks, int32_t *sel_out, int32_t *rem_out,
                       uint64_t *present_out) {
    if (!I) return fail(CSA_E_INVALID, "null instance");
    ScopedDevice sd(I->device);
    DevBuf<uint64_t> panels, present;
    DevBuf<int32_t> picks, sel, rem;
    DevBuf<uint32_t> status;
    int rc;
    if ((rc = dalloc(&panels.p, I->W)) || (rc = dalloc(&picks.p, std::max(k, 1))) || (rc = dalloc(&sel.p, I->F)) ||
        (rc = dalloc(&rem.p, I->F)) || (rc = dalloc(&present.p, I->W)) || (rc = dalloc(&status.p, 4)))
        return rc;
    HIPCHK(hipMemset(status.p, 0, 16));
    HIPCHK(hipMemset(picks.p, 0xFF, std::max(k, 1) * 4));
    if ((rc = launch_draw(I, k, seed, panel, 1, 1, attempt, 1, panels.p, nullptr, nullptr, picks.p, status.p, sel.p,
                          rem.p, present.p, nullptr)))
        return rc;
    uint32_t hs[4];
    if ((rc = read_status(status.p, nullptr, hs))) return rc;
    if (hs[0] == CSA_E_NO_CANDIDATE) return csa_status_decode(hs);
    if (hs[3] == kFail) return fail(CSA_E_SELECTION, "SelectionError (legacy.py:34)");
    std::vector<int32_t> pk(std::max(k, 1));
    HIPCHK(hipMemcpy(pk.data(), picks.p, pk.size() * 4, hipMemcpyDeviceToHost));
    int np = 0;
    for (int s = 0; s < k; ++s)
        if (pk[s] >= 0) {
            if (picks_out) picks_out[np] = pk[s];
            ++np;
        }
    if (n_picks) *n_picks = np;
    if (sel_out) HIPCHK(hipMemcpy(sel_out, sel.p, I->F * 4, hipMemcpyDeviceToHost));
    if (rem_out) HIPCHK(hipMemcpy(rem_out, rem.p, I->F * 4, hipMemcpyDeviceToHost));
    if (present_out) HIPCHK(hipMemcpy(present_out, present.p, I->W * 8, hipMemcpyDeviceToHost));
    return CSA_OK;
}

}  // extern "C"
