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
//   pair_mfma_kernel     X^T X on MFMA, panels as the K dimension: fp4 (e2m1, exact 0/1
//                        products, f32 accumulation) or int8 (v_mfma_i32_32x32x32_i8);
//                        upper-triangular 256x256 blocks, split-K, int32 partial tiles +
//                        pair_reduce_kernel
//                        (PairHistogram.add_portfolio_of_panels_to_histogram, analysis.py:90-95).
//   unique_kernel        open-addressing table of panel indices keyed by a 128-bit panel
//                        hash, exact full-bitmask compare (found_panels, analysis.py:171,186).
// The C ABI is declared in include/csa_legacy.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>
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

// position (0..63) of the rr-th (1-based) set bit of m; requires 1 <= rr <= popcount(m)
__device__ __forceinline__ int select_bit(uint64_t m, int rr) {
    // the 32-bit half first, then a binary search on 32-bit values (no 64-bit masks or shifts)
    uint32_t x = (uint32_t)m;
    int pos = 0;
    const int c0 = __popc(x);
    if (rr > c0) {
        rr -= c0;
        x = (uint32_t)(m >> 32);
        pos = 32;
    }
#pragma unroll
    for (int s = 16; s >= 1; s >>= 1) {
        const int c = __popc(x & ((1u << s) - 1u));
        if (rr > c) {
            rr -= c;
            x >>= s;
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
    const uint32_t *pmask;     // n person feature masks (bit f = holds feature f; F <= 32) or null
    const int32_t *addr_next;  // same-address rings (check_same_address, draw_kernel GENERAL) or null
    int32_t n, F, W, Ws, k;
    uint32_t max_attempts, attempt_base;
    int32_t single;            // 1: exactly one attempt, no min-quota check, write final state
    uint64_t seed, panel_begin, n_panels;
    uint64_t *panels;          // n_panels x W
    uint64_t *hashes;          // 2 x n_panels or null
    uint32_t *attempts;        // n_panels or null
    int32_t *picks;            // n_panels x k or null
    uint16_t *picks16;         // draw_lane_kernel: n_panels x k pick lists (picks_pack_kernel -> panels)
    uint32_t *status;          // 4 words
    // draw statistics (csa_instance_draw_stats): [0] SelectionError restarts, [1] min-quota
    // rejections; one fire-and-forget atomic per restart (null: not counted)
    unsigned long long *stats;
    // draw_kernel GENERAL only: draw the panels panel_list[i] (i < min(n_panels, *n_panels_dev)) into
    // row i instead of panel_begin + i (the multi-GPU owner's re-draw of hash-match candidates)
    const uint64_t *panel_list;
    const unsigned long long *n_panels_dev;
    int32_t *sel_out, *rem_out;
    uint64_t *present_out;
    // csa_draw_xt_async (draw_lane_kernel's fused pack only): the launch's panels also as XT (the
    // pair kernels' operand, csa_transpose_count_async's layout: two 32-bit planes per 64-panel block,
    // npad persons each) or null
    uint32_t *xt;
    int32_t npad;
};

// ---- sub-wave group primitives ------------------------------------------------------------
// A panel is drawn by a group of G lanes (G = 16: one DPP row; 32; 64 = whole wave).  All
// cross-lane traffic inside a group is DPP (quad_perm / row mirrors / row_shr / row_bcast)
// except the xor-16 / xor-32 butterfly levels of G = 32 / 64 (ds_bpermute).

template <int CTRL, int ROW_MASK = 0xF, bool BOUND_ZERO = false>
__device__ __forceinline__ int dpp(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, 0xF, BOUND_ZERO);
}

// butterfly partner at level LVL: quad xor1, quad xor2, half-row mirror, row mirror, xor16, xor32
template <int LVL>
__device__ __forceinline__ int partner(int v) {
    // every source lane of these patterns is valid, so bound_ctrl / old are irrelevant; (0, bc=1)
    // lets the compiler fold the DPP move into the consuming VALU op
    if constexpr (LVL == 0) return dpp<0xB1, 0xF, true>(0, v);
    else if constexpr (LVL == 1) return dpp<0x4E, 0xF, true>(0, v);
    else if constexpr (LVL == 2) return dpp<0x141, 0xF, true>(0, v);
    else if constexpr (LVL == 3) return dpp<0x140, 0xF, true>(0, v);
    else if constexpr (LVL == 4) return __shfl_xor(v, 16);
    else return __shfl_xor(v, 32);
}

template <int LVL>
__device__ __forceinline__ uint64_t partner64(uint64_t v) {
    const uint32_t lo = (uint32_t)partner<LVL>((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)partner<LVL>((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

constexpr int group_levels(int G) { return G == 16 ? 4 : (G == 32 ? 5 : 6); }

// strict-'>' argmax over need/den with lowest feature index on ties (legacy.py:145); branch-free,
// 24-bit multiplies (|need| < 2^23, den < 2^23 and need*den inside int32: checked on the host)
template <int LVL, int NL>
__device__ __forceinline__ void group_argmax(int &bn, int &bd, int &bi) {
    if constexpr (LVL < NL) {
        const int on = partner<LVL>(bn), od = partner<LVL>(bd), oi = partner<LVL>(bi);
        const int l = __mul24(on, bd), r = __mul24(bn, od);
        const bool take = (l > r) | ((l == r) & (oi < bi));
        bn = take ? on : bn;
        bd = take ? od : bd;
        bi = take ? oi : bi;
        group_argmax<LVL + 1, NL>(bn, bd, bi);
    }
}

template <int LVL, int NL>
__device__ __forceinline__ int group_max(int v) {
    if constexpr (LVL < NL) {
        return group_max<LVL + 1, NL>(max(v, partner<LVL>(v)));
    } else {
        return v;
    }
}

template <int LVL, int NL>
__device__ __forceinline__ uint64_t group_sum64(uint64_t v) {
    if constexpr (LVL < NL) {
        return group_sum64<LVL + 1, NL>(v + partner64<LVL>(v));
    } else {
        return v;
    }
}

// inclusive prefix sum inside the group (Hillis-Steele on DPP rows, row_bcast across rows)
template <int G>
__device__ __forceinline__ int group_scan(int v) {
    v += dpp<0x111, 0xF, true>(0, v);
    v += dpp<0x112, 0xF, true>(0, v);
    v += dpp<0x114, 0xF, true>(0, v);
    v += dpp<0x118, 0xF, true>(0, v);
    if constexpr (G >= 32) v += dpp<0x142, 0xA>(0, v);
    if constexpr (G == 64) v += dpp<0x143, 0xC>(0, v);
    return v;
}

template <int G>
__device__ __forceinline__ uint64_t group_bits(bool pred, int gbase) {
    const uint64_t b = __ballot(pred);
    if constexpr (G == 64) return b;
    else return (b >> gbase) & ((1ull << G) - 1);
}

template <int G>
__device__ __forceinline__ bool group_any(bool pred, int gbase) {
    return group_bits<G>(pred, gbase) != 0ull;
}

enum : int { kContinue = -1, kAccept = 0, kFail = 1, kReject = 2, kNoCandidate = 3 };

__device__ __forceinline__ void raise_status(uint32_t *status, uint32_t code, uint64_t panel) {
    // Materialise the operands here, on the rare path: left to itself the compiler keeps the constant
    // code (and the zero compare value) in a VGPR pair across the whole draw loop, which spilled it in
    // the register-bound kernels.
    uint32_t c = code, z = 0u;
    asm volatile("" : "+v"(c), "+v"(z));
    if (atomicCAS(&status[0], z, c) == 0u) {
        status[1] = (uint32_t)panel;
        status[2] = (uint32_t)(panel >> 32);
    }
}

// LDS image of the feature bitmasks: G*FPL rows (features >= F are all-zero rows with
// min = max = remaining = 0, i.e. never candidates) of Ls = G*WPL + 1 words (odd stride:
// lane-f reads of one word column are bank-conflict free; words >= W are zero).
// Then per group: KR Philox words (u32) and a W-word cascade scratch row (u64).
__host__ __device__ inline size_t draw_lds_bytes(int G, int FPL, int WPL, int W, int k, int groups) {
    const size_t KR = (size_t)((k + 3) & ~3);
    return (size_t)G * FPL * (G * WPL + 1) * 8 + (size_t)groups * KR * 4 + (size_t)groups * W * 8;
}

// One LEGACY draw per G-lane group, persistent over panels i = group, group + n_groups, ...
// Per group and step: find_max_ratio_cat (legacy.py:124-157) as a group argmax over
// FPL features per lane, the r-th remaining holder (legacy.py:186-197) as a group prefix
// sum over WPL bitset words per lane, delete_person + delete_all_in_cat (legacy.py:47-120)
// in bulk bitset form, and the SelectionError / rejection tests (legacy.py:132-137,
// 55, 73, 198-199; analysis.py:155-159).  Restarts re-key Philox with attempt + 1.
// GENERAL = false: batch mode only (panels / hashes / attempts); GENERAL = true adds pick
// order (legacy_find) and the single-attempt state outputs (find_random_sample_legacy).
// waves per SIMD requested from the register allocator: small instances fit 6 (80 VGPRs)
constexpr int draw_occupancy(int FPL, int WPL) { return FPL + WPL <= 4 ? 6 : 1; }
// threads per workgroup: the LDS feature rows are shared by the workgroup, so large instances
// (n = 8192: 66 KB of rows + 1.8 KB per group) get 512 threads = 2 waves per SIMD in one
// workgroup per CU, where 256 threads left 1 wave per SIMD (LDS-limited to one workgroup)
constexpr int draw_threads(int FPL, int WPL) { return (FPL + WPL > 4 && WPL <= 8) ? 2 * kDrawThreads : kDrawThreads; }

template <int G, int FPL, int WPL, bool GENERAL>
__global__ __launch_bounds__(draw_threads(FPL, WPL), draw_occupancy(FPL, WPL)) void draw_kernel(DrawArgs A) {
    constexpr int NL = group_levels(G);
    constexpr int FR = G * FPL;        // LDS feature rows
    constexpr int Ls = G * WPL + 1;    // LDS row stride (words)
    extern __shared__ uint64_t smem[];
    const int F = A.F, W = A.W, k = A.k;
    const int KR = (k + 3) & ~3;
    const int groups_wg = blockDim.x / G;
    // an index-list re-draw sized for its worst case: workgroups past the list's length (usually
    // all of them) leave before loading the feature rows
    if (GENERAL && A.n_panels_dev && (uint64_t)blockIdx.x * groups_wg >= (uint64_t)*A.n_panels_dev) return;
    uint64_t *fm = smem;
    uint32_t *rng_all = reinterpret_cast<uint32_t *>(smem + FR * Ls);
    uint64_t *dscr_all = reinterpret_cast<uint64_t *>(rng_all + (size_t)groups_wg * KR);
    for (int t = threadIdx.x; t < FR * Ls; t += blockDim.x) {
        const int f = t / Ls, w = t - f * Ls;
        fm[t] = (f < F && w < W) ? A.featmask[f * A.Ws + w] : 0ull;
    }
    __syncthreads();
    const uint32_t *fm32 = reinterpret_cast<const uint32_t *>(fm);

    const int lane = threadIdx.x & 63;
    const int glane = lane & (G - 1);
    const int gbase = lane - glane;
    const int gwg = threadIdx.x / G;
    uint32_t *rng = rng_all + (size_t)gwg * KR;
    uint64_t *dscr = dscr_all + (size_t)gwg * W;
    const uint64_t n_groups = (uint64_t)gridDim.x * groups_wg;

    int fmin[FPL], fmax[FPL], fid[FPL], sel0[FPL], rem0[FPL];
#pragma unroll
    for (int j = 0; j < FPL; ++j) {
        fid[j] = glane * FPL + j;
        const bool v = fid[j] < F;
        fmin[j] = v ? A.fmin[fid[j]] : 0;
        fmax[j] = v ? A.fmax[fid[j]] : 0;
        sel0[j] = v ? A.sel0[fid[j]] : 0;
        rem0[j] = v ? A.rem0[fid[j]] : 0;
    }
    uint64_t present0[WPL];
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
        const int w = glane * WPL + j;
        present0[j] = w < W ? A.present0[w] : 0ull;
    }

    int sel[FPL], rem[FPL];
    uint64_t rmn[WPL], pk[WPL];
    uint64_t i = (uint64_t)blockIdx.x * groups_wg + gwg;
    uint32_t a = 0;
    int s = 0;
    const uint64_t n_panels = (GENERAL && A.n_panels_dev) ? min(A.n_panels, (uint64_t)*A.n_panels_dev) : A.n_panels;
    bool active = i < n_panels;
    const bool single = GENERAL && A.single;
    const uint32_t max_att = single ? 1u : A.max_attempts;
    const uint32_t key0 = (uint32_t)A.seed, key1 = (uint32_t)(A.seed >> 32);
    if (active && __hip_atomic_load(&A.status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) active = false;

    while (__ballot(active) != 0ull) {
        if (active) {
            const uint64_t panel = (GENERAL && A.panel_list) ? A.panel_list[i] : A.panel_begin + i;
            if (s == 0) {  // start of an attempt (legacy_find's fresh deepcopy, analysis.py:147-148)
#pragma unroll
                for (int j = 0; j < FPL; ++j) {
                    sel[j] = sel0[j];
                    rem[j] = rem0[j];
                }
#pragma unroll
                for (int j = 0; j < WPL; ++j) {
                    rmn[j] = present0[j];
                    pk[j] = 0ull;
                }
                // Philox words of this attempt: block b covers steps 4b..4b+3 (oracle/philox.py)
                const uint32_t att = A.attempt_base + a;
                for (int b = glane; b < KR / 4; b += G) {
                    uint32_t x0 = (uint32_t)b, x1 = att, x2 = (uint32_t)panel, x3 = (uint32_t)(panel >> 32);
                    philox4x32_10(x0, x1, x2, x3, key0, key1);
                    *reinterpret_cast<uint4 *>(rng + 4 * b) = make_uint4(x0, x1, x2, x3);
                }
            }
            int outcome = kContinue;
            // --- find_max_ratio_cat (legacy.py:124-157) ------------------------------------
            int need[FPL];
            bool f1 = false;
#pragma unroll
            for (int j = 0; j < FPL; ++j) {
                need[j] = fmin[j] - sel[j];
                f1 |= (sel[j] < fmin[j]) & (rem[j] < need[j]);  // legacy.py:132-137
            }
            if (group_any<G>(f1, gbase)) {
                outcome = kFail;
            } else {
                // sentinel ratio -100/1 = the reference's initial best (legacy.py:125): every real
                // candidate (need > -100*rem, legacy.py:140-141) beats it, so the winner is the
                // sentinel iff no feature is a candidate
                int bn = -100, bd = 1, bi = fid[0];
#pragma unroll
                for (int j = 0; j < FPL; ++j) {
                    const bool cand = (rem[j] != 0) & (fmax[j] != 0) & (need[j] > __mul24(-100, rem[j]));
                    const bool take = cand & (__mul24(need[j], bd) > __mul24(bn, rem[j]));
                    bn = take ? need[j] : bn;
                    bd = take ? rem[j] : bd;
                    bi = take ? fid[j] : bi;
                }
                group_argmax<0, NL>(bn, bd, bi);
                bool ne = false;
#pragma unroll
                for (int j = 0; j < WPL; ++j) ne |= rmn[j] != 0ull;
                int p = -1;
                if ((bn == -100) & (bd == 1)) {
                    if (group_any<G>(ne, gbase)) outcome = kNoCandidate;  // KeyError, legacy.py:188
                } else {
                    // randint(1, remaining[f*]) (legacy.py:149), Philox verification mode
                    const uint32_t u = rng[s];
                    const int r = 1 + (int)__umulhi(u, (uint32_t)bd);
                    // r-th remaining holder of f* in agent order (legacy.py:186-197)
                    uint64_t m[WPL];
                    int c[WPL], cnt = 0;
#pragma unroll
                    for (int j = 0; j < WPL; ++j) {
                        m[j] = rmn[j] & fm[bi * Ls + glane * WPL + j];
                        c[j] = __popcll(m[j]);
                        cnt += c[j];
                    }
                    const int incl = group_scan<G>(cnt);
                    int rr = r - (incl - cnt);
                    const bool hit = (rr >= 1) & (rr <= cnt);
                    uint64_t ms = m[0];
                    int js = 0;
                    bool done = false;
#pragma unroll
                    for (int j = 1; j < WPL; ++j) {
                        const bool nxt = !done & (rr > c[j - 1]);
                        done |= !nxt;
                        rr = nxt ? rr - c[j - 1] : rr;
                        ms = nxt ? m[j] : ms;
                        js = nxt ? j : js;
                    }
                    const int pl = hit ? ((glane * WPL + js) * 64 + select_bit(ms, rr)) : -1;
                    p = group_max<0, NL>(pl);
                    if (p >= 0) {
                        // delete_person / really_delete_person (legacy.py:103-120, 67-75)
                        const int wi = p >> 6, bp = p & 63;
                        bool anyfull = false;
                        int has[FPL];
#pragma unroll
                        for (int j = 0; j < FPL; ++j) {
                            has[j] = (int)((fm32[2 * (fid[j] * Ls + wi) + (bp >> 5)] >> (bp & 31)) & 1u);
                            sel[j] += has[j];
                            rem[j] -= has[j];
                            anyfull |= (has[j] != 0) & (sel[j] == fmax[j]);
                        }
                        const uint64_t bit = 1ull << bp;
#pragma unroll
                        for (int j = 0; j < WPL; ++j) {
                            const uint64_t b = (glane * WPL + j == wi) ? bit : 0ull;
                            rmn[j] &= ~b;
                            pk[j] |= b;
                        }
                        // check_same_address (legacy.py:109-113): the remaining agents at the
                        // pick's address are deleted with selected=False before the cascades
                        // (walk of the pick's address ring; uniform across the group)
                        if constexpr (GENERAL) {
                            if (A.addr_next) {
                                for (int q = A.addr_next[p], guard = 0; q != p && guard < A.n;
                                     q = A.addr_next[q], ++guard) {
                                    const int wq = q >> 6, bq = q & 63;
                                    bool there = false;
#pragma unroll
                                    for (int j = 0; j < WPL; ++j)
                                        if (glane * WPL + j == wq) there = (rmn[j] >> bq) & 1ull;
                                    if (group_any<G>(there, gbase)) {
#pragma unroll
                                        for (int j = 0; j < WPL; ++j)
                                            if (glane * WPL + j == wq) rmn[j] &= ~(1ull << bq);
#pragma unroll
                                        for (int j = 0; j < FPL; ++j)
                                            rem[j] -= (int)((fm32[2 * (fid[j] * Ls + wq) + (bq >> 5)] >> (bq & 31)) & 1u);
                                    }
                                }
                            }
                        }
                        // delete_all_in_cat for every full feature of the pick (legacy.py:47-62,
                        // 115-119), bulk form D = remaining & OR(featmask[full])
                        if (group_any<G>(anyfull, gbase)) {
                            uint64_t D[WPL];
#pragma unroll
                            for (int j = 0; j < WPL; ++j) D[j] = 0ull;
#pragma unroll
                            for (int jf = 0; jf < FPL; ++jf) {
                                uint64_t bm = group_bits<G>((has[jf] != 0) & (sel[jf] == fmax[jf]), gbase);
                                while (bm) {
                                    const int f = (__ffsll((unsigned long long)bm) - 1) * FPL + jf;
                                    bm &= bm - 1;
#pragma unroll
                                    for (int j = 0; j < WPL; ++j) D[j] |= fm[f * Ls + glane * WPL + j];
                                }
                            }
#pragma unroll
                            for (int j = 0; j < WPL; ++j) {
                                D[j] &= rmn[j];
                                rmn[j] &= ~D[j];
                                if (glane * WPL + j < W) dscr[glane * WPL + j] = D[j];
                            }
                            int dec[FPL];
#pragma unroll
                            for (int j = 0; j < FPL; ++j) dec[j] = 0;
                            for (int w = 0; w < W; ++w) {
                                const uint64_t dw = dscr[w];
                                if (dw) {
#pragma unroll
                                    for (int j = 0; j < FPL; ++j) dec[j] += __popcll(dw & fm[fid[j] * Ls + w]);
                                }
                            }
#pragma unroll
                            for (int j = 0; j < FPL; ++j) rem[j] -= dec[j];
                        }
                        // remaining == 0 and selected < min inside the deletes (legacy.py:55, 73)
                        bool f2 = false;
#pragma unroll
                        for (int j = 0; j < FPL; ++j) f2 |= (rem[j] == 0) & (sel[j] < fmin[j]);
                        if (group_any<G>(f2, gbase)) outcome = kFail;
                    }
                }
                if (GENERAL && A.picks && glane == 0) A.picks[i * (uint64_t)k + s] = p;
                if (outcome == kContinue && s < k - 1) {  // legacy.py:198-199
                    bool ne2 = false;
#pragma unroll
                    for (int j = 0; j < WPL; ++j) ne2 |= rmn[j] != 0ull;
                    if (!group_any<G>(ne2, gbase)) outcome = kFail;
                }
            }
            if (outcome == kContinue) {
                ++s;
                if (s == k) {  // check_min_cats (legacy.py:160-168, analysis.py:155-159)
                    bool under = false;
#pragma unroll
                    for (int j = 0; j < FPL; ++j) under |= sel[j] < fmin[j];
                    outcome = group_any<G>(under, gbase) ? kReject : kAccept;
                }
            }
            if (outcome != kContinue) {
                // ---- attempt finished -------------------------------------------------------
                if (single) {  // find_random_sample_legacy: one attempt, report its state
                    if (glane == 0) {
                        A.status[3] = (uint32_t)outcome;
                        if (outcome == kNoCandidate) raise_status(A.status, CSA_E_NO_CANDIDATE, panel);
                    }
                    if (A.sel_out) {
#pragma unroll
                        for (int j = 0; j < FPL; ++j)
                            if (fid[j] < F) {
                                A.sel_out[fid[j]] = sel[j];
                                A.rem_out[fid[j]] = rem[j];
                            }
                    }
#pragma unroll
                    for (int j = 0; j < WPL; ++j)
                        if (glane * WPL + j < W) {
                            if (A.present_out) A.present_out[glane * WPL + j] = rmn[j];
                            A.panels[i * W + glane * WPL + j] = pk[j];
                        }
                    active = false;
                } else if (outcome == kNoCandidate) {
                    if (glane == 0) raise_status(A.status, CSA_E_NO_CANDIDATE, panel);
                    active = false;
                } else if (outcome != kAccept) {  // SelectionError restart / min-quota rejection
                    s = 0;
                    if (glane == 0 && A.stats) atomicAdd(A.stats + (outcome == kReject), 1ull);
                    if (++a >= max_att) {
                        if (glane == 0) raise_status(A.status, CSA_E_ATTEMPT_LIMIT, panel);
                        active = false;
                    }
                } else {
                    uint64_t h1 = 0, h2 = 0;
#pragma unroll
                    for (int j = 0; j < WPL; ++j) {
                        const uint64_t w = (uint64_t)(glane * WPL + j);
                        if (w < (uint64_t)W) {
                            A.panels[i * W + w] = pk[j];
                            h1 += fmix_a(pk[j] ^ (w * 0x9E3779B97F4A7C15ull));
                            h2 += fmix_b(pk[j] + (w + 1) * 0xD6E8FEB86659FD93ull);
                        }
                    }
                    if (A.hashes) {
                        h1 = group_sum64<0, NL>(h1);
                        h2 = group_sum64<0, NL>(h2);
                        if (glane == 0) {
                            A.hashes[2 * i] = h1;
                            A.hashes[2 * i + 1] = h2;
                        }
                    }
                    if (A.attempts && glane == 0) A.attempts[i] = a + 1;
                    i += n_groups;
                    a = 0;
                    s = 0;
                    active = i < n_panels;
                    if (active && __hip_atomic_load(&A.status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
                        active = false;
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Bit transpose + per-person counts
// ------------------------------------------------------------------------------------------
constexpr int kXtThreads = 256;
constexpr int kXtBlocksPerGroup = 16;  // at most 1024 panels per workgroup

// 64x64 bit-matrix transpose across a wavefront, in registers: lane i holds row i (bit j = column
// j) as (lo, hi) 32-bit halves; afterwards lane j holds column j (bit i = row i).  The six butterfly
// stages (stage s trades the bit-s half of the column index with lane bit s) run on VALU
// cross-lane moves only -- no ds_bpermute, no divergent branches (the round-2 form: 12 bpermutes and
// both sides of a lane-bit branch per stage):
//   s = 32: one v_permlane32_swap (lanes 32-63 of lo <-> lanes 0-31 of hi);
//   s = 16: the 16-bit fields each lane keeps / gives are gathered into two registers (v_perm), one
//           v_permlane16_swap trades the given ones between rows 2r and 2r+1, two v_perm re-interleave;
//   s = 8:  the given bytes gathered by a lane-dependent v_perm, DPP row_ror:8 (= lane ^ 8), two
//           lane-dependent v_perm merge;
//   s = 4, 2, 1: the partner's word by DPP (quad_perm xor 3 + row_half_mirror = lane ^ 4; quad_perm
//           for ^ 2, ^ 1), rotated into place by v_alignbit, merged by v_bfi with the lane's keep mask.
// 30 VALU per 64x64 block; the stage algebra is modelled lane by lane and checked in
// tests/test_host_logic.py::test_xt_register_transpose_network.
struct XtLane {
    uint32_t s8_send, s8_lo, s8_hi;  // stage 8 byte selectors
    uint32_t k4, k2, k1;             // keep masks of stages 4, 2, 1
    uint32_t r4, r2, r1;             // rotate amounts of stages 4, 2, 1
};
__device__ __forceinline__ XtLane xt_lane_consts(int lane) {
    XtLane c;
    const bool b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1, b1 = (lane >> 1) & 1, b0 = lane & 1;
    c.s8_send = b3 ? 0x06040200u : 0x07050301u;
    c.s8_lo = b3 ? 0x03050104u : 0x05020400u;
    c.s8_hi = b3 ? 0x03070106u : 0x07020600u;
    c.k4 = b2 ? 0xF0F0F0F0u : 0x0F0F0F0Fu;
    c.k2 = b1 ? 0xCCCCCCCCu : 0x33333333u;
    c.k1 = b0 ? 0xAAAAAAAAu : 0x55555555u;
    c.r4 = b2 ? 4u : 28u;
    c.r2 = b1 ? 2u : 30u;
    c.r1 = b0 ? 1u : 31u;
    return c;
}
template <int CTRL>
__device__ __forceinline__ uint32_t xt_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t xt_merge(uint32_t x, uint32_t y, uint32_t keep, uint32_t rot) {
    const uint32_t t = __builtin_amdgcn_alignbit(y, y, rot);  // y rotated right by rot
    return (keep & x) | (~keep & t);                        // v_bfi
}
__device__ __forceinline__ void wave_transpose64(uint32_t &lo, uint32_t &hi, const XtLane &c) {
    {  // s = 32
        const auto r = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
        lo = r[0];
        hi = r[1];
    }
    {  // s = 16
        const uint32_t A = __builtin_amdgcn_perm(hi, lo, 0x05040100u), B = __builtin_amdgcn_perm(hi, lo, 0x07060302u);
        const auto r = __builtin_amdgcn_permlane16_swap(A, B, false, false);
        lo = __builtin_amdgcn_perm(r[1], r[0], 0x05040100u);
        hi = __builtin_amdgcn_perm(r[1], r[0], 0x07060302u);
    }
    {  // s = 8
        const uint32_t R = xt_dpp<0x128>(__builtin_amdgcn_perm(hi, lo, c.s8_send));  // row_ror:8
        lo = __builtin_amdgcn_perm(R, lo, c.s8_lo);
        hi = __builtin_amdgcn_perm(R, hi, c.s8_hi);
    }
    // s = 4: quad_perm [3,2,1,0] then row_half_mirror = lane ^ 4
    lo = xt_merge(lo, xt_dpp<0x141>(xt_dpp<0x1B>(lo)), c.k4, c.r4);
    hi = xt_merge(hi, xt_dpp<0x141>(xt_dpp<0x1B>(hi)), c.k4, c.r4);
    lo = xt_merge(lo, xt_dpp<0x4E>(lo), c.k2, c.r2);  // s = 2: quad_perm [2,3,0,1]
    hi = xt_merge(hi, xt_dpp<0x4E>(hi), c.k2, c.r2);
    lo = xt_merge(lo, xt_dpp<0xB1>(lo), c.k1, c.r1);  // s = 1: quad_perm [1,0,3,2]
    hi = xt_merge(hi, xt_dpp<0xB1>(hi), c.k1, c.r1);
}

#include "draw_lane.inc"
#include "draw_wide.inc"
#include "draw_solo.inc"

// 128-bit panel hashes (the draw_kernel's in-kernel hash, for the batch kernel's panels): a
// quad of lanes per panel, words glane, glane+4, ... (coalesced within the quad), quad sum.
__global__ __launch_bounds__(256) void panel_hash_kernel(const uint64_t *__restrict__ panels, uint64_t S, int W,
                                                         uint64_t *__restrict__ hashes) {
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    const int q = threadIdx.x & 3;
    uint64_t h1 = 0, h2 = 0;
    if (i < S) {
        for (int w = q; w < W; w += 4) {
            const uint64_t pk = panels[i * W + w];
            h1 += fmix_a(pk ^ ((uint64_t)w * 0x9E3779B97F4A7C15ull));
            h2 += fmix_b(pk + ((uint64_t)w + 1) * 0xD6E8FEB86659FD93ull);
        }
    }
    h1 = group_sum64<0, 2>(h1);
    h2 = group_sum64<0, 2>(h2);
    if (i < S && q == 0) {
        hashes[2 * i] = h1;
        hashes[2 * i + 1] = h2;
    }
}

// blockIdx.y = column range: words [CW y, CW y + CW) of every panel, i.e. agents [64 CW y, ...).
// 32 words per range: a 17 KB tile + 8 KB of counts per workgroup, so ~6 workgroups share a CU and
// one's loads overlap another's transposes (128-word ranges at n = 8192 needed 98 KB, one
// workgroup per CU, and moved 2 GB per 10^6 panels at 0.9 TB/s).  Inside a workgroup the next
// block's panel words are loaded into registers while the current block is transposed (thread t
// loads rows t/32 + 8q, word t%32: no integer division per element).
constexpr int kXtCols = 32;
__global__ __launch_bounds__(kXtThreads) void xt_count_kernel(const uint64_t *__restrict__ panels,
                                                              uint64_t S, int n, int W, int npad,
                                                              uint64_t *__restrict__ xt,
                                                              int64_t *__restrict__ counts, int bpg) {
    extern __shared__ uint64_t smem[];
    const int c0 = (int)blockIdx.y * kXtCols, CW = min(kXtCols, W - c0);  // this block's word range
    const int Wp = CW | 1;
    const int p0 = 64 * c0, np = min(n - p0, 64 * CW);                   // its agents
    uint64_t *tile = smem;                                   // 64 x Wp
    uint32_t *cnt = reinterpret_cast<uint32_t *>(smem + 64 * Wp);  // np
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    const XtLane tc = xt_lane_consts(lane);
    for (int p = threadIdx.x; p < np; p += blockDim.x) cnt[p] = 0;
    const uint64_t nblk = (S + 63) / 64;
    const uint64_t b0 = (uint64_t)blockIdx.x * bpg;
    const uint64_t b1 = min(nblk, b0 + (uint64_t)bpg);
    const int ncol = min(npad / 64 - c0, kXtCols);  // transposed columns (padding included)
    static_assert(kXtThreads == 256 && kXtCols == 32, "loader: 8 rows of 32 words per pass");
    const int lr = threadIdx.x >> 5, lc = threadIdx.x & 31;
    uint64_t pre[8];
    auto load_blk = [&](uint64_t b) {
        const uint64_t row0 = b * 64;
        const int rows = (int)min<uint64_t>(64, S - row0);
        // branch-free: out-of-range rows / words load a clamped in-range address and are zeroed
        const uint64_t *src = panels + row0 * (uint64_t)W + c0 + min(lc, CW - 1);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int r = lr + 8 * q;
            const uint64_t v = src[(uint64_t)min(r, rows - 1) * W];
            pre[q] = (lc < CW && r < rows) ? v : 0ull;
        }
    };
    if (b0 < b1) load_blk(b0);
    for (uint64_t b = b0; b < b1; ++b) {
        __syncthreads();  // every wave is done with the previous block's tile
        if (lc < CW) {
#pragma unroll
            for (int q = 0; q < 8; ++q) tile[(lr + 8 * q) * Wp + lc] = pre[q];
        }
        __syncthreads();
        if (b + 1 < b1) load_blk(b + 1);  // in flight while this block is transposed
        for (int w = wv; w < ncol; w += nwv) {
            const uint64_t x = w < CW ? tile[lane * Wp + w] : 0ull;
            uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
            wave_transpose64(lo, hi, tc);
            const int p = 64 * w + lane;
            if (xt) {  // two 32-bit planes per panel block: panels 64b..64b+31, then 64b+32..64b+63
                uint32_t *x32 = reinterpret_cast<uint32_t *>(xt) + 2 * b * (uint64_t)npad + p0 + p;
                x32[0] = lo;
                x32[npad] = hi;
            }
            if (p < np) cnt[p] += (uint32_t)(__popc(lo) + __popc(hi));
        }
    }
    __syncthreads();
    for (int p = threadIdx.x; p < np; p += blockDim.x)
        if (cnt[p]) atomicAdd(reinterpret_cast<unsigned long long *>(counts + p0 + p), (unsigned long long)cnt[p]);
}

// ------------------------------------------------------------------------------------------
// Pair counts: X^T X on MFMA (PairHistogram.add_portfolio_of_panels_to_histogram, analysis.py:90-95)
// ------------------------------------------------------------------------------------------
// Panels are the K dimension; one 64-bit XT word = one agent over 64 panels = 64 k-values.
// Two engines share the tiling (256 x 256 upper-triangular output block per 512-thread
// workgroup, 8 waves of 128 rows x 64 columns, two waves per SIMD):
//   CSA_PAIR_FP4  v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1 operands (scale 2^0): one MFMA
//                 per 32x32 tile per word (K = 64), f32 accumulation.  A k-bit becomes an fp4
//                 nibble with one set bit at position 0 / 1 / 2 (0.5 / 1.0 / 2.0); A and B put
//                 the same bit at complementary positions, so every product of two set bits is
//                 exactly 1.0 and the accumulators hold exact integer counts while < 2^24
//                 (enforced per split on the host).  4-5 VALU per 32 operand bits.
//   CSA_PAIR_I8   v_mfma_i32_32x32x32_i8 with 0/1 bytes, int32 accumulation: two MFMAs per
//                 word (K = 32 each), 16 VALU per 32 operand bits.
// Per KB-block stage the workgroup stages the packed words of its 256 rows + 256 columns in
// LDS (double-buffered, one barrier per KB blocks); each wave expands its own fragments in
// registers.  Splits of the panel blocks write int32 partial tiles (plain coalesced stores)
// that pair_reduce_kernel sums into the int64 output, or (no scratch) int64 atomics.
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kPairBlock = 256;   // output block per workgroup
constexpr int kPairThreads = 512;
constexpr int kPairKB = 8;        // 64-panel blocks staged per barrier (8: 0.76 ms at sf_e vs 0.79 for 4 or 16)

// int8 fragment (k-half ks, lane half h) of one XT word: dword q holds bits 4h+q, 4h+q+8,
// 4h+q+16, 4h+q+24 of the 32-bit half ks as 0/1 bytes.  Any fixed bit -> k placement works
// because A and B use the same one (the k order cancels in the sum over k).
__device__ __forceinline__ v4i i8_frag(uint64_t w, int ks, int h) {
    const uint32_t x = (uint32_t)(w >> (32 * ks));
    v4i r;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = (int)((x >> (4 * h + q)) & 0x01010101u);
    return r;
}

// fp4 fragments of the 32 bits x = half h of a word (lane half h covers k = 32h .. 32h+31):
// bit 4i+p of x goes to nibble i of dword p (A: positions 0,1,2,2 -> 0.5,1,2,2;
// B: positions 2,1,0,0 -> 2,1,0.5,0.5).
__device__ __forceinline__ v8i f4_frag_a(uint32_t x) {
    v8i r;
    r[0] = (int)(x & 0x11111111u);
    r[1] = (int)(x & 0x22222222u);
    r[2] = (int)(x & 0x44444444u);
    r[3] = (int)((x >> 1) & 0x44444444u);
    r[4] = r[5] = r[6] = r[7] = 0;  // fp4 operands use 4 registers
    return r;
}
__device__ __forceinline__ v8i f4_frag_b(uint32_t x) {
    v8i r;
    r[0] = (int)((x << 2) & 0x44444444u);
    r[1] = (int)(x & 0x22222222u);
    r[2] = (int)((x >> 2) & 0x11111111u);
    r[3] = (int)((x >> 3) & 0x11111111u);
    r[4] = r[5] = r[6] = r[7] = 0;
    return r;
}

__device__ __forceinline__ void tri_block(int tri, int nbt, int &bi, int &bj) {
    bi = 0;
    int rem = tri;
    while (rem >= nbt - bi) {
        rem -= nbt - bi;
        ++bi;
    }
    bj = bi + rem;
}

template <bool FP4, bool PARTIAL, int KB>
__global__ __launch_bounds__(kPairThreads) void pair_mfma_kernel(const uint64_t *__restrict__ xt,
                                                                 uint64_t nblk, int n, int npad,
                                                                 int nbt, int nsplit,
                                                                 int64_t *__restrict__ pairs,
                                                                 int32_t *__restrict__ part) {
    __shared__ uint64_t words[2][KB][2 * kPairBlock];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    // Workgroup g runs on XCD g mod 8 (round-robin dispatch).  The (tile, split) items in
    // split-major order are cut into 8 contiguous chunks, one per XCD, sized to that XCD's share of
    // the grid: the ~32 workgroups of an XCD then cover one or two splits (their tiles share the
    // split's XT strips through that XCD's L2) instead of every XCD touching every split -- sf_e
    // (28 tiles x 9 splits) fetched 1.5 GB per launch for a 224 MB operand with the tile-major order.
    // (Round 2's grouping of ONE split per XCD needed nsplit % 8 == 0 and left 32 CUs idle.)
    const int g = (int)blockIdx.x, G = (int)gridDim.x, ntri = nbt * (nbt + 1) / 2;
    const int xcd = g & 7, it = xcd * (G >> 3) + min(xcd, G & 7) + (g >> 3);
    const int split = it / ntri, tri = it - split * ntri;
    const int item = tri * nsplit + split;
    int bi, bj;
    tri_block(tri, nbt, bi, bj);
    const int I0 = bi * kPairBlock, J0 = bj * kPairBlock;
    const uint64_t per = (nblk + nsplit - 1) / nsplit;
    const uint64_t kb0 = min(nblk, (uint64_t)split * per), kb1 = min(nblk, kb0 + per);

    using acc_t = typename std::conditional<FP4, v16f, v16i>::type;
    acc_t acc[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[a][b][v] = 0;

    const int wr = wave >> 2, wc = wave & 3;
    const int r32 = lane & 31, h = lane >> 5;
    const int src = t < kPairBlock ? I0 + t : J0 + t - kPairBlock;  // staging role of this thread
    uint64_t nw[KB];
    const uint64_t nst = (kb1 - kb0 + KB - 1) / KB;
    auto load_stage = [&](uint64_t s) {
#pragma unroll
        for (int j = 0; j < KB; ++j) {  // blocks past the split's end stage as zero words (no contribution)
            const uint64_t b = kb0 + s * KB + j;
            const uint32_t *x32 = reinterpret_cast<const uint32_t *>(xt) + 2 * b * (uint64_t)npad + src;
            nw[j] = b < kb1 ? ((uint64_t)x32[0] | ((uint64_t)x32[npad] << 32)) : 0ull;
        }
    };
    if (nst) {
        load_stage(0);
#pragma unroll
        for (int j = 0; j < KB; ++j) words[0][j][t] = nw[j];
        if (nst > 1) load_stage(1);
    }
    __syncthreads();
    for (uint64_t s = 0; s < nst; ++s) {
        const int buf = (int)(s & 1);
#pragma unroll
        for (int j = 0; j < KB; ++j) {
            {  // branch-free: the tail stage's missing blocks are zero words
                const uint64_t *w = words[buf][j];
                if constexpr (FP4) {
                    // lane half h needs only the 32-bit half h of each word: read it directly
                    // (a split into two 32-bit planes, conflict-free for these reads, measured
                    // 1-5 % slower: twice the staging stores)
                    const uint32_t *w32 = reinterpret_cast<const uint32_t *>(w) + h;
                    v8i fa[4], fb[2];
#pragma unroll
                    for (int x = 0; x < 4; ++x) fa[x] = f4_frag_a(w32[2 * (128 * wr + 32 * x + r32)]);
#pragma unroll
                    for (int x = 0; x < 2; ++x) fb[x] = f4_frag_b(w32[2 * (kPairBlock + 64 * wc + 32 * x + r32)]);
#pragma unroll
                    for (int a = 0; a < 4; ++a)
#pragma unroll
                        for (int b = 0; b < 2; ++b)
                            acc[a][b] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                                fa[a], fb[b], acc[a][b], 4, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
                } else {
                    uint64_t wa[4], wb[2];
#pragma unroll
                    for (int x = 0; x < 4; ++x) wa[x] = w[128 * wr + 32 * x + r32];
#pragma unroll
                    for (int x = 0; x < 2; ++x) wb[x] = w[kPairBlock + 64 * wc + 32 * x + r32];
#pragma unroll
                    for (int ks = 0; ks < 2; ++ks) {
                        v4i fa[4], fb[2];
#pragma unroll
                        for (int x = 0; x < 4; ++x) fa[x] = i8_frag(wa[x], ks, h);
#pragma unroll
                        for (int x = 0; x < 2; ++x) fb[x] = i8_frag(wb[x], ks, h);
#pragma unroll
                        for (int a = 0; a < 4; ++a)
#pragma unroll
                            for (int b = 0; b < 2; ++b)
                                acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a], fb[b], acc[a][b], 0, 0, 0);
                    }
                }
            }
            if (j == 0) {  // hand the prefetched stage to LDS, prefetch the one after
                if (s + 1 < nst) {
#pragma unroll
                    for (int jj = 0; jj < KB; ++jj) words[buf ^ 1][jj][t] = nw[jj];
                }
                if (s + 2 < nst) load_stage(s + 2);
            }
        }
        __syncthreads();
    }
    // C/D layout (gfx950, dtype-independent): col = lane & 31, row = (v&3) + 8*(v>>2) + 4*(lane>>5)
    const int rloc = 128 * wr + 4 * h, cloc = 64 * wc + r32;
    if constexpr (PARTIAL) {
        int32_t *dst = part + (size_t)item * kPairBlock * kPairBlock;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const int row = rloc + 32 * a + (v & 3) + 8 * (v >> 2);
                    dst[row * kPairBlock + cloc + 32 * b] = (int)acc[a][b][v];
                }
    } else {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int col = J0 + cloc + 32 * b;
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const int row = I0 + rloc + 32 * a + (v & 3) + 8 * (v >> 2);
                    const int val = (int)acc[a][b][v];
                    if (val != 0 && row < n && col < n)
                        atomicAdd(reinterpret_cast<unsigned long long *>(pairs + (uint64_t)row * n + col),
                                  (unsigned long long)(long long)val);
                }
                __builtin_amdgcn_sched_barrier(0);  // keep the atomic addresses from being hoisted (VGPR spill)
            }
    }
}

// Sum the nsplit int32 partial tiles of every upper-triangular block into the int64 output
// (+=, or = with overwrite; each output element is owned by exactly one thread).  HBM-bound.
__global__ __launch_bounds__(256) void pair_reduce_kernel(const int32_t *__restrict__ part, int n, int nbt,
                                                          int nsplit, int64_t *__restrict__ pairs,
                                                          int overwrite) {
    int bi, bj;
    tri_block((int)blockIdx.y, nbt, bi, bj);
    const int e = blockIdx.x * 256 + threadIdx.x;  // element of the 256 x 256 block
    const int row = bi * kPairBlock + (e >> 8), col = bj * kPairBlock + (e & 255);
    if (row >= n || col >= n) return;
    const int32_t *p = part + (size_t)blockIdx.y * nsplit * kPairBlock * kPairBlock + e;
    int64_t acc = 0;
    for (int k = 0; k < nsplit; ++k) acc += p[(size_t)k * kPairBlock * kPairBlock];
    // overwrite (CSA_PAIR_OVERWRITE): every element of the block is stored, so the caller needs
    // no zero-fill of the n x n output before a fresh batch
    if (overwrite) pairs[(size_t)row * n + col] = acc;
    else if (acc) pairs[(size_t)row * n + col] += acc;
}

// ---- pair_fp4_tile_kernel: X^T X with the tiles grouped by XCD (fp4 engine) ----------------
// One persistent 256-thread workgroup per CU (4 waves, one per SIMD, 256 accumulator registers
// each): wave (wr, wc) owns rows 128 wr .. and columns 128 wc .. of a 256 x 256 output tile, 16
// MFMAs per 64-panel block from 4 A and 4 B fragments (3 VALU of fragment expansion per MFMA,
// against 4.25 in pair_mfma_kernel's 128 x 64 wave tile).  XT arrives by LDS-DMA
// (global_load_lds_dwordx4, one 1 KiB piece per wave per block: A plane 0 / 1, B plane 0 / 1 --
// the planes make every fragment read conflict-free) into a ring of kP2Depth blocks, one raw
// barrier per block, the fragments of block j + 1 read while block j's MFMAs run.
// Work (PairMap): the upper-triangular tiles in locality order (bands of 4 tile rows, columns left
// to right) are cut into 8 contiguous chunks, one per XCD (workgroup g runs on XCD g mod 8), so the
// 32 workgroups of an XCD stream few XT strips through its L2 together; an XCD's chunk of T tiles
// runs as floor(T / 32) rounds of whole tiles (f32 accumulators, exact below 2^24 panels, stored
// straight into the int64 output); the T mod 32 leftover tiles of all XCDs are pooled and cut into
// 256 / (their number) k-pieces each, one per workgroup, written as int32 partial tiles that
// pair_reduce2_kernel sums -- no round runs part-empty (n = 8192: 2 rounds + 16 tiles x 16 pieces;
// sf_e, n = 1727: 28 tiles x 9 pieces).
constexpr int kP2Threads = 256;
constexpr int kP2Depth = 8;      // LDS ring slots = blocks in flight (4 KiB each)
constexpr int kP2Xcds = 8;
constexpr uint64_t kP2MaxBlocks = ((1ull << 24) - 1) / 64;  // whole-tile items stay exact in f32

struct PairMap {
    int nbt, ntri, P;   // tiles per side, upper-triangle tiles, workgroups per XCD
    int halves;         // work items per tile: 1 (256 x 256 items) or 2 (256 x 128 column halves)
    uint64_t nblk;      // 64-panel blocks
    __host__ __device__ int nitems() const { return ntri * halves; }
    // item idx = (tile idx / halves in locality order, column half idx % halves): its tile and the
    // first column of the half inside it
    __host__ __device__ void item_at(int idx, int &bi, int &bj, int &c0) const {
        tile_at(idx / halves, bi, bj);
        c0 = (idx % halves) * (kPairBlock / halves);
    }
    // tile at locality-order index idx
    __host__ __device__ void tile_at(int idx, int &bi, int &bj) const {
        int r0 = 0;
        for (;;) {
            const int hb = nbt - r0 < 4 ? nbt - r0 : 4;
            const int cnt = hb * (hb + 1) / 2 + (nbt - r0 - hb) * hb;
            if (idx < cnt) break;
            idx -= cnt;
            r0 += 4;
        }
        const int hb = nbt - r0 < 4 ? nbt - r0 : 4;
        const int tri = hb * (hb + 1) / 2;
        if (idx < tri) {  // the band's diagonal corner: column r0 + c holds rows r0 .. r0 + c
            int c = 0;
            while (idx > c) {
                idx -= c + 1;
                ++c;
            }
            bj = r0 + c;
            bi = r0 + idx;
        } else {
            idx -= tri;
            bj = r0 + hb + idx / hb;
            bi = r0 + idx % hb;
        }
    }
    __host__ __device__ void xcd_chunk(int x, int &t0, int &tx) const {
        t0 = (int)((int64_t)nitems() * x / kP2Xcds);
        tx = (int)((int64_t)nitems() * (x + 1) / kP2Xcds) - t0;
    }
    // leftover tiles (the last tx mod P of each XCD chunk) pooled over the XCDs: their number, the
    // k-pieces per tile (every workgroup takes at most one piece), and the tile of pooled index l
    __host__ __device__ int leftovers() const {
        int tl = 0;
        for (int x = 0; x < kP2Xcds; ++x) {
            int t0, tx;
            xcd_chunk(x, t0, tx);
            tl += tx % P;
        }
        return tl;
    }
    __host__ __device__ int pieces(int tl) const { return tl ? (kP2Xcds * P) / tl : 0; }
    __host__ __device__ int leftover_tile(int l) const {
        for (int x = 0;; ++x) {
            int t0, tx;
            xcd_chunk(x, t0, tx);
            const int lx = tx % P;
            if (l < lx || x == kP2Xcds - 1) return t0 + (tx - lx) + l;
            l -= lx;
        }
    }
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

// NB = B fragments per wave.  NB = 4 (every launch): 128 x 128 wave tiles, 256 x 256 items, 256
// accumulators (one wave fills its SIMD's 512 registers).  NB = 2 (CSA_P2_NB=2, A/B and tests): 128 x 64
// wave tiles, 256 x 128 items
// (the column halves of a tile, PairMap::halves = 2), 128 accumulators, at most 256 registers -- a draw
// workgroup's two 128-VGPR waves per SIMD fit beside it.
// Every wave streams its own operands -- its 128 A rows and 32 NB B columns of each 64-panel block, two
// LDS-DMAs (global_load_lds_dwordx4, 1 KiB each) into a private ring of kP2Depth 2 KiB slots -- so no
// wave ever waits for another: no workgroup barrier in the block loop (a shared ring with one barrier
// per block ran 10.4 / 14.8 ms vs 10.3 / 13.3 ms per 10^6 panels at n = 8192, NB = 4 / 2).  The A and B
// strips are fetched twice per workgroup (once per wave row / column); the second fetch hits L2.
// Step j waits for its own block j + 2 (vmcnt: blocks j + 3 .. j + D - 1, two DMAs each, may still be in
// flight), issues block j + D into the slot block j leaves (read in step j - 2, whose ds_reads the
// lgkmcnt(0) of step j - 1 retired), reads block j + 2's words, expands block j + 1's fragments (VALU
// interleaved with block j's MFMAs) and runs block j's MFMAs.  The DMA issue is branch-free (past the
// last block it re-loads the last block into a slot nobody reads), so the counted waits are constants.
template <int NB>
__global__ __launch_bounds__(kP2Threads, NB == 4 ? 1 : 2) void pair_fp4_tile_kernel(const uint32_t *__restrict__ xt,
                                                                                  int n, int npad, PairMap M,
                                                                                  int64_t *__restrict__ pairs,
                                                                                  int32_t *__restrict__ part,
                                                                                  int overwrite) {
    static_assert(NB == 2 || NB == 4, "B fragments per wave: 2 or 4");
    constexpr int BC = 32 * NB;  // B columns of a wave
    // slot (u32): A plane 0 rows 0..127, A plane 1, B plane 0 columns 0..BC-1, B plane 1, padding
    __shared__ uint32_t ring[4][kP2Depth][512];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = wave >> 1, wc = wave & 1, r32 = lane & 31, h = lane >> 5;
    const int x = (int)blockIdx.x % kP2Xcds, w = (int)blockIdx.x / kP2Xcds;
    int t0, tx;
    M.xcd_chunk(x, t0, tx);
    const int F = tx / M.P, tl = M.leftovers(), sp = M.pieces(tl), g = (int)blockIdx.x;
    const int items = F + (g < tl * sp ? 1 : 0);
    // DMA lanes: A chunk = lane (plane lane / 32, rows 4 (lane % 32) ..); B chunk = lane % (BC / 2)
    // (plane .. / (BC / 4)); at NB = 2 lanes 32..63 repeat lanes 0..31 into the slot's padding
    const int bl = lane % (BC / 2);
    const int offa = (lane >> 5) * npad + 128 * wr + 4 * (lane & 31);
    const int offb = (bl / (BC / 4)) * npad + BC * wc + 4 * (bl % (BC / 4));
    uint32_t(&myring)[kP2Depth][512] = ring[wave];
    for (int it = 0; it < items; ++it) {
        int idx, slot = -1;
        uint64_t kb0 = 0, kb1 = M.nblk;
        if (it < F) {
            idx = t0 + it * M.P + w;
        } else {
            const int q = g % sp;
            idx = M.leftover_tile(g / sp);
            kb0 = M.nblk * (uint64_t)q / (uint64_t)sp;
            kb1 = M.nblk * (uint64_t)(q + 1) / (uint64_t)sp;
            slot = g;
        }
        int bi, bj, c0;
        M.item_at(idx, bi, bj, c0);
        const int I0 = bi * kPairBlock, J0 = bj * kPairBlock + c0;
        v16f acc[4][NB];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.0f;
        const uint64_t bstride = 2 * (uint64_t)npad;
        const uint32_t *ga = xt + 2 * kb0 * (uint64_t)npad + I0 + offa;
        const uint32_t *gb = xt + 2 * kb0 * (uint64_t)npad + J0 + offb;
        asm volatile("" : "+v"(ga), "+v"(gb));
        const int nb = (int)(kb1 - kb0);  // <= kP2MaxBlocks
        // the previous item's trailing DMAs (re-loads of its last block) have landed
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        auto dma = [&](int blk, int sl) {
            const uint64_t o = (uint64_t)min(blk, nb - 1) * bstride;
            __builtin_amdgcn_global_load_lds((gbl_void_t *)(ga + o), (lds_void_t *)&myring[sl][0], 16, 0, 0);
            __builtin_amdgcn_global_load_lds((gbl_void_t *)(gb + o), (lds_void_t *)&myring[sl][256], 16, 0, 0);
        };
        static_assert((kP2Depth & (kP2Depth - 1)) == 0 && kP2Depth >= 4, "ring slots: power of two >= 4");
        auto read_blk = [&](int blk, uint32_t(&na)[4], uint32_t(&nbw)[NB]) {
            const uint32_t *sl = myring[blk & (kP2Depth - 1)];
#pragma unroll
            for (int q = 0; q < 4; ++q) na[q] = sl[128 * h + 32 * q + r32];
#pragma unroll
            for (int q = 0; q < NB; ++q) nbw[q] = sl[256 + BC * h + 32 * q + r32];
        };
        auto expand = [&](const uint32_t(&ca)[4], const uint32_t(&cb)[NB], v8i(&fa)[4], v8i(&fb)[NB]) {
#pragma unroll
            for (int q = 0; q < 4; ++q) fa[q] = f4_frag_a(ca[q]);
#pragma unroll
            for (int q = 0; q < NB; ++q) fb[q] = f4_frag_b(cb[q]);
        };
        auto mfma = [&](const v8i(&fa)[4], const v8i(&fb)[NB]) {
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < NB; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[a], fb[b], acc[a][b], 4, 4, 0,
                                                                                0x7F7F7F7F, 0, 0x7F7F7F7F);
        };
        if (nb > 0) {
#pragma unroll
            for (int j = 0; j < kP2Depth; ++j) dma(j, j);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (kP2Depth - 2)) : "memory");
            uint32_t r0a[4], r0b[NB], r1a[4], r1b[NB];
            v8i f0a[4], f0b[NB], f1a[4], f1b[NB];
            read_blk(0, r0a, r0b);
            read_blk(1, r1a, r1b);
            expand(r0a, r0b, f0a, f0b);
            auto step = [&](int j, const v8i(&fca)[4], const v8i(&fcb)[NB], const uint32_t(&rna)[4],
                            const uint32_t(&rnb)[NB], v8i(&fna)[4], v8i(&fnb)[NB], uint32_t(&rwa)[4],
                            uint32_t(&rwb)[NB]) {
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_waitcnt vmcnt(%0)" ::"n"(2 * (kP2Depth - 3)) : "memory");
                dma(j + kP2Depth, j & (kP2Depth - 1));
                read_blk(j + 2, rwa, rwb);
                expand(rna, rnb, fna, fnb);
                mfma(fca, fcb);
                // one MFMA, then its share of the expansion VALU (NB = 4: 56 VALU for 16 MFMAs; NB = 2: 42
                // for 8): an MFMA holds the wave's issue for 8 of its 32 cycles and this wave is alone on
                // its SIMD, so the fillers must sit in the gaps, not in runs (the compiler's own order left
                // runs of 7 VALU and of 7 bare MFMAs: 10.3 -> 8.7 ms at NB = 4, 13.4 -> 11.9 at NB = 2)
#pragma unroll
                for (int q = 0; q < 4 * NB; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, NB == 4 ? 4 : 5, 0);  // VALU
                }
                __builtin_amdgcn_sched_barrier(0);
            };
            int j = 0;
            for (; j + 2 <= nb; j += 2) {
                step(j, f0a, f0b, r1a, r1b, f1a, f1b, r0a, r0b);
                step(j + 1, f1a, f1b, r0a, r0b, f0a, f0b, r1a, r1b);
            }
            // an odd last block: its fragments are expanded and nothing is left to fetch or read
            if (j < nb) mfma(f0a, f0b);
        }
        int rloc = 128 * wr + 4 * h, cloc = BC * wc + r32;
        asm volatile("" : "+v"(rloc), "+v"(cloc));
        if (slot >= 0) {
            int32_t *dst = part + (size_t)slot * kPairBlock * kPairBlock;
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < NB; ++b)
#pragma unroll
                    for (int v = 0; v < 16; ++v)
                        dst[(rloc + 32 * a + (v & 3) + 8 * (v >> 2)) * kPairBlock + cloc + 32 * b] = (int)acc[a][b][v];
        } else {
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    const int col = J0 + cloc + 32 * b;
#pragma unroll
                    for (int v = 0; v < 16; ++v) {
                        const int row = I0 + rloc + 32 * a + (v & 3) + 8 * (v >> 2);
                        if (row < n && col < n) {
                            int64_t *o = pairs + (uint64_t)row * n + col;
                            const int64_t val = (int64_t)acc[a][b][v];
                            *o = overwrite ? val : *o + val;
                        }
                    }
                }
        }
    }
}

// Sums the k-pieces of the pooled leftover items of pair_fp4_tile_kernel (piece q of leftover item l
// in partial slot l * sp + q) into the int64 output: block (row, l) = row `row` of leftover item l.
__global__ __launch_bounds__(kPairBlock) void pair_reduce2_kernel(const int32_t *__restrict__ part, int n, PairMap M,
                                                                 int64_t *__restrict__ pairs, int overwrite) {
    const int l = (int)blockIdx.y, sp = M.pieces(M.leftovers());
    int bi, bj, c0;
    M.item_at(M.leftover_tile(l), bi, bj, c0);
    const int r = (int)blockIdx.x, c = (int)threadIdx.x;
    const int row = bi * kPairBlock + r, col = bj * kPairBlock + c0 + c;
    if (c >= kPairBlock / M.halves || row >= n || col >= n) return;
    const int32_t *p = part + (size_t)(l * sp) * kPairBlock * kPairBlock + r * kPairBlock + c;
    int64_t acc = 0;
    for (int q = 0; q < sp; ++q) acc += p[(size_t)q * kPairBlock * kPairBlock];
    int64_t *o = pairs + (uint64_t)row * n + col;
    *o = overwrite ? acc : *o + acc;
}

// ------------------------------------------------------------------------------------------
// Distinct panels
// ------------------------------------------------------------------------------------------
// Segmented input (the owner side of the multi-GPU exchange): entry i is valid iff
// i % seg_cap < seg_counts[i / seg_cap]; without seg_counts every entry is.
__device__ __forceinline__ bool uq_valid(uint64_t i, uint32_t seg_cap, const uint64_t *seg_counts) {
    if (!seg_counts) return true;
    const uint32_t s = (uint32_t)i / seg_cap;
    return (uint64_t)((uint32_t)i - s * seg_cap) < seg_counts[s];
}

// one thread per panel: open addressing on `panel index + 1`, keyed by the 128-bit hash, exact
// bitmask comparison on a hash match (small batches; the XMIN portfolio table)
// With rep (the exchange's local distinct set beyond the partitioned path's size): the index of every
// inserted (first-seen) panel goes to rep[], one rep_count atomic per wave.
__global__ void unique_kernel(const uint64_t *__restrict__ hashes, const uint64_t *__restrict__ panels,
                              uint64_t S, int W, unsigned long long *__restrict__ table,
                              uint64_t mask, unsigned long long *__restrict__ unique, uint32_t seg_cap,
                              const uint64_t *__restrict__ seg_counts, uint32_t *__restrict__ rep,
                              unsigned long long *__restrict__ rep_count) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool inserted = false;
    if (i < S && uq_valid(i, seg_cap, seg_counts)) {
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
                for (int w = 0; w < W && same; ++w) same = panels[i * W + w] == panels[j * W + w];
                if (same) break;
            }
            slot = (slot + 1) & mask;
        }
    }
    const uint64_t b = __ballot(inserted);
    if (unique && (threadIdx.x & 63) == 0 && b) atomicAdd(unique, (unsigned long long)__popcll(b));
    if (rep) {
        unsigned long long base = 0;
        if ((threadIdx.x & 63) == 0 && b) base = atomicAdd(rep_count, (unsigned long long)__popcll(b));
        base = __shfl(base, 0);
        if (inserted) rep[base + __popcll(b & ((1ull << (threadIdx.x & 63)) - 1ull))] = (uint32_t)i;
    }
}

// ---- partitioned distinct count (no global atomics per panel) -----------------------------
// unique_kernel's per-panel CAS runs at the memory side (MI355X global atomics are not performed
// in L2), ~0.22 ms per 10^6 panels.  For large batches the hashes are instead partitioned by
// their top bits (counting pass -> scans -> scatter, per-workgroup LDS histograms, plain stores)
// and each partition (<= ~1.5k panels on average) is deduplicated in an LDS hash table by one
// workgroup, with the same exact rule: equal 128-bit hashes AND equal bitmasks.
constexpr int kUqThreads = 256;
constexpr int kUqMaxParts = 8192;
constexpr int kUqTable = 8192;  // LDS slots per partition table (u32 panel index + 1)

__device__ __forceinline__ uint32_t uq_part(uint64_t h1, int pbits) { return (uint32_t)(h1 >> (64 - pbits)); }

__global__ __launch_bounds__(kUqThreads) void uq_count_kernel(const uint64_t *__restrict__ hashes, uint64_t S,
                                                              uint64_t CH, int pbits, uint32_t nwg,
                                                              uint32_t *__restrict__ hist, uint32_t seg_cap,
                                                              const uint64_t *__restrict__ seg_counts) {
    __shared__ uint32_t h[kUqMaxParts];
    const uint32_t P = 1u << pbits;
    for (uint32_t p = threadIdx.x; p < P; p += blockDim.x) h[p] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * CH, b1 = min(S, b0 + CH);
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x)
        if (uq_valid(i, seg_cap, seg_counts)) atomicAdd(&h[uq_part(hashes[2 * i], pbits)], 1u);
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < P; p += blockDim.x) hist[(uint64_t)p * nwg + blockIdx.x] = h[p];
}

// exclusive scan of one partition's per-workgroup counts (in place); tot[p] = the partition's size
__global__ __launch_bounds__(kUqThreads) void uq_scan_part_kernel(uint32_t *__restrict__ hist, uint32_t nwg,
                                                                  uint32_t *__restrict__ tot) {
    __shared__ uint32_t part_sum[kUqThreads];
    uint32_t *row = hist + (uint64_t)blockIdx.x * nwg;
    const uint32_t per = (nwg + kUqThreads - 1) / kUqThreads, a = threadIdx.x * per, b = min(nwg, a + per);
    uint32_t sum = 0;
    for (uint32_t k = a; k < b; ++k) sum += row[k];
    part_sum[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int t = 0; t < kUqThreads; ++t) {
            const uint32_t v = part_sum[t];
            part_sum[t] = acc;
            acc += v;
        }
        tot[blockIdx.x] = acc;
    }
    __syncthreads();
    uint32_t acc = part_sum[threadIdx.x];
    for (uint32_t k = a; k < b; ++k) {
        const uint32_t v = row[k];
        row[k] = acc;
        acc += v;
    }
}

// exclusive scan of the partition sizes -> partition bases (P + 1 entries)
__global__ __launch_bounds__(1024) void uq_scan_tot_kernel(const uint32_t *__restrict__ tot, uint32_t P,
                                                           uint32_t *__restrict__ base) {
    __shared__ uint32_t part_sum[1024];
    const uint32_t per = (P + 1023) / 1024, a = threadIdx.x * per, b = min(P, a + per);
    uint32_t sum = 0;
    for (uint32_t k = a; k < b; ++k) sum += tot[k];
    part_sum[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int t = 0; t < 1024; ++t) {
            const uint32_t v = part_sum[t];
            part_sum[t] = acc;
            acc += v;
        }
        base[P] = acc;
    }
    __syncthreads();
    uint32_t acc = part_sum[threadIdx.x];
    for (uint32_t k = a; k < b; ++k) {
        base[k] = acc;
        acc += tot[k];
    }
}

__global__ __launch_bounds__(kUqThreads) void uq_scatter_kernel(const uint64_t *__restrict__ hashes, uint64_t S,
                                                                uint64_t CH, int pbits, uint32_t nwg,
                                                                const uint32_t *__restrict__ hist,
                                                                const uint32_t *__restrict__ base,
                                                                uint32_t *__restrict__ idx, uint32_t seg_cap,
                                                                const uint64_t *__restrict__ seg_counts) {
    __shared__ uint32_t ctr[kUqMaxParts];
    const uint32_t P = 1u << pbits;
    for (uint32_t p = threadIdx.x; p < P; p += blockDim.x) ctr[p] = base[p] + hist[(uint64_t)p * nwg + blockIdx.x];
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * CH, b1 = min(S, b0 + CH);
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x)
        if (uq_valid(i, seg_cap, seg_counts)) idx[atomicAdd(&ctr[uq_part(hashes[2 * i], pbits)], 1u)] = (uint32_t)i;
}

// one workgroup per partition: exact dedupe in an LDS table of panel indices
__global__ __launch_bounds__(kUqThreads) void uq_dedupe_kernel(const uint64_t *__restrict__ hashes,
                                                               const uint64_t *__restrict__ panels, int W,
                                                               const uint32_t *__restrict__ idx,
                                                               const uint32_t *__restrict__ base,
                                                               unsigned long long *__restrict__ unique,
                                                               uint32_t *__restrict__ status,
                                                               uint32_t *__restrict__ rep,
                                                               unsigned long long *__restrict__ rep_count) {
    __shared__ uint32_t T[kUqTable];
    __shared__ uint32_t cnt, rbase, rpos;
    for (int t = threadIdx.x; t < kUqTable; t += blockDim.x) T[t] = 0;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const uint32_t b0 = base[blockIdx.x], b1 = base[blockIdx.x + 1];
    uint32_t mine = 0;
    for (uint32_t e = b0 + threadIdx.x; e < b1; e += blockDim.x) {
        const uint32_t i = idx[e];
        const uint64_t h1 = hashes[2 * (uint64_t)i], h2 = hashes[2 * (uint64_t)i + 1];
        uint32_t slot = (uint32_t)(h1 ^ (h2 >> 29)) & (kUqTable - 1);
        bool done = false;
        for (int probe = 0; probe < kUqTable && !done; ++probe) {
            const uint32_t v = atomicCAS(&T[slot], 0u, i + 1);
            if (v == 0u) {
                ++mine;
                done = true;
            } else {
                const uint64_t j = v - 1;
                if (hashes[2 * j] == h1 && hashes[2 * j + 1] == h2) {
                    bool same = true;
                    for (int w = 0; w < W && same; ++w) same = panels[(uint64_t)i * W + w] == panels[j * W + w];
                    done = same;
                }
                slot = (slot + 1) & (kUqTable - 1);
            }
        }
        // a full table (more than kUqTable distinct panels in one partition; csa_unique_async
        // sizes partitions at <= 2048 on average) fails the call through the status block
        if (!done) raise_status(status, CSA_E_UNSUPPORTED, 0xFFFFFFFFFFFFFFFFull);
    }
    atomicAdd(&cnt, mine);
    __syncthreads();
    if (threadIdx.x == 0 && cnt && unique) atomicAdd(unique, (unsigned long long)cnt);
    if (rep) {  // the partition's distinct panels (its table entries) -> rep[], one global atomic per workgroup
        if (threadIdx.x == 0) {
            rbase = cnt ? (uint32_t)atomicAdd(rep_count, (unsigned long long)cnt) : 0u;
            rpos = 0;
        }
        __syncthreads();
        for (int t = threadIdx.x; t < kUqTable; t += blockDim.x)
            if (T[t]) rep[rbase + atomicAdd(&rpos, 1u)] = T[t] - 1u;
    }
}

// Portfolio membership of drawn panels (xmin.py:468-469: `panel not in portfolio`): probe the
// portfolio table built by unique_kernel (slots hold portfolio index + 1) with each drawn panel's
// hash and compare full bitmasks on a hash match; the lowest non-member index wins (atomicMin).
__global__ void member_scan_kernel(const uint64_t *__restrict__ hashes, const uint64_t *__restrict__ panels,
                                   uint64_t S, int W, const unsigned long long *__restrict__ table, uint64_t mask,
                                   const uint64_t *__restrict__ port_hashes, const uint64_t *__restrict__ port_panels,
                                   unsigned long long *__restrict__ first) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    const uint64_t h1 = hashes[2 * i], h2 = hashes[2 * i + 1];
    uint64_t slot = (h1 ^ (h2 >> 29)) & mask;
    for (uint64_t probe = 0; probe <= mask; ++probe) {
        const unsigned long long v = table[slot];
        if (v == 0ull) break;  // empty slot: not a member
        const uint64_t j = v - 1;
        if (port_hashes[2 * j] == h1 && port_hashes[2 * j + 1] == h2) {
            bool same = true;
            for (int w = 0; w < W && same; ++w) same = panels[i * W + w] == port_panels[j * W + w];
            if (same) return;  // member
        }
        slot = (slot + 1) & mask;
    }
    atomicMin(first, (unsigned long long)i);
}

// Histogram of the pair counts i < j (the values plot_pair_probability_distribution_per_algorithm
// sorts, analysis.py:339-342): one workgroup per row i, coalesced reads of pairs[i][i+1..n),
// one 64-bit atomic per entry into hist[value] (value < n_bins is guaranteed by the caller:
// n_bins > max per-person count >= every pair count).  Values >= n_bins are counted in *overflow.
__global__ __launch_bounds__(256) void pair_histogram_kernel(const int64_t *__restrict__ pairs, int n,
                                                             unsigned long long *__restrict__ hist, uint64_t n_bins,
                                                             unsigned long long *__restrict__ overflow) {
    const int i = blockIdx.x;
    const int64_t *row = pairs + (size_t)i * n;
    for (int j = i + 1 + (int)threadIdx.x; j < n; j += blockDim.x) {
        const uint64_t v = (uint64_t)row[j];
        if (v < n_bins)
            atomicAdd(hist + v, 1ull);
        else
            atomicAdd(overflow, 1ull);
    }
}

// Multi-GPU distinct-panel exchange, send side (owner = h1 % world): the
// local distinct panels (rep[0 .. *rep_count), from the partitioned dedupe) go into fixed-capacity
// segments of send_hashes / send_panels, one segment per owner rank, so the all_to_all has equal
// splits and the host never reads a size.  send_counts[w] (zeroed by the caller) = entries reserved in
// segment w; a segment past its capacity raises CSA_E_UNSUPPORTED (kExchangeOverflow) in the status
// block.  Per workgroup: LDS histogram per owner, one global atomic per (workgroup, owner) to reserve
// ranges, the hashes, then the panel rows copied cooperatively (W contiguous words per row).
constexpr int kMaxWorld = 1024;
constexpr int kXbThreads = 256;
constexpr uint64_t kExchangeOverflow = 0xFFFFFFFFFFFFFFFEull;  // status "panel" of a full segment
__global__ __launch_bounds__(kXbThreads) void exchange_bucket_kernel(
    const uint64_t *__restrict__ hashes, const uint64_t *__restrict__ panels, int W, const uint32_t *__restrict__ rep,
    const unsigned long long *__restrict__ rep_count, uint32_t world, uint64_t capacity,
    uint64_t *__restrict__ send_hashes, uint64_t *__restrict__ send_panels,
    unsigned long long *__restrict__ send_counts, uint32_t *__restrict__ status) {
    __shared__ uint32_t hist[kMaxWorld];
    __shared__ unsigned long long rbase[kMaxWorld];
    __shared__ uint32_t src_row[kXbThreads];
    __shared__ uint64_t dst_row[kXbThreads];
    const uint64_t m = *rep_count;
    const uint64_t e0 = (uint64_t)blockIdx.x * kXbThreads;
    if (e0 >= m) return;  // whole workgroup
    for (uint32_t w = threadIdx.x; w < world; w += blockDim.x) hist[w] = 0;
    __syncthreads();
    const uint64_t e = e0 + threadIdx.x;
    const bool valid = e < m;
    uint32_t i = 0, owner = 0, local = 0;
    uint64_t h1 = 0, h2 = 0;
    if (valid) {
        i = rep[e];
        h1 = hashes[2 * (uint64_t)i];
        h2 = hashes[2 * (uint64_t)i + 1];
        owner = (uint32_t)(h1 % world);
        local = atomicAdd(&hist[owner], 1u);
    }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < world; w += blockDim.x)
        rbase[w] = hist[w] ? atomicAdd(&send_counts[w], (unsigned long long)hist[w]) : 0ull;
    __syncthreads();
    uint64_t dst = ~0ull;
    if (valid) {
        const uint64_t pos = rbase[owner] + local;
        if (pos < capacity) {
            dst = (uint64_t)owner * capacity + pos;
            send_hashes[2 * dst] = h1;
            send_hashes[2 * dst + 1] = h2;
        } else {
            raise_status(status, CSA_E_UNSUPPORTED, kExchangeOverflow);
        }
    }
    src_row[threadIdx.x] = i;
    dst_row[threadIdx.x] = dst;
    __syncthreads();
    const uint32_t rows = (uint32_t)min<uint64_t>(kXbThreads, m - e0);
    for (uint32_t t = threadIdx.x; t < rows * (uint32_t)W; t += blockDim.x) {
        const uint32_t r = t / (uint32_t)W, w = t - r * (uint32_t)W;
        const uint64_t d = dst_row[r];
        if (d != ~0ull) send_panels[d * W + w] = panels[(uint64_t)src_row[r] * W + w];
    }
}

// ---- the 24-byte exchange (keys instead of bitmasks) ---------------------------------------
// A panel is a pure function of (seed, global panel index) in the Philox stream, so a rank sends,
// per local distinct panel, its 128-bit hash and global index (24 B instead of 16 + 8W B); the
// owner counts distinct hashes and re-draws only the entries whose hash matched an earlier one
// (their bitmasks decide: a duplicate, or -- never seen in practice -- a 128-bit collision, whose
// mismatched members are then counted exactly by bitmask).
__global__ __launch_bounds__(kXbThreads) void exchange_keys_kernel(
    const uint64_t *__restrict__ hashes, const uint32_t *__restrict__ rep, const unsigned long long *__restrict__ rep_count,
    uint64_t panel_begin, uint32_t world, uint64_t capacity, uint64_t *__restrict__ send_keys,
    unsigned long long *__restrict__ send_counts, uint32_t *__restrict__ status) {
    __shared__ uint32_t hist[kMaxWorld];
    __shared__ unsigned long long rbase[kMaxWorld];
    const uint64_t m = *rep_count;
    const uint64_t e0 = (uint64_t)blockIdx.x * kXbThreads;
    if (e0 >= m) return;  // whole workgroup
    for (uint32_t w = threadIdx.x; w < world; w += blockDim.x) hist[w] = 0;
    __syncthreads();
    const uint64_t e = e0 + threadIdx.x;
    const bool valid = e < m;
    uint32_t i = 0, owner = 0, local = 0;
    uint64_t h1 = 0, h2 = 0;
    if (valid) {
        i = rep[e];
        h1 = hashes[2 * (uint64_t)i];
        h2 = hashes[2 * (uint64_t)i + 1];
        owner = (uint32_t)(h1 % world);
        local = atomicAdd(&hist[owner], 1u);
    }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < world; w += blockDim.x)
        rbase[w] = hist[w] ? atomicAdd(&send_counts[w], (unsigned long long)hist[w]) : 0ull;
    __syncthreads();
    if (valid) {
        const uint64_t pos = rbase[owner] + local;
        if (pos < capacity) {
            uint64_t *d = send_keys + 3 * ((uint64_t)owner * capacity + pos);
            d[0] = h1;
            d[1] = h2;
            d[2] = panel_begin + i;
        } else {
            raise_status(status, CSA_E_UNSUPPORTED, kExchangeOverflow);
        }
    }
}

// Owner, pass 1: distinct 128-bit hashes among the valid entries of the segmented keys (entry e
// valid iff e % seg_cap < seg_counts[e / seg_cap]); an entry whose hash equals an earlier-inserted
// entry's goes to the re-draw list as the pair (its panel index, that entry's panel index).
__global__ void key_unique_kernel(const uint64_t *__restrict__ keys, uint64_t total, uint32_t seg_cap,
                                  const uint64_t *__restrict__ seg_counts, unsigned long long *__restrict__ table,
                                  uint64_t mask, unsigned long long *__restrict__ unique, uint64_t *__restrict__ list,
                                  unsigned long long *__restrict__ list_len, uint64_t list_cap,
                                  uint32_t *__restrict__ status) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool inserted = false;
    if (e < total && uq_valid(e, seg_cap, seg_counts)) {
        const uint64_t h1 = keys[3 * e], h2 = keys[3 * e + 1];
        uint64_t slot = (h1 ^ (h2 >> 29)) & mask;
        for (uint64_t probe = 0; probe <= mask; ++probe) {
            const unsigned long long v = atomicCAS(table + slot, 0ull, (unsigned long long)(e + 1));
            if (v == 0ull) {
                inserted = true;
                break;
            }
            const uint64_t j = v - 1;
            if (keys[3 * j] == h1 && keys[3 * j + 1] == h2) {  // same hash: re-draw both to compare
                const unsigned long long c = atomicAdd(list_len, 2ull);
                if (c + 2 <= 2 * list_cap) {
                    list[c] = keys[3 * e + 2];
                    list[c + 1] = keys[3 * j + 2];
                } else {
                    raise_status(status, CSA_E_UNSUPPORTED, kExchangeOverflow);
                }
                break;
            }
            slot = (slot + 1) & mask;
        }
    }
    const uint64_t b = __ballot(inserted);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(unique, (unsigned long long)__popcll(b));
}

// Owner, pass 2 (after the re-draw of the list into rows): a candidate whose bitmask differs from
// its hash partner's is a different panel behind a 128-bit hash collision; those are counted
// exactly among themselves (table2, keyed by their own hash, bitmask comparison).
__global__ void key_verify_kernel(const uint64_t *__restrict__ rows, int W, const unsigned long long *__restrict__ list_len,
                                  unsigned long long *__restrict__ table2, uint64_t mask2,
                                  unsigned long long *__restrict__ unique) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool added = false;
    if (2 * c < *list_len) {
        const uint64_t *x = rows + 2 * c * (uint64_t)W, *y = x + W;
        bool same = true;
        for (int w = 0; w < W && same; ++w) same = x[w] == y[w];
        if (!same) {
            uint64_t h1 = 0, h2 = 0;
            for (int w = 0; w < W; ++w) {
                h1 += fmix_a(x[w] ^ ((uint64_t)w * 0x9E3779B97F4A7C15ull));
                h2 += fmix_b(x[w] + ((uint64_t)w + 1) * 0xD6E8FEB86659FD93ull);
            }
            uint64_t slot = (h1 ^ (h2 >> 29)) & mask2;
            for (uint64_t probe = 0; probe <= mask2; ++probe) {
                const unsigned long long v = atomicCAS(table2 + slot, 0ull, (unsigned long long)(c + 1));
                if (v == 0ull) {
                    added = true;
                    break;
                }
                const uint64_t *z = rows + 2 * (v - 1) * (uint64_t)W;
                bool eq = true;
                for (int w = 0; w < W && eq; ++w) eq = x[w] == z[w];
                if (eq) break;
                slot = (slot + 1) & mask2;
            }
        }
    }
    const uint64_t b = __ballot(added);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(unique, (unsigned long long)__popcll(b));
}

// Multi-GPU pair exchange: the upper triangle (incl. the diagonal) of the n x n int64 pair counts
// packed row-major into int32 (valid while every count < 2^31), so the all-reduce moves n(n+1)/2
// words of 4 B instead of n^2 of 8 B (6 MB instead of 24 MB at sf_e); unpack writes them back.
__device__ __forceinline__ uint64_t tri_offset(int i, int n) { return (uint64_t)i * n - (uint64_t)i * (i - 1) / 2; }
// dst[i] += src[i] (csa_legacy_sample_devices: shard counts / pairs summed on shard 0's device)
__global__ __launch_bounds__(256) void add_i64_kernel(int64_t *__restrict__ dst, const int64_t *__restrict__ src,
                                                      uint64_t m) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256ull) dst[i] += src[i];
}

__global__ __launch_bounds__(256) void pairs_pack_kernel(const int64_t *__restrict__ pairs, int n,
                                                         int32_t *__restrict__ packed) {
    const int i = blockIdx.x;
    const uint64_t off = tri_offset(i, n);
    for (int j = i + (int)threadIdx.x; j < n; j += blockDim.x) packed[off + (j - i)] = (int32_t)pairs[(uint64_t)i * n + j];
}
__global__ __launch_bounds__(256) void pairs_unpack_kernel(const int32_t *__restrict__ packed, int n,
                                                           int64_t *__restrict__ pairs) {
    const int i = blockIdx.x;
    const uint64_t off = tri_offset(i, n);
    for (int j = i + (int)threadIdx.x; j < n; j += blockDim.x) pairs[(uint64_t)i * n + j] = packed[off + (j - i)];
}

// per-person counts = the pair matrix's diagonal (sum over panels of x_i^2 = x_i): csa_pairs_diag_async,
// the counts of a draw whose XT came from the draw kernel (csa_draw_xt_async) instead of
// csa_transpose_count_async
__global__ __launch_bounds__(256) void pairs_diag_kernel(const int64_t *__restrict__ pairs, int n,
                                                         int64_t *__restrict__ counts) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) counts[i] = pairs[(size_t)i * n + i];
}

// PairHistogram materialisation (analysis.py:86-98): the STRICT upper triangle (i < j, the reference's
// key order, analysis.py:70) of the n x n int64 pair counts packed row-major -- as int64 counts, or as
// float64 count / divisor (IEEE division, correctly rounded: the value Python's int / int gives, as
// turn_into_probabilities_by_dividing_all_elements_by_given_number divides).  Row i starts at
// i (n - 1) - i (i - 1) / 2.  One workgroup per row, coalesced reads and writes; HBM-bound.
template <bool DIV>
__global__ __launch_bounds__(256) void pairs_upper_kernel(const int64_t *__restrict__ pairs, int n, double divisor,
                                                          void *__restrict__ out) {
    const int i = blockIdx.x;
    const uint64_t off = (uint64_t)i * (n - 1) - (uint64_t)i * (i - 1) / 2 - (uint64_t)(i + 1);
    const int64_t *row = pairs + (uint64_t)i * n;
    for (int j = i + 1 + (int)threadIdx.x; j < n; j += blockDim.x) {
        if constexpr (DIV) static_cast<double *>(out)[off + j] = (double)row[j] / divisor;
        else static_cast<int64_t *>(out)[off + j] = row[j];
    }
}

// Small-range variant (n_bins <= kHistLdsBins): per-workgroup LDS histogram over a stride of
// rows (u32 LDS atomics), flushed with one global atomic per non-zero bin -- few distinct values
// (n = 8192, S = 2e4: ~700 bins for 33.5 M pairs) would otherwise serialise on global atomics.
constexpr int kHistLdsBins = 16384;
__global__ __launch_bounds__(256) void pair_histogram_lds_kernel(const int64_t *__restrict__ pairs, int n,
                                                                 unsigned long long *__restrict__ hist,
                                                                 uint64_t n_bins,
                                                                 unsigned long long *__restrict__ overflow) {
    __shared__ uint32_t h[kHistLdsBins];
    __shared__ uint32_t over_s;
    for (int b = threadIdx.x; b < (int)n_bins; b += blockDim.x) h[b] = 0;
    if (threadIdx.x == 0) over_s = 0;
    __syncthreads();
    for (int i = blockIdx.x; i < n - 1; i += gridDim.x) {
        const int64_t *row = pairs + (size_t)i * n;
        for (int j = i + 1 + (int)threadIdx.x; j < n; j += blockDim.x) {
            const uint64_t v = (uint64_t)row[j];
            if (v < n_bins)
                atomicAdd(&h[v], 1u);
            else
                atomicAdd(&over_s, 1u);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < (int)n_bins; b += blockDim.x)
        if (h[b]) atomicAdd(hist + b, (unsigned long long)h[b]);
    if (threadIdx.x == 0 && over_s) atomicAdd(overflow, (unsigned long long)over_s);
}

}  // namespace

// library-internal: lets legacy_mt.cpp set the csa_last_error() message
void csa_set_last_error(const char *msg) { g_err = msg ? msg : ""; }

// ==========================================================================================
// Host side
// ==========================================================================================
struct csa_instance {
    int32_t n = 0, C = 0, F = 0, W = 0, Ws = 0;
    int device = 0;
    std::vector<int32_t> pf, fmin, fmax, fcat, pool;
    std::vector<int32_t> sel0;  // host copy of the initial "selected" counters (csa_instance_set_state)
    std::vector<uint64_t> featmask;  // F x Ws
    uint64_t *d_featmask = nullptr;
    int32_t *d_fmin = nullptr, *d_fmax = nullptr, *d_sel0 = nullptr, *d_rem0 = nullptr;
    uint64_t *d_present0 = nullptr;
    uint32_t *d_pmask = nullptr;  // n person feature masks (F <= 32 only)
    int32_t *d_addr_next = nullptr;  // same-address rings (csa_instance_set_address) or null
    int32_t max_abs = 0;  // max |fmin| / |sel0| bound for the cross-multiplication range check
    bool zero_max_min = false;  // some feature has max 0 and min > 0 (draw_batch_kernel excludes it)
    // some feature starts with selected >= max > 0: the lane / wide kernels test "selected == max" as
    // need < min - max + 1 (true past max too), so such start states take draw_kernel (exact ==)
    bool sel_over_max = false;
    int32_t max_slack = 0;      // max over live features of max - selected (draw_lane_kernel: <= 255)
    // every live feature's need = min - selected stays in [-127, 127] from the start state on (need
    // only falls, to min - max at worst): draw_lane_kernel's 8-bit need keys (CSA_LANE_KEY8)
    bool need8 = true;
    // grow-only device scratch + a stream for the repeated small host-API calls
    // (csa_first_panel_not_in: XMIN calls it 5n times)
    void *scratch[32] = {};   // slots 0-7: csa_first_panel_not_in; 8-19: csa_legacy_sample; 20-29: _devices
    size_t scratch_bytes[32] = {};
    hipStream_t stream = nullptr;
    hipStream_t sdraw = nullptr, spost = nullptr;  // csa_legacy_sample's pipeline
    hipEvent_t drawn = nullptr;
    // draw_lane_kernel's pick lists (u16, n_panels x k), reused across draws (lane_picks)
    uint16_t *d_picks16 = nullptr;
    size_t picks_bytes = 0;
    hipEvent_t picks_done = nullptr;
    bool picks_pending = false;
    // host copies of the draw state (empty = default) and address rings, bumped generation `gen`
    // on every set: csa_legacy_sample_devices' per-shard replicas re-mirror them when it changes
    std::vector<int32_t> rem0h, addr_h;
    std::vector<uint64_t> present0h;
    uint64_t gen = 1;
    std::vector<csa_instance *> replicas;  // [shard] (null: the instance itself / not created)
    std::vector<uint64_t> replica_gen;
    // draw statistics (csa_instance_draw_stats): device counters of SelectionError restarts and
    // min-quota rejections (DrawArgs::stats), host tally of the panels the batch draws accepted
    unsigned long long *d_stats = nullptr;
    uint64_t panels_drawn = 0;
};

namespace {

template <typename T>
int dalloc(T **p, size_t count) {
    HIPCHK(hipMalloc(reinterpret_cast<void **>(p), std::max<size_t>(count, 1) * sizeof(T)));
    return CSA_OK;
}

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

void update_need8(csa_instance *I) {
    I->need8 = true;
    for (int f = 0; f < I->F; ++f) {
        if (I->fmax[f] == 0) continue;  // dead (min = max = 0) or routed elsewhere (max = 0 < min)
        const int32_t hi = I->fmin[f] - I->sel0[f], lo = I->fmin[f] - I->fmax[f];
        if (hi > 127 || lo < -127) I->need8 = false;
    }
}

int check_k(const csa_instance *I, int32_t k) {
    if (k < 0) return fail(CSA_E_INVALID, "k must be >= 0 (got %d)", k);
    // need*den must stay inside int32 (need = fmin - sel, |need| <= max_abs + k, den <= n)
    const int64_t bound = (int64_t)(I->max_abs + k + 1) * (I->n + 1) * 100;
    if (bound >= (int64_t)1 << 31)
        return fail(CSA_E_UNSUPPORTED, "k=%d with n=%d exceeds the int32 ratio range", k, I->n);
    return CSA_OK;
}

struct DrawConfig {
    int G = 16, FPL = 1, WPL = 1;
    bool lane = false;  // draw_lane_kernel (2 lanes per panel): FPL / WPL hold its FN / WN
    bool wide = false;  // draw_wide_kernel (8 lanes per panel)
    bool solo = false;  // draw_solo_kernel (1 lane per panel): FPL / WPL hold its FN / WN
    bool k8 = false;    // lane / solo: the 8-bit need keys carrying their index (csa_instance::need8)
    const void *fn = nullptr;
    bool picks() const { return lane || wide || solo; }  // pick-list kernels (picks_pack_kernel builds the panels)
};

template <int FPL>
const void *wide_fn_w(int wpl) {
    switch (wpl) {
        case 4: return reinterpret_cast<const void *>(&draw_wide_kernel<8, FPL, 4>);
        case 8: return reinterpret_cast<const void *>(&draw_wide_kernel<8, FPL, 8>);
        case 16: return reinterpret_cast<const void *>(&draw_wide_kernel<8, FPL, 16>);
        default: return nullptr;
    }
}

const void *wide_fn(int fpl, int wpl) {
    switch (fpl) {
        case 2: return wide_fn_w<2>(wpl);
        case 4: return wide_fn_w<4>(wpl);
        case 5: return wide_fn_w<5>(wpl);
        case 8: return wide_fn_w<8>(wpl);
        default: return nullptr;
    }
}

// holder-scan batch of the lane kernel: all of a lane's row words in one LDS round trip
// (CSA_LANE_SKDIV > 1 splits them, trading a round trip for VGPRs)
#ifndef CSA_LANE_SKDIV
#define CSA_LANE_SKDIV 1
#endif
template <int FN, int WN, bool K8>
const void *lane_fn_wn() {
    constexpr int SK = (WN / 2 + CSA_LANE_SKDIV - 1) / CSA_LANE_SKDIV;
    return reinterpret_cast<const void *>(&draw_lane_kernel<FN, WN, SK, K8>);
}

template <int FN, bool K8>
const void *lane_fn_w(int wn) {
    switch (wn) {
        case 4: return lane_fn_wn<FN, 4, K8>();
        case 8: return lane_fn_wn<FN, 8, K8>();
        case 16: return lane_fn_wn<FN, 16, K8>();
        case 28: return lane_fn_wn<FN, 28, K8>();
        case 32: return lane_fn_wn<FN, 32, K8>();
        default: return nullptr;
    }
}

template <int FN, bool K8>
const void *solo_fn_w(int wn) {
    switch (wn) {
        case 4: return reinterpret_cast<const void *>(&draw_solo_kernel<FN, 4, K8>);
        case 8: return reinterpret_cast<const void *>(&draw_solo_kernel<FN, 8, K8>);
        case 16: return reinterpret_cast<const void *>(&draw_solo_kernel<FN, 16, K8>);
        case 28: return reinterpret_cast<const void *>(&draw_solo_kernel<FN, 28, K8>);
        case 32: return reinterpret_cast<const void *>(&draw_solo_kernel<FN, 32, K8>);
        default: return nullptr;
    }
}

// k8: the 8-bit need keys with the feature index inside (csa_instance::need8; draw_lane.inc)
const void *solo_fn(int fn_, int wn, bool k8) {
    switch (fn_) {
        case 8: return k8 ? solo_fn_w<8, true>(wn) : solo_fn_w<8, false>(wn);
        case 16: return k8 ? solo_fn_w<16, true>(wn) : solo_fn_w<16, false>(wn);
        default: return nullptr;
    }
}

const void *lane_fn(int fn_, int wn, bool k8) {
    switch (fn_) {
        case 32: return k8 ? lane_fn_w<32, true>(wn) : lane_fn_w<32, false>(wn);
        default: return nullptr;
    }
}

template <int G, int FPL, int WPL, bool GEN>
const void *draw_fn() {
    return reinterpret_cast<const void *>(&draw_kernel<G, FPL, WPL, GEN>);
}

template <int G, int FPL, bool GEN>
const void *draw_fn_w(int wpl) {
    switch (wpl) {
        case 1: return draw_fn<G, FPL, 1, GEN>();
        case 2: return draw_fn<G, FPL, 2, GEN>();
        case 4: return draw_fn<G, FPL, 4, GEN>();
        case 8: if constexpr (G == 16) return draw_fn<G, FPL, 8, GEN>(); else return nullptr;
        case 16: if constexpr (G == 16) return draw_fn<G, FPL, 16, GEN>(); else return nullptr;
        default: return nullptr;
    }
}

template <int G, bool GEN>
const void *draw_fn_fw(int fpl, int wpl) {
    switch (fpl) {
        case 1: return draw_fn_w<G, 1, GEN>(wpl);
        case 2: return draw_fn_w<G, 2, GEN>(wpl);
        case 4: return draw_fn_w<G, 4, GEN>(wpl);
        default: return nullptr;
    }
}

int pow2_ceil_int(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

// Batch draws: draw_solo_kernel (1 lane per panel) or draw_lane_kernel (2 lanes per panel, 32
// panels per wavefront) when the instance fits -- F <= 32, W <= 32, no max = 0 < min feature, |min|, |selected| < 2^15 (16-bit packed
// need / remaining) and no feature starting above max ("selected == max" is tested as
// need <= min - max) -- else draw_kernel with G = 16 (F <= 64, W <= 256) or 64.  Pick-order /
// single-attempt draws (general mode) use draw_kernel<64, ..., true>.  CSA_DRAW_KERNEL=solo|lane|wide|16|64
// forces a batch kernel the instance fits (parity tests of every layout).
int pick_draw_config(const csa_instance *I, bool general, DrawConfig &c) {
    general = general || I->d_addr_next;  // same-address deletions: draw_kernel<64, ..., true> only
    const bool reg_ok = I->F <= 32 && I->d_pmask && !I->zero_max_min && I->W <= 32 && I->max_abs < 32768 &&
                        !I->sel_over_max && I->max_slack <= 255;
    const bool lane_ok = reg_ok && I->F > 16;  // built for FN = 32 only
    const bool wide_ok = I->F <= 64 && I->W <= 128 && !I->zero_max_min && I->max_abs < 32768 && !I->sel_over_max;
    const bool g16_ok = I->F <= 64 && I->W <= 256;
    // one lane per panel when a lane holds few features (F <= 16: 142 VGPRs at W = 32, 3 waves/SIMD;
    // example_large_200 281 vs 252 M panels/s, example_small_20 2950 vs 2490); at F = 32 the state needs
    // 165 VGPRs and the two-lane kernel's 4 waves/SIMD win (sf_e 262 vs 247)
    const bool solo_ok = reg_ok && I->F <= 16;
    int choice = general ? 64 : solo_ok ? 1 : lane_ok ? 2 : wide_ok ? 8 : g16_ok ? 16 : 64;
    if (const char *e = getenv("CSA_DRAW_KERNEL")) {
        // the register kernels are built for the shapes they win on only (solo F <= 16, lane F > 16)
        if (!general && !strcmp(e, "solo") && solo_ok) choice = 1;
        else if (!general && !strcmp(e, "lane") && lane_ok && !solo_ok) choice = 2;
        else if (!general && !strcmp(e, "wide") && wide_ok) choice = 8;
        else if (!general && !strcmp(e, "16") && g16_ok) choice = 16;
        else if (!general && !strcmp(e, "64")) choice = 64;
    }
    c.G = choice;
    if (choice == 1) {
        c.solo = true;
        c.FPL = std::max(8, pow2_ceil_int(I->F));
        c.WPL = I->W <= 4 ? 4 : I->W <= 8 ? 8 : I->W <= 16 ? 16 : I->W <= 28 ? 28 : 32;
        c.k8 = I->need8;
        c.fn = solo_fn(c.FPL, c.WPL, c.k8);
        if (!c.fn) return fail(CSA_E_UNSUPPORTED, "no solo draw kernel for F=%d W=%d", I->F, I->W);
        return CSA_OK;
    }
    if (choice == 8) {  // draw_wide_kernel: FPL in {2, 4, 5, 8}, WPL in {4, 8, 16}
        const int fpl = (I->F + 7) / 8;
        c.wide = true;
        c.FPL = fpl <= 2 ? 2 : fpl <= 4 ? 4 : fpl <= 5 ? 5 : 8;
        c.WPL = I->W <= 32 ? 4 : I->W <= 64 ? 8 : 16;
        c.fn = wide_fn(c.FPL, c.WPL);
        if (!c.fn) return fail(CSA_E_UNSUPPORTED, "no wide draw kernel for F=%d W=%d", I->F, I->W);
        return CSA_OK;
    }
    if (choice == 2) {
        c.lane = true;
        c.FPL = std::max(8, pow2_ceil_int(I->F));
        c.WPL = I->W <= 4 ? 4 : I->W <= 8 ? 8 : I->W <= 16 ? 16 : I->W <= 28 ? 28 : 32;
        c.k8 = I->need8;
        c.fn = lane_fn(c.FPL, c.WPL, c.k8);
        if (!c.fn) return fail(CSA_E_UNSUPPORTED, "no lane draw kernel for F=%d W=%d", I->F, I->W);
        return CSA_OK;
    }
    c.FPL = pow2_ceil_int((I->F + c.G - 1) / c.G);
    c.WPL = pow2_ceil_int(std::max(1, (I->W + c.G - 1) / c.G));
    if (general)
        c.fn = draw_fn_fw<64, true>(c.FPL, c.WPL);
    else
        c.fn = c.G == 16 ? draw_fn_fw<16, false>(c.FPL, c.WPL) : draw_fn_fw<64, false>(c.FPL, c.WPL);
    if (!c.fn)
        return fail(CSA_E_UNSUPPORTED, "no draw kernel for F=%d n=%d (G=%d needs FPL=%d WPL=%d)", I->F, I->n, c.G,
                    c.FPL, c.WPL);
    return CSA_OK;
}

// k = 0 (legacy.py:184 loops zero times): every attempt returns the empty panel, accepted iff no
// feature is below its minimum (check_min_cats); otherwise the reference restarts forever.
__global__ void empty_panels_kernel(uint64_t n_panels, uint32_t *attempts, uint32_t *status, uint64_t panel_begin,
                                    int rejected) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_panels) return;
    if (rejected) {
        if (i == 0) raise_status(status, CSA_E_ATTEMPT_LIMIT, panel_begin);
    } else if (attempts) {
        attempts[i] = 1u;
    }
}

// per-instance pick-list scratch of the lane kernel, serialised across calls: a draw on any stream
// waits until the previous draw's picks_pack_kernel has consumed the lists
int lane_picks(csa_instance *I, uint64_t count, hipStream_t st, uint16_t **out) {
    if (!I->picks_done) HIPCHK(hipEventCreateWithFlags(&I->picks_done, hipEventDisableTiming));
    if (I->picks_pending) HIPCHK(hipStreamWaitEvent(st, I->picks_done, 0));
    const size_t bytes = std::max<uint64_t>(count, 1) * sizeof(uint16_t);
    if (I->picks_bytes < bytes) {
        if (I->picks_pending) HIPCHK(hipEventSynchronize(I->picks_done));
        if (I->d_picks16) HIPCHK(hipFree(I->d_picks16));
        I->d_picks16 = nullptr;
        I->picks_bytes = 0;
        HIPCHK(hipMalloc(reinterpret_cast<void **>(&I->d_picks16), bytes));
        I->picks_bytes = bytes;
    }
    *out = I->d_picks16;
    return CSA_OK;
}

int launch_pack(const uint16_t *d_picks, uint64_t n_panels, int k, int W, uint64_t *d_panels, uint64_t *d_hashes,
                hipStream_t stream) {
    if (n_panels == 0) return CSA_OK;
    // panels per wave: the largest power of two <= 64 whose tile (PK x (2W + 1) u32) stays near 8 KB
    const size_t row = (size_t)(2 * W + 1) * 4;
    const int pk = row * 64 <= 8704 ? 64 : row * 32 <= 8704 ? 32 : row * 16 <= 8704 ? 16 : row * 8 <= 8704 ? 8 : 4;
    const int wpb = 4;
    const uint64_t blocks = (n_panels + (uint64_t)pk * wpb - 1) / ((uint64_t)pk * wpb);
    const size_t plds = (size_t)wpb * pk * row;
    const void *fn = pk == 64   ? reinterpret_cast<const void *>(&picks_pack_kernel<64>)
                     : pk == 32 ? reinterpret_cast<const void *>(&picks_pack_kernel<32>)
                     : pk == 16 ? reinterpret_cast<const void *>(&picks_pack_kernel<16>)
                     : pk == 8  ? reinterpret_cast<const void *>(&picks_pack_kernel<8>)
                                : reinterpret_cast<const void *>(&picks_pack_kernel<4>);
    if (plds > 160 * 1024) return fail(CSA_E_UNSUPPORTED, "picks_pack: W=%d too large", W);
    void *args[] = {(void *)&d_picks, &n_panels, &k, &W, &d_panels, &d_hashes};
    HIPCHK(hipLaunchKernel(fn, dim3((unsigned)blocks), dim3(64 * wpb), args, plds, stream));
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

// d_picks_ext: the lane kernel's pick lists go to this caller buffer and are NOT packed (the caller
// runs csa_picks_pack_async); otherwise to the instance scratch, packed here into d_panels
int launch_draw(const csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                uint32_t max_attempts, uint32_t attempt_base, int single, uint64_t *d_panels,
                uint64_t *d_hashes, uint32_t *d_attempts, int32_t *d_picks, uint32_t *d_status,
                int32_t *d_sel_out, int32_t *d_rem_out, uint64_t *d_present_out, hipStream_t stream,
                uint16_t *d_picks_ext = nullptr, const uint64_t *d_panel_list = nullptr,
                const unsigned long long *d_list_len = nullptr, uint32_t *d_xt = nullptr,
                int32_t *xt_written = nullptr, bool count_stats = true) {
    if (xt_written) *xt_written = 0;
    if (d_panel_list) count_stats = false;  // (index-list re-draws are not new panels)
    int rc = check_k(I, k);
    if (rc) return rc;
    if ((!d_panels && !d_picks_ext) || !d_status) return fail(CSA_E_INVALID, "d_panels and d_status are required");
    if (n_panels == 0) return CSA_OK;
    if (k == 0 && !single && !d_sel_out && !d_present_out) {
        int rejected = 0;
        for (int f = 0; f < I->F; ++f) rejected |= I->sel0[f] < I->fmin[f];
        // draw statistics as the kernels keep them: accepted new panels only (an index-list re-draw of
        // the multi-GPU owner passes its list capacity as n_panels and draws no new panel)
        if (!rejected && count_stats) const_cast<csa_instance *>(I)->panels_drawn += n_panels;
        if (!d_panels) {  // pick-list draw of k = 0: nothing to write but the attempts / status
            hipLaunchKernelGGL(empty_panels_kernel, dim3((unsigned)((n_panels + 255) / 256)), dim3(256), 0, stream,
                               n_panels, d_attempts, d_status, panel_begin, rejected);
            HIPCHK(hipGetLastError());
            return CSA_OK;
        }
        HIPCHK(hipMemsetAsync(d_panels, 0, n_panels * I->W * 8, stream));
        hipLaunchKernelGGL(empty_panels_kernel, dim3((unsigned)((n_panels + 255) / 256)), dim3(256), 0, stream,
                           n_panels, d_attempts, d_status, panel_begin, rejected);
        HIPCHK(hipGetLastError());
        if (d_hashes) {
            hipLaunchKernelGGL(panel_hash_kernel, dim3((unsigned)((n_panels * 4 + 255) / 256)), dim3(256), 0, stream,
                               d_panels, n_panels, I->W, d_hashes);
            HIPCHK(hipGetLastError());
        }
        return CSA_OK;
    }
    DrawConfig cfg;
    int rc2 = pick_draw_config(I, single || d_picks || d_sel_out || d_present_out || d_panel_list, cfg);
    if (rc2) return rc2;
    DrawArgs A;
    A.featmask = I->d_featmask;
    A.fmin = I->d_fmin;
    A.fmax = I->d_fmax;
    A.sel0 = I->d_sel0;
    A.rem0 = I->d_rem0;
    A.present0 = I->d_present0;
    A.pmask = I->d_pmask;
    A.addr_next = I->d_addr_next;
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
    A.picks16 = nullptr;
    A.status = d_status;
    // legacy_find-semantics draws are counted; single attempts (csa_legacy_attempt) are not
    A.stats = (single || !count_stats) ? nullptr : I->d_stats;
    A.panel_list = d_panel_list;   // an index list: draw_kernel GENERAL (pick_draw_config above)
    A.n_panels_dev = d_list_len;
    A.sel_out = d_sel_out;
    A.rem_out = d_rem_out;
    A.present_out = d_present_out;
    A.xt = nullptr;
    A.npad = ((I->n + 255) / 256) * 256;  // csa_xt_pad
    if (d_picks_ext && !cfg.picks()) return fail(CSA_E_UNSUPPORTED, "this instance does not take the pick-list draw");
    csa_instance *M = const_cast<csa_instance *>(I);  // the lane kernel's pick-list scratch
    if (d_picks_ext)
        A.picks16 = d_picks_ext;
    // (the fused pack's chunked layout reserves whole workgroups of <= 256 panels)
    else if (cfg.picks() && (rc = lane_picks(M, ((n_panels + 255) & ~255ull) * (uint64_t)((k + 7) & ~7), stream,
                                             &A.picks16)))
        return rc;
    const int threads = cfg.lane   ? kLaneThreads
                        : cfg.solo ? kSoloThreads
                        : cfg.wide ? kWideThreads
                                   : draw_threads(cfg.FPL, cfg.WPL);
    const int groups_wg = threads / cfg.G;
    const size_t lds = cfg.lane   ? lane_lds_bytes(cfg.FPL, cfg.WPL, I->n)
                       : cfg.solo ? solo_lds_bytes(cfg.FPL, cfg.WPL, I->n)
                       : cfg.wide ? wide_lds_bytes(cfg.G, cfg.FPL, cfg.WPL)
                                  : draw_lds_bytes(cfg.G, cfg.FPL, cfg.WPL, I->W, k, groups_wg);
    if (lds > 160 * 1024) return fail(CSA_E_UNSUPPORTED, "draw kernel needs %zu B of LDS", lds);
    // CSA_DRAW_LDS_PAD (diagnostic A/B only): extra bytes of LDS per register-kernel workgroup, to price
    // the occupancy an LDS-resident pick-list tile would cost (128 panels x kpad u16 = 28 KB at sf_e)
    static const size_t lds_pad = [] {
        const char *e = getenv("CSA_DRAW_LDS_PAD");
        return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)0;
    }();
    const size_t lds_launch = (cfg.lane || cfg.solo || cfg.wide) && lds + lds_pad <= 160 * 1024 ? lds + lds_pad : lds;
    const uint64_t want = (n_panels + groups_wg - 1) / groups_wg;
    // the lane kernel: one workgroup per 128 panels, not persistent -- sf_e 10^6 panels: 4.47 ms vs
    // 5.05 ms for a persistent grid, and retiring workgroups let a concurrent stream's kernels in.
    // draw_kernel: one resident grid (its 66 KB of feature rows at n = 8192 load once per workgroup)
    uint64_t grid = want;
    if (!cfg.picks()) {
        int per_cu = 0, cus = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, cfg.fn, threads, lds));
        HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, I->device));
        grid = std::min(want, (uint64_t)std::max(per_cu, 1) * (uint64_t)std::max(cus, 1));
    }
    // the lane kernel packs its own panels (one workgroup per 128 panels, so every workgroup knows
    // its panel range); the wide kernel's pick lists are packed by picks_pack_kernel
    const bool fused = (cfg.lane || cfg.solo) && !d_picks_ext && d_panels;
    if ((cfg.lane || cfg.solo) && !fused) {
        A.panels = nullptr;
        A.hashes = nullptr;
    }
    if (d_xt && (cfg.lane || cfg.solo) && fused) {  // the register kernels' fused tail also writes XT
        A.xt = d_xt;
        if (xt_written) *xt_written = 1;
    }
    void *args[] = {&A};
    HIPCHK(hipLaunchKernel(cfg.fn, dim3((unsigned)std::max<uint64_t>(1, grid)), dim3(threads), args, lds_launch, stream));
    HIPCHK(hipGetLastError());
    if (!single && count_stats) M->panels_drawn += n_panels;
    if (cfg.picks() && !d_picks_ext) {  // pick lists -> packed panels (+ hashes)
        if (!fused && (rc = launch_pack(A.picks16, n_panels, k, I->W, d_panels, d_hashes, stream))) return rc;
        HIPCHK(hipEventRecord(M->picks_done, stream));
        M->picks_pending = true;
    }
    return CSA_OK;
}

// panels one full round of the batch draw's resident workgroups covers (CUs x resident workgroups
// per CU x panels per workgroup): a launch of a multiple of it ends without a part-empty last round
int draw_round_panels(const csa_instance *I, int32_t k, uint64_t *out) {
    *out = 0;
    int rc = check_k(I, k);
    if (rc) return rc;
    DrawConfig cfg;
    if ((rc = pick_draw_config(I, false, cfg))) return rc;
    const int threads = cfg.lane   ? kLaneThreads
                        : cfg.solo ? kSoloThreads
                        : cfg.wide ? kWideThreads
                                   : draw_threads(cfg.FPL, cfg.WPL);
    const size_t lds = cfg.lane   ? lane_lds_bytes(cfg.FPL, cfg.WPL, I->n)
                       : cfg.solo ? solo_lds_bytes(cfg.FPL, cfg.WPL, I->n)
                       : cfg.wide ? wide_lds_bytes(cfg.G, cfg.FPL, cfg.WPL)
                                  : draw_lds_bytes(cfg.G, cfg.FPL, cfg.WPL, I->W, k, threads / cfg.G);
    int per_cu = 0, cus = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, cfg.fn, threads, lds));
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, I->device));
    *out = (uint64_t)std::max(per_cu, 1) * (uint64_t)std::max(cus, 1) * (uint64_t)(threads / cfg.G);
    return CSA_OK;
}

int read_status(const uint32_t *d_status, hipStream_t stream, uint32_t *h) {
    HIPCHK(hipMemcpyAsync(h, d_status, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    return CSA_OK;
}

// csa_legacy_sample's pipeline chunk (panels): 2^20 = one bench step at sf_e
constexpr uint64_t kSampleChunk = 1ull << 20;
constexpr int kSampleSlot0 = 8, kScratchSlots = 32;          // instance scratch slots of csa_legacy_sample
constexpr size_t kSampleKeepBytes = (size_t)8 << 30;          // kept across calls up to 8 GiB

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

// instance scratch slot `slot` with at least `count` elements (grow-only)
template <typename T>
int scratch(csa_instance *I, int slot, size_t count, T **out) {
    if (slot < 0 || slot >= kScratchSlots) return fail(CSA_E_INVALID, "internal: scratch slot %d", slot);
    const size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
    if (I->scratch_bytes[slot] < bytes) {
        if (I->scratch[slot]) HIPCHK(hipFree(I->scratch[slot]));
        I->scratch[slot] = nullptr;
        I->scratch_bytes[slot] = 0;
        HIPCHK(hipMalloc(&I->scratch[slot], bytes));
        I->scratch_bytes[slot] = bytes;
    }
    *out = static_cast<T *>(I->scratch[slot]);
    return CSA_OK;
}

}  // namespace

namespace {
// Partitioned distinct pass (no per-panel global atomics): hashes partitioned by their top bits
// (counting pass -> scans -> scatter), then one workgroup per partition dedupes in an LDS table
// (equal 128-bit hashes AND equal bitmasks).  It counts (unique) and/or lists one index per
// distinct panel (rep); seg_counts restricts it to the valid entries of segmented input.
struct UqPlan {
    int pbits = 6;
    uint64_t P = 64, CH = 4096, scratch_bytes = 0;
    uint32_t nwg = 1;
    bool fits = true;  // partitions average <= 2048 entries (an 8192-slot LDS table each)
};

void uq_plan(uint64_t n, UqPlan &q) {
    q.pbits = 6;
    while ((1ull << q.pbits) * 1024 < n && q.pbits < 13) ++q.pbits;
    q.P = 1ull << q.pbits;
    q.CH = std::max<uint64_t>(4096, ((n + 1023) / 1024 + 255) / 256 * 256);
    q.nwg = (uint32_t)((n + q.CH - 1) / q.CH);
    q.scratch_bytes = 4 * n + 4 * q.P * q.nwg + 4 * q.P + 4 * (q.P + 1);
    q.fits = n < (1ull << 31) && n / q.P <= 2048;
}

int uq_partitioned(const uint64_t *d_hashes, const uint64_t *d_panels, uint64_t n, int W, const UqPlan &q,
                   uint32_t *scratch, uint64_t *d_unique, uint32_t *d_status, uint32_t seg_cap,
                   const uint64_t *seg_counts, uint32_t *rep, unsigned long long *rep_count, hipStream_t st) {
    if (!q.fits) return fail(CSA_E_UNSUPPORTED, "distinct panels: %llu entries exceed the partitioned path",
                             (unsigned long long)n);
    uint32_t *idx = scratch, *hist = idx + n, *tot = hist + q.P * q.nwg, *pbase = tot + q.P;
    hipLaunchKernelGGL(uq_count_kernel, dim3(q.nwg), dim3(kUqThreads), 0, st, d_hashes, n, q.CH, q.pbits, q.nwg, hist,
                       seg_cap, seg_counts);
    hipLaunchKernelGGL(uq_scan_part_kernel, dim3((unsigned)q.P), dim3(kUqThreads), 0, st, hist, q.nwg, tot);
    hipLaunchKernelGGL(uq_scan_tot_kernel, dim3(1), dim3(1024), 0, st, tot, (uint32_t)q.P, pbase);
    hipLaunchKernelGGL(uq_scatter_kernel, dim3(q.nwg), dim3(kUqThreads), 0, st, d_hashes, n, q.CH, q.pbits, q.nwg,
                       hist, pbase, idx, seg_cap, seg_counts);
    hipLaunchKernelGGL(uq_dedupe_kernel, dim3((unsigned)q.P), dim3(kUqThreads), 0, st, d_hashes, d_panels, W, idx,
                       pbase, reinterpret_cast<unsigned long long *>(d_unique), d_status, rep, rep_count);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

// csa_unique_async / csa_unique_segments_async: the partitioned path for large batches with a status
// block (its LDS tables report an overflow there), else one global open-addressing table
int unique_impl(const uint64_t *d_hashes, const uint64_t *d_panels, uint64_t n_panels, int32_t W, uint64_t *d_table,
                uint64_t table_slots, uint64_t *d_unique, uint32_t *d_status, uint32_t seg_cap,
                const uint64_t *seg_counts, hipStream_t st) {
    if (!d_hashes || !d_panels || !d_table || !d_unique || W <= 0) return fail(CSA_E_INVALID, "unique: bad arguments");
    if (table_slots < 2 * n_panels || (table_slots & (table_slots - 1)))
        return fail(CSA_E_INVALID, "unique: table_slots must be a power of two >= 2*n_panels");
    if (n_panels == 0) return CSA_OK;
    UqPlan q;
    uq_plan(n_panels, q);
    const char *ue = getenv("CSA_UNIQUE_PART");
    if (d_status && n_panels >= 65536 && q.fits && q.scratch_bytes <= table_slots * 8 && !(ue && atoi(ue) == 0))
        return uq_partitioned(d_hashes, d_panels, n_panels, W, q, reinterpret_cast<uint32_t *>(d_table), d_unique,
                              d_status, seg_cap, seg_counts, nullptr, nullptr, st);
    HIPCHK(hipMemsetAsync(d_table, 0, table_slots * 8, st));
    const unsigned grid = (unsigned)((n_panels + 255) / 256);
    hipLaunchKernelGGL(unique_kernel, dim3(grid), dim3(256), 0, st, d_hashes, d_panels, n_panels, W,
                       reinterpret_cast<unsigned long long *>(d_table), table_slots - 1,
                       reinterpret_cast<unsigned long long *>(d_unique), seg_cap, seg_counts, nullptr, nullptr);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}
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

int csa_current_device(int32_t *out) {
    if (!out) return fail(CSA_E_INVALID, "null out");
    int d = -1;
    hipError_t e = hipGetDevice(&d);
    *out = d;
    if (e != hipSuccess) return fail(CSA_E_HIP, "hipGetDevice: %s", hipGetErrorString(e));
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
    I->sel0.assign(F, 0);
    update_need8(I);
    I->featmask.assign((size_t)F * I->Ws, 0ull);
    for (int f = 1; f < F; ++f)
        if (feat_cat[f] < feat_cat[f - 1]) {
            delete I;
            return fail(CSA_E_INVALID, "features must be category-major (feat_cat non-decreasing)");
        }
    for (int f = 0; f < F; ++f) {
        I->max_abs = std::max(I->max_abs, std::abs(fmin[f]));
        if (fmax[f] > 0) I->max_slack = std::max(I->max_slack, fmax[f]);
        if (fmax[f] == 0 && fmin[f] != 0) I->zero_max_min = true;
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
        (rc = dalloc(&I->d_present0, I->W)) || (F <= 32 && (rc = dalloc(&I->d_pmask, n))) ||
        (rc = dalloc(&I->d_stats, 2))) {
        csa_instance_destroy(I);
        return rc;
    }
    std::vector<uint32_t> pmask(F <= 32 ? n : 0, 0u);
    for (int p = 0; p < (int)pmask.size(); ++p)
        for (int c = 0; c < C; ++c) pmask[p] |= 1u << person_feat[(size_t)p * C + c];
    hipError_t e = hipSuccess;
    e = e ? e : hipMemcpy(I->d_featmask, I->featmask.data(), I->featmask.size() * 8, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(I->d_fmin, fmin, F * 4, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(I->d_fmax, fmax, F * 4, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(I->d_sel0, zeros.data(), F * 4, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(I->d_rem0, I->pool.data(), F * 4, hipMemcpyHostToDevice);
    if (I->W) e = e ? e : hipMemcpy(I->d_present0, present.data(), I->W * 8, hipMemcpyHostToDevice);
    if (!pmask.empty()) e = e ? e : hipMemcpy(I->d_pmask, pmask.data(), pmask.size() * 4, hipMemcpyHostToDevice);
    e = e ? e : hipMemset(I->d_stats, 0, 16);
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
    // drain everything that may still use the instance's buffers, while its streams exist
    if (I->picks_done && I->picks_pending) (void)hipEventSynchronize(I->picks_done);
    if (I->sdraw) (void)hipStreamSynchronize(I->sdraw);
    if (I->spost) (void)hipStreamSynchronize(I->spost);
    if (I->stream) (void)hipStreamSynchronize(I->stream);
    if (I->d_featmask) (void)hipFree(I->d_featmask);
    if (I->d_fmin) (void)hipFree(I->d_fmin);
    if (I->d_fmax) (void)hipFree(I->d_fmax);
    if (I->d_sel0) (void)hipFree(I->d_sel0);
    if (I->d_rem0) (void)hipFree(I->d_rem0);
    if (I->d_present0) (void)hipFree(I->d_present0);
    if (I->d_pmask) (void)hipFree(I->d_pmask);
    if (I->d_addr_next) (void)hipFree(I->d_addr_next);
    if (I->d_picks16) (void)hipFree(I->d_picks16);
    if (I->d_stats) (void)hipFree(I->d_stats);
    for (int i = 0; i < kScratchSlots; ++i)
        if (I->scratch[i]) (void)hipFree(I->scratch[i]);
    if (I->picks_done) (void)hipEventDestroy(I->picks_done);
    if (I->drawn) (void)hipEventDestroy(I->drawn);
    if (I->stream) (void)hipStreamDestroy(I->stream);
    if (I->sdraw) (void)hipStreamDestroy(I->sdraw);
    if (I->spost) (void)hipStreamDestroy(I->spost);
    for (csa_instance *R : I->replicas)
        if (R) csa_instance_destroy(R);
    delete I;
}

int csa_instance_draw_stats(csa_instance *I, int32_t reset, uint64_t *out) {
    if (!I || !out) return fail(CSA_E_INVALID, "draw_stats: bad arguments");
    uint64_t acc[3] = {0, 0, 0};
    std::vector<csa_instance *> all{I};
    for (csa_instance *R : I->replicas)
        if (R) all.push_back(R);
    for (csa_instance *X : all) {
        ScopedDevice sd(X->device);
        HIPCHK(hipDeviceSynchronize());  // every stream that may still run a draw of X
        unsigned long long h[2];
        HIPCHK(hipMemcpy(h, X->d_stats, 16, hipMemcpyDeviceToHost));
        acc[0] += X->panels_drawn + h[0] + h[1];
        acc[1] += h[0];
        acc[2] += h[1];
        if (reset) {
            HIPCHK(hipMemset(X->d_stats, 0, 16));
            X->panels_drawn = 0;
        }
    }
    for (int j = 0; j < 3; ++j) out[j] = acc[j];
    return CSA_OK;
}

// d_out[0..2] = attempts, SelectionErrors, rejections of the instance's draws so far (not its
// replicas'), written on `stream` -- no host wait (the sharded legacy_probabilities folds them into
// its one host read)
__global__ void draw_stats_copy_kernel(const unsigned long long *__restrict__ st, uint64_t drawn,
                                       uint64_t *__restrict__ out) {
    if (threadIdx.x == 0) {
        out[0] = drawn + st[0] + st[1];
        out[1] = st[0];
        out[2] = st[1];
    }
}

int csa_instance_draw_stats_async(csa_instance *I, uint64_t *d_out, void *stream) {
    if (!I || !d_out) return fail(CSA_E_INVALID, "draw_stats_async: bad arguments");
    ScopedDevice sd(I->device);
    hipLaunchKernelGGL(draw_stats_copy_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, I->d_stats,
                       (uint64_t)I->panels_drawn, d_out);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_instance_draw_stats_reset(csa_instance *I, void *stream) {
    if (!I) return fail(CSA_E_INVALID, "draw_stats_reset: null instance");
    std::vector<csa_instance *> all{I};
    for (csa_instance *R : I->replicas)
        if (R) all.push_back(R);
    for (csa_instance *X : all) {
        ScopedDevice sd(X->device);
        if (stream && X == I) {  // ordered on the caller's stream: no host wait
            HIPCHK(hipMemsetAsync(X->d_stats, 0, 16, (hipStream_t)stream));
        } else {  // only the instance's own streams (csa_legacy_sample's pipeline), not the device
            for (hipStream_t s : {X->sdraw, X->spost, X->stream})
                if (s) HIPCHK(hipStreamSynchronize(s));
            if (!X->stream) HIPCHK(hipStreamCreateWithFlags(&X->stream, hipStreamNonBlocking));
            HIPCHK(hipMemsetAsync(X->d_stats, 0, 16, X->stream));
            HIPCHK(hipStreamSynchronize(X->stream));
        }
        X->panels_drawn = 0;
    }
    return CSA_OK;
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
    I->sel_over_max = false;
    I->max_slack = 0;
    for (int f = 0; f < I->F; ++f) {
        const int32_t s = sel ? sel[f] : 0;
        if (sel) mx = std::max(mx, std::abs(s));
        if (s > I->fmax[f] || (I->fmax[f] > 0 && s == I->fmax[f])) I->sel_over_max = true;
        if (I->fmax[f] > 0) I->max_slack = std::max(I->max_slack, I->fmax[f] - s);
    }
    I->max_abs = mx;
    update_need8(I);
    if (present)
        for (int w = 0; w < I->W; ++w)
            if (present[w] & ~all[w]) return fail(CSA_E_INVALID, "present mask has bits beyond n");
    HIPCHK(hipMemcpy(I->d_sel0, sel ? sel : zeros.data(), I->F * 4, hipMemcpyHostToDevice));
    I->sel0.assign(sel ? sel : zeros.data(), (sel ? sel : zeros.data()) + I->F);
    HIPCHK(hipMemcpy(I->d_rem0, rem ? rem : I->pool.data(), I->F * 4, hipMemcpyHostToDevice));
    if (I->W) HIPCHK(hipMemcpy(I->d_present0, present ? present : all.data(), I->W * 8, hipMemcpyHostToDevice));
    if (rem) I->rem0h.assign(rem, rem + I->F); else I->rem0h.clear();
    if (present) I->present0h.assign(present, present + I->W); else I->present0h.clear();
    ++I->gen;
    return CSA_OK;
}

int csa_instance_set_address(csa_instance *I, const int32_t *addr_next) {
    if (!I) return fail(CSA_E_INVALID, "null instance");
    ScopedDevice sd(I->device);
    if (I->picks_pending) HIPCHK(hipEventSynchronize(I->picks_done));
    if (!addr_next) {
        if (I->d_addr_next) HIPCHK(hipFree(I->d_addr_next));
        I->d_addr_next = nullptr;
        I->addr_h.clear();
        ++I->gen;
        return CSA_OK;
    }
    for (int p = 0; p < I->n; ++p)
        if (addr_next[p] < 0 || addr_next[p] >= I->n) return fail(CSA_E_INVALID, "addr_next[%d] out of range", p);
    if (!I->d_addr_next) {
        int rc = dalloc(&I->d_addr_next, (size_t)I->n);
        if (rc) return rc;
    }
    HIPCHK(hipMemcpy(I->d_addr_next, addr_next, (size_t)I->n * 4, hipMemcpyHostToDevice));
    I->addr_h.assign(addr_next, addr_next + I->n);
    ++I->gen;
    return CSA_OK;
}

int csa_pair_histogram_async(const int64_t *d_pairs, int32_t n, uint64_t *d_hist, uint64_t n_bins,
                             uint64_t *d_overflow, void *stream) {
    if (n < 0 || !d_pairs || !d_hist || !d_overflow || n_bins == 0) return fail(CSA_E_INVALID, "pair histogram: bad arguments");
    HIPCHK(hipMemsetAsync(d_hist, 0, n_bins * 8, (hipStream_t)stream));
    HIPCHK(hipMemsetAsync(d_overflow, 0, 8, (hipStream_t)stream));
    if (n < 2) return CSA_OK;
    if (n_bins <= (uint64_t)kHistLdsBins) {
        // ~2 workgroups per CU, each over a stride of rows (one LDS histogram flush per workgroup)
        const unsigned grid = (unsigned)std::min<int>(n - 1, 512);
        hipLaunchKernelGGL(pair_histogram_lds_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_pairs, n,
                           reinterpret_cast<unsigned long long *>(d_hist), n_bins,
                           reinterpret_cast<unsigned long long *>(d_overflow));
    } else {
        hipLaunchKernelGGL(pair_histogram_kernel, dim3((unsigned)(n - 1)), dim3(256), 0, (hipStream_t)stream, d_pairs,
                           n, reinterpret_cast<unsigned long long *>(d_hist), n_bins,
                           reinterpret_cast<unsigned long long *>(d_overflow));
    }
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_pairs_pack_async(const int64_t *d_pairs, int32_t n, int32_t *d_packed, void *stream) {
    if (n <= 0 || !d_pairs || !d_packed) return fail(CSA_E_INVALID, "pairs pack: bad arguments");
    hipLaunchKernelGGL(pairs_pack_kernel, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream, d_pairs, n, d_packed);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_pairs_diag_async(const int64_t *d_pairs, int32_t n, int64_t *d_counts, void *stream) {
    if (n <= 0 || !d_pairs || !d_counts) return fail(CSA_E_INVALID, "pairs_diag: bad arguments");
    hipLaunchKernelGGL(pairs_diag_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_pairs,
                       n, d_counts);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_pairs_upper_async(const int64_t *d_pairs, int32_t n, double divisor, void *d_out, void *stream) {
    if (n < 0 || (n > 1 && (!d_pairs || !d_out)) || divisor < 0.0) return fail(CSA_E_INVALID, "pairs upper: bad arguments");
    if (n < 2) return CSA_OK;
    if (divisor > 0.0)
        hipLaunchKernelGGL(pairs_upper_kernel<true>, dim3((unsigned)(n - 1)), dim3(256), 0, (hipStream_t)stream, d_pairs,
                           n, divisor, d_out);
    else
        hipLaunchKernelGGL(pairs_upper_kernel<false>, dim3((unsigned)(n - 1)), dim3(256), 0, (hipStream_t)stream, d_pairs,
                           n, 0.0, d_out);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_pairs_unpack_async(const int32_t *d_packed, int32_t n, int64_t *d_pairs, void *stream) {
    if (n <= 0 || !d_pairs || !d_packed) return fail(CSA_E_INVALID, "pairs unpack: bad arguments");
    hipLaunchKernelGGL(pairs_unpack_kernel, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream, d_packed, n, d_pairs);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

#ifdef CSA_LANE_STAMPS
// diagnostic builds only: the draw_lane_kernel segment totals (cycles summed over waves, [8] = waves,
// [9..19] = region execution counts summed over waves: loop, philox, step, pick, store, round, pass2,
// pass1, nocand, kcheck, ending)
int csa_debug_lane_stamps(uint64_t *out24, int reset) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out24, HIP_SYMBOL(g_lane_stamps), 24 * 8));
    if (reset) {
        static const unsigned long long zero[24] = {};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_lane_stamps), zero, 24 * 8));
    }
    return CSA_OK;
}
#endif

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
        case CSA_E_UNSUPPORTED:
            if (panel == kExchangeOverflow)
                return fail(CSA_E_UNSUPPORTED, "distinct-panel exchange: an owner segment exceeded its capacity");
            if (panel == 0xFFFFFFFFFFFFFFFFull)
                return fail(CSA_E_UNSUPPORTED, "distinct panels: a partition exceeded its LDS table");
            return fail(CSA_E_UNSUPPORTED, "device status %u at panel %llu", h[0], (unsigned long long)panel);
        default:
            return fail((int)h[0], "device status %u at panel %llu", h[0], (unsigned long long)panel);
    }
}

int csa_draw_round_panels(const csa_instance *I, int32_t k, uint64_t *out) {
    if (!I || !out) return fail(CSA_E_INVALID, "draw_round_panels: bad arguments");
    ScopedDevice sd(I->device);
    return draw_round_panels(I, k, out);
}

int csa_draw_async(const csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                   uint32_t max_attempts, uint64_t *d_panels, uint64_t *d_hashes, uint32_t *d_attempts,
                   int32_t *d_picks, uint32_t *d_status, void *stream) {
    if (!I) return fail(CSA_E_INVALID, "null instance");
    return launch_draw(I, k, seed, panel_begin, n_panels, max_attempts, 0, 0, d_panels, d_hashes, d_attempts,
                       d_picks, d_status, nullptr, nullptr, nullptr, (hipStream_t)stream);
}

int csa_draw_xt_async(const csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                      uint32_t max_attempts, uint64_t *d_panels, uint64_t *d_hashes, uint32_t *d_attempts,
                      uint32_t *d_status, uint32_t *d_xt, int32_t *xt_written, uint32_t flags, void *stream) {
    if (!I || !d_xt || !xt_written) return fail(CSA_E_INVALID, "draw_xt: null instance, d_xt or xt_written");
    if ((flags & CSA_DRAW_RESET_STATUS) && d_status) HIPCHK(hipMemsetAsync(d_status, 0, 4 * sizeof(uint32_t), (hipStream_t)stream));
    if (flags & CSA_DRAW_RESET_STATS) {  // this instance's statistics, ordered on the stream (no host wait)
        csa_instance *M = const_cast<csa_instance *>(I);
        ScopedDevice sd(M->device);
        HIPCHK(hipMemsetAsync(M->d_stats, 0, 16, (hipStream_t)stream));
        M->panels_drawn = 0;
    }
    return launch_draw(I, k, seed, panel_begin, n_panels, max_attempts, 0, 0, d_panels, d_hashes, d_attempts,
                       nullptr, d_status, nullptr, nullptr, nullptr, (hipStream_t)stream, nullptr, nullptr, nullptr,
                       d_xt, xt_written);
}

int csa_redraw_async(const csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                     uint32_t max_attempts, uint64_t *d_panels, uint32_t *d_status, void *stream) {
    if (!I || !d_panels || !d_status) return fail(CSA_E_INVALID, "redraw: null instance, d_panels or d_status");
    return launch_draw(I, k, seed, panel_begin, n_panels, max_attempts, 0, 0, d_panels, nullptr, nullptr, nullptr,
                       d_status, nullptr, nullptr, nullptr, (hipStream_t)stream, nullptr, nullptr, nullptr, nullptr,
                       nullptr, /*count_stats=*/false);
}

int32_t csa_picks_stride(int32_t k) { return (k + 7) & ~7; }

int csa_draw_picks_supported(const csa_instance *I, int32_t k) {
    if (!I || check_k(I, k)) return 0;
    DrawConfig cfg;
    return pick_draw_config(I, false, cfg) == CSA_OK && cfg.picks() ? 1 : 0;
}

int csa_draw_picks_async(const csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                         uint32_t max_attempts, uint16_t *d_picks, uint32_t *d_attempts, uint32_t *d_status,
                         void *stream) {
    if (!I || !d_picks) return fail(CSA_E_INVALID, "draw_picks: null instance or d_picks");
    return launch_draw(I, k, seed, panel_begin, n_panels, max_attempts, 0, 0, nullptr, nullptr, d_attempts, nullptr,
                       d_status, nullptr, nullptr, nullptr, (hipStream_t)stream, d_picks);
}

int csa_picks_pack_async(const uint16_t *d_picks, uint64_t n_panels, int32_t k, int32_t n, uint64_t *d_panels,
                         uint64_t *d_hashes, void *stream) {
    if (n <= 0 || n > 65536 || k < 0 || (k > 0 && !d_picks) || !d_panels)
        return fail(CSA_E_INVALID, "picks_pack: bad arguments");
    const int W = (n + 63) / 64;
    if ((size_t)4 * 4 * (2 * W + 1) * 4 > 160 * 1024) return fail(CSA_E_UNSUPPORTED, "picks_pack: n=%d too large", n);
    return launch_pack(d_picks, n_panels, k, W, d_panels, d_hashes, (hipStream_t)stream);
}

int csa_panel_hash_async(const uint64_t *d_panels, uint64_t n_panels, int32_t W, uint64_t *d_hashes,
                         void *stream) {
    if (W <= 0 || !d_panels || !d_hashes) return fail(CSA_E_INVALID, "panel hash: bad arguments");
    if (n_panels == 0) return CSA_OK;
    hipLaunchKernelGGL(panel_hash_kernel, dim3((unsigned)((n_panels * 4 + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d_panels, n_panels, W, d_hashes);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_draw_kernel_name(const csa_instance *I, int32_t k, char *buf, uint64_t len) {
    if (!I || !buf || len == 0) return fail(CSA_E_INVALID, "draw kernel name: bad arguments");
    int rc = check_k(I, k);
    if (rc) return rc;
    DrawConfig cfg;
    rc = pick_draw_config(I, false, cfg);
    if (rc) return rc;
    if (cfg.solo)
        snprintf(buf, (size_t)len, "draw_solo_kernel<%d, %d, %s>", cfg.FPL, cfg.WPL, cfg.k8 ? "true" : "false");
    else if (cfg.lane)
        snprintf(buf, (size_t)len, "draw_lane_kernel<%d, %d, %d, %s>", cfg.FPL, cfg.WPL,
                 (cfg.WPL / 2 + CSA_LANE_SKDIV - 1) / CSA_LANE_SKDIV, cfg.k8 ? "true" : "false");
    else if (cfg.wide)
        snprintf(buf, (size_t)len, "draw_wide_kernel<%d, %d, %d>", cfg.G, cfg.FPL, cfg.WPL);
    else
        snprintf(buf, (size_t)len, "draw_kernel<%d, %d, %d, false>", cfg.G, cfg.FPL, cfg.WPL);
    return CSA_OK;
}

int32_t csa_xt_pad(int32_t n) { return ((n + kPairBlock - 1) / kPairBlock) * kPairBlock; }

int csa_transpose_count_async(const uint64_t *d_panels, uint64_t n_panels, int32_t n, uint64_t *d_xt,
                              int64_t *d_counts, void *stream) {
    if (n <= 0 || !d_panels || !d_counts) return fail(CSA_E_INVALID, "transpose: bad arguments");
    if (n_panels == 0) return CSA_OK;
    const int W = (n + 63) / 64, CW = std::min(W, kXtCols), Wp = CW | 1;
    const size_t lds = (size_t)64 * Wp * 8 + (size_t)std::min(n, 64 * CW) * 4;
    if (lds > 160 * 1024) return fail(CSA_E_UNSUPPORTED, "transpose needs %zu B of LDS", lds);
    const uint64_t nblk = (n_panels + 63) / 64;
    const unsigned ranges = (unsigned)((W + kXtCols - 1) / kXtCols);
    // 64-panel blocks per workgroup: up to kXtBlocksPerGroup (fewer count flushes), but enough
    // workgroups for two per CU (n = 8192, 10^5 panels: 4 blocks per workgroup, not 16)
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    const uint64_t bpg = std::max<uint64_t>(1, std::min<uint64_t>(kXtBlocksPerGroup, nblk * ranges / (2 * (uint64_t)cus)));
    const unsigned grid = (unsigned)((nblk + bpg - 1) / bpg);
    hipLaunchKernelGGL(xt_count_kernel, dim3(grid, ranges), dim3(kXtThreads), lds, (hipStream_t)stream, d_panels,
                       n_panels, n, W, csa_xt_pad(n), d_xt, d_counts, (int)bpg);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

namespace {
struct PairPlan {
    int npad, nbt, ntri, nsplit;
};

// one 512-thread workgroup per CU (two waves per SIMD).  Splits of the panel blocks: the smallest count
// whose rounds of CU-wide workgroups, each 1/ns of a tile, come within 2 % of the best balance over
// ns <= 64 (ntri <= cus / 2: the CUs filled once, ns = cus / ntri as before -- sf_e 28 tiles x 9,
// n = 2000 36 x 7; 128 < ntri < 256: one split left up to half the CUs idle, n = 4096's 136 tiles
// 5.0 ms per 10^6 panels -- 15 splits make 8 rounds of 1/15 tile).  At least 8 panel blocks per
// split, and every split below the accumulator's exact range (f32: 2^24).
int pair_plan(int32_t n, uint64_t n_blocks, uint32_t engine, PairPlan &p) {
    if (engine != CSA_PAIR_FP4 && engine != CSA_PAIR_I8) return fail(CSA_E_INVALID, "pairs: unknown engine %u", engine);
    p.npad = csa_xt_pad(n);
    p.nbt = p.npad / kPairBlock;
    p.ntri = p.nbt * (p.nbt + 1) / 2;
    int cus = 256;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t ns_cap = std::max<uint64_t>(1, n_blocks / 8);
    uint64_t ns = std::max(1, cus / p.ntri);
    if (2 * p.ntri > cus) {  // time per split-round layout ~ ceil(ntri ns / cus) / ns
        auto cost = [&](uint64_t m) { return (double)((p.ntri * m + cus - 1) / cus) / (double)m; };
        const uint64_t hi = std::min<uint64_t>(64, ns_cap);
        double best = cost(1);
        for (uint64_t m = 2; m <= hi; ++m) best = std::min(best, cost(m));
        ns = 1;
        while (ns < hi && cost(ns) > 1.02 * best) ++ns;
    }
    ns = std::min<uint64_t>(ns, ns_cap);
    const uint64_t exact_blocks = engine == CSA_PAIR_FP4 ? (1ull << 24) / 64 : (1ull << 31) / 64;
    ns = std::max<uint64_t>(ns, (n_blocks + exact_blocks - 1) / exact_blocks);
    if (ns > (1u << 20)) return fail(CSA_E_UNSUPPORTED, "pairs: too many panel blocks per call");
    p.nsplit = (int)ns;
    return CSA_OK;
}
// pair_fp4_tile_kernel's plan (fp4 engine, whole-tile items exact in f32, CUs in 8 XCD groups):
// false when it does not apply (pair_mfma_kernel then runs).  It is taken when the triangle has at
// least one tile per CU (n >= ~5.7k): there pair_mfma_kernel's one-split launch ends in a part-empty
// round (n = 8192: 528 blocks = 2.06 rounds; 16.0 vs 10.3 ms alone, 29.3 vs 31.2 M panels/s end to
// end).  Below it the split kernel stays: alone the two are level, but its 2 waves/SIMD leave room
// for a draw wave beside it on a CU, and inside the pipelined step that is worth more (sf_e 263.4 vs
// 257.7 M panels/s, example_large_200 300.2 vs 289.4; tools/gpu_ab_env.sh).
// CSA_PAIR_KERNEL=1 forces pair_mfma_kernel, =2 this kernel wherever it applies.
struct Pair2Plan {
    PairMap M;
    int grid = 0, lmax = 0;  // persistent workgroups; leftover tiles (pooled over the XCDs)
};

// alone (CSA_PAIR_ALONE): no draw runs beside this launch, so the kernel fastest alone is taken.  This
// one wins alone only with several tiles per side and enough panel blocks to amortise its persistent
// grid (n = 1727: 0.60 vs 0.68 ms per 10^6 panels, 0.19 vs 0.20 per 2^18, level at 2^17, 0.053 vs
// 0.043 ms per 10^4; n <= 200 level at 10^6 and 4.5x slower at 10^4; profiles/r06_pair_alone/): below
// kP2AloneMinBlocks or kP2AloneMinTiles tiles per side the split kernel stays.  CSA_PAIR_ALONE_MIN_BLOCKS overrides the block bound (A/B).
constexpr uint64_t kP2AloneMinBlocks = 2048;  // 131072 panels: level there, the tile kernel ahead from 262144
constexpr int kP2AloneMinTiles = 4;           // n > 768
bool pair2_plan(int32_t n, uint64_t n_blocks, uint32_t engine, bool shared, Pair2Plan &q, bool alone = false) {
    if (engine != CSA_PAIR_FP4 || n_blocks == 0 || n_blocks > kP2MaxBlocks) return false;
    const char *e = getenv("CSA_PAIR_KERNEL");
    const int force = e ? atoi(e) : 0;
    if (force == 1) return false;
    int cus = 256, dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus < kP2Xcds || cus % kP2Xcds) return false;
    // B fragments per wave: 4 (512-register waves, one per SIMD) also when the launch shares the CUs with
    // draws (CSA_PAIR_SHARED): with the interleaved loop it beats the 256-register NB = 2 form beside the
    // n = 8192 draw (32.9 vs 31.7 M panels/s end to end); CSA_P2_NB=2|4 forces either (A/B)
    (void)shared;
    const char *enb = getenv("CSA_P2_NB");
    const int nbf = enb ? atoi(enb) : 4;
    q.M.halves = nbf == 2 ? 2 : 1;
    q.M.nbt = csa_xt_pad(n) / kPairBlock;
    q.M.ntri = q.M.nbt * (q.M.nbt + 1) / 2;
    q.M.P = cus / kP2Xcds;
    q.M.nblk = n_blocks;
    q.grid = cus;
    q.lmax = q.M.leftovers();  // pooled leftover tiles (each in pieces(lmax) int32 partial slots)
    static const uint64_t alone_min_blocks = [] {
        const char *v = getenv("CSA_PAIR_ALONE_MIN_BLOCKS");
        return v ? (uint64_t)strtoull(v, nullptr, 10) : kP2AloneMinBlocks;
    }();
    alone = alone && n_blocks >= alone_min_blocks && q.M.nbt >= kP2AloneMinTiles;
    return force == 2 || alone || q.M.ntri >= cus;
}

uint64_t pair2_scratch_bytes(const Pair2Plan &q) {
    return q.lmax ? (uint64_t)q.lmax * q.M.pieces(q.lmax) * kPairBlock * kPairBlock * sizeof(int32_t) : 0;
}
}  // namespace

uint64_t csa_pair_scratch_bytes(int32_t n, uint64_t n_blocks, uint32_t engine) {
    engine &= ~(CSA_PAIR_OVERWRITE | CSA_PAIR_SHARED | CSA_PAIR_ALONE);
    if (n <= 0 || n_blocks == 0) return 0;
    // enough for every form a call may take (per-CU kernel with or without CSA_PAIR_SHARED /
    // CSA_PAIR_ALONE, or the split kernel), so one buffer serves all of them
    uint64_t need = 0;
    Pair2Plan q;
    if (pair2_plan(n, n_blocks, engine, false, q, true)) need = std::max<uint64_t>(pair2_scratch_bytes(q), 4);
    if (pair2_plan(n, n_blocks, engine, false, q)) return need;
    PairPlan p;
    if (pair_plan(n, n_blocks, engine, p)) return need;
    return std::max<uint64_t>(need, (uint64_t)p.ntri * p.nsplit * kPairBlock * kPairBlock * sizeof(int32_t));
}

int csa_pair_counts_ex_async(const uint64_t *d_xt, uint64_t n_blocks, int32_t n, int64_t *d_pairs,
                             uint32_t engine, void *d_scratch, uint64_t scratch_bytes, void *stream) {
    if (n <= 0 || !d_xt || !d_pairs) return fail(CSA_E_INVALID, "pairs: bad arguments");
    const bool overwrite = (engine & CSA_PAIR_OVERWRITE) != 0u, shared = (engine & CSA_PAIR_SHARED) != 0u;
    const bool alone = (engine & CSA_PAIR_ALONE) != 0u && !shared;
    engine &= ~(CSA_PAIR_OVERWRITE | CSA_PAIR_SHARED | CSA_PAIR_ALONE);
    const hipStream_t st = (hipStream_t)stream;
    if (overwrite && (n_blocks == 0 || !d_scratch))  // no reduce pass to store every element
        HIPCHK(hipMemsetAsync(d_pairs, 0, (size_t)n * n * sizeof(int64_t), st));
    if (n_blocks == 0) return CSA_OK;
    Pair2Plan q;
    if (d_scratch && pair2_plan(n, n_blocks, engine, shared, q, alone)) {
        if (scratch_bytes < pair2_scratch_bytes(q))
            return fail(CSA_E_INVALID, "pairs: scratch of %llu B < csa_pair_scratch_bytes = %llu B",
                        (unsigned long long)scratch_bytes, (unsigned long long)pair2_scratch_bytes(q));
        int32_t *part = static_cast<int32_t *>(d_scratch);
        const uint32_t *xt32 = reinterpret_cast<const uint32_t *>(d_xt);
        const int npad = csa_xt_pad(n), ow = overwrite ? 1 : 0;
        const void *fn = q.M.halves == 2 ? reinterpret_cast<const void *>(&pair_fp4_tile_kernel<2>)
                                         : reinterpret_cast<const void *>(&pair_fp4_tile_kernel<4>);
        PairMap M = q.M;
        void *args[] = {(void *)&xt32, &n, (void *)&npad, &M, &d_pairs, &part, (void *)&ow};
        HIPCHK(hipLaunchKernel(fn, dim3(q.grid), dim3(kP2Threads), args, 0, st));
        HIPCHK(hipGetLastError());
        if (q.lmax) {
            hipLaunchKernelGGL(pair_reduce2_kernel, dim3(kPairBlock, q.lmax), dim3(kPairBlock), 0, st,
                               (const int32_t *)part, n, q.M, d_pairs, ow);
            HIPCHK(hipGetLastError());
        }
        return CSA_OK;
    }
    PairPlan p;
    int rc = pair_plan(n, n_blocks, engine, p);
    if (rc) return rc;
    const bool partial = d_scratch != nullptr;
    if (partial && scratch_bytes < csa_pair_scratch_bytes(n, n_blocks, engine))
        return fail(CSA_E_INVALID, "pairs: scratch of %llu B < csa_pair_scratch_bytes = %llu B",
                    (unsigned long long)scratch_bytes, (unsigned long long)csa_pair_scratch_bytes(n, n_blocks, engine));
    const dim3 grid(p.ntri * p.nsplit), block(kPairThreads);
    int32_t *part = static_cast<int32_t *>(d_scratch);
    const void *fn = engine == CSA_PAIR_FP4
                         ? (partial ? reinterpret_cast<const void *>(&pair_mfma_kernel<true, true, kPairKB>)
                                    : reinterpret_cast<const void *>(&pair_mfma_kernel<true, false, kPairKB>))
                         : (partial ? reinterpret_cast<const void *>(&pair_mfma_kernel<false, true, kPairKB>)
                                    : reinterpret_cast<const void *>(&pair_mfma_kernel<false, false, kPairKB>));
    uint64_t nb = n_blocks;
    int npad = p.npad, nbt = p.nbt, nsplit = p.nsplit;
    void *args[] = {(void *)&d_xt, &nb, &n, &npad, &nbt, &nsplit, &d_pairs, &part};
    HIPCHK(hipLaunchKernel(fn, grid, block, args, 0, st));
    HIPCHK(hipGetLastError());
    if (partial) {
        hipLaunchKernelGGL(pair_reduce_kernel, dim3(kPairBlock, p.ntri), dim3(256), 0, st, part, n, p.nbt, p.nsplit,
                           d_pairs, (int)overwrite);
        HIPCHK(hipGetLastError());
    }
    return CSA_OK;
}

int csa_pair_counts_async(const uint64_t *d_xt, uint64_t n_blocks, int32_t n, int64_t *d_pairs, void *stream) {
    return csa_pair_counts_ex_async(d_xt, n_blocks, n, d_pairs, CSA_PAIR_FP4, nullptr, 0, stream);
}

int csa_unique_async(const uint64_t *d_hashes, const uint64_t *d_panels, uint64_t n_panels, int32_t W,
                     uint64_t *d_table, uint64_t table_slots, uint64_t *d_unique, uint32_t *d_status, void *stream) {
    return unique_impl(d_hashes, d_panels, n_panels, W, d_table, table_slots, d_unique, d_status, 0, nullptr,
                       (hipStream_t)stream);
}

int csa_unique_segments_async(const uint64_t *d_hashes, const uint64_t *d_panels, uint32_t n_segments,
                              uint64_t capacity, const uint64_t *d_seg_counts, int32_t W, uint64_t *d_table,
                              uint64_t table_slots, uint64_t *d_unique, uint32_t *d_status, void *stream) {
    if (!d_seg_counts || capacity == 0 || capacity > 0xFFFFFFFFull)
        return fail(CSA_E_INVALID, "unique segments: bad arguments");
    return unique_impl(d_hashes, d_panels, (uint64_t)n_segments * capacity, W, d_table, table_slots, d_unique,
                       d_status, (uint32_t)capacity, d_seg_counts, (hipStream_t)stream);
}

// scratch of csa_exchange_pack_async: rep_count, rep[n], then the partitioned pass's scratch or --
// for a shard beyond it (more than 2048 panels per partition at the 8192-partition maximum, i.e.
// above 16.8 M panels) -- one global open-addressing table of pow2 >= 2n slots
static uint64_t exchange_dedupe_bytes(uint64_t n) {
    UqPlan q;
    uq_plan(n, q);
    return q.fits ? q.scratch_bytes : 8 * pow2_at_least(std::max<uint64_t>(2 * n, 64));
}

uint64_t csa_exchange_scratch_bytes(uint64_t n_panels) {
    const uint64_t n = std::max<uint64_t>(n_panels, 1);
    return 8 + 4 * (n + 1) + exchange_dedupe_bytes(n) + 8;
}

int csa_exchange_pack_async(const uint64_t *d_hashes, const uint64_t *d_panels, uint64_t n_panels, int32_t W,
                            uint32_t world, uint64_t capacity, void *d_scratch, uint64_t scratch_bytes,
                            uint64_t *d_send_hashes, uint64_t *d_send_panels, uint64_t *d_send_counts,
                            uint32_t *d_status, void *stream) {
    if (!d_hashes || !d_panels || W <= 0 || world == 0 || world > (uint32_t)kMaxWorld || capacity == 0 ||
        !d_scratch || !d_send_hashes || !d_send_panels || !d_send_counts || !d_status)
        return fail(CSA_E_INVALID, "exchange pack: bad arguments");
    if (n_panels >= (1ull << 31)) return fail(CSA_E_UNSUPPORTED, "exchange pack: n_panels >= 2^31 (u32 indices)");
    if (scratch_bytes < csa_exchange_scratch_bytes(n_panels))
        return fail(CSA_E_INVALID, "exchange pack: scratch_bytes < csa_exchange_scratch_bytes(n_panels)");
    const hipStream_t st = (hipStream_t)stream;
    unsigned long long *rep_count = reinterpret_cast<unsigned long long *>(d_scratch);
    uint32_t *rep = reinterpret_cast<uint32_t *>(rep_count + 1);
    uint32_t *part = rep + ((std::max<uint64_t>(n_panels, 1) + 1) & ~1ull);  // 8-byte aligned
    HIPCHK(hipMemsetAsync(rep_count, 0, 8, st));
    HIPCHK(hipMemsetAsync(d_send_counts, 0, (size_t)world * 8, st));
    if (n_panels == 0) return CSA_OK;
    // 1. the local distinct panels (exact: hash AND bitmask), their indices into rep[]
    UqPlan q;
    uq_plan(n_panels, q);
    if (q.fits) {
        int rc = uq_partitioned(d_hashes, d_panels, n_panels, W, q, part, nullptr, d_status, 0, nullptr, rep, rep_count,
                                st);
        if (rc) return rc;
    } else {  // beyond the partitioned path: one global table, first-seen indices listed in rep[]
        const uint64_t slots = pow2_at_least(std::max<uint64_t>(2 * n_panels, 64));
        unsigned long long *table = reinterpret_cast<unsigned long long *>(part);
        HIPCHK(hipMemsetAsync(table, 0, slots * 8, st));
        hipLaunchKernelGGL(unique_kernel, dim3((unsigned)((n_panels + 255) / 256)), dim3(256), 0, st, d_hashes, d_panels,
                           n_panels, W, table, slots - 1, nullptr, 0u, nullptr, rep, rep_count);
        HIPCHK(hipGetLastError());
    }
    // 2. bucket them by owner into the fixed-capacity segments
    const unsigned grid = (unsigned)((n_panels + kXbThreads - 1) / kXbThreads);
    hipLaunchKernelGGL(exchange_bucket_kernel, dim3(grid), dim3(kXbThreads), 0, st, d_hashes, d_panels, W, rep,
                       rep_count, world, capacity, d_send_hashes, d_send_panels,
                       reinterpret_cast<unsigned long long *>(d_send_counts), d_status);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

int csa_exchange_keys_async(const uint64_t *d_hashes, const uint64_t *d_panels, uint64_t n_panels, int32_t W,
                            uint64_t panel_begin, uint32_t world, uint64_t capacity, void *d_scratch,
                            uint64_t scratch_bytes, uint64_t *d_send_keys, uint64_t *d_send_counts, uint32_t *d_status,
                            void *stream) {
    if (!d_hashes || !d_panels || W <= 0 || world == 0 || world > (uint32_t)kMaxWorld || capacity == 0 ||
        !d_scratch || !d_send_keys || !d_send_counts || !d_status)
        return fail(CSA_E_INVALID, "exchange keys: bad arguments");
    if (n_panels >= (1ull << 31)) return fail(CSA_E_UNSUPPORTED, "exchange keys: n_panels >= 2^31 (u32 indices)");
    if (scratch_bytes < csa_exchange_scratch_bytes(n_panels))
        return fail(CSA_E_INVALID, "exchange keys: scratch_bytes < csa_exchange_scratch_bytes(n_panels)");
    const hipStream_t st = (hipStream_t)stream;
    unsigned long long *rep_count = reinterpret_cast<unsigned long long *>(d_scratch);
    uint32_t *rep = reinterpret_cast<uint32_t *>(rep_count + 1);
    uint32_t *part = rep + ((std::max<uint64_t>(n_panels, 1) + 1) & ~1ull);
    HIPCHK(hipMemsetAsync(rep_count, 0, 8, st));
    HIPCHK(hipMemsetAsync(d_send_counts, 0, (size_t)world * 8, st));
    if (n_panels == 0) return CSA_OK;
    UqPlan q;
    uq_plan(n_panels, q);
    if (q.fits) {
        int rc = uq_partitioned(d_hashes, d_panels, n_panels, W, q, part, nullptr, d_status, 0, nullptr, rep, rep_count,
                                st);
        if (rc) return rc;
    } else {
        const uint64_t slots = pow2_at_least(std::max<uint64_t>(2 * n_panels, 64));
        unsigned long long *table = reinterpret_cast<unsigned long long *>(part);
        HIPCHK(hipMemsetAsync(table, 0, slots * 8, st));
        hipLaunchKernelGGL(unique_kernel, dim3((unsigned)((n_panels + 255) / 256)), dim3(256), 0, st, d_hashes, d_panels,
                           n_panels, W, table, slots - 1, nullptr, 0u, nullptr, rep, rep_count);
        HIPCHK(hipGetLastError());
    }
    const unsigned grid = (unsigned)((n_panels + kXbThreads - 1) / kXbThreads);
    hipLaunchKernelGGL(exchange_keys_kernel, dim3(grid), dim3(kXbThreads), 0, st, d_hashes, rep, rep_count, panel_begin,
                       world, capacity, d_send_keys, reinterpret_cast<unsigned long long *>(d_send_counts), d_status);
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

// owner scratch: table | list (2 n) | list_len | re-drawn rows (2 n x W) | table2
static void unique_keys_layout(uint64_t n_keys, int32_t W, uint64_t &slots, uint64_t &slots2, uint64_t &words) {
    const uint64_t n = std::max<uint64_t>(n_keys, 1);
    slots = pow2_at_least(std::max<uint64_t>(2 * n, 64));
    slots2 = slots;
    words = slots + 2 * n + 1 + 2 * n * (uint64_t)std::max(W, 1) + slots2;
}

uint64_t csa_unique_keys_scratch_bytes(uint64_t n_keys, int32_t W) {
    uint64_t slots, slots2, words;
    unique_keys_layout(n_keys, W, slots, slots2, words);
    return 8 * words;
}

int csa_unique_keys_async(const csa_instance *I, int32_t k, uint64_t seed, uint32_t max_attempts, const uint64_t *d_keys,
                          uint32_t n_segments, uint64_t capacity, const uint64_t *d_seg_counts, void *d_scratch,
                          uint64_t scratch_bytes, uint64_t *d_unique, uint32_t *d_status, void *stream) {
    if (!I || !d_keys || !d_seg_counts || !d_scratch || !d_unique || !d_status || capacity == 0 ||
        capacity > 0xFFFFFFFFull || n_segments == 0)
        return fail(CSA_E_INVALID, "unique keys: bad arguments");
    const uint64_t total = (uint64_t)n_segments * capacity;
    const int W = I->W;
    if (scratch_bytes < csa_unique_keys_scratch_bytes(total, W))
        return fail(CSA_E_INVALID, "unique keys: scratch_bytes < csa_unique_keys_scratch_bytes");
    uint64_t slots, slots2, words;
    unique_keys_layout(total, W, slots, slots2, words);
    uint64_t *base = static_cast<uint64_t *>(d_scratch);
    unsigned long long *table = reinterpret_cast<unsigned long long *>(base);
    uint64_t *list = base + slots;
    unsigned long long *list_len = reinterpret_cast<unsigned long long *>(list + 2 * total);
    uint64_t *rows = list + 2 * total + 1;
    unsigned long long *table2 = reinterpret_cast<unsigned long long *>(rows + 2 * total * (uint64_t)W);
    const hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipMemsetAsync(table, 0, slots * 8, st));
    HIPCHK(hipMemsetAsync(list_len, 0, 8, st));
    HIPCHK(hipMemsetAsync(table2, 0, slots2 * 8, st));
    const unsigned grid = (unsigned)((total + 255) / 256);
    hipLaunchKernelGGL(key_unique_kernel, dim3(grid), dim3(256), 0, st, d_keys, total, (uint32_t)capacity, d_seg_counts,
                       table, slots - 1, reinterpret_cast<unsigned long long *>(d_unique), list, list_len, total,
                       d_status);
    HIPCHK(hipGetLastError());
    // re-draw the listed panels (a persistent index-list draw: workgroups past the list leave at once)
    int rc = launch_draw(I, k, seed, 0, 2 * total, max_attempts, 0, 0, rows, nullptr, nullptr, nullptr, d_status,
                         nullptr, nullptr, nullptr, st, nullptr, list, list_len);
    if (rc) return rc;
    hipLaunchKernelGGL(key_verify_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, (const uint64_t *)rows,
                       W, (const unsigned long long *)list_len, table2, slots2 - 1,
                       reinterpret_cast<unsigned long long *>(d_unique));
    HIPCHK(hipGetLastError());
    return CSA_OK;
}

// analysis.py:174-176: sum(min) <= k <= sum(max) in every category
static int check_quotas(const csa_instance *I, int32_t k) {
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
    return CSA_OK;
}

// Every exit of a sample call leaves the instance's streams idle, so the next call may reuse the
// buffers; a batch above kSampleKeepBytes of device memory frees its buffers again.
static void sample_drain(csa_instance *I) {
    ScopedDevice sd(I->device);
    if (I->sdraw) (void)hipStreamSynchronize(I->sdraw);
    if (I->spost) (void)hipStreamSynchronize(I->spost);
    size_t held = 0;
    for (int j = kSampleSlot0; j < kScratchSlots; ++j) held += I->scratch_bytes[j];
    if (held > kSampleKeepBytes)
        for (int j = kSampleSlot0; j < kScratchSlots; ++j)
            if (I->scratch[j]) {
                (void)hipFree(I->scratch[j]);
                I->scratch[j] = nullptr;
                I->scratch_bytes[j] = 0;
            }
}

// device results of one enqueued batch (instance scratch; valid until the next call)
struct SampleRun {
    uint64_t *panels = nullptr, *hashes = nullptr, *table = nullptr, *uniq = nullptr;
    int64_t *counts = nullptr, *pairs = nullptr;
    uint32_t *attempts = nullptr, *status = nullptr;
    uint64_t slots = 0;
    int next_slot = kSampleSlot0;  // first instance scratch slot the batch left free
};

// Enqueue one batch on the instance's two streams, no host synchronisation.  Chunked pipeline:
// chunk c + 1 is drawn (sdraw) while chunk c is transposed, counted and paired (spost); panels and
// hashes hold the whole batch, XT and the pair scratch one chunk.  count_unique: the exact distinct
// count into r.uniq (else only the hashes are written, for the caller's own dedupe).  On return
// spost is ordered after every draw.
static int sample_enqueue(csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                          uint32_t flags, uint32_t max_attempts, bool want_attempts, bool count_unique,
                          SampleRun &r) {
    const int n = I->n, W = I->W;
    const int npad = csa_xt_pad(std::max(n, 1));
    uint64_t chunk = kSampleChunk;
    if (const char *e = getenv("CSA_SAMPLE_CHUNK")) chunk = std::max<uint64_t>(64, strtoull(e, nullptr, 10));
    chunk = std::min(chunk, std::max<uint64_t>(n_panels, 1));
    const uint64_t cblk = (chunk + 63) / 64;
    if (!I->sdraw) HIPCHK(hipStreamCreateWithFlags(&I->sdraw, hipStreamNonBlocking));
    if (!I->spost) HIPCHK(hipStreamCreateWithFlags(&I->spost, hipStreamNonBlocking));
    if (!I->drawn) HIPCHK(hipEventCreateWithFlags(&I->drawn, hipEventDisableTiming));
    hipStream_t sdraw = I->sdraw, spost = I->spost;
    int rc;
    const bool want_hashes = flags & CSA_WANT_UNIQUE, want_pairs = flags & CSA_WANT_PAIRS;
    const bool want_counts = flags & CSA_WANT_COUNTS;
    r.slots = pow2_at_least(std::max<uint64_t>(2 * n_panels, 64));
    const uint64_t sb = want_pairs ? csa_pair_scratch_bytes(n, cblk, CSA_PAIR_FP4) : 0;
    uint64_t *xt = nullptr;
    int32_t *pscratch = nullptr;
    int &sl = r.next_slot;
    if ((rc = scratch(I, sl++, std::max<uint64_t>(n_panels, 1) * W, &r.panels)) ||
        (rc = scratch(I, sl++, 4, &r.status)))
        return rc;
    if (want_hashes && (rc = scratch(I, sl++, 2 * std::max<uint64_t>(n_panels, 1), &r.hashes))) return rc;
    if (want_hashes && count_unique &&
        ((rc = scratch(I, sl++, r.slots, &r.table)) || (rc = scratch(I, sl++, 1, &r.uniq))))
        return rc;
    if (want_attempts && (rc = scratch(I, sl++, std::max<uint64_t>(n_panels, 1), &r.attempts))) return rc;
    if ((want_counts || want_pairs) && (rc = scratch(I, sl++, (size_t)n, &r.counts))) return rc;
    if (want_pairs && ((rc = scratch(I, sl++, cblk * npad, &xt)) || (rc = scratch(I, sl++, (size_t)n * n, &r.pairs)) ||
                       (rc = scratch(I, sl++, sb / sizeof(int32_t) + 1, &pscratch))))
        return rc;
    HIPCHK(hipMemsetAsync(r.status, 0, 16, sdraw));
    if (r.counts) HIPCHK(hipMemsetAsync(r.counts, 0, (size_t)n * 8, spost));
    if (r.uniq) HIPCHK(hipMemsetAsync(r.uniq, 0, 8, spost));
    for (uint64_t off = 0; off < n_panels; off += chunk) {
        const uint64_t len = std::min(chunk, n_panels - off);
        uint64_t *cp = r.panels + off * W;
        // the draw also writes the panels' 128-bit hashes (picks_pack_kernel / draw_kernel)
        if ((rc = launch_draw(I, k, seed, panel_begin + off, len, max_attempts, 0, 0, cp,
                              r.hashes ? r.hashes + 2 * off : nullptr, r.attempts ? r.attempts + off : nullptr,
                              nullptr, r.status, nullptr, nullptr, nullptr, sdraw)))
            return rc;
        HIPCHK(hipEventRecord(I->drawn, sdraw));
        HIPCHK(hipStreamWaitEvent(spost, I->drawn, 0));
        if (r.counts && (rc = csa_transpose_count_async(cp, len, n, xt, r.counts, spost))) return rc;
        // the first chunk stores its pair counts (no n*n zero-fill), later chunks add theirs
        if (r.pairs && (rc = csa_pair_counts_ex_async(xt, (len + 63) / 64, n, r.pairs,
                                                      CSA_PAIR_FP4 | (off == 0 ? CSA_PAIR_OVERWRITE : 0u), pscratch,
                                                      sb, spost)))
            return rc;
    }
    if (r.pairs && n_panels == 0) HIPCHK(hipMemsetAsync(r.pairs, 0, (size_t)n * n * 8, spost));
    HIPCHK(hipEventRecord(I->drawn, sdraw));
    HIPCHK(hipStreamWaitEvent(spost, I->drawn, 0));
    if (r.uniq && (rc = csa_unique_async(r.hashes, r.panels, n_panels, W, r.table, r.slots, r.uniq, r.status, spost)))
        return rc;
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
    int rc = check_quotas(I, k);
    if (rc) return rc;
    ScopedDevice sd(I->device);
    struct Drain {
        csa_instance *I;
        ~Drain() { sample_drain(I); }
    } drain{I};
    SampleRun r;
    if ((rc = sample_enqueue(I, k, seed, panel_begin, n_panels, flags, max_attempts, attempts_out != nullptr, true, r)))
        return rc;
    const hipStream_t spost = I->spost;
    const int n = I->n, W = I->W;
    uint32_t hs[4];
    if ((rc = read_status(r.status, spost, hs))) return rc;
    if ((rc = csa_status_decode(hs))) return rc;
    if (flags & CSA_WANT_PANELS)
        HIPCHK(hipMemcpyAsync(panels_out, r.panels, n_panels * W * 8, hipMemcpyDeviceToHost, spost));
    if (flags & CSA_WANT_COUNTS)
        HIPCHK(hipMemcpyAsync(person_counts, r.counts, (size_t)n * 8, hipMemcpyDeviceToHost, spost));
    if (flags & CSA_WANT_PAIRS)
        HIPCHK(hipMemcpyAsync(pair_counts, r.pairs, (size_t)n * n * 8, hipMemcpyDeviceToHost, spost));
    if (flags & CSA_WANT_UNIQUE) HIPCHK(hipMemcpyAsync(unique_out, r.uniq, 8, hipMemcpyDeviceToHost, spost));
    if (attempts_out) HIPCHK(hipMemcpyAsync(attempts_out, r.attempts, n_panels * 4, hipMemcpyDeviceToHost, spost));
    HIPCHK(hipStreamSynchronize(spost));
    return CSA_OK;
}

// The instance's copy on device `dev` for shard s of csa_legacy_sample_devices (shard 0 on the
// instance's own device is the instance itself).  A replica mirrors the instance's draw state and
// address rings as of the last csa_instance_set_state / csa_instance_set_address (generation).
static int shard_instance(csa_instance *I, int s, int dev, csa_instance **out) {
    if (s == 0 && dev == I->device) {
        *out = I;
        return CSA_OK;
    }
    if ((int)I->replicas.size() <= s) {
        I->replicas.resize(s + 1, nullptr);
        I->replica_gen.resize(s + 1, 0);
    }
    csa_instance *&R = I->replicas[s];
    if (R && R->device != dev) {
        csa_instance_destroy(R);
        R = nullptr;
    }
    int rc;
    if (!R) {
        ScopedDevice sd(dev);
        if ((rc = csa_instance_create(I->n, I->C, I->F, I->pf.data(), I->fmin.data(), I->fmax.data(), I->fcat.data(),
                                      &R)))
            return rc;
        I->replica_gen[s] = 0;
    }
    if (I->replica_gen[s] != I->gen) {
        if ((rc = csa_instance_set_state(R, I->sel0.data(), I->rem0h.empty() ? nullptr : I->rem0h.data(),
                                         I->present0h.empty() ? nullptr : I->present0h.data())) ||
            (rc = csa_instance_set_address(R, I->addr_h.empty() ? nullptr : I->addr_h.data())))
            return rc;
        I->replica_gen[s] = I->gen;
    }
    *out = R;
    return CSA_OK;
}

// Scratch slots of the multi-device combine (above the batch's own, kSampleSlot0..)
constexpr int kShardSlot0 = 20, kRootSlot0 = 24;

int csa_legacy_sample_devices(csa_instance *I, const int32_t *devices, int32_t n_shards, int32_t k, uint64_t seed,
                              uint64_t panel_begin, uint64_t n_panels, uint32_t flags, uint32_t max_attempts,
                              uint64_t *panels_out, int64_t *person_counts, int64_t *pair_counts,
                              uint64_t *unique_out, uint32_t *attempts_out) {
    if (!I) return fail(CSA_E_INVALID, "null instance");
    if (n_shards <= 0 || n_shards > kMaxWorld) return fail(CSA_E_INVALID, "n_shards must be in [1, %d]", kMaxWorld);
    if ((flags & CSA_WANT_PANELS) && !panels_out) return fail(CSA_E_INVALID, "panels_out is NULL");
    if ((flags & CSA_WANT_COUNTS) && !person_counts) return fail(CSA_E_INVALID, "person_counts is NULL");
    if ((flags & CSA_WANT_PAIRS) && !pair_counts) return fail(CSA_E_INVALID, "pair_counts is NULL");
    if ((flags & CSA_WANT_UNIQUE) && !unique_out) return fail(CSA_E_INVALID, "unique_out is NULL");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    std::vector<int> dev(n_shards);
    for (int s = 0; s < n_shards; ++s) {
        dev[s] = devices ? devices[s] : s;
        if (dev[s] < 0 || dev[s] >= ndev)
            return fail(CSA_E_INVALID, "shard %d: device %d outside [0, %d)", s, dev[s], ndev);
    }
    int rc = check_quotas(I, k);
    if (rc) return rc;
    const int n = I->n, W = I->W;
    std::vector<csa_instance *> R(n_shards, nullptr);
    for (int s = 0; s < n_shards; ++s)
        if ((rc = shard_instance(I, s, dev[s], &R[s]))) return rc;
    struct DrainAll {
        std::vector<csa_instance *> &R;
        ~DrainAll() {
            for (csa_instance *x : R)
                if (x) sample_drain(x);
        }
    } drain{R};
    // 1. every shard draws, counts and pairs its contiguous panel range and reduces it to its exact
    //    local distinct panels (csa_exchange_pack_async with one owner), all enqueued before any wait
    const bool want_unique = flags & CSA_WANT_UNIQUE, want_pairs = flags & CSA_WANT_PAIRS;
    const bool want_counts = flags & CSA_WANT_COUNTS;
    const uint32_t sflags = flags & (CSA_WANT_COUNTS | CSA_WANT_PAIRS | CSA_WANT_UNIQUE);
    std::vector<uint64_t> b(n_shards + 1);
    for (int s = 0; s <= n_shards; ++s) b[s] = n_panels * (uint64_t)s / (uint64_t)n_shards;
    uint64_t cap = 1;
    for (int s = 0; s < n_shards; ++s) cap = std::max(cap, b[s + 1] - b[s]);
    std::vector<SampleRun> run(n_shards);
    std::vector<uint64_t *> sh(n_shards, nullptr), sp(n_shards, nullptr), sc(n_shards, nullptr);
    for (int s = 0; s < n_shards; ++s) {
        csa_instance *X = R[s];
        ScopedDevice sd(X->device);
        const uint64_t len = b[s + 1] - b[s];
        if ((rc = sample_enqueue(X, k, seed, panel_begin + b[s], len, sflags, max_attempts, attempts_out != nullptr,
                                 false, run[s])))
            return rc;
        if (!want_unique) continue;
        const uint64_t xb = csa_exchange_scratch_bytes(len);
        void *xs = nullptr;
        if ((rc = scratch(X, kShardSlot0, 2 * cap, &sh[s])) || (rc = scratch(X, kShardSlot0 + 1, cap * W, &sp[s])) ||
            (rc = scratch(X, kShardSlot0 + 2, 1, &sc[s])) ||
            (rc = scratch(X, kShardSlot0 + 3, xb, reinterpret_cast<uint8_t **>(&xs))))
            return rc;
        if ((rc = csa_exchange_pack_async(run[s].hashes, run[s].panels, len, W, 1, cap, xs, xb, sh[s], sp[s], sc[s],
                                          run[s].status, X->spost)))
            return rc;
    }
    // 2. every shard's status, its panels / attempts straight into the caller's buffers
    for (int s = 0; s < n_shards; ++s) {
        csa_instance *X = R[s];
        ScopedDevice sd(X->device);
        const uint64_t len = b[s + 1] - b[s];
        uint32_t hs[4];
        if ((rc = read_status(run[s].status, X->spost, hs))) return rc;
        if ((rc = csa_status_decode(hs))) return rc;
        if ((flags & CSA_WANT_PANELS) && len)
            HIPCHK(hipMemcpyAsync(panels_out + b[s] * W, run[s].panels, len * W * 8, hipMemcpyDeviceToHost, X->spost));
        if (attempts_out && len)
            HIPCHK(hipMemcpyAsync(attempts_out + b[s], run[s].attempts, len * 4, hipMemcpyDeviceToHost, X->spost));
    }
    // 3. combine on shard 0's device: counts and pairs summed (peer copies over xGMI + one add
    //    kernel per shard), the local distinct sets gathered as segments and counted exactly
    //    (hash AND bitmask) by csa_unique_segments_async
    csa_instance *X0 = R[0];
    ScopedDevice sd0(X0->device);
    const hipStream_t st = X0->spost;
    const size_t nn = want_pairs ? (size_t)n * n : 0, nc = (want_counts || want_pairs) ? (size_t)n : 0;
    int64_t *tmp = nullptr;
    if (n_shards > 1 && nc && (rc = scratch(X0, kRootSlot0, nc + nn, &tmp))) return rc;
    uint64_t *gh = nullptr, *gp = nullptr, *gc = nullptr, *table = nullptr, *uniq = nullptr;
    const uint64_t total = (uint64_t)n_shards * cap, slots = pow2_at_least(std::max<uint64_t>(2 * total, 64));
    if (want_unique &&
        ((rc = scratch(X0, kRootSlot0 + 1, 2 * total, &gh)) || (rc = scratch(X0, kRootSlot0 + 2, total * W, &gp)) ||
         (rc = scratch(X0, kRootSlot0 + 3, (size_t)n_shards, &gc)) || (rc = scratch(X0, kRootSlot0 + 4, slots, &table)) ||
         (rc = scratch(X0, kRootSlot0 + 5, 1, &uniq))))
        return rc;
    for (int s = 0; s < n_shards; ++s) {
        const int d = R[s]->device;
        if (s > 0 && nc) {
            HIPCHK(hipMemcpyPeerAsync(tmp, X0->device, run[s].counts, d, nc * 8, st));
            if (nn) HIPCHK(hipMemcpyPeerAsync(tmp + nc, X0->device, run[s].pairs, d, nn * 8, st));
            // counts and pairs are adjacent in tmp but not in the shard-0 buffers: two adds
            hipLaunchKernelGGL(add_i64_kernel, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, st, run[0].counts,
                               (const int64_t *)tmp, (uint64_t)nc);
            if (nn)
                hipLaunchKernelGGL(add_i64_kernel, dim3((unsigned)std::min<uint64_t>((nn + 255) / 256, 65536)), dim3(256),
                                   0, st, run[0].pairs, (const int64_t *)(tmp + nc), (uint64_t)nn);
            HIPCHK(hipGetLastError());
        }
        if (want_unique) {
            HIPCHK(hipMemcpyPeerAsync(gh + 2 * cap * s, X0->device, sh[s], d, 2 * cap * 8, st));
            HIPCHK(hipMemcpyPeerAsync(gp + cap * W * s, X0->device, sp[s], d, cap * W * 8, st));
            HIPCHK(hipMemcpyPeerAsync(gc + s, X0->device, sc[s], d, 8, st));
        }
    }
    if (want_unique) {
        HIPCHK(hipMemsetAsync(uniq, 0, 8, st));
        if ((rc = csa_unique_segments_async(gh, gp, (uint32_t)n_shards, cap, gc, W, table, slots, uniq, run[0].status,
                                            st)))
            return rc;
    }
    uint32_t hs[4];
    if ((rc = read_status(run[0].status, st, hs))) return rc;
    if ((rc = csa_status_decode(hs))) return rc;
    if (want_counts) HIPCHK(hipMemcpyAsync(person_counts, run[0].counts, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    if (want_pairs) HIPCHK(hipMemcpyAsync(pair_counts, run[0].pairs, nn * 8, hipMemcpyDeviceToHost, st));
    if (want_unique) HIPCHK(hipMemcpyAsync(unique_out, uniq, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return CSA_OK;
}

int csa_first_panel_not_in(csa_instance *I, int32_t k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                           uint32_t max_attempts, const uint64_t *portfolio, uint64_t m, uint64_t chunk,
                           int64_t *index_out, uint64_t *panel_out) {
    if (!I || !index_out || !panel_out || (m && !portfolio)) return fail(CSA_E_INVALID, "first_panel_not_in: bad arguments");
    *index_out = -1;
    if (n_panels == 0) return CSA_OK;
    ScopedDevice sd(I->device);
    const int W = I->W;
    if (chunk == 0) chunk = 256;
    if (!I->stream) HIPCHK(hipStreamCreateWithFlags(&I->stream, hipStreamNonBlocking));
    hipStream_t st = I->stream;
    const uint64_t cap = std::min(n_panels, std::max<uint64_t>(chunk, 1) << 12);  // largest chunk
    const uint64_t slots = pow2_at_least(std::max<uint64_t>(2 * m, 64));
    uint64_t *pport, *phash, *table, *cnt, *panels, *hashes, *first;
    uint32_t *status;
    int rc;
    if ((rc = scratch(I, 0, std::max<uint64_t>(m, 1) * W, &pport)) ||
        (rc = scratch(I, 1, 2 * std::max<uint64_t>(m, 1), &phash)) || (rc = scratch(I, 2, slots, &table)) ||
        (rc = scratch(I, 3, 2, &cnt)) || (rc = scratch(I, 4, cap * W, &panels)) ||
        (rc = scratch(I, 5, 2 * cap, &hashes)) || (rc = scratch(I, 6, 1, &first)) ||
        (rc = scratch(I, 7, 4, &status)))
        return rc;
    HIPCHK(hipMemsetAsync(table, 0, slots * 8, st));
    if (m) {  // portfolio table: panel_hash_kernel + unique_kernel insertion (exact)
        HIPCHK(hipMemcpyAsync(pport, portfolio, m * W * 8, hipMemcpyHostToDevice, st));
        if ((rc = csa_panel_hash_async(pport, m, W, phash, st))) return rc;
        HIPCHK(hipMemsetAsync(cnt, 0, 8, st));
        if ((rc = csa_unique_async(phash, pport, m, W, table, slots, cnt, nullptr, st))) return rc;
    }
    // chunks of growing size: the expected first non-member is near the start
    uint64_t done = 0, len = std::min(chunk, n_panels);
    while (done < n_panels) {
        len = std::min(len, n_panels - done);
        HIPCHK(hipMemsetAsync(status, 0, 16, st));
        HIPCHK(hipMemsetAsync(first, 0xFF, 8, st));
        if ((rc = launch_draw(I, k, seed, panel_begin + done, len, max_attempts, 0, 0, panels, hashes, nullptr,
                              nullptr, status, nullptr, nullptr, nullptr, st)))
            return rc;
        hipLaunchKernelGGL(member_scan_kernel, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, st, hashes,
                           panels, len, W, reinterpret_cast<const unsigned long long *>(table), slots - 1,
                           phash, pport, reinterpret_cast<unsigned long long *>(first));
        HIPCHK(hipGetLastError());
        uint32_t hs[4];
        if ((rc = read_status(status, st, hs))) return rc;
        if (hs[0] != 0u) {
            // a draw error (KeyError / attempt limit) at panel e: the reference meets it only if
            // every panel before e is a member, so re-scan the panels before e first (the error
            // stops other groups, leaving later panels of this chunk undrawn)
            const uint64_t e = (uint64_t)hs[1] | ((uint64_t)hs[2] << 32), start = panel_begin + done;
            if (e > start && e < start + len) {
                len = e - start;
                continue;
            }
            return csa_status_decode(hs);
        }
        uint64_t f = 0;
        HIPCHK(hipMemcpyAsync(&f, first, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (f != ~0ull) {
            HIPCHK(hipMemcpyAsync(panel_out, panels + f * W, (size_t)W * 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            *index_out = (int64_t)(done + f);
            return CSA_OK;
        }
        done += len;
        len = std::min<uint64_t>(len * 2, cap);
    }
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
