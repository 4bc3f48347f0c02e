// legacy_mt.cpp -- MT19937 mode of the LEGACY draw, host code.
//
// The reference draws from the global stdlib `random` stream: random.seed(seed) at
// analysis.py:169, random.randint(1, remaining) at EVERY improvement of the argmax in
// find_max_ratio_cat (legacy.py:149), one stream across restarts and panels.  That stream is
// sequential -- how many words a step consumes depends on every earlier step -- so this mode
// runs on the host, one panel after another; it reproduces the reference's published
// probabilities (reference_output/*_ratio_product_data.csv) bit for bit.  The device path uses
// the Philox verification-mode stream instead (oracle/philox.py contract).
//
// The generator state is CPython's own (random.getstate()[1]: 624 words + the position), so
// the Python layer seeds with the stdlib and hands the state over; this file only advances it:
//   getrandbits(k <= 32) = genrand_uint32() >> (32 - k)             (Modules/_randommodule.c)
//   randint(a, b) = a + _randbelow(b - a + 1), _randbelow(m): k = m.bit_length(), draw
//   getrandbits(k) until < m                                         (Lib/random.py)
// Step semantics follow legacy.py:124-200 with every SelectionError raised where the reference
// raises it, so that no randint call is consumed past it:
//   * find_max_ratio_cat: features in CSV order; the FAIL test (selected < min and remaining <
//     min - selected) stops the scan at that feature; candidates (remaining != 0, max != 0)
//     compare (min - selected) / remaining against the best with strict '>' from -100.0 (exact
//     cross-multiplication), each improvement consuming one randint(1, remaining);
//   * no candidate while people remain -> KeyError (legacy.py:188) = CSA_E_NO_CANDIDATE; no
//     candidate and nobody left -> no pick this step;
//   * the r-th remaining holder of the winner in agent order (legacy.py:186-197);
//   * delete_person + delete_all_in_cat in bulk form, then the remaining == 0 and selected < min
//     test (legacy.py:55, 73: no randint is consumed inside a step after the pick, so the order
//     of the deletions inside the step does not matter); the emptied pool (legacy.py:198-199);
//   * legacy_find (analysis.py:141-159): restart on SelectionError and on check_min_cats failure.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/csa_legacy.h"

void csa_set_last_error(const char *msg);  // csa_legacy.hip (library-internal)

namespace {

constexpr int kMtN = 624, kMtM = 397;

struct Mt {
    uint32_t *mt;   // 624 words
    uint32_t *idx;  // position
    uint32_t next() {
        static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
        uint32_t y;
        if (*idx >= (uint32_t)kMtN) {
            int kk;
            for (kk = 0; kk < kMtN - kMtM; kk++) {
                y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
                mt[kk] = mt[kk + kMtM] ^ (y >> 1) ^ mag01[y & 1u];
            }
            for (; kk < kMtN - 1; kk++) {
                y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
                mt[kk] = mt[kk + (kMtM - kMtN)] ^ (y >> 1) ^ mag01[y & 1u];
            }
            y = (mt[kMtN - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
            mt[kMtN - 1] = mt[kMtM - 1] ^ (y >> 1) ^ mag01[y & 1u];
            *idx = 0;
        }
        y = mt[(*idx)++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    // random.randint(1, m) for 1 <= m < 2^31
    int randint1(uint32_t m) {
        int k = 0;
        while ((m >> k) != 0u) ++k;  // m.bit_length()
        uint32_t r;
        do {
            r = next() >> (32 - k);
        } while (r >= m);
        return 1 + (int)r;
    }
};

enum { kOk = 0, kFail = 1, kNoCand = 2 };

struct Inst {
    int n, C, F, W;
    const int32_t *pf, *fmin, *fmax;
    const int32_t *addr_next;    // same-address ring (check_same_address) or null
    std::vector<uint64_t> rows;  // F x W feature bitmasks
};

// one find_random_sample_legacy call (legacy.py:178-200) from (sel, rem, pool); picks in pick order
int attempt(const Inst &I, int k, Mt &rng, std::vector<int32_t> &sel, std::vector<int32_t> &rem,
            std::vector<uint64_t> &pool, std::vector<int32_t> &picks) {
    const int F = I.F, W = I.W, C = I.C;
    picks.clear();
    for (int step = 0; step < k; ++step) {
        int64_t bn = -100, bd = 1;
        int fs = -1, r = -1;
        for (int f = 0; f < F; ++f) {
            const int64_t need = (int64_t)I.fmin[f] - sel[f];
            if (sel[f] < I.fmin[f] && rem[f] < need) return kFail;  // legacy.py:132-137
            if (rem[f] != 0 && I.fmax[f] != 0) {                     // legacy.py:140
                if (need > rem[f]) return kFail;                     // ratio > 1, legacy.py:143-144
                if (need * bd > bn * rem[f]) {                       // strict '>', legacy.py:145
                    bn = need;
                    bd = rem[f];
                    fs = f;
                    r = rng.randint1((uint32_t)rem[f]);              // legacy.py:149
                }
            }
        }
        bool any = false;
        for (int w = 0; w < W; ++w) any |= pool[w] != 0ull;
        if (fs < 0) {
            if (any) return kNoCand;  // pvalue[""]: KeyError, legacy.py:188
        } else {
            int p = -1;  // r-th remaining holder of fs in agent order
            for (int w = 0; w < W && p < 0; ++w) {
                uint64_t m = pool[w] & I.rows[(size_t)fs * W + w];
                const int c = __builtin_popcountll(m);
                if (r > c) {
                    r -= c;
                    continue;
                }
                while (--r > 0) m &= m - 1;
                p = w * 64 + __builtin_ctzll(m);
            }
            if (p >= 0) {
                picks.push_back(p);
                pool[p >> 6] &= ~(1ull << (p & 63));
                const int32_t *pfp = I.pf + (size_t)p * C;
                for (int c = 0; c < C; ++c) {  // really_delete_person(selected=True)
                    ++sel[pfp[c]];
                    --rem[pfp[c]];
                }
                // check_same_address (legacy.py:109-113): everyone left at the pick's address is
                // deleted with really_delete_person(selected=False), before the cascades
                if (I.addr_next)
                    for (int q = I.addr_next[p]; q != p; q = I.addr_next[q])
                        if ((pool[q >> 6] >> (q & 63)) & 1ull) {
                            pool[q >> 6] &= ~(1ull << (q & 63));
                            const int32_t *pq = I.pf + (size_t)q * C;
                            for (int c = 0; c < C; ++c) --rem[pq[c]];
                        }
                // delete_all_in_cat for every full feature of the pick, bulk form
                std::vector<uint64_t> del(W, 0ull);
                bool cascade = false;
                for (int c = 0; c < C; ++c) {
                    const int g = pfp[c];
                    if (sel[g] == I.fmax[g]) {
                        cascade = true;
                        for (int w = 0; w < W; ++w) del[w] |= I.rows[(size_t)g * W + w];
                    }
                }
                if (cascade)
                    for (int w = 0; w < W; ++w) {
                        uint64_t d = del[w] & pool[w];
                        pool[w] &= ~d;
                        while (d) {
                            const int q = w * 64 + __builtin_ctzll(d);
                            d &= d - 1;
                            const int32_t *pq = I.pf + (size_t)q * C;
                            for (int c = 0; c < C; ++c) --rem[pq[c]];
                        }
                    }
                for (int g = 0; g < F; ++g)  // legacy.py:55, 73
                    if (rem[g] == 0 && sel[g] < I.fmin[g]) return kFail;
            }
        }
        if (step < k - 1) {  // legacy.py:198-199
            bool left = false;
            for (int w = 0; w < W; ++w) left |= pool[w] != 0ull;
            if (!left) return kFail;
        }
    }
    return kOk;
}

int fail(int code, const std::string &msg) {
    csa_set_last_error(msg.c_str());  // csa_legacy.hip: the thread-local csa_last_error() message
    return code;
}

}  // namespace

extern "C" {

int csa_legacy_draw_mt(int32_t n, int32_t C, int32_t F, const int32_t *person_feat, const int32_t *fmin,
                       const int32_t *fmax, const int32_t *sel0, const int32_t *rem0, const uint64_t *present0,
                       const int32_t *addr_next, int32_t k, uint32_t *mt_state, uint64_t n_panels,
                       uint32_t max_attempts, int32_t single, int32_t *picks_out, uint64_t *panels_out,
                       uint32_t *attempts_out, int32_t *sel_out, int32_t *rem_out, uint64_t *present_out,
                       uint64_t *stats_out) {
    if (stats_out) stats_out[0] = stats_out[1] = stats_out[2] = 0;
    if (n < 0 || C <= 0 || F <= 0 || k < 0 || !person_feat || !fmin || !fmax || !mt_state ||
        mt_state[kMtN] > (uint32_t)kMtN) {
        return fail(CSA_E_INVALID, "draw_mt: bad arguments");
    }
    Inst I;
    I.n = n;
    I.C = C;
    I.F = F;
    I.W = (n + 63) / 64;
    I.pf = person_feat;
    I.fmin = fmin;
    I.fmax = fmax;
    I.addr_next = addr_next;
    if (addr_next)
        for (int p = 0; p < n; ++p)
            if (addr_next[p] < 0 || addr_next[p] >= n) return fail(CSA_E_INVALID, "draw_mt: addr_next out of range");
    I.rows.assign((size_t)F * I.W, 0ull);
    std::vector<int32_t> pool0(F, 0);
    for (int p = 0; p < n; ++p)
        for (int c = 0; c < C; ++c) {
            const int g = person_feat[(size_t)p * C + c];
            if (g < 0 || g >= F) {
                return fail(CSA_E_INVALID, "draw_mt: feature id out of range");
            }
            I.rows[(size_t)g * I.W + (p >> 6)] |= 1ull << (p & 63);
            ++pool0[g];
        }
    std::vector<uint64_t> all(I.W, 0ull);
    for (int p = 0; p < n; ++p) all[p >> 6] |= 1ull << (p & 63);
    Mt rng{mt_state, mt_state + kMtN};
    const uint32_t cap = single ? 1u : (max_attempts ? max_attempts : 100000u);
    std::vector<int32_t> sel, rem, picks;
    std::vector<uint64_t> pool;
    for (uint64_t i = 0; i < n_panels; ++i) {
        uint32_t a = 0;
        for (;;) {
            // a fresh copy of the start state per attempt (legacy_find's deepcopy, analysis.py:147-148)
            if (sel0) sel.assign(sel0, sel0 + F);
            else sel.assign(F, 0);
            const int32_t *r0 = rem0 ? rem0 : pool0.data();
            rem.assign(r0, r0 + F);
            const uint64_t *q0 = present0 ? present0 : all.data();
            pool.assign(q0, q0 + I.W);
            const int st = attempt(I, k, rng, sel, rem, pool, picks);
            ++a;
            if (stats_out) ++stats_out[0];
            if (st == kNoCand) {
                return fail(CSA_E_NO_CANDIDATE, "panel " + std::to_string(i) +
                                                    ": no candidate feature while agents remain (KeyError, legacy.py:188)");
            }
            if (single) {
                if (st == kFail) {
                    if (stats_out) ++stats_out[1];
                    return fail(CSA_E_SELECTION, "SelectionError (legacy.py:34)");
                }
                break;
            }
            bool under = false;  // check_min_cats (legacy.py:160-168)
            for (int f = 0; f < F; ++f) under |= sel[f] < fmin[f];
            if (st == kOk && !under) break;
            if (stats_out) ++stats_out[st == kOk ? 2 : 1];  // rejection ("Rejected") / SelectionError
            if (a >= cap) {
                return fail(CSA_E_ATTEMPT_LIMIT,
                            "panel " + std::to_string(i) + ": attempt limit reached without an accepted panel");
            }
        }
        if (picks_out) {
            int32_t *row = picks_out + i * (uint64_t)k;
            for (int s = 0; s < k; ++s) row[s] = s < (int)picks.size() ? picks[s] : -1;
        }
        if (panels_out) {
            uint64_t *row = panels_out + i * (uint64_t)I.W;
            std::memset(row, 0, (size_t)I.W * 8);
            for (int p : picks) row[p >> 6] |= 1ull << (p & 63);
        }
        if (attempts_out) attempts_out[i] = a;
    }
    if (single) {
        if (sel_out) std::memcpy(sel_out, sel.data(), (size_t)F * 4);
        if (rem_out) std::memcpy(rem_out, rem.data(), (size_t)F * 4);
        if (present_out) std::memcpy(present_out, pool.data(), (size_t)I.W * 8);
    }
    return CSA_OK;
}

}  // extern "C"
