/*
 * legacy_oracle.c -- plain-C restatement of the reference LEGACY Monte Carlo
 * path, Philox verification mode.  TEST INFRASTRUCTURE ONLY: loaded by tests/
 * (as the checker) and by bench.py's cpu_baseline leg (as the timed CPU port).
 * The product library never links or calls this file.
 *
 * Restates (reference file:line):
 *   find_max_ratio_cat        legacy.py:124-157   strict '>' argmax from -100.0,
 *                                                 exact integer cross-multiplication
 *   holder scan               legacy.py:186-197   r-th remaining holder, ascending id
 *   delete_person             legacy.py:103-120   sel+=1 / rem-=1 on the picked row
 *   delete_all_in_cat         legacy.py:47-62     bulk cascade over full features
 *   find_random_sample_legacy legacy.py:178-200   k steps + empty-pool SelectionError
 *   check_min_cats            legacy.py:160-168
 *   legacy_find               analysis.py:141-159 restart / reject loop
 *   legacy_probabilities      analysis.py:162-191 counts, pairs, distinct panels
 * RNG: oracle/philox.py contract (Philox4x32-10, key=(seed), ctr=(step>>2,
 * attempt, panel), word step&3; r = 1 + ((word*rem) >> 32)).
 *
 * Pinned by tests/test_oracle_golden.py against tests/golden/philox_*.json,
 * which tools/make_goldens.py produced by driving the unmodified reference.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_OK 0
#define OR_E_INVALID 1
#define OR_E_NO_CANDIDATE 3
#define OR_E_ATTEMPT_LIMIT 4

static inline uint32_t mulhi32(uint32_t a, uint32_t b, uint32_t *lo) {
    uint64_t p = (uint64_t)a * b;
    *lo = (uint32_t)p;
    return (uint32_t)(p >> 32);
}

void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint32_t lo0, lo1;
        uint32_t hi0 = mulhi32(0xD2511F53u, c0, &lo0);
        uint32_t hi1 = mulhi32(0xCD9E8D57u, c2, &lo1);
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

typedef struct {
    int n, C, F, W;
    const int32_t *pf, *fmin, *fmax, *fcat;
    uint64_t *featmask;   /* F * W */
    int32_t *pool;        /* F */
} oinst;

/* one attempt; returns 0 accepted, 1 SelectionError, 2 min-quota rejection, -1 no candidate */
static int attempt_once(const oinst *I, int k, uint64_t seed, uint64_t panel, uint32_t attempt,
                        uint64_t *remaining, int32_t *sel, int32_t *rem, uint64_t *picked,
                        uint64_t *del, int32_t *picks) {
    const int F = I->F, W = I->W, n = I->n, C = I->C;
    memset(sel, 0, sizeof(int32_t) * F);
    memcpy(rem, I->pool, sizeof(int32_t) * F);
    memset(picked, 0, sizeof(uint64_t) * W);
    for (int w = 0; w < W; ++w) {
        int bits = n - 64 * w;
        remaining[w] = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    }
    uint32_t blk[4];
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int step = 0; step < k; ++step) {
        if ((step & 3) == 0) {
            uint32_t ctr[4] = {(uint32_t)(step >> 2), attempt, (uint32_t)panel, (uint32_t)(panel >> 32)};
            oracle_philox(ctr, key, blk);
        }
        int fs = -1;
        int64_t bn = 0, bd = 1;
        for (int f = 0; f < F; ++f) {
            int64_t need = (int64_t)I->fmin[f] - sel[f];
            if (sel[f] < I->fmin[f] && rem[f] < need) return 1;
            if (rem[f] != 0 && I->fmax[f] != 0) {
                int better = fs < 0 ? (need > -100 * (int64_t)rem[f]) : (need * bd > bn * (int64_t)rem[f]);
                if (better) { fs = f; bn = need; bd = rem[f]; }
            }
        }
        int any = 0;
        for (int w = 0; w < W; ++w) any |= remaining[w] != 0;
        if (fs < 0) {
            if (any) return -1;
        } else {
            uint64_t r = 1 + (((uint64_t)blk[step & 3] * (uint64_t)rem[fs]) >> 32);
            const uint64_t *fm = I->featmask + (size_t)fs * W;
            int p = -1;
            for (int w = 0; w < W && p < 0; ++w) {
                uint64_t m = remaining[w] & fm[w];
                uint64_t c = (uint64_t)__builtin_popcountll(m);
                if (r <= c) {
                    for (uint64_t j = 1; j < r; ++j) m &= m - 1;
                    p = 64 * w + __builtin_ctzll(m);
                } else {
                    r -= c;
                }
            }
            if (p >= 0) {
                if (picks) picks[step] = p;
                remaining[p >> 6] &= ~(1ull << (p & 63));
                picked[p >> 6] |= 1ull << (p & 63);
                const int32_t *row = I->pf + (size_t)p * C;
                int nfull = 0;
                memset(del, 0, sizeof(uint64_t) * W);
                for (int c = 0; c < C; ++c) {
                    int g = row[c];
                    sel[g] += 1;
                    rem[g] -= 1;
                }
                for (int c = 0; c < C; ++c) {
                    int g = row[c];
                    if (sel[g] == I->fmax[g]) {
                        ++nfull;
                        const uint64_t *gm = I->featmask + (size_t)g * W;
                        for (int w = 0; w < W; ++w) del[w] |= gm[w];
                    }
                }
                if (nfull) {
                    for (int w = 0; w < W; ++w) { del[w] &= remaining[w]; remaining[w] &= ~del[w]; }
                    for (int g = 0; g < F; ++g) {
                        const uint64_t *gm = I->featmask + (size_t)g * W;
                        int d = 0;
                        for (int w = 0; w < W; ++w) d += __builtin_popcountll(del[w] & gm[w]);
                        rem[g] -= d;
                    }
                }
                for (int g = 0; g < F; ++g)
                    if (rem[g] == 0 && sel[g] < I->fmin[g]) return 1;
            }
        }
        if (step < k - 1) {
            any = 0;
            for (int w = 0; w < W; ++w) any |= remaining[w] != 0;
            if (!any) return 1;
        }
    }
    for (int f = 0; f < F; ++f)
        if (sel[f] < I->fmin[f]) return 2;
    return 0;
}

int oracle_draw(int n, int C, int F, const int32_t *pf, const int32_t *fmin, const int32_t *fmax,
                const int32_t *fcat, int k, uint64_t seed, uint64_t panel_begin, uint64_t n_panels,
                uint32_t max_attempts, uint64_t *panels_out, int32_t *picks_out, uint32_t *attempts_out,
                uint32_t *rejects_out, int nthreads) {
    if (n <= 0 || C <= 0 || F <= 0 || k < 0 || !pf || !fmin || !fmax || !fcat) return OR_E_INVALID;
    oinst I;
    I.n = n; I.C = C; I.F = F; I.W = (n + 63) / 64;
    I.pf = pf; I.fmin = fmin; I.fmax = fmax; I.fcat = fcat;
    I.featmask = (uint64_t *)calloc((size_t)F * I.W, sizeof(uint64_t));
    I.pool = (int32_t *)calloc((size_t)F, sizeof(int32_t));
    for (int p = 0; p < n; ++p)
        for (int c = 0; c < C; ++c) {
            int g = pf[(size_t)p * C + c];
            if (g < 0 || g >= F || fcat[g] != c) { free(I.featmask); free(I.pool); return OR_E_INVALID; }
            I.featmask[(size_t)g * I.W + (p >> 6)] |= 1ull << (p & 63);
            I.pool[g] += 1;
        }
    int status = OR_OK;
    if (nthreads <= 0) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
    {
        const int W = I.W;
        uint64_t *remaining = (uint64_t *)malloc(sizeof(uint64_t) * W);
        uint64_t *picked = (uint64_t *)malloc(sizeof(uint64_t) * W);
        uint64_t *del = (uint64_t *)malloc(sizeof(uint64_t) * W);
        int32_t *sel = (int32_t *)malloc(sizeof(int32_t) * F);
        int32_t *rem = (int32_t *)malloc(sizeof(int32_t) * F);
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = 0; i < (int64_t)n_panels; ++i) {
            uint64_t panel = panel_begin + (uint64_t)i;
            int32_t *picks = picks_out ? picks_out + (size_t)i * k : NULL;
            uint32_t a = 0, rejects = 0;
            int rc = 1;
            for (; a < max_attempts; ++a) {
                rc = attempt_once(&I, k, seed, panel, a, remaining, sel, rem, picked, del, picks);
                if (rc == 0 || rc < 0) break;
                rejects += rc == 2;  /* check_min_cats failed: "Rejected" (analysis.py:155-159) */
            }
            if (rc < 0) {
#pragma omp atomic write
                status = OR_E_NO_CANDIDATE;
            } else if (rc != 0) {
#pragma omp atomic write
                status = OR_E_ATTEMPT_LIMIT;
            }
            if (panels_out) memcpy(panels_out + (size_t)i * W, picked, sizeof(uint64_t) * W);
            if (attempts_out) attempts_out[i] = a + 1;
            if (rejects_out) rejects_out[i] = rejects;
        }
        free(remaining); free(picked); free(del); free(sel); free(rem);
    }
    free(I.featmask);
    free(I.pool);
    return status;
}

/* per-person counts: counts[p] = number of panels containing p */
void oracle_counts(const uint64_t *panels, uint64_t S, int n, int64_t *counts) {
    const int W = (n + 63) / 64;
    memset(counts, 0, sizeof(int64_t) * n);
    for (uint64_t i = 0; i < S; ++i)
        for (int w = 0; w < W; ++w) {
            uint64_t m = panels[i * W + w];
            while (m) { counts[64 * w + __builtin_ctzll(m)] += 1; m &= m - 1; }
        }
}

/* pair counts (full symmetric n x n, diagonal = counts) */
void oracle_pairs(const uint64_t *panels, uint64_t S, int n, int64_t *pairs, int nthreads) {
    const int W = (n + 63) / 64;
    memset(pairs, 0, sizeof(int64_t) * (size_t)n * n);
    if (nthreads <= 0) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 4)
    for (int i = 0; i < n; ++i) {
        int64_t *row = pairs + (size_t)i * n;
        const uint64_t bi = 1ull << (i & 63);
        for (uint64_t s = 0; s < S; ++s) {
            const uint64_t *pan = panels + s * W;
            if (!(pan[i >> 6] & bi)) continue;
            for (int w = 0; w < W; ++w) {
                uint64_t m = pan[w];
                while (m) { row[64 * w + __builtin_ctzll(m)] += 1; m &= m - 1; }
            }
        }
    }
}

static int g_cmp_words;
static int cmp_rows(const void *a, const void *b) {
    return memcmp(a, b, sizeof(uint64_t) * (size_t)g_cmp_words);
}

/* number of distinct panels (exact, by sorting full bitmasks); not thread-safe */
uint64_t oracle_unique(const uint64_t *panels, uint64_t S, int n) {
    const int W = (n + 63) / 64;
    if (S == 0) return 0;
    uint64_t *copy = (uint64_t *)malloc(sizeof(uint64_t) * W * S);
    memcpy(copy, panels, sizeof(uint64_t) * W * S);
    g_cmp_words = W;
    qsort(copy, S, sizeof(uint64_t) * W, cmp_rows);
    uint64_t u = 1;
    for (uint64_t i = 1; i < S; ++i)
        if (memcmp(copy + i * W, copy + (i - 1) * W, sizeof(uint64_t) * W)) ++u;
    free(copy);
    return u;
}
