/*
 * gca_oracle.c — plain-C restatement of the Alexandridis step (reference
 * ca_alexandridis_jax.py:164-206, 321-460) in the exact f32 evaluation order the
 * device kernel documents, plus Philox4x32-10 and the deterministic exp_f32.
 * TEST INFRASTRUCTURE ONLY (bit-exact checker of libgca_hip.so and the CPU baseline
 * of bench.py); it shares no source with the product and is never linked into it.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; no -ffast-math).
 *
 * Restated algorithm, per cell (r, c) of env e, zero (EMPTY) padding:
 *   B_k   = #FIRE in the (2k+1)^2 box, D_k = sum of dousing in the box (k = 1, 2)
 *   heat  = sum_{k=0..R} dw_k * B_k         (dw_k = w_k - w_{k+1}: ring weights, f32; ph = fmaf(dw_k, B_k, ph))
 *   dous  = (inner - border) * D_1 + border * D_2   (the second term by fmaf)
 *   p_h   = heat - dous                      (:198)
 *   p_d   = ((((p_h * av) * ad) * wind[d]) * p_slope[d])                       (:206)
 *   injected: TREE -> FIRE iff exists fire neighbour d with u[d] < p_d (:379-383)
 *   philox  : TREE -> FIRE iff u(main) < 1 - q, q = prod_{fire d} (1 - clamp01(p_d)) accumulated in d order as
 *             q = fmaf(-q, clamp01(p_d), q) (one rounding per factor). Draws (r05): one Philox block per group of
 *             4 cells of a row, X = Philox(r * ceil(W / 4) + (c >> 2), env, step, ALXC); cell j = c & 3 tests
 *             main = X[j] (its high 24 bits). The group's new fires take their ages in column order: the first
 *             from the spare word X[0].b0 | X[1].b0 << 8 | X[2].b0 << 16 | X[3].b0 << 24 (the low bytes, which
 *             no decision reads), the k-th (k = 2..4) from word k-2 of Y = Philox(same counter, ALXA)
 *   EMPTY -> TREE iff u < p_tree; FIRE -> EMPTY iff age <= 1 (age == 1 with burnout_eq1, the
 *   classic ca_alexandridis.py:181-183); ages (:394-423). heat starts at heat0 (0, or the classic
 *   constant p_h = 0.58 of ca_alexandridis.py:94 with zero heat / dousing weights).
 */
#include <math.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#define TAG_ALEX_CELL 0x414C5843u
#define TAG_ALEX_AGE 0x414C5841u
#define TAG_ALEX_WIND 0x414C5857u

typedef struct {
    int32_t R;
    float heat_dw[9];
    float dous_inner, dous_border;
    float veg1p[6], den1p[6];
    float p_tree;
    int32_t age_lo, age_hi;
    uint64_t seed;
    int32_t env_offset;
    int32_t empty, tree, fire;
    int32_t n_winds;
    float winds[16][9];
    float heat0;
    int32_t burnout_eq1;
    int32_t vd_uniform; /* gca.h; the oracle reads per-cell layers */
} oracle_alex_params;

/* ------------------------------------------------------------------ Philox4x32-10 */
static void philox(const uint32_t in[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
    uint32_t c0 = in[0], c1 = in[1], c2 = in[2], c3 = in[3];
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n1 = (uint32_t)p1;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1, n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

void oracle_philox(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out, long n) {
    for (long i = 0; i < n; ++i) philox(ctr + 4 * i, k0, k1, out + 4 * i);
}

static float u01(uint32_t x) { return (float)(x >> 8) * 0x1.0p-24f; }
static int32_t randint_ms(uint32_t x, int32_t lo, int32_t hi) {
    if (hi <= lo) return lo;
    return lo + (int32_t)(((uint64_t)x * (uint32_t)(hi - lo)) >> 32);
}

/* ------------------------------------------------------------------ exp_f32 */
float oracle_exp_f32(float x) {
    x = fminf(fmaxf(x, -80.0f), 80.0f);
    const float kf = rintf(x * 1.44269504088896341f);
    const int k = (int)kf;
    float r = fmaf(kf, -0.693145751953125f, x);
    r = fmaf(kf, -1.42860682030941723212e-6f, r);
    float p = 1.98412698412698413e-4f;
    p = fmaf(p, r, 1.38888888888888889e-3f);
    p = fmaf(p, r, 8.33333333333333333e-3f);
    p = fmaf(p, r, 4.16666666666666667e-2f);
    p = fmaf(p, r, 1.66666666666666667e-1f);
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r * r, r);
    p = p + 1.0f;
    uint32_t bits;
    memcpy(&bits, &p, 4);
    bits += (uint32_t)k << 23;
    float y;
    memcpy(&y, &bits, 4);
    return y;
}

/* p_slope factor of a = 0.078f * slope (device slope_factor, gca_common.h): exp_f32(a) for a >= 0,
 * 1 / exp_f32(-a) (IEEE division) for a < 0 — so the two directions of one edge are exact reciprocals */
float oracle_slope_factor(float a) { return a >= 0.0f ? oracle_exp_f32(a) : 1.0f / oracle_exp_f32(-a); }

/* the edge layout's signed factor V = +exp_f32(a) (a >= 0) / -exp_f32(-a) (a < 0), a = 0.078f * slope */
void oracle_signed_factors(const float* slope, float* v, long n) {
    for (long i = 0; i < n; ++i) {
        const float a = 0.078f * slope[i];
        v[i] = a >= 0.0f ? oracle_exp_f32(a) : -oracle_exp_f32(-a);
    }
}

/* the factor of the neighbour direction from V (the kernel's rule): P(-a) = |V| if V < 0 else 1/|V|,
 * and the own direction P(a) = V if V > 0 else 1/|V| */
void oracle_factor_pairs(const float* v, float* own, float* nbr, long n) {
    for (long i = 0; i < n; ++i) {
        const float x = fabsf(v[i]);
        own[i] = v[i] > 0.0f ? x : 1.0f / x;
        nbr[i] = v[i] < 0.0f ? x : 1.0f / x;
    }
}

void oracle_alex_prepare_slope(const float* slope, float* p_slope, int E, int H, int W) {
    const long HW = (long)H * W;
    for (int e = 0; e < E; ++e)
        for (long cell = 0; cell < HW; ++cell)
            for (int d = 0; d < 8; ++d) {
                const float s = slope[((long)e * HW + cell) * 9 + (d < 4 ? d : d + 1)];
                p_slope[((long)e * 8 + d) * HW + cell] = oracle_slope_factor(0.078f * s);
            }
}

static float clamp01(float v) { return fminf(fmaxf(v, 0.0f), 1.0f); }

/* one env, one step */
static void alex_env(const oracle_alex_params* p, int e, int H, int W, const uint8_t* g, uint8_t* go,
                     const int16_t* age, int16_t* ageo, const uint8_t* veg, const uint8_t* den, const uint8_t* dous,
                     const float* ps, int widx, uint32_t step, const float* ib, const float* ig, const int32_t* ia,
                     float* po, int32_t* counts) {
    const long HW = (long)H * W;
    const int R = p->R;
    const float in_minus_bd = p->dous_inner - p->dous_border;
    const uint32_t k0 = (uint32_t)p->seed, k1 = (uint32_t)(p->seed >> 32);
    const uint32_t env_id = (uint32_t)(p->env_offset + e);
    float wind[8];
    for (int d = 0; d < 8; ++d) wind[d] = p->winds[widx][d < 4 ? d : d + 1];
    int cE = 0, cT = 0, cF = 0;
    /* summed-area tables of FIRE indicators and dousing values, (H+1) x (W+1) */
    int64_t* satf = (int64_t*)calloc((size_t)(H + 1) * (W + 1), sizeof(int64_t));
    int64_t* satd = (int64_t*)calloc((size_t)(H + 1) * (W + 1), sizeof(int64_t));
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c) {
            const long i = (long)(r + 1) * (W + 1) + (c + 1);
            satf[i] = (g[(long)r * W + c] == p->fire) + satf[i - 1] + satf[i - (W + 1)] - satf[i - (W + 1) - 1];
            satd[i] = dous[(long)r * W + c] + satd[i - 1] + satd[i - (W + 1)] - satd[i - (W + 1) - 1];
        }
    const uint32_t GW4 = (uint32_t)(W + 3) >> 2;
    for (int r = 0; r < H; ++r) {
        uint32_t gX[4] = {0u, 0u, 0u, 0u};
        int g_have = 0, g_n = 0;
        long g_cell[4];
        for (int c = 0; c < W; ++c) {
            const long cell = (long)r * W + c;
            const uint32_t grp = (uint32_t)r * GW4 + ((uint32_t)c >> 2);
            if ((c & 3) == 0) g_have = g_n = 0;
            /* box sums from the summed-area tables (clamped to the grid = zero padding) */
            float ph = p->heat0, dz = 0.0f;
            const int KS = R < 2 ? 2 : R;
            for (int k = 0; k <= KS; ++k) {
                const int r0 = r - k < 0 ? 0 : r - k, r1 = r + k + 1 > H ? H : r + k + 1;
                const int c0 = c - k < 0 ? 0 : c - k, c1 = c + k + 1 > W ? W : c + k + 1;
                const long W1 = W + 1;
                const int64_t fire_n = satf[r1 * W1 + c1] - satf[r0 * W1 + c1] - satf[r1 * W1 + c0] + satf[r0 * W1 + c0];
                const int64_t dsum = satd[r1 * W1 + c1] - satd[r0 * W1 + c1] - satd[r1 * W1 + c0] + satd[r0 * W1 + c0];
                if (k <= R) ph = fmaf(p->heat_dw[k], (float)fire_n, ph);
                if (k == 1) dz = in_minus_bd * (float)dsum;
                if (k == 2) dz = fmaf(p->dous_border, (float)dsum, dz);
            }
            ph = ph - dz;
            /* neighbourhood fire mask, d = (a,b) row-major without the centre */
            uint32_t fm = 0;
            int d = 0;
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) {
                    if (a == 1 && b == 1) continue;
                    const int rr = r + a - 1, cc = c + b - 1;
                    if (rr >= 0 && rr < H && cc >= 0 && cc < W && g[(long)rr * W + cc] == p->fire) fm |= 1u << d;
                    ++d;
                }
            const int vv = veg[cell], dd = den[cell];
            const int vi = vv < 1 ? 1 : (vv > 5 ? 5 : vv), di = dd < 1 ? 1 : (dd > 5 ? 5 : dd);
            const float base = (ph * p->veg1p[vi]) * p->den1p[di];
            float pd[8];
            for (int q = 0; q < 8; ++q) pd[q] = (base * wind[q]) * ps[(long)q * HW + cell];
            if (po)
                for (int q = 0; q < 8; ++q) po[cell * 8 + q] = pd[q];
            const int x = g[cell];
            const int is_tree = x == p->tree, is_empty = x == p->empty, is_fire = x == p->fire;
            int burn = 0, grow = 0, new_age = p->age_lo;
            if (ib) {
                if (is_tree && fm) {
                    for (int q = 0; q < 8; ++q)
                        if (((fm >> q) & 1u) && ib[cell * 9 + (q < 4 ? q : q + 1)] < pd[q]) burn = 1;
                    if (burn) new_age = ia[cell];
                }
                if (is_empty) grow = ig[cell] < p->p_tree;
            } else if ((is_tree && fm) || (is_empty && p->p_tree > 0.0f)) {
                /* the group's block (r * ceil(W/4) + c/4, env, step, ALXC): cell j = c & 3 reads word j */
                if (!g_have) {
                    const uint32_t ctr[4] = {grp, env_id, step, TAG_ALEX_CELL};
                    philox(ctr, k0, k1, gX);
                    g_have = 1;
                }
                const uint32_t main_w = gX[c & 3];
                if (is_tree) {
                    float qn = 1.0f;
                    for (int q = 0; q < 8; ++q)
                        if ((fm >> q) & 1u) qn = fmaf(-qn, clamp01(pd[q]), qn);
                    burn = u01(main_w) < 1.0f - qn;
                    if (burn) g_cell[g_n++] = cell; /* its age: at the end of the group, by rank */
                } else {
                    grow = u01(main_w) < p->p_tree;
                }
            }
            int nx = x;
            if (is_tree && burn) nx = p->fire;
            else if (is_empty && grow) nx = p->tree;
            else if (is_fire && (p->burnout_eq1 ? age[cell] == 1 : age[cell] <= 1)) nx = p->empty;
            int na = (nx == p->fire && !is_fire) ? new_age : age[cell];
            if (is_fire) na -= 1;
            go[cell] = (uint8_t)nx;
            ageo[cell] = (int16_t)na;
            cE += nx == p->empty;
            cT += nx == p->tree;
            cF += nx == p->fire;
            if (g_n && ((c & 3) == 3 || c == W - 1)) {
                /* the group's new fires in column order: the spare word of X, then words 0.. of Y (ALXA) */
                const uint32_t spare = (gX[0] & 0xFFu) | ((gX[1] & 0xFFu) << 8) | ((gX[2] & 0xFFu) << 16) |
                                       (gX[3] << 24);
                uint32_t gY[4] = {0u, 0u, 0u, 0u};
                if (g_n > 1) {
                    const uint32_t ctr[4] = {grp, env_id, step, TAG_ALEX_AGE};
                    philox(ctr, k0, k1, gY);
                }
                for (int k = 0; k < g_n; ++k)
                    ageo[g_cell[k]] = (int16_t)randint_ms(k == 0 ? spare : gY[k - 1], p->age_lo, p->age_hi);
                g_n = 0;
            }
        }
    }
    free(satf);
    free(satd);
    if (counts) {
        counts[0] = cE;
        counts[1] = cT;
        counts[2] = cF;
    }
}

void oracle_alex_step(const oracle_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                      const int16_t* age_in, int16_t* age_out, const uint8_t* veg, const uint8_t* den,
                      const uint8_t* dousing, const float* p_slope, const int32_t* wind_index,
                      const uint32_t* rng_step, const float* inj_burn, const float* inj_grow, const int32_t* inj_age,
                      float* prob_out, int32_t* counts) {
    const long HW = (long)H * W;
    for (int e = 0; e < E; ++e) {
        alex_env(p, e, H, W, grid_in + e * HW, grid_out + e * HW, age_in + e * HW, age_out + e * HW, veg + e * HW,
                 den + e * HW, dousing + e * HW, p_slope + e * 8 * HW, wind_index[e], rng_step ? rng_step[e] : 0u,
                 inj_burn ? inj_burn + e * HW * 9 : 0, inj_grow ? inj_grow + e * HW : 0,
                 inj_age ? inj_age + e * HW : 0, prob_out ? prob_out + e * HW * 8 : 0, counts ? counts + 3 * e : 0);
    }
}

/* wind change (ca_alexandridis_jax.py:442-451) with the device's Philox convention */
void oracle_alex_wind_change(float p_change, int n_winds, uint64_t seed, int env_offset, const uint32_t* rng_step,
                             int32_t* wind_index, int E) {
    for (int e = 0; e < E; ++e) {
        const uint32_t ctr[4] = {0u, (uint32_t)(env_offset + e), rng_step ? rng_step[e] : 0u, TAG_ALEX_WIND};
        uint32_t x[4];
        philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32), x);
        if (u01(x[0]) < p_change) wind_index[e] = (wind_index[e] + randint_ms(x[1], 1, 8)) % n_winds;
    }
}

/* ------------------------------------------------------------------ pinecone spotting
 * Restates ca_alexandridis_jax.py:229-319 + the scatter of :400-420 with the device's draw convention
 * (gca_pine.hip): every FIRE cell of grid_in (row-major) throws n = min(Poisson(1), max) pinecones; pinecone m
 * lands at (clip(r + dx[d] s), clip(c + dy[d] s)) and, if that cell of grid_out is TREE and u < prob, ignites
 * it with age randint(age_lo, age_hi) of the target's own draw. Sequential application = the device's
 * any-pinecone-ignites rule (an ignited target is no longer TREE). */
#define PINE_MAX 8
#define PINE_CDF 17
#define TAG_PINE 0x50494E45u
#define TAG_PINE_AGE 0x50494E41u
typedef struct {
    uint32_t n_cdf[PINE_MAX];
    int32_t max_pinecones;
    int32_t dx[8], dy[8];
    float scale;
    float veg1p[6], den1p[6];
    int32_t age_lo, age_hi;
    uint64_t seed;
    int32_t env_offset;
    int32_t empty, tree, fire;
} oracle_pine_params;

static int cdf_pick(uint32_t x, const uint32_t* thr, int n) {
    int k = 0;
    for (int j = 0; j < n; ++j) k += x >= thr[j];
    return k;
}

void oracle_alex_pinecones(const oracle_pine_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                           int16_t* age_out, const uint8_t* veg, const uint8_t* den, const int32_t* wind_index,
                           const uint32_t* s_cdf, const uint32_t* rng_step, int32_t* counts) {
    const long HW = (long)H * W;
    const uint32_t k0 = (uint32_t)p->seed, k1 = (uint32_t)(p->seed >> 32);
    for (int e = 0; e < E; ++e) {
        const uint32_t env_id = (uint32_t)(p->env_offset + e), step = rng_step ? rng_step[e] : 0u;
        const uint32_t* tab = s_cdf + (long)wind_index[e] * 8 * PINE_CDF;
        for (long lin = 0; lin < HW; ++lin) {
            if (grid_in[e * HW + lin] != p->fire) continue;
            const int r = (int)(lin / W), c = (int)(lin % W);
            uint32_t b0[4];
            const uint32_t c0[4] = {(uint32_t)lin, env_id, step, TAG_PINE};
            philox(c0, k0, k1, b0);
            int n = cdf_pick(b0[0], p->n_cdf, PINE_MAX);
            if (n > p->max_pinecones) n = p->max_pinecones;
            for (int m = 0; m < n; ++m) {
                uint32_t x[4];
                const uint32_t cm[4] = {(uint32_t)lin, env_id, step, TAG_PINE + 1u + (uint32_t)m};
                philox(cm, k0, k1, x);
                const int d = (int)(x[2] >> 29);
                const uint32_t* t = tab + d * PINE_CDF;
                const int s = cdf_pick(x[0], t + 1, (int)t[0]) - (int)(t[0] >> 1);
                int tr = r + p->dx[d] * s, tc = c + p->dy[d] * s;
                tr = tr < 0 ? 0 : (tr > H - 1 ? H - 1 : tr);
                tc = tc < 0 ? 0 : (tc > W - 1 ? W - 1 : tc);
                const long tl = (long)tr * W + tc;
                int vv = veg[e * HW + tl], dd = den[e * HW + tl];
                vv = vv < 1 ? 1 : (vv > 5 ? 5 : vv);
                dd = dd < 1 ? 1 : (dd > 5 ? 5 : dd);
                const float prob = (p->scale * p->veg1p[vv]) * p->den1p[dd];
                if (!(u01(x[1]) < prob)) continue;
                if (grid_out[e * HW + tl] != p->tree) continue;
                grid_out[e * HW + tl] = (uint8_t)p->fire;
                uint32_t a[4];
                const uint32_t ca[4] = {(uint32_t)tl, env_id, step, TAG_PINE_AGE};
                philox(ca, k0, k1, a);
                age_out[e * HW + tl] = (int16_t)randint_ms(a[0], p->age_lo, p->age_hi);
                if (counts) {
                    counts[3 * e + 1] -= 1;
                    counts[3 * e + 2] += 1;
                }
            }
        }
    }
}

/* ------------------------------------------------------------------ classic pinecone spotting
 * The sequential skip-list loop of PartiallyObservableForestFire.update (ca_alexandridis.py:149-210) restricted
 * to its pinecone part, on the output of the classic step: cells are visited in row-major order, a visited FIRE
 * cell of grid_in throws its pinecones (the device's draw convention, gca_pine.hip), a landing inside the grid and
 * not on the thrower ignites its target whatever its state (u24 < burn_thr), and an ignited target later in the
 * order is put on the skip list (a skipped FIRE cell throws nothing). Ages of ignited targets: the target-keyed
 * draw. The device resolves the same order dependence in parallel; this loop is the literal order. */
#define PINEC_NMAX 16
#define PINEC_CDF 48
#define TAG_PINEC 0x50434C00u
#define TAG_PINEC_AGE 0x50434C41u
typedef struct {
    uint32_t n_cdf[PINEC_NMAX];
    int32_t dx[8], dy[8];
    uint32_t burn_thr[6][6];
    int32_t age_lo, age_hi;
    uint64_t seed;
    int32_t env_offset;
    int32_t empty, tree, fire;
} oracle_pine_classic_params;

void oracle_alex_pinecones_classic(const oracle_pine_classic_params* p, int E, int H, int W, const uint8_t* grid_in,
                                   uint8_t* grid_out, int16_t* age_out, const uint8_t* veg, const uint8_t* den,
                                   const int32_t* wind_index, const uint32_t* s_cdf, const uint32_t* rng_step,
                                   int32_t* counts, int32_t* n_skipped_sources) {
    const long HW = (long)H * W;
    const uint32_t k0 = (uint32_t)p->seed, k1 = (uint32_t)(p->seed >> 32);
    uint8_t* skip = (uint8_t*)malloc((size_t)HW);
    for (int e = 0; e < E; ++e) {
        memset(skip, 0, (size_t)HW);
        const uint32_t env_id = (uint32_t)(p->env_offset + e), step = rng_step ? rng_step[e] : 0u;
        const uint32_t* tab = s_cdf + (long)wind_index[e] * 8 * PINEC_CDF;
        int skipped_sources = 0;
        for (long lin = 0; lin < HW; ++lin) {
            if (grid_in[e * HW + lin] != p->fire) continue;
            if (skip[lin]) {
                ++skipped_sources;
                continue;
            }
            const int r = (int)(lin / W), c = (int)(lin % W);
            uint32_t b0[4];
            const uint32_t c0[4] = {(uint32_t)lin, env_id, step, TAG_PINEC};
            philox(c0, k0, k1, b0);
            const int n = cdf_pick(b0[0], p->n_cdf, PINEC_NMAX);
            for (int m = 0; m < n; ++m) {
                uint32_t x[4];
                const uint32_t cm[4] = {(uint32_t)lin, env_id, step, TAG_PINEC + 1u + (uint32_t)m};
                philox(cm, k0, k1, x);
                const int d = (int)(x[2] >> 29);
                const uint32_t* t = tab + d * PINEC_CDF;
                const int s = cdf_pick(x[0], t + 1, (int)t[0]) - (int)(t[0] >> 1);
                const int tr = r + p->dx[d] * s, tc = c + p->dy[d] * s;
                if (tr < 0 || tr >= H || tc < 0 || tc >= W || (tr == r && tc == c)) continue;
                const long tl = (long)tr * W + tc;
                int vv = veg[e * HW + tl], dd = den[e * HW + tl];
                vv = vv < 1 ? 1 : (vv > 5 ? 5 : vv);
                dd = dd < 1 ? 1 : (dd > 5 ? 5 : dd);
                if (!((x[1] >> 8) < p->burn_thr[vv][dd])) continue;
                const uint8_t prev = grid_out[e * HW + tl];
                grid_out[e * HW + tl] = (uint8_t)p->fire;
                uint32_t a[4];
                const uint32_t ca[4] = {(uint32_t)tl, env_id, step, TAG_PINEC_AGE};
                philox(ca, k0, k1, a);
                age_out[e * HW + tl] = (int16_t)randint_ms(a[0], p->age_lo, p->age_hi);
                if (counts && prev != p->fire) {
                    if (prev == p->empty) counts[3 * e] -= 1;
                    else if (prev == p->tree) counts[3 * e + 1] -= 1;
                    counts[3 * e + 2] += 1;
                }
                if (tl > lin) skip[tl] = 1;
            }
        }
        if (n_skipped_sources) n_skipped_sources[e] = skipped_sources;
    }
    free(skip);
}
