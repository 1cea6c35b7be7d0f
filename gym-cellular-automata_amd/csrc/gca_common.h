// gca_common.h — shared device helpers for the gfx950 forest-fire kernels.
// Product code: not shared with oracle/ (the oracle restates these independently).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/gca.h"

// ----------------------------------------------------------------- errors
void gca_set_error(const char* fmt, ...);

#define GCA_CHECK_ARG(cond, msg)                 \
    do {                                         \
        if (!(cond)) {                           \
            gca_set_error("argument: %s", msg);  \
            return GCA_ERR_ARG;                  \
        }                                        \
    } while (0)

#define GCA_CHECK_LAUNCH(name)                                                      \
    do {                                                                            \
        hipError_t _e = hipGetLastError();                                          \
        if (_e != hipSuccess) {                                                     \
            gca_set_error("%s: %s", name, hipGetErrorString(_e));                   \
            return GCA_ERR_HIP;                                                     \
        }                                                                           \
    } while (0)

#define GCA_WAVE 64

// ----------------------------------------------------------------- Philox4x32-10
// Random123 Philox4x32 with 10 rounds. Key (k0,k1) is wave-uniform in every kernel
// here (seed), so the key schedule stays in SGPRs.
struct u32x4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)M0 * c.x;
        const uint64_t p1 = (uint64_t)M1 * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        // one v_bitop3_b32 (3-input xor, table 0x96) each; the builtin (not inline asm) lets the hazard
        // recogniser and the scheduler see it: inline asm cost an s_nop before every following v_mad_u64_u32
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96);
        c = u32x4{n0, lo1, n2, lo0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// 24-bit float uniform in [0,1): exact in f32.
__device__ __forceinline__ float u01_f32(uint32_t x) { return (float)(x >> 8) * 0x1.0p-24f; }
// 53-bit double uniform in [0,1) from two words (hi first).
__device__ __forceinline__ double u01_f64(uint32_t hi, uint32_t lo) {
    const uint64_t v = (((uint64_t)hi << 32) | lo) >> 11;
    return (double)v * 0x1.0p-53;
}
// Integer in [lo, hi) by multiply-shift (hi <= lo -> lo): branch-free, span 0 gives lo (one v_mul_hi_u32 + add).
__device__ __forceinline__ int32_t randint_ms(uint32_t x, int32_t lo, int32_t hi) {
    const uint32_t span = hi > lo ? (uint32_t)(hi - lo) : 0u;
    return lo + (int32_t)__umulhi(x, span);
}

// ----------------------------------------------------------------- env helpers (gca_env.hip, gca_windy.hip)
__device__ __forceinline__ int clampi_dev(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
// Move.update (move_modify.py:37-67): the four set tests run in order on the running (row, col).
__device__ __forceinline__ void move_pos(int a, int& row, int& col, int H, int W, int up, int down, int left,
                                         int right) {
    const bool valid_up = row > 0, valid_down = row < H - 1, valid_left = col > 0, valid_right = col < W - 1;
    if (((up >> a) & 1) && valid_up) row -= 1;
    if (((down >> a) & 1) && valid_down) row += 1;
    if (((left >> a) & 1) && valid_left) col -= 1;
    if (((right >> a) & 1) && valid_right) col += 1;
}
// count slot of a cell code: 0 EMPTY, 1 TREE, 2 FIRE, -1 other
__device__ __forceinline__ int cell_category(int v, int empty, int tree, int fire) {
    return v == empty ? 0 : (v == tree ? 1 : (v == fire ? 2 : -1));
}

// WindyForestFire active-direction mask (ca_windy.py:53-77): bit d set iff roll[d] < wind[d]
// (the reference marks d as failed iff wind <= roll). d indexes the 3x3 row-major, centre skipped.
__device__ __forceinline__ uint32_t windy_mask(const double* __restrict__ w, const double* __restrict__ roll,
                                               uint32_t k0, uint32_t k1, uint32_t env_id, uint32_t step) {
    uint32_t m = 0;
    if (roll) {
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            const int idx = d < 4 ? d : d + 1;
            if (roll[idx] < w[idx]) m |= 1u << d;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32x4 x = philox4x32_10(u32x4{(uint32_t)j, env_id, step, GCA_TAG_WINDY_ROLL}, k0, k1);
            const int d0 = 2 * j, d1 = 2 * j + 1;
            const int i0 = d0 < 4 ? d0 : d0 + 1, i1 = d1 < 4 ? d1 : d1 + 1;
            if (u01_f64(x.x, x.y) < w[i0]) m |= 1u << d0;
            if (u01_f64(x.z, x.w) < w[i1]) m |= 1u << d1;
        }
    }
    return m;
}

// ----------------------------------------------------------------- deterministic expf
// exp_f32(x): Cody–Waite reduction x = k*ln2 + r (|r| <= ln2/2), degree-7 Taylor
// polynomial evaluated with explicit fmaf, then exact 2^k scaling. Every step is a
// correctly rounded IEEE op, so the C oracle's restatement (C99 fmaf, rintf,
// -ffp-contract=off) is bit-identical. |error| <= 1 ulp on the clamped range [-80, 80].
__device__ __forceinline__ float exp_f32(float x) {
    x = fminf(fmaxf(x, -80.0f), 80.0f);
    const float kf = rintf(x * 1.44269504088896341f);
    const int k = (int)kf;
    float r = fmaf(kf, -0.693145751953125f, x);          // ln2 hi
    r = fmaf(kf, -1.42860682030941723212e-6f, r);         // ln2 lo
    float p = 1.98412698412698413e-4f;                    // 1/7!
    p = fmaf(p, r, 1.38888888888888889e-3f);              // 1/6!
    p = fmaf(p, r, 8.33333333333333333e-3f);              // 1/5!
    p = fmaf(p, r, 4.16666666666666667e-2f);              // 1/4!
    p = fmaf(p, r, 1.66666666666666667e-1f);              // 1/3!
    p = fmaf(p, r, 0.5f);                                 // 1/2!
    p = fmaf(p, r * r, r);                                // r + r^2 * p
    p = p + 1.0f;
    return __uint_as_float(__float_as_uint(p) + ((uint32_t)k << 23));
}

// ----------------------------------------------------------------- slope factor
// p_slope = P(a), a = 0.078f * slope (ca_alexandridis_jax.py:199-200: exp(0.078 * slope)):
//   P(a) = exp_f32(a) for a >= 0,  1 / exp_f32(-a) (IEEE division) for a < 0.
// Within 2 ulp of exp(a); defined through exp_f32 of |a| so that the two directions of one edge
// (slopes s and -s) share one exp: P(-a) = 1 / P(a) exactly (the edge-slope layout stores one value
// per edge). The C oracle restates it (oracle_slope_factor).
__device__ __forceinline__ float slope_factor(float a) {
    return a >= 0.0f ? exp_f32(a) : __fdiv_rn(1.0f, exp_f32(-a));
}
// 1 / x correctly rounded for x in [1, 2048): v_rcp_f32 (<= 1 ulp) + one Newton step in fma.
// Verified against IEEE division for every f32 in [1, 1121] (tests/test_gpu_edge_slope.py), the range
// of exp_f32(|0.078 * slope|) for |slope| < 90 degrees.
__device__ __forceinline__ float recip_ge1(float x) {
    const float r0 = __builtin_amdgcn_rcpf(x);
    const float e = fmaf(-x, r0, 1.0f);
    return fmaf(e, r0, r0);
}

// ----------------------------------------------------------------- SWAR byte helpers
// Per-byte equality with a replicated pattern: returns 0x01 in each byte where x == pat.
__device__ __forceinline__ uint32_t bytes_eq01(uint32_t x, uint32_t pat) {
    const uint32_t t = x ^ pat;
    const uint32_t y = ((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t;   // high bit set iff byte != 0
    return (~y >> 7) & 0x01010101u;
}
__host__ __device__ __forceinline__ uint32_t rep4(uint32_t v) { return (v & 0xFFu) * 0x01010101u; }
