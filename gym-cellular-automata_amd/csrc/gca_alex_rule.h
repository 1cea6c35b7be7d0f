// gca_alex_rule.h — per-cell arithmetic of the Alexandridis step shared by its two mappings (the tiled kernel of
// gca_alex.hip and the marching kernel of gca_alex_march.hip), so that both evaluate the rule with the same
// instructions in the same order. Reference: ca_alexandridis_jax.py:164-206 (_compute_burn_probability), :321-424.
#pragma once
#include "gca_common.h"

typedef float gca_f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float gca_clamp01(float v) { return fminf(fmaxf(v, 0.0f), 1.0f); }
// clamp01(a * b) on both halves: one v_pk_mul_f32 with the clamp output modifier; the product is
// rounded first, then clamped (= clamp01(__fmul_rn(a, b)), NaN -> 0 like fminf(fmaxf(NaN, 0), 1))
__device__ __forceinline__ gca_f2 gca_pk_mul_clamp01(gca_f2 a, gca_f2 b) {
    gca_f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// 4-bit mask of the bytes of x equal to the byte of pat (bit j <-> byte j)
__device__ __forceinline__ uint32_t gca_eq_nib(uint32_t x, uint32_t pat) {
    return (bytes_eq01(x, pat) * 0x01020408u) >> 24;
}
// nibble (bit j) -> 0x01 in byte j; the four partial products never overlap
__device__ __forceinline__ uint32_t gca_spread4(uint32_t n) { return ((n & 0xFu) * 0x00204081u) & 0x01010101u; }
__device__ __forceinline__ uint32_t gca_bfi32(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
// bit i of w as an all-ones / all-zeros word (v_bfe_i32)
__device__ __forceinline__ uint32_t gca_sbit(uint32_t w, int i) { return (uint32_t)((int32_t)(w << (31 - i)) >> 31); }

// p_slope factors of a cell pair from edge-layout values V = +-exp_f32(|a|) (gca.h: gca_alex_step_es): own direction
// (the edge's slope a): P(a) = V if V > 0 else 1/|V|; the neighbour's edge seen from the other end
// (slope -a): P(-a) = |V| if V < 0 else 1/|V|. With rc = 1/V (signed: v_rcp_f32 + one packed Newton
// step, the exact negation of the same steps on |V|) and |V| >= 1 >= |rc|, the selections are
// P(a) = max(V, -rc) and P(-a) = max(-V, rc): one v_max_f32 per cell instead of a compare and a select.
__device__ __forceinline__ gca_f2 gca_edge_factor_pair(float v0, float v1, bool own) {
    const gca_f2 x = {v0, v1};
    const gca_f2 r0 = {__builtin_amdgcn_rcpf(v0), __builtin_amdgcn_rcpf(v1)};
    // ee = 1 - x * r0 on both halves (neg modifiers in the instruction; the compiler sometimes emits sign
    // xors). The s_nop covers the v_rcp_f32 (trans) -> VALU read hazard, which the hazard recogniser does
    // not apply to inline-asm operands (without it the high half read a stale r0).
    gca_f2 ee;
    asm("s_nop 1\n\tv_pk_fma_f32 %0, %1, %2, 1.0 op_sel_hi:[1,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0]"
        : "=v"(ee) : "v"(x), "v"(r0));
    const gca_f2 rc = __builtin_elementwise_fma(ee, r0, r0);
    gca_f2 o;  // v_max_f32 with a neg source modifier (fmaxf would add canonicalising maxes and sign xors)
    if (own) {
        asm("v_max_f32_e64 %0, %1, -%2" : "=v"(o.x) : "v"(v0), "v"(rc.x));
        asm("v_max_f32_e64 %0, %1, -%2" : "=v"(o.y) : "v"(v1), "v"(rc.y));
    } else {
        asm("v_max_f32_e64 %0, -%1, %2" : "=v"(o.x) : "v"(v0), "v"(rc.x));
        asm("v_max_f32_e64 %0, -%1, %2" : "=v"(o.y) : "v"(v1), "v"(rc.y));
    }
    return o;
}

// Both factors of the edges (v0, v1) from one reciprocal: own = P(a) and nb = P(-a), each bit-identical to
// gca_edge_factor_pair(v0, v1, true / false) (the same instructions on the same rc)
__device__ __forceinline__ void gca_edge_factors_both(float v0, float v1, gca_f2& own, gca_f2& nb) {
    const gca_f2 x = {v0, v1};
    const gca_f2 r0 = {__builtin_amdgcn_rcpf(v0), __builtin_amdgcn_rcpf(v1)};
    gca_f2 ee;
    asm("s_nop 1\n\tv_pk_fma_f32 %0, %1, %2, 1.0 op_sel_hi:[1,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0]"
        : "=v"(ee) : "v"(x), "v"(r0));
    const gca_f2 rc = __builtin_elementwise_fma(ee, r0, r0);
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(own.x) : "v"(v0), "v"(rc.x));
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(own.y) : "v"(v1), "v"(rc.y));
    asm("v_max_f32_e64 %0, -%1, %2" : "=v"(nb.x) : "v"(v0), "v"(rc.x));
    asm("v_max_f32_e64 %0, -%1, %2" : "=v"(nb.y) : "v"(v1), "v"(rc.y));
}
// own factors only (P(a)), as gca_edge_factor_pair(v0, v1, true)
__device__ __forceinline__ gca_f2 gca_edge_factors_own(float v0, float v1) { return gca_edge_factor_pair(v0, v1, true); }

// LUT[0..7] = 1 + p_veg[clip(v, 1, 5)] for v = 0..7, LUT[8..15] the same for density (:170-184): entry t of 16
__device__ __forceinline__ float gca_alex_lut_entry(const gca_alex_params& p, int t) {
    const int v = t & 7;
    // selects on the (SGPR) kernel arguments only: no dynamic indexing into the argument struct
    const float av = v <= 1 ? p.veg1p[1] : v == 2 ? p.veg1p[2] : v == 3 ? p.veg1p[3] : v == 4 ? p.veg1p[4] : p.veg1p[5];
    const float ad = v <= 1 ? p.den1p[1] : v == 2 ? p.den1p[2] : v == 3 ? p.den1p[3] : v == 4 ? p.den1p[4] : p.den1p[5];
    return t < 8 ? av : ad;
}
