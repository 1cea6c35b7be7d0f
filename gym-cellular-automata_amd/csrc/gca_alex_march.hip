// gca_alex_march.hip — the Alexandridis CA step on the Advanced env's packed layout, marching form (W = 256 * NSEG).
// Reference: PartiallyObservableForestFireJax._update_grid (ca_alexandridis_jax.py:321-424) with
// _compute_burn_probability (:164-206): the rule, the f32 arithmetic in its order and the Philox draws of
// alex_step_kernel's packed mode (gca_alex.hip), bit for bit; only the work mapping differs.
//
// Mapping: one wave = one activity-map tile = 16 rows x 256 columns of one env. Lane l owns columns 4l .. 4l+3 of
// every row and the wave walks its tile top to bottom, one row per iteration, with every input of row r+1 in
// flight while row r is computed. No LDS staging and no workgroup barrier (the tiled kernel spent 31 % of a wave's
// life staging its halo and building the column prefix, profiles/r03i):
//   fire ring   FIRE flags (0x01 bytes, one dword per row) of rows r-R-1 .. r+R;
//   V_k         per column, the FIRE count of the 2k+1 rows around r: V_k += row r+k - row r-1-k per row;
//   B_k         the (2k+1) x (2k+1) box sum = the (2k+1)-column window of V_k: v_dot4_u32_u8 of the lane's dword
//               and its DPP neighbours (lanes l-2 .. l+2, wave_shr / wave_shl) against constant 0/1 byte masks;
//   D_1, D_2    the same on the dousing flags (3 x 3 and 5 x 5 boxes, a ring of 6 rows);
//   heat = sum_k dw_k * B_k, dous = (inner - border) * D_1 + border * D_2, fma-chained as in gca_alex.hip.
// Edge slopes in the natural edge layout (E, 4, H, W) (gca_alex_edge_slope_from_altitude): row r+1's four planes
// arrive while row r is computed; they are row r's 'down' factors (directions 5, 6, 7) and then row r+1's own, so
// every slope byte is read once (the tiled kernel re-reads three planes of row r+1 through L2: 27.4 B/cell of
// traffic against 23.1 algorithmic, profiles/pmc_traffic.json). Lane reads are 16 B / 4 B / 8 B at 16 / 4 / 8 B
// strides: 1 KiB, 256 B, 512 B contiguous per wave instruction.
// The edge halo of a 256-column segment is the grid's zero border at W = 256: lane 0's left and lane 63's right
// DPP neighbours read 0 (EMPTY / no dousing), and the border cells' slope factors are 1.
// W = 256 * NSEG (NSEG = 2, 4: the reference's R = 7 grids at 512^2, R = 8 at 1024^2): one workgroup = the NSEG waves of
// one 16-row strip, wave g marching segment g (columns 256g .. 256g + 255) in step with its neighbours. After each row's
// running sums move, every wave's edge lanes (0, 1, 62, 63) post what the neighbour segment's edge lanes take by DPP
// from across the boundary — V_1..V_R, the two dousing sums, the FIRE flags of rows r-1, r, r+1 and three raw edge-slope
// values — into a per-row-parity LDS exchange, one barrier, and each wave reads its neighbours' values straight into the
// `old` operand of its edge DPPs (lane 0 <- the left segment's lane 63 / 62, lane 63 <- the right segment's lane 0 / 1;
// the grid's border reads a slot of zeros and slope 1.0). Nothing else changes: the same cells, the same arithmetic.
#include "gca_alex_rule.h"

#include <type_traits>

#ifndef GCA_MARCH_FLAT_OCC
#define GCA_MARCH_FLAT_OCC 4  // waves / SIMD of the flat-terrain step (no slope planes in registers: ~110 VGPRs)
#endif
#ifndef GCA_MARCH_OBS_FLAT_OCC
#define GCA_MARCH_OBS_FLAT_OCC 3  // waves / SIMD of the flat-terrain step with the fused frame (r06: 2 -> 3, -18 %)
#endif
#ifndef GCA_MARCH_XROW
#define GCA_MARCH_XROW 1  // the 17th slope row of a tile from the next tile's wave through LDS (r06; 0: from HBM again)
#endif

namespace {

constexpr int MW = 256;  // segment width (one wave per segment of a row; W = MW * NSEG)
constexpr int SH = 16;   // rows per wave = one tile of the activity map (gca.h: gca_alex_step_packed)

struct MarchObs {
    const float4* col;     // [2 nights][3 kinds][2 dousing] colours (gca_obs_color_table)
    const int32_t* night;  // [E] pre-step is_night
    float* rgb;            // [E][H][W][3]
    // the extension pipeline (gca_alex_step_march_rgb_ext, W = 256): per extension choice (the action's third
    // column, clamped to [0, n_choices)) 4 bits of OBS_* below; refit[e] = 1 when env e's frame must be rendered by
    // gca_adv_observation instead (its display needs the blur, or the speculation "row 0 of an enabled extension
    // channel is nonzero" failed)
    const int32_t* action;
    int action_stride, n_choices;
    uint32_t mode_bits;
    uint8_t* refit;
};
// frame modes of an extension choice (advanced_bulldozer.py:1035-1101 with the display scan of gca_obs.hip): the
// display is channel min(first row with a positive extension value, n_ext - 1); the kernel speculates that row 0 has
// one, so channel 0 is shown: the grid itself (channel 0 enabled and unblurred: visibility changes only code 3, which
// renders EMPTY either way) or zeros (channel 0 disabled); the check bits say how row 0 is tested
constexpr uint32_t OBS_GRID = 0u, OBS_ZERO = 1u, OBS_NONE = 2u;  // bits 0-1: what the kernel renders
constexpr uint32_t OBS_CHK_GRID = 4u, OBS_CHK_BLUR = 8u;        // speculation checks (row 0 of the new grid)

// DPP across the whole wave (gfx9 wave_shr:1 / wave_shl:1); the lane without a source reads 0 (bound_ctrl: no
// `old` operand to materialise, one v_mov_b32_dpp each)
__device__ __forceinline__ uint32_t from_prev(uint32_t v) {  // lane l <- lane l-1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t from_next(uint32_t v) {  // lane l <- lane l+1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xF, 0xF, true);
}
// the same with a halo: the lane without a source keeps `old` (lane 0: the left segment's value, lane 63: the right's)
__device__ __forceinline__ uint32_t from_prev_or(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t from_next_or(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x130, 0xF, 0xF, false);
}

// byte mask of dword o (lane l+o, o in -2..2) inside the window of radius k around the lane's column j
__host__ __device__ constexpr uint32_t win_mask(int o, int j, int k) {
    uint32_t m = 0;
    for (int b = 0; b < 4; ++b) {
        const int c = 4 * o + b - j;
        if (c >= -k && c <= k) m |= 1u << (8 * b);
    }
    return m;
}
// is dword o (lane l+o) entirely inside the window of radius k around column j?
__host__ __device__ constexpr bool win_full(int o, int j, int k) { return j - k <= 4 * o && 4 * o + 3 <= j + k; }
// B[j] = sum of the byte counts X over columns 4l+j-k .. 4l+j+k (k <= 8: lanes l-2 .. l+2), v_dot4_u32_u8 chains. The
// dwords a window covers fully (always a run around the lane's own: {0}, {-1,0}, {0,1} or {-1,0,1} for k >= 2) are summed
// once and shared by the four windows; the partial dwords are added with their byte masks (k = 6: 10 dot4 instead of 16)
// HALO (NSEG > 1): h1 / h2 are the dwords beyond the segment's edges (lane 0: left segment's lanes 63 / 62, lane 63:
// right segment's lanes 0 / 1)
template <bool HALO = false>
__device__ __forceinline__ void window4(uint32_t X, int k, uint32_t (&B)[4], uint32_t z = 0u, uint32_t h1 = 0u,
                                        uint32_t h2 = 0u) {
    uint32_t n[5] = {0u, 0u, X, 0u, 0u};
    if (k >= 1) {
        n[1] = HALO ? from_prev_or(h1, X) : from_prev(X);
        n[3] = HALO ? from_next_or(h1, X) : from_next(X);
    }
    if (k >= 5) {
        n[0] = HALO ? from_prev_or(h2, n[1]) : from_prev(n[1]);
        n[4] = HALO ? from_next_or(h2, n[3]) : from_next(n[3]);
    }
    constexpr uint32_t ONES = 0x01010101u;
    // which full runs the four windows use (compile-time after unrolling)
    bool use0 = false, useL = false, useR = false, useLR = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool f0 = win_full(0, j, k), fl = win_full(-1, j, k), fr = win_full(1, j, k);
        if (f0 && fl && fr) useLR = true;
        else if (f0 && fl) useL = true;
        else if (f0 && fr) useR = true;
        else if (f0) use0 = true;
    }
    uint32_t S0 = 0u, SL = 0u, SR = 0u, SLR = 0u;
    if (use0 || useL || useR || useLR) S0 = __builtin_amdgcn_udot4(n[2], ONES, z, false);
    if (useL || useLR) SL = __builtin_amdgcn_udot4(n[1], ONES, S0, false);
    if (useR) SR = __builtin_amdgcn_udot4(n[3], ONES, S0, false);
    if (useLR) SLR = __builtin_amdgcn_udot4(n[3], ONES, SL, false);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool f0 = win_full(0, j, k), fl = win_full(-1, j, k), fr = win_full(1, j, k);
        const bool run = f0;  // the full dwords of a window with the lane's own are a run containing it
        uint32_t acc = !run ? z : (fl && fr) ? SLR : fl ? SL : fr ? SR : S0;
#pragma unroll
        for (int o = -2; o <= 2; ++o) {
            if (run && (o == 0 || (o == -1 && fl) || (o == 1 && fr))) continue;  // inside the shared sum
            const uint32_t m = win_mask(o, j, k);
            if (m) acc = __builtin_amdgcn_udot4(n[o + 2], m, acc, false);
        }
        B[j] = acc;
    }
}

__device__ __forceinline__ float4 ldf4(const float* p) { return *reinterpret_cast<const float4*>(p); }
// gca_edge_factors_both / _own (gca_alex_rule.h) with the first Newton fma as a builtin (v_pk_fma_f32 with the neg
// modifier, the same instruction) instead of inline asm with its own s_nop: the hazard recogniser then spaces the
// v_rcp_f32 -> v_pk_fma_f32 reads only where the schedule leaves them adjacent
__device__ __forceinline__ gca_f2 m_recip(float v0, float v1) {
    const gca_f2 x = {v0, v1};
    const gca_f2 r0 = {__builtin_amdgcn_rcpf(v0), __builtin_amdgcn_rcpf(v1)};
    const gca_f2 ee = __builtin_elementwise_fma(-x, r0, (gca_f2){1.0f, 1.0f});
    return __builtin_elementwise_fma(ee, r0, r0);
}
__device__ __forceinline__ void m_edge_both(float v0, float v1, gca_f2& own, gca_f2& nb) {
    const gca_f2 rc = m_recip(v0, v1);
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(own.x) : "v"(v0), "v"(rc.x));
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(own.y) : "v"(v1), "v"(rc.y));
    asm("v_max_f32_e64 %0, -%1, %2" : "=v"(nb.x) : "v"(v0), "v"(rc.x));
    asm("v_max_f32_e64 %0, -%1, %2" : "=v"(nb.y) : "v"(v1), "v"(rc.y));
}
// both cell pairs of a float4 at once: the two reciprocal chains interleaved (each v_pk_fma_f32 result is read two
// instructions later, not by the next one)
__device__ __forceinline__ void m_edge_both4(const float4& v, gca_f2& oa, gca_f2& na, gca_f2& ob, gca_f2& nb) {
    const gca_f2 x0 = {v.x, v.y}, x1 = {v.z, v.w};
    const gca_f2 r0 = {__builtin_amdgcn_rcpf(v.x), __builtin_amdgcn_rcpf(v.y)};
    const gca_f2 r1 = {__builtin_amdgcn_rcpf(v.z), __builtin_amdgcn_rcpf(v.w)};
    const gca_f2 e0 = __builtin_elementwise_fma(-x0, r0, (gca_f2){1.0f, 1.0f});
    const gca_f2 e1 = __builtin_elementwise_fma(-x1, r1, (gca_f2){1.0f, 1.0f});
    const gca_f2 c0 = __builtin_elementwise_fma(e0, r0, r0);
    const gca_f2 c1 = __builtin_elementwise_fma(e1, r1, r1);
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(oa.x) : "v"(v.x), "v"(c0.x));
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(oa.y) : "v"(v.y), "v"(c0.y));
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(ob.x) : "v"(v.z), "v"(c1.x));
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(ob.y) : "v"(v.w), "v"(c1.y));
    asm("v_max_f32_e64 %0, -%1, %2" : "=v"(na.x) : "v"(v.x), "v"(c0.x));
    asm("v_max_f32_e64 %0, -%1, %2" : "=v"(na.y) : "v"(v.y), "v"(c0.y));
    asm("v_max_f32_e64 %0, -%1, %2" : "=v"(nb.x) : "v"(v.z), "v"(c1.x));
    asm("v_max_f32_e64 %0, -%1, %2" : "=v"(nb.y) : "v"(v.w), "v"(c1.y));
}
__device__ __forceinline__ void m_edge_own4(const float4& v, gca_f2& oa, gca_f2& ob) {
    const gca_f2 x0 = {v.x, v.y}, x1 = {v.z, v.w};
    const gca_f2 r0 = {__builtin_amdgcn_rcpf(v.x), __builtin_amdgcn_rcpf(v.y)};
    const gca_f2 r1 = {__builtin_amdgcn_rcpf(v.z), __builtin_amdgcn_rcpf(v.w)};
    const gca_f2 e0 = __builtin_elementwise_fma(-x0, r0, (gca_f2){1.0f, 1.0f});
    const gca_f2 e1 = __builtin_elementwise_fma(-x1, r1, (gca_f2){1.0f, 1.0f});
    const gca_f2 c0 = __builtin_elementwise_fma(e0, r0, r0);
    const gca_f2 c1 = __builtin_elementwise_fma(e1, r1, r1);
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(oa.x) : "v"(v.x), "v"(c0.x));
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(oa.y) : "v"(v.y), "v"(c0.y));
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(ob.x) : "v"(v.z), "v"(c1.x));
    asm("v_max_f32_e64 %0, %1, -%2" : "=v"(ob.y) : "v"(v.w), "v"(c1.y));
}
// *(T*)((char*)base + off): a wave-uniform base and a 32-bit lane byte offset (global_load ... v_off, s[base])
template <class T, class B> __device__ __forceinline__ T ld_at(const B* base, uint32_t off) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const unsigned char*>(base) + off);
}
// the same load, non-temporal (global_load ... nt): the streamed slope / age / vegetation-density rows are read once
// and should not displace the grid rows re-read R rows later from L2 (r04: with the non-temporal stores below and
// the skipped slope loads sent to one shared row, 26.2 -> 24.8 B/cell of HBM traffic, -4 % at 256^2, -13 % at 512^2)
template <class T, class B> __device__ __forceinline__ T ld_nt(const B* base, uint32_t off) {
    constexpr int N = (int)(sizeof(T) / 4);
    typedef uint32_t vt __attribute__((ext_vector_type(N)));
    typedef const __attribute__((address_space(1))) unsigned char gbyte;
    typedef const __attribute__((address_space(1))) vt gvt;
    const vt v = __builtin_nontemporal_load((gvt*)((gbyte*)base + off));
    return __builtin_bit_cast(T, v);
}
// Window sums as f32 pairs: the dot4 chains start from 2^23 (as f32 bits), so the sum's bits read as the float
// 2^23 + B exactly (B < 2^23) and one packed subtract gives (float)B for two cells instead of a v_cvt_f32_u32 each
constexpr uint32_t WZ = 0x4B000000u;
__device__ __forceinline__ gca_f2 wsum_f2(uint32_t b0, uint32_t b1) {
    return (gca_f2){__uint_as_float(b0), __uint_as_float(b1)} - (gca_f2){8388608.0f, 8388608.0f};
}
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef int16_t i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ i16x2 bitcast_i16x2(uint32_t v) { return __builtin_bit_cast(i16x2, v); }
__device__ __forceinline__ u16x2 bitcast_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
template <class T> __device__ __forceinline__ uint32_t bitcast_u32(T v) { return __builtin_bit_cast(uint32_t, v); }

// exchange items per edge lane (NSEG > 1): V_1..V_8, D_1, D_2, FIRE flags of rows r-1, r, r+1, two raw slopes, pad
constexpr int XI = 16;
constexpr int XS_ONE = 13, XS_TWO = 14;  // items holding raw slopes (1.0 in the border slots: factor 1)

// FLATM 1 / 2 (FLAT): every slope factor is 1 (flat terrain: edge_slope = NULL, e.g. use_hidden=False's
// init_altitude_same) -- no slope planes are streamed and every row takes the KILL pass (clamp01(base * wind) per
// direction), bit for bit what the general pass computes with factors of exactly 1.0. FLATM 2 (UNI): also every cell's
// vegetation / density byte is p.vd_uniform (vd = NULL; use_hidden=False's init_vegetation_same / init_density_same):
// the vd stream and the per-cell LUT reads go, the two factors are wave constants (the same f32 products in order)
template <int R, bool OBS, bool GROW, int NSEG, int FLATM>  // GROW: p_tree > 0 (EMPTY cells draw too); W = 256 * NSEG
// occupancy: 3 waves / SIMD for the step (VGPR-bound, <= 168; 4 would spill), 2 for the fused frame: its 3 KiB per
// wave-row of f32 RGB stores run faster from fewer concurrent waves (r05g, same box: 1.760 -> 1.723 ms per 4096 x 256^2
// step with the frame; the plain step at 2 waves: +8 %)
__global__ __launch_bounds__(NSEG == 1 ? 256 : 64 * NSEG) __attribute__((amdgpu_waves_per_eu(OBS ? (FLATM ? GCA_MARCH_OBS_FLAT_OCC : 2) : (FLATM ? GCA_MARCH_FLAT_OCC : 3), OBS ? (FLATM ? GCA_MARCH_OBS_FLAT_OCC : 2) : (FLATM ? GCA_MARCH_FLAT_OCC : 3)))) void alex_march_kernel(
    gca_alex_params p, int H, int nwaves, const uint8_t* __restrict__ grid_in, uint8_t* __restrict__ grid_out,
    const int16_t* age_in, int16_t* age_out,  // no __restrict__: the env updates ages in place
    const uint8_t* __restrict__ vd, const uint16_t* __restrict__ dbits, const float* __restrict__ es,
    const int32_t* __restrict__ wind_index, const uint32_t* __restrict__ rng_step, int32_t* __restrict__ counts,
    const uint8_t* __restrict__ act_in, uint8_t* __restrict__ act_out, MarchObs obs) {
    constexpr int NF = 2 * R + 2;  // fire ring rows r-R-1 .. r+R
    constexpr bool HALO = NSEG > 1;
    constexpr int WPB = HALO ? NSEG : 4;  // waves per workgroup: 4 independent tiles, or the NSEG segments of a strip
    constexpr int W = MW * NSEG;
    __shared__ float lut[WPB][16];
    __shared__ float4 colw[WPB][8];
    __shared__ float4 img[OBS ? WPB : 1][OBS ? 192 : 1];  // OBS: one RGB row (3 KiB) per wave
    __shared__ uint32_t fring[WPB][2 * NF * 64];              // per wave: the fire ring, each row twice
    // HALO: [row parity][segment + 1][edge lane 0, 1, 62, 63][item]; segments 0 and NSEG + 1 are the grid's border
    __shared__ uint32_t xch[HALO ? 2 : 1][HALO ? NSEG + 2 : 1][4][HALO ? XI : 1];
    __shared__ uint32_t qfl[HALO ? NSEG : 1];
    // XROW (NSEG = 1, the fused-frame kernel): the raw planes 0..2 of each wave's first row, for the wave of the tile
    // above, whose last rows need them as row r + 2 (the "17th row": otherwise loaded from HBM a second time, 0.75 B /
    // cell; 3 of a workgroup's 4 tile boundaries); xok: slot valid. r06 A/B (profiles/r06a, r06b): HBM traffic 24.70 ->
    // 24.15 B / cell; the fused-frame step -1.2 %, but the plain step +0-1.2 % (the one workgroup barrier aligns the
    // four waves' starts) and the reset state's quiet tiles +46 % (0.345 -> 0.503 ms): the plain kernel keeps the 17th row
    constexpr bool FLAT = FLATM >= 1, UNI = FLATM == 2;
    constexpr bool XROW = GCA_MARCH_XROW && !HALO && OBS && !FLAT;
    __shared__ float4 xrow[XROW ? 4 : 1][3][XROW ? 64 : 1];
    __shared__ uint32_t xok[XROW ? 4 : 1];

    // the wave index in SGPRs: everything derived from it (env, rows, base pointers, wind) stays scalar
    const int tid = threadIdx.x, wl = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    // XCD-aware order (as gca_alex.hip): blocks b, b+8, ... share an XCD; give each XCD a contiguous block range
    const int nb = (int)gridDim.x;
    const int xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
    const int qn8 = nb >> 3, rn8 = nb & 7;
    const int lb = (xcd < rn8 ? xcd * (qn8 + 1) : rn8 * (qn8 + 1) + (xcd - rn8) * qn8) + slot;
    int strips, e, s, g;
    if constexpr (!HALO) {
        const int wv = lb * 4 + wl;
        if (wv >= nwaves) {  // wave-uniform; no barrier follows -- but XROW's one barrier per live wave: join it
            if constexpr (XROW) {
                if (lane == 0) xok[wl] = 0u;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                __builtin_amdgcn_s_barrier();
            }
            return;
        }
        strips = H / SH;
        // (env-major wave order: one env's tiles back to back. A tile-major order inside chunks of 128 / 256 / 512
        //  envs, meant to turn the tiles' shared halo rows into L2 hits, measured 5 / 8 / 12 % slower, profiles/r03p)
        e = wv / strips;
        s = wv - e * strips;
        g = 0;
    } else {
        if (lb * NSEG >= nwaves) return;  // workgroup-uniform: every barrier below is reached by all its waves or none
        strips = H / SH;
        e = lb / strips;
        s = lb - e * strips;
        g = wl;
    }
    const int s0 = s * SH;
    const uint32_t HW = (uint32_t)H * W;
    const uint8_t* gE = grid_in + (size_t)e * HW;
    uint8_t* gO = grid_out + (size_t)e * HW;
    const int16_t* aE = age_in + (size_t)e * HW;
    int16_t* aO = age_out + (size_t)e * HW;
    const uint8_t* vE = UNI ? vd : vd + (size_t)e * HW;  // UNI: vd is NULL, never read
    const uint16_t* dE = dbits + (size_t)e * (HW >> 4);
    const float* sE = FLAT ? es : es + (size_t)e * 4 * HW;  // FLAT: es is NULL, never read
    // column of the lane's cell 0 (= its grid byte offset in a row) and its dousing-bit word (u16) in a row
    const uint32_t lc = HALO ? (uint32_t)(MW * g) + 4u * (uint32_t)lane : 4u * (uint32_t)lane;
    const uint32_t ld16 = HALO ? lc >> 4 : (uint32_t)(lane >> 2);
    const uint32_t lane_a = 2u * lc, lane_s = 4u * lc, lane_d = 2u * ld16;  // ages, slopes, dousing
    const uint32_t Fp = rep4((uint32_t)p.fire), Ep = rep4((uint32_t)p.empty), Tp = rep4((uint32_t)p.tree);

    if (lane < 16) lut[wl][lane] = gca_alex_lut_entry(p, lane);
    if (OBS && lane < 6) colw[wl][lane] = obs.col[6 * (obs.night[e] != 0 ? 1 : 0) + lane];
    // the env's frame mode (OBS_*; 0 = the plain frame of the grid)
    uint32_t omode = 0u;
    if constexpr (OBS && !HALO) {
        if (obs.action) {
            const int choice = min(max(obs.action[(size_t)e * obs.action_stride + 2], 0), obs.n_choices - 1);
            omode = (uint32_t)__builtin_amdgcn_readfirstlane((int)((obs.mode_bits >> (4 * choice)) & 0xFu));
        }
    }
    // the speculation check (tile 0 of the env; values 0..2 expected, any other code in rows 0 / 1 refits): some
    // enabled channel is positive in row 0 -- the grid (a TREE or FIRE) or its 3 x 3 edge-padded blur (round(S / 9)
    // >= 1 <=> S >= 5, S = 2 x (row 0's three columns) + (row 1's), the f32 arithmetic of apply_blur, gca_obs.hip)
    auto row0_refit = [&](uint32_t x0, uint32_t x1) -> uint8_t {
        const uint32_t odd = ((x0 + 0x7D7D7D7Du) | x0 | (x1 + 0x7D7D7D7Du) | x1) & 0x80808080u;  // a byte > 2
        bool pos = false;
        if (omode & OBS_CHK_GRID) pos |= __ballot(x0 != 0u) != 0ull;
        if (omode & OBS_CHK_BLUR) {
            auto hsum = [&](uint32_t x) {  // columns c-1 + c + c+1 per byte, the grid's edge columns replicated
                uint32_t L = __builtin_amdgcn_alignbyte(x, from_prev(x), 3);
                uint32_t Rt = __builtin_amdgcn_alignbyte(from_next(x), x, 1);
                if (lane == 0) L = (x << 8) | (x & 0xFFu);
                if (lane == 63) Rt = (x >> 8) | (x & 0xFF000000u);
                return L + x + Rt;
            };
            const uint32_t S = 2u * hsum(x0) + hsum(x1);
            pos |= __ballot(((S + 0x7B7B7B7Bu) & 0x80808080u) != 0u) != 0ull;
        }
        const bool bad = __ballot(odd != 0u) != 0ull;
        return ((omode & 3u) == OBS_NONE || bad || ((omode & (OBS_CHK_GRID | OBS_CHK_BLUR)) && !pos)) ? 1 : 0;
    };
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    auto graw = [&](int r) -> uint32_t {  // grid bytes of the lane's 4 cells in row r (EMPTY outside the grid)
        return (r >= 0 && r < H) ? *reinterpret_cast<const uint32_t*>(gE + (uint32_t)r * W + lc) : Ep;
    };
    auto draw_bits = [&](int r) -> uint32_t {  // the u16 of dousing bits holding the lane's 4 cells
        return (r >= 0 && r < H) ? (uint32_t)dE[(uint32_t)r * (W / 16) + ld16] : 0u;
    };
    auto dflags = [&](uint32_t w16) -> uint32_t { return gca_spread4(w16 >> (4 * (lane & 3))); };
    // The RGB row r of the lane's 4 cells (kinds from the new TREE / FIRE nibbles, pre-step dousing flags) through the
    // wave's LDS row: the 4 colours read back to back (one index byte per cell: 2 * kind + dousing), 3 x 16 B written,
    // then 3 x 1 KiB contiguous non-temporal stores (r03k: two rows per flush, or plain stores, measured slower)
    auto write_rgb_row = [&](int r, uint32_t tB, uint32_t fB, uint32_t dfl) {
        if constexpr (OBS) {
            if ((omode & 3u) == OBS_NONE) return;  // rendered by gca_adv_observation (refit)
            if ((omode & 3u) == OBS_ZERO) tB = fB = 0u;  // the display is an all-zero channel: EMPTY colours
            const uint32_t kidx = 2u * gca_spread4(tB) + 4u * gca_spread4(fB) + (dfl & 0x01010101u);
            // one cell at a time (3 live VGPRs instead of the 16 of four colours: the frame is written at the end of
            // the row, where row r+1's loads are in flight and the register file is full)
            float* im = reinterpret_cast<float*>(img[wl]) + 12 * lane;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 c = colw[wl][(kidx >> (8 * j)) & 0xFFu];
                im[3 * j + 0] = c.x;
                im[3 * j + 1] = c.y;
                im[3 * j + 2] = c.z;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            typedef float f4t __attribute__((ext_vector_type(4)));
            float* row = obs.rgb + ((size_t)e * H + r) * (W * 3) + (HALO ? (size_t)(MW * 3) * g : 0);
            float4 v[3];
#pragma unroll
            for (int t = 0; t < 3; ++t) v[t] = img[wl][64 * t + lane];
            // (r05 A/B, profiles/r05c/ab.txt: plain stores +4 %; the frame written before the grid / age stores: equal)
#pragma unroll
            for (int t = 0; t < 3; ++t)
                __builtin_nontemporal_store((f4t){v[t].x, v[t].y, v[t].z, v[t].w},
                                            reinterpret_cast<f4t*>(row + 4 * (64 * t + lane)));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // this row's reads before the next row's writes
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    };

    // XROW: every live wave of the workgroup passes exactly one workgroup barrier, after publishing its first row's
    // planes (or, a quiet tile, that it has none): the tile above reads them after its own barrier
    auto xrow_publish = [&](bool ok, const float4* planes) {
        if constexpr (XROW) {
            if (ok) {
#pragma unroll
                for (int k = 0; k < 3; ++k) xrow[wl][k][lane] = planes[k];
            }
            if (lane == 0) xok[wl] = ok ? 1u : 0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        }
    };

    // ---- quiet tiles: no FIRE in this tile's rows or the row on either side at the step's input -> with p_tree = 0
    //      nothing in the tile can change (a TREE burns only next to a FIRE; pinecones are a separate pass); copy it.
    //      Known from the tile activity map when the caller keeps one (gca_alex_step_packed; act_in only with
    //      p_tree == 0, host-checked), otherwise from the rows themselves: two rows first (in a dense state they
    //      already hold a FIRE, so the check costs a few VALU), then the other 16 at once
    //      (r03ac: the episode's first steps, where most tiles are quiet, no longer run the full step on them)
    // the fire ring's first rows (s0 - R - 1 .. s0 + R - 1) are loaded before the check, which reads two of them: a
    // dense tile pays no extra round trip
    uint32_t g_init[NF - 1];
#pragma unroll
    for (int t = 0; t < NF - 1; ++t) g_init[t] = graw(s0 - R - 1 + t);
    // a quiet tile: the input rows copied (grid, ages when not in place, the frame) and counted; row(i) gives row s0+i
    auto quiet_copy = [&](auto row) {
        int cE = 0, cT = 0;
#pragma unroll
        for (int i = 0; i < SH; ++i) {
            const int r = s0 + i;
            const uint32_t o = (uint32_t)r * W + lc;
            const uint32_t gw = row(i);
            __builtin_nontemporal_store(gw, reinterpret_cast<uint32_t*>(gO + o));
            if (age_in != age_out) *reinterpret_cast<uint2*>(aO + o) = *reinterpret_cast<const uint2*>(aE + o);
            cE += __builtin_popcount(bytes_eq01(gw, Ep));
            cT += __builtin_popcount(bytes_eq01(gw, Tp));
            if (OBS) write_rgb_row(r, gca_eq_nib(gw, Tp), 0u, dflags(draw_bits(r)));
        }
        if constexpr (OBS && !HALO) {
            if (obs.refit && s0 == 0) {
                const uint8_t rf = row0_refit(row(0), row(1));
                if (lane == 0) obs.refit[e] = rf;
            }
        }
        if (act_out && lane == 0) act_out[((size_t)e * strips + s) * NSEG + g] = 0;
        if (counts) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                cE += __shfl_xor(cE, off);
                cT += __shfl_xor(cT, off);
            }
            if (lane == 0) {
                if (cE) atomicAdd(counts + 3 * e + 0, cE);
                if (cT) atomicAdd(counts + 3 * e + 1, cT);
            }
        }
    };
    bool quiet = false;
    if (!HALO && act_out && act_in) {
        const uint8_t* A = act_in + (size_t)e * strips;
        quiet = !(A[s] | (s > 0 ? A[s - 1] : 0) | (s + 1 < strips ? A[s + 1] : 0));
    } else if constexpr (!GROW) {
        auto has_fire = [&](uint32_t x) {  // some byte of x is the FIRE code (exact: the zero-byte test of x ^ Fp)
            const uint32_t v = x ^ Fp;
            return (v - 0x01010101u) & ~v & 0x80808080u;
        };
        if (__ballot((has_fire(g_init[R]) | has_fire(g_init[R + 1])) != 0u) == 0ull) {  // rows s0 - 1, s0
            uint32_t gq[SH];  // rows s0 .. s0+SH-1, kept for the copy (no second load round trip, r04)
            gq[0] = g_init[R + 1];
            uint32_t f = has_fire(graw(s0 + SH));
#pragma unroll
            for (int i = 1; i < SH; ++i) {
                gq[i] = graw(s0 + i);
                f |= has_fire(gq[i]);
            }
            quiet = __ballot(f != 0u) == 0ull;
            if constexpr (!HALO) {
                if (quiet) {
                    xrow_publish(false, nullptr);
                    quiet_copy([&](int i) { return gq[i]; });
                    return;
                }
            }
        }
    }
    if constexpr (HALO) {
        // the strip is quiet only when every segment is (a FIRE in a neighbour segment's edge column can ignite this
        // one): one consensus, so all waves of the workgroup take the same path through the barriers below. Wave 0
        // also fills the border slots of the exchange (both parities): zero sums / flags, raw slope 1.0 (factor 1)
        if (wl == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int idx = 4 * lane + j;  // 256 = 2 parities x 2 border slots x 4 edge lanes x 16 items
                const int item = idx & 15, li = (idx >> 4) & 3, sl = ((idx >> 6) & 1) ? NSEG + 1 : 0, pa = idx >> 7;
                xch[pa][sl][li][item] = (item == XS_ONE || item == XS_TWO) ? 0x3F800000u : 0u;
            }
        }
        if (lane == 0) qfl[wl] = quiet ? 1u : 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        uint32_t all = 1u;
#pragma unroll
        for (int w = 0; w < NSEG; ++w) all &= qfl[w];
        quiet = all != 0u;
    }
    if (quiet) {  // the tile map's verdict, or every segment of a strip quiet (HALO): rows loaded again
        xrow_publish(false, nullptr);
        quiet_copy([&](int i) { return *reinterpret_cast<const uint32_t*>(gE + (uint32_t)(s0 + i) * W + lc); });
        return;
    }

    // ---- fire ring in LDS: the FIRE flags (0x01 bytes) of rows r-R-1 .. r+R, one dword per lane and row, each row
    //      stored twice (slots t and t + NF), so that the rows around r sit at fixed offsets from one base that moves
    //      by one slot per row: immediate-offset ds_read_b32, no register rotation. Rows are stored in DESCENDING
    //      order (the base moves down one slot per row): the entering row sits at the base and its copy at base + NF,
    //      both immediate offsets off the address the reads use (ascending order put the copy at base - 1, which took
    //      a second per-lane address register and, in the fused-frame variant, a spill, r03p)
    uint32_t* FR = fring[wl];
    auto ring_put = [&](int t, uint32_t v) {  // relative row t = row - (s0 - R - 1): slot NF - 1 - t (row 0's base)
        const int sl = (2 * NF - 2 - t) % NF;
        FR[sl * 64 + lane] = v;
        FR[(sl + NF) * 64 + lane] = v;
    };
#pragma unroll
    for (int t = 0; t < NF - 1; ++t) ring_put(t, bytes_eq01(g_init[t], Fp));
    uint32_t dring[6];
#pragma unroll
    for (int t = 0; t < 5; ++t) dring[t] = dflags(draw_bits(s0 - 3 + t));
    // loads of row s0 (and the slopes of rows s0, s0+1)
    // row r's own codes are re-read one row ahead (nOwn) although the ring saw them R rows earlier: a per-wave LDS ring
    // of the codes instead cuts the traffic by 1.0 B / cell (26.2 -> 25.2) but measured 0.6-2 % slower (r03q/r03r)
    uint32_t nG = graw(s0 + R), nD = draw_bits(s0 + 2), nOwn = graw(s0);
    uint32_t nVD = UNI ? 0u : *reinterpret_cast<const uint32_t*>(vE + (size_t)s0 * W + lc);
    uint2 nAge = *reinterpret_cast<const uint2*>(aE + (size_t)s0 * W + lc);
    float4 sc[4], sn[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if constexpr (FLAT) {
            sc[k] = sn[k] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
        } else {
            sc[k] = ldf4(sE + (size_t)k * HW + (size_t)s0 * W + lc);
            sn[k] = ldf4(sE + (size_t)k * HW + (size_t)min(s0 + 1, H - 1) * W + lc);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    xrow_publish(true, sc);  // (raw planes: prep_own below rewrites sc)
    // the tile below is the next wave of this workgroup, in the same env, and published its first row
    const bool xuse = XROW && wl < 3 && s0 + SH < H && xok[XROW ? wl + 1 : 0] != 0u;
    uint32_t V[R + 1];
#pragma unroll
    for (int k = 1; k <= R; ++k) {
        uint32_t v = 0u;
#pragma unroll
        for (int t = R - k; t <= R + k; ++t) v += FR[((2 * NF - 2 - t) % NF) * 64 + lane];
        V[k] = v;
    }
    uint32_t Dv1 = dring[1] + dring[2] + dring[3];
    uint32_t Dv2 = dring[0] + Dv1 + dring[4];

    // border columns 0 and W-1 (lanes 0 / 63 of the first / last segment, elements 0 / 3): slope factor 1 (the rows
    // 0 / H-1: kill_row below)
    const bool col_lo = lane == 0 && (!HALO || g == 0), col_hi = lane == 63 && (!HALO || g == NSEG - 1);
    // HALO: the lane's read offset into a parity of the exchange: lane 63 reads the right segment's lane 0 (and 1),
    // every other lane the left segment's lane 63 (and 62) — only lane 0's value is used; the rest read it broadcast
    const uint32_t xo1 = HALO ? (lane == 63 ? (uint32_t)(((g + 2) * 4 + 0) * XI) : (uint32_t)((g * 4 + 3) * XI)) : 0u;
    const uint32_t xo2 = HALO ? (lane == 63 ? (uint32_t)(((g + 2) * 4 + 1) * XI) : (uint32_t)((g * 4 + 2) * XI)) : 0u;
    // row s0's own factors of planes 0..2 (row r's directions 0..2 read prepared own factors; plane 3 stays raw)
    auto prep_own = [&](float4& v) {
        gca_f2 a, b;
        m_edge_own4(v, a, b);
        v = make_float4(col_lo ? 1.0f : a.x, a.y, b.x, col_hi ? 1.0f : b.y);
    };
    if constexpr (!FLAT) {
#pragma unroll
        for (int k = 0; k < 3; ++k) prep_own(sc[k]);
    }

    // the per-env constants of the packed f32 arithmetic, two per VGPR pair, held in VGPRs: as SGPR operands hipcc
    // materialises every (x, x) pair as two SGPRs, and the 30-odd of them were spilled to VGPR lanes and read back per
    // row. A constant is used as the pair (x, x) through op_sel (one half of the pair broadcast), so the 8 winds and
    // R + 1 heat weights take 8 + 2 ceil((R + 1) / 2) VGPRs instead of 16 + 2 (R + 1) (r03p: the fused-frame variant
    // spilled two VGPRs, whose per-row reloads waited for the row-ahead loads)
    constexpr int NHW = (R + 2) / 2;
    gca_f2 windp[4], hdwp[NHW];
    {
        const int widx = wind_index[e];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int d0 = 2 * q, d1 = 2 * q + 1;
            windp[q] = (gca_f2){p.winds[widx][d0 < 4 ? d0 : d0 + 1], p.winds[widx][d1 < 4 ? d1 : d1 + 1]};
            asm volatile("" : "+v"(windp[q]));
        }
#pragma unroll
        for (int q = 0; q < NHW; ++q) {
            hdwp[q] = (gca_f2){p.heat_dw[2 * q], 2 * q + 1 <= R ? p.heat_dw[2 * q + 1] : 0.0f};
            asm volatile("" : "+v"(hdwp[q]));
        }
    }
    // UNI: the two layer factors (1 + p_veg, 1 + p_den) of every cell, as the LUT entries of the uniform vd byte
    gca_f2 avd = {1.0f, 1.0f};
    if constexpr (UNI) {
        const int b = p.vd_uniform & 0xFF;
        avd = (gca_f2){gca_alex_lut_entry(p, b & 7), gca_alex_lut_entry(p, 8 + ((b >> 4) & 7))};
        asm volatile("" : "+v"(avd));
    }
    auto bcast = [](gca_f2 v, int h) -> gca_f2 {
        return h ? __builtin_shufflevector(v, v, 1, 1) : __builtin_shufflevector(v, v, 0, 0);
    };
    const uint32_t step = rng_step ? rng_step[e] : 0u;
    const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
    const uint32_t env_id = (uint32_t)(p.env_offset + e);
    // Philox4x32-10 of the counter (cell pair, env, step, tag) (gca_common.h philox4x32_10, bit for bit): words 1..3
    // are the same for every block of the wave, so the first round's M1 x step product (words 0 / 1 after round 1)
    // and the second round's M0 product of word 0 are wave constants, computed once here on the scalar unit; per block
    // the lane does one multiply in each of the first two rounds instead of two (r04)
    constexpr uint32_t PM0 = 0xD2511F53u, PM1 = 0xCD9E8D57u, PW0 = 0x9E3779B9u, PW1 = 0xBB67AE85u;
    const uint64_t pq1 = (uint64_t)PM1 * step;
    const uint32_t pu0 = (uint32_t)(pq1 >> 32) ^ env_id ^ k0;  // word 0 after round 1 (uniform)
    const uint64_t pq2 = (uint64_t)PM0 * pu0;                   // round 2's word-0 product (uniform)
    const uint32_t pkc = (uint32_t)GCA_TAG_ALEX_CELL ^ k1;      // round 1: word 2 = hi0 ^ tag ^ k1
    const uint32_t pkc_age = (uint32_t)GCA_TAG_ALEX_AGE ^ k1;   // the same for the rare second block (tag ALXA)
    const uint32_t pka = (uint32_t)pq1 ^ (k0 + PW0);            // round 2: word 0 = hi1 ^ (word 1 = lo(M1 step)) ^ key
    const uint32_t pkb = (uint32_t)(pq2 >> 32) ^ (k1 + PW1);    // round 2: word 2 = hi(M0 pu0) ^ (word 3 = lo0) ^ key
    const uint32_t pl2 = (uint32_t)pq2;                         // round 2: word 3 = lo(M0 pu0)
    auto philox_cell = [&](uint32_t x0, uint32_t rk0, uint32_t rk1, uint32_t ktag) -> u32x4 {
        const uint64_t p0 = (uint64_t)PM0 * x0;  // round 1
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint64_t p1 = (uint64_t)PM1 * (hi0 ^ ktag);  // round 2 (word 2 after round 1)
        u32x4 c = u32x4{(uint32_t)(p1 >> 32) ^ pka, (uint32_t)p1, lo0 ^ pkb, pl2};
#pragma unroll
        for (int i = 2; i < 10; ++i) {  // rounds 3..10 as philox4x32_10, keys (k0 + i W0, k1 + i W1)
            const uint64_t a = (uint64_t)PM0 * c.x;
            const uint64_t b = (uint64_t)PM1 * c.z;
            const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(b >> 32), c.y, rk0 + (uint32_t)i * PW0, 0x96);
            const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), c.w, rk1 + (uint32_t)i * PW1, 0x96);
            c = u32x4{n0, (uint32_t)b, n2, (uint32_t)a};
        }
        return c;
    };
    const float pt24 = __fmul_rn(p.p_tree, 16777216.0f);
    const float w_in_minus_bd = __fsub_rn(p.dous_inner, p.dous_border);
    const uint32_t codes = (p.empty & 0xFFu) | ((p.tree & 0xFFu) << 8) | ((p.fire & 0xFFu) << 16);
    int cntE = 0, cntT = 0, cntF = 0;
    uint32_t out_row0 = 0u;  // OBS refit check: the new codes of row 0 (tile 0)

    // one row of the tile. SC: row r's planes (0..2 as prepared own factors, 3 raw); SN: row r+1's raw planes.
    // After the row, SN holds row r+1's prepared planes and SC row r+2's raw planes (loaded once direction 4 has
    // read SC): the caller swaps the roles.
    auto row = [&](const int i, float4 (&SC)[4], float4 (&SN)[4], auto parity) {
        const int r = s0 + i;
        // ---- this row's inputs (loaded one row ago); issue row r+1's (rows clamped into the grid: the last row's
        //      loads are unused, and unconditional loads keep the two rows of the loop body branch-free)
        const uint32_t gnew = nG, dnew = nD, own = nOwn, vdw = nVD;
        const uint2 agep = nAge;
        {  // (wave-uniform row base pointers + a 32-bit lane byte offset; raw buffer loads with SGPR row offsets were
           //  measured 2.5 % slower, profiles/r03n/ab_buffer_loads.txt)
            // (the tile's last row loads the next tile's row r+1 here, unused; reading one shared row instead -- ~0.2
            //  B / cell less HBM traffic -- measured 1 % slower, profiles/r05c/ab.txt: ~3000 waves on the same
            //  few hundred bytes)
            const int rg = r + 1 + R, rd = r + 3;
            const uint32_t r1 = (uint32_t)min(r + 1, H - 1);
            const uint32_t gl = ld_at<uint32_t>(gE + (size_t)min(rg, H - 1) * W, lc);
            const uint32_t d = ld_at<uint16_t>(dE + (size_t)min(rd, H - 1) * (W / 16), lane_d);
            nOwn = ld_at<uint32_t>(gE + (size_t)r1 * W, lc);
            if constexpr (!UNI) nVD = ld_nt<uint32_t>(vE + (size_t)r1 * W, lc);
            nAge = ld_nt<uint2>(aE + (size_t)r1 * W, lane_a);
            nG = rg < H ? gl : Ep;
            nD = rd < H ? d : 0u;
        }
        // Row r+2's slope planes (loaded during this row) serve rows r+1 and r+2, which can only need them with a FIRE
        // in rows r..r+3, and only inside the tile (the last row's row r+2 is the next tile's): otherwise the load
        // reads one shared row (below; a branch around the load would keep SC live and cost registers), and the
        // values are never used (those rows' row_need is false). The ring holds rows up to r+R; R < 3 always loads.
        // (Until r04 a skipped load re-read the tile's first row, taken to be L2-resident: it was not — the tile's
        // last rows re-fetched it from HBM, ~1 B/cell.)
        bool need_next = i + 1 < SH;
        auto load_next_slopes = [&]() {  // row r+2's raw planes into SC
            if constexpr (XROW) {
                if (i == SH - 2 && xuse) {  // row r+2 = the next tile's first row: from its wave's LDS slot
#pragma unroll
                    for (int k = 0; k < 3; ++k) SC[k] = xrow[wl + 1][k][lane];
                    SC[3] = SC[2];  // plane 3 of row r+2 serves row r+2 only (the next tile's): unused here
                    return;
                }
            }
            // plane 3 of row r+2 serves row r+2 itself only: the next tile's first row (i = SH - 2) skips it too.
            // A skipped load reads row 0 of env 0's planes instead (the same 4 KiB for every wave: L2-resident,
            // while the streamed planes are loaded non-temporally and do not stay)
            const bool need3 = need_next && i + 2 < SH;
            const float* sb = need_next ? sE : es;
            const float* sb3 = need3 ? sE : es;
            const uint32_t rs = need_next ? (uint32_t)min(r + 2, H - 1) : 0u;
            const uint32_t rs3 = need3 ? rs : 0u;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                SC[k] = ld_nt<float4>((k == 3 ? sb3 : sb) + (size_t)k * HW + (size_t)(k == 3 ? rs3 : rs) * W, lane_s);
        };
        // ---- fire ring: row r+R enters; the running vertical sums move to row r
        uint32_t* Fb = FR + (NF - 1 - (uint32_t)i % NF) * 64;  // slot of row r+R; row r+R-t at slot + t
        {
            const uint32_t fnew = bytes_eq01(gnew, Fp);  // row r+R: offset 0 and its copy at +NF (both immediates off
            Fb[lane] = fnew;                             // the one address the reads use)
            Fb[NF * 64 + lane] = fnew;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t fm1, f0, fp1;  // FIRE flags of rows r-1, r, r+1
        {
            uint32_t rw[NF];
#pragma unroll
            for (int t = 0; t < NF; ++t) rw[t] = Fb[(NF - 1 - t) * 64 + lane];  // rw[t] = row r-R-1+t
#pragma unroll
            for (int k = 1; k <= R; ++k) V[k] += rw[R + 1 + k] - rw[R - k];
            fm1 = rw[R];
            f0 = rw[R + 1];
            fp1 = rw[R + 2];
            if constexpr (R >= 3)
                need_next = need_next && __ballot((rw[R + 1] | rw[R + 2] | rw[R + 3] | rw[R + 4]) != 0u) != 0ull;
        }
        dring[5] = dflags(dnew);
        Dv1 += dring[4] - dring[1];
        Dv2 += dring[5] - dring[0];

        // ---- HALO: post this row's edge values for the neighbour segments, one barrier, and read theirs. xr / xr2:
        //      the neighbours' items (lane 0: left segment's lanes 63 / 62; lane 63: right segment's lanes 0 / 1).
        //      Raw slopes posted: lane 0 the plane 3 value of (r, first column) and plane 0 of (r+1, first column),
        //      lane 63 plane 2 of (r+1, last column) — what the neighbour's directions 4 / 7 and 5 read across the edge
        //      (if the neighbour needs one, its cell there burns, so this wave loaded real planes: need_next above)
        const uint32_t* xr = nullptr;
        const uint32_t* xr2 = nullptr;
        uint32_t hfm1 = 0u, hf0 = 0u, hfp1 = 0u;
        if constexpr (HALO) {
            constexpr int PAR = decltype(parity)::value;
            if (lane < 2 || lane >= 62) {
                const int xl = lane < 2 ? lane : lane - 60;
                uint4* xd = reinterpret_cast<uint4*>(&xch[PAR][g + 1][xl][0]);
                uint32_t vv[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) vv[k] = k + 1 <= R ? V[k + 1] : 0u;
                const uint32_t sA = lane < 32 ? __float_as_uint(SC[3].x) : __float_as_uint(SN[2].w);
                xd[0] = make_uint4(vv[0], vv[1], vv[2], vv[3]);
                xd[1] = make_uint4(vv[4], vv[5], vv[6], vv[7]);
                xd[2] = make_uint4(Dv1, Dv2, fm1, f0);
                xd[3] = make_uint4(fp1, sA, __float_as_uint(SN[0].x), 0u);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
            xr = &xch[PAR][0][0][0] + xo1;
            xr2 = &xch[PAR][0][0][0] + xo2;
            hfm1 = xr[10];
            hf0 = xr[11];
            hfp1 = xr[12];
        }

        // ---- masks of the row: own kinds, FIRE neighbourhood (3 rows x 6 columns per lane)
        const uint32_t treeB = gca_eq_nib(own, Tp), emptyB = gca_eq_nib(own, Ep);
        // burning-neighbour masks: 0xFF in byte j iff cell j's neighbour d is FIRE, from the row dwords shifted one
        // column across lanes ([prev.b3, X.b0..b2] / [X.b1..b3, next.b0]); built per direction inside the pass (8
        // live masks cost registers), and masked into the products with one SDWA v_and per cell
        auto shl_c = [](uint32_t x, uint32_t h) {  // column c-1 (HALO: lane 0's from the left segment)
            return __builtin_amdgcn_alignbyte(x, HALO ? from_prev_or(h, x) : from_prev(x), 3);
        };
        auto shr_c = [](uint32_t x, uint32_t h) {  // column c+1 (HALO: lane 63's from the right segment)
            return __builtin_amdgcn_alignbyte(HALO ? from_next_or(h, x) : from_next(x), x, 1);
        };
        auto dir_mask = [&](int d) -> uint32_t {
            const uint32_t row = d < 3 ? fm1 : (d < 5 ? f0 : fp1);
            const uint32_t hrow = d < 3 ? hfm1 : (d < 5 ? hf0 : hfp1);
            const int dc = d < 3 ? d - 1 : (d == 3 ? -1 : (d == 4 ? 1 : d - 6));
            uint32_t m = dc < 0 ? shl_c(row, hrow) : (dc > 0 ? shr_c(row, hrow) : row);
            m *= 0xFFu;
            asm volatile("" : "+v"(m));  // opaque: hipcc would fold the byte extractions into per-byte multiplies
            return m;
        };
        const uint32_t fireB = (f0 * 0x01020408u) >> 24;
        // a FIRE anywhere in the 3 x 3 block (the centre too: it only matters for TREE cells, which are not FIRE)
        const uint32_t vor = fm1 | f0 | fp1, hvor = hfm1 | hf0 | hfp1;
        const uint32_t anyfire = (((vor | shl_c(vor, hvor) | shr_c(vor, hvor)) & 0x01010101u) * 0x01020408u) >> 24;
        gca_f2 qn[2] = {{1.0f, 1.0f}, {1.0f, 1.0f}};
        const bool row_need = __ballot((treeB & anyfire) != 0u) != 0ull;
        const bool kill_row = r == 0 || r == H - 1;       // every factor of row r is 1
        const bool kill_next = r + 1 == H - 1;            // row r+1's own factors are 1 (prepared here)
        // own factors of SN's plane k for row r+1 (and, when `nb`, the neighbour factors row r's directions 5..7 use)
        auto prep_next = [&](int k, bool want_nb, float (&nbv)[4]) {
            gca_f2 oa, ob, na, nb2;
            if (want_nb) {
                m_edge_both4(SN[k], oa, na, ob, nb2);
                nbv[0] = na.x; nbv[1] = na.y; nbv[2] = nb2.x; nbv[3] = nb2.y;
            } else {
                m_edge_own4(SN[k], oa, ob);
            }
            SN[k] = make_float4(col_lo ? 1.0f : oa.x, oa.y, ob.x, col_hi ? 1.0f : ob.y);
        };
        if (!row_need) {
            if constexpr (!FLAT) {
                load_next_slopes();
                float unused[4];
#pragma unroll
                for (int k = 0; k < 3; ++k) prep_next(k, false, unused);
            }
        } else {
            // ---- heat = heat0 + sum_k dw_k * B_k (k = 0..R, fma chain), minus the dousing term
            gca_f2 ph[2] = {{p.heat0, p.heat0}, {p.heat0, p.heat0}};
#pragma unroll
            for (int k = 0; k <= R; ++k) {
                uint32_t B[4];
                if (k == 0) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) B[j] = (f0 >> (8 * j)) & 0xFFu;
                } else {
                    if constexpr (HALO)
                        window4<true>(V[k], k, B, WZ, xr[k - 1], k >= 5 ? xr2[k - 1] : 0u);
                    else
                        window4(V[k], k, B, WZ);
                }
                gca_f2 bs[2];  // both pairs converted first, then both fmas (no dependent back-to-back packed op)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    bs[h] = k == 0 ? (gca_f2){(float)B[2 * h], (float)B[2 * h + 1]} : wsum_f2(B[2 * h], B[2 * h + 1]);
#pragma unroll
                for (int h = 0; h < 2; ++h) ph[h] = __builtin_elementwise_fma(bcast(hdwp[k >> 1], k & 1), bs[h], ph[h]);
                // one radius at a time (hipcc would otherwise interleave all the radii's DPP / dot4 work)
                asm volatile("" : "+v"(ph[0]), "+v"(ph[1]));
                __builtin_amdgcn_sched_barrier(0);
            }
            // the dousing term only where the wave sees a doused cell in its 5 x 5 windows (the 5-row sums Dv2 contain
            // the 3-row Dv1; HALO: the neighbour segments' edge sums too). Dousing is sparse (one bulldozer per env):
            // most wave-rows skip the two windows. Skipping subtracts nothing instead of +-0, which can differ only in
            // the sign of a zero heat; a zero heat gives every direction's factor +-0, which leaves qn unchanged either
            // way, so the step's outputs are the same bit for bit
            const bool dous_any = __ballot((Dv2 | (HALO ? xr[8] | xr[9] : 0u)) != 0u) != 0ull;
            if (dous_any) {  // the two pairs interleaved step by step (no packed result read by the next instruction)
                uint32_t D1[4], D2[4];
                if constexpr (HALO) {
                    window4<true>(Dv1, 1, D1, WZ, xr[8]);
                    window4<true>(Dv2, 2, D2, WZ, xr[9]);
                } else {
                    window4(Dv1, 1, D1, WZ);
                    window4(Dv2, 2, D2, WZ);
                }
                gca_f2 d1[2], d2[2], dz[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) d1[h] = wsum_f2(D1[2 * h], D1[2 * h + 1]);
#pragma unroll
                for (int h = 0; h < 2; ++h) d2[h] = wsum_f2(D2[2 * h], D2[2 * h + 1]);
#pragma unroll
                for (int h = 0; h < 2; ++h) dz[h] = (gca_f2){w_in_minus_bd, w_in_minus_bd} * d1[h];
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    dz[h] = __builtin_elementwise_fma((gca_f2){p.dous_border, p.dous_border}, d2[h], dz[h]);
#pragma unroll
                for (int h = 0; h < 2; ++h) ph[h] = ph[h] - dz[h];
            }
            // ---- base = (p_h * (1 + p_veg)) * (1 + p_den)
            if constexpr (UNI) {
#pragma unroll
                for (int h = 0; h < 2; ++h) ph[h] = ph[h] * bcast(avd, 0);
#pragma unroll
                for (int h = 0; h < 2; ++h) ph[h] = ph[h] * bcast(avd, 1);
            } else {
                gca_f2 av[2], ad[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t b0 = (vdw >> (16 * h)) & 0xFFu, b1 = (vdw >> (16 * h + 8)) & 0xFFu;
                    av[h] = (gca_f2){lut[wl][b0 & 7u], lut[wl][b1 & 7u]};
                    ad[h] = (gca_f2){lut[wl][8 + (b0 >> 4)], lut[wl][8 + (b1 >> 4)]};
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) ph[h] = ph[h] * av[h];
#pragma unroll
                for (int h = 0; h < 2; ++h) ph[h] = ph[h] * ad[h];
            }
            // ---- directions, in order: qn = prod over burning d of (1 - clamp01(base * wind[d] * p_slope[d])), each
            //      factor as qn = fma(-qn, c, qn);
            //      rows 0 and H-1 (KILL: every factor 1, no edge arithmetic) take their own copy of the pass
            auto dir_pass = [&](auto kill_tag) {
                constexpr bool KILL = decltype(kill_tag)::value;
                auto apply = [&](int d, const float (&a)[4]) {
                    // pin base and the product: otherwise the direction-independent work of all 8 directions is
                    // hoisted (as in gca_alex.hip)
                    asm volatile("" : "+v"(ph[0]), "+v"(ph[1]), "+v"(qn[0]), "+v"(qn[1]));
                    const gca_f2 wd2 = bcast(windp[d >> 1], d & 1);
                    const uint32_t Md = dir_mask(d);
                    // the two cell pairs' chains interleaved step by step (a packed f32 result read by the next
                    // instruction costs a wait state; two independent chains hide it)
                    // (KILL: every factor 1, so clamp01(base * wind) is the product's own clamp modifier -- one packed
                    //  op per pair; with the flat-terrain step every row takes it)
                    gca_f2 c[2];
                    if constexpr (KILL) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) c[h] = gca_pk_mul_clamp01(ph[h], wd2);
                    } else {
                        gca_f2 t[2];
#pragma unroll
                        for (int h = 0; h < 2; ++h) t[h] = ph[h] * wd2;
#pragma unroll
                        for (int h = 0; h < 2; ++h) c[h] = gca_pk_mul_clamp01(t[h], (gca_f2){a[2 * h], a[2 * h + 1]});
                    }
                    // qn <- fma(-qn, c, qn) = qn * (1 - c), one rounding (the oracle's order); no burning
                    // neighbour d: c -> +0 and qn is unchanged exactly (the oracle skips the factor)
                    uint32_t cm[2][2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        cm[h][0] = __float_as_uint(c[h].x) & (uint32_t)(int32_t)(int8_t)(Md >> (16 * h));
                        cm[h][1] = __float_as_uint(c[h].y) & (uint32_t)(int32_t)(int8_t)(Md >> (16 * h + 8));
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        qn[h] = __builtin_elementwise_fma(-qn[h], (gca_f2){__uint_as_float(cm[h][0]), __uint_as_float(cm[h][1])},
                                                          qn[h]);
                    __builtin_amdgcn_sched_barrier(0);
                };
                const float one[4] = {1.0f, 1.0f, 1.0f, 1.0f};
                // HALO: the neighbour factors across the segment's edges (lane 63: planes 3 of (r, c+1) and 0 of
                // (r+1, c+1) for directions 4 / 7; lane 0: plane 2 of (r+1, c-1) for direction 5), from the raw values
                // the neighbour segments posted; at the grid's border the posted raw 1.0 gives factor 1
                uint32_t h45 = 0x3F800000u, h7 = 0x3F800000u;
                if constexpr (HALO && !KILL) {
                    gca_f2 o_, n_;
                    m_edge_both(__uint_as_float(xr[XS_ONE]), __uint_as_float(xr[XS_TWO]), o_, n_);
                    h45 = __float_as_uint(n_.x);
                    h7 = __float_as_uint(n_.y);
                }
#pragma unroll
                for (int d = 0; d < 3; ++d) {  // prepared own factors of planes 0..2
                    const float a[4] = {SC[d].x, SC[d].y, SC[d].z, SC[d].w};
                    apply(d, KILL ? one : a);
                }
                if (KILL) {
                    apply(3, one);
                    apply(4, one);
                } else {  // plane 3 of row r: own factor (d = 3) and, one column on, the neighbour factor (d = 4)
                    gca_f2 oa, ob, na, nb2;
                    m_edge_both4(SC[3], oa, na, ob, nb2);
                    const float a3[4] = {col_lo ? 1.0f : oa.x, oa.y, ob.x, col_hi ? 1.0f : ob.y};
                    apply(3, a3);
                    // (r, c+1)'s plane 3; lane 63's last cell is column 255 (DPP old = 1.0; HALO: the right segment's)
                    const float nx = __uint_as_float((uint32_t)__builtin_amdgcn_update_dpp(
                        (int)h45, (int)__float_as_uint(na.x), 0x130, 0xF, 0xF, false));
                    const float a4[4] = {col_lo ? 1.0f : na.y, nb2.x, nb2.y, nx};
                    apply(4, a4);
                }
                if constexpr (!FLAT) load_next_slopes();
                float nb[4];
                // plane 2 of (r+1, c-1): lane 0's first cell is column 0 (DPP old = 1.0)
                if constexpr (!FLAT) prep_next(2, !KILL, nb);
                if (KILL) {
                    apply(5, one);
                } else {
                    const float pv = __uint_as_float((uint32_t)__builtin_amdgcn_update_dpp(
                        (int)h45, (int)__float_as_uint(nb[3]), 0x138, 0xF, 0xF, false));
                    const float a5[4] = {pv, nb[0], nb[1], col_hi ? 1.0f : nb[2]};
                    apply(5, a5);
                }
                // plane 1 of (r+1, c)
                if constexpr (!FLAT) prep_next(1, !KILL, nb);
                if (KILL) {
                    apply(6, one);
                } else {
                    const float a6[4] = {col_lo ? 1.0f : nb[0], nb[1], nb[2], col_hi ? 1.0f : nb[3]};
                    apply(6, a6);
                }
                // plane 0 of (r+1, c+1): lane 63's last cell is column 255 (DPP old = 1.0)
                if constexpr (!FLAT) prep_next(0, !KILL, nb);
                if (KILL) {
                    apply(7, one);
                } else {
                    const float nx = __uint_as_float((uint32_t)__builtin_amdgcn_update_dpp(
                        (int)h7, (int)__float_as_uint(nb[0]), 0x130, 0xF, 0xF, false));
                    const float a7[4] = {col_lo ? 1.0f : nb[1], nb[2], nb[3], nx};
                    apply(7, a7);
                }
            };
            if (FLAT || kill_row)
                dir_pass(std::true_type{});
            else
                dir_pass(std::false_type{});
        }
        if (kill_next) {  // row H-1: its own factors are 1 (its neighbour factors come from outside the grid)
#pragma unroll
            for (int k = 0; k < 3; ++k) SN[k] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
        }

        // ---- draws (r05): one Philox block per lane-row -- the lane's 4 cells are the group (r, 4l .. 4l+3), counter
        //      r * W/4 + l = lin0 >> 2 (gca.h GCA_TAG_ALEX_CELL; as gca_alex.hip and the C oracle). Cell j's burn / grow
        //      uniform is word j's high 24 bits; the low bytes, which no decision reads, make the spare word whose
        //      randint is the age of the lane's first new fire. Until r04 every cell pair took a block (its second
        //      word the cell's age draw): 2 blocks per lane-row, ~100 of ~640 VALU per wave-row
        const uint32_t needB = (treeB & anyfire) | (GROW ? emptyB : 0u);
        const uint32_t lin0 = (uint32_t)r * W + lc;
        uint32_t burn = 0u, grow = 0u, NA[2];
        // every lane draws when any lane of the wave needs to (a wave-uniform branch instead of a masked one per
        // lane): the draws of cells that need none are discarded (qn = 1 gives thr = 0; grow is masked by EMPTY)
        const bool wave_draws = __ballot(needB != 0u) != 0ull;
        // the Philox round keys are rebuilt per row by s_add (hoisted, the 20 of them were spilled to VGPR lanes
        // and read back per row)
        uint32_t rk0 = k0, rk1 = k1;
        asm volatile("" : "+s"(rk0), "+s"(rk1));
        u32x4 X = u32x4{0u, 0u, 0u, 0u};
        if (wave_draws) X = philox_cell(lin0 >> 2, rk0, rk1, pkc);
        const uint32_t xw[4] = {X.x, X.y, X.z, X.w};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            // thr = fl(1 - qn) * 2^24 = fl(2^24 - qn * 2^24) (power-of-two scaling commutes with the rounding)
            const gca_f2 thr = __builtin_elementwise_fma(qn[h], (gca_f2){-16777216.0f, -16777216.0f},
                                                         (gca_f2){16777216.0f, 16777216.0f});
            const float u0 = (float)(xw[2 * h] >> 8), u1 = (float)(xw[2 * h + 1] >> 8);
            burn |= (u0 < thr.x ? 1u : 0u) << (2 * h);
            burn |= (u1 < thr.y ? 1u : 0u) << (2 * h + 1);
            if constexpr (GROW) {
                grow |= (u0 < pt24 ? 1u : 0u) << (2 * h);
                grow |= (u1 < pt24 ? 1u : 0u) << (2 * h + 1);
            }
        }
        burn &= treeB;
        grow &= emptyB;
        {
            const uint32_t spare = __builtin_amdgcn_perm(__builtin_amdgcn_perm(X.w, X.z, 0x0c0c0400u),
                                                         __builtin_amdgcn_perm(X.y, X.x, 0x0c0c0400u), 0x05040100u);
            const uint32_t n0 = (uint32_t)randint_ms(spare, p.age_lo, p.age_hi);
            NA[0] = NA[1] = __builtin_amdgcn_perm(n0, n0, 0x05040100u);
            // a lane with two or more new fires (dense state: ~5 % of the wave-rows): the 2nd..4th in column order
            // take words 0..2 of the group's second block (tag ALXA)
            if (__ballot((burn & (burn - 1u)) != 0u) != 0ull) {
                const u32x4 Y = philox_cell(lin0 >> 2, rk0, rk1, pkc_age);
                const uint32_t nk[4] = {n0, (uint32_t)randint_ms(Y.x, p.age_lo, p.age_hi),
                                        (uint32_t)randint_ms(Y.y, p.age_lo, p.age_hi),
                                        (uint32_t)randint_ms(Y.z, p.age_lo, p.age_hi)};
                uint32_t a[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t rank = (uint32_t)__builtin_popcount(burn & ((1u << j) - 1u));
                    a[j] = rank == 0 ? nk[0] : (rank == 1 ? nk[1] : (rank == 2 ? nk[2] : nk[3]));
                }
                NA[0] = __builtin_amdgcn_perm(a[1], a[0], 0x05040100u);
                NA[1] = __builtin_amdgcn_perm(a[3], a[2], 0x05040100u);
            }
        }

        // ---- the rule on 4-bit masks: TREE -> FIRE (burn), EMPTY -> TREE (grow), FIRE -> EMPTY (age <= 1;
        //      classic: age == 1); age <= 1 <=> sat(age - 2) < 0 (saturating i16 pairs, exact for every int16)
        const uint32_t agw[2] = {agep.x, agep.y};
        uint32_t le1;
        if (!p.burnout_eq1) {
            const uint32_t y0 = bitcast_u32(__builtin_elementwise_sub_sat(bitcast_i16x2(agw[0]), (i16x2){2, 2}));
            const uint32_t y1 = bitcast_u32(__builtin_elementwise_sub_sat(bitcast_i16x2(agw[1]), (i16x2){2, 2}));
            le1 = ((y0 >> 15) & 1u) | ((y0 >> 30) & 2u) | ((y1 >> 13) & 4u) | ((y1 >> 28) & 8u);
        } else {
            le1 = 0u;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                le1 |= ((int32_t)(int16_t)(agw[j >> 1] >> (16 * (j & 1))) == 1) ? (1u << j) : 0u;
        }
        const uint32_t newF = burn | (fireB & ~le1);
        const uint32_t newT = (treeB & ~burn) | grow;
        const uint32_t newE = (emptyB & ~grow) | (fireB & le1);
        const uint32_t keepB = ~(treeB | emptyB | fireB) & 0xFu;  // codes outside {empty, tree, fire}: unchanged
        uint32_t sel = gca_spread4(newT) + 2u * gca_spread4(newF);
        sel |= (gca_spread4(keepB) * 0xFFu) & 0x07060504u;
        const uint32_t outw = __builtin_amdgcn_perm(own, codes, sel);
        // ages: FIRE cells age - 1 (also when they burn out), new fires the drawn age, others unchanged
        uint32_t nag[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t fh = ((fireB >> (2 * h)) & 1u) | (((fireB >> (2 * h + 1)) & 1u) << 16);
            const uint32_t a1 = bitcast_u32(bitcast_u16x2(agw[h]) - bitcast_u16x2(fh));
            const uint32_t bm = (((burn >> (2 * h)) & 1u) * 0xFFFFu) | (((burn >> (2 * h + 1)) & 1u) * 0xFFFF0000u);
            nag[h] = gca_bfi32(bm, NA[h], a1);
        }
        const size_t o = (size_t)r * W + lc;
        // the new grid and ages are read back only by the next step: non-temporal stores
        __builtin_nontemporal_store(outw, reinterpret_cast<uint32_t*>(gO + o));
        { typedef uint32_t u2v __attribute__((ext_vector_type(2)));
          __builtin_nontemporal_store((u2v){nag[0], nag[1]}, reinterpret_cast<u2v*>(aO + o)); }
        write_rgb_row(r, newT, newF, dring[3]);
        if constexpr (OBS && !HALO) {
            if (obs.refit && r < 2) {  // tile 0's rows 0 and 1 (wave-uniform)
                if (r == 0) {
                    out_row0 = outw;
                } else {
                    const uint8_t rf = row0_refit(out_row0, outw);
                    if (lane == 0) obs.refit[e] = rf;
                }
            }
        }
        cntT += __builtin_popcount(newT);
        cntF += __builtin_popcount(newF);
        cntE += __builtin_popcount(newE);

#pragma unroll
        for (int t = 0; t < 5; ++t) dring[t] = dring[t + 1];
    };
#pragma unroll 1
    for (int i = 0; i < SH; i += 2) {
        row(i, sc, sn, std::integral_constant<int, 0>{});
        row(i + 1, sn, sc, std::integral_constant<int, 1>{});
    }

    if (counts || act_out) {
        const bool anyF = __ballot(cntF != 0) != 0ull;
        if (act_out && lane == 0) act_out[((size_t)e * strips + s) * NSEG + g] = anyF ? 1 : 0;
        if (counts) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                cntT += __shfl_xor(cntT, off);
                cntF += __shfl_xor(cntF, off);
                cntE += __shfl_xor(cntE, off);
            }
            if (lane == 0) {
                if (cntE) atomicAdd(counts + 3 * e + 0, cntE);
                if (cntT) atomicAdd(counts + 3 * e + 1, cntT);
                if (cntF) atomicAdd(counts + 3 * e + 2, cntF);
            }
        }
    }
}

template <int R, bool OBS, bool GROW, int NSEG, int FLATM>
void launch_march_n(const gca_alex_params& p, int E, int H, const uint8_t* gi, uint8_t* go, const int16_t* ai,
                    int16_t* ao, const uint8_t* vd, const uint16_t* db, const float* es, const int32_t* wi,
                    const uint32_t* rs, int32_t* counts, const uint8_t* act_in, uint8_t* act_out, MarchObs obs,
                    hipStream_t st) {
    const int nwaves = E * (H / SH) * NSEG;
    if constexpr (NSEG == 1)  // four independent tiles per workgroup
        hipLaunchKernelGGL((alex_march_kernel<R, OBS, GROW, 1, FLATM>), dim3((unsigned)((nwaves + 3) / 4)), dim3(256), 0, st, p,
                           H, nwaves, gi, go, ai, ao, vd, db, es, wi, rs, counts, act_in, act_out, obs);
    else  // one strip (NSEG segment waves) per workgroup
        hipLaunchKernelGGL((alex_march_kernel<R, OBS, GROW, NSEG, FLATM>), dim3((unsigned)(nwaves / NSEG)), dim3(64 * NSEG), 0,
                           st, p, H, nwaves, gi, go, ai, ao, vd, db, es, wi, rs, counts, act_in, act_out, obs);
}
template <int R, bool OBS, bool GROW, int FLATM>
void launch_march_g(const gca_alex_params& p, int E, int H, int W, const uint8_t* gi, uint8_t* go, const int16_t* ai,
                    int16_t* ao, const uint8_t* vd, const uint16_t* db, const float* es, const int32_t* wi,
                    const uint32_t* rs, int32_t* counts, const uint8_t* act_in, uint8_t* act_out, MarchObs obs,
                    hipStream_t st) {
    if (W == MW)
        launch_march_n<R, OBS, GROW, 1, FLATM>(p, E, H, gi, go, ai, ao, vd, db, es, wi, rs, counts, act_in, act_out, obs, st);
    else if (W == 2 * MW)
        launch_march_n<R, OBS, GROW, 2, FLATM>(p, E, H, gi, go, ai, ao, vd, db, es, wi, rs, counts, act_in, act_out, obs, st);
    else
        launch_march_n<R, OBS, GROW, 4, FLATM>(p, E, H, gi, go, ai, ao, vd, db, es, wi, rs, counts, act_in, act_out, obs, st);
}
template <int R, bool OBS>
void launch_march(const gca_alex_params& p, int E, int H, int W, const uint8_t* gi, uint8_t* go, const int16_t* ai,
                  int16_t* ao, const uint8_t* vd, const uint16_t* db, const float* es, const int32_t* wi,
                  const uint32_t* rs, int32_t* counts, const uint8_t* act_in, uint8_t* act_out, MarchObs obs,
                  hipStream_t st) {
    // edge_slope NULL: flat terrain; vd NULL as well: uniform layers (march_impl checks the pairing)
    const bool grow = p.p_tree > 0.0f;
    const int fm = es ? 0 : (vd ? 1 : 2);
#define GCA_MARCH_FM(FM)                                                                                                \
    if (grow)                                                                                                         \
        launch_march_g<R, OBS, true, FM>(p, E, H, W, gi, go, ai, ao, vd, db, es, wi, rs, counts, act_in, act_out, obs, st); \
    else                                                                                                              \
        launch_march_g<R, OBS, false, FM>(p, E, H, W, gi, go, ai, ao, vd, db, es, wi, rs, counts, act_in, act_out, obs, st);
    if (fm == 0) {
        GCA_MARCH_FM(0)
    } else if (fm == 1) {
        GCA_MARCH_FM(1)
    } else {
        GCA_MARCH_FM(2)
    }
#undef GCA_MARCH_FM
}

template <bool OBS>
void dispatch_march(const gca_alex_params& p, int E, int H, int W, const uint8_t* gi, uint8_t* go, const int16_t* ai,
                    int16_t* ao, const uint8_t* vd, const uint16_t* db, const float* es, const int32_t* wi,
                    const uint32_t* rs, int32_t* counts, const uint8_t* act_in, uint8_t* act_out, MarchObs obs,
                    hipStream_t st) {
#define GCA_MARCH_CASE(RV) \
    case RV: launch_march<RV, OBS>(p, E, H, W, gi, go, ai, ao, vd, db, es, wi, rs, counts, act_in, act_out, obs, st); break;
    switch (p.R) {
#ifdef GCA_MARCH_ANALYSIS_R6  // ISA analysis builds (scripts/isa_rows.py): the R = 6 instances only
        GCA_MARCH_CASE(6)
#else
        GCA_MARCH_CASE(1) GCA_MARCH_CASE(2) GCA_MARCH_CASE(3) GCA_MARCH_CASE(4)
        GCA_MARCH_CASE(5) GCA_MARCH_CASE(6) GCA_MARCH_CASE(7) GCA_MARCH_CASE(8)
#endif
    }
#undef GCA_MARCH_CASE
}

int march_impl(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
               const int16_t* age_in, int16_t* age_out, const uint8_t* vd, const uint16_t* dous_bits,
               const float* edge_slope, const int32_t* wind_index, const uint32_t* rng_step, int32_t* counts,
               const uint8_t* act_in, uint8_t* act_out, MarchObs obs, void* stream) {
    GCA_CHECK_ARG(p && grid_in && grid_out && age_in && age_out && dous_bits && wind_index,
                  "alex_step_march: null argument");  // edge_slope NULL: flat terrain (every slope factor 1)
    GCA_CHECK_ARG(vd || (!edge_slope && p->vd_uniform >= 0 && p->vd_uniform <= 255 && (p->vd_uniform & 0x88) == 0),
                  "alex_step_march: vd = NULL (uniform layers) needs edge_slope = NULL and p->vd_uniform = "
                  "vegetation | density << 4 with both in 0..7");
    GCA_CHECK_ARG(E > 0 && H > 0 && (W == MW || W == 2 * MW || W == 4 * MW) && H % SH == 0,
                  "alex_step_march: W must be 256, 512 or 1024 and H a multiple of 16");
    GCA_CHECK_ARG(p->R >= 1 && p->R <= GCA_MAX_RADIUS, "alex_step_march: burn radius must be in [1, 8]");
    GCA_CHECK_ARG(p->n_winds >= 1 && p->n_winds <= 16, "alex_step_march: 1..16 wind matrices");
    GCA_CHECK_ARG((int64_t)E * (H / SH) * (W / MW) < (int64_t)1 << 31, "alex_step_march: too many tiles");
    GCA_CHECK_ARG(!act_in || W == MW, "alex_step_march: the tile activity map (act_in) is read at W = 256 only (wider "
                                      "grids find quiet strips from the grid itself; act_out is still written)");
    GCA_CHECK_ARG(grid_in != grid_out, "alex_step_march: the grid cannot be updated in place");
    GCA_CHECK_ARG(((((uintptr_t)grid_in) | ((uintptr_t)grid_out) | ((uintptr_t)age_in) | ((uintptr_t)age_out) |
                    ((uintptr_t)vd) | ((uintptr_t)edge_slope) | ((uintptr_t)obs.rgb) | ((uintptr_t)obs.col)) & 15u) == 0 &&
                      ((uintptr_t)dous_bits & 1u) == 0,
                  "alex_step_march: arrays must be 16-B aligned");
    GCA_CHECK_ARG(!obs.action || (obs.rgb && obs.refit && W == MW && obs.action_stride >= 3 && obs.n_choices >= 1 &&
                                  p->empty == 0 && p->tree == 1 && p->fire == 2),
                  "alex_step_march_rgb_ext: needs rgb, refit, W = 256, full actions (stride >= 3) and the codes 0 / 1 / 2");
    GCA_CHECK_ARG(!act_in || act_out, "alex_step_march: act_in needs act_out");
    GCA_CHECK_ARG(act_in != act_out || !act_in, "alex_step_march: act_in and act_out must differ");
    hipStream_t st = (hipStream_t)stream;
    if (counts && hipMemsetAsync(counts, 0, sizeof(int32_t) * 3 * (size_t)E, st) != hipSuccess) {
        gca_set_error("alex_step_march: counts memset failed");
        return GCA_ERR_HIP;
    }
    const uint8_t* ain = (p->p_tree > 0.0f) ? nullptr : act_in;  // growth can change a fire-free tile
    if (obs.rgb)
        dispatch_march<true>(*p, E, H, W, grid_in, grid_out, age_in, age_out, vd, dous_bits, edge_slope, wind_index,
                             rng_step, counts, ain, act_out, obs, st);
    else
        dispatch_march<false>(*p, E, H, W, grid_in, grid_out, age_in, age_out, vd, dous_bits, edge_slope, wind_index,
                              rng_step, counts, ain, act_out, obs, st);
    GCA_CHECK_LAUNCH(obs.rgb ? "alex_step_march_rgb" : "alex_step_march");
    return GCA_OK;
}

// OBS_* bits of every extension choice (see MarchObs): the display of advanced_bulldozer.py:1035-1101 under the
// speculation that row 0 of an enabled channel is positive (then channel 0 is shown everywhere, gca_obs.hip's scan
// stops at row 0); what needs the blurred grid, or a single channel, is left to gca_adv_observation (OBS_NONE)
uint32_t obs_mode_bits(const gca_obs_params& op, int& n_choices) {
    const bool ext = op.enable_extensions && op.n_choices > 0;
    n_choices = ext ? (op.n_choices < 8 ? op.n_choices : 8) : 1;
    uint32_t bits = 0u;
    for (int c = 0; c < n_choices; ++c) {
        uint32_t on = 0u;
        if (ext)
            for (int i = 0; i < op.n_ext && i < GCA_OBS_MAX_EXT; ++i) on |= (op.ext_lookup[c][i] != 0 ? 1u : 0u) << i;
        uint32_t m;
        if (!on) {
            m = op.should_transform ? OBS_NONE : OBS_GRID;  // the base channel: blurred, or the grid
        } else if (op.n_ext < 2) {
            m = OBS_NONE;  // one channel: shown whenever any row is positive (not a row-0 question)
        } else {
            uint32_t chk = 0u;
            for (int i = 0; i < op.n_ext && i < GCA_OBS_MAX_EXT; ++i)
                if ((on >> i) & 1u) chk |= op.ext_skip_blur[i] ? OBS_CHK_GRID : OBS_CHK_BLUR;
            m = (on & 1u) ? (op.ext_skip_blur[0] ? OBS_GRID : OBS_NONE) : OBS_ZERO;
            if (m != OBS_NONE) m |= chk;
        }
        bits |= m << (4 * c);
    }
    return bits;
}

}  // namespace

extern "C" int gca_alex_step_march(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in,
                                   uint8_t* grid_out, const int16_t* age_in, int16_t* age_out, const uint8_t* vd,
                                   const uint16_t* dous_bits, const float* edge_slope, const int32_t* wind_index,
                                   const uint32_t* rng_step, int32_t* counts, const uint8_t* act_in, uint8_t* act_out,
                                   void* stream) {
    return march_impl(p, E, H, W, grid_in, grid_out, age_in, age_out, vd, dous_bits, edge_slope, wind_index, rng_step,
                      counts, act_in, act_out, MarchObs{nullptr, nullptr, nullptr, nullptr, 0, 1, 0u, nullptr}, stream);
}

extern "C" int gca_alex_step_march_rgb(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in,
                                       uint8_t* grid_out, const int16_t* age_in, int16_t* age_out, const uint8_t* vd,
                                       const uint16_t* dous_bits, const float* edge_slope, const int32_t* wind_index,
                                       const uint32_t* rng_step, int32_t* counts, const uint8_t* act_in,
                                       uint8_t* act_out, const float* color_table, const int32_t* is_night, float* rgb,
                                       void* stream) {
    GCA_CHECK_ARG(color_table && is_night && rgb, "alex_step_march_rgb: color_table, is_night and rgb required");
    return march_impl(p, E, H, W, grid_in, grid_out, age_in, age_out, vd, dous_bits, edge_slope, wind_index, rng_step,
                      counts, act_in, act_out,
                      MarchObs{reinterpret_cast<const float4*>(color_table), is_night, rgb, nullptr, 0, 1, 0u, nullptr},
                      stream);
}

extern "C" int gca_alex_step_march_rgb_ext(const gca_alex_params* p, const gca_obs_params* op, int E, int H, int W,
                                           const uint8_t* grid_in, uint8_t* grid_out, const int16_t* age_in,
                                           int16_t* age_out, const uint8_t* vd, const uint16_t* dous_bits,
                                           const float* edge_slope, const int32_t* wind_index, const uint32_t* rng_step,
                                           int32_t* counts, const uint8_t* act_in, uint8_t* act_out,
                                           const float* color_table, const int32_t* is_night, float* rgb,
                                           const int32_t* action, int action_stride, uint8_t* refit, void* stream) {
    GCA_CHECK_ARG(op && color_table && is_night && rgb && action && refit,
                  "alex_step_march_rgb_ext: obs params, color_table, is_night, rgb, action and refit required");
    int n_choices = 1;
    const uint32_t bits = obs_mode_bits(*op, n_choices);
    return march_impl(p, E, H, W, grid_in, grid_out, age_in, age_out, vd, dous_bits, edge_slope, wind_index, rng_step,
                      counts, act_in, act_out,
                      MarchObs{reinterpret_cast<const float4*>(color_table), is_night, rgb, action, action_stride,
                               n_choices, bits, refit},
                      stream);
}
