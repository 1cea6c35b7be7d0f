// gca_windy.hip — WindyForestFire CA step on gfx950 (reference: ca_windy.py:41-139).
//
// Reference semantics (scipy.signal.convolve2d, mode="same", boundary fill = empty):
//   S[r,c] = 2048*x[r,c] + sum_{(a,b)!=(1,1)} K[a,b] * x[r-(a-1), c-(b-1)]
//   K[a,b] = 8 if direction (a,b) is active this step (roll < wind), else `empty`.
//   new = EMPTY (S<2048T) | TREE (S<2048T+8F) | FIRE (S<2048F) | EMPTY.
// Direction bit d of dir_mask indexes (a,b) row-major with the centre skipped.
//
// Two kernels:
//  * windy_exact_kernel : the formula above, literally, one thread per cell. Any H, W,
//    any u8 cell codes (covers empty != 0, where failed directions still weigh `empty`).
//  * windy_fast_kernel  : empty == 0 and W = 16*LPR (LPR | 64). Then, for grids whose
//    cells are in {0,T,F} (checked at the boundary) and the constructor's asserted
//    ordering (ca_windy.py:141-173), the thresholds reduce EXACTLY to
//      TREE -> FIRE iff some active direction sees FIRE;  FIRE -> EMPTY;  else unchanged.
//    Each lane owns 16 consecutive cells (one 16-B load/store per row), a wave covers
//    RPW = 64/LPR rows per step and marches down a strip of SH rows. Fire flags are
//    SWAR bytes; vertical neighbours come from the adjacent lane group (ds_bpermute),
//    horizontal ones from byte funnel shifts plus the neighbour lane's edge dword.
//    Reward/done counts of the new grid are fused (wave reduction + 3 atomics).
#include "gca_common.h"

// windy_fast_kernel: row chunks in flight ahead of the one being computed (r01o: 2 / 4 / 8 measured slower than 1)
constexpr int WINDY_AHEAD = 1;

// ------------------------------------------------------------------ dir mask
__global__ void windy_dirmask_kernel(const double* __restrict__ wind, int64_t wind_stride,
                                     const double* __restrict__ roll, uint32_t k0, uint32_t k1,
                                     const uint32_t* __restrict__ rng_step, const int32_t* __restrict__ steps,
                                     int pass, int env_offset, uint8_t* __restrict__ dir_mask, int E) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    if (steps && steps[e] <= pass) return;
    const uint32_t step = (rng_step ? rng_step[e] : 0u) + (uint32_t)pass;
    dir_mask[e] = (uint8_t)windy_mask(wind + (int64_t)e * wind_stride, roll ? roll + (int64_t)e * 9 : nullptr, k0, k1,
                                      (uint32_t)(env_offset + e), step);
}

// ------------------------------------------------------------------ exact kernel
__global__ __launch_bounds__(256) void windy_exact_kernel(uint8_t* __restrict__ buf0, uint8_t* __restrict__ buf1,
                                                          const uint8_t* __restrict__ parity,
                                                          const int32_t* __restrict__ steps, int pass,
                                                          const uint8_t* __restrict__ dir_mask, int E, int H, int W,
                                                          int empty, int tree, int fire, int32_t* __restrict__ counts) {
    const int64_t HW = (int64_t)H * W;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in_range = idx < (int64_t)E * HW;
    const int e = in_range ? (int)(idx / HW) : E - 1;
    const bool active = in_range && (!steps || steps[e] > pass);
    int out_code = -1;
    if (active) {
        const int64_t cell = idx - (int64_t)e * HW;
        const int r = (int)(cell / W), c = (int)(cell - (int64_t)r * W);
        const bool odd = parity && parity[e];
        const uint8_t* src = (odd ? buf1 : buf0) + (int64_t)e * HW;
        uint8_t* dst = (odd ? buf0 : buf1) + (int64_t)e * HW;
        const uint32_t m = dir_mask[e];
        int32_t S = 2048 * (int32_t)src[cell];
        int d = 0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                if (a == 1 && b == 1) continue;
                const int sr = r - (a - 1), sc = c - (b - 1);
                const int32_t nb = (sr >= 0 && sr < H && sc >= 0 && sc < W) ? (int32_t)src[(int64_t)sr * W + sc] : empty;
                const int32_t k = ((m >> d) & 1u) ? 8 : empty;
                S += k * nb;
                ++d;
            }
        }
        const int32_t keep = 2048 * tree, prop = 2048 * tree + 8 * fire, cons = 2048 * fire;
        int v = empty;
        if (S >= keep && S < prop) v = tree;
        if (S >= prop && S < cons) v = fire;
        if (S >= cons) v = empty;
        dst[cell] = (uint8_t)v;
        out_code = v;
    }
    if (counts) {
        // waves whose lanes all belong to one env reduce first; mixed waves fall back to per-lane atomics
        const int e0 = __shfl(e, 0), e63 = __shfl(e, 63);
        const bool uniform = (e0 == e63) && __all(active || !in_range);
        if (uniform) {
            const int nE = __popcll(__ballot(out_code == empty));
            const int nT = __popcll(__ballot(out_code == tree && tree != empty));
            const int nF = __popcll(__ballot(out_code == fire));
            if ((threadIdx.x & 63) == 0 && __any(active)) {
                atomicAdd(counts + 3 * e0 + 0, nE);
                atomicAdd(counts + 3 * e0 + 1, nT);
                atomicAdd(counts + 3 * e0 + 2, nF);
            }
        } else if (active) {
            if (out_code == empty) atomicAdd(counts + 3 * e + 0, 1);
            else if (out_code == tree) atomicAdd(counts + 3 * e + 1, 1);
            else if (out_code == fire) atomicAdd(counts + 3 * e + 2, 1);
        }
    }
}

// ------------------------------------------------------------------ fast kernel
struct Row16 {
    uint32_t f[4];  // 0x01 per byte where cell == FIRE
    uint32_t t[4];  // 0x01 per byte where cell == TREE
};

__device__ __forceinline__ Row16 classify(uint4 v, uint32_t Tp, uint32_t Fp, bool valid) {
    Row16 o;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        o.f[j] = valid ? bytes_eq01(w[j], Fp) : 0u;
        o.t[j] = valid ? bytes_eq01(w[j], Tp) : 0u;
    }
    return o;
}

__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

template <int LPR>
__global__ __launch_bounds__(256) void windy_fast_kernel(uint8_t* __restrict__ buf0, uint8_t* __restrict__ buf1,
                                                         const uint8_t* __restrict__ parity,
                                                         const int32_t* __restrict__ steps, int pass,
                                                         const uint8_t* __restrict__ dir_mask, int H, int SH,
                                                         int blocks_per_env, uint32_t Ep, uint32_t Tp, uint32_t Fp,
                                                         int32_t* __restrict__ counts) {
    constexpr int W = 16 * LPR;
    constexpr int RPW = 64 / LPR;
    const int env = blockIdx.x / blocks_per_env;
    const int sblk = blockIdx.x - env * blocks_per_env;
    if (steps && steps[env] <= pass) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane / LPR, q = lane - g * LPR;
    const int s0 = (sblk * 4 + wave) * SH;
    if (s0 >= H) return;
    const int s_end = min(s0 + SH, H);
    const int nT = (s_end - s0 + RPW - 1) / RPW;

    const bool odd = parity && parity[env];
    const int64_t HW = (int64_t)H * W;
    const uint8_t* __restrict__ S = (odd ? buf1 : buf0) + (int64_t)env * HW + 16 * q;
    uint8_t* __restrict__ D = (odd ? buf0 : buf1) + (int64_t)env * HW + 16 * q;

    const uint32_t m = dir_mask[env];
    const uint32_t m0 = (m & 1u) ? ~0u : 0u, m1 = (m & 2u) ? ~0u : 0u, m2 = (m & 4u) ? ~0u : 0u,
                   m3 = (m & 8u) ? ~0u : 0u, m4 = (m & 16u) ? ~0u : 0u, m5 = (m & 32u) ? ~0u : 0u,
                   m6 = (m & 64u) ? ~0u : 0u, m7 = (m & 128u) ? ~0u : 0u;

    auto load_row = [&](int R, bool want) -> uint4 {
        if (want && R >= 0 && R < H) return *reinterpret_cast<const uint4*>(S + (int64_t)R * W);
        return make_uint4(0u, 0u, 0u, 0u);
    };

    // chunk c of the strip = rows s0 + c*RPW + g; chunk nT only for its first row (the strip's lower halo)
    auto chunk_row = [&](int c) { return s0 + c * RPW + g; };
    auto wanted = [&](int c) { return c < nT || (c == nT && g == 0); };
    // prologue: chunk -1 (only the row just above the strip), chunk 0, and chunks 1..AHEAD in flight
    const int Rprev = s0 - RPW + g;
    Row16 prv = classify(load_row(Rprev, g == RPW - 1), Tp, Fp, g == RPW - 1 && Rprev >= 0);
    Row16 cur = classify(load_row(chunk_row(0), true), Tp, Fp, chunk_row(0) < H);
    uint4 ring[WINDY_AHEAD];  // ring[u] holds chunk t + 1 when t % AHEAD == u
#pragma unroll
    for (int u = 0; u < WINDY_AHEAD; ++u) ring[u] = load_row(chunk_row(u + 1), wanted(u + 1));

    const int lane_up = (lane - LPR) & 63, lane_dn = (lane + LPR) & 63;
    const int lane_l = (lane - 1) & 63, lane_r = (lane + 1) & 63;
    const bool has_l = q > 0, has_r = q < LPR - 1;

    int32_t cntT = 0, cntF = 0, cntV = 0;
    for (int t0 = 0; t0 < nT; t0 += WINDY_AHEAD) {
#pragma unroll
    for (int u = 0; u < WINDY_AHEAD; ++u) {
        const int t = t0 + u;
        if (t >= nT) break;  // wave-uniform
        const int Rc = chunk_row(t), Rn = chunk_row(t + 1);
        Row16 nxt = classify(ring[u], Tp, Fp, wanted(t + 1) && Rn < H);
        // refill the slot just consumed: the load AHEAD + 1 chunks ahead, issued before computing this chunk
        ring[u] = load_row(chunk_row(t + 1 + WINDY_AHEAD), wanted(t + 1 + WINDY_AHEAD));

        uint32_t up[4], dn[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            up[j] = shfl_u32(g == RPW - 1 ? prv.f[j] : cur.f[j], lane_up);
            dn[j] = shfl_u32(g == 0 ? nxt.f[j] : cur.f[j], lane_dn);
        }
        // edge dwords of the neighbouring 16-cell chunks (same row) for +-1 column shifts
        // (bpermutes run in every lane: a lane switched off in EXEC would not serve its value)
        const uint32_t s_upL = shfl_u32(up[3], lane_l), s_upR = shfl_u32(up[0], lane_r);
        const uint32_t s_cuL = shfl_u32(cur.f[3], lane_l), s_cuR = shfl_u32(cur.f[0], lane_r);
        const uint32_t s_dnL = shfl_u32(dn[3], lane_l), s_dnR = shfl_u32(dn[0], lane_r);
        const uint32_t upL = has_l ? s_upL : 0u, upR = has_r ? s_upR : 0u;
        const uint32_t cuL = has_l ? s_cuL : 0u, cuR = has_r ? s_cuR : 0u;
        const uint32_t dnL = has_l ? s_dnL : 0u, dnR = has_r ? s_dnR : 0u;

        uint32_t outw[4];
        int32_t rowT = 0, rowF = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // X_l: byte i holds X[i-1] (source column c-1); X_r: byte i holds X[i+1] (column c+1)
            const uint32_t up_l = __builtin_amdgcn_alignbyte(up[j], j ? up[j - 1] : upL, 3);
            const uint32_t up_r = __builtin_amdgcn_alignbyte(j < 3 ? up[j + 1] : upR, up[j], 1);
            const uint32_t cu_l = __builtin_amdgcn_alignbyte(cur.f[j], j ? cur.f[j - 1] : cuL, 3);
            const uint32_t cu_r = __builtin_amdgcn_alignbyte(j < 3 ? cur.f[j + 1] : cuR, cur.f[j], 1);
            const uint32_t dn_l = __builtin_amdgcn_alignbyte(dn[j], j ? dn[j - 1] : dnL, 3);
            const uint32_t dn_r = __builtin_amdgcn_alignbyte(j < 3 ? dn[j + 1] : dnR, dn[j], 1);
            // d -> source (r+1-a, c+1-b): d0 down/c+1, d1 down, d2 down/c-1, d3 cur/c+1,
            //                             d4 cur/c-1, d5 up/c+1, d6 up, d7 up/c-1
            const uint32_t any = (dn_r & m0) | (dn[j] & m1) | (dn_l & m2) | (cu_r & m3) | (cu_l & m4) |
                                 (up_r & m5) | (up[j] & m6) | (up_l & m7);
            const uint32_t ign = cur.t[j] & any;          // TREE -> FIRE
            const uint32_t keep = cur.t[j] & ~any;        // TREE stays
            const uint32_t ignm = (ign << 8) - ign;       // 0x01 -> 0xFF per byte
            const uint32_t keepm = (keep << 8) - keep;
            outw[j] = (ignm & Fp) | (keepm & Tp) | (~(ignm | keepm) & Ep);
            rowF += __popc(ign);
            rowT += __popc(keep);
        }
        if (Rc < s_end) {  // rows of the last partial chunk past the strip are neither stored nor counted
            *reinterpret_cast<uint4*>(D + (int64_t)Rc * W) = make_uint4(outw[0], outw[1], outw[2], outw[3]);
            cntV += 16;
            cntT += rowT;
            cntF += rowF;
        }
        prv = cur;
        cur = nxt;
    }
    }
    if (counts) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            cntT += __shfl_xor(cntT, off);
            cntF += __shfl_xor(cntF, off);
            cntV += __shfl_xor(cntV, off);
        }
        if (lane == 0) {
            atomicAdd(counts + 3 * env + 0, cntV - cntT - cntF);
            atomicAdd(counts + 3 * env + 1, cntT);
            atomicAdd(counts + 3 * env + 2, cntF);
        }
    }
}

// ------------------------------------------------------------------ row-stream kernel (W = 256 NW, NW = 1, 2)
// The fast kernel's rule with a different lane map: a wave holds WHOLE image rows, lane l owning columns
// [4 NW l, 4 NW l + 4 NW) (one dword per row at W = 256), and marches down a strip of SH rows. The vertical
// neighbours are then the lane's own previous / next row (registers: no cross-lane traffic at all) and the horizontal
// ones the neighbour lanes' edge dwords, moved by DPP whole-wave shifts (wave_shr:1 / wave_shl:1, lanes 0 / 63 read 0 =
// the grid's left / right border) instead of ds_bpermute. Each row's fire flags and their two column shifts are built
// once and used by the three output rows that see them. Loads run WINDY_RD rows ahead (one dword per lane each, so
// many rows fit in flight); row indices are clamped, not branched, so hipcc keeps the counted waits.
constexpr int WINDY_RSH = 16;  // strip height per wave (r02j: 16 / 32 / 64 rows -> config 5 CA 105.9 / 109.7 / 110.5 us)
constexpr int WINDY_RD = 8;    // rows in flight ahead of the row being classified

template <int NW>
struct RowRaw {
    uint32_t w[NW];
};
template <int NW>
struct RowCls {
    uint32_t f[NW], fl[NW], fr[NW];  // FIRE flags (0x01 per byte); byte i = flag of column c-1 (fl), c+1 (fr)
    uint32_t t[NW];                  // TREE flags
};

__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {  // lane l <- lane l-1, lane 0 <- 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v) {  // lane l <- lane l+1, lane 63 <- 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);
}

// S: the env's wave-uniform base (SGPRs), lofs: the lane's 32-bit column offset, R wave-uniform: the clamp and the row
// offset stay scalar and the load is one global_load with an SGPR base and a 32-bit VGPR offset (no 64-bit address
// VGPRs, no per-lane row arithmetic)
template <int NW>
__device__ __forceinline__ RowRaw<NW> load_rowraw(const uint8_t* __restrict__ S, uint32_t lofs, int R, int H) {
    constexpr int W = 256 * NW;
    const int Rc = min(max(R, 0), H - 1);  // clamped: the value of an out-of-grid row is discarded by classify
    const uint8_t* p = S + (uint32_t)Rc * (uint32_t)W + lofs;
    RowRaw<NW> x;
    if (NW == 1) {
        x.w[0] = *reinterpret_cast<const uint32_t*>(p);
    } else if (NW == 2) {
        const uint2 v = *reinterpret_cast<const uint2*>(p);
        x.w[0] = v.x; x.w[1 % NW] = v.y;
    } else {
        const uint4 v = *reinterpret_cast<const uint4*>(p);
        x.w[0] = v.x; x.w[1 % NW] = v.y; x.w[2 % NW] = v.z; x.w[3 % NW] = v.w;
    }
    return x;
}

// STD: the bulldozer's codes EMPTY 0, TREE 3 (0b00011), FIRE 25 (0b11001): on these three byte values FIRE is bit 4
// and TREE is bit 0 without bit 4, so both flags cost 3 VALU (shift, and, one bitop3) instead of two byte compares
// (~9); the fast rule's contract already restricts the cells to the three codes
template <int NW, bool STD>
__device__ __forceinline__ RowCls<NW> classify_row(const RowRaw<NW>& x, bool valid, uint32_t Tp, uint32_t Fp) {
    RowCls<NW> o;
#pragma unroll
    for (int j = 0; j < NW; ++j) {
        if constexpr (STD) {
            const uint32_t h = x.w[j] >> 4;
            o.f[j] = valid ? (h & 0x01010101u) : 0u;
            o.t[j] = valid ? __builtin_amdgcn_bitop3_b32(x.w[j], h, 0x01010101u, 0x20) : 0u;  // a & ~b & c
        } else {
            o.f[j] = valid ? bytes_eq01(x.w[j], Fp) : 0u;
            o.t[j] = valid ? bytes_eq01(x.w[j], Tp) : 0u;
        }
    }
    const uint32_t prev = wave_shr1(o.f[NW - 1]), next = wave_shl1(o.f[0]);
#pragma unroll
    for (int j = 0; j < NW; ++j) {
        o.fl[j] = __builtin_amdgcn_alignbyte(o.f[j], j ? o.f[j - 1] : prev, 3);
        o.fr[j] = __builtin_amdgcn_alignbyte(j < NW - 1 ? o.f[j + 1] : next, o.f[j], 1);
    }
    return o;
}

// One wave's strip of SH rows [s0, s0 + SH) of one env: S the input grid, Dst the output, m the env's direction mask;
// the strip's new-grid counts are added to (cntT, cntF, cntV = cells written). Shared by windy_rows_kernel (one
// launch per CA pass) and bulldozer_step_fused_kernel (the whole env step), so both write the same bytes. RD: rows of
// loads in flight ahead of the row being classified (RD = SH: the whole strip at once), SH: the strip's height.
template <int NW, int SH, int RD, bool STD, class MaskFn>
__device__ __forceinline__ void windy_rows_strip_f(const uint8_t* __restrict__ S, uint8_t* __restrict__ Dst, int s0,
                                                   int H, MaskFn get_mask, uint32_t lofs, uint32_t Ep, uint32_t Tp,
                                                   uint32_t Fp, int32_t& cntT, int32_t& cntF, int32_t& cntV) {
    constexpr int W = 256 * NW;
    static_assert(RD >= 1 && RD <= SH, "rows in flight: 1 .. SH");
    // the strip's first rows are requested before the direction mask is known (its draw overlaps their latency)
    RowRaw<NW> ring[RD];
    const RowRaw<NW> r_up = load_rowraw<NW>(S, lofs, s0 - 1, H), r_cur = load_rowraw<NW>(S, lofs, s0, H);
#pragma unroll
    for (int k = 0; k < RD; ++k) ring[k] = load_rowraw<NW>(S, lofs, s0 + 1 + k, H);
    const uint32_t m = get_mask();
    // all-ones / zero per direction, made opaque (readfirstlane) so that hipcc keeps `(x & m) | acc` as one
    // v_and_or_b32 per direction instead of turning each mask into a v_cndmask plus a separate or
    auto dm = [&](uint32_t bit) {
        uint32_t v = (m & bit) ? ~0u : 0u;
        asm volatile("" : "+s"(v));  // opaque SGPR value
        return v;
    };
    const uint32_t m0 = dm(1u), m1 = dm(2u), m2 = dm(4u), m3 = dm(8u), m4 = dm(16u), m5 = dm(32u), m6 = dm(64u),
                   m7 = dm(128u);

    const uint32_t codes = (Ep & 0xFFu) | ((Tp & 0xFFu) << 8) | ((Fp & 0xFFu) << 16);
    // ring[k % RD] holds row s0 + 1 + k (k = 0 .. SH): the strip's rows below row s0 up to its lower halo row
    RowCls<NW> A = classify_row<NW, STD>(r_up, s0 >= 1, Tp, Fp);
    RowCls<NW> B = classify_row<NW, STD>(r_cur, true, Tp, Fp);

#pragma unroll
    for (int t = 0; t < SH; ++t) {
        const int Rc = s0 + t;
        // row Rc + 1: loaded RD rows ago; its slot is refilled with row Rc + 1 + RD right away
        const RowCls<NW> C = classify_row<NW, STD>(ring[t % RD], Rc + 1 < H, Tp, Fp);
        if (t + RD < SH) ring[t % RD] = load_rowraw<NW>(S, lofs, Rc + 1 + RD, H);
        uint32_t outw[NW];
        int32_t rowT = 0, rowF = 0;
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            // d -> source (r+1-a, c+1-b): d0 down/c+1, d1 down, d2 down/c-1, d3 cur/c+1, d4 cur/c-1, d5 up/c+1,
            // d6 up, d7 up/c-1 (as windy_fast_kernel)
            // any = OR_d (flags_d & m_d): one v_bitop3 (a & b) | c (table 0xEA) per direction
            uint32_t any = C.fr[j] & m0;
            any = __builtin_amdgcn_bitop3_b32(C.f[j], m1, any, 0xEA);
            any = __builtin_amdgcn_bitop3_b32(C.fl[j], m2, any, 0xEA);
            any = __builtin_amdgcn_bitop3_b32(B.fr[j], m3, any, 0xEA);
            any = __builtin_amdgcn_bitop3_b32(B.fl[j], m4, any, 0xEA);
            any = __builtin_amdgcn_bitop3_b32(A.fr[j], m5, any, 0xEA);
            any = __builtin_amdgcn_bitop3_b32(A.f[j], m6, any, 0xEA);
            any = __builtin_amdgcn_bitop3_b32(A.fl[j], m7, any, 0xEA);
            const uint32_t ign = B.t[j] & any;  // TREE -> FIRE
            const uint32_t keep = B.t[j] ^ ign;  // TREE stays
            // output byte = code[2 ign + keep] (0 EMPTY, 1 TREE, 2 FIRE): one v_perm_b32 on the packed codes (hipcc
            // turned the previous (x << 8) - x byte masks into quarter-rate v_mul_lo_u32)
            outw[j] = __builtin_amdgcn_perm(codes, codes, (ign << 1) + keep);
            rowF += __popc(ign);
            rowT += __popc(keep);
        }
        if (Rc < H && t < SH) {
            uint8_t* p = Dst + (uint32_t)Rc * (uint32_t)W + lofs;
            // W >= 512: non-temporal stores (1024 x 512^2 is 256 MiB per grid, past the Infinity Cache: 105 -> 98 us
            // per CA-only step, profiles/r04p); W = 256 keeps plain stores (1024 x 256^2 in + out stays cache-resident
            // across steps; non-temporal: 24 -> 30 us)
            typedef uint32_t u2v __attribute__((ext_vector_type(2)));
            typedef uint32_t u4v __attribute__((ext_vector_type(4)));
            if (NW == 1) *reinterpret_cast<uint32_t*>(p) = outw[0];
            else if (NW == 2) __builtin_nontemporal_store((u2v){outw[0], outw[1 % NW]}, reinterpret_cast<u2v*>(p));
            else __builtin_nontemporal_store((u4v){outw[0], outw[1 % NW], outw[2 % NW], outw[3 % NW]},
                                             reinterpret_cast<u4v*>(p));
            cntV += 4 * NW;
            cntT += rowT;
            cntF += rowF;
        }
        A = B;
        B = C;
    }
}

template <int NW, int SH, int RD, bool STD>
__device__ __forceinline__ void windy_rows_strip(const uint8_t* __restrict__ S, uint8_t* __restrict__ Dst, int s0,
                                                 int H, uint32_t m, uint32_t lofs, uint32_t Ep, uint32_t Tp,
                                                 uint32_t Fp, int32_t& cntT, int32_t& cntF, int32_t& cntV) {
    windy_rows_strip_f<NW, SH, RD, STD>(S, Dst, s0, H, [m]() { return m; }, lofs, Ep, Tp, Fp, cntT, cntF, cntV);
}

template <int NW, bool STD>
__global__ __launch_bounds__(256) void windy_rows_kernel(uint8_t* __restrict__ buf0, uint8_t* __restrict__ buf1,
                                                         const uint8_t* __restrict__ parity,
                                                         const int32_t* __restrict__ steps, int pass,
                                                         const uint8_t* __restrict__ dir_mask, int H,
                                                         int blocks_per_env, uint32_t Ep, uint32_t Tp, uint32_t Fp,
                                                         int32_t* __restrict__ counts) {
    constexpr int W = 256 * NW;
    const int env = blockIdx.x / blocks_per_env;
    const int sblk = blockIdx.x - env * blocks_per_env;
    if (steps && steps[env] <= pass) return;
    // the wave index is wave-uniform: readfirstlane keeps s0 and every row index in SGPRs
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int s0 = (sblk * 4 + wave) * WINDY_RSH;
    if (s0 >= H) return;
    const bool odd = parity && parity[env];
    const int64_t HW = (int64_t)H * W;
    const uint8_t* __restrict__ S = (odd ? buf1 : buf0) + (int64_t)env * HW;
    uint8_t* __restrict__ Dst = (odd ? buf0 : buf1) + (int64_t)env * HW;
    const uint32_t lofs = 4 * NW * (uint32_t)lane;
    // the env's direction mask, forced into an SGPR (a VGPR copy made hipcc rebuild some masks per row)
    const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)dir_mask[env]);
    int32_t cntT = 0, cntF = 0, cntV = 0;
    windy_rows_strip<NW, WINDY_RSH, WINDY_RD, STD>(S, Dst, s0, H, m, lofs, Ep, Tp, Fp, cntT, cntF, cntV);
    if (counts) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            cntT += __shfl_xor(cntT, off);
            cntF += __shfl_xor(cntF, off);
            cntV += __shfl_xor(cntV, off);
        }
        if (lane == 0) {
            atomicAdd(counts + 3 * env + 0, cntV - cntT - cntF);
            atomicAdd(counts + 3 * env + 1, cntT);
            atomicAdd(counts + 3 * env + 2, cntF);
        }
    }
}

// ------------------------------------------------------------------ the whole ForestFireBulldozer env step, fused
// The env's direction mask (windy_mask bit for bit) drawn inside one wave, no barrier: lane j < 4 draws Philox block j
// (directions 2j, 2j+1) against the env's wind, two ballots gather the bits; the result is wave-uniform (an SGPR).
// Shared by both fused step kernels so their draw order cannot drift apart.
__device__ __forceinline__ uint32_t wave_windy_mask(const gca_bulldozer_params& p, const double (&wl)[9], int e,
                                                    uint32_t rs, int lane) {
    bool b0 = false, b1 = false;
    if (lane < 4) {
        const u32x4 xr = philox4x32_10(u32x4{(uint32_t)lane, (uint32_t)(p.env_offset + e), rs, GCA_TAG_WINDY_ROLL},
                                       (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
        const int d0 = 2 * lane, d1 = 2 * lane + 1;
        const int i0 = d0 < 4 ? d0 : d0 + 1, i1 = d1 < 4 ? d1 : d1 + 1;
        double w0 = wl[0], w1 = wl[0];
#pragma unroll
        for (int k = 1; k < 9; ++k) {
            w0 = k == i0 ? wl[k] : w0;
            w1 = k == i1 ? wl[k] : w1;
        }
        b0 = u01_f64(xr.x, xr.y) < w0;
        b1 = u01_f64(xr.z, xr.w) < w1;
    }
    const uint32_t g0 = (uint32_t)__ballot(b0), g1 = (uint32_t)__ballot(b1);
    uint32_t mm = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) mm |= (((g0 >> j) & 1u) << (2 * j)) | (((g1 >> j) & 1u) << (2 * j + 1));
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)mm);
}

// strips of the fused step: 32 rows with 16 in flight at W = 256 (8 waves per env: four workgroups per CU, so the
// launch's 1024 workgroups are resident at once), 16 rows with 8 in flight (the rows kernel's) at W = 512 (16 waves)
template <int NW> constexpr int FUSED_SH = NW == 1 ? 32 : 16;
template <int NW> constexpr int FUSED_RD = NW == 1 ? 16 : 8;

// The launch is latency-bound (the stepping envs are few), so the per-env inputs are all loaded up front, before any
// branch or barrier: one round trip to memory instead of a chain of dependent ones (the env's action, then its
// accu, then the wind, after the CA the position, the counts ... measured 13.6 us per 1024 x 256^2 env step with
// the loads where they are used, r03u). A launch of fewer, resident workgroups looping over the envs measured
// slower still (16.3 us, r03v: each workgroup then pays its envs' chains one after the other).
// The env's action: the caller's (action != NULL), or -- gca_bulldozer_step_fused_random, a random policy -- drawn here
// exactly as gca_random_actions draws it (Philox (0, global env id, rng_step[e], ACTI) under the policy's seed: move =
// randint[0, 9), shoot = top bit of word 1), and written to pol.out when given.
struct FusedPolicy {
    uint64_t seed;
    int32_t* out;
};
__device__ __forceinline__ void fused_action(const int32_t* __restrict__ action, const FusedPolicy& pol, int e,
                                             uint32_t env_id, uint32_t rs, int32_t& a0, int32_t& a1) {
    if (action) {
        a0 = action[2 * e];
        a1 = action[2 * e + 1];
    } else {
        const u32x4 x = philox4x32_10(u32x4{0u, env_id, rs, GCA_TAG_ACTION}, (uint32_t)pol.seed,
                                      (uint32_t)(pol.seed >> 32));
        a0 = randint_ms(x.x, 0, 9);
        a1 = (int32_t)(x.y >> 31);
    }
}

template <int NW, bool STD>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void bulldozer_step_fused_kernel(
    gca_bulldozer_params p, const int32_t* __restrict__ action, double* __restrict__ accu, int32_t* __restrict__ steps,
    uint8_t* __restrict__ done, const double* __restrict__ wind, int64_t wind_stride, uint32_t* __restrict__ rng_step,
    uint8_t* __restrict__ parity, uint8_t* __restrict__ buf0, uint8_t* __restrict__ buf1, int H,
    int32_t* __restrict__ pos, int32_t* __restrict__ counts, uint8_t* __restrict__ hit, double* __restrict__ reward,
    int64_t* __restrict__ steps_elapsed, FusedPolicy pol) {
    constexpr int W = 256 * NW;
    __shared__ int32_t wave_cnt[16][3];  // per wave (no zeroing, no atomics): summed by thread 0 after the barrier
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    // ---- every per-env input (wave-uniform addresses: scalar loads), issued together
    const bool was_done = done[e] != 0;
    const uint32_t rs = rng_step[e];
    int32_t act0, act1;
    fused_action(action, pol, e, (uint32_t)(p.env_offset + e), rs, act0, act1);
    if (pol.out && tid == 0) {
        pol.out[2 * e] = act0;
        pol.out[2 * e + 1] = act1;
    }
    const double acc = accu[e];
    const bool odd = parity[e] != 0;
    const int32_t prow = pos[2 * e], pcol = pos[2 * e + 1];
    const int32_t c0 = counts[3 * e + 0], c1 = counts[3 * e + 1], c2 = counts[3 * e + 2];
    const int64_t se = steps_elapsed ? steps_elapsed[e] : 0;
    double wl[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) wl[k] = wind[(int64_t)e * wind_stride + k];
    // ---- RepeatCA bookkeeping (repeat_ca.py:32-45, as gca_bulldozer_pre) and the Move (move_modify.py:37-67, as
    //      gca_bulldozer_post), which does not depend on the CA
    const int a0 = clampi_dev(act0, 0, 8), a1s = clampi_dev(act1, 0, 1);
    const double x = acc + ((p.t_move[a0] + p.t_shoot[a1s]) + p.t_any);
    const double reps = trunc(x);  // math.modf
    const int n = was_done ? -1 : (int)reps;
    int row = prow, col = pcol;
    move_pos(a0, row, col, H, W, p.up_mask, p.down_mask, p.left_mask, p.right_mask);
    const int64_t HW = (int64_t)H * W;
    uint8_t* grid = (odd ? buf1 : buf0) + e * HW;  // the env's grid after this step
    if (n > 0) {
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, nw = (int)(blockDim.x >> 6);
        // the direction mask (windy_mask, bit for bit) in every wave, no barrier: lane j < 4 draws Philox block j
        // (directions 2j, 2j+1), two ballots gather the bits; drawn after the strip's first row loads are issued
        auto get_mask = [&]() -> uint32_t { return wave_windy_mask(p, wl, e, rs, lane); };
        const uint8_t* __restrict__ S = grid;
        uint8_t* __restrict__ Dst = (odd ? buf0 : buf1) + e * HW;
        const uint32_t lofs = 4 * NW * (uint32_t)lane;
        int32_t cntT = 0, cntF = 0, cntV = 0;
        for (int s0 = wave * FUSED_SH<NW>; s0 < H; s0 += nw * FUSED_SH<NW>)
            windy_rows_strip_f<NW, FUSED_SH<NW>, FUSED_RD<NW>, STD>(S, Dst, s0, H, get_mask, lofs, rep4(p.empty),
                                                                   rep4(p.tree), rep4(p.fire), cntT, cntF, cntV);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            cntT += __shfl_xor(cntT, off);
            cntF += __shfl_xor(cntF, off);
            cntV += __shfl_xor(cntV, off);
        }
        if (lane == 0) {
            wave_cnt[wave][0] = cntV - cntT - cntF;
            wave_cnt[wave][1] = cntT;
            wave_cnt[wave][2] = cntF;
        }
        __syncthreads();  // the new grid (every wave's stores) and the counts are complete
        grid = Dst;
    }
    if (tid != 0) return;
    steps[e] = n;
    if (n < 0) {  // finished before this step: graceful no-op (ca_env.py:50-62)
        reward[e] = 0.0;
        return;
    }
    accu[e] = x - reps;
    int32_t cE = c0, cT = c1, cF = c2;
    if (n > 0) {
        parity[e] = odd ? 0 : 1;
        cE = cT = cF = 0;
        const int nw = (int)(blockDim.x >> 6);
        for (int w = 0; w < nw; ++w) {
            cE += wave_cnt[w][0];
            cT += wave_cnt[w][1];
            cF += wave_cnt[w][2];
        }
    }
    // MoveModify (move_modify.py:128-134): Modify at the new position, on the post-CA grid
    pos[2 * e] = row;
    pos[2 * e + 1] = col;
    uint8_t h = 0;
    // a position outside the grid (a caller's own, never produced by Move from inside) writes nothing
    if (act1 && row >= 0 && row < H && col >= 0 && col < W) {
        const int v = grid[(int64_t)row * W + col];
        const int nv = p.effect[v];
        if (nv >= 0) {
            grid[(int64_t)row * W + col] = (uint8_t)nv;
            h = 1;
            const int c_old = cell_category(v, p.empty, p.tree, p.fire), c_new = cell_category(nv, p.empty, p.tree, p.fire);
            if (c_old == 0) cE -= 1; else if (c_old == 1) cT -= 1; else if (c_old == 2) cF -= 1;
            if (c_new == 0) cE += 1; else if (c_new == 1) cT += 1; else if (c_new == 2) cF += 1;
        }
    }
    counts[3 * e + 0] = cE;
    counts[3 * e + 1] = cT;
    counts[3 * e + 2] = cF;
    hit[e] = h;
    reward[e] = (cT + cF) > 0 ? -((double)cF / (double)(cT + cF)) : (double)NAN;
    done[e] = cF == 0 ? 1 : 0;
    rng_step[e] = rs + (uint32_t)n;
    if (steps_elapsed) steps_elapsed[e] = se + 1;
}

// The fused step spread over P workgroups per env (W = 512: one CU's four SIMDs ran a stepping env's 16 waves four deep,
// ~12 us of VALU; P = 4 workgroups of 4 waves on four CUs). Every part reads the env's inputs and decides the same
// n; the CA rows are split by strips; the part holding the bulldozer's row applies Modify. The parts meet in one 64-bit
// atomic per env (E | T | F counts, 20 bits each, the hit bit, and an arrival count in the top 3 bits): the last to
// arrive writes every per-env output (only then has every part read its inputs) and clears the slot for the next step.
// `meet`: the caller's per-env slots (zero on entry; every launch leaves them zero). Measured (profiles/r04s-u, one
// restored mid-episode state, hipGraph of 8 steps with device random actions): 1024 x 512^2 18.3 -> 14.9 us per env
// step (P = 4; P = 8: 16.5), 1024 x 256^2 14.1 -> 12.7 us (P = 2). Only launched for H*W + 1 < 2^20 (the fields' width;
// gca_bulldozer_step_fused takes the one-workgroup kernel beyond).
template <int NW, bool STD, int P>
__global__ __launch_bounds__(256) void bulldozer_step_fused_parts_kernel(
    gca_bulldozer_params p, const int32_t* __restrict__ action, double* __restrict__ accu, int32_t* __restrict__ steps,
    uint8_t* __restrict__ done, const double* __restrict__ wind, int64_t wind_stride, uint32_t* __restrict__ rng_step,
    uint8_t* __restrict__ parity, uint8_t* __restrict__ buf0, uint8_t* __restrict__ buf1, int H,
    int32_t* __restrict__ pos, int32_t* __restrict__ counts, uint8_t* __restrict__ hit, double* __restrict__ reward,
    int64_t* __restrict__ steps_elapsed, unsigned long long* __restrict__ meet, FusedPolicy pol) {
    constexpr int W = 256 * NW;
    constexpr int SHv = (NW == 1 && P >= 4) ? 16 : FUSED_SH<NW>;
    constexpr int RDv = SHv < FUSED_RD<NW> ? SHv : FUSED_RD<NW>;
    __shared__ int32_t wave_cnt[4][3];
    const int e = blockIdx.x / P, part = blockIdx.x - e * P;
    const int tid = threadIdx.x;
    const bool was_done = done[e] != 0;
    const uint32_t rs = rng_step[e];
    int32_t act0, act1;
    fused_action(action, pol, e, (uint32_t)(p.env_offset + e), rs, act0, act1);
    if (pol.out && part == 0 && tid == 0) {
        pol.out[2 * e] = act0;
        pol.out[2 * e + 1] = act1;
    }
    const double acc = accu[e];
    const bool odd = parity[e] != 0;
    const int32_t prow = pos[2 * e], pcol = pos[2 * e + 1];
    const int32_t c0 = counts[3 * e + 0], c1 = counts[3 * e + 1], c2 = counts[3 * e + 2];
    const int64_t se = steps_elapsed ? steps_elapsed[e] : 0;
    double wl[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) wl[k] = wind[(int64_t)e * wind_stride + k];
    const int a0 = clampi_dev(act0, 0, 8), a1s = clampi_dev(act1, 0, 1);
    const double x = acc + ((p.t_move[a0] + p.t_shoot[a1s]) + p.t_any);
    const double reps = trunc(x);
    const int n = was_done ? -1 : (int)reps;
    int row = prow, col = pcol;
    move_pos(a0, row, col, H, W, p.up_mask, p.down_mask, p.left_mask, p.right_mask);
    const int64_t HW = (int64_t)H * W;
    const int strips = (H + SHv - 1) / SHv, spp = (strips + P - 1) / P;
    const int s_begin = part * spp, s_end = min(strips, s_begin + spp);
    uint8_t* grid = (odd ? buf1 : buf0) + e * HW;
    if (n > 0) {
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
        auto get_mask = [&]() -> uint32_t { return wave_windy_mask(p, wl, e, rs, lane); };
        const uint8_t* __restrict__ S = grid;
        uint8_t* __restrict__ Dst = (odd ? buf0 : buf1) + e * HW;
        const uint32_t lofs = 4 * NW * (uint32_t)lane;
        int32_t cntT = 0, cntF = 0, cntV = 0;
        for (int s = s_begin + wave; s < s_end; s += 4)
            windy_rows_strip_f<NW, SHv, RDv, STD>(S, Dst, s * SHv, H, get_mask, lofs, rep4(p.empty),
                                                           rep4(p.tree), rep4(p.fire), cntT, cntF, cntV);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            cntT += __shfl_xor(cntT, off);
            cntF += __shfl_xor(cntF, off);
            cntV += __shfl_xor(cntV, off);
        }
        if (lane == 0) {
            wave_cnt[wave][0] = cntV - cntT - cntF;
            wave_cnt[wave][1] = cntT;
            wave_cnt[wave][2] = cntF;
        }
        __syncthreads();
        grid = Dst;
    }
    if (tid != 0) return;
    // this part's contribution: n > 0 its rows' counts (+ Modify when it holds the bulldozer's row); n == 0 the Modify's
    // count changes + 1 (owner only); n < 0 nothing
    int32_t pE = 0, pT = 0, pF = 0;
    uint32_t h = 0;
    if (n > 0) {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            pE += wave_cnt[w][0];
            pT += wave_cnt[w][1];
            pF += wave_cnt[w][2];
        }
    } else if (n == 0) {
        pE = pT = pF = 1;
    }
    const int owner = min((row / SHv) / spp, P - 1);
    if (n >= 0 && part == owner && act1 && row >= 0 && row < H && col >= 0 && col < W) {  // (no write outside the grid)
        const int v = grid[(int64_t)row * W + col];
        const int nv = p.effect[v];
        if (nv >= 0) {
            grid[(int64_t)row * W + col] = (uint8_t)nv;
            h = 1;
            const int c_old = cell_category(v, p.empty, p.tree, p.fire), c_new = cell_category(nv, p.empty, p.tree, p.fire);
            if (c_old == 0) pE -= 1; else if (c_old == 1) pT -= 1; else if (c_old == 2) pF -= 1;
            if (c_new == 0) pE += 1; else if (c_new == 1) pT += 1; else if (c_new == 2) pF += 1;
        }
    }
    if (n == 0 && part != owner) pE = pT = pF = 0;
    const unsigned long long pk = (unsigned long long)(uint32_t)pE | ((unsigned long long)(uint32_t)pT << 20) |
                                  ((unsigned long long)(uint32_t)pF << 40) | ((unsigned long long)h << 60) |
                                  (1ull << 61);
    const unsigned long long old = atomicAdd(&meet[e], pk);
    if ((int)(old >> 61) != P - 1) return;  // not the last part to arrive
    const unsigned long long tot = old + pk;
    meet[e] = 0ull;
    steps[e] = n;
    if (n < 0) {
        reward[e] = 0.0;
        return;
    }
    accu[e] = x - reps;
    int32_t cE = (int32_t)(tot & 0xFFFFFu), cT = (int32_t)((tot >> 20) & 0xFFFFFu), cF = (int32_t)((tot >> 40) & 0xFFFFFu);
    if (n > 0) {
        parity[e] = odd ? 0 : 1;
    } else {
        cE = c0 + cE - 1;
        cT = c1 + cT - 1;
        cF = c2 + cF - 1;
    }
    const uint8_t hh = (uint8_t)((tot >> 60) & 1u);
    pos[2 * e] = row;
    pos[2 * e + 1] = col;
    counts[3 * e + 0] = cE;
    counts[3 * e + 1] = cT;
    counts[3 * e + 2] = cF;
    hit[e] = hh;
    reward[e] = (cT + cF) > 0 ? -((double)cF / (double)(cT + cF)) : (double)NAN;
    done[e] = cF == 0 ? 1 : 0;
    rng_step[e] = rs + (uint32_t)n;
    if (steps_elapsed) steps_elapsed[e] = se + 1;
}

// K env steps of every env in ONE launch under the random policy of gca_bulldozer_step_fused_random (r06): one
// workgroup per env marches its env through the K steps with the per-env state in registers (read once, written once):
// the action drawn from (env, rng_step) exactly as gca_random_actions does, RepeatCA's time, the Windy CA over the env's
// strips when the step takes one (every wave, one workgroup barrier before the counts), Move / Modify (thread 0) and
// reward / done, broadcast to the workgroup through LDS behind one barrier per step. Bit for bit K calls of
// gca_bulldozer_step_fused_random (tests/test_gpu_windy.py). Workgroups never wait for each other, so an env whose fire
// burns out or whose CA steps are few runs ahead: the K x E env steps cost the slowest env's chain, not K launches of
// the slowest step. Per-step outputs (optional): the actions (K, E, 2), rewards (K, E) and done flags (K, E).
// SOLO (the host proves that Modify never changes the FIRE count: no effect maps a FIRE cell or onto FIRE -- the
// bulldozer's {TREE: EMPTY}): thread 0 alone applies Modify and keeps the E / T counts, hit and reward; every other
// thread needs only the FIRE count (done), which then changes only in CA steps, whose counts all threads sum. A step
// without a CA pass needs no barrier at all; a CA step opens with one (thread 0's Modify writes since the last barrier,
// before the other waves' CA reads) and closes with one (the new grid and the counts). Otherwise thread 0 applies
// Modify and broadcasts its counts through LDS behind a barrier per step. (Every thread applying Modify itself was
// tried first: a slow wave then reads the cell a fast wave already rewrote and miscounts, r06f.)
template <int NW, bool STD, bool SOLO>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void bulldozer_rollout_random_kernel(
    gca_bulldozer_params p, int K, uint64_t seed, int32_t* __restrict__ action_out, double* __restrict__ reward_out,
    uint8_t* __restrict__ done_out, double* __restrict__ accu, int32_t* __restrict__ steps, uint8_t* __restrict__ done,
    const double* __restrict__ wind, int64_t wind_stride, uint32_t* __restrict__ rng_step, uint8_t* __restrict__ parity,
    uint8_t* buf0, uint8_t* buf1, int H, int32_t* __restrict__ pos, int32_t* __restrict__ counts,
    uint8_t* __restrict__ hit, double* __restrict__ reward, int64_t* __restrict__ steps_elapsed, int E) {
    constexpr int W = 256 * NW;
    __shared__ int32_t wave_cnt[2][16][3];  // per CA step, double-buffered (no barrier after the counts are read)
    __shared__ int32_t bc[2][4];  // !SOLO: thread 0 -> the workgroup, per step (double-buffered): E, T, F counts, hit
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, nw = (int)(blockDim.x >> 6);
    const uint32_t env_id = (uint32_t)(p.env_offset + e);
    bool was_done = done[e] != 0;
    uint32_t rs = rng_step[e];
    double acc = accu[e];
    bool odd = parity[e] != 0;
    int32_t row = pos[2 * e], col = pos[2 * e + 1];
    int32_t cE = counts[3 * e + 0], cT = counts[3 * e + 1], cF = counts[3 * e + 2];
    int64_t se = steps_elapsed ? steps_elapsed[e] : 0;
    uint8_t h = hit[e];
    double rew = reward[e];
    int last_n = 0, ca = 0;
    double wl[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) wl[k] = wind[(int64_t)e * wind_stride + k];
    const int64_t HW = (int64_t)H * W;
    const uint32_t lofs = 4 * NW * (uint32_t)lane;
    for (int k = 0; k < K; ++k) {
        int32_t act0, act1;
        fused_action(nullptr, FusedPolicy{seed, nullptr}, e, env_id, rs, act0, act1);
        const size_t ke = (size_t)k * E + e;
        if (action_out && tid == 0) {
            action_out[2 * ke] = act0;
            action_out[2 * ke + 1] = act1;
        }
        const int a0 = clampi_dev(act0, 0, 8), a1s = clampi_dev(act1, 0, 1);
        const double x = acc + ((p.t_move[a0] + p.t_shoot[a1s]) + p.t_any);
        const double reps = trunc(x);
        const int n = was_done ? -1 : (int)reps;
        last_n = n;
        if (n < 0) {  // finished: a graceful no-op step (ca_env.py:50-62), nothing but the reward changes
            rew = 0.0;
            if (tid == 0) {
                if (reward_out) reward_out[ke] = 0.0;
                if (done_out) done_out[ke] = 1;
            }
            continue;
        }
        int nrow = row, ncol = col;
        move_pos(a0, nrow, ncol, H, W, p.up_mask, p.down_mask, p.left_mask, p.right_mask);
        uint8_t* grid = (odd ? buf1 : buf0) + e * HW;
        if (n > 0) {
            if constexpr (SOLO) __syncthreads();  // thread 0's Modify writes since the last barrier, before the CA reads
            auto get_mask = [&]() -> uint32_t { return wave_windy_mask(p, wl, e, rs, lane); };
            const uint8_t* S = grid;
            uint8_t* Dst = (odd ? buf0 : buf1) + e * HW;
            int32_t cntT = 0, cntF = 0, cntV = 0;
            for (int s0 = wave * FUSED_SH<NW>; s0 < H; s0 += nw * FUSED_SH<NW>)
                windy_rows_strip_f<NW, FUSED_SH<NW>, FUSED_RD<NW>, STD>(S, Dst, s0, H, get_mask, lofs, rep4(p.empty),
                                                                       rep4(p.tree), rep4(p.fire), cntT, cntF, cntV);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                cntT += __shfl_xor(cntT, off);
                cntF += __shfl_xor(cntF, off);
                cntV += __shfl_xor(cntV, off);
            }
            int32_t (*WC)[3] = wave_cnt[ca & 1];  // a wave that runs ahead writes the other buffer at the next CA step
            ++ca;
            if (lane == 0) {
                WC[wave][0] = cntV - cntT - cntF;
                WC[wave][1] = cntT;
                WC[wave][2] = cntF;
            }
            __syncthreads();  // the new grid (every wave's stores) and the counts are complete
            grid = Dst;
            odd = !odd;
            cE = cT = cF = 0;
            for (int w = 0; w < nw; ++w) {
                cE += WC[w][0];
                cT += WC[w][1];
                cF += WC[w][2];
            }
        }
        acc = x - reps;
        row = nrow;
        col = ncol;
        // MoveModify (move_modify.py:128-134): Modify at the new position, on the post-CA grid
        auto modify = [&](int32_t& mE, int32_t& mT, int32_t& mF) -> uint8_t {
            uint8_t hh = 0;
            if (act1 && row >= 0 && row < H && col >= 0 && col < W) {
                const int v = grid[(int64_t)row * W + col];
                const int nv = p.effect[v];
                if (nv >= 0) {
                    grid[(int64_t)row * W + col] = (uint8_t)nv;
                    hh = 1;
                    const int c_old = cell_category(v, p.empty, p.tree, p.fire);
                    const int c_new = cell_category(nv, p.empty, p.tree, p.fire);
                    if (c_old == 0) mE -= 1; else if (c_old == 1) mT -= 1; else if (c_old == 2) mF -= 1;
                    if (c_new == 0) mE += 1; else if (c_new == 1) mT += 1; else if (c_new == 2) mF += 1;
                }
            }
            return hh;
        };
        if constexpr (SOLO) {
            if (tid == 0) h = modify(cE, cT, cF);  // FIRE count unchanged (host-checked): the other threads' cF holds
        } else {
            int32_t* B = bc[k & 1];
            if (tid == 0) {
                const uint8_t hh = modify(cE, cT, cF);
                B[0] = cE;
                B[1] = cT;
                B[2] = cF;
                B[3] = hh;
            }
            __syncthreads();  // the Modify write and its counts, for every wave's next step
            cE = B[0];
            cT = B[1];
            cF = B[2];
            h = (uint8_t)B[3];
        }
        rew = (cT + cF) > 0 ? -((double)cF / (double)(cT + cF)) : (double)NAN;
        was_done = cF == 0;
        rs += (uint32_t)n;
        se += 1;
        if (tid == 0) {
            if (reward_out) reward_out[ke] = rew;
            if (done_out) done_out[ke] = was_done ? 1 : 0;
        }
    }
    if (tid != 0 || K == 0) return;
    steps[e] = last_n;
    reward[e] = rew;
    accu[e] = acc;
    parity[e] = odd ? 1 : 0;
    pos[2 * e] = row;
    pos[2 * e + 1] = col;
    counts[3 * e + 0] = cE;
    counts[3 * e + 1] = cT;
    counts[3 * e + 2] = cF;
    hit[e] = h;
    done[e] = was_done ? 1 : 0;
    rng_step[e] = rs;
    if (steps_elapsed) steps_elapsed[e] = se;
}

template <int NW>
static void launch_rows(uint8_t* b0, uint8_t* b1, const uint8_t* parity, const int32_t* steps, int pass,
                        const uint8_t* dm, int E, int H, int empty, int tree, int fire, int32_t* counts,
                        hipStream_t st) {
    const int strips = (H + WINDY_RSH - 1) / WINDY_RSH;
    const int bpe = (strips + 3) / 4;
    if (empty == 0 && tree == 3 && fire == 25)
        hipLaunchKernelGGL((windy_rows_kernel<NW, true>), dim3((unsigned)((int64_t)E * bpe)), dim3(256), 0, st, b0, b1,
                           parity, steps, pass, dm, H, bpe, rep4(empty), rep4(tree), rep4(fire), counts);
    else
        hipLaunchKernelGGL((windy_rows_kernel<NW, false>), dim3((unsigned)((int64_t)E * bpe)), dim3(256), 0, st, b0, b1,
                           parity, steps, pass, dm, H, bpe, rep4(empty), rep4(tree), rep4(fire), counts);
}

// ------------------------------------------------------------------ host API
extern "C" int gca_windy_dirmask(const double* wind, int64_t wind_stride, const double* roll, uint64_t seed,
                                 const uint32_t* rng_step, const int32_t* steps, int pass, int env_offset,
                                 uint8_t* dir_mask, int E, void* stream) {
    GCA_CHECK_ARG(E > 0 && wind && dir_mask, "E > 0, wind and dir_mask required");
    GCA_CHECK_ARG(wind_stride >= 0, "wind_stride >= 0");
    const int threads = 256, blocks = (E + threads - 1) / threads;
    hipLaunchKernelGGL(windy_dirmask_kernel, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, wind, wind_stride,
                       roll, (uint32_t)seed, (uint32_t)(seed >> 32), rng_step, steps, pass, env_offset, dir_mask, E);
    GCA_CHECK_LAUNCH("windy_dirmask");
    return GCA_OK;
}

template <int LPR>
static void launch_fast(uint8_t* b0, uint8_t* b1, const uint8_t* parity, const int32_t* steps, int pass,
                        const uint8_t* dm, int E, int H, int empty, int tree, int fire, int32_t* counts,
                        hipStream_t st) {
    constexpr int RPW = 64 / LPR;
    // strip height: >= 32 rows when there is enough work, multiple of RPW
    const int64_t rows = (int64_t)E * H;
    int SH = 32;
    while (SH > RPW && rows / SH < 8192) SH >>= 1;
    if (SH < RPW) SH = RPW;
    SH = ((SH + RPW - 1) / RPW) * RPW;
    const int strips = (H + SH - 1) / SH;
    const int bpe = (strips + 3) / 4;
    hipLaunchKernelGGL(windy_fast_kernel<LPR>, dim3((unsigned)((int64_t)E * bpe)), dim3(256), 0, st, b0, b1, parity,
                       steps, pass, dm, H, SH, bpe, rep4(empty), rep4(tree), rep4(fire), counts);
}

extern "C" int gca_windy_step(uint8_t* buf0, uint8_t* buf1, const uint8_t* parity, const int32_t* steps, int pass,
                              const uint8_t* dir_mask, int E, int H, int W, int empty, int tree, int fire,
                              int force_exact, int32_t* counts, void* stream) {
    GCA_CHECK_ARG(buf0 && buf1 && dir_mask, "buffers and dir_mask required");
    GCA_CHECK_ARG(E > 0 && H > 0 && W > 0, "E, H, W must be positive");
    GCA_CHECK_ARG(empty >= 0 && empty < 256 && tree >= 0 && tree < 256 && fire >= 0 && fire < 256,
                  "cell codes must fit in u8");
    GCA_CHECK_ARG(empty < tree && tree < fire, "cell codes must satisfy empty < tree < fire (ca_windy.py:158)");
    hipStream_t st = (hipStream_t)stream;
    const bool aligned = ((((uintptr_t)buf0) | ((uintptr_t)buf1)) & 15u) == 0;
    const int LPR = W / 16;
    const bool fast = !force_exact && empty == 0 && aligned && (W % 16 == 0) && LPR >= 1 && LPR <= 64 && (64 % LPR) == 0;
    if (fast && (W == 256 || W == 512)) {
        if (W == 256) launch_rows<1>(buf0, buf1, parity, steps, pass, dir_mask, E, H, empty, tree, fire, counts, st);
        else launch_rows<2>(buf0, buf1, parity, steps, pass, dir_mask, E, H, empty, tree, fire, counts, st);
        GCA_CHECK_LAUNCH("windy_rows");
    } else if (fast) {
        switch (LPR) {
            case 1: launch_fast<1>(buf0, buf1, parity, steps, pass, dir_mask, E, H, empty, tree, fire, counts, st); break;
            case 2: launch_fast<2>(buf0, buf1, parity, steps, pass, dir_mask, E, H, empty, tree, fire, counts, st); break;
            case 4: launch_fast<4>(buf0, buf1, parity, steps, pass, dir_mask, E, H, empty, tree, fire, counts, st); break;
            case 8: launch_fast<8>(buf0, buf1, parity, steps, pass, dir_mask, E, H, empty, tree, fire, counts, st); break;
            case 16: launch_fast<16>(buf0, buf1, parity, steps, pass, dir_mask, E, H, empty, tree, fire, counts, st); break;
            case 32: launch_fast<32>(buf0, buf1, parity, steps, pass, dir_mask, E, H, empty, tree, fire, counts, st); break;
            case 64: launch_fast<64>(buf0, buf1, parity, steps, pass, dir_mask, E, H, empty, tree, fire, counts, st); break;
        }
        GCA_CHECK_LAUNCH("windy_fast");
    } else {
        const int64_t n = (int64_t)E * H * W;
        const int threads = 256;
        const int64_t blocks = (n + threads - 1) / threads;
        GCA_CHECK_ARG(blocks < (int64_t)1 << 31, "grid too large for the exact kernel");
        hipLaunchKernelGGL(windy_exact_kernel, dim3((unsigned)blocks), dim3(threads), 0, st, buf0, buf1, parity, steps,
                           pass, dir_mask, E, H, W, empty, tree, fire, counts);
        GCA_CHECK_LAUNCH("windy_exact");
    }
    return GCA_OK;
}

static int bulldozer_step_fused_impl(const gca_bulldozer_params* p, const int32_t* action, FusedPolicy pol,
                                     double* accu, int32_t* steps, uint8_t* done, const double* wind,
                                     int64_t wind_stride, uint32_t* rng_step, uint8_t* parity, uint8_t* buf0,
                                     uint8_t* buf1, int H, int W, int32_t* pos, int32_t* counts, uint8_t* hit,
                                     double* reward, int64_t* steps_elapsed, uint64_t* meet, int E, void* stream) {
    GCA_CHECK_ARG(p && accu && steps && done && wind && rng_step && parity && buf0 && buf1 && pos && counts &&
                      hit && reward && E > 0 && H > 0,
                  "bulldozer_step_fused: null argument or empty batch");
    GCA_CHECK_ARG(W == 256 || W == 512, "bulldozer_step_fused: W must be 256 or 512 (the row-stream CA)");
    GCA_CHECK_ARG(p->empty == 0 && p->empty < p->tree && p->tree < p->fire && p->fire < 256,
                  "bulldozer_step_fused: cell codes must be empty = 0 < tree < fire < 256 (the closed-form rule)");
    GCA_CHECK_ARG(((((uintptr_t)buf0) | ((uintptr_t)buf1)) & 15u) == 0, "bulldozer_step_fused: buffers 16-B aligned");
    GCA_CHECK_ARG(wind_stride >= 0, "bulldozer_step_fused: wind_stride >= 0");
    // at most one CA step per env step: accu < 1 on entry, so (t_move + t_shoot) + t_any < 1 for every action
    double tmax = 0.0;
    for (int a = 0; a < 9; ++a)
        for (int b = 0; b < 2; ++b) tmax = fmax(tmax, (p->t_move[a] + p->t_shoot[b]) + p->t_any);
    GCA_CHECK_ARG(tmax < 1.0, "bulldozer_step_fused: an action can take >= 1 time unit (several CA passes per step): "
                              "use gca_bulldozer_pre / gca_windy_step / gca_bulldozer_post");
    const int fsh = W == 256 ? FUSED_SH<1> : FUSED_SH<2>;
    const int strips = (H + fsh - 1) / fsh;
    const int threads = 64 * (strips < 16 ? strips : 16);
    hipStream_t st = (hipStream_t)stream;
    const bool std_codes = p->empty == 0 && p->tree == 3 && p->fire == 25;
#define GCA_FUSED_LAUNCH(NWV, STDV)                                                                                 \
    hipLaunchKernelGGL((bulldozer_step_fused_kernel<NWV, STDV>), dim3((unsigned)E), dim3(threads), 0, st, *p, action, \
                       accu, steps, done, wind, wind_stride, rng_step, parity, buf0, buf1, H, pos, counts, hit, reward,   \
                       steps_elapsed, pol)
    // with the caller's meeting slots: P workgroups per env (2 at W = 256, 4 at 512); without: one
#define GCA_FUSED_PARTS_LAUNCH(NWV, STDV, PV)                                                                     \
    hipLaunchKernelGGL((bulldozer_step_fused_parts_kernel<NWV, STDV, PV>), dim3((unsigned)E * PV), dim3(256), 0, st, *p, \
                       action, accu, steps, done, wind, wind_stride, rng_step, parity, buf0, buf1, H, pos, counts, hit,  \
                       reward, steps_elapsed, (unsigned long long*)meet, pol)
    // the parts meet in 20-bit E / T / F fields of one 64-bit word per env: a field's total reaches H*W (+1 when Modify
    // moves an uncategorised code to a category), so grids of 2^20 - 1 cells or more take the one-workgroup kernel,
    // which sums in int32 (W = 256 at H >= 4096, W = 512 at H >= 2048); `meet` is then left untouched
    // (zero, as the contract requires)
    const bool parts_fit = (int64_t)H * W + 1 < ((int64_t)1 << 20);
    if (meet && parts_fit) {
        GCA_CHECK_ARG((int64_t)E * 4 < ((int64_t)1 << 31), "bulldozer_step_fused: too many envs");
        if (W == 256) {
            if (std_codes) GCA_FUSED_PARTS_LAUNCH(1, true, 2); else GCA_FUSED_PARTS_LAUNCH(1, false, 2);
        } else {
            if (std_codes) GCA_FUSED_PARTS_LAUNCH(2, true, 4); else GCA_FUSED_PARTS_LAUNCH(2, false, 4);
        }
    } else if (W == 256) {
        if (std_codes) GCA_FUSED_LAUNCH(1, true); else GCA_FUSED_LAUNCH(1, false);
    } else {
        if (std_codes) GCA_FUSED_LAUNCH(2, true); else GCA_FUSED_LAUNCH(2, false);
    }
#undef GCA_FUSED_LAUNCH
#undef GCA_FUSED_PARTS_LAUNCH
    GCA_CHECK_LAUNCH("bulldozer_step_fused");
    return GCA_OK;
}

extern "C" int gca_bulldozer_step_fused(const gca_bulldozer_params* p, const int32_t* action, double* accu,
                                        int32_t* steps, uint8_t* done, const double* wind, int64_t wind_stride,
                                        uint32_t* rng_step, uint8_t* parity, uint8_t* buf0, uint8_t* buf1, int H, int W,
                                        int32_t* pos, int32_t* counts, uint8_t* hit, double* reward,
                                        int64_t* steps_elapsed, uint64_t* meet, int E, void* stream) {
    GCA_CHECK_ARG(action, "bulldozer_step_fused: action required");
    return bulldozer_step_fused_impl(p, action, FusedPolicy{0u, nullptr}, accu, steps, done, wind, wind_stride, rng_step,
                                     parity, buf0, buf1, H, W, pos, counts, hit, reward, steps_elapsed, meet, E, stream);
}

extern "C" int gca_bulldozer_step_fused_random(const gca_bulldozer_params* p, uint64_t action_seed, int32_t* action_out,
                                               double* accu, int32_t* steps, uint8_t* done, const double* wind,
                                               int64_t wind_stride, uint32_t* rng_step, uint8_t* parity, uint8_t* buf0,
                                               uint8_t* buf1, int H, int W, int32_t* pos, int32_t* counts, uint8_t* hit,
                                               double* reward, int64_t* steps_elapsed, uint64_t* meet, int E,
                                               void* stream) {
    return bulldozer_step_fused_impl(p, nullptr, FusedPolicy{action_seed, action_out}, accu, steps, done, wind,
                                     wind_stride, rng_step, parity, buf0, buf1, H, W, pos, counts, hit, reward,
                                     steps_elapsed, meet, E, stream);
}

extern "C" int gca_bulldozer_rollout_random(const gca_bulldozer_params* p, uint64_t action_seed, int K,
                                            int32_t* action_out, double* reward_out, uint8_t* done_out, double* accu,
                                            int32_t* steps, uint8_t* done, const double* wind, int64_t wind_stride,
                                            uint32_t* rng_step, uint8_t* parity, uint8_t* buf0, uint8_t* buf1, int H,
                                            int W, int32_t* pos, int32_t* counts, uint8_t* hit, double* reward,
                                            int64_t* steps_elapsed, int E, void* stream) {
    GCA_CHECK_ARG(p && accu && steps && done && wind && rng_step && parity && buf0 && buf1 && pos && counts && hit &&
                      reward && E > 0 && H > 0 && K >= 0,
                  "bulldozer_rollout_random: null argument, empty batch or K < 0");
    GCA_CHECK_ARG(W == 256 || W == 512, "bulldozer_rollout_random: W must be 256 or 512 (the row-stream CA)");
    GCA_CHECK_ARG(p->empty == 0 && p->empty < p->tree && p->tree < p->fire && p->fire < 256,
                  "bulldozer_rollout_random: cell codes must be empty = 0 < tree < fire < 256 (the closed-form rule)");
    GCA_CHECK_ARG(((((uintptr_t)buf0) | ((uintptr_t)buf1)) & 15u) == 0, "bulldozer_rollout_random: buffers 16-B aligned");
    GCA_CHECK_ARG(wind_stride >= 0, "bulldozer_rollout_random: wind_stride >= 0");
    GCA_CHECK_ARG((int64_t)K * E < ((int64_t)1 << 40), "bulldozer_rollout_random: K x E too large");
    double tmax = 0.0;
    for (int a = 0; a < 9; ++a)
        for (int b = 0; b < 2; ++b) tmax = fmax(tmax, (p->t_move[a] + p->t_shoot[b]) + p->t_any);
    GCA_CHECK_ARG(tmax < 1.0, "bulldozer_rollout_random: an action can take >= 1 time unit (several CA passes per step)");
    if (K == 0) return GCA_OK;
    const int fsh = W == 256 ? FUSED_SH<1> : FUSED_SH<2>;
    const int strips = (H + fsh - 1) / fsh;
    const int threads = 64 * (strips < 16 ? strips : 16);
    hipStream_t st = (hipStream_t)stream;
    const bool std_codes = p->empty == 0 && p->tree == 3 && p->fire == 25;
    // SOLO: Modify never changes the FIRE count (the kernel's comment)
    bool solo = true;
    auto fire_cat = [&](int v) { return v == p->fire; };
    for (int v = 0; v < 256; ++v) {
        const int nv = p->effect[v];
        if (nv >= 0 && fire_cat(v) != fire_cat(nv)) solo = false;
    }
#define GCA_ROLLOUT_LAUNCH(NWV, STDV, SOLOV)                                                                             \
    hipLaunchKernelGGL((bulldozer_rollout_random_kernel<NWV, STDV, SOLOV>), dim3((unsigned)E), dim3(threads), 0, st, *p, \
                       K, action_seed, action_out, reward_out, done_out, accu, steps, done, wind, wind_stride, rng_step,  \
                       parity, buf0, buf1, H, pos, counts, hit, reward, steps_elapsed, E)
    if (W == 256) {
        if (std_codes && solo) GCA_ROLLOUT_LAUNCH(1, true, true);
        else if (solo) GCA_ROLLOUT_LAUNCH(1, false, true);
        else GCA_ROLLOUT_LAUNCH(1, false, false);
    } else {
        if (std_codes && solo) GCA_ROLLOUT_LAUNCH(2, true, true);
        else if (solo) GCA_ROLLOUT_LAUNCH(2, false, true);
        else GCA_ROLLOUT_LAUNCH(2, false, false);
    }
#undef GCA_ROLLOUT_LAUNCH
    GCA_CHECK_LAUNCH("bulldozer_rollout_random");
    return GCA_OK;
}
