// gca_alex.hip — Alexandridis fire-spread CA step on gfx950.
// Reference: PartiallyObservableForestFireJax._update_grid (ca_alexandridis_jax.py:321-424),
//            _compute_burn_probability (:164-206), kernels (:54-160).
//
// Per cell (r,c) of env e, with the reference's zero ("EMPTY") padding:
//   heat   = sum_{|dr|,|dc|<=R} [x(r+dr,c+dc)==FIRE] * K(max(|dr|,|dc|))       (13x13 @256)
//   dous   = inner * D3 + border * (D5 - D3),  Dk = sum of dousing over the kxk box  (5x5)
//   p_d    = ((((heat - dous) * (1+veg)) * (1+den)) * wind[d]) * p_slope[d]   (left-to-right f32)
//   TREE -> FIRE iff some neighbour d is FIRE and draw_d < p_d; EMPTY -> TREE iff u < p_tree;
//   FIRE -> EMPTY iff age <= 1; new fires get age randint[lo,hi); old fires age -= 1.
//
// Mapping (one workgroup = 256 threads = TH x TW = 16 x 256 cells of one env):
//   thread (tr = tid/16, q = tid%16) owns 16 consecutive cells of one row -> 16-B loads.
//   LDS: the grid rows [r0-R, r0+TH+R) x cols [c0-16, c0+TW+16) staged once, and the
//   column-prefix CP of packed v = fire | dousing<<16 (u32). Box sums of radius k are
//   sum over 16+2k columns of (CP[row+k+1] - CP[row-k]) with a sliding window; fire and
//   dousing fields never interfere because every box sum of either field is < 2^16.
//   Ring counts n_k = B_k - B_{k-1} are exact integers; heat is then
//   ((w0*n0 + w1*n1) + w2*n2) + ...  in f32 (fixed order, no fma): deterministic.
// Draws: INJECT = the reference's own uniform/randint arrays (exact rule);
//        Philox = one Philox4x32-10 block per cell that needs it: x0 burn, x1 grow, x2 age;
//        burn iff u0 < 1 - prod_{fire d}(1 - clamp01(p_d)) (same law as independent draws).
#include "gca_common.h"

namespace {

constexpr int TH = 16;
constexpr int TW = 256;
constexpr int CW = TW + 32;  // staged columns: [c0-16, c0+TW+16)

__device__ __forceinline__ float clamp01(float v) { return fminf(fmaxf(v, 0.0f), 1.0f); }

template <int R, bool INJECT>
__global__ __launch_bounds__(256, 2) void alex_step_kernel(
    gca_alex_params p, int H, int W, int tiles_r, int tiles_c, const uint8_t* __restrict__ grid_in,
    uint8_t* __restrict__ grid_out, const int16_t* __restrict__ age_in, int16_t* __restrict__ age_out,
    const uint8_t* __restrict__ veg, const uint8_t* __restrict__ den, const uint8_t* __restrict__ dousing,
    const float* __restrict__ p_slope, const int32_t* __restrict__ wind_index, const uint32_t* __restrict__ rng_step,
    const float* __restrict__ inj_burn, const float* __restrict__ inj_grow, const int32_t* __restrict__ inj_age,
    float* __restrict__ prob_out, int32_t* __restrict__ counts) {
    constexpr int RS = R < 2 ? 2 : R;  // staged halo: heat radius, at least the 5x5 dousing box
    constexpr int RR = TH + 2 * RS;    // staged rows
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* CP = reinterpret_cast<uint32_t*>(smem);            // [RR+1][CW]
    uint8_t* G = smem + sizeof(uint32_t) * (RR + 1) * CW;        // [RR][CW]

    const int tiles = tiles_r * tiles_c;
    const int e = blockIdx.x / tiles;
    const int tile = blockIdx.x - e * tiles;
    const int r0 = (tile / tiles_c) * TH, c0 = (tile % tiles_c) * TW;
    const int64_t HW = (int64_t)H * W;
    const uint8_t* gE = grid_in + (int64_t)e * HW;
    const uint8_t* dE = dousing + (int64_t)e * HW;
    const int tid = threadIdx.x;
    const bool rows16 = ((W & 15) == 0) &&
                        ((((uintptr_t)grid_in) | ((uintptr_t)dousing) | ((uintptr_t)grid_out) | ((uintptr_t)veg) |
                          ((uintptr_t)den) | ((uintptr_t)age_in) | ((uintptr_t)age_out) | ((uintptr_t)p_slope)) &
                         15u) == 0;

    // ---------------- per-thread cells
    const int tr = tid >> 4, q = tid & 15;
    const int r = r0 + tr;
    const int cbase = c0 + 16 * q;
    const bool row_ok = r < H;
    const int rr = RS + tr;          // staged row of r
    const int cc0 = 16 + 16 * q;     // staged column of cbase

    // ---- per-cell contexts (packed)
    const int64_t rowoff = (int64_t)e * HW + (int64_t)r * W + cbase;
    const bool vec = row_ok && rows16 && (cbase + 16 <= W);
    uint32_t agew[8], vgw[4], dnw[4];
    if (vec) {
        const uint4 a0 = *reinterpret_cast<const uint4*>(age_in + rowoff);
        const uint4 a1 = *reinterpret_cast<const uint4*>(age_in + rowoff + 8);
        const uint4 v4 = *reinterpret_cast<const uint4*>(veg + rowoff);
        const uint4 d4 = *reinterpret_cast<const uint4*>(den + rowoff);
        agew[0] = a0.x; agew[1] = a0.y; agew[2] = a0.z; agew[3] = a0.w;
        agew[4] = a1.x; agew[5] = a1.y; agew[6] = a1.z; agew[7] = a1.w;
        vgw[0] = v4.x; vgw[1] = v4.y; vgw[2] = v4.z; vgw[3] = v4.w;
        dnw[0] = d4.x; dnw[1] = d4.y; dnw[2] = d4.z; dnw[3] = d4.w;
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) agew[k] = 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) vgw[k] = dnw[k] = 0x01010101u;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (row_ok && cbase + i < W) {
                agew[i >> 1] |= (uint32_t)(uint16_t)age_in[rowoff + i] << (16 * (i & 1));
                const uint32_t sh = 8 * (i & 3);
                vgw[i >> 2] = (vgw[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)veg[rowoff + i] << sh);
                dnw[i >> 2] = (dnw[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)den[rowoff + i] << sh);
            }
        }
    }

    // ---------------- stage: grid bytes -> G, packed fire|dousing<<16 -> CP rows 1..RR
    const uint32_t Fp = rep4((uint32_t)p.fire);
    for (int ch = tid; ch < RR * (CW / 16); ch += 256) {
        const int rr = ch / (CW / 16), cq = ch - rr * (CW / 16);
        const int gr = r0 - RS + rr, gc = c0 - 16 + 16 * cq;
        uint32_t gw[4] = {0u, 0u, 0u, 0u}, dw[4] = {0u, 0u, 0u, 0u};
        const uint32_t Ep = rep4((uint32_t)p.empty);
        gw[0] = gw[1] = gw[2] = gw[3] = Ep;
        if (gr >= 0 && gr < H) {
            if (rows16 && gc >= 0 && gc + 16 <= W) {
                const uint4 a = *reinterpret_cast<const uint4*>(gE + (int64_t)gr * W + gc);
                const uint4 b = *reinterpret_cast<const uint4*>(dE + (int64_t)gr * W + gc);
                gw[0] = a.x; gw[1] = a.y; gw[2] = a.z; gw[3] = a.w;
                dw[0] = b.x; dw[1] = b.y; dw[2] = b.z; dw[3] = b.w;
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int c = gc + i;
                    if (c >= 0 && c < W) {
                        const uint32_t sh = 8 * (i & 3);
                        gw[i >> 2] = (gw[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)gE[(int64_t)gr * W + c] << sh);
                        dw[i >> 2] |= (uint32_t)dE[(int64_t)gr * W + c] << sh;
                    }
                }
            }
        }
        *reinterpret_cast<uint4*>(G + rr * CW + 16 * cq) = make_uint4(gw[0], gw[1], gw[2], gw[3]);
        uint32_t* cp = CP + (rr + 1) * CW + 16 * cq;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t f = bytes_eq01(gw[j], Fp);
            uint4 v;
            v.x = (f & 1u) | ((dw[j] & 0xFFu) << 16);
            v.y = ((f >> 8) & 1u) | (((dw[j] >> 8) & 0xFFu) << 16);
            v.z = ((f >> 16) & 1u) | (((dw[j] >> 16) & 0xFFu) << 16);
            v.w = ((f >> 24) & 1u) | (((dw[j] >> 24) & 0xFFu) << 16);
            *reinterpret_cast<uint4*>(cp + 4 * j) = v;
        }
    }
    for (int cc = tid; cc < CW; cc += 256) CP[cc] = 0u;
    __syncthreads();
    // ---------------- column prefix (in place)
    for (int cc = tid; cc < CW; cc += 256) {
        uint32_t run = 0u;
#pragma unroll 4
        for (int rr = 1; rr <= RR; ++rr) {
            run += CP[rr * CW + cc];
            CP[rr * CW + cc] = run;
        }
    }
    __syncthreads();

    // ---- 3x3 neighbour FIRE mask per cell, one byte per cell: bit d = neighbourhood entry
    //      (a,b) row-major without the centre, entry (a,b) = cell (r+a-1, c+b-1) (:332-337)
    uint32_t fm[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const uint8_t* gp = G + (rr - 1 + a) * CW + cc0 - 4;
        const uint4 mid = *reinterpret_cast<const uint4*>(gp + 4);
        const uint32_t f[6] = {bytes_eq01(*reinterpret_cast<const uint32_t*>(gp), Fp), bytes_eq01(mid.x, Fp),
                               bytes_eq01(mid.y, Fp), bytes_eq01(mid.z, Fp), bytes_eq01(mid.w, Fp),
                               bytes_eq01(*reinterpret_cast<const uint32_t*>(gp + 20), Fp)};
        const int dbase = a * 3 - (a > 1 ? 1 : 0);  // d of (a, 0)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t left = __builtin_amdgcn_alignbyte(f[j + 1], f[j], 3);   // column c-1
            const uint32_t right = __builtin_amdgcn_alignbyte(f[j + 2], f[j + 1], 1);  // column c+1
            fm[j] |= left << dbase;
            if (a != 1) fm[j] |= f[j + 1] << (dbase + 1);
            fm[j] |= right << (dbase + (a == 1 ? 1 : 2));
        }
    }
    const uint4 own = *reinterpret_cast<const uint4*>(G + rr * CW + cc0);
    const uint32_t ownw[4] = {own.x, own.y, own.z, own.w};

    __builtin_amdgcn_sched_barrier(0);
    // ---- heat and dousing from box sums B_k (fire field) and D_1, D_2 (dousing field):
    //   heat = sum_k n_k*w_k = sum_{k=0..R} B_k * dw_k   (dw_k = w_k - w_{k+1}, w_{R+1} = 0: p.heat_dw)
    //   dous = inner*D_1 + border*(D_2 - D_1) = (inner - border)*D_1 + border*D_2
    // Fixed evaluation order, every op separately rounded: bit-identical with the C oracle.
    float ph[16], dz[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        ph[i] = 0.0f;
        dz[i] = 0.0f;
    }
    const float w_in_minus_bd = __fsub_rn(p.dous_inner, p.dous_border);
#pragma unroll
    for (int k = 0; k <= RS; ++k) {
        uint32_t V[16 + 2 * RS];
        const uint32_t* top = CP + (rr - k) * CW + cc0 - k;
        const uint32_t* bot = CP + (rr + k + 1) * CW + cc0 - k;
#pragma unroll
        for (int j = 0; j < 16 + 2 * RS; ++j)
            if (j < 16 + 2 * k) V[j] = bot[j] - top[j];
        uint32_t s = 0u;
#pragma unroll
        for (int j = 0; j <= 2 * RS; ++j)
            if (j <= 2 * k) s += V[j];
        const float wk = k <= R ? p.heat_dw[k] : 0.0f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (i > 0) s += V[i + 2 * k] - V[i - 1];
            if (k <= R) ph[i] = __fadd_rn(ph[i], __fmul_rn(wk, (float)(s & 0xFFFFu)));
            if (k == 1) dz[i] = __fmul_rn(w_in_minus_bd, (float)(s >> 16));
            if (k == 2) dz[i] = __fadd_rn(dz[i], __fmul_rn(p.dous_border, (float)(s >> 16)));
        }
        // materialise this radius' partial sums now: without it hipcc keeps all (R+1)x16 window
        // sums live and evaluates the f32 chains at the end (-> spills at R >= 4)
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(ph[i]), "+v"(dz[i]));
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) ph[i] = __fsub_rn(ph[i], dz[i]);  // p_h = heat - dousing (:198)

    const int widx = wind_index[e];
    float wind[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) wind[d] = p.winds[widx][d < 4 ? d : d + 1];
    const uint32_t step = rng_step ? rng_step[e] : 0u;
    const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
    const uint32_t env_id = (uint32_t)(p.env_offset + e);
    const bool want_prob = prob_out != nullptr;

    uint32_t outw[4] = {0u, 0u, 0u, 0u}, nagew[8];
    int cntT = 0, cntF = 0, cntE = 0;
    const float* ps_base = p_slope + ((int64_t)e * 8 * H + r) * W + cbase;  // + d*HW

#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
        float ps[8][4];
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            const float* src = ps_base + (int64_t)d * HW + 4 * g4;
            if (vec) {
                const float4 v = *reinterpret_cast<const float4*>(src);
                ps[d][0] = v.x; ps[d][1] = v.y; ps[d][2] = v.z; ps[d][3] = v.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) ps[d][j] = (row_ok && cbase + 4 * g4 + j < W) ? src[j] : 0.0f;
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = 4 * g4 + j;
            const bool ok = row_ok && cbase + i < W;
            const int x = (int)((ownw[g4] >> (8 * j)) & 0xFFu);
            const uint32_t nbm = (fm[g4] >> (8 * j)) & 0xFFu;
            const int age = (int)(int16_t)(agew[i >> 1] >> (16 * (i & 1)));
            // lookups with clip(idx, 1, 5) (:176-178) as select chains (no per-lane indexing)
            const int vv = (int)((vgw[g4] >> (8 * j)) & 0xFFu), dd = (int)((dnw[g4] >> (8 * j)) & 0xFFu);
            const float av = vv <= 1 ? p.veg1p[1] : vv == 2 ? p.veg1p[2] : vv == 3 ? p.veg1p[3] : vv == 4 ? p.veg1p[4] : p.veg1p[5];
            const float ad = dd <= 1 ? p.den1p[1] : dd == 2 ? p.den1p[2] : dd == 3 ? p.den1p[3] : dd == 4 ? p.den1p[4] : p.den1p[5];
            // p = p_h * (1 + p_veg) * (1 + p_den) * wind * p_slope, left to right (:206)
            const float base = __fmul_rn(__fmul_rn(ph[i], av), ad);
            if (want_prob && ok) {
                float* po = prob_out + (rowoff + i) * 8;
#pragma unroll
                for (int d = 0; d < 8; ++d) po[d] = __fmul_rn(__fmul_rn(base, wind[d]), ps[d][j]);
            }
            const bool is_tree = x == p.tree, is_empty = x == p.empty, is_fire = x == p.fire;
            bool burn = false, grow = false;
            int new_age_draw = p.age_lo;
            if (INJECT) {
                if (ok && is_tree && nbm) {
                    const float* u = inj_burn + (rowoff + i) * 9;
#pragma unroll
                    for (int d = 0; d < 8; ++d) {
                        const float pd = __fmul_rn(__fmul_rn(base, wind[d]), ps[d][j]);
                        if (((nbm >> d) & 1u) && u[d < 4 ? d : d + 1] < pd) burn = true;
                    }
                    if (burn) new_age_draw = inj_age[rowoff + i];
                }
                if (ok && is_empty) grow = inj_grow[rowoff + i] < p.p_tree;
            } else {
                const bool need = ok && ((is_tree && nbm) || (is_empty && p.p_tree > 0.0f));
                if (need) {
                    const u32x4 rx =
                        philox4x32_10(u32x4{(uint32_t)(r * W + cbase + i), env_id, step, GCA_TAG_ALEX_CELL}, k0, k1);
                    if (is_tree) {
                        float qn = 1.0f;
#pragma unroll
                        for (int d = 0; d < 8; ++d) {
                            const float pd = __fmul_rn(__fmul_rn(base, wind[d]), ps[d][j]);
                            if ((nbm >> d) & 1u) qn = __fmul_rn(qn, __fsub_rn(1.0f, clamp01(pd)));
                        }
                        burn = u01_f32(rx.x) < __fsub_rn(1.0f, qn);
                        new_age_draw = randint_ms(rx.z, p.age_lo, p.age_hi);
                    } else {
                        grow = u01_f32(rx.y) < p.p_tree;
                    }
                }
            }
            int nx = x;
            if (is_tree && burn) nx = p.fire;
            else if (is_empty && grow) nx = p.tree;
            else if (is_fire && age <= 1) nx = p.empty;
            int na = (nx == p.fire && !is_fire) ? new_age_draw : age;
            if (is_fire) na -= 1;
            if (i & 1) nagew[i >> 1] |= (uint32_t)(uint16_t)na << 16;
            else nagew[i >> 1] = (uint32_t)(uint16_t)na;
            outw[g4] |= (uint32_t)(nx & 0xFF) << (8 * j);
            if (ok) {
                cntT += nx == p.tree;
                cntF += nx == p.fire;
                cntE += nx == p.empty;
            }
        }    __builtin_amdgcn_sched_barrier(0);  // one group of 4 cells (8 x 16-B p_slope loads) in flight at a time
    }

    // ---------------- stores
    if (vec) {
        *reinterpret_cast<uint4*>(grid_out + rowoff) = make_uint4(outw[0], outw[1], outw[2], outw[3]);
        *reinterpret_cast<uint4*>(age_out + rowoff) = make_uint4(nagew[0], nagew[1], nagew[2], nagew[3]);
        *reinterpret_cast<uint4*>(age_out + rowoff + 8) = make_uint4(nagew[4], nagew[5], nagew[6], nagew[7]);
    } else if (row_ok) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (cbase + i < W) {
                grid_out[rowoff + i] = (uint8_t)(outw[i >> 2] >> (8 * (i & 3)));
                age_out[rowoff + i] = (int16_t)(nagew[i >> 1] >> (16 * (i & 1)));
            }
        }
    }
    if (counts) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            cntT += __shfl_xor(cntT, off);
            cntF += __shfl_xor(cntF, off);
            cntE += __shfl_xor(cntE, off);
        }
        if ((tid & 63) == 0) {
            if (cntE) atomicAdd(counts + 3 * e + 0, cntE);
            if (cntT) atomicAdd(counts + 3 * e + 1, cntT);
            if (cntF) atomicAdd(counts + 3 * e + 2, cntF);
        }
    }
}

// p_slope[e][d][r][c] = exp_f32(0.078f * slope[e][r][c][d'])
__global__ void alex_prepare_slope_kernel(const float* __restrict__ slope, float* __restrict__ p_slope, int64_t HW,
                                          int E) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= HW * E) return;
    const int e = (int)(idx / HW);
    const int64_t cell = idx - (int64_t)e * HW;
    const float* s = slope + idx * 9;
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        const float a = __fmul_rn(0.078f, s[d < 4 ? d : d + 1]);
        p_slope[((int64_t)e * 8 + d) * HW + cell] = exp_f32(a);
    }
}

template <int R, bool INJ>
void launch_alex(const gca_alex_params& p, int E, int H, int W, const uint8_t* gi, uint8_t* go, const int16_t* ai,
                 int16_t* ao, const uint8_t* veg, const uint8_t* den, const uint8_t* dous, const float* ps,
                 const int32_t* wi, const uint32_t* rs, const float* ib, const float* ig, const int32_t* ia, float* po,
                 int32_t* counts, hipStream_t st) {
    const int tiles_r = (H + TH - 1) / TH, tiles_c = (W + TW - 1) / TW;
    constexpr int RS = R < 2 ? 2 : R;
    constexpr int RR = TH + 2 * RS;
    const size_t lds = sizeof(uint32_t) * (RR + 1) * CW + (size_t)RR * CW;
    hipLaunchKernelGGL((alex_step_kernel<R, INJ>), dim3((unsigned)((int64_t)E * tiles_r * tiles_c)), dim3(256), lds, st,
                       p, H, W, tiles_r, tiles_c, gi, go, ai, ao, veg, den, dous, ps, wi, rs, ib, ig, ia, po, counts);
}

template <bool INJ>
void dispatch_r(int R, const gca_alex_params& p, int E, int H, int W, const uint8_t* gi, uint8_t* go, const int16_t* ai,
                int16_t* ao, const uint8_t* veg, const uint8_t* den, const uint8_t* dous, const float* ps,
                const int32_t* wi, const uint32_t* rs, const float* ib, const float* ig, const int32_t* ia, float* po,
                int32_t* counts, hipStream_t st) {
#define GCA_ALEX_CASE(RV) \
    case RV: launch_alex<RV, INJ>(p, E, H, W, gi, go, ai, ao, veg, den, dous, ps, wi, rs, ib, ig, ia, po, counts, st); break;
    switch (R) {
        GCA_ALEX_CASE(1) GCA_ALEX_CASE(2) GCA_ALEX_CASE(3) GCA_ALEX_CASE(4)
        GCA_ALEX_CASE(5) GCA_ALEX_CASE(6) GCA_ALEX_CASE(7) GCA_ALEX_CASE(8)
    }
#undef GCA_ALEX_CASE
}

}  // namespace

extern "C" int gca_alex_prepare_slope(const float* slope, float* p_slope, int E, int H, int W, void* stream) {
    GCA_CHECK_ARG(slope && p_slope && E > 0 && H > 0 && W > 0, "prepare_slope: bad arguments");
    const int64_t n = (int64_t)E * H * W;
    hipLaunchKernelGGL(alex_prepare_slope_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       slope, p_slope, (int64_t)H * W, E);
    GCA_CHECK_LAUNCH("alex_prepare_slope");
    return GCA_OK;
}

extern "C" int gca_alex_step(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                             const int16_t* age_in, int16_t* age_out, const uint8_t* veg, const uint8_t* den,
                             const uint8_t* dousing, const float* p_slope, const int32_t* wind_index,
                             const uint32_t* rng_step, const float* inj_burn, const float* inj_grow,
                             const int32_t* inj_age, float* prob_out, int32_t* counts, void* stream) {
    GCA_CHECK_ARG(p && grid_in && grid_out && age_in && age_out && veg && den && dousing && p_slope && wind_index,
                  "alex_step: null argument");
    GCA_CHECK_ARG(E > 0 && H > 0 && W > 0, "alex_step: sizes must be positive");
    GCA_CHECK_ARG(p->R >= 1 && p->R <= GCA_MAX_RADIUS, "alex_step: burn radius must be in [1, 8] (N in [5, 1024])");
    GCA_CHECK_ARG(p->n_winds >= 1 && p->n_winds <= 16, "alex_step: 1..16 wind matrices");
    GCA_CHECK_ARG(grid_in != grid_out && age_in != age_out, "alex_step: in-place update is not supported");
    const bool inj = inj_burn || inj_grow || inj_age;
    GCA_CHECK_ARG(!inj || (inj_burn && inj_grow && inj_age), "alex_step: injected mode needs all three draw arrays");
    GCA_CHECK_ARG(((uintptr_t)age_in & 1u) == 0 && ((uintptr_t)age_out & 1u) == 0, "alex_step: age arrays misaligned");
    hipStream_t st = (hipStream_t)stream;
    if (counts && hipMemsetAsync(counts, 0, sizeof(int32_t) * 3 * (size_t)E, st) != hipSuccess) {
        gca_set_error("alex_step: counts memset failed");
        return GCA_ERR_HIP;
    }
    if (inj)
        dispatch_r<true>(p->R, *p, E, H, W, grid_in, grid_out, age_in, age_out, veg, den, dousing, p_slope, wind_index,
                         rng_step, inj_burn, inj_grow, inj_age, prob_out, counts, st);
    else
        dispatch_r<false>(p->R, *p, E, H, W, grid_in, grid_out, age_in, age_out, veg, den, dousing, p_slope, wind_index,
                          rng_step, nullptr, nullptr, nullptr, prob_out, counts, st);
    GCA_CHECK_LAUNCH("alex_step");
    return GCA_OK;
}

// ------------------------------------------------------------------ slope from altitude
// get_slope (init_utils.py:166-200) on the device, then p_slope = exp_f32(0.078f * f32(slope)):
// slope[r,c,i,j] = degrees(atan((alt[r,c] - alt[r+i-1,c+j-1]) / (1.414 if diagonal))) in f64
// for interior cells (border cells and the centre are 0); the f32 cast follows jnp.array
// (advanced_bulldozer.py:204). altitude == NULL means altitude 0 (slope 0 everywhere).
namespace {
__global__ void alex_slope_from_altitude_kernel(const double* __restrict__ alt, float* __restrict__ p_slope,
                                                float* __restrict__ slope_out, int H, int W, int E) {
    const int64_t HW = (int64_t)H * W;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= HW * E) return;
    const int e = (int)(idx / HW);
    const int64_t cell = idx - (int64_t)e * HW;
    const int r = (int)(cell / W), c = (int)(cell - (int64_t)r * W);
    const bool interior = alt && r >= 1 && r < H - 1 && c >= 1 && c < W - 1;
    const double* a = alt ? alt + (int64_t)e * HW : nullptr;
    int d = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            float s = 0.0f;
            if (interior && !(i == 1 && j == 1)) {
                double diff = a[cell] - a[(int64_t)(r + i - 1) * W + (c + j - 1)];
                if (i != 1 && j != 1) diff /= 1.414;
                s = (float)(atan(diff) * (180.0 / 3.14159265358979323846));
            }
            if (slope_out) slope_out[idx * 9 + 3 * i + j] = s;
            if (i == 1 && j == 1) continue;
            p_slope[((int64_t)e * 8 + d) * HW + cell] = exp_f32(__fmul_rn(0.078f, s));
            ++d;
        }
    }
}
}  // namespace

extern "C" int gca_alex_slope_from_altitude(const double* altitude, float* p_slope, float* slope_out, int E, int H,
                                            int W, void* stream) {
    GCA_CHECK_ARG(p_slope && E > 0 && H > 0 && W > 0, "slope_from_altitude: bad arguments");
    const int64_t n = (int64_t)E * H * W;
    hipLaunchKernelGGL(alex_slope_from_altitude_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, altitude, p_slope, slope_out, H, W, E);
    GCA_CHECK_LAUNCH("alex_slope_from_altitude");
    return GCA_OK;
}
