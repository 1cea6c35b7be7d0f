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
// LDS row layout of the column prefix: one pad dword after every 16 columns (column c at
// c + c/16) and a row stride = 16 (mod 32) dwords, so the 64 lanes of a heat-window read
// (4 rows x 16 lanes, 16 columns apart) hit 64 distinct banks of a ds_read_b32 lane group.
constexpr int CWP = 336;
__host__ __device__ constexpr int pcol(int c) { return c + (c >> 4); }
static_assert(pcol(CW - 1) < CWP && CWP % 32 == 16, "padded row");

__device__ __forceinline__ float clamp01(float v) { return fminf(fmaxf(v, 0.0f), 1.0f); }

// MODE: 0 = Philox draws (production), 1 = Philox + debug burn probabilities, 2 = injected draws
// (+ probabilities when prob_out != NULL). The debug store is compiled out of mode 0.
template <int R, int MODE>
__global__ __launch_bounds__(256, 4) void alex_step_kernel(
    gca_alex_params p, int H, int W, int tiles_r, int tiles_c, const uint8_t* __restrict__ grid_in,
    uint8_t* __restrict__ grid_out, const int16_t* __restrict__ age_in, int16_t* __restrict__ age_out,
    const uint8_t* __restrict__ veg, const uint8_t* __restrict__ den, const uint8_t* __restrict__ dousing,
    const float* __restrict__ p_slope, const int32_t* __restrict__ wind_index, const uint32_t* __restrict__ rng_step,
    const float* __restrict__ inj_burn, const float* __restrict__ inj_grow, const int32_t* __restrict__ inj_age,
    float* __restrict__ prob_out, int32_t* __restrict__ counts) {
    constexpr bool INJECT = MODE == 2;
    constexpr bool PROB = MODE != 0;
    constexpr int RS = R < 2 ? 2 : R;  // staged halo: heat radius, at least the 5x5 dousing box
    constexpr int RR = TH + 2 * RS;    // staged rows
    constexpr int NCH = CW / 16;       // 16-column chunks per staged row
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* CP = reinterpret_cast<uint32_t*>(smem);                             // [RR+1][CWP] column prefix
    uint16_t* FB = reinterpret_cast<uint16_t*>(smem + sizeof(uint32_t) * (RR + 1) * CWP);  // [RR][NCH] fire bits

    // XCD-aware order: blocks b, b+8, b+16, ... share an XCD (and its L2) under round-robin
    // dispatch; give each XCD a contiguous range of (env, tile) so the halo rows a tile stages
    // were just fetched into the same L2 by its neighbour tile. Bijective for any grid size.
    const int tiles = tiles_r * tiles_c;
    const int nb = (int)gridDim.x;
    const int xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
    const int qn8 = nb >> 3, rn8 = nb & 7;
    const int lb = (xcd < rn8 ? xcd * (qn8 + 1) : rn8 * (qn8 + 1) + (xcd - rn8) * qn8) + slot;
    const int e = lb / tiles;
    const int tile = lb - e * tiles;
    const int r0 = (tile / tiles_c) * TH, c0 = (tile % tiles_c) * TW;
    const int64_t HW = (int64_t)H * W;
    const uint8_t* gE = grid_in + (int64_t)e * HW;
    const uint8_t* dE = dousing + (int64_t)e * HW;
    const int tid = threadIdx.x;
    const bool rows16 = ((W & 15) == 0) &&
                        ((((uintptr_t)grid_in) | ((uintptr_t)dousing) | ((uintptr_t)grid_out) | ((uintptr_t)veg) |
                          ((uintptr_t)den) | ((uintptr_t)age_in) | ((uintptr_t)age_out) | ((uintptr_t)p_slope)) &
                         15u) == 0;
    const uint32_t Fp = rep4((uint32_t)p.fire), Ep = rep4((uint32_t)p.empty);

    // ---------------- this thread's 16 cells: row r, columns [cbase, cbase+16)
    const int tr = tid >> 4, q = tid & 15;
    const int r = r0 + tr;
    const int cbase = c0 + 16 * q;
    const bool row_ok = r < H;
    const int rr = RS + tr;  // staged row of r
    // global addressing: wave-uniform per-env base pointers (SGPRs) + 32-bit lane offsets,
    // so no 64-bit address VGPRs stay live across the kernel
    const uint32_t lo = (uint32_t)(r * W + cbase);  // cell offset of cell 0 within the env
    const uint8_t* gEi = grid_in + (size_t)e * HW;
    const int16_t* aEi = age_in + (size_t)e * HW;
    const uint8_t* vE = veg + (size_t)e * HW;
    const uint8_t* nE = den + (size_t)e * HW;
    const int64_t rowoff = (int64_t)e * HW + lo;  // debug / injected arrays only
    const bool vec = row_ok && rows16 && (cbase + 16 <= W);

    // per-cell inputs, issued before the LDS phases so their latency overlaps them
    // (fire ages are loaded later, after the direction pass, to keep them out of its VGPR peak)
    uint32_t own[4], vgw[4], dnw[4];
    if (vec) {
        const uint4 g4 = *reinterpret_cast<const uint4*>(gEi + lo);
        const uint4 v4 = *reinterpret_cast<const uint4*>(vE + lo);
        const uint4 d4 = *reinterpret_cast<const uint4*>(nE + lo);
        own[0] = g4.x; own[1] = g4.y; own[2] = g4.z; own[3] = g4.w;
        vgw[0] = v4.x; vgw[1] = v4.y; vgw[2] = v4.z; vgw[3] = v4.w;
        dnw[0] = d4.x; dnw[1] = d4.y; dnw[2] = d4.z; dnw[3] = d4.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            vgw[k] = dnw[k] = 0x01010101u;
            own[k] = Ep;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (row_ok && cbase + i < W) {
                const uint32_t sh = 8 * (i & 3);
                vgw[i >> 2] = (vgw[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)vE[lo + i] << sh);
                dnw[i >> 2] = (dnw[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)nE[lo + i] << sh);
                own[i >> 2] = (own[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)gEi[lo + i] << sh);
            }
        }
    }

    // ---------------- stage rows [r0-RS, r0+TH+RS) x cols [c0-16, c0+TW+16):
    //                  packed fire | dousing<<16 -> CP rows 1..RR, fire bitmask -> FB
    for (int ch = tid; ch < RR * NCH; ch += 256) {
        const int sr = ch / NCH, cq = ch - sr * NCH;
        const int gr = r0 - RS + sr, gc = c0 - 16 + 16 * cq;
        uint32_t gw[4] = {Ep, Ep, Ep, Ep}, dw[4] = {0u, 0u, 0u, 0u};
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
        uint32_t* cp = CP + (sr + 1) * CWP + 17 * cq;  // = pcol(16 * cq)
        uint32_t bits = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t f = bytes_eq01(gw[j], Fp);
            bits |= ((f & 1u) | ((f >> 7) & 2u) | ((f >> 14) & 4u) | ((f >> 21) & 8u)) << (4 * j);
            cp[4 * j + 0] = (f & 1u) | ((dw[j] & 0xFFu) << 16);
            cp[4 * j + 1] = ((f >> 8) & 1u) | (((dw[j] >> 8) & 0xFFu) << 16);
            cp[4 * j + 2] = ((f >> 16) & 1u) | (((dw[j] >> 16) & 0xFFu) << 16);
            cp[4 * j + 3] = ((f >> 24) & 1u) | (((dw[j] >> 24) & 0xFFu) << 16);
        }
        FB[sr * NCH + cq] = (uint16_t)bits;
    }
    for (int cc = tid; cc < CWP; cc += 256) CP[cc] = 0u;
    __syncthreads();
    // ---------------- column prefix: columns t and t + CW/2 per thread, every load before the adds
    if (tid < CW / 2) {
        const int pa = pcol(tid), pb = pcol(tid + CW / 2);
        uint32_t va[RR], vb[RR];
#pragma unroll
        for (int k = 0; k < RR; ++k) {
            va[k] = CP[(k + 1) * CWP + pa];
            vb[k] = CP[(k + 1) * CWP + pb];
        }
        uint32_t ra = 0u, rb = 0u;
#pragma unroll
        for (int k = 0; k < RR; ++k) {
            ra += va[k];
            rb += vb[k];
            CP[(k + 1) * CWP + pa] = ra;
            CP[(k + 1) * CWP + pb] = rb;
        }
    }
    __syncthreads();

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
        const uint32_t* top = CP + (rr - k) * CWP + 17 * (q + 1);  // = pcol(cc0)
        const uint32_t* bot = CP + (rr + k + 1) * CWP + 17 * (q + 1);
#pragma unroll
        for (int j = 0; j < 16 + 2 * RS; ++j) {
            if (j < 16 + 2 * k) {
                const int t = j - k;                        // column cc0 + t, t in [-k, 16 + k)
                const int off = t + (t >= 16 ? 1 : 0) - (t < 0 ? 1 : 0);  // pcol(cc0 + t) - pcol(cc0)
                V[j] = bot[off] - top[off];
            }
            if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // <= 16 LDS reads in flight (VGPR budget)
        }
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

    // ---- FIRE bits of rows r-1, r, r+1: bit j of nbw[a] <-> staged column cc0 - 1 + j (j = 0..17)
    uint32_t nbw[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const uint16_t* fb = FB + (rr - 1 + a) * NCH + q;
        nbw[a] = ((uint32_t)fb[0] >> 15) | ((uint32_t)fb[1] << 1) | (((uint32_t)fb[2] & 1u) << 17);
    }
    asm volatile("" : "+v"(nbw[0]), "+v"(nbw[1]), "+v"(nbw[2]));  // build the 3 words now (no 9 live halfwords)

    const int widx = wind_index[e];
    float wind[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) wind[d] = p.winds[widx][d < 4 ? d : d + 1];
    const uint32_t step = rng_step ? rng_step[e] : 0u;
    const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
    const uint32_t env_id = (uint32_t)(p.env_offset + e);
    const bool want_prob = PROB && prob_out != nullptr;
    const uint32_t lin0 = lo;  // cell index of cell 0 within the env

    // ---- base[i] = (p_h * (1 + p_veg)) * (1 + p_den)   (left-to-right product of :206)
    uint32_t treebits = 0u, emptybits = 0u, okbits = 0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int x = (int)((own[i >> 2] >> (8 * (i & 3))) & 0xFFu);
        treebits |= (uint32_t)(x == p.tree) << i;
        emptybits |= (uint32_t)(x == p.empty) << i;
        okbits |= (uint32_t)(row_ok && cbase + i < W) << i;
        // lookups with clip(idx, 1, 5) (:176-178) as select chains (no per-lane indexing)
        const int vv = (int)((vgw[i >> 2] >> (8 * (i & 3))) & 0xFFu), dd = (int)((dnw[i >> 2] >> (8 * (i & 3))) & 0xFFu);
        const float av = vv <= 1 ? p.veg1p[1] : vv == 2 ? p.veg1p[2] : vv == 3 ? p.veg1p[3] : vv == 4 ? p.veg1p[4] : p.veg1p[5];
        const float ad = dd <= 1 ? p.den1p[1] : dd == 2 ? p.den1p[2] : dd == 3 ? p.den1p[3] : dd == 4 ? p.den1p[4] : p.den1p[5];
        ph[i] = __fmul_rn(__fmul_rn(ph[i], av), ad);  // ph now holds base
    }
    // burning-neighbour mask of direction d for all 16 cells: bit i <-> cell i
    // d = (a, b) row-major without the centre; entry (a, b) = cell (r + a - 1, c + b - 1) (:332-337)
    auto dir_bits = [&](int d) -> uint32_t {
        const int a = d < 3 ? 0 : (d < 5 ? 1 : 2);
        const int b = d < 3 ? d : (d == 3 ? 0 : (d == 4 ? 2 : d - 5));
        return (nbw[a] >> b) & 0xFFFFu;
    };
    uint32_t anyfire = 0u;
#pragma unroll
    for (int d = 0; d < 8; ++d) anyfire |= dir_bits(d);

    // ---- direction-outer pass: each p_slope row segment (16 floats = 64 B per lane, 1 KiB per
    //      16 lanes) is read in one burst, so every HBM line is consumed by one wave instruction group
    float qn[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) qn[i] = 1.0f;
    uint32_t burnbits = 0u;
    const float* psE = p_slope + (size_t)e * 8 * HW;  // wave-uniform
    auto load_ps = [&](int d, float4 (&v)[4]) {
        const float* src = psE + (uint32_t)(d * (uint32_t)HW) + lo;
        if (vec) {
#pragma unroll
            for (int m = 0; m < 4; ++m) v[m] = *reinterpret_cast<const float4*>(src + 4 * m);
        } else {
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                float t4[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) t4[j] = (row_ok && cbase + 4 * m + j < W) ? src[4 * m + j] : 0.0f;
                v[m] = make_float4(t4[0], t4[1], t4[2], t4[3]);
            }
        }
    };
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        float4 psc[4];
        load_ps(d, psc);
        const uint32_t fb = dir_bits(d) & treebits & okbits;
        const float wd = wind[d];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float4 v4 = psc[i >> 2];
            const float ps = (i & 3) == 0 ? v4.x : (i & 3) == 1 ? v4.y : (i & 3) == 2 ? v4.z : v4.w;
            const float pd = __fmul_rn(__fmul_rn(ph[i], wd), ps);
            if (PROB && want_prob && ((okbits >> i) & 1u)) prob_out[(rowoff + i) * 8 + d] = pd;
            const bool f = (fb >> i) & 1u;
            if (INJECT) {
                if (f && inj_burn[(rowoff + i) * 9 + (d < 4 ? d : d + 1)] < pd) burnbits |= 1u << i;
            } else {
                qn[i] = f ? __fmul_rn(qn[i], __fsub_rn(1.0f, clamp01(pd))) : qn[i];
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // one direction's 64 B per lane in flight at a time
    }

    uint32_t agew[8];
    if (vec) {
        const uint4 a0 = *reinterpret_cast<const uint4*>(aEi + lo);
        const uint4 a1 = *reinterpret_cast<const uint4*>(aEi + lo + 8);
        agew[0] = a0.x; agew[1] = a0.y; agew[2] = a0.z; agew[3] = a0.w;
        agew[4] = a1.x; agew[5] = a1.y; agew[6] = a1.z; agew[7] = a1.w;
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) agew[k] = 0u;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (row_ok && cbase + i < W) agew[i >> 1] |= (uint32_t)(uint16_t)aEi[lo + i] << (16 * (i & 1));
    }

    // ---- draws and the rule, two cells (one Philox block) at a time
    uint32_t outw[4] = {0u, 0u, 0u, 0u}, nagew[8];
    int cntT = 0, cntF = 0, cntE = 0;
#pragma unroll
    for (int pp = 0; pp < 8; ++pp) {
        bool burn[2] = {false, false}, grow[2] = {false, false}, need[2];
        int new_age[2] = {p.age_lo, p.age_lo};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = 2 * pp + h;
            const bool ok = (okbits >> i) & 1u, is_tree = (treebits >> i) & 1u, is_empty = (emptybits >> i) & 1u;
            const bool nb = (anyfire >> i) & 1u;
            if (INJECT) {
                need[h] = false;
                burn[h] = (burnbits >> i) & 1u;
                if (burn[h]) new_age[h] = inj_age[rowoff + i];
                if (ok && is_empty) grow[h] = inj_grow[rowoff + i] < p.p_tree;
            } else {
                need[h] = ok && ((is_tree && nb) || (is_empty && p.p_tree > 0.0f));
            }
        }
        if (!INJECT) {
            // Philox block for cell index pair lin>>1; word pair (2h, 2h+1) for h = lin & 1
            const uint32_t linA = lin0 + (uint32_t)(2 * pp);
            const uint32_t cA = linA >> 1, cB = (linA + 1u) >> 1;
            u32x4 XA = u32x4{0u, 0u, 0u, 0u}, XB;
            if (need[0] || (need[1] && cA == cB))
                XA = philox4x32_10(u32x4{cA, env_id, step, GCA_TAG_ALEX_CELL}, k0, k1);
            XB = XA;
            if (need[1] && cA != cB) XB = philox4x32_10(u32x4{cB, env_id, step, GCA_TAG_ALEX_CELL}, k0, k1);
            const bool hA = linA & 1u, hB = (linA + 1u) & 1u;
            const uint32_t mains[2] = {hA ? XA.z : XA.x, hB ? XB.z : XB.x};
            const uint32_t auxs[2] = {hA ? XA.w : XA.y, hB ? XB.w : XB.y};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 2 * pp + h;
                if (need[h]) {
                    if ((treebits >> i) & 1u) {
                        burn[h] = u01_f32(mains[h]) < __fsub_rn(1.0f, qn[i]);
                        new_age[h] = randint_ms(auxs[h], p.age_lo, p.age_hi);
                    } else {
                        grow[h] = u01_f32(mains[h]) < p.p_tree;
                    }
                }
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = 2 * pp + h;
            const int x = (int)((own[i >> 2] >> (8 * (i & 3))) & 0xFFu);
            const int age = (int)(int16_t)(agew[i >> 1] >> (16 * (i & 1)));
            const bool is_tree = x == p.tree, is_empty = x == p.empty, is_fire = x == p.fire;
            int nx = x;
            if (is_tree && burn[h]) nx = p.fire;
            else if (is_empty && grow[h]) nx = p.tree;
            else if (is_fire && age <= 1) nx = p.empty;
            int na = (nx == p.fire && !is_fire) ? new_age[h] : age;
            if (is_fire) na -= 1;
            if (h) nagew[pp] |= (uint32_t)(uint16_t)na << 16;
            else nagew[pp] = (uint32_t)(uint16_t)na;
            outw[i >> 2] |= (uint32_t)(nx & 0xFF) << (8 * (i & 3));
            if ((okbits >> i) & 1u) {
                cntT += nx == p.tree;
                cntF += nx == p.fire;
                cntE += nx == p.empty;
            }
        }
    }

    // ---------------- stores
    if (vec) {
        uint8_t* gEo = grid_out + (size_t)e * HW;
        int16_t* aEo = age_out + (size_t)e * HW;
        *reinterpret_cast<uint4*>(gEo + lo) = make_uint4(outw[0], outw[1], outw[2], outw[3]);
        *reinterpret_cast<uint4*>(aEo + lo) = make_uint4(nagew[0], nagew[1], nagew[2], nagew[3]);
        *reinterpret_cast<uint4*>(aEo + lo + 8) = make_uint4(nagew[4], nagew[5], nagew[6], nagew[7]);
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

template <int R, int MODE>
void launch_alex(const gca_alex_params& p, int E, int H, int W, const uint8_t* gi, uint8_t* go, const int16_t* ai,
                 int16_t* ao, const uint8_t* veg, const uint8_t* den, const uint8_t* dous, const float* ps,
                 const int32_t* wi, const uint32_t* rs, const float* ib, const float* ig, const int32_t* ia, float* po,
                 int32_t* counts, hipStream_t st) {
    const int tiles_r = (H + TH - 1) / TH, tiles_c = (W + TW - 1) / TW;
    constexpr int RS = R < 2 ? 2 : R;
    constexpr int RR = TH + 2 * RS;
    const size_t lds = sizeof(uint32_t) * (RR + 1) * CWP + sizeof(uint16_t) * RR * (CW / 16);
    hipLaunchKernelGGL((alex_step_kernel<R, MODE>), dim3((unsigned)((int64_t)E * tiles_r * tiles_c)), dim3(256), lds, st,
                       p, H, W, tiles_r, tiles_c, gi, go, ai, ao, veg, den, dous, ps, wi, rs, ib, ig, ia, po, counts);
}

template <int MODE>
void dispatch_r(int R, const gca_alex_params& p, int E, int H, int W, const uint8_t* gi, uint8_t* go, const int16_t* ai,
                int16_t* ao, const uint8_t* veg, const uint8_t* den, const uint8_t* dous, const float* ps,
                const int32_t* wi, const uint32_t* rs, const float* ib, const float* ig, const int32_t* ia, float* po,
                int32_t* counts, hipStream_t st) {
#define GCA_ALEX_CASE(RV) \
    case RV: launch_alex<RV, MODE>(p, E, H, W, gi, go, ai, ao, veg, den, dous, ps, wi, rs, ib, ig, ia, po, counts, st); break;
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
        dispatch_r<2>(p->R, *p, E, H, W, grid_in, grid_out, age_in, age_out, veg, den, dousing, p_slope, wind_index,
                         rng_step, inj_burn, inj_grow, inj_age, prob_out, counts, st);
    else if (prob_out)
        dispatch_r<1>(p->R, *p, E, H, W, grid_in, grid_out, age_in, age_out, veg, den, dousing, p_slope, wind_index,
                      rng_step, nullptr, nullptr, nullptr, prob_out, counts, st);
    else
        dispatch_r<0>(p->R, *p, E, H, W, grid_in, grid_out, age_in, age_out, veg, den, dousing, p_slope, wind_index,
                      rng_step, nullptr, nullptr, nullptr, nullptr, counts, st);
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
