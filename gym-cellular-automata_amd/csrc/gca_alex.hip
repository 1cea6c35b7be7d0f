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
//   LDS: the grid rows [r0-R, r0+TH+R) x cols [c0-16, c0+TW+16) staged once as the
//   column prefix CP of packed v = fire | dousing<<16 (u32; v_perm_b32 builds each word) plus
//   a FIRE bitmask FB. Box sums B_k of radius k = sliding window over 16+2k columns of
//   (CP[row+k+1] - CP[row-k]); fire and dousing fields never interfere (box sums < 2^16).
//   heat = sum_k dw_k * B_k in f32 (fixed order, separately rounded, packed over cell pairs).
// Lane work: per-cell decisions are single compares; the state update, output bytes (v_perm),
//   ages (SWAR i16 pairs) and counts (popcount) are word-level operations on 16-bit cell masks.
// p_slope (78% of the bytes) streams through a depth-2 register pipeline: direction d+2 is in
//   flight while direction d+1 is consumed; direction 0 rides with the staging loads.
// Draws: INJECT = the reference's own uniform/randint arrays (exact rule);
//        Philox = one Philox4x32-10 block per cell pair: words (main, aux) per cell;
//        burn iff u(main) < 1 - prod_{fire d}(1 - clamp01(p_d)) (same law as independent draws),
//        grow iff u(main) < p_tree, new fire age = randint(aux).
#include "gca_alex_rule.h"

namespace {

// tile rows (r02n: 32-row tiles of 512 threads, two workgroups per CU, measured 1.82 vs 1.44 ms)
constexpr int TH = 16;
constexpr int NT = 16 * TH;  // threads per workgroup (16 lanes per image row)
constexpr int TW = 256;
constexpr int CW = TW + 32;  // staged columns: [c0-16, c0+TW+16)
// LDS row layout of the column prefix: rows of CWP dwords, one 16-dword chunk per 16 columns (16-B
// aligned: the heat phase reads a lane's 16 columns as 4 x ds_read_b128). Inside chunk q, the 4-column
// group g is stored at group slot (g + q/4) & 3, so the 16 chunks q = 1..16 of one g cover 64 distinct
// banks, and so do 64 consecutive columns read as b32 (prefix phase). A ds_read_b128 is serviced in lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... (MI355X_MICROARCH.md §LDS): each group mixes two image
// rows (tr, tr+1) of the wave, so the row pitch must be a multiple of 64 dwords for those 16 lanes to stay
// on 16 distinct q's: CWP = 320 (the unpadded 288 ≡ 32 mod 64 put lanes q and q' = q+-8 of adjacent rows
// on one bank: 2-way conflicts on every heat-phase read, 7.9e7 conflict cycles per launch in r01o).
constexpr int CWP = 320;
static_assert(CWP >= CW, "staged row fits");
__host__ __device__ constexpr int pcol(int c) { return 16 * (c >> 4) + 4 * ((((c >> 2) & 3) + (c >> 6)) & 3) + (c & 3); }
static_assert(CWP % 4 == 0, "16-B aligned rows");

typedef gca_f2 f2;
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef int16_t i16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float clamp01(float v) { return gca_clamp01(v); }
__device__ __forceinline__ f2 pk_mul_clamp01(f2 a, f2 b) { return gca_pk_mul_clamp01(a, b); }
// bits = 2 * bits + (a < b): v_cmp into VCC + add-with-carry (cell 0 lands in the top bit; reversed later)
__device__ __forceinline__ uint32_t push_lt(uint32_t bits, float a, float b) {
    asm("v_cmp_lt_f32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(bits) : "v"(a), "v"(b) : "vcc");
    return bits;
}
__device__ __forceinline__ uint32_t eq_nib(uint32_t x, uint32_t pat) { return gca_eq_nib(x, pat); }
__device__ __forceinline__ uint32_t spread4(uint32_t n) { return gca_spread4(n); }
__device__ __forceinline__ uint32_t bfi32(uint32_t m, uint32_t a, uint32_t b) { return gca_bfi32(m, a, b); }
__device__ __forceinline__ uint32_t sbit(uint32_t w, int i) { return gca_sbit(w, i); }
__device__ __forceinline__ f2 edge_factor_pair(float v0, float v1, bool own) { return gca_edge_factor_pair(v0, v1, own); }
// DPP moves inside a 16-lane row (= one image row of a workgroup: lanes q = 0..15)
__device__ __forceinline__ float dpp_from_next(float old, float src) {  // lane q <- lane q+1; lane 15 keeps old
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), 0x101, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_from_prev(float old, float src) {  // lane q <- lane q-1; lane 0 keeps old
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), 0x111, 0xF, 0xF, false));
}
template <class T, class S> __device__ __forceinline__ T bitcast_(S s) {
    static_assert(sizeof(T) == sizeof(S), "size");
    T t;
    __builtin_memcpy(&t, &s, sizeof(T));
    return t;
}

// MODE: 0 = Philox draws (production), 1 = Philox + debug burn probabilities, 2 = injected draws
// (+ probabilities when prob_out != NULL). The debug store is compiled out of mode 0.
//
// Lane work is organised around 16-bit cell masks (bit i <-> the lane's cell i) and packed f32 pairs:
// per-cell decisions are single compares; the state update, the output bytes, the ages and the counts
// are word-level bit operations (see the rule section). Every f32 op keeps the oracle's order and
// rounding (packed ops round each half like the scalar op; -ffp-contract=off).
// FAST: W % TW == 0, H % TH == 0, every array 16-B aligned (checked on the host): all per-lane bounds
// checks and byte-wise fallbacks compile away, which also lets the waitcnt pass keep loads in flight.
//
// ES (edge slopes): `p_slope` is the antisymmetric edge layout of gca_alex_edge_slope_from_altitude,
// es[e][k][r][c] = V = +-exp_f32(|a|), a = 0.078f * f32(raw slope of (r,c) toward neighbour k),
// k = 0..3 <-> (-1,-1), (-1,0), (-1,+1), (0,-1), sign = sign of a — 16 B per cell instead of 32.
// get_slope's f64 difference, division, atan and degree scaling are odd, and so are the f32 cast and
// the 0.078f product, so the neighbour sees exactly -a. With p_slope = slope_factor(a) (gca_common.h:
// exp_f32(a) for a >= 0, 1 / exp_f32(-a) otherwise), direction d < 4 of cell X is P(a) = V > 0 ? V :
// 1/|V| and direction d >= 4 is P(-a) of the neighbour X + off_d's edge: |V| if V < 0, else 1/|V|;
// 1/x is recip_ge1 (v_rcp_f32 + one Newton step, correctly rounded on [1, 1121], tested exhaustively).
// Cells on the grid border get p_slope = 1 (get_slope leaves their slopes 0).
// Bit-identical to the 8-plane layout built from the same altitude (tests/test_gpu_edge_slope.py).
//
// Fire sparsity (MODE 0): p_slope, vegetation, density, the heat field and the per-direction products
// only matter for TREE cells with a burning neighbour. A workgroup with no FIRE within one cell of its tile
// skips the heat phase; a wave with no such TREE cell skips the direction pass and its loads (a real
// episode's fire front covers a few tiles of 256). Results are unchanged (the skipped values are unused).
//
// PK (packed env layout, ES + FAST + Philox mode only: gca_alex_step_packed): `veg` holds vd = min(veg, 7) |
// min(den, 7) << 4 (one byte per cell), `dousing` one bit per cell (a u16 per 16-column chunk, bit i = column
// 16j + i; the env's dousing counts are 0/1) and the edge slopes are stored coalesced: inside every 256-column
// row segment of a plane, column 16q + 4m + j sits at position 64m + 4q + j, so the 16 lanes of an image row
// read 256 contiguous bytes per load instruction. 23.125 B of HBM traffic per cell instead of 25.
constexpr int WGS = 4;  // workgroups per CU (launch bounds)
// Wave priorities (s_setprio) along a tile's phase chain: 3 while a tile issues its staging loads, 2 through the LDS
// writes and the column prefix (the phases in front of the workgroup's last barrier), 0 from the heat phase on, so the
// SIMD arbiter lets waves that hold up a barrier issue ahead of the barrier-free heat / slope / Philox work of the other
// workgroups. r02r (profiles/r02r): 1.405 vs 1.434 ms (-2.0 %) on the headline, +4 % on the sparse episode-start state;
// the slope-streaming pass at 2 above the heat phase measured +21 %. (r02h: two of the seven slope loads by LDS-DMA into
// the dead column prefix, four loads in flight per wave, measured 2 % slower and was removed.)
// bytes of the column-prefix region: (RR + 1) rows of CWP dwords
__host__ __device__ constexpr int cp_bytes(int RR, bool) { return 4 * (RR + 1) * CWP; }
// OBS colour table: after the column prefix, the fire bitmask and the 16-float LUT, 16-B aligned (6 float4)
__host__ __device__ constexpr int obs_col_off(int RR, bool pk) {
    return (cp_bytes(RR, pk) + 2 * RR * (TW + 32) / 16 + 64 + 15) & ~15;
}
// OBS (PK only): the step also writes the env's RGB observation of the plain case (no extension channel, no grid
// transform — advanced_bulldozer.py:1035-1101 with enable_extensions=False, the reference's default): every cell's
// colour is a function of its NEW state (grid_to_rgb of the post-step grid, :1120) and its PRE-step dousing bit and
// day / night (the MDP renders with the input per_env_context, :1121) — all of which this kernel holds — so the
// frame costs its 12 B/cell of writes and nothing else. The bulldozer's pixel (:1099) is written afterwards by
// gca_obs_position (the position is only known after the env step's Move).
struct AlexObs {
    const float4* col;       // [2 nights][3 kinds][2 dousing] colours (gca_obs_color_table)
    const int32_t* night;    // [E] pre-step is_night
    float* rgb;              // [E][H][W][3]
};


template <int R, int MODE, bool FAST, bool ES, bool PK = false, bool OBS = false>
__global__ __launch_bounds__(NT, WGS) void alex_step_kernel(
    gca_alex_params p, int H, int W, int tiles_r, int tiles_c, const uint8_t* __restrict__ grid_in,
    uint8_t* __restrict__ grid_out, const int16_t* age_in, int16_t* age_out,  // no __restrict__: PK updates in place
    const uint8_t* __restrict__ veg, const uint8_t* __restrict__ den, const uint8_t* __restrict__ dousing,
    const float* __restrict__ p_slope, const int32_t* __restrict__ wind_index, const uint32_t* __restrict__ rng_step,
    const float* __restrict__ inj_burn, const float* __restrict__ inj_grow, const int32_t* __restrict__ inj_age,
    float* __restrict__ prob_out, int32_t* __restrict__ counts, const uint8_t* __restrict__ act_in,
    uint8_t* __restrict__ act_out, AlexObs obs) {
    static_assert(!OBS || PK, "the fused observation runs on the packed env layout");
    constexpr bool INJECT = MODE == 2;
    constexpr bool PROB = MODE != 0;
    constexpr int RS = R < 2 ? 2 : R;  // staged halo: heat radius, at least the 5x5 dousing box
    constexpr int RR = TH + 2 * RS;    // staged rows
    constexpr int NCH = CW / 16;       // 16-column chunks per staged row
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* CP = reinterpret_cast<uint32_t*>(smem);                                        // [RR+1][CWP]
    constexpr int CPB = cp_bytes(RR, PK);                                                    // CP (+ GLDS slots)
    uint16_t* FB = reinterpret_cast<uint16_t*>(smem + CPB);                                  // [RR][NCH] fire bits
    float* LUT = reinterpret_cast<float*>(smem + CPB + sizeof(uint16_t) * RR * NCH);
    // LUT[0..7] = 1 + p_veg[clip(v, 1, 5)] for v = min(byte, 7); LUT[8..15] the same for density
    float4* COL = reinterpret_cast<float4*>(smem + obs_col_off(RR, PK));
    static_assert(!OBS || cp_bytes(RR, PK) >= 4 * 6144, "OBS: 6 KiB of dead column prefix per wave");  // OBS: the env's 6 colours (kind x dousing)

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
    const uint16_t* dbE = reinterpret_cast<const uint16_t*>(dousing) + (int64_t)e * (HW >> 4);  // PK: dousing bits
    static_assert(!PK || (ES && FAST && MODE == 0), "packed layout: edge slopes, FAST shape, Philox mode");
    const int tid = threadIdx.x;
    __builtin_amdgcn_s_setprio(3);  // issue this tile's loads ahead of other waves' compute
    const bool rows16 = FAST || (((W & 15) == 0) &&
                                 ((((uintptr_t)grid_in) | ((uintptr_t)dousing) | ((uintptr_t)grid_out) |
                                   ((uintptr_t)veg) | ((uintptr_t)den) | ((uintptr_t)age_in) | ((uintptr_t)age_out) |
                                   ((uintptr_t)p_slope)) & 15u) == 0);
    const uint32_t Fp = rep4((uint32_t)p.fire), Ep = rep4((uint32_t)p.empty), Tp = rep4((uint32_t)p.tree);

    // ---------------- this thread's 16 cells: row r, columns [cbase, cbase+16)
    const int tr = tid >> 4, q = tid & 15;
    const int r = r0 + tr;
    const int cbase = c0 + 16 * q;
    const bool row_ok = FAST || r < H;
    const int rr = RS + tr;  // staged row of r
    // global addressing: wave-uniform per-env base pointers (SGPRs) + 32-bit lane offsets,
    // so no 64-bit address VGPRs stay live across the kernel
    const uint32_t lo = (uint32_t)(r * W + cbase);  // cell offset of cell 0 within the env
    const uint8_t* gEi = grid_in + (size_t)e * HW;
    const int16_t* aEi = age_in + (size_t)e * HW;
    const uint8_t* vE = veg + (size_t)e * HW;
    const uint8_t* nE = den + (size_t)e * HW;
    const int64_t rowoff = (int64_t)e * HW + lo;  // debug / injected arrays only
    const bool vec = FAST || (row_ok && rows16 && (cbase + 16 <= W));
    const int nvalid = row_ok ? min(16, W - cbase) : 0;
    const uint32_t okB = FAST ? 0xFFFFu : nvalid >= 16 ? 0xFFFFu : (nvalid > 0 ? (1u << nvalid) - 1u : 0u);

    // per-cell inputs: the own cells now; vegetation / density once the wave knows it needs them
    // (fire ages are loaded later, after the direction pass, to keep them out of its VGPR peak)
    uint32_t own[4], vgw[4], dnw[4];
    if (vec) {
        const uint4 g4 = *reinterpret_cast<const uint4*>(gEi + lo);
        own[0] = g4.x; own[1] = g4.y; own[2] = g4.z; own[3] = g4.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) own[k] = Ep;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (row_ok && cbase + i < W) {
                const uint32_t sh = 8 * (i & 3);
                own[i >> 2] = (own[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)gEi[lo + i] << sh);
            }
        }
    }
    auto load_vd = [&]() {
        if (PK) {  // vd = veg | den << 4 (both already min(., 7))
            const uint4 v4 = *reinterpret_cast<const uint4*>(vE + lo);
            vgw[0] = v4.x & 0x0F0F0F0Fu; vgw[1] = v4.y & 0x0F0F0F0Fu; vgw[2] = v4.z & 0x0F0F0F0Fu; vgw[3] = v4.w & 0x0F0F0F0Fu;
            dnw[0] = (v4.x >> 4) & 0x0F0F0F0Fu; dnw[1] = (v4.y >> 4) & 0x0F0F0F0Fu;
            dnw[2] = (v4.z >> 4) & 0x0F0F0F0Fu; dnw[3] = (v4.w >> 4) & 0x0F0F0F0Fu;
        } else if (vec) {
            const uint4 v4 = *reinterpret_cast<const uint4*>(vE + lo);
            const uint4 d4 = *reinterpret_cast<const uint4*>(nE + lo);
            vgw[0] = v4.x; vgw[1] = v4.y; vgw[2] = v4.z; vgw[3] = v4.w;
            dnw[0] = d4.x; dnw[1] = d4.y; dnw[2] = d4.z; dnw[3] = d4.w;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) vgw[k] = dnw[k] = 0x01010101u;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (row_ok && cbase + i < W) {
                    const uint32_t sh = 8 * (i & 3);
                    vgw[i >> 2] = (vgw[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)vE[lo + i] << sh);
                    dnw[i >> 2] = (dnw[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)nE[lo + i] << sh);
                }
            }
        }
    };

    // ---- p_slope software pipeline (depth 2): the first load is issued before the heat phase,
    //      the second right after it, so their HBM latency overlaps the heat computation; load k+2 is
    //      issued as soon as load k is consumed. p_slope is the bulk of the kernel's bytes, so keeping
    //      two loads in flight per wave is what keeps HBM busy while the waves compute.
    //      8-plane layout: load k = plane k, row r.  Edge layout (ES): loads L0..L6 =
    //      (plane 0, r) (1, r) (2, r) (3, r) (2, r+1) (1, r+1) (0, r+1); direction d uses load
    //      LOAD_OF(d) = 0 1 2 3 3 4 5 6 (d = 3 and 4 share plane 3 of row r).
    constexpr int NPL = ES ? 4 : 8;
    const float* psE = p_slope + (size_t)e * NPL * HW;  // wave-uniform
    auto load_ps = [&](int k, float4 (&v)[4]) {
        const int plane = ES ? (k < 4 ? k : 6 - k) : k;
        // ES rows r+1 (k >= 4): row H-1 (a border row: every value killed) reads itself instead
        const int dr = (ES && k >= 4 && r + 1 < H) ? 1 : 0;
        const float* src = psE + (uint32_t)(plane * (uint32_t)HW) + lo + (uint32_t)(dr * W);
        if (vec) {
            // PK: coalesced segment order, lane q's columns 16q + 4m .. +3 at segment position 64m + 4q
#pragma unroll
            for (int m = 0; m < 4; ++m) v[m] = *reinterpret_cast<const float4*>(src + (PK ? 64 * m - 12 * q : 4 * m));
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
    float4 psbuf[2][4];
    uint32_t agew[8];
    auto load_ages = [&]() {
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
    };
    // ---- OBS epilogue: RGB f32 of the lane's 16 cells (tB / fB: new TREE / FIRE masks, bit i <-> cell i) through a
    //      per-wave transposition in the column-prefix LDS (dead after the heat phase: a workgroup barrier orders every
    //      wave's reads before the first write), two rounds of two image rows, so that every non-temporal store
    //      instruction writes 1 KiB of contiguous RGB (per-lane 192-B stores were 4x slower in gca_obs.hip, r01m)
    auto write_rgb = [&](uint32_t tB, uint32_t fB) {
        if constexpr (OBS) {
            if (tid < 6) {
                const int nt = obs.night[e] != 0 ? 1 : 0;
                COL[tid] = obs.col[6 * nt + tid];
            }
            const uint32_t dbits = dbE[lo >> 4];  // PRE-step dousing bits of this lane's 16 cells
            __syncthreads();
            const int lane = tid & 63, wv = tid >> 6;
            float4* img = reinterpret_cast<float4*>(smem) + wv * 384;  // 6 KiB per wave
            typedef float f4t __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if ((lane >> 5) == h) {  // lanes 32h .. 32h+31 hold this wave's image rows 2h, 2h+1
                    float4* dst = img + ((lane >> 4) & 1) * 192 + q * 12;
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        float c[12];
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int i = 4 * g + j;
                            const int kind = ((tB >> i) & 1u) ? 1 : (((fB >> i) & 1u) ? 2 : 0);
                            const float4 cl = COL[2 * kind + (int)((dbits >> i) & 1u)];
                            c[3 * j] = cl.x;
                            c[3 * j + 1] = cl.y;
                            c[3 * j + 2] = cl.z;
                        }
                        dst[3 * g] = make_float4(c[0], c[1], c[2], c[3]);
                        dst[3 * g + 1] = make_float4(c[4], c[5], c[6], c[7]);
                        dst[3 * g + 2] = make_float4(c[8], c[9], c[10], c[11]);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int jj = 0; jj < 6; ++jj) {
                    const int lr = jj / 3;  // image row of the round (3 x 1 KiB per 256-column row segment)
                    const int row = r0 + 4 * wv + 2 * h + lr;
                    float* gdst = obs.rgb + (((size_t)e * H + row) * W + c0) * 3 + 4 * (64 * (jj - 3 * lr) + lane);
                    const float4 v = img[64 * jj + lane];
                    __builtin_nontemporal_store((f4t){v.x, v.y, v.z, v.w}, reinterpret_cast<f4t*>(gdst));
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // this round's reads before the next writes
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    };
    // ---------------- stage rows [r0-RS, r0+TH+RS) x cols [c0-16, c0+TW+16):
    //                  packed fire | dousing<<16 -> CP rows 1..RR, fire bitmask -> FB
    //                  every load of the thread's chunks is issued before any is processed
    constexpr int NIT = (RR * NCH + NT - 1) / NT;
    uint32_t sgw[NIT][4], sdw[NIT][4];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int ch = tid + NT * it;
        const int sr = ch / NCH, cq = ch - sr * NCH;
        const int gr = r0 - RS + sr, gc = c0 - 16 + 16 * cq;
        uint32_t* gw = sgw[it];
        uint32_t* dw = sdw[it];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            gw[j] = Ep;
            dw[j] = 0u;
        }
        if (ch < RR * NCH && gr >= 0 && gr < H) {
            if (rows16 && gc >= 0 && gc + 16 <= W) {  // FAST: a chunk is entirely inside or outside
                const uint4 a = *reinterpret_cast<const uint4*>(gE + (int64_t)gr * W + gc);
                gw[0] = a.x; gw[1] = a.y; gw[2] = a.z; gw[3] = a.w;
                if (PK) {  // 16 dousing bits -> 0x01 bytes
                    const uint32_t b16 = dbE[((uint32_t)gr * (uint32_t)W + (uint32_t)gc) >> 4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) dw[j] = spread4(b16 >> (4 * j));
                } else {
                    const uint4 b = *reinterpret_cast<const uint4*>(dE + (int64_t)gr * W + gc);
                    dw[0] = b.x; dw[1] = b.y; dw[2] = b.z; dw[3] = b.w;
                }
            } else if (!FAST) {
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
    }
    // ---- tile activity map (PK, the env's path; act_in only with p_tree == 0, checked on the host): a tile with
    //      no FIRE in itself or its 8 neighbour tiles at the step's input cannot change — no tree has a burning
    //      neighbour, no fire ages, nothing grows — so it is copied instead of stepped: the grid (own cells, loaded
    //      above), and the ages only when they are not updated in place (the env's ages are). Checked here, after
    //      the staging loads are issued, so the flags' latency hides under them. act_out[tile] = any FIRE in the
    //      step's output tile: 0 here, set to 1 below by every wave that leaves a FIRE (ordered after this store
    //      by the workgroup barrier).
    if (PK && act_out) {
        const int tiles_all = tiles_r * tiles_c;
        if (act_in) {
            const int ti = tile / tiles_c, tj = tile - ti * tiles_c;
            const uint8_t* A = act_in + (size_t)e * tiles_all;
            int anyf = 0;
#pragma unroll
            for (int di = -1; di <= 1; ++di)
#pragma unroll
                for (int dj = -1; dj <= 1; ++dj) {
                    const int a = ti + di, b = tj + dj;
                    if (a >= 0 && a < tiles_r && b >= 0 && b < tiles_c) anyf |= A[a * tiles_c + b];
                }
            if (!anyf) {
                *reinterpret_cast<uint4*>(grid_out + (size_t)e * HW + lo) = make_uint4(own[0], own[1], own[2], own[3]);
                if (age_in != age_out) {
                    const uint4 a0 = *reinterpret_cast<const uint4*>(age_in + (size_t)e * HW + lo);
                    const uint4 a1 = *reinterpret_cast<const uint4*>(age_in + (size_t)e * HW + lo + 8);
                    *reinterpret_cast<uint4*>(age_out + (size_t)e * HW + lo) = a0;
                    *reinterpret_cast<uint4*>(age_out + (size_t)e * HW + lo + 8) = a1;
                }
                if (tid == 0) act_out[(size_t)e * tiles_all + tile] = 0;
                if (counts) {
                    int cE = 0, cT = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        cE += __builtin_popcount(bytes_eq01(own[j], Ep));
                        cT += __builtin_popcount(bytes_eq01(own[j], Tp));
                    }
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) {
                        cE += __shfl_xor(cE, off);
                        cT += __shfl_xor(cT, off);
                    }
                    if ((tid & 63) == 0) {
                        if (cE) atomicAdd(counts + 3 * e + 0, cE);
                        if (cT) atomicAdd(counts + 3 * e + 1, cT);
                    }
                }
                if constexpr (OBS) {  // the copied tile has no FIRE (it holds none and none reaches it)
                    uint32_t tB = 0u;
#pragma unroll
                    for (int j = 0; j < 4; ++j) tB |= eq_nib(own[j], Tp) << (4 * j);
                    write_rgb(tB, 0u);
                }
                return;  // the whole workgroup (anyf is workgroup-uniform)
            }
        }
        if (tid == 0) act_out[(size_t)e * tiles_all + tile] = 0;
    }
    __builtin_amdgcn_s_setprio(2);
    int near_fire = 0;  // a FIRE cell within one row of the tile (rows r0-1 .. r0+TH) in this thread's chunks
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int ch = tid + NT * it;
        if (ch >= RR * NCH) break;
        const int sr = ch / NCH, cq = ch - sr * NCH;
        uint32_t* cp = CP + (sr + 1) * CWP + 16 * cq;  // chunk cq; word j (columns 4j..4j+3) at slot (j + cq/4) & 3
        uint32_t bits = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t f = bytes_eq01(sgw[it][j], Fp);  // 0x01 in every FIRE byte
            bits |= ((f * 0x01020408u) >> 24) << (4 * j);
            // cell m of this word: (fire flag) | (dousing byte) << 16, one v_perm_b32 each; one ds_write_b128
            uint32_t w[4];
#pragma unroll
            for (int m = 0; m < 4; ++m)
                w[m] = __builtin_amdgcn_perm(sdw[it][j], f, 0x0C000C00u | ((4u + (uint32_t)m) << 16) | (uint32_t)m);
            *reinterpret_cast<uint4*>(cp + 4 * ((j + (cq >> 2)) & 3)) = make_uint4(w[0], w[1], w[2], w[3]);
        }
        FB[sr * NCH + cq] = (uint16_t)bits;
        near_fire |= (bits != 0u && sr >= RS - 1 && sr <= RS + TH) ? 1 : 0;
    }
    for (int cc = tid; cc < CWP; cc += NT) CP[cc] = 0u;
    if (tid < 16) LUT[tid] = gca_alex_lut_entry(p, tid);
    // MODE 0: does any TREE cell of this workgroup (wg_need) / this wave (wave_need) have a burning
    // neighbour? The other modes evaluate every probability.
    bool wg_need = true;
    if (MODE == 0)
        wg_need = __syncthreads_or(near_fire) != 0;
    else
        __syncthreads();
    uint32_t treeB = 0u, emptyB = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        treeB |= eq_nib(own[j], Tp) << (4 * j);
        emptyB |= eq_nib(own[j], Ep) << (4 * j);
    }
    // FIRE bits of rows r-1, r, r+1: bit j of nbw[a] <-> staged column cc0 - 1 + j (j = 0..17)
    auto fire_rows = [&](uint32_t (&nbw)[3]) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const uint16_t* fb = FB + (rr - 1 + a) * NCH + q;
            nbw[a] = ((uint32_t)fb[0] >> 15) | ((uint32_t)fb[1] << 1) | (((uint32_t)fb[2] & 1u) << 17);
        }
    };
    // burning-neighbour mask of direction d for all 16 cells: bit i <-> cell i
    // d = (a, b) row-major without the centre; entry (a, b) = cell (r + a - 1, c + b - 1) (:332-337)
    auto dir_bits_of = [](const uint32_t (&nbw)[3], int d) -> uint32_t {
        const int a = d < 3 ? 0 : (d < 5 ? 1 : 2);
        const int b = d < 3 ? d : (d == 3 ? 0 : (d == 4 ? 2 : d - 5));
        return (nbw[a] >> b) & 0xFFFFu;
    };
    bool wave_need = true;
    if (MODE == 0) {
        uint32_t anyf = 0u;
        if (wg_need) {
            uint32_t nb0[3];
            fire_rows(nb0);
#pragma unroll
            for (int d = 0; d < 8; ++d) anyf |= dir_bits_of(nb0, d);
        }
        wave_need = __ballot((treeB & anyf & okB) != 0u) != 0ull;
    }
    // ES: the three edge values a lane's shifted directions take from outside its row segment
    float e4 = 0.0f, e5 = 0.0f, e7 = 0.0f;
    if (wave_need) {
        load_vd();
        load_ps(0, psbuf[0]);  // first p_slope load: in flight during the prefix and heat phases
        if (ES) {
            const float* es = psE + lo;
            if (q == 15 && row_ok && cbase + 16 < W) {
                e4 = es[3 * (uint32_t)HW + 16];                              // es[3][r][cbase+16]
                if (r + 1 < H) e7 = es[(uint32_t)W + 16];                    // es[0][r+1][cbase+16]
            }
            if (q == 0 && row_ok && cbase >= 1 && r + 1 < H) e5 = es[2 * (uint32_t)HW + (uint32_t)W - 1];  // es[2][r+1][cbase-1]
        }
    }
    // ---------------- column prefix: columns t and t + CW/2 per thread, every load before the adds
    if constexpr (NT >= CW) {  // tall tiles: one column per thread
        if (wg_need && tid < CW) {
            const int pa = pcol(tid);
            uint32_t va[RR];
#pragma unroll
            for (int k = 0; k < RR; ++k) va[k] = CP[(k + 1) * CWP + pa];
            uint32_t ra = 0u;
#pragma unroll
            for (int k = 0; k < RR; ++k) {
                ra += va[k];
                CP[(k + 1) * CWP + pa] = ra;
            }
        }
    } else if (wg_need && tid < CW / 2) {
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
    __builtin_amdgcn_s_setprio(0);  // past the last barrier

    __builtin_amdgcn_sched_barrier(0);

    // ---- heat and dousing from box sums B_k (fire field) and D_1, D_2 (dousing field):
    //   heat = sum_k n_k*w_k = sum_{k=0..R} B_k * dw_k   (dw_k = w_k - w_{k+1}, w_{R+1} = 0: p.heat_dw)
    //   dous = inner*D_1 + border*(D_2 - D_1) = (inner - border)*D_1 + border*D_2
    // Fixed evaluation order: heat accumulates by fma (ph = fma(dw_k, B_k, ph)), dous = fma(border, D_2,
    // (inner - border) * D_1); bit-identical with the C oracle (fmaf).
    // Pairs of cells share one packed mul / add; B_k <= (2R+1)^2 <= 225 for R <= 7 -> v_cvt_f32_ubyte0.
    f2 ph2[8], dz2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        ph2[j] = (f2){p.heat0, p.heat0};  // 0 (JAX rule) or the classic constant p_h
        dz2[j] = (f2){0.0f, 0.0f};
    }
    const float w_in_minus_bd = __fsub_rn(p.dous_inner, p.dous_border);
    auto fire_f = [](uint32_t s) -> float { return R <= 7 ? (float)(s & 0xFFu) : (float)(s & 0xFFFFu); };
    if (wave_need) {
        // Window sums by lane-local prefix + DPP halo: lane q reads only its own 16 columns of the two
        // prefix rows (4 + 4 ds_read_b128), V = bottom - top; P = inclusive prefix of V over the 16
        // columns. The k columns left of the lane are the left lane's suffix T(m) = P(15) - P(15 - m)
        // (DPP row_shr:1), those right of it the right lane's P(m - 1) (DPP row_shl:1); the 16-lane DPP
        // row is the image row of the workgroup. Lanes 0 / 15 keep the DPP `old` value: 0 (columns
        // outside the grid when the tile spans the grid's width) or, when tiles_c > 1, the staged halo
        // chunk's sums. All sums are exact u32 arithmetic on the packed fire | dousing << 16 columns.
        const bool halo_lds = tiles_c > 1;  // grid-uniform
        int goff[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) goff[g] = 16 * (q + 1) + 4 * ((g + ((q + 1) >> 2)) & 3);
#pragma unroll
        for (int k = 0; k <= RS; ++k) {
            const uint32_t* top = CP + (rr - k) * CWP;
            const uint32_t* bot = CP + (rr + k + 1) * CWP;
            uint32_t P[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint4 b4 = *reinterpret_cast<const uint4*>(bot + goff[g]);
                const uint4 t4 = *reinterpret_cast<const uint4*>(top + goff[g]);
                P[4 * g + 0] = b4.x - t4.x;
                P[4 * g + 1] = b4.y - t4.y;
                P[4 * g + 2] = b4.z - t4.z;
                P[4 * g + 3] = b4.w - t4.w;
            }
#pragma unroll
            for (int i = 1; i < 16; ++i) P[i] += P[i - 1];
            uint32_t Lh[RS + 1], Rh[RS + 1];  // Lh[m]: sum of the m columns left of the lane, Rh[m]: right
#pragma unroll
            for (int m = 1; m <= k; ++m) {
                Lh[m] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(P[15] - P[15 - m]), 0x111, 0xF, 0xF, false);
                Rh[m] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)P[m - 1], 0x101, 0xF, 0xF, false);
            }
            if (halo_lds && k > 0) {  // lanes 0 / 15: the staged chunks left / right of the tile
                uint32_t al = 0u, ar = 0u;
#pragma unroll
                for (int m = 1; m <= k; ++m) {
                    const int cl = pcol(16 * q + 16 - m), cr = pcol(16 * (q + 2) + m - 1);
                    al += bot[cl] - top[cl];
                    ar += bot[cr] - top[cr];
                    Lh[m] = q == 0 ? al : Lh[m];
                    Rh[m] = q == 15 ? ar : Rh[m];
                }
            }
            const float wk = k <= R ? p.heat_dw[k] : 0.0f;
            uint32_t sprev = 0u;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int hi = i + k < 15 ? i + k : 15, lo = i - k - 1;
                uint32_t s = P[hi];
                if (lo >= 0) s -= P[lo];
                if (i < k) s += Lh[k - i];
                if (i + k > 15) s += Rh[i + k - 15];
                if (i & 1) {
                    const int j = i >> 1;
                    if (k <= R) ph2[j] = __builtin_elementwise_fma((f2){wk, wk}, (f2){fire_f(sprev), fire_f(s)}, ph2[j]);
                    // PK: dousing is 0 / 1 per cell, so the D_1 / D_2 box sums are <= 25 and one v_cvt_f32_ubyte2 converts
                    // them; the plain layouts' u8 counts can sum past 255 (full 16-bit field)
                    const f2 dsum = PK ? (f2){(float)((sprev >> 16) & 0xFFu), (float)((s >> 16) & 0xFFu)}
                                       : (f2){(float)(sprev >> 16), (float)(s >> 16)};
                    if (k == 1) dz2[j] = (f2){w_in_minus_bd, w_in_minus_bd} * dsum;
                    if (k == 2) dz2[j] = __builtin_elementwise_fma((f2){p.dous_border, p.dous_border}, dsum, dz2[j]);
                }
                sprev = s;
            }
            // materialise this radius' partial sums now: without it hipcc keeps all (R+1)x16 window
            // sums live and evaluates the f32 chains at the end (-> spills at R >= 4)
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(ph2[j]), "+v"(dz2[j]));
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ph2[j] = ph2[j] - dz2[j];  // p_h = heat - dousing (:198)
        load_ps(1, psbuf[1]);
    }
    // ---- FIRE bits of rows r-1, r, r+1: bit j of nbw[a] <-> staged column cc0 - 1 + j (j = 0..17)
    uint32_t nbw[3];
    fire_rows(nbw);
    asm volatile("" : "+v"(nbw[0]), "+v"(nbw[1]), "+v"(nbw[2]));  // build the 3 words now (no 9 live halfwords)

    const int widx = wind_index[e];
    float wind[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) wind[d] = p.winds[widx][d < 4 ? d : d + 1];
    const uint32_t step = rng_step ? rng_step[e] : 0u;
    const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
    const uint32_t env_id = (uint32_t)(p.env_offset + e);
    const bool want_prob = PROB && prob_out != nullptr;

    const uint32_t fireB = (nbw[1] >> 1) & 0xFFFFu;
    auto dir_bits = [&](int d) -> uint32_t { return dir_bits_of(nbw, d); };
    uint32_t anyfire = 0u;
#pragma unroll
    for (int d = 0; d < 8; ++d) anyfire |= dir_bits(d);

    // ---- direction-outer pass: each p_slope row segment (16 floats = 64 B per lane, 1 KiB per
    //      16 lanes) is read in one burst, so every HBM line is consumed by one wave instruction group.
    //      qn = prod over burning directions of (1 - clamp01(p_d)), each factor applied as qn = fma(-qn, c, qn);
    //      a non-burning direction's c is masked to +0 (qn unchanged exactly), the oracle's skip-form.
    f2 qn2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) qn2[j] = (f2){1.0f, 1.0f};
    uint32_t burn_inj = 0u;
    __builtin_amdgcn_s_setprio(0);  // (kept: it also fixes hipcc's schedule of the pass, measured r02r)
    if (wave_need) {
        // ---- base = (p_h * (1 + p_veg)) * (1 + p_den)   (left-to-right product of :206), clip(idx, 1, 5)
        //      (:176-178) through the LDS table
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i0 = 2 * j, i1 = 2 * j + 1;
            const uint32_t v0 = min((vgw[i0 >> 2] >> (8 * (i0 & 3))) & 0xFFu, 7u);
            const uint32_t v1 = min((vgw[i1 >> 2] >> (8 * (i1 & 3))) & 0xFFu, 7u);
            const uint32_t d0 = min((dnw[i0 >> 2] >> (8 * (i0 & 3))) & 0xFFu, 7u);
            const uint32_t d1 = min((dnw[i1 >> 2] >> (8 * (i1 & 3))) & 0xFFu, 7u);
            const f2 av = {LUT[v0], LUT[v1]}, ad = {LUT[8 + d0], LUT[8 + d1]};
            ph2[j] = (ph2[j] * av) * ad;  // ph2 now holds base
        }
        // ES border handling: cells in rows 0 / H-1 or columns 0 / W-1 get p_slope = 1 (exponent 0).
        // Rows: lane-uniform, and only the waves holding row 0 or H-1 branch into the select.
        const int wrow0 = r0 + 4 * __builtin_amdgcn_readfirstlane(tid >> 6);
        const bool wave_rowkill = ES && (wrow0 == 0 || wrow0 + 3 >= H - 1);
        const bool rowkill = r == 0 || r >= H - 1;
        const bool kill_lo = cbase == 0;
        const int hi_idx = W - 1 - cbase;  // element holding column W-1, if in [0, 16)
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            const int ld = ES ? (d < 4 ? d : d - 1) : d;  // load consumed by direction d
            float4 (&psc)[4] = psbuf[ld & 1];
            f2 ps2[8];
            if (!ES) {
#pragma unroll
                for (int j = 0; j < 8; ++j) ps2[j] = (j & 1) ? (f2){psc[j >> 1].z, psc[j >> 1].w}
                                                             : (f2){psc[j >> 1].x, psc[j >> 1].y};
            } else {
                float a[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float4 v = psc[i >> 2];
                    a[i] = (i & 3) == 0 ? v.x : (i & 3) == 1 ? v.y : (i & 3) == 2 ? v.z : v.w;
                }
                // d = 4, 7: element i <- i + 1 (cell i's right / down-right neighbour);
                // d = 5: element i <- i - 1; the row segment's outer element comes from the next /
                // previous lane of the 16-lane row (DPP) or, at the segment's end, from e4 / e7 / e5
                if (d == 4 || d == 7) {
                    const float nx = dpp_from_next(d == 4 ? e4 : e7, a[0]);
#pragma unroll
                    for (int i = 0; i < 15; ++i) a[i] = a[i + 1];
                    a[15] = nx;
                } else if (d == 5) {
                    const float pv = dpp_from_prev(e5, a[15]);
#pragma unroll
                    for (int i = 15; i > 0; --i) a[i] = a[i - 1];
                    a[0] = pv;
                }
                // border cells: factor +1 (slope 0 -> p_slope = 1 either way round)
                if (wave_rowkill) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) a[i] = rowkill ? 1.0f : a[i];
                }
                a[0] = kill_lo ? 1.0f : a[0];
                if (FAST) {
                    a[15] = hi_idx == 15 ? 1.0f : a[15];
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) a[i] = hi_idx == i ? 1.0f : a[i];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) ps2[j] = edge_factor_pair(a[2 * j], a[2 * j + 1], d < 4);
            }
            // pin base here: otherwise the 64 direction-independent products base*wind[d] are hoisted
            // above the loop (128 live VGPRs -> spills)
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(ph2[j]));
            // qn of non-tree / out-of-range cells is never used (burn is masked by treeB & okB)
            const uint32_t fbd = INJECT ? (dir_bits(d) & treeB & okB) : dir_bits(d);
            const f2 wd2 = {wind[d], wind[d]};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const f2 ps = ps2[j];
                const f2 t = ph2[j] * wd2;
                f2 c;
                if (PROB) {
                    const f2 pd = t * ps;
                    if (want_prob) {
                        if ((okB >> (2 * j)) & 1u) prob_out[(rowoff + 2 * j) * 8 + d] = pd.x;
                        if ((okB >> (2 * j + 1)) & 1u) prob_out[(rowoff + 2 * j + 1) * 8 + d] = pd.y;
                    }
                    if (INJECT) {
                        const int dd = d < 4 ? d : d + 1;
                        if (((fbd >> (2 * j)) & 1u) && inj_burn[(rowoff + 2 * j) * 9 + dd] < pd.x)
                            burn_inj |= 1u << (2 * j);
                        if (((fbd >> (2 * j + 1)) & 1u) && inj_burn[(rowoff + 2 * j + 1) * 9 + dd] < pd.y)
                            burn_inj |= 1u << (2 * j + 1);
                    }
                    c = (f2){clamp01(pd.x), clamp01(pd.y)};
                } else {
                    c = pk_mul_clamp01(t, ps);
                }
                if (!INJECT) {
                    // q <- fma(-q, c, q) = q * (1 - c) with one rounding; a non-burning direction has c masked to +0,
                    // so q is unchanged exactly (the oracle skips the factor)
                    const uint32_t c0 = __float_as_uint(c.x) & sbit(fbd, 2 * j);
                    const uint32_t c1 = __float_as_uint(c.y) & sbit(fbd, 2 * j + 1);
                    qn2[j] = __builtin_elementwise_fma(-qn2[j], (f2){__uint_as_float(c0), __uint_as_float(c1)}, qn2[j]);
                }
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(qn2[j]));  // finish this direction's products here
            // refill the buffer just consumed with load ld + 2 (ES: not after d = 3, whose load d = 4 reuses)
            const int last = ES ? 6 : 7;
            if (ld + 2 <= last && !(ES && d == 3)) {
                load_ps(ld + 2, psc);
            }
            if (d == 6) load_ages();            // its buffer is free from here on
            __builtin_amdgcn_sched_barrier(0);  // two loads' 64 B per lane in flight
        }
    } else {
        load_ages();
    }

    // ---- draws: burn / grow masks and the packed new-fire ages NA (two cells per word)
    uint32_t burn, grow, NA[8];
    if (INJECT) {
        burn = burn_inj;
        grow = 0u;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (((okB & emptyB) >> i) & 1u) grow |= (uint32_t)(inj_grow[rowoff + i] < p.p_tree) << i;
#pragma unroll
        for (int pp = 0; pp < 8; ++pp) {
            const uint32_t n0 = ((burn >> (2 * pp)) & 1u) ? (uint32_t)inj_age[rowoff + 2 * pp] : 0u;
            const uint32_t n1 = ((burn >> (2 * pp + 1)) & 1u) ? (uint32_t)inj_age[rowoff + 2 * pp + 1] : 0u;
            NA[pp] = __builtin_amdgcn_perm(n1, n0, 0x05040100u);
        }
    } else {
        // Philox (r05): one block per group of 4 cells (r, 4g .. 4g+3), counter r * ceil(W/4) + g (the lane's 16
        // cells are 4 whole groups: cbase % 16 == 0; the march kernel and the C oracle use the same groups); cell j
        // of a group tests word j: burn iff u < 1 - qn <=> (word >> 8) < (1 - qn) * 2^24 (exact power-of-two
        // scaling); grow iff u < p_tree. Cells that need no draw cannot change through them (qn = 1 -> 1-qn = 0).
        // The group's first new fire takes randint of its spare word (the words' low bytes, read by no decision),
        // the 2nd..4th words 0..2 of the group's ALXA block (rare: only computed when some lane needs it).
        const uint32_t needB = okB & ((treeB & anyfire) | (p.p_tree > 0.0f ? emptyB : 0u));
        const float pt24 = __fmul_rn(p.p_tree, 16777216.0f);
        const uint32_t grp0 = (uint32_t)r * (((uint32_t)W + 3u) >> 2) + ((uint32_t)cbase >> 2);
        uint32_t Dt = 0u, Dg = 0u, spare[4];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            const uint32_t nd = (needB >> (4 * gq)) & 0xFu;
            u32x4 X = u32x4{0u, 0u, 0u, 0u};
            if (nd) X = philox4x32_10(u32x4{grp0 + (uint32_t)gq, env_id, step, GCA_TAG_ALEX_CELL}, k0, k1);
            const uint32_t mw[4] = {X.x, X.y, X.z, X.w};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int pp = 2 * gq + h;
                const f2 thr = ((f2){1.0f, 1.0f} - qn2[pp]) * (f2){16777216.0f, 16777216.0f};
                const float u0 = (float)(mw[2 * h] >> 8), u1 = (float)(mw[2 * h + 1] >> 8);
                Dt = push_lt(Dt, u0, thr.x);
                Dt = push_lt(Dt, u1, thr.y);
                Dg = push_lt(Dg, u0, pt24);
                Dg = push_lt(Dg, u1, pt24);
            }
            spare[gq] = __builtin_amdgcn_perm(__builtin_amdgcn_perm(X.w, X.z, 0x0c0c0400u),
                                              __builtin_amdgcn_perm(X.y, X.x, 0x0c0c0400u), 0x05040100u);
            __builtin_amdgcn_sched_barrier(0);  // one Philox block in flight per lane (2 or 4 interleaved: same time, r02h)
        }
        burn = (__builtin_bitreverse32(Dt) >> 16) & treeB & okB;
        grow = (__builtin_bitreverse32(Dg) >> 16) & emptyB & okB;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            const uint32_t n0 = (uint32_t)randint_ms(spare[gq], p.age_lo, p.age_hi);
            NA[2 * gq] = NA[2 * gq + 1] = __builtin_amdgcn_perm(n0, n0, 0x05040100u);
            const uint32_t b4 = (burn >> (4 * gq)) & 0xFu;
            if (__ballot((b4 & (b4 - 1u)) != 0u) != 0ull) {  // a lane with 2+ new fires in this group
                const u32x4 Y = philox4x32_10(u32x4{grp0 + (uint32_t)gq, env_id, step, GCA_TAG_ALEX_AGE}, k0, k1);
                const uint32_t nk[4] = {n0, (uint32_t)randint_ms(Y.x, p.age_lo, p.age_hi),
                                        (uint32_t)randint_ms(Y.y, p.age_lo, p.age_hi),
                                        (uint32_t)randint_ms(Y.z, p.age_lo, p.age_hi)};
                uint32_t a[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t rank = (uint32_t)__builtin_popcount(b4 & ((1u << j) - 1u));
                    a[j] = rank == 0 ? nk[0] : (rank == 1 ? nk[1] : (rank == 2 ? nk[2] : nk[3]));
                }
                NA[2 * gq] = __builtin_amdgcn_perm(a[1], a[0], 0x05040100u);
                NA[2 * gq + 1] = __builtin_amdgcn_perm(a[3], a[2], 0x05040100u);
            }
        }
    }

    // ---- the rule on masks: TREE -> FIRE (burn), EMPTY -> TREE (grow), FIRE -> EMPTY (age <= 1)
    uint32_t le1acc = 0u;  // age <= 1  <=>  sat(age - 2) < 0 (saturating i16: exact for every int16)
#pragma unroll
    for (int pp = 0; pp < 8; ++pp) {
        const i16x2 y = __builtin_elementwise_sub_sat(bitcast_<i16x2>(agew[pp]), (i16x2){2, 2});
        le1acc |= (bitcast_<uint32_t>(y) >> (15 - 2 * pp)) & ((1u << (2 * pp)) | (1u << (16 + 2 * pp)));
    }
    uint32_t le1 = (le1acc & 0x5555u) | ((le1acc >> 15) & 0xAAAAu);
    if (p.burnout_eq1) {  // classic rule: burn out iff age == 1 (uniform branch)
        uint32_t eqacc = 0u;
#pragma unroll
        for (int pp = 0; pp < 8; ++pp) {
            const u16x2 x = bitcast_<u16x2>(agew[pp] ^ 0x00010001u);  // half == 0 <=> age == 1
            const uint32_t z = bitcast_<uint32_t>(x - (u16x2){1, 1}) & ~bitcast_<uint32_t>(x) & 0x80008000u;
            eqacc |= (z >> (15 - 2 * pp)) & ((1u << (2 * pp)) | (1u << (16 + 2 * pp)));
        }
        le1 = (eqacc & 0x5555u) | ((eqacc >> 15) & 0xAAAAu);
    }
    const uint32_t newF = burn | (fireB & ~le1);
    const uint32_t newT = (treeB & ~burn) | grow;
    const uint32_t newE = (emptyB & ~grow) | (fireB & le1);
    const uint32_t keepB = ~(treeB | emptyB | fireB) & 0xFFFFu;  // codes outside {empty, tree, fire}: unchanged
    // output bytes: one v_perm_b32 per word, selector 0/1/2 -> empty/tree/fire code, 4+m -> own byte m
    const uint32_t codes = (p.empty & 0xFFu) | ((p.tree & 0xFFu) << 8) | ((p.fire & 0xFFu) << 16);
    uint32_t sel[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) sel[j] = spread4(newT >> (4 * j)) + 2u * spread4(newF >> (4 * j));
    if (keepB) {
#pragma unroll
        for (int j = 0; j < 4; ++j) sel[j] |= (spread4(keepB >> (4 * j)) * 0xFFu) & 0x07060504u;
    }
    uint32_t outw[4], nagew[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) outw[j] = __builtin_amdgcn_perm(own[j], codes, sel[j]);
    // ages: FIRE cells age - 1 (also when they burn out), new fires the drawn age, others unchanged
    const uint32_t CF = (fireB & 0x5555u) | (((fireB >> 1) & 0x5555u) << 16);
    const uint32_t CB = (burn & 0x5555u) | (((burn >> 1) & 0x5555u) << 16);
#pragma unroll
    for (int pp = 0; pp < 8; ++pp) {
        const u16x2 fh = bitcast_<u16x2>((CF >> (2 * pp)) & 0x00010001u);
        const uint32_t a1 = bitcast_<uint32_t>(bitcast_<u16x2>(agew[pp]) - fh);
        const uint32_t bm = ((CB >> (2 * pp)) & 0x00010001u) * 0xFFFFu;
        nagew[pp] = bfi32(bm, NA[pp], a1);
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
    write_rgb(newT, newF);
    if (counts || (PK && act_out)) {
        int cntT = __builtin_popcount(newT & okB), cntF = __builtin_popcount(newF & okB),
            cntE = __builtin_popcount(newE & okB);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            cntT += __shfl_xor(cntT, off);
            cntF += __shfl_xor(cntF, off);
            cntE += __shfl_xor(cntE, off);
        }
        if ((tid & 63) == 0) {
            if (counts) {
                if (cntE) atomicAdd(counts + 3 * e + 0, cntE);
                if (cntT) atomicAdd(counts + 3 * e + 1, cntT);
                if (cntF) atomicAdd(counts + 3 * e + 2, cntF);
            }
            if (PK && act_out && cntF) act_out[(size_t)e * tiles_r * tiles_c + tile] = 1;
        }
    }
}

// p_slope[e][d][r][c] = slope_factor(0.078f * slope[e][r][c][d'])
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
        p_slope[((int64_t)e * 8 + d) * HW + cell] = slope_factor(a);
    }
}

template <int R, int MODE, bool ES, bool PK = false, bool OBS = false>
void launch_alex(const gca_alex_params& p, int E, int H, int W, const uint8_t* gi, uint8_t* go, const int16_t* ai,
                 int16_t* ao, const uint8_t* veg, const uint8_t* den, const uint8_t* dous, const float* ps,
                 const int32_t* wi, const uint32_t* rs, const float* ib, const float* ig, const int32_t* ia, float* po,
                 int32_t* counts, hipStream_t st, const uint8_t* act_in = nullptr, uint8_t* act_out = nullptr,
                 AlexObs obs = AlexObs{nullptr, nullptr, nullptr}) {
    const int tiles_r = (H + TH - 1) / TH, tiles_c = (W + TW - 1) / TW;
    constexpr int RS = R < 2 ? 2 : R;
    constexpr int RR = TH + 2 * RS;
    const size_t lds = OBS ? (size_t)obs_col_off(RR, PK) + 6 * sizeof(float4)
                           : (size_t)cp_bytes(RR, PK) + sizeof(uint16_t) * RR * (CW / 16) + sizeof(float) * 16;
    const dim3 grid((unsigned)((int64_t)E * tiles_r * tiles_c));
    const bool fast = MODE == 0 && W % TW == 0 && H % TH == 0 &&
                      ((((uintptr_t)gi) | ((uintptr_t)go) | ((uintptr_t)ai) | ((uintptr_t)ao) | ((uintptr_t)veg) |
                        ((uintptr_t)den) | ((uintptr_t)dous) | ((uintptr_t)ps)) & 15u) == 0;
    if (PK)  // packed env layout (the host checked the FAST shape and alignment)
        hipLaunchKernelGGL((alex_step_kernel<R, 0, true, true, true, OBS>), grid, dim3(NT), lds, st, p, H, W, tiles_r,
                           tiles_c, gi, go, ai, ao, veg, den, dous, ps, wi, rs, ib, ig, ia, po, counts, act_in, act_out,
                           obs);
    else if (fast)  // production shape: no per-lane bounds checks (instantiated for the Philox mode only)
        hipLaunchKernelGGL((alex_step_kernel<R, MODE, MODE == 0, ES>), grid, dim3(NT), lds, st, p, H, W, tiles_r,
                           tiles_c, gi, go, ai, ao, veg, den, dous, ps, wi, rs, ib, ig, ia, po, counts, act_in, act_out,
                           obs);
    else
        hipLaunchKernelGGL((alex_step_kernel<R, MODE, false, ES>), grid, dim3(NT), lds, st, p, H, W, tiles_r, tiles_c,
                           gi, go, ai, ao, veg, den, dous, ps, wi, rs, ib, ig, ia, po, counts, act_in, act_out, obs);
}

template <int MODE, bool ES, bool PK = false, bool OBS = false>
void dispatch_r(int R, const gca_alex_params& p, int E, int H, int W, const uint8_t* gi, uint8_t* go, const int16_t* ai,
                int16_t* ao, const uint8_t* veg, const uint8_t* den, const uint8_t* dous, const float* ps,
                const int32_t* wi, const uint32_t* rs, const float* ib, const float* ig, const int32_t* ia, float* po,
                int32_t* counts, hipStream_t st, const uint8_t* act_in = nullptr, uint8_t* act_out = nullptr,
                AlexObs obs = AlexObs{nullptr, nullptr, nullptr}) {
#define GCA_ALEX_CASE(RV) \
    case RV: launch_alex<RV, MODE, ES, PK, OBS>(p, E, H, W, gi, go, ai, ao, veg, den, dous, ps, wi, rs, ib, ig, ia, po, counts, st, act_in, act_out, obs); break;
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

static int alex_step_impl(bool es, const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
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
        (es ? dispatch_r<2, true> : dispatch_r<2, false>)(p->R, *p, E, H, W, grid_in, grid_out, age_in, age_out, veg, den, dousing, p_slope, wind_index,
                         rng_step, inj_burn, inj_grow, inj_age, prob_out, counts, st, nullptr, nullptr, AlexObs{});
    else if (prob_out)
        (es ? dispatch_r<1, true> : dispatch_r<1, false>)(p->R, *p, E, H, W, grid_in, grid_out, age_in, age_out, veg, den, dousing, p_slope, wind_index,
                      rng_step, nullptr, nullptr, nullptr, prob_out, counts, st, nullptr, nullptr, AlexObs{});
    else
        (es ? dispatch_r<0, true> : dispatch_r<0, false>)(p->R, *p, E, H, W, grid_in, grid_out, age_in, age_out, veg, den, dousing, p_slope, wind_index,
                      rng_step, nullptr, nullptr, nullptr, nullptr, counts, st, nullptr, nullptr, AlexObs{});
    GCA_CHECK_LAUNCH(es ? "alex_step_es" : "alex_step");
    return GCA_OK;
}

extern "C" int gca_alex_step(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                             const int16_t* age_in, int16_t* age_out, const uint8_t* veg, const uint8_t* den,
                             const uint8_t* dousing, const float* p_slope, const int32_t* wind_index,
                             const uint32_t* rng_step, const float* inj_burn, const float* inj_grow,
                             const int32_t* inj_age, float* prob_out, int32_t* counts, void* stream) {
    return alex_step_impl(false, p, E, H, W, grid_in, grid_out, age_in, age_out, veg, den, dousing, p_slope,
                          wind_index, rng_step, inj_burn, inj_grow, inj_age, prob_out, counts, stream);
}

extern "C" int gca_alex_step_es(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in,
                                uint8_t* grid_out, const int16_t* age_in, int16_t* age_out, const uint8_t* veg,
                                const uint8_t* den, const uint8_t* dousing, const float* edge_slope,
                                const int32_t* wind_index, const uint32_t* rng_step, const float* inj_burn,
                                const float* inj_grow, const int32_t* inj_age, float* prob_out, int32_t* counts,
                                void* stream) {
    return alex_step_impl(true, p, E, H, W, grid_in, grid_out, age_in, age_out, veg, den, dousing, edge_slope,
                          wind_index, rng_step, inj_burn, inj_grow, inj_age, prob_out, counts, stream);
}

static int alex_step_packed_impl(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in,
                                 uint8_t* grid_out, const int16_t* age_in, int16_t* age_out, const uint8_t* vd,
                                 const uint16_t* dous_bits, const float* edge_slope_coal, const int32_t* wind_index,
                                 const uint32_t* rng_step, int32_t* counts, const uint8_t* act_in, uint8_t* act_out,
                                 AlexObs obs, void* stream) {
    GCA_CHECK_ARG(p && grid_in && grid_out && age_in && age_out && vd && dous_bits && edge_slope_coal && wind_index,
                  "alex_step_packed: null argument");
    GCA_CHECK_ARG(E > 0 && H > 0 && W > 0 && W % TW == 0 && H % TH == 0,
                  "alex_step_packed: W must be a multiple of 256 and H of 16");
    GCA_CHECK_ARG(p->R >= 1 && p->R <= GCA_MAX_RADIUS, "alex_step_packed: burn radius must be in [1, 8]");
    GCA_CHECK_ARG(p->n_winds >= 1 && p->n_winds <= 16, "alex_step_packed: 1..16 wind matrices");
    // ages may be updated in place (each lane reads and writes only its own cells); the grid may not (halos)
    GCA_CHECK_ARG(grid_in != grid_out, "alex_step_packed: the grid cannot be updated in place");
    GCA_CHECK_ARG(((((uintptr_t)grid_in) | ((uintptr_t)grid_out) | ((uintptr_t)age_in) | ((uintptr_t)age_out) |
                    ((uintptr_t)vd) | ((uintptr_t)edge_slope_coal) | ((uintptr_t)obs.rgb) | ((uintptr_t)obs.col)) & 15u) == 0
                      && ((uintptr_t)dous_bits & 1u) == 0,
                  "alex_step_packed: arrays must be 16-B aligned");
    hipStream_t st = (hipStream_t)stream;
    if (counts && hipMemsetAsync(counts, 0, sizeof(int32_t) * 3 * (size_t)E, st) != hipSuccess) {
        gca_set_error("alex_step_packed: counts memset failed");
        return GCA_ERR_HIP;
    }
    GCA_CHECK_ARG(!act_in || act_out, "alex_step_packed: act_in needs act_out");
    GCA_CHECK_ARG(act_in != act_out || !act_in, "alex_step_packed: act_in and act_out must differ");
    // a tile without fire nearby can still change when EMPTY cells grow: the skip needs p_tree == 0
    const uint8_t* ain = (p->p_tree > 0.0f) ? nullptr : act_in;
    if (obs.rgb)
        dispatch_r<0, true, true, true>(p->R, *p, E, H, W, grid_in, grid_out, age_in, age_out, vd, nullptr,
                                        reinterpret_cast<const uint8_t*>(dous_bits), edge_slope_coal, wind_index, rng_step,
                                        nullptr, nullptr, nullptr, nullptr, counts, st, ain, act_out, obs);
    else
        dispatch_r<0, true, true>(p->R, *p, E, H, W, grid_in, grid_out, age_in, age_out, vd, nullptr,
                                  reinterpret_cast<const uint8_t*>(dous_bits), edge_slope_coal, wind_index, rng_step, nullptr,
                                  nullptr, nullptr, nullptr, counts, st, ain, act_out);
    GCA_CHECK_LAUNCH(obs.rgb ? "alex_step_packed_rgb" : "alex_step_packed");
    return GCA_OK;
}

extern "C" int gca_alex_step_packed(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in,
                                    uint8_t* grid_out, const int16_t* age_in, int16_t* age_out, const uint8_t* vd,
                                    const uint16_t* dous_bits, const float* edge_slope_coal, const int32_t* wind_index,
                                    const uint32_t* rng_step, int32_t* counts, const uint8_t* act_in, uint8_t* act_out,
                                    void* stream) {
    return alex_step_packed_impl(p, E, H, W, grid_in, grid_out, age_in, age_out, vd, dous_bits, edge_slope_coal,
                                 wind_index, rng_step, counts, act_in, act_out, AlexObs{nullptr, nullptr, nullptr}, stream);
}

extern "C" int gca_alex_step_packed_rgb(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in,
                                        uint8_t* grid_out, const int16_t* age_in, int16_t* age_out, const uint8_t* vd,
                                        const uint16_t* dous_bits, const float* edge_slope_coal,
                                        const int32_t* wind_index, const uint32_t* rng_step, int32_t* counts,
                                        const uint8_t* act_in, uint8_t* act_out, const float* color_table,
                                        const int32_t* is_night, float* rgb, void* stream) {
    GCA_CHECK_ARG(color_table && is_night && rgb, "alex_step_packed_rgb: color_table, is_night and rgb required");
    return alex_step_packed_impl(p, E, H, W, grid_in, grid_out, age_in, age_out, vd, dous_bits, edge_slope_coal,
                                 wind_index, rng_step, counts, act_in, act_out,
                                 AlexObs{reinterpret_cast<const float4*>(color_table), is_night, rgb}, stream);
}


// ------------------------------------------------------------------ packed env layers
namespace {
// one thread per 16-cell chunk: vd = min(veg, 7) | min(den, 7) << 4, dousing bit = (count != 0)
__global__ void alex_pack_layers_kernel(const uint8_t* __restrict__ veg, const uint8_t* __restrict__ den,
                                        const uint8_t* __restrict__ dous, uint8_t* __restrict__ vd,
                                        uint16_t* __restrict__ dbits, int64_t nchunks) {
    const int64_t ch = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ch >= nchunks) return;
    uint16_t b = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int64_t c = ch * 16 + i;
        if (vd) vd[c] = (uint8_t)(min((int)veg[c], 7) | (min((int)den[c], 7) << 4));
        b |= (uint16_t)((dous[c] != 0 ? 1u : 0u) << i);
    }
    dbits[ch] = b;
}
// coalesced edge-slope order: inside every 256-column segment, column 16q + 4m + j -> position 64m + 4q + j
__global__ void alex_edge_coalesce_kernel(const float* __restrict__ in, float* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t seg = i >> 8;
    const int c = (int)(i & 255), q = c >> 4, m = (c >> 2) & 3, j = c & 3;
    out[(seg << 8) + 64 * m + 4 * q + j] = in[i];
}
}  // namespace

extern "C" int gca_alex_pack_layers(const uint8_t* veg, const uint8_t* den, const uint8_t* dousing, uint8_t* vd,
                                    uint16_t* dous_bits, int E, int H, int W, void* stream) {
    GCA_CHECK_ARG(dousing && dous_bits && E > 0 && H > 0 && W > 0 && W % 16 == 0,
                  "pack_layers: dousing, dous_bits and W % 16 == 0 required");
    GCA_CHECK_ARG(!vd || (veg && den), "pack_layers: vd needs veg and den");
    const int64_t nch = (int64_t)E * H * W / 16;
    hipLaunchKernelGGL(alex_pack_layers_kernel, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       veg, den, dousing, vd, dous_bits, nch);
    GCA_CHECK_LAUNCH("pack_layers");
    return GCA_OK;
}

extern "C" int gca_alex_edge_slope_coalesce(const float* edge_slope, float* edge_slope_coal, int E, int H, int W,
                                            void* stream) {
    GCA_CHECK_ARG(edge_slope && edge_slope_coal && edge_slope != edge_slope_coal && E > 0 && H > 0 && W > 0 &&
                      W % TW == 0,
                  "edge_slope_coalesce: distinct arrays and W % 256 == 0 required");
    const int64_t n = (int64_t)E * 4 * H * W;
    hipLaunchKernelGGL(alex_edge_coalesce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       edge_slope, edge_slope_coal, n);
    GCA_CHECK_LAUNCH("edge_slope_coalesce");
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
            p_slope[((int64_t)e * 8 + d) * HW + cell] = slope_factor(__fmul_rn(0.078f, s));
            ++d;
        }
    }
}
}  // namespace

// Edge layout of the same slopes (see alex_step_kernel, ES): es[e][k][r][c] = the signed slope factor
// of (r,c) toward neighbour k (+exp_f32(a) for a >= 0, -exp_f32(-a) for a < 0, a = 0.078f * f32(raw slope)), k = 0..3 <-> (-1,-1), (-1,0), (-1,+1), (0,-1), with get_slope's arithmetic
// but WITHOUT its border zeroing (the step kernel applies that per cell); 0 where the neighbour is outside.
namespace {
__global__ void alex_edge_slope_from_altitude_kernel(const double* __restrict__ alt, float* __restrict__ es, int H,
                                                     int W, int E) {
    const int64_t HW = (int64_t)H * W;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= HW * E) return;
    const int e = (int)(idx / HW);
    const int64_t cell = idx - (int64_t)e * HW;
    const int r = (int)(cell / W), c = (int)(cell - (int64_t)r * W);
    const double* a = alt ? alt + (int64_t)e * HW : nullptr;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int dr = k < 3 ? -1 : 0, dc = k < 3 ? k - 1 : -1;
        const int nr = r + dr, nc = c + dc;
        float s = 0.0f;
        if (a && nr >= 0 && nc >= 0 && nc < W) {
            double diff = a[cell] - a[(int64_t)nr * W + nc];
            if (dr != 0 && dc != 0) diff /= 1.414;
            s = (float)(atan(diff) * (180.0 / 3.14159265358979323846));
        }
        // signed factor: +exp_f32(a) for a >= 0, -exp_f32(-a) for a < 0, a = 0.078f * slope
        const float a = __fmul_rn(0.078f, s);
        es[((int64_t)e * 4 + k) * HW + cell] = a >= 0.0f ? exp_f32(a) : -exp_f32(-a);
    }
}
}  // namespace

namespace {
__global__ void alex_edge_factors_kernel(const float* __restrict__ v, float* __restrict__ own, float* __restrict__ nbr,
                                         int64_t n) {
    const int64_t i = 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const float v0 = v[i], v1 = i + 1 < n ? v[i + 1] : 1.0f;
    const f2 o = edge_factor_pair(v0, v1, true), b = edge_factor_pair(v0, v1, false);
    own[i] = o.x;
    nbr[i] = b.x;
    if (i + 1 < n) {
        own[i + 1] = o.y;
        nbr[i + 1] = b.y;
    }
}
}  // namespace

extern "C" int gca_alex_edge_factors(const float* v, float* own, float* nbr, int64_t n, void* stream) {
    GCA_CHECK_ARG(v && own && nbr && n > 0, "edge_factors: bad arguments");
    const int64_t pairs = (n + 1) / 2;
    hipLaunchKernelGGL(alex_edge_factors_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, v, own, nbr, n);
    GCA_CHECK_LAUNCH("alex_edge_factors");
    return GCA_OK;
}

extern "C" int gca_alex_edge_slope_from_altitude(const double* altitude, float* edge_slope, int E, int H, int W,
                                                 void* stream) {
    GCA_CHECK_ARG(edge_slope && E > 0 && H > 0 && W > 0, "edge_slope_from_altitude: bad arguments");
    const int64_t n = (int64_t)E * H * W;
    hipLaunchKernelGGL(alex_edge_slope_from_altitude_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, altitude, edge_slope, H, W, E);
    GCA_CHECK_LAUNCH("alex_edge_slope_from_altitude");
    return GCA_OK;
}

namespace {
__global__ void alex_altitude_apply_kernel(double* __restrict__ alt, int H, int W, int E,
                                           const int32_t* __restrict__ n_hills, const double* __restrict__ hills,
                                           const int32_t* __restrict__ n_slopes, const double* __restrict__ slopes) {
    const int64_t HW = (int64_t)H * W;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= HW * E) return;
    const int e = (int)(idx / HW);
    const int64_t cell = idx - (int64_t)e * HW;
    const int i = (int)(cell / W), j = (int)(cell - (int64_t)i * W);
    double a = alt[idx];
    const int nh = min(n_hills[e], GCA_MAX_HILLS);
    for (int h = 0; h < nh; ++h) {
        const double* hp = hills + ((int64_t)e * GCA_MAX_HILLS + h) * 4;
        const int cr = (int)hp[0], cc = (int)hp[1], radius = (int)hp[2];
        const int64_t dr = i - cr, dc = j - cc;
        const double distance = sqrt((double)(dr * dr + dc * dc));
        if (distance < (double)radius) a = __dadd_rn(a, __dmul_rn(hp[3], cos(distance / (double)radius * M_PI / 2)));
    }
    const int ns = min(n_slopes[e], GCA_MAX_SLOPES);
    for (int k = 0; k < ns; ++k) {
        const double* sp = slopes + ((int64_t)e * GCA_MAX_SLOPES + k) * 5;
        const int sr = (int)sp[0], sc = (int)sp[1], width = (int)sp[2], height = (int)sp[3];
        if (i >= sr && i < min(sr + height, H) && j >= sc && j < min(sc + width, W))
            a = __dadd_rn(a, __dmul_rn(sp[4], (double)(i - sr) / (double)height));
    }
    alt[idx] = a / 10.0;
}
}  // namespace

extern "C" int gca_alex_altitude_apply(double* altitude, int E, int H, int W, const int32_t* n_hills,
                                       const double* hills, const int32_t* n_slopes, const double* slopes,
                                       void* stream) {
    GCA_CHECK_ARG(altitude && n_hills && hills && n_slopes && slopes && E > 0 && H > 0 && W > 0,
                  "altitude_apply: bad arguments");
    const int64_t n = (int64_t)E * H * W;
    hipLaunchKernelGGL(alex_altitude_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, altitude, H, W, E, n_hills, hills, n_slopes, slopes);
    GCA_CHECK_LAUNCH("alex_altitude_apply");
    return GCA_OK;
}

extern "C" int gca_alex_slope_from_altitude(const double* altitude, float* p_slope, float* slope_out, int E, int H,
                                            int W, void* stream) {
    GCA_CHECK_ARG(p_slope && E > 0 && H > 0 && W > 0, "slope_from_altitude: bad arguments");
    const int64_t n = (int64_t)E * H * W;
    hipLaunchKernelGGL(alex_slope_from_altitude_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, altitude, p_slope, slope_out, H, W, E);
    GCA_CHECK_LAUNCH("alex_slope_from_altitude");
    return GCA_OK;
}
