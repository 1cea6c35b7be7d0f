// gca_pine.hip — pinecone spotting of the Alexandridis CA on gfx950.
// Reference: PartiallyObservableForestFireJax._handle_pinecone_spread (ca_alexandridis_jax.py:229-319)
//            + _compute_pinecone_burn_probability (:208-227) and the scatter of _update_grid (:400-420,
//            commented out in the reference's live path; enabled here on request).
//
// Every cell burning in the step's INPUT grid (fire_mask) throws n = min(Poisson(1), max_pinecones)
// pinecones. Pinecone m: direction d in [0, 8), thrust t = N(0, 1) * ft[ft_lookup[d]] (the env's current
// wind ft matrix), landing (clip(round(r + dx[d] t)), clip(round(c + dy[d] t))). A pinecone landing on a
// TREE of the step's OUTPUT grid ignites it with probability 0.48 (1 + p_veg) (1 + p_den) of the target.
// round(r + dx t) = r + dx * round(t) for dx in {-1, 0, 1} (t continuous), so the kernel draws the integer
// s = round(t) directly from its exact law P(s = k) = Phi((k + .5) / f) - Phi((k - .5) / f): 32-bit
// inverse-CDF thresholds built on the host in f64 (gymca_amd/forest_fire/operators/pinecones.py) and one
// integer compare per threshold, so the C oracle reproduces every landing bit for bit.
//
// Draws (Philox4x32-10): block (lin, env, step, PINE) word 0 -> n (Poisson CDF thresholds); block
// (lin, env, step, PINE + 1 + m) -> s (word 0), burn uniform (word 1 >> 8), direction (word 2 >> 29).
// Duplicates (the reference's .at[].set scatter leaves their order unspecified): a target ignites iff ANY
// pinecone landing on it burns; its age is randint(age_lo, age_hi) of word 0 of block (target lin, env,
// step, PINA), whichever pinecone wins. The ignition is an atomicCAS of the target's byte (TREE -> FIRE),
// so exactly one thread writes the age and moves one count from tree to fire.
// Cost: 1 B/cell of input grid read + ~2 Philox blocks per burning cell + scattered byte CAS per landing.
#include "gca_common.h"

namespace {

__device__ __forceinline__ int cdf_pick(uint32_t x, const uint32_t* thr, int n) {
    int k = 0;
    for (int j = 0; j < n; ++j) k += x >= thr[j] ? 1 : 0;
    return k;
}

// one thread per 16-cell chunk of the input grid; the loops run only over its burning cells
__global__ __launch_bounds__(256) void alex_pinecones_kernel(gca_pine_params p, int H, int W,
                                                             const uint8_t* __restrict__ grid_in,
                                                             uint8_t* __restrict__ grid_out,
                                                             int16_t* __restrict__ age_out,
                                                             const uint8_t* __restrict__ veg,
                                                             const uint8_t* __restrict__ den,
                                                             const int32_t* __restrict__ wind_index,
                                                             const uint32_t* __restrict__ s_cdf,
                                                             const uint32_t* __restrict__ rng_step,
                                                             int32_t* __restrict__ counts, uint8_t* __restrict__ act,
                                                             int64_t chunks_per_env, int E) {
    const int64_t gch = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int e = (int)(gch / chunks_per_env);
    if (e >= E) return;
    const int64_t ch = gch - (int64_t)e * chunks_per_env;
    const int64_t HW = (int64_t)H * W;
    const int64_t c0 = ch * 16;
    const uint8_t* gi = grid_in + (int64_t)e * HW;
    uint32_t fire = 0u;
    for (int i = 0; i < 16; ++i)
        if (c0 + i < HW && gi[c0 + i] == (uint8_t)p.fire) fire |= 1u << i;
    if (!fire) return;
    const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
    const uint32_t env_id = (uint32_t)(p.env_offset + e);
    const uint32_t step = rng_step ? rng_step[e] : 0u;
    const uint32_t* tab = s_cdf + (int64_t)wind_index[e] * 8 * GCA_PINE_CDF;
    uint8_t* go = grid_out + (int64_t)e * HW;
    const uint8_t* vE = veg + (int64_t)e * HW;
    const uint8_t* dE = den + (int64_t)e * HW;
    while (fire) {
        const int i = __builtin_ctz(fire);
        fire &= fire - 1u;
        const uint32_t lin = (uint32_t)(c0 + i);
        const int r = (int)(lin / (uint32_t)W), c = (int)(lin - (uint32_t)r * (uint32_t)W);
        const u32x4 B0 = philox4x32_10(u32x4{lin, env_id, step, GCA_TAG_PINE}, k0, k1);
        const int n = min(cdf_pick(B0.x, p.n_cdf, GCA_PINE_MAX), p.max_pinecones);
        for (int m = 0; m < n; ++m) {
            const u32x4 X = philox4x32_10(u32x4{lin, env_id, step, GCA_TAG_PINE + 1u + (uint32_t)m}, k0, k1);
            const int d = (int)(X.z >> 29);
            const uint32_t* t = tab + d * GCA_PINE_CDF;  // t[0] = 2K thresholds, then t[1..2K]; s in [-K, K]
            const int s = cdf_pick(X.x, t + 1, (int)t[0]) - (int)(t[0] >> 1);
            const int tr = min(max(r + p.dx[d] * s, 0), H - 1), tc = min(max(c + p.dy[d] * s, 0), W - 1);
            const int64_t tl = (int64_t)tr * W + tc;
            // the target's pinecone burn probability (:209-227): (0.48 * (1 + p_veg)) * (1 + p_den), clip 1..5
            const int vv = min(max((int)vE[tl], 1), 5), dd = min(max((int)dE[tl], 1), 5);
            const float prob = __fmul_rn(__fmul_rn(p.scale, p.veg1p[vv]), p.den1p[dd]);
            if (!((float)(X.y >> 8) * 0x1.0p-24f < prob)) continue;
            // TREE -> FIRE on the output grid, once: atomicCAS of the aligned word holding the byte
            uint8_t* bp = go + tl;
            uint32_t* wp = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(bp) & ~(uintptr_t)3);
            const uint32_t sh = 8u * (uint32_t)(reinterpret_cast<uintptr_t>(bp) & 3);
            uint32_t old = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool won = false;
            while (((old >> sh) & 0xFFu) == (uint32_t)p.tree) {
                const uint32_t nw = (old & ~(0xFFu << sh)) | ((uint32_t)p.fire << sh);
                const uint32_t prev = atomicCAS(wp, old, nw);
                if (prev == old) {
                    won = true;
                    break;
                }
                old = prev;
            }
            if (won) {
                const u32x4 A = philox4x32_10(u32x4{(uint32_t)tl, env_id, step, GCA_TAG_PINE_AGE}, k0, k1);
                age_out[(int64_t)e * HW + tl] = (int16_t)randint_ms(A.x, p.age_lo, p.age_hi);
                if (counts) {
                    atomicSub(counts + 3 * e + 1, 1);
                    atomicAdd(counts + 3 * e + 2, 1);
                }
                if (act) {  // the step's tile activity map (16 x 256 tiles): the target's tile now burns
                    const int tcw = (W + 255) / 256, tch = (H + 15) / 16;
                    act[(int64_t)e * tch * tcw + (tr / 16) * tcw + tc / 256] = 1;
                }
            }
        }
    }
}

}  // namespace

extern "C" int gca_alex_pinecones(const gca_pine_params* p, int E, int H, int W, const uint8_t* grid_in,
                                  uint8_t* grid_out, int16_t* age_out, const uint8_t* veg, const uint8_t* den,
                                  const int32_t* wind_index, const uint32_t* s_cdf, const uint32_t* rng_step,
                                  int32_t* counts, uint8_t* act_tiles, void* stream) {
    GCA_CHECK_ARG(p && grid_in && grid_out && age_out && veg && den && wind_index && s_cdf,
                  "alex_pinecones: null argument");
    GCA_CHECK_ARG(E > 0 && H > 0 && W > 0 && grid_in != grid_out, "alex_pinecones: bad sizes or aliased grids");
    GCA_CHECK_ARG(p->max_pinecones >= 0 && p->max_pinecones <= GCA_PINE_MAX, "alex_pinecones: max_pinecones in [0, 8]");
    GCA_CHECK_ARG(((uintptr_t)grid_out & 3u) == 0 && ((int64_t)H * W) % 4 == 0,
                  "alex_pinecones: grid_out 4-B aligned and H*W % 4 == 0 (byte CAS on whole words)");
    const int64_t cpe = ((int64_t)H * W + 15) / 16;
    const int64_t n = cpe * E;
    hipLaunchKernelGGL(alex_pinecones_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *p,
                       H, W, grid_in, grid_out, age_out, veg, den, wind_index, s_cdf, rng_step, counts, act_tiles, cpe, E);
    GCA_CHECK_LAUNCH("alex_pinecones");
    return GCA_OK;
}

// ============================================================================ classic pinecone spotting
// PartiallyObservableForestFire.update (ca_alexandridis.py:135-221) throws pinecones from every FIRE cell it
// VISITS, in row-major order, and a pinecone that ignites a cell later in that order puts the cell on the
// skip list (:151-152, :209-210): the later cell is then not visited at all — when it is a FIRE cell of the
// input grid it throws nothing. Whether source s throws therefore depends on the sources before it:
//     active(s) = NOT OR { active(s') : s' < s, a pinecone of s' ignites s }.
// The landings of a source are a function of its own counter-keyed draws, so this is a DAG in scan order, and
// the Jacobi iteration sup_{k+1} = ignitions by {s : not sup_k(s)} reaches its unique fixed point after at most
// (longest chain + 1) rounds. One workgroup per env keeps four bitmaps (FIRE of grid_in, sup_k, sup_{k+1},
// edge = "s ignites some later FIRE cell when it throws") in LDS or, for grids above GCA_PINEC_LDS_MAX_HW cells,
// in the caller's scratch. Round 0 runs every source once; later rounds re-run only edge sources (the others
// can never change a bit); the final pass applies the landings of the active sources, one writer per target
// (atomicOr on an "ignited" bitmap picks it).
namespace {

enum { PC_ROUND0 = 0, PC_ROUND = 1, PC_APPLY = 2 };

template <bool IN_LDS>
__device__ __forceinline__ void pc_sync() {
    if (!IN_LDS) __threadfence();  // global bitmaps: atomics live in L2; drop stale L1 lines after the barrier
    __syncthreads();
    if (!IN_LDS) __threadfence();
}

__device__ __forceinline__ bool bm_test(const uint32_t* bm, uint32_t i) { return (bm[i >> 5] >> (i & 31u)) & 1u; }

struct PcEnv {
    int H, W;
    uint32_t env_id, step, k0, k1;
    const uint32_t* tab;  // [8][GCA_PINEC_CDF] of this env's wind
    const uint8_t* veg;
    const uint8_t* den;
};

// The pinecones of source s (ca_alexandridis.py:184-210). ROUND0 / ROUND: OR the ignited later FIRE cells into
// `out` (ROUND0 also records s in `edge`); APPLY: ignite every target (first writer per target wins).
template <int MODE>
__device__ __forceinline__ void pc_throw(const gca_pine_classic_params& p, const PcEnv& v, uint32_t s,
                                         const uint32_t* fireb, uint32_t* out, uint32_t* edge, uint8_t* go,
                                         int16_t* ao, int32_t* cnt) {
    const int r = (int)(s / (uint32_t)v.W), c = (int)(s - (uint32_t)r * (uint32_t)v.W);
    const u32x4 B0 = philox4x32_10(u32x4{s, v.env_id, v.step, GCA_TAG_PINEC}, v.k0, v.k1);
    const int n = cdf_pick(B0.x, p.n_cdf, GCA_PINEC_NMAX);
    bool later_fire = false;
    for (int m = 0; m < n; ++m) {
        const u32x4 X = philox4x32_10(u32x4{s, v.env_id, v.step, GCA_TAG_PINEC + 1u + (uint32_t)m}, v.k0, v.k1);
        const int d = (int)(X.z >> 29);
        const uint32_t* t = v.tab + d * GCA_PINEC_CDF;
        const int sv = cdf_pick(X.x, t + 1, (int)t[0]) - (int)(t[0] >> 1);
        const int tr = r + p.dx[d] * sv, tc = c + p.dy[d] * sv;
        // inside the grid and not the source itself (:194-200; (dx, dy) != (0, 0), so s_m == 0 is the source)
        if (sv == 0 || tr < 0 || tr >= v.H || tc < 0 || tc >= v.W) continue;
        const uint32_t tl = (uint32_t)tr * (uint32_t)v.W + (uint32_t)tc;
        const int vv = min(max((int)v.veg[tl], 1), 5), dd = min(max((int)v.den[tl], 1), 5);
        if ((X.y >> 8) >= p.burn_thr[vv][dd]) continue;  // p_burn > uniform (:126-127)
        const uint32_t bit = 1u << (tl & 31u);
        if (MODE != PC_APPLY) {
            if (tl > s && bm_test(fireb, tl)) {
                atomicOr(out + (tl >> 5), bit);
                later_fire = true;
            }
        } else if (!(atomicOr(out + (tl >> 5), bit) & bit)) {
            const uint8_t prev = go[tl];
            go[tl] = (uint8_t)p.fire;
            const u32x4 A = philox4x32_10(u32x4{tl, v.env_id, v.step, GCA_TAG_PINEC_AGE}, v.k0, v.k1);
            ao[tl] = (int16_t)randint_ms(A.x, p.age_lo, p.age_hi);
            if (cnt && prev != (uint8_t)p.fire) {
                const int from = prev == (uint8_t)p.empty ? 0 : (prev == (uint8_t)p.tree ? 1 : -1);
                if (from >= 0) atomicSub(cnt + from, 1);
                atomicAdd(cnt + 2, 1);
            }
        }
    }
    if (MODE == PC_ROUND0 && later_fire) atomicOr(edge + (s >> 5), 1u << (s & 31u));
}

template <bool IN_LDS>
__global__ __launch_bounds__(512) void alex_pinecones_classic_kernel(
    gca_pine_classic_params p, int H, int W, int NW, const uint8_t* __restrict__ grid_in, uint8_t* grid_out,
    int16_t* age_out, const uint8_t* __restrict__ veg, const uint8_t* __restrict__ den,
    const int32_t* __restrict__ wind_index, const uint32_t* __restrict__ s_cdf, const uint32_t* __restrict__ rng_step,
    int32_t* counts, uint32_t* scratch) {
    extern __shared__ uint32_t pc_lds[];
    const int e = blockIdx.x;
    const int64_t HW = (int64_t)H * W;
    uint32_t* bm = IN_LDS ? pc_lds : scratch + (int64_t)e * 4 * NW;
    uint32_t* fireb = bm;
    uint32_t* supA = bm + NW;
    uint32_t* supB = bm + 2 * NW;
    uint32_t* edge = bm + 3 * NW;
    const uint8_t* gi = grid_in + e * HW;
    const PcEnv v{H, W, (uint32_t)(p.env_offset + e), rng_step ? rng_step[e] : 0u, (uint32_t)p.seed,
                  (uint32_t)(p.seed >> 32), s_cdf + (int64_t)wind_index[e] * 8 * GCA_PINEC_CDF, veg + e * HW,
                  den + e * HW};
    uint8_t* go = grid_out + e * HW;
    int16_t* ao = age_out + e * HW;
    int32_t* cnt = counts ? counts + 3 * e : nullptr;
    const int T = blockDim.x;

    // FIRE bitmap of the input grid; clear the others
    for (int w = threadIdx.x; w < NW; w += T) {
        uint32_t bits = 0;
        const int64_t b = (int64_t)w * 32;
        for (int i = 0; i < 32; ++i)
            if (b + i < HW && gi[b + i] == (uint8_t)p.fire) bits |= 1u << i;
        fireb[w] = bits;
        supA[w] = 0u;
        supB[w] = 0u;
        edge[w] = 0u;
    }
    pc_sync<IN_LDS>();
    // round 0: every source throws
    for (int w = threadIdx.x; w < NW; w += T)
        for (uint32_t bits = fireb[w]; bits; bits &= bits - 1u)
            pc_throw<PC_ROUND0>(p, v, (uint32_t)w * 32u + (uint32_t)__builtin_ctz(bits), fireb, supA, edge, go, ao,
                                cnt);
    pc_sync<IN_LDS>();
    // rounds k >= 1 over the edge sources, until sup stops changing (every wave sees the same `changed`)
    uint32_t* A = supA;
    uint32_t* B = supB;
    for (int64_t round = 0; round <= HW; ++round) {
        for (int w = threadIdx.x; w < NW; w += T)
            for (uint32_t bits = edge[w] & ~A[w]; bits; bits &= bits - 1u)
                pc_throw<PC_ROUND>(p, v, (uint32_t)w * 32u + (uint32_t)__builtin_ctz(bits), fireb, B, edge, go, ao,
                                   cnt);
        pc_sync<IN_LDS>();
        int changed = 0;
        for (int w = threadIdx.x; w < NW; w += T) {
            changed |= A[w] != B[w];
            A[w] = 0u;
        }
        if (!IN_LDS) __threadfence();
        changed = __syncthreads_or(changed);
        if (!IN_LDS) __threadfence();
        uint32_t* t = A;
        A = B;
        B = t;
        if (!changed) break;
    }
    // A = the fixed point; B (cleared) becomes the "ignited" bitmap of the apply pass
    for (int w = threadIdx.x; w < NW; w += T)
        for (uint32_t bits = fireb[w] & ~A[w]; bits; bits &= bits - 1u)
            pc_throw<PC_APPLY>(p, v, (uint32_t)w * 32u + (uint32_t)__builtin_ctz(bits), fireb, B, edge, go, ao,
                               cnt);
}

}  // namespace

extern "C" int gca_alex_pinecones_classic(const gca_pine_classic_params* p, int E, int H, int W,
                                          const uint8_t* grid_in, uint8_t* grid_out, int16_t* age_out,
                                          const uint8_t* veg, const uint8_t* den, const int32_t* wind_index,
                                          const uint32_t* s_cdf, const uint32_t* rng_step, int32_t* counts,
                                          uint32_t* scratch, void* stream) {
    GCA_CHECK_ARG(p && grid_in && grid_out && age_out && veg && den && wind_index && s_cdf,
                  "alex_pinecones_classic: null argument");
    GCA_CHECK_ARG(E > 0 && H > 0 && W > 0 && grid_in != grid_out, "alex_pinecones_classic: bad sizes or aliased grids");
    const int64_t HW = (int64_t)H * W;
    GCA_CHECK_ARG(HW < ((int64_t)1 << 31), "alex_pinecones_classic: H * W < 2^31");
    const int NW = (int)((HW + 31) / 32);
    const bool in_lds = HW <= GCA_PINEC_LDS_MAX_HW;
    GCA_CHECK_ARG(in_lds || scratch, "alex_pinecones_classic: scratch (E * 4 * ceil(H W / 32) u32) required above "
                                     "GCA_PINEC_LDS_MAX_HW cells");
    hipStream_t st = (hipStream_t)stream;
    if (in_lds) {
        const size_t lds = (size_t)16 * NW;
        // raise the dynamic-LDS ceiling on every launch above 64 KiB: the attribute is per device (and cheap), so a
        // process-wide "already set" cache would skip it on a second GPU. GCA_PINEC_LDS_MAX_HW = 512 * 512 keeps the
        // bitmaps at <= 128 KiB, leaving room under the 160 KiB per-workgroup limit for the static LDS of
        // __syncthreads_or's work-group reduction.
        if (lds > 65536 && hipFuncSetAttribute(reinterpret_cast<const void*>(&alex_pinecones_classic_kernel<true>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
            gca_set_error("alex_pinecones_classic: hipFuncSetAttribute(%zu B LDS) failed", lds);
            return GCA_ERR_HIP;
        }
        hipLaunchKernelGGL(alex_pinecones_classic_kernel<true>, dim3(E), dim3(512), lds, st, *p, H, W, NW, grid_in,
                           grid_out, age_out, veg, den, wind_index, s_cdf, rng_step, counts, nullptr);
    } else {
        hipLaunchKernelGGL(alex_pinecones_classic_kernel<false>, dim3(E), dim3(512), 0, st, *p, H, W, NW, grid_in,
                           grid_out, age_out, veg, den, wind_index, s_cdf, rng_step, counts, scratch);
    }
    GCA_CHECK_LAUNCH("alex_pinecones_classic");
    return GCA_OK;
}
