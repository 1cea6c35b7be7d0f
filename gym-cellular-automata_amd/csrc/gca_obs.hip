// gca_obs.hip — observation builders of the Advanced bulldozer env on gfx950.
// Reference: MDP.build_observation_on_extensions / grid_to_rgb_with_extensions / grid_to_rgb
//            (advanced_bulldozer.py:988-1101), apply_blur / apply_visibility / transform_grid /
//            apply_extensions (bulldozer/utils/extension_utils.py:89-196), the reset observation
//            (advanced_bulldozer.py:401-411).
//
// Grid: one workgroup (256 threads) per (env, block of up to OBS_RB = 16 rows):
//   A. (step mode, only when an extension channel can be non-zero) the first row holding a positive
//      extension value — the reference's `has_extension` is a vmap over the ROWS of the channel-last
//      (H, W, 3 + n_ext) stack, and the row index found is then used as the channel index (clamped to
//      the last channel, like JAX's out-of-bounds gather). Every block of the env repeats this scan;
//      it normally ends at row 0;
//   B. the block's rows (+1 halo row each side) and its dousing rows staged in LDS (all loads in one
//      batch; the render rounds then read LDS only), then per cell the display
//      value and its f32 RGB: empty/tree/fire colour of the pre-step day/night, the water tint blended
//      in where dousing_count == 1 (rgb*0.25 + tint*0.75 — exact in f32 for these integer colours, so
//      the order of the reference's ops cannot matter), the position colour on the bulldozer's cell;
//      4 cells per thread, 3 float4 stores. Optionally the u8 channel stack itself.
// HBM bytes per cell: grid 1 + dousing 1 read, 12 written (14 B/cell).
// Cell transforms (values are the env's integer codes):
//   blur(g)[r,c] = round(S / 9), S = 3x3 sum with edge padding (the reference's f32 sum of
//   (1/9)*(g/3) times 3 is S/9 to within 1e-6 relative; S/9 is never within 0.05 of a .5 tie for
//   S < 5000, so the integer rounding floor((2S + 9) / 18) is the reference's result);
//   vis(v) = (v == 3 && !is_night) ? 0 : v   (the reference's literal 3, extension_utils.py:93).
#include "gca_common.h"

// Measured choices (the A/B variants were removed after the measurement):
//   wave-local RGB transposition (each wave stores its own 3 KiB, no barriers per round; r01p: 0.713 vs 0.722 ms for
//   the block-wide one, two block-wide buffers with one barrier per round 1.08 ms); non-temporal RGB stores (r01i:
//   1.07 vs 1.10 ms); full rounds batched as 3 LDS reads, one wait, 3 stores
constexpr int OBS_RB = 16;   // rows per workgroup (r02f at W = 256: 8 / 12 / 16 / 32 rows -> 0.84 / 0.70 / 0.64 / 0.70 ms)
constexpr int OBS_PRE = 5;   // staged 16-B chunks per thread issued before the display scan (W = 256, 32 rows: 4.1)
constexpr int OBS_PLAIN = 1; // chunks of 256 cells per wave in adv_obs_plain_kernel (r02k: 1 / 8 / 16 chunks ->
                             // 0.633 / 0.726 / 0.726 ms, the staged kernel 0.688 ms)

namespace {

// blur of cell (lr, c) from the LDS copy of the block's rows (staged row lr+1 <-> grid row r), edge padding
__device__ __forceinline__ int blur_lds(const uint8_t* __restrict__ T, int W, int lr, int c) {
    int s = 0;
#pragma unroll
    for (int dr = 0; dr < 3; ++dr) {
        const uint8_t* row = T + (lr + dr) * W;
#pragma unroll
        for (int dc = -1; dc <= 1; ++dc) s += row[min(max(c + dc, 0), W - 1)];
    }
    return (2 * s + 9) / 18;
}
// the same from global memory (display selection scan)
__device__ __forceinline__ int blur_at(const uint8_t* __restrict__ g, int H, int W, int r, int c) {
    int s = 0;
#pragma unroll
    for (int dr = -1; dr <= 1; ++dr) {
        const int rr = min(max(r + dr, 0), H - 1);
#pragma unroll
        for (int dc = -1; dc <= 1; ++dc) s += g[(int64_t)rr * W + min(max(c + dc, 0), W - 1)];
    }
    return (2 * s + 9) / 18;
}

__device__ __forceinline__ int transform(int raw, int blurred, bool night, int skip_vis, int skip_blur) {
    int v = skip_blur ? raw : blurred;
    if (!skip_vis && v == 3 && !night) v = 0;
    return v;
}

struct ObsCfg {
    bool need_blur;  // some channel in use blurs
    uint32_t on;     // active extension channels
    bool night;      // pre-step day/night
};

// base channel + active extension channels of one cell from its raw value and blur
__device__ __forceinline__ int ext_value(const gca_obs_params& p, const ObsCfg& k, int i, int raw, int bl) {
    return ((k.on >> i) & 1u) ? transform(raw, bl, k.night, p.ext_skip_visibility[i], p.ext_skip_blur[i]) : 0;
}

__device__ __forceinline__ int colour_kind(const gca_obs_params& p, int v, bool at_pos) {
    return at_pos ? 3 : (v == p.tree ? 1 : (v == p.fire ? 2 : 0));
}
// colour of kind k (empty / tree / fire / position) with the dousing tint
__device__ __forceinline__ void render_kind(const gca_obs_params& p, float* __restrict__ out, int k, int dous,
                                            bool night) {
    const float(*col)[3] = night ? p.color_night : p.color_day;
    const bool at_pos = k == 3;
    float rgb[3] = {col[k][0], col[k][1], col[k][2]};
    if (!at_pos && dous > 0) {
        const float s = dous == 1 ? 0.75f : 0.0f;
        const float* tint = night ? p.tint_night : p.tint_day;
#pragma unroll
        for (int j = 0; j < 3; ++j) rgb[j] = __fadd_rn(__fmul_rn(rgb[j], __fsub_rn(1.0f, s)), __fmul_rn(tint[j], s));
    }
    out[0] = rgb[0];
    out[1] = rgb[1];
    out[2] = rgb[2];
}
__device__ __forceinline__ void render(const gca_obs_params& p, float* __restrict__ out, int v, int dous, bool night,
                                       bool at_pos) {
    render_kind(p, out, colour_kind(p, v, at_pos), dous, night);
}

// Grid: (env, block of RB rows); 256 threads. The display selection (a scan from row 0 that normally
// stops at the first row) is recomputed by every block of the env instead of a separate pass; the
// block's rows plus one halo row on each side are staged in LDS for the blur; W % 4 == 0 renders
// 4 cells per thread (3 float4 stores, 48-B aligned).
__global__ __launch_bounds__(256) void adv_observation_kernel(gca_obs_params p, int mode, int H, int W, int RB,
                                                              int blocks_per_env, const uint8_t* __restrict__ grid,
                                                              const uint8_t* __restrict__ dousing,
                                                              const int32_t* __restrict__ pos,
                                                              const int32_t* __restrict__ is_night,
                                                              const int32_t* __restrict__ time_step,
                                                              const int32_t* __restrict__ action, int action_stride,
                                                              float* __restrict__ rgb, uint8_t* __restrict__ channels,
                                                              const uint8_t* __restrict__ env_mask) {
    extern __shared__ uint8_t T[];  // [(RB + 2) * W] grid rows r0-1 .. r0+RB (edge-clamped), then [RB * W] dousing
    uint8_t* D = T + (RB + 2) * W;
    const int e = blockIdx.x / blocks_per_env;
    if (env_mask && !env_mask[e]) return;  // whole block: envs outside the mask keep their observation
    const int r0 = (blockIdx.x - e * blocks_per_env) * RB;
    const int rows = min(RB, H - r0);
    const int64_t HW = (int64_t)H * W;
    const uint8_t* g = grid + e * HW;
    const uint8_t* du = dousing ? dousing + e * HW : nullptr;
    ObsCfg k;
    // the observation uses the PRE-step is_night; the env step toggled it when time_step % day_length == 0
    k.night = is_night[e] != 0;
    if (time_step && p.day_length > 0 && time_step[e] % p.day_length == 0) k.night = !k.night;
    const int pr = pos[2 * e], pc = pos[2 * e + 1];
    k.on = 0u;
    if (mode == 0 && p.enable_extensions && action && action_stride >= 3 && p.n_choices > 0) {
        const int choice = min(max(action[(int64_t)e * action_stride + 2], 0), min(p.n_choices, 8) - 1);
        for (int i = 0; i < p.n_ext; ++i) k.on |= (p.ext_lookup[choice][i] != 0 ? 1u : 0u) << i;
    }
    k.need_blur = mode == 0 && p.should_transform != 0;
    for (int i = 0; i < p.n_ext; ++i) k.need_blur |= ((k.on >> i) & 1u) && !p.ext_skip_blur[i];
    const int nch = 3 + p.n_ext;

    // ---- staging loads first (W % 16 == 0, 16-B aligned: the production shape): up to OBS_PRE 16-B
    //      chunks per thread go to registers now and to LDS after the display scan, so the scan's loads and
    //      these overlap instead of queueing one HBM round trip behind the other at the head of every block
    const bool stage_all = (W & 3) == 0;  // the 4-cells-per-thread path reads both arrays from LDS
    const bool do_stage = mode == 0 && (stage_all || k.need_blur);
    const bool al16 = ((((uintptr_t)grid) | ((uintptr_t)dousing)) & 15u) == 0;
    const bool fast16 = do_stage && (W & 15) == 0 && al16;
    const int w16 = W >> 4;
    const int ng16 = (rows + 2) * w16, nd16 = du ? rows * w16 : 0;
    const int nst = fast16 ? ng16 + nd16 : 0;
    // byte offset of staged 16-B chunk idx (grid rows r0-1 .. r0+rows edge-clamped, then the dousing rows)
    // from g; the dousing array is addressed relative to the grid (same env, same layout)
    const int64_t dgap = du ? (int64_t)(du - g) : 0;
    auto src16 = [&](int idx) -> int64_t {
        const int lr = idx / w16, cq = idx - lr * w16;
        const int r = min(max(r0 - 1 + lr, 0), H - 1);
        return idx < ng16 ? (int64_t)r * W + 16 * cq : dgap + (int64_t)r0 * W + 16 * (int64_t)(idx - ng16);
    };
    uint4 pre[OBS_PRE];
#pragma unroll
    for (int j = 0; j < OBS_PRE; ++j) {  // unconditional loads of clamped chunks: pre stays in VGPRs
        const int idx = min((int)threadIdx.x + 256 * j, max(nst - 1, 0));
        pre[j] = nst ? *reinterpret_cast<const uint4*>(g + src16(idx)) : make_uint4(0u, 0u, 0u, 0u);
    }

    // ---- display selection (see the header comment in include/gca.h). Every wave scans on its own (the
    //      result is a function of the grid alone, so all waves agree): no workgroup barrier per scanned row
    const int lane = (int)threadIdx.x & 63;
    int sel = -1;     // mode 0: -1 = base channel, else the extension channel shown everywhere
    int col_sel = 0;  // mode 1: column of the raw grid shown
    if (mode == 0 && k.on) {
        bool scan_blur = false;
        for (int i = 0; i < p.n_ext; ++i) scan_blur |= ((k.on >> i) & 1u) && !p.ext_skip_blur[i];
        int fv = -1;
        for (int r = 0; r < H && fv < 0; ++r) {
            int any = 0;
            if ((W & 3) == 0) {
                for (int c4 = 4 * lane; c4 < W; c4 += 256) {
                    const uint32_t w = *reinterpret_cast<const uint32_t*>(g + (int64_t)r * W + c4);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int raw = (int)((w >> (8 * j)) & 0xFFu);
                        const int bl = scan_blur ? blur_at(g, H, W, r, c4 + j) : raw;
                        for (int i = 0; i < p.n_ext; ++i) any |= ext_value(p, k, i, raw, bl) > 0;
                    }
                }
            } else {
                for (int c = lane; c < W; c += 64) {
                    const int raw = g[(int64_t)r * W + c];
                    const int bl = scan_blur ? blur_at(g, H, W, r, c) : raw;
                    for (int i = 0; i < p.n_ext; ++i) any |= ext_value(p, k, i, raw, bl) > 0;
                }
            }
            if (__ballot(any) != 0ull) fv = r;
        }
        if (fv >= 0) sel = min(fv, p.n_ext - 1);
    } else if (mode == 1 && W > 3) {
        int fv = -1;
        for (int r = 0; r < H && fv < 0; ++r) {
            int any = 0;
            for (int c = 3 + lane; c < W; c += 64) any |= g[(int64_t)r * W + c] > 0;
            if (__ballot(any) != 0ull) fv = r;
        }
        col_sel = fv >= 0 ? 3 + min(fv, W - 4) : 0;
    }

    if (mode == 1) {  // rgb[r][c] = colour(grid[c][col_sel]) (+ dousing of (r, c), position)
        for (int idx = threadIdx.x; idx < rows * W; idx += blockDim.x) {
            const int lr = idx / W, c = idx - lr * W, r = r0 + lr;
            const int64_t cell = (int64_t)r * W + c;
            render(p, rgb + (e * HW + cell) * 3, g[(int64_t)c * W + col_sel], du ? du[cell] : 0, k.night,
                   r == pr && c == pc);
        }
        return;
    }

    // ---- stage grid rows [r0 - 1, r0 + rows] (clamped: edge padding, for the blur) and the block's dousing
    //      rows in LDS: the render rounds below then read LDS only and never wait on HBM between their stores
    // the block's 12 colours (kind x dousing 0 / 1 / >= 2) in LDS: the render rounds then index LDS instead of
    // the kernel arguments (a per-lane index into them is a vector memory load, whose wait would also drain
    // the previous round's stores)
    __shared__ float4 COLT[12];
    if (stage_all && threadIdx.x < 12) {
        float c3[3];
        render_kind(p, c3, (int)threadIdx.x / 3, (int)threadIdx.x % 3, k.night);
        COLT[threadIdx.x] = make_float4(c3[0], c3[1], c3[2], 0.0f);
    }
    if (do_stage) {
        if (fast16) {
#pragma unroll
            for (int j = 0; j < OBS_PRE; ++j) {
                const int idx = (int)threadIdx.x + 256 * j;
                if (idx < ng16 + nd16) reinterpret_cast<uint4*>(idx < ng16 ? T : D - 16 * ng16)[idx] = pre[j];
            }
            for (int idx = (int)threadIdx.x + 256 * OBS_PRE; idx < ng16 + nd16; idx += 256)
                reinterpret_cast<uint4*>(idx < ng16 ? T : D - 16 * ng16)[idx] =
                    *reinterpret_cast<const uint4*>(g + src16(idx));
        } else if (stage_all) {
            const int wq = W >> 2;
            const int ng = (rows + 2) * wq, nd = du ? rows * wq : 0;
            for (int idx = threadIdx.x; idx < ng + nd; idx += blockDim.x) {
                if (idx < ng) {
                    const int lr = idx / wq, cq = idx - lr * wq;
                    const int r = min(max(r0 - 1 + lr, 0), H - 1);
                    reinterpret_cast<uint32_t*>(T)[lr * wq + cq] = reinterpret_cast<const uint32_t*>(g + (int64_t)r * W)[cq];
                } else {
                    const int j = idx - ng;
                    reinterpret_cast<uint32_t*>(D)[j] = reinterpret_cast<const uint32_t*>(du + (int64_t)r0 * W)[j];
                }
            }
        } else {
            for (int idx = threadIdx.x; idx < (rows + 2) * W; idx += blockDim.x) {
                const int lr = idx / W, c = idx - lr * W;
                T[idx] = g[(int64_t)min(max(r0 - 1 + lr, 0), H - 1) * W + c];
            }
        }
    }
    __syncthreads();

    auto values_of = [&](int raw, int bl, int* extv) -> int {
        const int base = p.should_transform ? transform(raw, bl, k.night, 0, 0) : raw;
        for (int i = 0; i < GCA_OBS_MAX_EXT; ++i) extv[i] = i < p.n_ext ? ext_value(p, k, i, raw, bl) : 0;
        return base;
    };
    auto cell_value = [&](int lr, int c, int raw, int* extv) -> int {
        return values_of(raw, k.need_blur ? blur_lds(T, W, lr, c) : raw, extv);
    };
    if ((W & 3) == 0) {
        // 256 threads x 4 cells per round; the 12 floats of each thread go through LDS so that every store
        // instruction writes 1 KiB of contiguous RGB (the rows of a block are contiguous in HBM)
        __shared__ float4 OUT4s[256 * 3];
        const int wq = W >> 2;
        for (int base_q = 0; base_q < rows * wq; base_q += 256) {
            float4* OUT4 = OUT4s;
            const int idx = base_q + (int)threadIdx.x;
            if (idx < rows * wq) {
                const int lr = idx / wq, c0 = (idx - lr * wq) * 4, r = r0 + lr;
                const int64_t cell0 = (int64_t)r * W + c0;
                const uint32_t gw = *reinterpret_cast<const uint32_t*>(T + (lr + 1) * W + c0);
                const uint32_t dw = du ? *reinterpret_cast<const uint32_t*>(D + lr * W + c0) : 0u;
                // blur of the 4 cells: column sums of columns c0-1 .. c0+4 over the 3 staged rows
                // (one aligned word + the two edge bytes per row; edge padding at the grid border)
                int bl4[4] = {0, 0, 0, 0};
                if (k.need_blur) {
                    int cs[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
                    for (int dr = 0; dr < 3; ++dr) {
                        const uint8_t* row = T + (lr + dr) * W;
                        const uint32_t w = reinterpret_cast<const uint32_t*>(row)[c0 >> 2];
                        cs[0] += c0 > 0 ? row[c0 - 1] : (int)(w & 0xFF);
#pragma unroll
                        for (int j = 0; j < 4; ++j) cs[1 + j] += (int)((w >> (8 * j)) & 0xFF);
                        cs[5] += c0 + 4 < W ? row[c0 + 4] : (int)(w >> 24);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) bl4[j] = (2 * (cs[j] + cs[j + 1] + cs[j + 2]) + 9) / 18;
                }
                float out[12];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int raw = (gw >> (8 * j)) & 0xFF;
                    int extv[GCA_OBS_MAX_EXT];
                    const int base = values_of(raw, k.need_blur ? bl4[j] : raw, extv);
                    int v = base;
#pragma unroll
                    for (int i = 0; i < GCA_OBS_MAX_EXT; ++i)
                        if (sel == i) v = extv[i];
                    const float4 cl = COLT[3 * colour_kind(p, v, r == pr && c0 + j == pc) +
                                           (int)min((dw >> (8 * j)) & 0xFFu, 2u)];
                    out[3 * j] = cl.x;
                    out[3 * j + 1] = cl.y;
                    out[3 * j + 2] = cl.z;
                    if (channels) {
                        uint8_t* ch = channels + (e * HW + cell0 + j) * nch;
                        ch[0] = (uint8_t)base;
                        ch[1] = 0;
                        ch[2] = 0;
                        for (int i = 0; i < p.n_ext; ++i) ch[3 + i] = (uint8_t)extv[i];
                    }
                }
                OUT4[3 * threadIdx.x + 0] = make_float4(out[0], out[1], out[2], out[3]);
                OUT4[3 * threadIdx.x + 1] = make_float4(out[4], out[5], out[6], out[7]);
                OUT4[3 * threadIdx.x + 2] = make_float4(out[8], out[9], out[10], out[11]);
            }
            // a wave's 64 threads own 256 consecutive cells = 3 KiB of contiguous RGB: the transposition stays
            // inside the wave (LDS operations of one wave complete in order), so no workgroup barrier
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int n4 = 3 * min(256, rows * wq - base_q);
            float4* dst = reinterpret_cast<float4*>(rgb + (e * HW + (int64_t)r0 * W + 4 * (int64_t)base_q) * 3);
            typedef float f4v __attribute__((ext_vector_type(4)));
            if (n4 == 768) {
                // a full round (all but a block's ragged last one): the three LDS reads issue back to back, one
                // wait, then the three 1-KiB stores — not read / wait / store three times over
                const int q0 = 192 * ((int)threadIdx.x >> 6) + ((int)threadIdx.x & 63);
                const float4 v0 = OUT4[q0], v1 = OUT4[q0 + 64], v2 = OUT4[q0 + 128];
                __builtin_nontemporal_store((f4v){v0.x, v0.y, v0.z, v0.w}, reinterpret_cast<f4v*>(dst + q0));
                __builtin_nontemporal_store((f4v){v1.x, v1.y, v1.z, v1.w}, reinterpret_cast<f4v*>(dst + q0 + 64));
                __builtin_nontemporal_store((f4v){v2.x, v2.y, v2.z, v2.w}, reinterpret_cast<f4v*>(dst + q0 + 128));
            } else
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int q4 = 192 * ((int)threadIdx.x >> 6) + ((int)threadIdx.x & 63) + 64 * j;
                if (q4 < n4) {
                    const float4 v = OUT4[q4];
                    __builtin_nontemporal_store((f4v){v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(dst + q4));
                }
            }
            // this round's LDS reads before the next round's writes (same wave)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    } else {
        for (int idx = threadIdx.x; idx < rows * W; idx += blockDim.x) {
            const int lr = idx / W, c = idx - lr * W, r = r0 + lr;
            const int64_t cell = (int64_t)r * W + c;
            int extv[GCA_OBS_MAX_EXT];
            const int base = cell_value(lr, c, g[cell], extv);
            int v = base;
            for (int i = 0; i < p.n_ext; ++i)
                if (sel == i) v = extv[i];
            render(p, rgb + (e * HW + cell) * 3, v, du ? du[cell] : 0, k.night, r == pr && c == pc);
            if (channels) {
                uint8_t* ch = channels + (e * HW + cell) * nch;
                ch[0] = (uint8_t)base;
                ch[1] = 0;
                ch[2] = 0;
                for (int i = 0; i < p.n_ext; ++i) ch[3 + i] = (uint8_t)extv[i];
            }
        }
    }
}

// Plain step observation (no extension channels, no grid transform — the env's default, enable_extensions = False):
// every cell's colour depends on its own grid and dousing bytes (and the bulldozer's position) only, so there is no
// halo and nothing to stage. Each wave renders CW chunks of 256 consecutive cells of one env (64 lanes x 4 cells: one
// dword of grid and one of dousing per lane per chunk, all CW chunks' loads issued up front), looks the colours up in a
// per-block LDS table (day and night x kind x dousing 0 / 1 / >= 2, built by the same `render_kind` arithmetic) and
// writes each chunk's 3 KiB of RGB through its own LDS slice so that every non-temporal store instruction writes 1 KiB
// contiguous. Straight-line code (CW is a template constant): hipcc's counted waits then let the stores of earlier
// chunks stay in flight while later chunks render (a rolled loop made it wait for them: 0.65 ms per frame).
// Requires (H*W / 256) % CW == 0 (a wave's chunks lie in one env; checked on the host).
template <int CW>
__global__ __launch_bounds__(256) void adv_obs_plain_kernel(gca_obs_params p, int64_t chunks, int chunks_per_env,
                                                            int W, const uint8_t* __restrict__ grid,
                                                            const uint8_t* __restrict__ dousing,
                                                            const int32_t* __restrict__ pos,
                                                            const int32_t* __restrict__ is_night,
                                                            const int32_t* __restrict__ time_step,
                                                            float* __restrict__ rgb, const uint8_t* __restrict__ env_mask) {
    __shared__ float4 COL[2][12];
    __shared__ float4 OUT4s[4][192];
    if (threadIdx.x < 24) {
        float c3[3];
        const int nt = (int)threadIdx.x / 12, i = (int)threadIdx.x % 12;
        render_kind(p, c3, i / 3, i % 3, nt != 0);
        COL[nt][i] = make_float4(c3[0], c3[1], c3[2], 0.0f);
    }
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = (int)threadIdx.x & 63;
    float4* OUT4 = OUT4s[wave];
    typedef float f4v __attribute__((ext_vector_type(4)));
    const int64_t c0 = ((int64_t)blockIdx.x * 4 + wave) * CW;  // this wave's chunks [c0, c0 + CW)
    if (c0 >= chunks) return;
    const int e = (int)(c0 / chunks_per_env);  // wave-uniform: scalar loads of the env's values
    if (env_mask && !env_mask[e]) return;
    bool night = is_night[e] != 0;  // the PRE-step is_night (see adv_observation_kernel)
    if (time_step && p.day_length > 0 && time_step[e] % p.day_length == 0) night = !night;
    const int64_t pcell = (int64_t)pos[2 * e] * W + pos[2 * e + 1];
    const float4* colt = COL[night ? 1 : 0];
    const uint8_t* dsrc = dousing ? dousing : grid;  // no dousing: read the grid again and mask it (no branch)
    const uint32_t dmask = dousing ? ~0u : 0u;
    uint32_t gw[CW], dw[CW];
#pragma unroll
    for (int i = 0; i < CW; ++i) {
        gw[i] = *reinterpret_cast<const uint32_t*>(grid + 256 * (c0 + i) + 4 * lane);
        dw[i] = *reinterpret_cast<const uint32_t*>(dsrc + 256 * (c0 + i) + 4 * lane);
    }
#pragma unroll
    for (int i = 0; i < CW; ++i) {
        const int64_t c = c0 + i;
        const int64_t cell0 = 256 * (c - (int64_t)e * chunks_per_env) + 4 * lane;  // cell of this lane within the env
        const uint32_t g4 = gw[i], d4 = dw[i] & dmask;
        float out[12];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int v = (int)((g4 >> (8 * j)) & 0xFFu);
            const int kind = colour_kind(p, v, cell0 + j == pcell);
            const float4 cl = colt[3 * kind + (int)min((d4 >> (8 * j)) & 0xFFu, 2u)];
            out[3 * j] = cl.x;
            out[3 * j + 1] = cl.y;
            out[3 * j + 2] = cl.z;
        }
        OUT4[3 * lane + 0] = make_float4(out[0], out[1], out[2], out[3]);
        OUT4[3 * lane + 1] = make_float4(out[4], out[5], out[6], out[7]);
        OUT4[3 * lane + 2] = make_float4(out[8], out[9], out[10], out[11]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float4 v0 = OUT4[lane], v1 = OUT4[lane + 64], v2 = OUT4[lane + 128];
        f4v* dst = reinterpret_cast<f4v*>(rgb + 768 * c);
        __builtin_nontemporal_store((f4v){v0.x, v0.y, v0.z, v0.w}, dst + lane);
        __builtin_nontemporal_store((f4v){v1.x, v1.y, v1.z, v1.w}, dst + lane + 64);
        __builtin_nontemporal_store((f4v){v2.x, v2.y, v2.z, v2.w}, dst + lane + 128);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // this chunk's LDS reads before the next one's writes
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// colour table of the fused step observation (gca_alex_step_packed_rgb): [night][kind][dousing 0 / 1] as float4
__global__ void obs_color_table_kernel(gca_obs_params p, float4* __restrict__ table) {
    const int i = (int)threadIdx.x;
    if (i >= 12) return;
    float c3[3];
    render_kind(p, c3, (i % 6) / 2, i % 2, i >= 6);
    table[i] = make_float4(c3[0], c3[1], c3[2], 0.0f);
}

// the bulldozer's pixel (grid_to_rgb's .at[position].set, advanced_bulldozer.py:1095-1099) over a frame the fused step
// wrote: position colour of the PRE-step day / night (the step toggled is_night when time_step % day_length == 0)
__global__ void obs_position_kernel(gca_obs_params p, int E, int H, int W, const int32_t* __restrict__ pos,
                                    const int32_t* __restrict__ is_night, const int32_t* __restrict__ time_step,
                                    float* __restrict__ rgb) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    bool night = is_night[e] != 0;
    if (time_step && p.day_length > 0 && time_step[e] % p.day_length == 0) night = !night;
    const int r = pos[2 * e], c = pos[2 * e + 1];
    if (r < 0 || r >= H || c < 0 || c >= W) return;  // JAX drops out-of-bounds updates
    float c3[3];
    render_kind(p, c3, 3, 0, night);
    float* o = rgb + (((int64_t)e * H + r) * W + c) * 3;
    o[0] = c3[0];
    o[1] = c3[1];
    o[2] = c3[2];
}

}  // namespace

extern "C" int gca_obs_color_table(const gca_obs_params* p, float* table, void* stream) {
    GCA_CHECK_ARG(p && table && ((uintptr_t)table & 15u) == 0, "obs_color_table: bad arguments");
    hipLaunchKernelGGL(obs_color_table_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, *p,
                       reinterpret_cast<float4*>(table));
    GCA_CHECK_LAUNCH("obs_color_table");
    return GCA_OK;
}

extern "C" int gca_obs_position(const gca_obs_params* p, int E, int H, int W, const int32_t* pos,
                                const int32_t* is_night, const int32_t* time_step, float* rgb, void* stream) {
    GCA_CHECK_ARG(p && pos && is_night && rgb && E > 0 && H > 0 && W > 0, "obs_position: bad arguments");
    hipLaunchKernelGGL(obs_position_kernel, dim3((E + 255) / 256), dim3(256), 0, (hipStream_t)stream, *p, E, H, W, pos,
                       is_night, time_step, rgb);
    GCA_CHECK_LAUNCH("obs_position");
    return GCA_OK;
}

extern "C" int gca_adv_observation(const gca_obs_params* p, int mode, int E, int H, int W, const uint8_t* grid,
                                   const uint8_t* dousing, const int32_t* pos, const int32_t* is_night,
                                   const int32_t* time_step, const int32_t* action, int action_stride, float* rgb,
                                   uint8_t* channels, const uint8_t* env_mask, void* stream) {
    GCA_CHECK_ARG(p && grid && pos && is_night && rgb && E > 0 && H > 0 && W > 0, "adv_observation: bad arguments");
    GCA_CHECK_ARG(mode == 0 || mode == 1, "adv_observation: mode is 0 (step) or 1 (reset)");
    GCA_CHECK_ARG(p->n_ext >= 0 && p->n_ext <= GCA_OBS_MAX_EXT, "adv_observation: 0..4 extension channels");
    GCA_CHECK_ARG(mode == 0 || H == W, "adv_observation: the reset observation needs a square grid (reference broadcast)");
    GCA_CHECK_ARG(mode == 0 || channels == nullptr, "adv_observation: no channel stack in reset mode");
    GCA_CHECK_ARG(W <= 16384, "adv_observation: W <= 16384");
    GCA_CHECK_ARG(((uintptr_t)rgb & 15u) == 0 && ((uintptr_t)grid & 3u) == 0 && ((uintptr_t)dousing & 3u) == 0,
                  "adv_observation: rgb must be 16-B and grid/dousing 4-B aligned");
    // rows per block; (2 RB + 2) * W bytes of dynamic LDS (grid + dousing), at most 48 KiB
    const int64_t HW = (int64_t)H * W;
    constexpr int CWP = OBS_PLAIN;  // chunks of 256 cells per wave
    if (CWP > 0 && mode == 0 && !p->enable_extensions && !p->should_transform && channels == nullptr &&
        HW % 256 == 0 && (HW / 256) % (CWP > 0 ? CWP : 1) == 0) {
        const int64_t chunks = (int64_t)E * (HW / 256);
        const int64_t waves = chunks / (CWP > 0 ? CWP : 1);
        hipLaunchKernelGGL(adv_obs_plain_kernel<(CWP > 0 ? CWP : 1)>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                           (hipStream_t)stream, *p, chunks, (int)(HW / 256), W, grid, dousing, pos, is_night, time_step,
                           rgb, env_mask);
        GCA_CHECK_LAUNCH("adv_obs_plain");
        return GCA_OK;
    }
    const int RB = max(1, min(OBS_RB, 24576 / W - 1));
    const int bpe = (H + RB - 1) / RB;
    hipLaunchKernelGGL(adv_observation_kernel, dim3((unsigned)((int64_t)E * bpe)), dim3(256), (size_t)(2 * RB + 2) * W,
                       (hipStream_t)stream, *p, mode, H, W, RB, bpe, grid, dousing, pos, is_night, time_step, action,
                       action_stride, rgb, channels, env_mask);
    GCA_CHECK_LAUNCH("adv_observation");
    return GCA_OK;
}
