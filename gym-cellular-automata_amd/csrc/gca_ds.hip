// gca_ds.hip — Drossel–Schwabl forest fire (helicopter env CA), ForestFire.update
// (ca_DrosselSchwabl.py:32-66) on gfx950.
//
// The reference walks the grid row-major and, per cell:
//   TREE with a FIRE neighbour (Moore, padding = EMPTY) -> FIRE           (no draw)
//   TREE otherwise -> FIRE iff u < thr_fire                               (one f64 draw)
//   EMPTY -> TREE iff u < thr_tree                                        (one f64 draw)
//   FIRE -> EMPTY                                                         (no draw)
// with u from op.np_random (Generator.choice with p = [p, 1-p]: one random() per call,
// True iff u < cdf[0]; thr_* = that cdf[0], computed on the host exactly as numpy does).
// Exact-stream mode: uniforms[uniform_offset[e] + j] is the j-th draw of env e; a
// workgroup per env scans the draw flags in row-major order to find j for each cell,
// so the device consumes the same stream as the reference.
// Philox mode (uniforms == NULL): u = 53-bit double of Philox((cell, env_offset+e, step, DSCE)).
#include "gca_common.h"

namespace {

__device__ __forceinline__ bool ds_has_fire_nb(const uint8_t* __restrict__ g, int r, int c, int H, int W, int fire) {
#pragma unroll
    for (int dr = -1; dr <= 1; ++dr) {
#pragma unroll
        for (int dc = -1; dc <= 1; ++dc) {
            if (dr == 0 && dc == 0) continue;
            const int rr = r + dr, cc = c + dc;
            if (rr >= 0 && rr < H && cc >= 0 && cc < W && g[rr * W + cc] == fire) return true;
        }
    }
    return false;
}

// 0 = no draw, 1 = draw (tree w/o burning neighbour, or empty)
__device__ __forceinline__ int ds_draw_flag(const uint8_t* __restrict__ g, int cell, int H, int W, int empty, int tree,
                                            int fire) {
    const int x = g[cell];
    if (x == tree) return ds_has_fire_nb(g, cell / W, cell % W, H, W, fire) ? 0 : 1;
    return x == empty ? 1 : 0;
}

__device__ __forceinline__ int block_excl_scan(int v, int* sh, int& total) {
    // 256 threads = 4 waves: wave inclusive scan via shuffles, then wave offsets in LDS
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) sh[wave] = x;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wave; ++w) base += sh[w];
    total = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
    return base + x - v;
}

__global__ __launch_bounds__(256) void ds_count_kernel(const uint8_t* __restrict__ grid, int H, int W, int empty,
                                                       int tree, int fire, int32_t* __restrict__ n_draws) {
    __shared__ int sh[4];
    const int e = blockIdx.x;
    const uint8_t* g = grid + (int64_t)e * H * W;
    int acc = 0;
    for (int base = 0; base < H * W; base += 256) {
        const int cell = base + threadIdx.x;
        acc += cell < H * W ? ds_draw_flag(g, cell, H, W, empty, tree, fire) : 0;
    }
    int total;
    block_excl_scan(acc, sh, total);
    if (threadIdx.x == 0) n_draws[e] = total;
}

__global__ __launch_bounds__(256) void ds_step_kernel(const uint8_t* __restrict__ grid_in, uint8_t* __restrict__ grid_out,
                                                      int H, int W, int empty, int tree, int fire,
                                                      const double* __restrict__ thr, const double* __restrict__ uniforms,
                                                      const int64_t* __restrict__ uoff, uint32_t k0, uint32_t k1,
                                                      const uint32_t* __restrict__ rng_step, int env_offset,
                                                      int32_t* __restrict__ counts) {
    __shared__ int sh[4];
    const int e = blockIdx.x;
    const int64_t HW = (int64_t)H * W;
    const uint8_t* g = grid_in + e * HW;
    uint8_t* o = grid_out + e * HW;
    const double thr_fire = thr[2 * e], thr_tree = thr[2 * e + 1];
    const uint32_t step = rng_step ? rng_step[e] : 0u;
    int64_t consumed = uniforms ? uoff[e] : 0;
    int cE = 0, cT = 0, cF = 0;
    for (int base = 0; base < HW; base += 256) {
        const int cell = base + threadIdx.x;
        const bool in = cell < HW;
        const int flag = in ? ds_draw_flag(g, cell, H, W, empty, tree, fire) : 0;
        int total;
        const int j = block_excl_scan(flag, sh, total);
        if (in) {
            const int x = g[cell];
            int nx = x;
            if (x == fire) {
                nx = empty;
            } else if (x == tree && !flag) {
                nx = fire;
            } else if (flag) {
                double u;
                if (uniforms) {
                    u = uniforms[consumed + j];
                } else {
                    const u32x4 rx = philox4x32_10(u32x4{(uint32_t)cell, (uint32_t)(env_offset + e), step, GCA_TAG_DS_CELL}, k0, k1);
                    u = u01_f64(rx.x, rx.y);
                }
                if (x == tree) nx = (u < thr_fire) ? fire : tree;
                else nx = (u < thr_tree) ? tree : empty;
            }
            o[cell] = (uint8_t)nx;
            cE += nx == empty;
            cT += nx == tree;
            cF += nx == fire;
        }
        consumed += total;
    }
    if (counts) {
        atomicAdd(counts + 3 * e + 0, cE);
        atomicAdd(counts + 3 * e + 1, cT);
        atomicAdd(counts + 3 * e + 2, cF);
    }
}

}  // namespace

extern "C" int gca_ds_count_draws(const uint8_t* grid, int E, int H, int W, int empty, int tree, int fire,
                                  int32_t* n_draws, void* stream) {
    GCA_CHECK_ARG(grid && n_draws && E > 0 && H > 0 && W > 0, "ds_count_draws: bad arguments");
    GCA_CHECK_ARG((int64_t)H * W < (1 << 30), "ds_count_draws: grid too large");
    hipLaunchKernelGGL(ds_count_kernel, dim3(E), dim3(256), 0, (hipStream_t)stream, grid, H, W, empty, tree, fire,
                       n_draws);
    GCA_CHECK_LAUNCH("ds_count_draws");
    return GCA_OK;
}

extern "C" int gca_ds_step(const uint8_t* grid_in, uint8_t* grid_out, int E, int H, int W, int empty, int tree,
                           int fire, const double* thresholds, const double* uniforms, const int64_t* uniform_offset,
                           uint64_t seed, const uint32_t* rng_step, int env_offset, int32_t* counts, void* stream) {
    GCA_CHECK_ARG(grid_in && grid_out && thresholds && E > 0 && H > 0 && W > 0, "ds_step: bad arguments");
    GCA_CHECK_ARG(grid_in != grid_out, "ds_step: in-place update is not supported");
    GCA_CHECK_ARG(!uniforms || uniform_offset, "ds_step: uniforms need uniform_offset");
    GCA_CHECK_ARG((int64_t)H * W < (1 << 30), "ds_step: grid too large");
    hipStream_t st = (hipStream_t)stream;
    if (counts && hipMemsetAsync(counts, 0, sizeof(int32_t) * 3 * (size_t)E, st) != hipSuccess) {
        gca_set_error("ds_step: counts memset failed");
        return GCA_ERR_HIP;
    }
    hipLaunchKernelGGL(ds_step_kernel, dim3(E), dim3(256), 0, st, grid_in, grid_out, H, W, empty, tree, fire, thresholds,
                       uniforms, uniform_offset, (uint32_t)seed, (uint32_t)(seed >> 32), rng_step, env_offset, counts);
    GCA_CHECK_LAUNCH("ds_step");
    return GCA_OK;
}
