// gca_init.hip — hidden context layers of the Advanced env drawn on the device (init_utils.py:10-116).
// The reference draws them with np.random per pixel / patch / hill in Python loops (4.7 s for 4096 envs
// at 256^2 even vectorised on the host, dominated by 268M sequential MT19937 noise draws and a 2 GB
// upload). Here every draw is Philox keyed by (global env id, slot), so the layers are independent of
// the launch shape and of the env sharding; the recipe (ranges, patch order, zero fill, hills, slopes)
// is the reference's. Stream compatibility with np.random is the host path's job (init_utils.py).
#include "gca_common.h"

namespace {

constexpr int kMaxPatches = 7;  // randint(4, 8)

struct Patch {
    int16_t r0, r1, c0, c1;
    int16_t value;
};

__device__ __forceinline__ u32x4 plan_draw(uint32_t slot, uint32_t gid, uint32_t k0, uint32_t k1) {
    return philox4x32_10(u32x4{slot, gid, 0u, GCA_TAG_HIDDEN}, k0, k1);
}

// Patches of one layer (0 vegetation, 1 density): slot 64 * layer + 8 + 2 p (+1) per patch, 64 * layer: count.
__device__ int layer_patches(int layer, uint32_t gid, int R, int C, uint32_t k0, uint32_t k1, Patch* out) {
    const uint32_t base = 64u * (uint32_t)layer;
    const int n = randint_ms(plan_draw(base, gid, k0, k1).x, 4, 8);
    for (int p = 0; p < n; ++p) {
        const u32x4 a = plan_draw(base + 8u + 2u * p, gid, k0, k1);
        const u32x4 b = plan_draw(base + 9u + 2u * p, gid, k0, k1);
        const int cr = randint_ms(a.x, 0, R), cc = randint_ms(a.y, 0, C);
        const int ph = randint_ms(a.z, 3, max(4, R / 2)), pw = randint_ms(a.w, 3, max(4, C / 2));
        out[p].r0 = (int16_t)max(0, cr - ph / 2);
        out[p].r1 = (int16_t)min(R, cr + ph / 2);
        out[p].c0 = (int16_t)max(0, cc - pw / 2);
        out[p].c1 = (int16_t)min(C, cc + pw / 2);
        out[p].value = (int16_t)randint_ms(b.x, 1, 6);
    }
    return n;
}

__device__ __forceinline__ double uniform_f64(u32x4 x, double lo, double hi) {
    return lo + (hi - lo) * u01_f64(x.x, x.y);
}

// One thread per env: the altitude plan (hills slot 128 + h, slopes slot 160 + k, counts slot 127).
__global__ void hidden_plan_kernel(uint32_t k0, uint32_t k1, int env_offset, int E, int R, int C,
                                   int32_t* __restrict__ n_hills, double* __restrict__ hills,
                                   int32_t* __restrict__ n_slopes, double* __restrict__ slopes) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const uint32_t gid = (uint32_t)(env_offset + e);
    const u32x4 cnt = plan_draw(127u, gid, k0, k1);
    const int nh = randint_ms(cnt.x, 6, 10), ns = randint_ms(cnt.y, 4, 8);
    n_hills[e] = nh;
    n_slopes[e] = ns;
    for (int h = 0; h < GCA_MAX_HILLS; ++h) {
        double* hp = hills + ((int64_t)e * GCA_MAX_HILLS + h) * 4;
        if (h >= nh) {
            hp[0] = hp[1] = hp[2] = hp[3] = 0.0;
            continue;
        }
        const u32x4 a = plan_draw(128u + h, gid, k0, k1);
        hp[0] = (double)randint_ms(a.x, 0, R);
        hp[1] = (double)randint_ms(a.y, 0, C);
        hp[2] = (double)randint_ms(a.z, 2, max(3, min(R, C) / 4));
        hp[3] = uniform_f64(plan_draw(144u + h, gid, k0, k1), 2.0, 6.0);
    }
    for (int k = 0; k < GCA_MAX_SLOPES; ++k) {
        double* sp = slopes + ((int64_t)e * GCA_MAX_SLOPES + k) * 5;
        if (k >= ns) {
            sp[0] = sp[1] = sp[2] = sp[3] = sp[4] = 0.0;
            continue;
        }
        const u32x4 a = plan_draw(160u + k, gid, k0, k1);
        sp[0] = (double)randint_ms(a.x, 0, max(1, R - 4));
        sp[1] = (double)randint_ms(a.y, 0, max(1, C - 4));
        sp[2] = (double)randint_ms(a.z, 3, max(4, C / 4));
        sp[3] = (double)randint_ms(a.w, 3, max(4, R / 4));
        sp[4] = uniform_f64(plan_draw(176u + k, gid, k0, k1), 1.0, 4.0);
    }
}

// Block = (env, 16 rows), 256 threads. Lanes 0 / 1 draw the vegetation / density patch lists into LDS.
constexpr int kRowsPerBlock = 16;

__global__ __launch_bounds__(256) void hidden_cells_kernel(uint32_t k0, uint32_t k1, int env_offset, int R, int C,
                                                           int blocks_per_env, uint8_t* __restrict__ veg,
                                                           uint8_t* __restrict__ den, double* __restrict__ noise) {
    __shared__ Patch P[2][kMaxPatches];
    __shared__ int NP[2];
    const int e = blockIdx.x / blocks_per_env;
    const int r0 = (blockIdx.x - e * blocks_per_env) * kRowsPerBlock;
    const uint32_t gid = (uint32_t)(env_offset + e);
    if (threadIdx.x < 2) NP[threadIdx.x] = layer_patches(threadIdx.x, gid, R, C, k0, k1, P[threadIdx.x]);
    __syncthreads();
    const int rows = min(kRowsPerBlock, R - r0);
    const int64_t base = (int64_t)e * R * C;
    for (int idx = threadIdx.x; idx < rows * C; idx += blockDim.x) {
        const int r = r0 + idx / C, c = idx % C;
        const int64_t lin = (int64_t)r * C + c;
        const u32x4 x = philox4x32_10(u32x4{(uint32_t)lin, gid, 0u, GCA_TAG_HIDDEN_CELL}, k0, k1);
        int v[2] = {0, 0};
#pragma unroll
        for (int l = 0; l < 2; ++l) {
            for (int p = 0; p < NP[l]; ++p)
                if (r >= P[l][p].r0 && r < P[l][p].r1 && c >= P[l][p].c0 && c < P[l][p].c1) v[l] = P[l][p].value;
        }
        veg[base + lin] = (uint8_t)(v[0] ? v[0] : randint_ms(x.x, 1, 4));
        den[base + lin] = (uint8_t)(v[1] ? v[1] : randint_ms(x.y, 1, 4));
        noise[base + lin] = 5.0 * u01_f64(x.z, x.w);
    }
}

}  // namespace

extern "C" int gca_hidden_init(uint64_t seed, int env_offset, int E, int H, int W, uint8_t* vegetation,
                               uint8_t* density, double* altitude, int32_t* n_hills, double* hills, int32_t* n_slopes,
                               double* slopes, void* stream) {
    GCA_CHECK_ARG(vegetation && density && altitude && n_hills && hills && n_slopes && slopes, "hidden_init: null");
    GCA_CHECK_ARG(E > 0 && H > 0 && W > 0 && H < 32768 && W < 32768 && env_offset >= 0, "hidden_init: sizes");
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(hidden_plan_kernel, dim3((E + 63) / 64), dim3(64), 0, st, k0, k1, env_offset, E, H, W, n_hills,
                       hills, n_slopes, slopes);
    GCA_CHECK_LAUNCH("hidden_plan");
    const int bpe = (H + kRowsPerBlock - 1) / kRowsPerBlock;
    hipLaunchKernelGGL(hidden_cells_kernel, dim3((unsigned)((int64_t)E * bpe)), dim3(256), 0, st, k0, k1, env_offset,
                       H, W, bpe, vegetation, density, altitude);
    GCA_CHECK_LAUNCH("hidden_cells");
    return GCA_OK;
}
