// gca_util.hip — error plumbing, Philox KAT entry point, cell counting, synthetic inputs.
#include <stdarg.h>

#include "gca_common.h"

static thread_local char g_err[512] = "";

void gca_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

extern "C" const char* gca_last_error(void) { return g_err; }
extern "C" int gca_version(void) { return 1; }

// ------------------------------------------------------------------ Philox KAT
__global__ void philox_kernel(const uint32_t* __restrict__ ctr, uint32_t k0, uint32_t k1, uint32_t* __restrict__ out,
                              int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32x4 c{ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]};
    const u32x4 x = philox4x32_10(c, k0, k1);
    out[4 * i] = x.x;
    out[4 * i + 1] = x.y;
    out[4 * i + 2] = x.z;
    out[4 * i + 3] = x.w;
}

extern "C" int gca_philox(const uint32_t* ctr, uint32_t key0, uint32_t key1, uint32_t* out, int64_t n, void* stream) {
    GCA_CHECK_ARG(ctr && out && n >= 0, "ctr/out required");
    if (n == 0) return GCA_OK;
    hipLaunchKernelGGL(philox_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ctr, key0,
                       key1, out, n);
    GCA_CHECK_LAUNCH("philox");
    return GCA_OK;
}

// ------------------------------------------------------------------ count_cells
// One block per (env, chunk of 16 KiB); 16-B loads, SWAR byte compares, wave reduce, atomics.
__global__ __launch_bounds__(256) void count_kernel(const uint8_t* __restrict__ grid, int64_t HW, int chunks_per_env,
                                                    uint32_t p0, uint32_t p1, uint32_t p2, int32_t* __restrict__ counts) {
    const int env = blockIdx.x / chunks_per_env;
    const int chunk = blockIdx.x - env * chunks_per_env;
    const uint8_t* g = grid + (int64_t)env * HW;
    const int64_t begin = (int64_t)chunk * 16384, end = min(begin + 16384, HW);
    int32_t c0 = 0, c1 = 0, c2 = 0;
    const bool vec = ((((uintptr_t)g) & 15u) == 0) && (HW % 16 == 0);
    if (vec) {
        for (int64_t i = begin + 16 * threadIdx.x; i < end; i += 16 * 256) {
            const uint4 v = *reinterpret_cast<const uint4*>(g + i);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                c0 += __popc(bytes_eq01(w[j], p0));
                c1 += __popc(bytes_eq01(w[j], p1));
                c2 += __popc(bytes_eq01(w[j], p2));
            }
        }
    } else {
        for (int64_t i = begin + threadIdx.x; i < end; i += 256) {
            const uint32_t v = g[i];
            c0 += v == (p0 & 0xFFu);
            c1 += v == (p1 & 0xFFu);
            c2 += v == (p2 & 0xFFu);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        c0 += __shfl_xor(c0, off);
        c1 += __shfl_xor(c1, off);
        c2 += __shfl_xor(c2, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(counts + 3 * env + 0, c0);
        atomicAdd(counts + 3 * env + 1, c1);
        atomicAdd(counts + 3 * env + 2, c2);
    }
}

extern "C" int gca_count_cells(const uint8_t* grid, int E, int H, int W, int v0, int v1, int v2, int32_t* counts,
                               void* stream) {
    GCA_CHECK_ARG(grid && counts && E > 0 && H > 0 && W > 0, "grid/counts and positive sizes required");
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(counts, 0, sizeof(int32_t) * 3 * (size_t)E, st) != hipSuccess) {
        gca_set_error("count_cells: memset failed");
        return GCA_ERR_HIP;
    }
    const int64_t HW = (int64_t)H * W;
    const int cpe = (int)((HW + 16383) / 16384);
    hipLaunchKernelGGL(count_kernel, dim3((unsigned)((int64_t)E * cpe)), dim3(256), 0, st, grid, HW, cpe, rep4(v0),
                       rep4(v1), rep4(v2), counts);
    GCA_CHECK_LAUNCH("count_cells");
    return GCA_OK;
}

// ------------------------------------------------------------------ synthetic inputs
// out[e][i] = values[j] where j is the first index with u < cdf[j], u = u01_f32 of
// Philox((i>>2, env_offset+e, 0, INIT))[i&3]. Used by bench/tests for seeded grids.
__global__ void fill_categorical_kernel(uint8_t* __restrict__ out, int64_t n_per_env, int env_offset, uint32_t k0,
                                        uint32_t k1, const float* __restrict__ cdf, const uint8_t* __restrict__ values,
                                        int n_values, int E) {
    const int64_t quads = (n_per_env + 3) / 4;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= quads * E) return;
    const int e = (int)(gid / quads);
    const int64_t qd = gid - (int64_t)e * quads;
    const u32x4 x = philox4x32_10(u32x4{(uint32_t)qd, (uint32_t)(env_offset + e), 0u, GCA_TAG_INIT}, k0, k1);
    const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t i = 4 * qd + j;
        if (i >= n_per_env) break;
        const float u = u01_f32(xs[j]);
        int k = 0;
        while (k < n_values - 1 && !(u < cdf[k])) ++k;
        out[(int64_t)e * n_per_env + i] = values[k];
    }
}

extern "C" int gca_fill_categorical(uint8_t* out, int64_t n_per_env, int E, int env_offset, uint64_t seed,
                                    const float* cdf, const uint8_t* values, int n_values, void* stream) {
    GCA_CHECK_ARG(out && cdf && values && n_values > 0 && E > 0 && n_per_env > 0, "bad fill_categorical args");
    const int64_t n = ((n_per_env + 3) / 4) * E;
    hipLaunchKernelGGL(fill_categorical_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       out, n_per_env, env_offset, (uint32_t)seed, (uint32_t)(seed >> 32), cdf, values, n_values, E);
    GCA_CHECK_LAUNCH("fill_categorical");
    return GCA_OK;
}

// action[e] = (move in [0,9), shoot in {0,1}) from Philox((0, env_offset+e, rng_step[e], ACTION)).
__global__ void random_actions_kernel(int32_t* __restrict__ action, int E, int env_offset, uint32_t k0, uint32_t k1,
                                      const uint32_t* __restrict__ rng_step) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const u32x4 x = philox4x32_10(u32x4{0u, (uint32_t)(env_offset + e), rng_step ? rng_step[e] : 0u, GCA_TAG_ACTION},
                                  k0, k1);
    action[2 * e] = randint_ms(x.x, 0, 9);
    action[2 * e + 1] = (int32_t)(x.y >> 31);
}

extern "C" int gca_random_actions(int32_t* action, int E, int env_offset, uint64_t seed, const uint32_t* rng_step,
                                  void* stream) {
    GCA_CHECK_ARG(action && E > 0, "action required");
    hipLaunchKernelGGL(random_actions_kernel, dim3((E + 255) / 256), dim3(256), 0, (hipStream_t)stream, action, E,
                       env_offset, (uint32_t)seed, (uint32_t)(seed >> 32), rng_step);
    GCA_CHECK_LAUNCH("random_actions");
    return GCA_OK;
}
