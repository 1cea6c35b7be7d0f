// gca_env.hip — per-env O(1) work of the batched env steps: RepeatCA time bookkeeping,
// Move, Modify, reward/done, wind change, conditional reset. One thread per env.
//
// References: repeat_ca.py:32-45, move_modify.py:37-134, bulldozer.py:180-216,393-400,
//             repeat_ca_jax.py:34-71, move_modify_jax.py:39-157,
//             ca_alexandridis_jax.py:442-451, advanced_bulldozer.py:422-633,1103-1133.
#include <math.h>

#include "gca_common.h"

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return clampi_dev(v, lo, hi); }
__device__ __forceinline__ int category(int v, int empty, int tree, int fire) { return cell_category(v, empty, tree, fire); }

// ================================================================== ForestFireBulldozer
__global__ void bulldozer_pre_kernel(gca_bulldozer_params p, const int32_t* __restrict__ action,
                                     double* __restrict__ accu, int32_t* __restrict__ steps,
                                     const uint8_t* __restrict__ done, const double* __restrict__ wind,
                                     int64_t wind_stride, const uint32_t* __restrict__ rng_step,
                                     uint8_t* __restrict__ dir_mask, int32_t* __restrict__ counts, int E) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    if (done && done[e]) {  // ca_env.py:50-62: stepping a finished env changes nothing
        steps[e] = -1;
        return;
    }
    const int a0 = clampi(action[2 * e], 0, 8), a1 = clampi(action[2 * e + 1], 0, 1);
    // RepeatCA.update: time_taken = t_acting(action) + t_perception(state); accu += time_taken
    const double time_action = p.t_move[a0] + p.t_shoot[a1];
    const double x = accu[e] + (time_action + p.t_any);
    const double reps = trunc(x);  // math.modf
    accu[e] = x - reps;
    const int n = (int)reps;
    steps[e] = n;
    if (n > 0) {
        counts[3 * e + 0] = 0;
        counts[3 * e + 1] = 0;
        counts[3 * e + 2] = 0;
        dir_mask[e] = (uint8_t)windy_mask(wind + (int64_t)e * wind_stride, nullptr, (uint32_t)p.seed,
                                          (uint32_t)(p.seed >> 32), (uint32_t)(p.env_offset + e), rng_step[e]);
    }
}

__global__ void bulldozer_interpass_kernel(gca_bulldozer_params p, int pass, const int32_t* __restrict__ steps,
                                           uint8_t* __restrict__ parity, const double* __restrict__ wind,
                                           int64_t wind_stride, const uint32_t* __restrict__ rng_step,
                                           uint8_t* __restrict__ dir_mask, int32_t* __restrict__ counts, int E) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int n = steps[e];
    if (n > pass) parity[e] ^= 1;
    if (n > pass + 1) {
        // the next pass recounts this env's new grid from zero
        counts[3 * e + 0] = 0;
        counts[3 * e + 1] = 0;
        counts[3 * e + 2] = 0;
        dir_mask[e] = (uint8_t)windy_mask(wind + (int64_t)e * wind_stride, nullptr, (uint32_t)p.seed,
                                          (uint32_t)(p.seed >> 32), (uint32_t)(p.env_offset + e),
                                          rng_step[e] + (uint32_t)(pass + 1));
    }
}

__global__ void bulldozer_post_kernel(gca_bulldozer_params p, int last_pass, const int32_t* __restrict__ action,
                                      const int32_t* __restrict__ steps, uint8_t* __restrict__ parity,
                                      uint8_t* __restrict__ buf0, uint8_t* __restrict__ buf1, int H, int W,
                                      int32_t* __restrict__ pos, int32_t* __restrict__ counts,
                                      uint32_t* __restrict__ rng_step, uint8_t* __restrict__ done,
                                      uint8_t* __restrict__ hit, double* __restrict__ reward, int E) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int n = steps[e];
    if (n < 0) {  // finished before this step: graceful no-op (ca_env.py:50-62)
        reward[e] = 0.0;
        return;
    }
    if (parity && n > last_pass) parity[e] ^= 1;
    uint8_t* grid = ((parity && parity[e]) ? buf1 : buf0) + (int64_t)e * H * W;
    // MoveModify (move_modify.py:128-134): Move, then Modify at the new position
    const int a0 = clampi(action[2 * e], 0, 8), a1 = action[2 * e + 1];
    int row = pos[2 * e], col = pos[2 * e + 1];
    move_pos(a0, row, col, H, W, p.up_mask, p.down_mask, p.left_mask, p.right_mask);
    pos[2 * e] = row;
    pos[2 * e + 1] = col;
    uint8_t h = 0;
    if (a1 && row >= 0 && row < H && col >= 0 && col < W) {  // a caller's own out-of-grid position writes nothing
        const int v = grid[(int64_t)row * W + col];
        const int nv = p.effect[v];
        if (nv >= 0) {
            grid[(int64_t)row * W + col] = (uint8_t)nv;
            h = 1;
            const int c_old = category(v, p.empty, p.tree, p.fire), c_new = category(nv, p.empty, p.tree, p.fire);
            if (c_old >= 0) counts[3 * e + c_old] -= 1;
            if (c_new >= 0) counts[3 * e + c_new] += 1;
        }
    }
    hit[e] = h;
    // _award (bulldozer.py:180-213) and _is_done (:215-216) on the post-Modify grid
    const int t = counts[3 * e + 1], f = counts[3 * e + 2];
    reward[e] = (t + f) > 0 ? -((double)f / (double)(t + f)) : (double)NAN;
    done[e] = f == 0 ? 1 : 0;
    rng_step[e] += (uint32_t)n;
}

static const int kEnvThreads = 256;
#define ENV_GRID(E) dim3((unsigned)(((E) + kEnvThreads - 1) / kEnvThreads)), dim3(kEnvThreads)

extern "C" int gca_bulldozer_pre(const gca_bulldozer_params* p, const int32_t* action, double* accu, int32_t* steps,
                                 const uint8_t* done, const double* wind, int64_t wind_stride,
                                 const uint32_t* rng_step, uint8_t* dir_mask, int32_t* counts, int E, void* stream) {
    GCA_CHECK_ARG(p && action && accu && steps && wind && rng_step && dir_mask && counts && E > 0,
                  "bulldozer_pre: null argument");
    hipLaunchKernelGGL(bulldozer_pre_kernel, ENV_GRID(E), 0, (hipStream_t)stream, *p, action, accu, steps, done, wind,
                       wind_stride, rng_step, dir_mask, counts, E);
    GCA_CHECK_LAUNCH("bulldozer_pre");
    return GCA_OK;
}

extern "C" int gca_bulldozer_interpass(const gca_bulldozer_params* p, int pass, const int32_t* steps, uint8_t* parity,
                                       const double* wind, int64_t wind_stride, const uint32_t* rng_step,
                                       uint8_t* dir_mask, int32_t* counts, int E, void* stream) {
    GCA_CHECK_ARG(p && steps && parity && wind && rng_step && dir_mask && counts && E > 0,
                  "bulldozer_interpass: null argument");
    hipLaunchKernelGGL(bulldozer_interpass_kernel, ENV_GRID(E), 0, (hipStream_t)stream, *p, pass, steps, parity, wind,
                       wind_stride, rng_step, dir_mask, counts, E);
    GCA_CHECK_LAUNCH("bulldozer_interpass");
    return GCA_OK;
}

extern "C" int gca_bulldozer_post(const gca_bulldozer_params* p, int last_pass, const int32_t* action,
                                  const int32_t* steps, uint8_t* parity, uint8_t* buf0, uint8_t* buf1, int H, int W,
                                  int32_t* pos, int32_t* counts, uint32_t* rng_step, uint8_t* done, uint8_t* hit,
                                  double* reward, int E, void* stream) {
    GCA_CHECK_ARG(p && action && steps && buf0 && pos && counts && rng_step && done && hit && reward && E > 0,
                  "bulldozer_post: null argument");
    GCA_CHECK_ARG(!parity || buf1, "bulldozer_post: parity needs buf1");
    hipLaunchKernelGGL(bulldozer_post_kernel, ENV_GRID(E), 0, (hipStream_t)stream, *p, last_pass, action, steps,
                       parity, buf0, buf1, H, W, pos, counts, rng_step, done, hit, reward, E);
    GCA_CHECK_LAUNCH("bulldozer_post");
    return GCA_OK;
}

// ================================================================== Advanced env (JAX)
__global__ void advenv_post_kernel(gca_advenv_params p, const int32_t* __restrict__ action, int32_t* __restrict__ pos,
                                   float* __restrict__ accu, int32_t* __restrict__ wind_index,
                                   int32_t* __restrict__ time_step, int32_t* __restrict__ is_night,
                                   uint8_t* __restrict__ dousing, uint16_t* __restrict__ dous_bits, int H, int W,
                                   const int32_t* __restrict__ counts,
                                   uint32_t* __restrict__ rng_step, float* __restrict__ reward,
                                   uint8_t* __restrict__ done, float* __restrict__ steps_elapsed,
                                   float* __restrict__ reward_acc, int E) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const uint32_t step = rng_step[e];
    // wind change (ca_alexandridis_jax.py:442-451): u < p_wind_change -> (idx + randint[1,8)) % n_winds
    const u32x4 x = philox4x32_10(u32x4{0u, (uint32_t)(p.env_offset + e), step, GCA_TAG_ALEX_WIND}, (uint32_t)p.seed,
                                  (uint32_t)(p.seed >> 32));
    if (u01_f32(x.x) < p.p_wind_change) wind_index[e] = (wind_index[e] + randint_ms(x.y, 1, 8)) % p.n_winds;
    // RepeatCAJax time bookkeeping (repeat_ca_jax.py:191-198), f32 like the JAX env
    const int a0 = clampi(action[2 * e], 0, 8), a1 = clampi(action[2 * e + 1], 0, 1);
    const float time_taken = __fadd_rn(__fadd_rn(p.t_move[a0], p.t_shoot[a1]), p.t_any);
    const float na = __fadd_rn(accu[e], time_taken);
    accu[e] = __fsub_rn(na, truncf(na));
    // MoveJax then ModifyJax (dousing_count[row, col] = 1 when shoot == 1)
    int row = pos[2 * e], col = pos[2 * e + 1];
    move_pos(a0, row, col, H, W, p.up_mask, p.down_mask, p.left_mask, p.right_mask);
    pos[2 * e] = row;
    pos[2 * e + 1] = col;
    if (a1 == 1 && row >= 0 && row < H && col >= 0 && col < W) {  // JAX drops out-of-bounds scatter updates
        const int64_t cell = (int64_t)e * H * W + (int64_t)row * W + col;
        dousing[cell] = 1;
        if (dous_bits) dous_bits[cell >> 4] |= (uint16_t)(1u << (cell & 15));  // packed layout (one writer per env)
    }
    // time_step / is_night (advanced_bulldozer.py:1118,1123-1127)
    const int ts = time_step[e] + 1;
    time_step[e] = ts;
    if (p.day_length > 0 && ts % p.day_length == 0) is_night[e] = 1 - is_night[e];
    // _award (:597-630): -(f / (t + f + 1e-8)) in f32; _is_done (:632-633)
    const int t = counts[3 * e + 1], f = counts[3 * e + 2];
    const float denom = __fadd_rn((float)(t + f), 1e-8f);
    const float rw = -__fdiv_rn((float)f, denom);
    reward[e] = rw;
    done[e] = f == 0 ? 1 : 0;
    if (steps_elapsed) steps_elapsed[e] = __fadd_rn(steps_elapsed[e], 1.0f);
    if (reward_acc) reward_acc[e] = __fadd_rn(reward_acc[e], rw);
    rng_step[e] = step + 1u;
}

extern "C" int gca_advenv_post(const gca_advenv_params* p, const int32_t* action, int32_t* pos, float* accu,
                               int32_t* wind_index, int32_t* time_step, int32_t* is_night, uint8_t* dousing,
                               uint16_t* dous_bits, int H, int W, const int32_t* counts, uint32_t* rng_step,
                               float* reward, uint8_t* done, float* steps_elapsed, float* reward_accumulated, int E,
                               void* stream) {
    GCA_CHECK_ARG(p && action && pos && accu && wind_index && time_step && is_night && dousing && counts && rng_step &&
                      reward && done && E > 0,
                  "advenv_post: null argument");
    GCA_CHECK_ARG(p->n_winds > 0, "advenv_post: n_winds > 0");
    GCA_CHECK_ARG(!dous_bits || (W % 16 == 0), "advenv_post: dousing bits need W % 16 == 0");
    hipLaunchKernelGGL(advenv_post_kernel, ENV_GRID(E), 0, (hipStream_t)stream, *p, action, pos, accu, wind_index,
                       time_step, is_night, dousing, dous_bits, H, W, counts, rng_step, reward, done, steps_elapsed,
                       reward_accumulated, E);
    GCA_CHECK_LAUNCH("advenv_post");
    return GCA_OK;
}

// ================================================================== conditional reset
// Grid-sized copies: block = (env, 4 KiB chunk); blocks of live envs exit at once.
__global__ __launch_bounds__(256) void reset_cells_kernel(const uint8_t* __restrict__ done, int64_t HW, int cpe,
                                                          uint8_t* __restrict__ grid, const uint8_t* __restrict__ grid0,
                                                          int16_t* __restrict__ age, const int16_t* __restrict__ age0,
                                                          uint8_t* __restrict__ dous, const uint8_t* __restrict__ dous0,
                                                          uint16_t* __restrict__ dbits) {
    const int e = blockIdx.x / cpe;
    if (!done[e]) return;
    const int64_t base = (int64_t)e * HW;
    const int64_t begin = (int64_t)(blockIdx.x - e * cpe) * 4096, end = min(begin + 4096, HW);
    for (int64_t i = begin + threadIdx.x; i < end; i += 256) {
        if (grid) grid[base + i] = grid0[base + i];
        if (age) age[base + i] = age0[base + i];
        if (dous) dous[base + i] = dous0 ? dous0[base + i] : 0;
    }
    if (dbits)  // packed dousing bits of this chunk (zeroed: the reset state has no dousing)
        for (int64_t i = begin / 16 + threadIdx.x; i < end / 16; i += 256) dbits[(base >> 4) + i] = 0;
}

__global__ void reset_env_kernel(uint8_t* __restrict__ done, int32_t* __restrict__ pos,
                                 const int32_t* __restrict__ pos0, float* __restrict__ accu,
                                 int32_t* __restrict__ wind_index, const int32_t* __restrict__ wind_index0, int E) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E || !done[e]) return;
    if (pos) {
        pos[2 * e] = pos0[2 * e];
        pos[2 * e + 1] = pos0[2 * e + 1];
    }
    if (accu) accu[e] = 0.0f;
    if (wind_index) wind_index[e] = wind_index0[e];
    done[e] = 0;
}

extern "C" int gca_reset_where(const uint8_t* done, int E, int H, int W, uint8_t* grid, const uint8_t* grid0,
                               int16_t* age, const int16_t* age0, uint8_t* dousing, const uint8_t* dousing0,
                               uint16_t* dous_bits, int32_t* pos, const int32_t* pos0, float* accu, int32_t* wind_index,
                               const int32_t* wind_index0, void* stream) {
    GCA_CHECK_ARG(done && E > 0 && H > 0 && W > 0, "reset_where: done and sizes required");
    GCA_CHECK_ARG(!grid || grid0, "reset_where: grid needs grid0");
    GCA_CHECK_ARG(!age || age0, "reset_where: age needs age0");
    GCA_CHECK_ARG(!pos || pos0, "reset_where: pos needs pos0");
    GCA_CHECK_ARG(!wind_index || wind_index0, "reset_where: wind_index needs wind_index0");
    GCA_CHECK_ARG(!dous_bits || (!dousing0 && W % 16 == 0), "reset_where: dousing bits are zeroed (no dousing0), W % 16 == 0");
    hipStream_t st = (hipStream_t)stream;
    const int64_t HW = (int64_t)H * W;
    const int cpe = (int)((HW + 4095) / 4096);
    if (grid || age || dousing || dous_bits) {
        hipLaunchKernelGGL(reset_cells_kernel, dim3((unsigned)((int64_t)E * cpe)), dim3(256), 0, st, done, HW, cpe, grid,
                           grid0, age, age0, dousing, dousing0, dous_bits);
        GCA_CHECK_LAUNCH("reset_cells");
    }
    hipLaunchKernelGGL(reset_env_kernel, ENV_GRID(E), 0, st, (uint8_t*)done, pos, pos0, accu, wind_index, wind_index0, E);
    GCA_CHECK_LAUNCH("reset_env");
    return GCA_OK;
}

// ================================================================== Move / Modify (batched)
// MoveModify.update (move_modify.py:128-134) for E envs: Move then Modify at the new position.
__global__ void move_modify_kernel(const int32_t* __restrict__ action, int32_t* __restrict__ pos,
                                   uint8_t* __restrict__ grid, int H, int W, gca_bulldozer_params p,
                                   uint8_t* __restrict__ hit, int E) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    int row = pos[2 * e], col = pos[2 * e + 1];
    const int a0 = action[2 * e], a1 = action[2 * e + 1];
    if (a0 >= 0 && a0 < 32) move_pos(a0, row, col, H, W, p.up_mask, p.down_mask, p.left_mask, p.right_mask);
    pos[2 * e] = row;
    pos[2 * e + 1] = col;
    uint8_t h = 0;
    // a caller's own start outside the grid that no move brings inside: no write (the host build and the Python
    // layer refuse it with GCA_ERR_ARG before any launch; a kernel cannot, so it only stays inside the buffer)
    if (grid && a1 && row >= 0 && row < H && col >= 0 && col < W) {
        uint8_t* g = grid + (int64_t)e * H * W + (int64_t)row * W + col;
        const int nv = p.effect[*g];
        if (nv >= 0) {
            *g = (uint8_t)nv;
            h = 1;
        }
    }
    if (hit) hit[e] = h;
}

extern "C" int gca_move_modify(const gca_bulldozer_params* p, const int32_t* action, int32_t* pos, uint8_t* grid, int H,
                               int W, uint8_t* hit, int E, void* stream) {
    GCA_CHECK_ARG(p && action && pos && E > 0 && H > 0 && W > 0, "move_modify: bad arguments");
    hipLaunchKernelGGL(move_modify_kernel, ENV_GRID(E), 0, (hipStream_t)stream, action, pos, grid, H, W, *p, hit, E);
    GCA_CHECK_LAUNCH("move_modify");
    return GCA_OK;
}

// ================================================================== Alexandridis wind change
// PartiallyObservableForestFireJax.update (ca_alexandridis_jax.py:442-451) for E envs:
// u < p_wind_change -> wind_index = (wind_index + randint[1,8)) % n_winds.
// Draws: inj_u / inj_k (nullable, injected) or Philox((0, env_offset+e, rng_step[e], ALXW)).
__global__ void alex_wind_change_kernel(float p_change, int n_winds, uint32_t k0, uint32_t k1, int env_offset,
                                        const uint32_t* __restrict__ rng_step, const float* __restrict__ inj_u,
                                        const int32_t* __restrict__ inj_k, int32_t* __restrict__ wind_index, int E) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    float u;
    int k;
    if (inj_u) {
        u = inj_u[e];
        k = inj_k[e];
    } else {
        const u32x4 x = philox4x32_10(u32x4{0u, (uint32_t)(env_offset + e), rng_step ? rng_step[e] : 0u,
                                            GCA_TAG_ALEX_WIND}, k0, k1);
        u = u01_f32(x.x);
        k = randint_ms(x.y, 1, 8);
    }
    if (u < p_change) wind_index[e] = (wind_index[e] + k) % n_winds;
}

extern "C" int gca_alex_wind_change(float p_wind_change, int n_winds, uint64_t seed, int env_offset,
                                    const uint32_t* rng_step, const float* inj_u, const int32_t* inj_k,
                                    int32_t* wind_index, int E, void* stream) {
    GCA_CHECK_ARG(wind_index && E > 0 && n_winds > 0, "alex_wind_change: bad arguments");
    GCA_CHECK_ARG((inj_u == nullptr) == (inj_k == nullptr), "alex_wind_change: inj_u and inj_k go together");
    hipLaunchKernelGGL(alex_wind_change_kernel, ENV_GRID(E), 0, (hipStream_t)stream, p_wind_change, n_winds,
                       (uint32_t)seed, (uint32_t)(seed >> 32), env_offset, rng_step, inj_u, inj_k, wind_index, E);
    GCA_CHECK_LAUNCH("alex_wind_change");
    return GCA_OK;
}
