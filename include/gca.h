/*
 * gca.h — C-ABI of libgca_hip.so, the MI355X (gfx950) forest-fire CA hot path.
 *
 * Boundary contract:
 *   - plain extern "C", int status (GCA_OK = 0), gca_last_error() for the message;
 *   - every array argument is a DEVICE pointer owned by the caller (e.g. a torch
 *     tensor's data_ptr()); parameter structs are HOST pointers read at call time;
 *   - `stream` is a hipStream_t (NULL = legacy default stream); calls only enqueue
 *     work: no allocation, no synchronisation, so they can be captured in a hipGraph;
 *   - one caller per stream (thread-compatible, not thread-safe).
 *
 * Cell grids are u8, laid out (env, row, col) row-major. Cell codes are the
 * reference's integer values (ForestFireBulldozer EMPTY=0 TREE=3 FIRE=25,
 * Advanced/Helicopter 0/1/2); the host side checks they fit in u8.
 *
 * RNG: counter-based Philox4x32-10 (Random123), key = (seed lo, seed hi),
 * counter = (slot, global env id, per-env step, stream tag). See DESIGN.md §RNG.
 */
#ifndef GCA_H
#define GCA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GCA_OK 0
#define GCA_ERR_ARG 1
#define GCA_ERR_HIP 2
#define GCA_ERR_UNSUPPORTED 3

#define GCA_MAX_RADIUS 8     /* heat-kernel radius ceil(log2 N)-2 <= 8  <=>  N <= 1024 */

/* Philox stream tags (counter word 3). */
#define GCA_TAG_WINDY_ROLL 0x574E4459u /* 'WNDY' : 3x3 roll of WindyForestFire      */
#define GCA_TAG_ALEX_CELL  0x414C5843u /* 'ALXC' : per-cell draws of Alexandridis (one block per 4 cells) */
#define GCA_TAG_ALEX_AGE   0x414C5841u /* 'ALXA' : ages of a 4-cell group's 2nd..4th new fires            */
#define GCA_TAG_ALEX_WIND  0x414C5857u /* 'ALXW' : per-env wind change               */
#define GCA_TAG_ACTION     0x41435449u /* 'ACTI' : synthetic actions (bench)          */
#define GCA_TAG_INIT       0x494E4954u /* 'INIT' : synthetic initial states           */
#define GCA_TAG_DS_CELL    0x44534345u /* 'DSCE' : Drossel-Schwabl per-cell draws     */
#define GCA_TAG_PINE       0x50494E45u /* 'PINE' (+1+m): pinecone count / pinecone m  */
#define GCA_TAG_PINE_AGE   0x50494E41u /* 'PINA' : age of a pinecone-ignited cell     */
#define GCA_TAG_HIDDEN     0x48494444u /* 'HIDD' : per-env hidden-layer plan (patches, hills, slopes) */
#define GCA_TAG_HIDDEN_CELL 0x48494443u /* 'HIDC' : per-cell hidden-layer draws          */
#define GCA_TAG_PINEC      0x50434C00u /* 'PCL\0' (+1+m): classic pinecone count / pinecone m */
#define GCA_TAG_PINEC_AGE  0x50434C41u /* 'PCLA' : age of a classic pinecone ignition        */

/* ------------------------------------------------------------------ generic */

const char* gca_last_error(void);
int gca_version(void);

/* Philox4x32-10 over n counters (ctr[n][4] device, out[n][4] device). KAT hook. */
int gca_philox(const uint32_t* ctr, uint32_t key0, uint32_t key1, uint32_t* out, int64_t n, void* stream);

/* counts[e][0..2] = #cells == v0/v1/v2 in grid e (overwrites). ca_env.py:94-99 count_cells. */
int gca_count_cells(const uint8_t* grid, int E, int H, int W, int v0, int v1, int v2, int32_t* counts, void* stream);

/* ------------------------------------------------------- WindyForestFire ---
 * Replaces WindyForestFire._get_failed_propagations_mask + _get_kernel
 * (ca_windy.py:53-77): dir_mask[e] bit d (d = 3x3 index row-major, centre
 * skipped) is set iff roll[d] < wind[d]  (the reference keeps d iff NOT wind<=roll).
 * wind: [E][9] f64 with env stride wind_stride (0 = one wind shared by all envs).
 * roll: [E][9] f64 injected uniforms, or NULL -> Philox(seed, (d/2, env_offset+e,
 *       rng_step[e] + pass, GCA_TAG_WINDY_ROLL)), 53-bit doubles.
 * Only envs with steps == NULL || steps[e] > pass are written.                */
int gca_windy_dirmask(const double* wind, int64_t wind_stride, const double* roll, uint64_t seed,
                      const uint32_t* rng_step, const int32_t* steps, int pass, int env_offset,
                      uint8_t* dir_mask, int E, void* stream);

/* One WindyForestFire CA step (ca_windy.py:41-51, scipy convolve2d mode="same",
 * fill=empty, then the 3 thresholds of _translate_analogic_to_discrete :102-139).
 * Env e participates iff steps == NULL || steps[e] > pass; it reads
 * buf[parity ? parity[e] : 0] and writes the other buffer (parity is NOT flipped here).
 * force_exact = 1 selects the literal threshold kernel; 0 lets the library use the
 * SWAR kernel when it is exact (empty == 0, all cells in {empty, tree, fire}: the
 * caller guarantees the latter; W = 16*2^j <= 1024, 16-B aligned buffers).
 * counts (nullable, [E][3] empty/tree/fire of the NEW grid) are ACCUMULATED with
 * atomics: the caller zeroes the participating rows first.                    */
int gca_windy_step(uint8_t* buf0, uint8_t* buf1, const uint8_t* parity, const int32_t* steps, int pass,
                   const uint8_t* dir_mask, int E, int H, int W, int empty, int tree, int fire,
                   int force_exact, int32_t* counts, void* stream);

/* --------------------------------------------- ForestFireBulldozer (batched)
 * bulldozer.py:393-400 MDP = RepeatCA (repeat_ca.py:32-45) then MoveModify
 * (move_modify.py:128-134); reward/done bulldozer.py:180-216.                 */
typedef struct {
    double t_move[9];        /* _movement_timings (bulldozer.py:277-286)      */
    double t_shoot[2];       /* _shooting_timings                              */
    double t_any;            /* time_per_state (bulldozer.py:297)              */
    uint64_t seed;           /* Philox key for the windy roll                  */
    int32_t env_offset;      /* global id of env 0 of this shard               */
    int32_t empty, tree, fire;
    int32_t up_mask, down_mask, left_mask, right_mask; /* action sets as bitmasks over 0..8 */
    int16_t effect[256];     /* Modify effects: new value, or -1 if not a key  */
} gca_bulldozer_params;

/* Before the CA passes: for live envs (done[e]==0) accu += (t_move[a0]+t_shoot[a1]) + t_any,
 * (accu, steps) = modf(accu); zero counts of stepping envs; dir_mask for pass 0.
 * Done envs get steps = 0.                                                      */
int gca_bulldozer_pre(const gca_bulldozer_params* p, const int32_t* action, double* accu, int32_t* steps,
                      const uint8_t* done, const double* wind, int64_t wind_stride, const uint32_t* rng_step,
                      uint8_t* dir_mask, int32_t* counts, int E, void* stream);
/* Between CA passes `pass` and `pass+1`: flip parity of envs that stepped in `pass`;
 * for envs stepping again, zero their counts and draw the dir_mask for pass+1.  */
int gca_bulldozer_interpass(const gca_bulldozer_params* p, int pass, const int32_t* steps, uint8_t* parity,
                            const double* wind, int64_t wind_stride, const uint32_t* rng_step, uint8_t* dir_mask,
                            int32_t* counts, int E, void* stream);
/* After the last pass (index last_pass): flip parity, Move, Modify (in place on the
 * current buffer), adjust counts, reward = -(f/(t+f)) (NaN if t+f==0), done = (f==0),
 * rng_step += steps. Done-on-entry envs: reward 0, nothing moves.                  */
int gca_bulldozer_post(const gca_bulldozer_params* p, int last_pass, const int32_t* action, const int32_t* steps,
                       uint8_t* parity, uint8_t* buf0, uint8_t* buf1, int H, int W, int32_t* pos,
                       int32_t* counts, uint32_t* rng_step, uint8_t* done, uint8_t* hit, double* reward,
                       int E, void* stream);

/* The whole ForestFireBulldozer env step in one launch (bulldozer.py:393-400 MDP.update + ca_env.py:27-62 reward /
 * done), one workgroup per env: the gca_bulldozer_pre bookkeeping, when a CA step is due (steps[e] = 1) the Windy
 * direction mask and the row-stream CA of gca_windy_step on the env's grid, then gca_bulldozer_post's Move / Modify,
 * counts, reward, done, hit, rng_step and parity; steps_elapsed (nullable) += 1 for live envs. Identical results to
 * the three-kernel sequence. Requires W = 256 or 512, empty = 0 < tree < fire, 16-B aligned buffers and one CA pass
 * at most per env step ((t_move + t_shoot) + t_any < 1 for every action; otherwise GCA_ERR_ARG).
 * meet (nullable): E 64-bit slots, zero-initialised once by the caller (every launch leaves them zero); with them the
 * step runs as 2 (W = 256) / 4 (W = 512) workgroups per env that meet in one atomic per env, the last to arrive writing
 * the env's outputs — the same results; NULL: one workgroup per env. Not shared between concurrent launches. The
 * slots pack 20-bit counts, so grids with H*W + 1 >= 2^20 cells ignore `meet` and run one workgroup per env.   */
int gca_bulldozer_step_fused(const gca_bulldozer_params* p, const int32_t* action, double* accu, int32_t* steps,
                             uint8_t* done, const double* wind, int64_t wind_stride, uint32_t* rng_step,
                             uint8_t* parity, uint8_t* buf0, uint8_t* buf1, int H, int W, int32_t* pos,
                             int32_t* counts, uint8_t* hit, double* reward, int64_t* steps_elapsed, uint64_t* meet,
                             int E, void* stream);
/* gca_bulldozer_step_fused under a random policy: every env's action is drawn inside the step exactly as
 * gca_random_actions(action, E, p->env_offset, action_seed, rng_step) draws it before the step (move randint[0, 9),
 * shoot the top bit, Philox keyed by the global env id and rng_step[e]) -- the pair of launches in one, bit for bit --
 * and written to action_out (nullable, [E][2]). For random rollouts (action_space.sample() per env per step).       */
int gca_bulldozer_step_fused_random(const gca_bulldozer_params* p, uint64_t action_seed, int32_t* action_out,
                                    double* accu, int32_t* steps, uint8_t* done, const double* wind,
                                    int64_t wind_stride, uint32_t* rng_step, uint8_t* parity, uint8_t* buf0,
                                    uint8_t* buf1, int H, int W, int32_t* pos, int32_t* counts, uint8_t* hit,
                                    double* reward, int64_t* steps_elapsed, uint64_t* meet, int E, void* stream);
/* K env steps of every env in ONE launch under gca_bulldozer_step_fused_random's random policy (r06): bit for bit K
 * consecutive gca_bulldozer_step_fused_random calls with the same action_seed (the batched form of K iterations of the
 * reference loop `env.step(env.action_space.sample())`, bulldozer.py:393-400, ca_env.py:27-62); one workgroup per env
 * keeps the env's state in registers across the K steps. Optional per-step outputs: action_out (K, E, 2) int32,
 * reward_out (K, E) f64, done_out (K, E) u8 (as `done` after each step). Same contract as gca_bulldozer_step_fused
 * (W = 256 / 512, one CA pass at most per env step, empty = 0 < tree < fire). */
int gca_bulldozer_rollout_random(const gca_bulldozer_params* p, uint64_t action_seed, int K, int32_t* action_out,
                                 double* reward_out, uint8_t* done_out, double* accu, int32_t* steps, uint8_t* done,
                                 const double* wind, int64_t wind_stride, uint32_t* rng_step, uint8_t* parity,
                                 uint8_t* buf0, uint8_t* buf1, int H, int W, int32_t* pos, int32_t* counts, uint8_t* hit,
                                 double* reward, int64_t* steps_elapsed, int E, void* stream);

/* Move then Modify for E envs (move_modify.py:37-134): action[e] = (move, shoot);
 * uses p->up/down/left/right_mask and p->effect; grid may be NULL (Move only); hit nullable. */
int gca_move_modify(const gca_bulldozer_params* p, const int32_t* action, int32_t* pos, uint8_t* grid, int H, int W,
                    uint8_t* hit, int E, void* stream);

/* -------------------------------------------- Alexandridis (advanced env CA) */
typedef struct {
    int32_t R;                 /* burn_kernel_radius (ca_alexandridis_jax.py:62)              */
    float heat_dw[GCA_MAX_RADIUS + 1]; /* w_k - w_{k+1} (f32), w_k = heat weight at Chebyshev distance k (k=0 centre, w_{R+1}=0), :108-153 */
    float dous_inner, dous_border;    /* 5x5 dousing weights :64-105                          */
    float veg1p[6], den1p[6];  /* 1 + veg_probs / den_probs, f32 (:170-184, clip 1..5)        */
    float p_tree;              /* shared_context["p_tree"] (:386)                              */
    int32_t age_lo, age_hi;    /* randint(fire_age_min, fire_age_max) bounds, truncated (:368) */
    uint64_t seed;
    int32_t env_offset;
    int32_t empty, tree, fire; /* 0, 1, 2 in AdvancedForestFireBulldozerEnv                  */
    int32_t n_winds;
    float winds[16][9];        /* shared_context["winds"][i][0] wind matrices (row-major 3x3)  */
    float heat0;               /* initial value of the heat sum: 0 for the JAX rule; the classic
                                  PartiallyObservableForestFire's constant p_h = 0.58 with every
                                  heat_dw / dousing weight 0 (ca_alexandridis.py:94)             */
    int32_t burnout_eq1;       /* 0: FIRE -> EMPTY iff age <= 1 (ca_alexandridis_jax.py:389);
                                  1: iff age == 1, i.e. the decremented age hits 0 (classic
                                  ca_alexandridis.py:181-183). Ages are decremented either way. */
    int32_t vd_uniform;        /* gca_alex_step_march* with vd = NULL (uniform layers, flat terrain only): the packed
                                  byte vegetation | density << 4 of every cell of every env (init_vegetation_same /
                                  init_density_same, advanced_bulldozer.py:190-195); unused otherwise */
} gca_alex_params;

/* p_slope[e][d][r][c] = slope_factor(0.078f * slope[e][r][c][d']) for the 8 non-centre d'
 * (ca_alexandridis_jax.py:199-200: exp(0.078 * slope)); slope_factor(a) = exp_f32(a) for a >= 0 and
 * 1 / exp_f32(-a) for a < 0 (IEEE division), exp_f32 the deterministic expf of DESIGN.md. */
int gca_alex_prepare_slope(const float* slope, float* p_slope, int E, int H, int W, void* stream);

/* One CA step of PartiallyObservableForestFireJax._update_grid (ca_alexandridis_jax.py:321-424).
 * grid u8, fire_age i16, vegetation/density/dousing u8 (E,H,W); p_slope (E,8,H,W) f32.
 * Draws: inj_burn [E][H][W][9] f32, inj_grow [E][H][W] f32, inj_age [E][H][W] i32 (all three
 *        given = injected mode, the reference rule verbatim), or all NULL = Philox mode
 *        (burn test against 1 - prod(1 - clamp01(p_d)); one Philox4x32-10 block per 4 cells (r, 4g .. 4g+3),
 *        counter (r * ceil(W/4) + g, env_offset + e, rng_step[e], ALXC): cell j tests word j's high 24 bits,
 *        the group's first new fire takes randint of the words' low bytes, its 2nd..4th words 0..2 of the
 *        ALXA block of the same counter).
 * prob_out (nullable, debug) [E][H][W][8] f32 burn probabilities of every cell.
 * counts (nullable) [E][3] of the NEW grid, OVERWRITTEN (memset inside).          */
int gca_alex_step(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                  const int16_t* age_in, int16_t* age_out, const uint8_t* veg, const uint8_t* den,
                  const uint8_t* dousing, const float* p_slope, const int32_t* wind_index, const uint32_t* rng_step,
                  const float* inj_burn, const float* inj_grow, const int32_t* inj_age, float* prob_out,
                  int32_t* counts, void* stream);

/* gca_alex_step with the slopes in the antisymmetric edge layout of gca_alex_edge_slope_from_altitude
 * (16 B per cell instead of p_slope's 32): edge_slope (E,4,H,W) f32. Valid for slopes that come from an
 * altitude field through get_slope (init_utils.py:166-200), the only slopes the Advanced env has
 * (advanced_bulldozer.py:182-204); results are bit-identical to gca_alex_step on the p_slope that
 * gca_alex_slope_from_altitude builds from the same altitude. Same replaced code and draws as above. */
int gca_alex_step_es(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                     const int16_t* age_in, int16_t* age_out, const uint8_t* veg, const uint8_t* den,
                     const uint8_t* dousing, const float* edge_slope, const int32_t* wind_index,
                     const uint32_t* rng_step, const float* inj_burn, const float* inj_grow, const int32_t* inj_age,
                     float* prob_out, int32_t* counts, void* stream);

/* gca_alex_step_es on the Advanced env's packed layout (Philox mode, W % 256 == 0, H % 16 == 0, 16-B aligned
 * arrays): vd[e][r][c] = min(veg, 7) | min(den, 7) << 4; dous_bits[e][r][c / 16] bit c % 16 = (dousing != 0)
 * (the env's dousing counts are 0/1: ModifyJax writes 1, move_modify_jax.py:102-114); edge_slope_coal = the edge
 * layout with every 256-column row segment of a plane in coalesced order (gca_alex_edge_slope_coalesce).
 * Results are bit-identical to gca_alex_step_es on the unpacked arrays. Same replaced code as gca_alex_step.
 * Tile activity map (nullable): act_out[e][tile] (u8, tiles of 16 rows x 256 columns, row-major) receives 1 iff
 * the step leaves a FIRE in that tile; with act_in = the previous step's act_out (or all ones), a tile whose 3 x 3
 * tile neighbourhood has no fire is copied instead of stepped (exact when p_tree == 0: act_in is ignored
 * otherwise). act_out is required with act_in; act_out alone just records the map. */
int gca_alex_step_packed(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                         const int16_t* age_in, int16_t* age_out, const uint8_t* vd, const uint16_t* dous_bits,
                         const float* edge_slope_coal, const int32_t* wind_index, const uint32_t* rng_step,
                         int32_t* counts, const uint8_t* act_in, uint8_t* act_out, void* stream);
/* gca_alex_step_packed that ALSO writes the env's step observation of the plain case (enable_extensions = False, the
 * reference's default; advanced_bulldozer.py:1035-1101, :1120): rgb [E][H][W][3] f32 of every cell = the colour of its
 * NEW state (empty / tree / fire; other codes the empty colour) under the PRE-step is_night[e], water-tinted where its
 * PRE-step dousing bit is set (the MDP renders with the input per_env_context, :1121) — the frame gca_adv_observation
 * (mode 0) renders from the same inputs, minus the bulldozer's pixel, which gca_obs_position adds once the env step
 * has moved it. color_table [2][3][2][4] f32 from gca_obs_color_table (16-B aligned, like rgb). */
int gca_alex_step_packed_rgb(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                             const int16_t* age_in, int16_t* age_out, const uint8_t* vd, const uint16_t* dous_bits,
                             const float* edge_slope_coal, const int32_t* wind_index, const uint32_t* rng_step,
                             int32_t* counts, const uint8_t* act_in, uint8_t* act_out, const float* color_table,
                             const int32_t* is_night, float* rgb, void* stream);
/* gca_alex_step_packed / _rgb in marching form for W == 256 (H % 16 == 0): one wave walks one 16 x 256 tile row by
 * row (gca_alex_march.hip), every slope byte read once. Same replaced code, arguments, results (bit for bit), tile
 * activity map and frame, except edge_slope: the edge layout (E,4,H,W) in natural column order (the output of
 * gca_alex_edge_slope_from_altitude, not coalesced), or NULL for flat terrain: every slope factor 1, as when every edge
 * value is +-1 (use_hidden=False: init_altitude_same, advanced_bulldozer.py:190-197, gives zero slopes) — no slope
 * planes are read (7.125 instead of 23.125 B / cell) and the results are those of the all-ones planes, bit for bit.
 * With edge_slope = NULL, vd may be NULL too: every cell's packed layer byte is p->vd_uniform (6.125 B / cell). */
int gca_alex_step_march(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                        const int16_t* age_in, int16_t* age_out, const uint8_t* vd, const uint16_t* dous_bits,
                        const float* edge_slope, const int32_t* wind_index, const uint32_t* rng_step, int32_t* counts,
                        const uint8_t* act_in, uint8_t* act_out, void* stream);
int gca_alex_step_march_rgb(const gca_alex_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                            const int16_t* age_in, int16_t* age_out, const uint8_t* vd, const uint16_t* dous_bits,
                            const float* edge_slope, const int32_t* wind_index, const uint32_t* rng_step,
                            int32_t* counts, const uint8_t* act_in, uint8_t* act_out, const float* color_table,
                            const int32_t* is_night, float* rgb, void* stream);
/* vd (nullable) and dous_bits of gca_alex_step_packed from veg / den / dousing (E,H,W) u8; W % 16 == 0. */
int gca_alex_pack_layers(const uint8_t* veg, const uint8_t* den, const uint8_t* dousing, uint8_t* vd,
                         uint16_t* dous_bits, int E, int H, int W, void* stream);
/* edge_slope (E,4,H,W) -> coalesced order: inside every 256-column segment of a row, column 16q + 4m + j moves
 * to position 64m + 4q + j (W % 256 == 0). */
int gca_alex_edge_slope_coalesce(const float* edge_slope, float* edge_slope_coal, int E, int H, int W, void* stream);

/* Edge-slope layout for gca_alex_step_es from altitude [E][H][W] f64 (NULL = flat): edge_slope[e][k][r][c] =
 * V = +exp_f32(a) if a >= 0 else -exp_f32(-a), a = 0.078f * s, s = f32(degrees(atan((alt[r][c] - alt[n]) /
 * (1.414 if diagonal)))) toward neighbour n = k-th of (-1,-1), (-1,0), (-1,+1), (0,-1) (s = 0 where n is
 * outside the grid): get_slope (init_utils.py:166-200) without its border zeroing, which the step applies
 * per cell. p_slope everywhere is slope_factor(a) = exp_f32(a) (a >= 0) or 1/exp_f32(-a) (a < 0), so
 * both directions of an edge come from V: P(a) = V > 0 ? V : 1/|V|, P(-a) = V < 0 ? |V| : 1/|V|.      */
int gca_alex_edge_slope_from_altitude(const double* altitude, float* edge_slope, int E, int H, int W, void* stream);
/* (own, neighbour) factors the step derives from n edge values V, with the step's own arithmetic
 * (v_rcp_f32 + Newton reciprocal): the hook the exhaustive reciprocal test calls.                   */
int gca_alex_edge_factors(const float* v, float* own, float* nbr, int64_t n, void* stream);

/* Wind change of PartiallyObservableForestFireJax.update (ca_alexandridis_jax.py:442-451) for E envs:
 * u < p_wind_change -> wind_index = (wind_index + k) % n_winds, k in [1, 8).
 * inj_u/inj_k injected draws, or both NULL -> Philox((0, env_offset+e, rng_step[e], ALXW)) words 0/1. */
int gca_alex_wind_change(float p_wind_change, int n_winds, uint64_t seed, int env_offset, const uint32_t* rng_step,
                         const float* inj_u, const int32_t* inj_k, int32_t* wind_index, int E, void* stream);

/* get_slope (init_utils.py:166-200) on the device from altitude [E][H][W] f64 (NULL = flat),
 * f64 -> f32 like jnp.array, then p_slope as in gca_alex_prepare_slope. slope_out (nullable)
 * receives the f32 slope [E][H][W][3][3]. */
int gca_alex_slope_from_altitude(const double* altitude, float* p_slope, float* slope_out, int E, int H, int W,
                                 void* stream);

/* init_altitude's arithmetic (bulldozer/utils/init_utils.py:76-116) on the device. altitude [E][H][W]
 * holds the noise field on entry (the reference's uniform(0, 5) draws) and the altitude on return:
 * per cell, in the reference's order, += height * cos(dist / radius * pi / 2) for every hill with
 * dist < radius, += height_diff * (row - start_row) / height inside every slope rectangle, then / 10.
 * hills [E][GCA_MAX_HILLS][4] = (centre row, centre col, radius, height), n_hills [E] (<= 10);
 * slopes [E][GCA_MAX_SLOPES][5] = (start row, start col, width, height, height_diff), n_slopes [E] (<= 8).
 * Integer fields are stored as doubles. The random draws stay on the host (legacy np.random order). */
#define GCA_MAX_HILLS 10
#define GCA_MAX_SLOPES 8
int gca_alex_altitude_apply(double* altitude, int E, int H, int W, const int32_t* n_hills, const double* hills,
                            const int32_t* n_slopes, const double* slopes, void* stream);

/* Hidden layers drawn on the device (init_utils.py:10-116's recipe, Philox draws keyed by the GLOBAL env id,
 * so sharded runs draw what the unsharded run draws; not the reference's np.random stream — the envs'
 * hidden_rng="philox" mode). Per env (counter (slot, env_offset + e, 0, GCA_TAG_HIDDEN)):
 *   vegetation / density: randint(4, 8) patches (centre randint(0, R) x randint(0, C), size randint(3, max(4,
 *     R//2)) x randint(3, max(4, C//2)), value randint(1, 6)), later patches over earlier ones, uncovered cells
 *     randint(1, 4);
 *   altitude: noise uniform(0, 5) per cell into `altitude`, and the hills / slopes plan of
 *     gca_alex_altitude_apply (randint(6, 10) hills: centre, radius randint(2, max(3, min(R, C)//4)), height
 *     uniform(2, 6); randint(4, 8) slopes: start randint(0, max(1, R-4)) x randint(0, max(1, C-4)), width
 *     randint(3, max(4, C//4)), height randint(3, max(4, R//4)), height_diff uniform(1, 4)).
 * Per cell (counter (r * W + c, env_offset + e, 0, GCA_TAG_HIDDEN_CELL)): word 0 -> vegetation fill, word 1
 * -> density fill, words 2:3 -> noise. Follow with gca_alex_altitude_apply to finish the altitude.          */
int gca_hidden_init(uint64_t seed, int env_offset, int E, int H, int W, uint8_t* vegetation, uint8_t* density,
                    double* altitude, int32_t* n_hills, double* hills, int32_t* n_slopes, double* slopes,
                    void* stream);

/* Pinecone spotting (ca_alexandridis_jax.py:229-319, the scatter :400-420 — disabled in the reference's
 * live path, enabled in our env / operator with pinecones=True), after gca_alex_step* on its output:
 * every FIRE cell of grid_in throws n = min(Poisson(1), max_pinecones) pinecones in direction d (uniform
 * over 8) with integer thrust s = round(N(0,1) * ft[ft_lookup[d]]) of the env's current wind; a pinecone
 * landing on a TREE of grid_out at (clip(r + dx[d] s), clip(c + dy[d] s)) burns it with probability
 * (scale * veg1p[clip(veg)]) * den1p[clip(den)] of the target; the target becomes FIRE with age
 * randint(age_lo, age_hi) and one count moves tree -> fire. Any burning pinecone ignites its target
 * (duplicates). s_cdf [n_winds][8][GCA_PINE_CDF] u32: per (wind, direction) t[0] = 2K, t[1..2K] = 32-bit
 * thresholds of P(s <= -K + j) (gymca_amd/forest_fire/operators/pinecones.py). Draws: Philox blocks
 * (lin, env, step, PINE + 0 / 1 + m) and (target lin, env, step, PINA), see gca_pine.hip. act_tiles
 * (nullable): gca_alex_step_packed's act_out of the same step — the tile of every ignited target is set to 1. */
#define GCA_PINE_MAX 8
#define GCA_PINE_CDF 17
typedef struct {
    uint32_t n_cdf[GCA_PINE_MAX]; /* P(Poisson(1) <= j) * 2^32, j = 0..7                         */
    int32_t max_pinecones;        /* 5 (:230)                                                      */
    int32_t dx[8], dy[8];         /* E, NE, N, NW, W, SW, S, SE tables (:259-260)                  */
    float scale;                  /* 0.48 (:227)                                                    */
    float veg1p[6], den1p[6];     /* 1 + veg_probs / den_probs, f32 (:211-214)                     */
    int32_t age_lo, age_hi;       /* randint(4, 11) (:409)                                          */
    uint64_t seed;
    int32_t env_offset;
    int32_t empty, tree, fire;
} gca_pine_params;
int gca_alex_pinecones(const gca_pine_params* p, int E, int H, int W, const uint8_t* grid_in, uint8_t* grid_out,
                       int16_t* age_out, const uint8_t* veg, const uint8_t* den, const int32_t* wind_index,
                       const uint32_t* s_cdf, const uint32_t* rng_step, int32_t* counts, uint8_t* act_tiles, void* stream);

/* Classic pinecone spotting: PartiallyObservableForestFire.update's sequential skip-list pass
 * (ca_alexandridis.py:184-210, sampling :35-69, ignition :113-133), after gca_alex_step (classic params) on
 * its output. Every FIRE cell s of grid_in, in row-major order, throws N ~ Poisson(1) pinecones (tail folded at
 * GCA_PINEC_NMAX); pinecone m has direction d uniform over 8 and integer thrust s_m = round(3 N(0,1) ft[lookup[d]])
 * (:189-190, ft of the env's current wind), landing at (r + dx[d] s_m, c + dy[d] s_m). A landing inside the grid
 * and not on s itself ignites its target - WHATEVER the target's state - iff u < 0.58 (1 + p_veg) (1 + p_den)
 * of the target (burn_thr: u24 < thr), with a fresh age randint(4, 11). A target that ignites and comes LATER
 * in the scan is skipped by the reference's loop (:151-152): when that target is itself a FIRE cell of grid_in it
 * throws no pinecones. The device resolves that order dependence exactly: one workgroup per env iterates
 * "s is active iff no active earlier source ignites it" to its fixed point (the dependence is a DAG in scan
 * order), then applies the landings of the active sources. Ages are keyed by the target (the last of several
 * ignitions of one target draws a fresh uniform age in the reference: the same law). counts (nullable):
 * one count moves from the target's previous state to FIRE per ignited target.
 * s_cdf [n_winds][8][GCA_PINEC_CDF] u32: per (wind, direction) t[0] = 2K, t[1..2K] thresholds of
 * P(round(3 ft Z) <= -K + j) * 2^32. scratch: NULL when 16 * ceil(H W / 32) bytes fit one workgroup's LDS
 * (H W <= 262144 = 512 x 512), else E * 4 * ceil(H W / 32) u32 of device memory (the kernel clears it).
 * Draws: Philox (lin, env, step, PINEC + 0) -> N, (lin, env, step, PINEC + 1 + m) -> s (word 0), u (word 1 >> 8),
 * d (word 2 >> 29); (target lin, env, step, PINEC_AGE) word 0 -> age. */
#define GCA_PINEC_NMAX 16
#define GCA_PINEC_CDF 48
#define GCA_PINEC_LDS_MAX_HW 262144
typedef struct {
    uint32_t n_cdf[GCA_PINEC_NMAX]; /* P(Poisson(1) <= j) * 2^32, j = 0..15 (N_p = poisson(), :37)              */
    int32_t dx[8], dy[8];           /* dx_lookup / dy_lookup (:63-64)                                          */
    uint32_t burn_thr[6][6];        /* [veg][den]: ceil(p * 2^24), p = 0.58 * (1 + p_veg) * (1 + p_den) in f64 */
    int32_t age_lo, age_hi;         /* integers(4, 11) (:131)                                                  */
    uint64_t seed;
    int32_t env_offset;
    int32_t empty, tree, fire;
} gca_pine_classic_params;
int gca_alex_pinecones_classic(const gca_pine_classic_params* p, int E, int H, int W, const uint8_t* grid_in,
                               uint8_t* grid_out, int16_t* age_out, const uint8_t* veg, const uint8_t* den,
                               const int32_t* wind_index, const uint32_t* s_cdf, const uint32_t* rng_step,
                               int32_t* counts, uint32_t* scratch, void* stream);

/* --------------------------------- AdvancedForestFireBulldozer env step (batched)
 * advanced_bulldozer.py:1103-1133 minus observations, + _award/_is_done :597-633.  */
typedef struct {
    float t_move[9], t_shoot[2], t_any;  /* f32 like the JAX env (all moves cost t_move: :745-760) */
    float p_wind_change;                 /* 0.06 (:210)                                            */
    int32_t day_length;                  /* 400 (:733)                                             */
    uint64_t seed;
    int32_t env_offset;
    int32_t n_winds;
    int32_t up_mask, down_mask, left_mask, right_mask;
} gca_advenv_params;

/* After gca_alex_step: wind change (repeat: ca_alexandridis_jax.py:442-451), time
 * accumulation (repeat_ca_jax.py:191-198, f32), MoveJax, ModifyJax (dousing[r][c] = 1
 * if shoot==1), time_step += 1, is_night toggle, reward = -(f/(t+f+1e-8)) f32,
 * done = no fire, rng_step += 1. dous_bits (nullable): the packed layout's dousing bits, set with dousing.
 * steps_elapsed / reward_accumulated (nullable, f32 [E]): stateless_step's episode statistics
 * info["steps_elapsed"] += 1, info["reward_accumulated"] += reward (advanced_bulldozer.py:396-397).    */
int gca_advenv_post(const gca_advenv_params* p, const int32_t* action, int32_t* pos, float* accu,
                    int32_t* wind_index, int32_t* time_step, int32_t* is_night, uint8_t* dousing, uint16_t* dous_bits,
                    int H, int W, const int32_t* counts, uint32_t* rng_step, float* reward, uint8_t* done,
                    float* steps_elapsed, float* reward_accumulated, int E, void* stream);

/* conditional_reset (advanced_bulldozer.py:422-518): envs with done[e] copy their
 * initial grid/age/dousing/position/time/wind_index (and clear done); dous_bits (nullable, packed layout)
 * are zeroed (only without dousing0).                                             */
int gca_reset_where(const uint8_t* done, int E, int H, int W, uint8_t* grid, const uint8_t* grid0,
                    int16_t* age, const int16_t* age0, uint8_t* dousing, const uint8_t* dousing0,
                    uint16_t* dous_bits, int32_t* pos, const int32_t* pos0, float* accu, int32_t* wind_index,
                    const int32_t* wind_index0, void* stream);

/* ------------------------------------------- Advanced env observations (RGB)
 * MDP.build_observation_on_extensions + grid_to_rgb_with_extensions + grid_to_rgb
 * (advanced_bulldozer.py:988-1101) with apply_blur / apply_visibility / transform_grid /
 * apply_extensions (bulldozer/utils/extension_utils.py:89-196).                       */
#define GCA_OBS_MAX_EXT 4
typedef struct {
    int32_t empty, tree, fire;
    int32_t n_ext;                              /* extension channels (reference registry: 2)       */
    int32_t ext_skip_visibility[GCA_OBS_MAX_EXT];
    int32_t ext_skip_blur[GCA_OBS_MAX_EXT];     /* (unblur: 0/1, see_invisible_fires: 1/0)          */
    int32_t enable_extensions;                  /* MDP.enable_extensions                             */
    int32_t should_transform;                   /* MDP.should_transform_grid                         */
    int32_t day_length;                         /* > 0 with time_step: undo the step's is_night toggle */
    float color_day[4][3];                      /* empty, tree, fire, position (0..255 as f32)       */
    float color_night[4][3];
    float tint_day[3], tint_night[3];           /* water tint of doused cells                        */
    int32_t n_choices;                          /* extension-choice ids (create_up_to_k_mappings)     */
    int32_t ext_lookup[8][GCA_OBS_MAX_EXT];     /* id -> binary extension flags                       */
} gca_obs_params;

/* rgb [E][H][W][3] f32 (and, nullable, channels [E][H][W][3 + n_ext] u8 = transformed grid, 0, 0,
 * extension channels) for E envs.
 * mode 0 (env step, advanced_bulldozer.py:1120): grid/position after the step, dousing and is_night
 *   before it (pass the post-step is_night with time_step to undo its toggle); action [E][action_stride]
 *   full actions (move, shoot, extension choice): the choice (column 2, clamped to n_choices - 1) maps
 *   to binary extension flags through ext_lookup (_create_full_actions :308-330); action NULL or
 *   action_stride < 3 = no extension active.
 * mode 1 (reset, :401-411): the reference applies grid_to_rgb_with_extensions to the raw (H, W)
 *   grid; its broadcasting gives rgb[r][c] = colour(grid[c][k]) with k = 3 + the first row holding a
 *   positive value in columns 3.. (clamped), or k = 0 — reproduced as is (square grids only).
 * env_mask (nullable, u8 [E]): only envs with env_mask[e] != 0 are rendered, the others' rgb/channels
 *   are left untouched — conditional_reset's per-env jnp.where(terminated, new obs, old obs) (:464-481). */
int gca_adv_observation(const gca_obs_params* p, int mode, int E, int H, int W, const uint8_t* grid,
                        const uint8_t* dousing, const int32_t* pos, const int32_t* is_night, const int32_t* time_step,
                        const int32_t* action, int action_stride, float* rgb, uint8_t* channels,
                        const uint8_t* env_mask, void* stream);

/* gca_alex_step_march_rgb for the extension pipeline (W = 256, codes 0 / 1 / 2): the frame of gca_adv_observation
 * mode 0 (action = the full actions, action_stride >= 3) from the CA step's epilogue, minus the bulldozer's pixel
 * (gca_obs_position), for every env whose display is channel 0 of the extended grid -- the grid itself (the unblur
 * choice) or all zeros (see_invisible_fires: its blur is shown only when row 0 of the blur is empty; the reference's
 * row-vs-channel display scan, advanced_bulldozer.py:1035-1064). The kernel checks that speculation on row 0 of the
 * new grid and sets refit[e] = 1 (else 0) when it fails or when the display needs the blurred grid (no extension
 * chosen with should_transform): those envs' frames are left for gca_adv_observation with env_mask = refit, after
 * the env step. Results of the pair are bit for bit gca_adv_observation's. */
int gca_alex_step_march_rgb_ext(const gca_alex_params* p, const gca_obs_params* op, int E, int H, int W,
                                const uint8_t* grid_in, uint8_t* grid_out, const int16_t* age_in, int16_t* age_out,
                                const uint8_t* vd, const uint16_t* dous_bits, const float* edge_slope,
                                const int32_t* wind_index, const uint32_t* rng_step, int32_t* counts,
                                const uint8_t* act_in, uint8_t* act_out, const float* color_table,
                                const int32_t* is_night, float* rgb, const int32_t* action, int action_stride,
                                uint8_t* refit, void* stream);

/* [night][kind empty / tree / fire][dousing 0 / 1] float4 colours (rgb, 0) of grid_to_rgb (advanced_bulldozer.py:1041-1093),
 * the table gca_alex_step_packed_rgb reads: table[12][4] f32 device, 16-B aligned. */
int gca_obs_color_table(const gca_obs_params* p, float* table, void* stream);
/* rgb[e][pos[e]] = the position colour of the PRE-step day / night (is_night after the env step, time_step to undo its
 * toggle; time_step NULL = is_night as given): grid_to_rgb's .at[position].set (:1095-1099) over a fused frame. */
int gca_obs_position(const gca_obs_params* p, int E, int H, int W, const int32_t* pos, const int32_t* is_night,
                     const int32_t* time_step, float* rgb, void* stream);

/* Synthetic inputs for benches/tests (Philox, GCA_TAG_INIT / GCA_TAG_ACTION). */
int gca_fill_categorical(uint8_t* out, int64_t n_per_env, int E, int env_offset, uint64_t seed,
                         const float* cdf, const uint8_t* values, int n_values, void* stream);
int gca_random_actions(int32_t* action, int E, int env_offset, uint64_t seed, const uint32_t* rng_step,
                       void* stream);

/* ------------------------------------------ Drossel-Schwabl (helicopter CA)
 * ForestFire.update (ca_DrosselSchwabl.py:32-66). The reference draws one f64
 * uniform per TREE-without-burning-neighbour and per EMPTY cell, in row-major
 * order, from op.np_random. Exact-stream mode: uniforms[] holds those draws in
 * order (n = gca_ds_count_draws). One workgroup per env (scan over the grid).   */
int gca_ds_count_draws(const uint8_t* grid, int E, int H, int W, int empty, int tree, int fire,
                       int32_t* n_draws, void* stream);
int gca_ds_step(const uint8_t* grid_in, uint8_t* grid_out, int E, int H, int W, int empty, int tree, int fire,
                const double* thresholds /*[E][2]: cdf0 of choice([T,F], p=[p_fire,1-p_fire]), same for p_tree*/,
                const double* uniforms, const int64_t* uniform_offset, uint64_t seed, const uint32_t* rng_step,
                int env_offset, int32_t* counts, void* stream);

/* ------------------------------------------ measurement yardsticks (bench.py; no reference counterpart)
 * gca_bench_copy: a 16-B device copy of nbytes (one element per thread, one pass) (a multiple of 16, 16-B aligned), nt != 0 non-temporal
 * loads and stores: the practical HBM ceiling the bench reports beside the 8 TB/s spec.
 * gca_bench_march_pattern: the loads and stores of gca_alex_step_march at W = 256 (radius R in 4..7; with rgb != NULL
 * also the fused frame's f32 RGB stores) with trivial arithmetic, on the env's packed-layout buffers: the floor of
 * that access pattern on this device; edge_slopes = NULL: the flat-terrain step's pattern (no slope planes), and vd =
 * NULL with it the uniform-layers step's (no vd layer either). Outputs are scratch (their values mean nothing). */
int gca_bench_copy(const void* src, void* dst, int64_t nbytes, int nt, void* stream);
int gca_bench_march_pattern(int R, int E, int H, int W, const uint8_t* grid, uint8_t* grid_out, const int16_t* age,
                            int16_t* age_out, const uint8_t* vd, const uint16_t* dous_bits, const float* edge_slopes,
                            float* rgb, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GCA_H */
