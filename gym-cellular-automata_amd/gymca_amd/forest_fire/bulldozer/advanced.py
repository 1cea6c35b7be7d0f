"""AdvancedForestFireBulldozerEnv — the batched Alexandridis env, resident in HBM.

Reference: advanced_bulldozer.py:63-1133 (JAX, vmap over num_envs). One env step is

    gca_alex_step     RepeatCAJax's single CA step (repeat_ca_jax.py:218-220) of
                      PartiallyObservableForestFireJax._update_grid (ca_alexandridis_jax.py:321-424),
                      new-grid tree/fire counts fused
    gca_advenv_post   wind change (:442-451), f32 time accumulation (repeat_ca_jax.py:191-198),
                      MoveJax/ModifyJax (move_modify_jax.py:39-157), time_step/is_night
                      (advanced_bulldozer.py:1116-1127), reward -(f/(t+f+1e-8)) and done (:597-633),
                      info["steps_elapsed"] / info["reward_accumulated"] (:396-397)

Reference batched API (the drop-in surface, advanced_bulldozer.py:332-518):

    obs, info = env.reset()
    obs, reward, terminated, truncated, info = env.stateless_step(action, obs, info)
    obs, reward, terminated, truncated, info = env.conditional_reset(step_tuple, action)

obs = (rgb f32 (E, H, W, 3), context) with context = {"per_env_context": {...}, "shared_context": {...},
"position": (E, 2), "time": (E,)} — the reference's key sets (:109-129). The tensors are device views of
the env's own HBM state: the JAX env threads state through obs/info functionally, here the state stays
resident and `stateless_step` adopts whatever obs/info it is handed (a tensor that IS the env's buffer costs
nothing; any other value — an older obs, a host array — is copied in). Returned tensors stay valid until the
env's next step (they are the buffers the next step writes), as in other device-resident vector envs.
observation="rgb" (default, the reference's) renders gca_adv_observation: RGB f32 of the
extension/blur/visibility pipeline (:988-1101) and the reset observation (:401-411);
observation="grid" returns the true u8 grid instead (cheaper; not the reference's obs).

Device layout per env: grid u8 (ping-pong), fire_age i16 (ping-pong), vegetation /
density / dousing u8, the slopes in the antisymmetric edge layout f32 [4][H][W]
(0.078 * slope toward the 4 preceding neighbours, built once from altitude; the step
derives the other 4 directions and exp in-kernel: gca_alex_step_es), plus per-env
scalars: 25 B of HBM traffic per cell-update. slope_layout="packed" (the default
"auto" when W % 256 == 0 and H % 16 == 0) runs gca_alex_step_packed on the same state with
vegetation|density in one byte, the 0/1 dousing counts as bits and the edge slopes in coalesced
segment order (23.1 B per cell-update; the u8 layers stay the API's context). At W = 256 the packed
layout's step is the marching kernel (gca_alex_step_march: one wave walks a 16 x 256 tile row by row,
the edge slopes in natural column order); step_kernel="tiled" keeps gca_alex_step_packed there.
slope_layout="planes" keeps the general 8-plane p_slope f32 [8][H][W] = exp(0.078*slope) (41 B per
cell-update).
"""
import numpy as np

from ... import _device as dev
from ..._lib import AdvEnvParams, call
from ..._seeding import env_integers
from ..operators.ca_alexandridis import make_alex_params
from .bulldozer import ACTION_SETS, bulldozer_timings
from .init_utils import altitude_plan, device_altitude, get_winds, init_density, init_vegetation
from .observation import make_obs_params


class AdvancedForestFireBulldozerEnv:
    def __init__(self, nrows, ncols, key=0, num_envs=8, speed_move=0.12, speed_act=0.03, speed_multiplier=1.0,
                 pos_bull=None, pos_fire=None, t_move=None, t_shoot=None, t_any=0.001, p_tree=0.90, p_empty=0.10,
                 use_hidden=True, middle_fire=False, enable_extensions=False, device=None, env_offset=0,
                 hidden_rng=None, slope_layout="auto", observation="rgb", pinecones=False, tile_skip=False,
                 step_kernel="auto"):
        import torch

        self.device = dev.require_device(device)
        self.nrows, self.ncols, self.num_envs = int(nrows), int(ncols), int(num_envs)
        E, H, W = self.num_envs, self.nrows, self.ncols
        self.key = int(key)
        self.env_offset = int(env_offset)
        self.use_hidden = use_hidden
        self.middle_fire = middle_fire
        self._empty, self._tree, self._fire = 0, 1, 2
        self._p_tree_init, self._p_empty_init = p_tree, p_empty
        self._pos_bull = _per_env_bull(pos_bull, self.num_envs)
        self._pos_fire = _per_env_fire(pos_fire, self.num_envs)
        self._p_fire = 0.00033
        self._p_tree = 0.0  # advanced_bulldozer.py:209
        self._p_wind_change = 0.06
        self._day_length = 400
        self._winds = np.asarray(get_winds(use_hidden), dtype=np.float32)  # (8, 2, 3, 3)
        t_act_move, t_act_shoot = bulldozer_timings(H, W, speed_move, speed_act, t_move, t_shoot, t_any)
        self.alex_params, self.constants = make_alex_params(H, self._empty, self._tree, self._fire, self._winds,
                                                            self._p_tree, self.key, self.env_offset)
        ep = AdvEnvParams()
        for a in range(9):  # all moves, not_move included, cost t_move (:753-754)
            ep.t_move[a] = float(np.float32(t_act_move))
        ep.t_shoot[0] = ep.t_shoot[1] = float(np.float32(t_act_shoot))
        ep.t_any = float(np.float32(t_any))
        ep.p_wind_change = float(np.float32(self._p_wind_change))
        ep.day_length = self._day_length
        ep.seed = self.key & (2**64 - 1)
        ep.env_offset = self.env_offset
        ep.n_winds = len(self._winds)
        from ..operators.move_modify import make_params

        mp = make_params(ACTION_SETS)
        ep.up_mask, ep.down_mask, ep.left_mask, ep.right_mask = mp.up_mask, mp.down_mask, mp.left_mask, mp.right_mask
        self.env_params = ep
        # pinecone spotting after each CA step (ca_alexandridis_jax.py:229-319, :400-420; commented out in the
        # reference's _update_grid, so off by default): gca_alex_pinecones with the step's wind
        self.pinecones = bool(pinecones)
        if self.pinecones:
            from ..operators.pinecones import make_pine_params, s_cdf_tables

            self.pine_params = make_pine_params(self.key, self._empty, self._tree, self._fire, self.env_offset)

        kw = dict(device=self.device)
        self.grid = torch.zeros((2, E, H, W), dtype=torch.uint8, **kw)
        self.age = torch.zeros((2, E, H, W), dtype=torch.int16, **kw)
        self.cur = 0
        self.vegetation = torch.full((E, H, W), 3, dtype=torch.uint8, **kw)
        self.density = torch.full((E, H, W), 3, dtype=torch.uint8, **kw)
        self.dousing = torch.zeros((E, H, W), dtype=torch.uint8, **kw)
        if slope_layout == "auto":
            slope_layout = "packed" if (W % 256 == 0 and H % 16 == 0) else "edge"
        if slope_layout not in ("edge", "planes", "packed"):
            raise ValueError("slope_layout must be 'auto', 'edge', 'packed' or 'planes'")
        if slope_layout == "packed" and (W % 256 or H % 16):
            raise ValueError("slope_layout='packed' needs W % 256 == 0 and H % 16 == 0")
        self.slope_layout = slope_layout
        if step_kernel not in ("auto", "march", "tiled"):
            raise ValueError("step_kernel must be 'auto', 'march' or 'tiled'")
        if step_kernel == "march" and (slope_layout != "packed" or W not in (256, 512, 1024)):
            raise ValueError("step_kernel='march' needs the packed layout at W = 256, 512 or 1024")
        self._step_kernel = step_kernel
        if slope_layout == "packed":  # the packed step updates ages in place: both "buffers" are one (stride 0)
            self.age = torch.zeros((E, H, W), dtype=torch.int16, **kw).unsqueeze(0).expand(2, E, H, W)
        # edge: (E, 4, H, W) edge values for gca_alex_step_es (packed: the same in coalesced order);
        # planes: (E, 8, H, W) p_slope for gca_alex_step
        self.slope_data = torch.zeros((E, 8 if slope_layout == "planes" else 4, H, W), dtype=torch.float32, **kw)
        # packed layout extras: vd = min(veg, 7) | min(den, 7) << 4 and the dousing bits (u16 per 16 columns)
        self.vd = torch.zeros((E, H, W), dtype=torch.uint8, **kw) if slope_layout == "packed" else None
        self.dous_bits = torch.zeros((E, H * W // 16), dtype=torch.int16, **kw) if slope_layout == "packed" else None
        # tile activity map of the tiled packed step (16 x 256 tiles; ping-pong with the grid): tiles whose 3 x 3 tile
        # neighbourhood holds no fire are copied instead of stepped (exact: p_tree = 0 here); all ones = unknown.
        # Opt-in, tiled step only (the marching step derives the same from the grid)
        self.act = None
        self.set_tile_skip(tile_skip)
        self.wind_index = torch.zeros(E, dtype=torch.int32, **kw)
        self.pine_tables = (torch.as_tensor(s_cdf_tables(self._winds).view(np.int32), **kw) if self.pinecones
                            else None)
        self.pos = torch.zeros((E, 2), dtype=torch.int32, **kw)
        self.accu = torch.zeros(E, dtype=torch.float32, **kw)
        self.time_step = torch.ones(E, dtype=torch.int32, **kw)
        self.is_night = torch.zeros(E, dtype=torch.int32, **kw)
        self.rng_step = torch.zeros(E, dtype=torch.int32, **kw)
        self.counts = torch.zeros((E, 3), dtype=torch.int32, **kw)
        self.reward = torch.zeros(E, dtype=torch.float32, **kw)
        self.done = torch.zeros(E, dtype=torch.uint8, **kw)
        self.steps_elapsed = torch.zeros(E, dtype=torch.float32, **kw)
        self.reward_accumulated = torch.zeros(E, dtype=torch.float32, **kw)
        self.truncated = torch.zeros(E, dtype=torch.bool, **kw)  # the reference never truncates (:392)
        self._winds_dev = torch.as_tensor(self._winds, device=self.device)
        self._initial = None
        self._mdp = None
        if observation not in ("grid", "rgb"):
            raise ValueError("observation must be 'grid' or 'rgb'")
        if observation == "rgb" and H != W:
            # the reference's reset observation broadcasts the raw (H, W) grid against (W, W)-shaped colour
            # arrays (advanced_bulldozer.py:405-409), so it only exists for square grids
            raise ValueError("observation='rgb' (the reference's) needs a square grid; use observation='grid'")
        self.observation = observation
        self.enable_extensions = bool(enable_extensions)
        # MDP(should_transform_grid = transform_grid and enable_extensions, ...) (advanced_bulldozer.py:293-302)
        self.obs_params = make_obs_params(self._empty, self._tree, self._fire, self.enable_extensions,
                                          self.enable_extensions, self._day_length)
        self.rgb = torch.zeros((E, H, W, 3), dtype=torch.float32, **kw) if observation == "rgb" else None
        # the plain observation (no extension channel, no transform: the reference's default) is written by the CA
        # step itself on the packed layout (gca_alex_step_packed_rgb) and the bulldozer's pixel by gca_obs_position;
        # extensions, other layouts and pinecones (which ignite cells after the step) render it in its own pass
        # the extension pipeline's fused frame: envs whose display the step's epilogue cannot render (refit = 1) are
        # rendered by gca_adv_observation after the env step (gca_alex_step_march_rgb_ext)
        self._refit = torch.zeros(E, dtype=torch.uint8, **kw) if self.rgb is not None else None
        self._no_ext = torch.zeros((E, 3), dtype=torch.int32, **kw) if self.rgb is not None else None
        self.obs_colors = torch.zeros((12, 4), dtype=torch.float32, **kw)
        call("gca_obs_color_table", self.obs_params, dev.ptr(self.obs_colors), dev.stream_ptr(self.device))
        self._build_context_layers(hidden_rng)

    # ------------------------------------------------------------------ init
    def _build_context_layers(self, rng):
        """density / vegetation / altitude -> slope, once per env instance like the reference's
        constructor (advanced_bulldozer.py:182-204). With use_hidden the layers come from the
        init_utils restatement, which consumes `rng` (default: the global np.random state, as the
        reference does) draw for draw; altitude's arithmetic and get_slope run on the device.
        rng="philox" draws the same recipe on the device instead (gca_hidden_init)."""
        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        self.altitude = None
        if self.use_hidden and isinstance(rng, str):
            if rng != "philox":
                raise ValueError("hidden_rng: None, a numpy random source, or 'philox'")
            import torch

            # the same recipe drawn on the device, keyed by the global env id (gca_hidden_init): milliseconds
            # instead of seconds at E = 4096, and shard-invariant; not the reference's np.random stream
            self.altitude = torch.empty((E, H, W), dtype=torch.float64, device=self.device)
            nh = torch.empty(E, dtype=torch.int32, device=self.device)
            ns = torch.empty(E, dtype=torch.int32, device=self.device)
            hills = torch.empty((E, 10, 4), dtype=torch.float64, device=self.device)
            slopes = torch.empty((E, 8, 5), dtype=torch.float64, device=self.device)
            call("gca_hidden_init", self.key & (2**64 - 1), self.env_offset, E, H, W, dev.ptr(self.vegetation),
                 dev.ptr(self.density), dev.ptr(self.altitude), dev.ptr(nh), dev.ptr(hills), dev.ptr(ns),
                 dev.ptr(slopes), st)
            call("gca_alex_altitude_apply", dev.ptr(self.altitude), E, H, W, dev.ptr(nh), dev.ptr(hills), dev.ptr(ns),
                 dev.ptr(slopes), st)
        elif self.use_hidden:
            import torch

            den = init_density(H, W, E, rng)
            veg = init_vegetation(H, W, E, rng)
            self.density.copy_(torch.as_tensor(np.clip(den, 0, 255).astype(np.uint8), device=self.device))
            self.vegetation.copy_(torch.as_tensor(np.clip(veg, 0, 255).astype(np.uint8), device=self.device))
            self.altitude = device_altitude(altitude_plan(H, W, E, rng), self.device)
        else:
            self.density.fill_(3)
            self.vegetation.fill_(3)
        self._slopes_from(self.altitude)
        self._pack_layers()

    def set_tile_skip(self, on):
        """Switch the packed step's tile activity map on / off (the map restarts as "every tile active"). The marching
        step finds its quiet tiles from the grid itself (cheaper than keeping the map: 0.41 vs 0.51 ms per 4096 x 256^2
        step from the reset state, BENCH r03), so there tile_skip keeps no map and changes nothing; the map serves the
        tiled step (step_kernel="tiled")."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        if on and self.slope_layout != "packed":
            raise ValueError("tile skipping needs the packed layout (W % 256 == 0, H % 16 == 0)")
        self.tile_skip = bool(on)
        self.act = (torch.ones((2, E, (H // 16) * (W // 256)), dtype=torch.uint8, device=self.device)
                    if on and not self.march else None)

    def _pack_layers(self, layers=True):
        """vd and dousing bits of the packed layout from the u8 layers (no-op for the other layouts); `layers`:
        vegetation / density may have changed (uniform_layers is re-derived), not only the dousing."""
        if self.vd is None:
            return
        E, H, W = self.num_envs, self.nrows, self.ncols
        call("gca_alex_pack_layers", dev.ptr(self.vegetation), dev.ptr(self.density), dev.ptr(self.dousing),
             dev.ptr(self.vd), dev.ptr(self.dous_bits), E, H, W, dev.stream_ptr(self.device))
        if layers and hasattr(self, "flat_terrain"):  # (construction packs before the slopes; _slopes_from refreshes)
            self._refresh_layers()

    @property
    def march(self):
        """True when the packed step runs the marching kernel (W = 256, 512, 1024; edge slopes in natural column
        order); other widths (W % 256 == 0) run the tiled kernel on the coalesced layout."""
        return self.slope_layout == "packed" and self.ncols in (256, 512, 1024) and self._step_kernel != "tiled"

    def _slopes_from(self, altitude):
        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        if self.slope_layout == "edge" or self.march:
            call("gca_alex_edge_slope_from_altitude", dev.ptr(altitude), dev.ptr(self.slope_data), E, H, W, st)
        elif self.slope_layout == "packed":
            import torch

            tmp = torch.empty_like(self.slope_data)
            call("gca_alex_edge_slope_from_altitude", dev.ptr(altitude), dev.ptr(tmp), E, H, W, st)
            call("gca_alex_edge_slope_coalesce", dev.ptr(tmp), dev.ptr(self.slope_data), E, H, W, st)
            del tmp
        else:
            call("gca_alex_slope_from_altitude", dev.ptr(altitude), dev.ptr(self.slope_data), None, E, H, W, st)
        self.refresh_terrain()

    def refresh_terrain(self):
        """Re-derive `flat_terrain` from the slope buffer: True when every edge value is +-1, i.e. every slope factor of
        every env is exactly 1 (use_hidden=False: init_altitude_same gives zero slopes, exp_f32(0) = 1). The marching
        step then streams no slope planes (gca_alex_step_march with edge_slope = NULL; bit for bit the same step).
        On flat terrain `uniform_layers` says whether every cell of every env has the same packed vegetation / density
        byte (use_hidden=False: init_vegetation_same / init_density_same); then the step reads no vd layer either (vd =
        NULL, the byte in alex_params.vd_uniform). The env calls it whenever it sets the slopes or the layers
        (construction, set_state(altitude= / vegetation= / density=), adopted contexts); call it after writing
        `slope_data` or `vd` in place (new vegetation / density go through set_state, which repacks vd)."""
        self.flat_terrain = self.slope_layout != "planes" and bool((self.slope_data.abs() == 1.0).all())
        self._refresh_layers()

    def _refresh_layers(self):
        """`uniform_layers` from the packed vd layer (flat terrain only; see refresh_terrain)."""
        self.uniform_layers = False
        vd = getattr(self, "vd", None)
        if self.flat_terrain and vd is not None:
            v0 = int(vd.reshape(-1)[0])
            if (v0 & 0x88) == 0 and bool((vd == v0).all()):
                self.alex_params.vd_uniform = v0
                self.uniform_layers = True

    def p_slope_planes(self):
        """The general 8-plane p_slope (E, 8, H, W) = exp_f32(0.078 * slope) of this env's altitude
        (gca_alex_slope_from_altitude), e.g. for the oracle; the step itself may use the edge layout."""
        import torch

        if self.slope_layout == "planes":
            return self.slope_data
        E, H, W = self.num_envs, self.nrows, self.ncols
        out = torch.empty((E, 8, H, W), dtype=torch.float32, device=self.device)
        call("gca_alex_slope_from_altitude", dev.ptr(self.altitude), dev.ptr(out), None, E, H, W,
             dev.stream_ptr(self.device))
        return out

    def reset(self, *, seed=None, options=None):
        """Initial state of advanced_bulldozer.py:650-743 for every env; returns (obs, info) like :401-420."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        # grid iid over {EMPTY, TREE} (p_empty, p_tree), two fires with age (N + N//2) * 2 (:650-688)
        cdf = torch.tensor([self._p_empty_init, self._p_empty_init + self._p_tree_init, 1.0], dtype=torch.float32,
                           device=self.device)
        vals = torch.tensor([self._empty, self._tree, self._fire], dtype=torch.uint8, device=self.device)
        self.cur = 0
        call("gca_fill_categorical", dev.ptr(self.grid[0]), H * W, E, self.env_offset,
             (self.key if seed is None else int(seed)) & (2**64 - 1), dev.ptr(cdf), dev.ptr(vals), 3, st)
        self.age[0].zero_()
        # fires: per env the cells of pos_fire[env] (default (3N/4, N/4) and its left neighbour, or the middle),
        # age (N + N//2) * 2 (:664-688). Negative indices wrap as in the reference's .at[].set; a cell outside
        # the grid raises here (JAX would drop the update silently)
        if self._pos_fire is not None:
            fires = self._pos_fire
        else:
            r, c = (H // 2, W // 2) if self.middle_fire else (3 * H // 4, W // 4)
            fires = [[(r, c), (r, c - 1)]] * E
        ei = np.array([e for e in range(E) for _ in fires[e]], np.int64)
        rc = np.array([p for e in range(E) for p in fires[e]], np.int64).reshape(-1, 2)
        if rc.size and ((rc[:, 0] < -H).any() or (rc[:, 0] >= H).any() or (rc[:, 1] < -W).any() or
                        (rc[:, 1] >= W).any()):
            raise ValueError("pos_fire holds a cell outside the grid")
        rc = rc % np.array([H, W])
        idx = (torch.as_tensor(ei, device=self.device), torch.as_tensor(rc[:, 0], device=self.device),
               torch.as_tensor(rc[:, 1], device=self.device))
        self.grid[0].index_put_(idx, torch.tensor(self._fire, dtype=torch.uint8, device=self.device))
        self.age[0].index_put_(idx, torch.tensor((H + H // 2) * 2, dtype=torch.int16, device=self.device))
        # bulldozer: pos_bull[env], default (int(0.15 N), int(0.85 N)) (:690-700)
        bull = self._pos_bull if self._pos_bull is not None else [(int(H * 0.15), int(W * 0.85))] * E
        b = np.asarray(bull, np.int64).reshape(E, 2)
        if ((b[:, 0] < 0) | (b[:, 0] >= H) | (b[:, 1] < 0) | (b[:, 1] >= W)).any():
            raise ValueError(f"pos_bull holds a position outside the {H}x{W} grid")
        self.pos.copy_(torch.as_tensor(np.asarray(bull, np.int32).reshape(E, 2), device=self.device))
        # initial wind index per env (:703-709), keyed by the global env id (shard-invariant)
        wi = (env_integers(self.key if seed is None else int(seed), self.env_offset, E, 0x57494E44, 0, 8)
              if self.use_hidden else np.zeros(E))
        self.wind_index.copy_(torch.as_tensor(wi.astype(np.int32), device=self.device))
        self.dousing.zero_()
        if self.dous_bits is not None:
            self.dous_bits.zero_()
        if self.act is not None:
            self.act.fill_(1)
        self.accu.zero_()
        self.time_step.fill_(1)
        self.is_night.zero_()
        self.rng_step.zero_()
        self.done.zero_()
        self.reward.zero_()
        self.steps_elapsed.zero_()
        self.reward_accumulated.zero_()
        call("gca_count_cells", dev.ptr(self.grid[0]), E, H, W, self._empty, self._tree, self._fire,
             dev.ptr(self.counts), st)
        self._initial = dict(grid=self.grid[0].clone(), age=self.age[0].clone(), pos=self.pos.clone(),
                             wind_index=self.wind_index.clone(), counts=self.counts.clone())
        if self.rgb is not None:  # the reference's reset observation (advanced_bulldozer.py:405-409)
            call("gca_adv_observation", self.obs_params, 1, E, H, W, dev.ptr(self.grid[0]), dev.ptr(self.dousing),
                 dev.ptr(self.pos), dev.ptr(self.is_night), None, None, 0, dev.ptr(self.rgb), None, None, st)
        return self._obs(), self._info()

    def set_state(self, grid=None, fire_age=None, vegetation=None, density=None, wind_index=None, dousing=None,
                  altitude=None, position=None):
        """Overwrite parts of the device state (synthetic mid-episode states for benches/tests)."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)

        def put(dst, x, dtype):
            dst.copy_(x.to(dst.device, dtype) if dev.is_device_tensor(x) else torch.as_tensor(np.asarray(x), dtype=dtype,
                                                                                           device=self.device))

        if grid is not None:
            put(self.grid[self.cur], grid, torch.uint8)
        if fire_age is not None:
            put(self.age[self.cur], fire_age, torch.int16)
        if vegetation is not None:
            put(self.vegetation, vegetation, torch.uint8)
        if density is not None:
            put(self.density, density, torch.uint8)
        if wind_index is not None:
            wt = wind_index if dev.is_device_tensor(wind_index) else torch.as_tensor(np.asarray(wind_index))
            if wt.numel() and (bool((wt < 0).any()) or bool((wt >= len(self._winds)).any())):
                raise ValueError(f"wind_index: values must index the env's {len(self._winds)} wind matrices")
            put(self.wind_index, wind_index, torch.int32)
        if dousing is not None:
            put(self.dousing, dousing, torch.uint8)
            if self.dous_bits is not None and bool((self.dousing > 1).any()):
                raise ValueError("the packed layout stores dousing counts as bits: values must be 0/1 "
                                 "(use slope_layout='edge' for other counts)")
        if position is not None:
            pt = (position if dev.is_device_tensor(position) else torch.as_tensor(np.asarray(position))).reshape(-1, 2)
            if bool(((pt[:, 0] < 0) | (pt[:, 0] >= self.nrows) | (pt[:, 1] < 0) | (pt[:, 1] >= self.ncols)).any()):
                raise ValueError(f"position: every (row, col) must lie inside the {self.nrows}x{self.ncols} grid")
            put(self.pos, position, torch.int32)
        if altitude is not None:
            alt = altitude if dev.is_device_tensor(altitude) else torch.as_tensor(np.asarray(altitude, np.float64),
                                                                                 device=self.device)
            self.altitude = alt.to(self.device, torch.float64).contiguous()
            self._slopes_from(self.altitude)
        if vegetation is not None or density is not None or dousing is not None:
            self._pack_layers(layers=vegetation is not None or density is not None)
        if self.act is not None:  # the state may have fire anywhere now
            self.act.fill_(1)
        call("gca_count_cells", dev.ptr(self.grid[self.cur]), E, H, W, self._empty, self._tree, self._fire,
             dev.ptr(self.counts), st)

    # ------------------------------------------------------------------ obs / info (reference layout)
    def _context(self):
        """The reference's context dict (advanced_bulldozer.py:109-129, :711-743) over device views.
        Layout differences: "key" is the per-env Philox step counter (the JAX PRNG key's role), "slope" the
        step's slope layout (edge values (E, 4, H, W), coalesced when packed off W = 256, or p_slope planes
        (E, 8, H, W)
        instead of (E, H, W, 3, 3)), "fire_age" i16, "true_grid" / "dousing_count" / "vegetation" / "density"
        u8; "altitude" is None without hidden layers."""
        per_env = {"wind_index": self.wind_index, "density": self.density, "vegetation": self.vegetation,
                   "altitude": self.altitude, "slope": self.slope_data, "fire_age": self.age[self.cur],
                   "key": self.rng_step, "is_night": self.is_night, "true_grid": self.grid[self.cur],
                   "time_step": self.time_step, "dousing_count": self.dousing}
        shared = {"winds": self._winds_dev, "p_fire": self._p_fire, "p_tree": self._p_tree,
                  "p_wind_change": self._p_wind_change, "day_length": self._day_length}
        return {"per_env_context": per_env, "shared_context": shared, "position": self.pos, "time": self.accu}

    def reference_context(self):
        """The context in the reference's own layout (advanced_bulldozer.py:109-129, :711-743), materialised on the
        device: true_grid / fire_age f32, density / vegetation / dousing_count / wind_index / time_step / is_night
        int32, altitude f64, slope (E, H, W, 3, 3) f32 (get_slope of the altitude; zeros without one), "key" the
        per-env Philox step counter. For callers of env.MDP.update or code that reads the reference's keys; the
        step itself keeps the compact layout of _context()."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        i32 = torch.int32
        slope = torch.zeros((E, H, W, 3, 3), dtype=torch.float32, device=self.device)
        alt = self.altitude if self.altitude is not None else torch.zeros((E, H, W), dtype=torch.float64,
                                                                          device=self.device)
        if self.altitude is not None:
            tmp = torch.empty((E, 8, H, W), dtype=torch.float32, device=self.device)
            call("gca_alex_slope_from_altitude", dev.ptr(self.altitude), dev.ptr(tmp), dev.ptr(slope), E, H, W,
                 dev.stream_ptr(self.device))
        per_env = {"wind_index": self.wind_index.clone(), "density": self.density.to(i32),
                   "vegetation": self.vegetation.to(i32), "altitude": alt.clone(), "slope": slope,
                   "fire_age": self.age[self.cur].to(torch.float32), "key": self.rng_step.clone(),
                   "is_night": self.is_night.clone(), "true_grid": self.grid[self.cur].to(torch.float32),
                   "time_step": self.time_step.clone(), "dousing_count": self.dousing.to(i32)}
        shared = {"winds": self._winds_dev, "p_fire": self._p_fire, "p_tree": self._p_tree,
                  "p_wind_change": self._p_wind_change, "day_length": self._day_length}
        return {"per_env_context": per_env, "shared_context": shared, "position": self.pos.clone(),
                "time": self.accu.clone()}

    def _obs(self):
        return (self.rgb if self.rgb is not None else self.grid[self.cur]), self._context()

    def _info(self):
        return {"reward": self.reward, "terminated": self.done.bool(), "TimeLimit.truncated": self.truncated,
                "steps_elapsed": self.steps_elapsed, "reward_accumulated": self.reward_accumulated}

    @property
    def MDP(self):
        """The per-env MDP operator (advanced_bulldozer.py:66-68, 956-1133) wired to this env:
        MDP.update(grid, action, per_env_context, shared_context, position, time) on the reference's context
        layout, one env or a leading env axis (stateless_step's vmap). See advanced_mdp.py."""
        if self._mdp is None:
            from .advanced_mdp import make_env_mdp

            self._mdp = make_env_mdp(self)
        return self._mdp

    def _is_own(self, x, buf):
        return (dev.is_device_tensor(x) and x.data_ptr() == buf.data_ptr() and x.dtype == buf.dtype
                and tuple(x.shape) == tuple(buf.shape))

    def _adopt(self, obs=None, info=None):
        """Make the env's device state the one `obs` / `info` describe (the functional reference threads state
        through them, :332-399). Values that are this env's own buffers are skipped (zero cost in the usual loop
        that passes back what the last call returned); anything else is validated first — nothing is written
        when any value is refused — and then copied in. Honoured beyond the step state: a foreign "slope" (the
        env's own layout, or the reference's (E, H, W, 3, 3) / (E, H, W, 9), which switches the env to the general
        8-plane layout), "altitude" (carried, unread by the step as in the reference) and the shared context's
        "winds", "p_tree", "p_wind_change" and "day_length". Refused with ValueError: shapes that match neither
        layout, non-integer or out-of-range cell codes / fire ages, dousing counts > 1 on the packed layout."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        plan = []  # (name, source tensor on the device, destination buffer)

        def src_of(x, name, buf, integral=None):
            if x is None or self._is_own(x, buf):
                return
            t = x if dev.is_device_tensor(x) else torch.as_tensor(np.asarray(x))
            if tuple(t.shape) != tuple(buf.shape):
                raise ValueError(f"{name}: shape {tuple(t.shape)} does not match the env's {tuple(buf.shape)}")
            t = t.to(self.device)
            if integral is not None and t.numel():
                lo, hi = integral
                if t.is_floating_point() and not bool(torch.equal(t, torch.round(t))):
                    raise ValueError(f"{name}: values must be integers (the reference's states are integer-valued)")
                if bool((t < lo).any()) or bool((t > hi).any()):
                    raise ValueError(f"{name}: values outside [{lo}, {hi}] do not fit the env's layout")
            plan.append((name, t, buf))

        slope_src = altitude_src = None
        shared = {}
        if obs is not None:
            ctx = obs[1]
            pe = ctx.get("per_env_context", {})
            # the slope source and the shared context first: a reference-layout slope switches the env to the
            # 8-plane layout (dousing counts beyond 1 allowed), and adopted winds set the wind_index range
            slope_src = self._slope_source(pe.get("slope"))
            shared = self._shared_changes(ctx.get("shared_context"))
            n_winds = len(shared["winds"]) if "winds" in shared else len(self._winds)
            src_of(pe.get("true_grid"), "true_grid", self.grid[self.cur], (0, 255))
            src_of(pe.get("fire_age"), "fire_age", self.age[self.cur], (-32768, 32767))
            to_planes = slope_src is not None and slope_src[0] == "ref"
            dous_hi = 1 if (self.dous_bits is not None and not to_planes) else 255
            src_of(pe.get("dousing_count"), "dousing_count", self.dousing, (0, dous_hi))
            src_of(pe.get("vegetation"), "vegetation", self.vegetation, (0, 255))
            src_of(pe.get("density"), "density", self.density, (0, 255))
            src_of(pe.get("wind_index"), "wind_index", self.wind_index, (0, n_winds - 1))
            if "winds" in shared and not any(name == "wind_index" for name, _, _ in plan):
                if int(self.wind_index.max().item()) >= n_winds:
                    raise ValueError("winds: fewer wind matrices than the current wind indices need")
            src_of(pe.get("is_night"), "is_night", self.is_night, (0, 1))
            src_of(pe.get("time_step"), "time_step", self.time_step)
            src_of(pe.get("key"), "key", self.rng_step)
            src_of(ctx.get("position"), "position", self.pos, (0, max(H, W) - 1))
            for name, t, _ in plan:  # rows and columns each inside the grid (the kernels' scatters assume it)
                if name == "position" and t.numel() and (bool((t[:, 0] >= H).any()) or bool((t[:, 1] >= W).any())):
                    raise ValueError(f"position: every (row, col) must lie inside the {H}x{W} grid")
            src_of(ctx.get("time"), "time", self.accu)
            if obs[0] is not None and self.rgb is not None:
                src_of(obs[0], "rgb", self.rgb)
            alt = pe.get("altitude")
            if alt is not None and not (self.altitude is not None and self._is_own(alt, self.altitude)):
                a = alt if dev.is_device_tensor(alt) else torch.as_tensor(np.asarray(alt))
                if tuple(a.shape) != (E, H, W):
                    raise ValueError(f"altitude: shape {tuple(a.shape)} is not ({E}, {H}, {W})")
                altitude_src = a
        if info is not None:
            src_of(info.get("steps_elapsed"), "steps_elapsed", self.steps_elapsed)
            src_of(info.get("reward_accumulated"), "reward_accumulated", self.reward_accumulated)
            src_of(info.get("reward"), "reward", self.reward)
        # everything validated: apply
        touched = set()
        for name, t, buf in plan:
            buf.copy_(t.to(dtype=buf.dtype))
            touched.add(name)
        if altitude_src is not None:  # carried like the reference's context; the step reads the slopes only
            self.altitude = altitude_src.to(self.device, torch.float64).contiguous().clone()
        if slope_src is not None:
            self._adopt_slope(*slope_src)
        if shared:
            self._apply_shared(shared)
        if {"vegetation", "density", "dousing_count"} & touched:
            self._pack_layers(layers=bool({"vegetation", "density"} & touched))
        if "true_grid" in touched:
            if self.act is not None:
                self.act.fill_(1)
            call("gca_count_cells", dev.ptr(self.grid[self.cur]), self.num_envs, self.nrows, self.ncols, self._empty,
                 self._tree, self._fire, dev.ptr(self.counts), dev.stream_ptr(self.device))

    def _slope_source(self, x):
        """None (own buffer / absent) or (kind, tensor): kind "env" = this env's slope layout, "ref" = the
        reference's f32 slopes (E, H, W, 9)."""
        import torch

        if x is None or self._is_own(x, self.slope_data):
            return None
        E, H, W = self.num_envs, self.nrows, self.ncols
        t = x if dev.is_device_tensor(x) else torch.as_tensor(np.asarray(x))
        shp = tuple(t.shape)
        if shp == tuple(self.slope_data.shape):
            return "env", t.to(self.device, torch.float32).contiguous()
        if shp in ((E, H, W, 3, 3), (E, H, W, 9)):
            t = t.to(self.device, torch.float32).reshape(E, H, W, 9).contiguous()
            if bool((t.abs() > 90).any()):
                raise ValueError("slope: degrees outside [-90, 90] (the reference's slope space)")
            return "ref", t
        raise ValueError(f"slope: shape {shp} is neither the env's layout {tuple(self.slope_data.shape)} nor the "
                         f"reference's ({E}, {H}, {W}, 3, 3)")

    def _adopt_slope(self, kind, t):
        import torch

        if kind == "env":
            self.slope_data.copy_(t)
            self.refresh_terrain()
            return
        # arbitrary slopes need the general layout: 8 p_slope planes (gca_alex_step, 41 B per cell-update)
        if self.slope_layout != "planes":
            self._to_planes_layout()
        E, H, W = self.num_envs, self.nrows, self.ncols
        call("gca_alex_prepare_slope", dev.ptr(t), dev.ptr(self.slope_data), E, H, W, dev.stream_ptr(self.device))
        self.refresh_terrain()

    def _to_planes_layout(self):
        """Switch the step to the 8-plane p_slope layout (gca_alex_step) keeping the state: separate age buffers,
        no packed vd / dousing bits / tile map."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        ages = torch.zeros((2, E, H, W), dtype=torch.int16, device=self.device)
        ages[self.cur].copy_(self.age[self.cur])
        self.age = ages
        self.slope_data = torch.zeros((E, 8, H, W), dtype=torch.float32, device=self.device)
        self.slope_layout = "planes"
        self.vd = self.dous_bits = self.act = None

    def _shared_changes(self, sc):
        """The shared-context values that differ from the env's (validated, not yet applied)."""
        if not sc:
            return {}
        out = {}
        w = sc.get("winds")
        if w is not None and w is not self._winds_dev:
            wn = (w.cpu().numpy() if dev.is_device_tensor(w) else np.asarray(w)).astype(np.float32)
            if wn.ndim != 4 or wn.shape[1:] != (2, 3, 3) or not 1 <= wn.shape[0] <= 16:
                raise ValueError("winds: expected (n, 2, 3, 3) with 1 <= n <= 16 (wind matrix, ft pairs)")
            if not np.array_equal(wn, self._winds):
                out["winds"] = wn
        for k, cur in (("p_tree", self._p_tree), ("p_wind_change", self._p_wind_change),
                       ("day_length", self._day_length)):
            v = sc.get(k)
            if v is None:
                continue
            v = float(v.item()) if dev.is_device_tensor(v) else float(np.asarray(v))
            if v != cur:
                if k == "day_length" and (v != int(v) or v < 1):
                    raise ValueError("day_length must be a positive integer")
                out[k] = v
        return out

    def _apply_shared(self, ch):
        import torch

        if "winds" in ch:  # (the wind_index range was checked against these winds before anything was written)
            w = ch["winds"]
            self._winds = w
            self._winds_dev = torch.as_tensor(w, device=self.device)
            self.alex_params.n_winds = self.env_params.n_winds = len(w)
            for i, m in enumerate(w[:, 0]):
                for j in range(9):
                    self.alex_params.winds[i][j] = float(m.reshape(9)[j])
            if self.pinecones:
                from ..operators.pinecones import s_cdf_tables

                self.pine_tables = torch.as_tensor(s_cdf_tables(w).view(np.int32), device=self.device)
        if "p_tree" in ch:
            self._p_tree = ch["p_tree"]
            self.alex_params.p_tree = float(np.float32(ch["p_tree"]))
        if "p_wind_change" in ch:
            self._p_wind_change = ch["p_wind_change"]
            self.env_params.p_wind_change = float(np.float32(ch["p_wind_change"]))
        if "day_length" in ch:
            self._day_length = int(ch["day_length"])
            self.env_params.day_length = self._day_length
            self.obs_params.day_length = self._day_length
        self._mdp = None

    def _full_action(self, action):
        import torch

        full = action if dev.is_device_tensor(action) else torch.as_tensor(np.asarray(action), device=self.device)
        return full.to(device=self.device, dtype=torch.int32).reshape(self.num_envs, -1).contiguous()

    def render_observation(self, action=None, channels=None):
        """The step observation (gca_adv_observation mode 0) of the current state into self.rgb; `action`
        (E, >= 3) int32 device tensor carries the extension choice; `channels` (E, H, W, 5) u8 receives the
        channel stack. Uses the post-step is_night / time_step to recover the pre-step day/night."""
        E, H, W = self.num_envs, self.nrows, self.ncols
        a = action if (action is not None and action.shape[-1] >= 3) else None
        call("gca_adv_observation", self.obs_params, 0, E, H, W, dev.ptr(self.grid[self.cur]), dev.ptr(self.dousing),
             dev.ptr(self.pos), dev.ptr(self.is_night), dev.ptr(self.time_step), dev.ptr(a),
             0 if a is None else int(a.shape[-1]), dev.ptr(self.rgb), dev.ptr(channels), None,
             dev.stream_ptr(self.device))
        return self.rgb

    @property
    def _ext_frame(self):
        """The extension pipeline (enable_extensions / should_transform) is rendered by the step's epilogue too: the
        marching step at W = 256 (gca_alex_step_march_rgb_ext), with gca_adv_observation refitting the envs whose
        display needs the blurred grid (finish_frame)."""
        return ((self.enable_extensions or bool(self.obs_params.should_transform)) and bool(self.march)
                and self.ncols == 256 and (self._empty, self._tree, self._fire) == (0, 1, 2))

    @property
    def fused_observation(self):
        """True when env.step's RGB observation comes out of the CA step's own epilogue (see __init__)."""
        if self.rgb is None or self.slope_layout != "packed" or self.pinecones:
            return False
        plain = not self.enable_extensions and not self.obs_params.should_transform
        return plain or self._ext_frame

    def ca_step(self, render=False, action=None):
        """The CA step alone (RepeatCAJax's one step) for every env; swaps the ping-pong buffers. render=True (with
        fused_observation) also writes the step's RGB frame, all but the bulldozer's pixel; with the extension
        pipeline on, `action` holds the full actions (E, >= 3) whose third column chooses the extension, and
        finish_frame(action) completes the frame after the env step."""
        E, H, W = self.num_envs, self.nrows, self.ncols
        a, b = self.cur, 1 - self.cur
        if self.slope_layout == "packed":
            flat = self.march and self.flat_terrain
            args = (self.alex_params, E, H, W, dev.ptr(self.grid[a]), dev.ptr(self.grid[b]),
                    dev.ptr(self.age[a]), dev.ptr(self.age[b]),
                    dev.ptr(None if flat and self.uniform_layers else self.vd), dev.ptr(self.dous_bits),
                    dev.ptr(None if flat else self.slope_data), dev.ptr(self.wind_index),
                    dev.ptr(self.rng_step), dev.ptr(self.counts),
                    dev.ptr(None if self.act is None else self.act[a]), dev.ptr(None if self.act is None else self.act[b]))
            fn = "gca_alex_step_march" if self.march else "gca_alex_step_packed"
            if render:
                if not self.fused_observation:
                    raise ValueError("ca_step(render=True) needs fused_observation")
                if self._ext_frame:
                    full = self._ext_action(action)
                    call("gca_alex_step_march_rgb_ext", args[0], self.obs_params, *args[1:], dev.ptr(self.obs_colors),
                         dev.ptr(self.is_night), dev.ptr(self.rgb), dev.ptr(full), int(full.shape[1]),
                         dev.ptr(self._refit), dev.stream_ptr(self.device))
                else:
                    call(fn + "_rgb", *args, dev.ptr(self.obs_colors), dev.ptr(self.is_night), dev.ptr(self.rgb),
                         dev.stream_ptr(self.device))
            else:
                call(fn, *args, dev.stream_ptr(self.device))
            self._pinecones(a, b)
            self.cur = b
            return
        fn = "gca_alex_step_es" if self.slope_layout == "edge" else "gca_alex_step"
        call(fn, self.alex_params, E, H, W, dev.ptr(self.grid[a]), dev.ptr(self.grid[b]),
             dev.ptr(self.age[a]), dev.ptr(self.age[b]), dev.ptr(self.vegetation), dev.ptr(self.density),
             dev.ptr(self.dousing), dev.ptr(self.slope_data), dev.ptr(self.wind_index), dev.ptr(self.rng_step),
             None, None, None, None, dev.ptr(self.counts), dev.stream_ptr(self.device))
        self._pinecones(a, b)
        self.cur = b

    def _pinecones(self, a, b):
        if self.pinecones:
            E, H, W = self.num_envs, self.nrows, self.ncols
            call("gca_alex_pinecones", self.pine_params, E, H, W, dev.ptr(self.grid[a]), dev.ptr(self.grid[b]),
                 dev.ptr(self.age[b]), dev.ptr(self.vegetation), dev.ptr(self.density), dev.ptr(self.wind_index),
                 dev.ptr(self.pine_tables), dev.ptr(self.rng_step), dev.ptr(self.counts),
                 dev.ptr(None if self.act is None else self.act[b]), dev.stream_ptr(self.device))

    def _ext_action(self, action):
        """The full actions (E, >= 3) int32 device tensor the extension frame reads (no extension: choice 0)."""
        if action is None or action.dim() != 2 or action.shape[1] < 3:
            return self._no_ext
        return action

    def finish_frame(self, action=None):
        """After ca_step(render=True) and post_step: the bulldozer's pixel at its new position, and (extension
        pipeline) the frames of the envs the step's epilogue left to gca_adv_observation (refit)."""
        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        call("gca_obs_position", self.obs_params, E, H, W, dev.ptr(self.pos), dev.ptr(self.is_night),
             dev.ptr(self.time_step), dev.ptr(self.rgb), st)
        if self._ext_frame:
            full = self._ext_action(action)
            call("gca_adv_observation", self.obs_params, 0, E, H, W, dev.ptr(self.grid[self.cur]), dev.ptr(self.dousing),
                 dev.ptr(self.pos), dev.ptr(self.is_night), dev.ptr(self.time_step), dev.ptr(full),
                 int(full.shape[1]), dev.ptr(self.rgb), None, dev.ptr(self._refit), st)

    def step(self, action):
        """Gymnasium-style step of every env: action (E, 2) or (E, 3) ints (move, shoot[, extension choice]),
        device tensor or numpy. Returns (obs, reward, terminated, truncated, info) like stateless_step."""
        full = self._full_action(action)
        fused = self.fused_observation
        self.ca_step(render=fused, action=full)
        self.post_step(full[:, :2].contiguous(), stats=True)
        if fused:  # the frame came with the CA step; the bulldozer's pixel at its new position (+ refits)
            self.finish_frame(full)
        elif self.rgb is not None:
            self.render_observation(full)
        return self._obs(), self.reward, self.done.bool(), self.truncated, self._info()

    def stateless_step(self, action, obs=None, info=None):
        """The reference's batched step (advanced_bulldozer.py:332-399): action (E, 3) = (move, shoot, extension
        choice); obs / info as returned by reset / the previous call (their state is adopted, see _adopt).
        Returns (obs, reward, terminated, truncated, info) with info["reward" / "terminated" /
        "TimeLimit.truncated" / "steps_elapsed" / "reward_accumulated"]."""
        self._adopt(obs, info)
        return self.step(action)

    def post_step(self, action2, stats=False):
        """gca_advenv_post for (E, 2) int32 device actions: wind change, time, Move/Modify, reward, done
        (+ the info episode statistics steps_elapsed / reward_accumulated when `stats`)."""
        E, H, W = self.num_envs, self.nrows, self.ncols
        call("gca_advenv_post", self.env_params, dev.ptr(action2), dev.ptr(self.pos), dev.ptr(self.accu),
             dev.ptr(self.wind_index), dev.ptr(self.time_step), dev.ptr(self.is_night), dev.ptr(self.dousing),
             dev.ptr(self.dous_bits), H, W, dev.ptr(self.counts), dev.ptr(self.rng_step), dev.ptr(self.reward),
             dev.ptr(self.done), dev.ptr(self.steps_elapsed if stats else None),
             dev.ptr(self.reward_accumulated if stats else None), E, dev.stream_ptr(self.device))

    def conditional_reset(self, step_tuple=None, action=None, *, seed=None, options=None):
        """The reference's conditional_reset (advanced_bulldozer.py:422-518): envs whose `terminated` flag is
        set in `step_tuple` (default: this env's last step) get their initial state back — grid, fire ages,
        dousing, wind index, position, time, RNG key; time_step / is_night are kept (:497-507) — and their
        observation is rebuilt from the initial grid with `action`'s extension choice and the step's (pre-reset)
        per-env context (:455-481). info steps_elapsed / reward_accumulated restart at 0 for them, the reward
        is the award of the resulting grid and `terminated` comes back all False (:509-516). Every launch exits
        at once for live envs, so nothing syncs with the host (the reference's lax.cond, :518-523). `seed` and
        `options` are accepted for signature parity; like the reference's traced initial_state they change
        nothing."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        if step_tuple is not None:
            obs, _, terminated, _, info = step_tuple
            self._adopt(obs, info)
            if terminated is not None:
                t = terminated if dev.is_device_tensor(terminated) else torch.as_tensor(np.asarray(terminated))
                if not (dev.is_device_tensor(t) and t.data_ptr() == self.done.data_ptr()):
                    self.done.copy_(t.reshape(E).to(device=self.device, dtype=torch.uint8))
        init = self._initial
        mask = self.done.bool()
        if self.rgb is not None:
            # the re-injected envs' observation: initial grid and position, the step's dousing and is_night
            # (no day/night undo: the context is the post-step one), action's extension choice; others untouched
            a = None if action is None else self._full_action(action)
            call("gca_adv_observation", self.obs_params, 0, E, H, W, dev.ptr(init["grid"]), dev.ptr(self.dousing),
                 dev.ptr(init["pos"]), dev.ptr(self.is_night), None, dev.ptr(a), 0 if a is None else int(a.shape[-1]),
                 dev.ptr(self.rgb), None, dev.ptr(self.done), st)
        self.steps_elapsed.masked_fill_(mask, 0)
        self.reward_accumulated.masked_fill_(mask, 0.0)
        self.rng_step.masked_fill_(mask, 0)  # the reference re-injects the initial JAX key
        if self.act is not None:  # re-injected envs: their fire is back, every tile active
            self.act[self.cur].masked_fill_(mask[:, None], 1)
        self.counts.copy_(torch.where(mask[:, None], init["counts"], self.counts))
        t, f = self.counts[:, 1].float(), self.counts[:, 2].float()
        self.reward.copy_(torch.where(mask, -(f / (t + f + 1e-8)), self.reward))
        call("gca_reset_where", dev.ptr(self.done), E, H, W, dev.ptr(self.grid[self.cur]), dev.ptr(init["grid"]),
             dev.ptr(self.age[self.cur]), dev.ptr(init["age"]), dev.ptr(self.dousing), None,
             dev.ptr(self.dous_bits), dev.ptr(self.pos),
             dev.ptr(init["pos"]), dev.ptr(self.accu), dev.ptr(self.wind_index), dev.ptr(init["wind_index"]), st)
        return self._obs(), self.reward, self.done.bool(), self.truncated, self._info()


def _per_env_bull(pos_bull, E):
    """pos_bull as the reference takes it — a list of E (row, col) pairs (advanced_bulldozer.py:690-700) — or one
    (row, col) pair for every env; None = the default. Returns a list of E pairs or None."""
    if pos_bull is None:
        return None
    a = np.asarray(pos_bull, dtype=np.int64)
    if a.shape == (2,):
        return [tuple(int(v) for v in a)] * E
    if a.shape == (E, 2):
        return [tuple(int(v) for v in row) for row in a]
    raise ValueError(f"pos_bull must be (row, col) or a list of {E} (row, col) pairs, got shape {a.shape}")


def _per_env_fire(pos_fire, E):
    """pos_fire as the reference takes it — per env a list of (row, col) fire cells (advanced_bulldozer.py:664-688:
    [[(r, c), (r, c - 1)], ...]) — or one (row, col) pair, meaning (r, c) and (r, c - 1) in every env (the
    reference's default pattern). None = the default. Returns a list of E lists of pairs or None."""
    if pos_fire is None:
        return None
    if np.asarray(pos_fire, dtype=object).shape == (2,) and all(np.isscalar(v) for v in pos_fire):
        r, c = int(pos_fire[0]), int(pos_fire[1])
        return [[(r, c), (r, c - 1)]] * E
    if len(pos_fire) != E:
        raise ValueError(f"pos_fire must be (row, col) or a list of {E} per-env lists of (row, col) cells")
    out = []
    for cells in pos_fire:
        a = np.asarray(cells, dtype=np.int64).reshape(-1, 2) if len(cells) else np.zeros((0, 2), np.int64)
        out.append([tuple(int(v) for v in row) for row in a])
    return out
