"""AdvancedForestFireBulldozerEnv — the batched Alexandridis env, resident in HBM.

Reference: advanced_bulldozer.py:63-1133 (JAX, vmap over num_envs). One env step is

    gca_alex_step     RepeatCAJax's single CA step (repeat_ca_jax.py:218-220) of
                      PartiallyObservableForestFireJax._update_grid (ca_alexandridis_jax.py:321-424),
                      new-grid tree/fire counts fused
    gca_advenv_post   wind change (:442-451), f32 time accumulation (repeat_ca_jax.py:191-198),
                      MoveJax/ModifyJax (move_modify_jax.py:39-157), time_step/is_night
                      (advanced_bulldozer.py:1116-1127), reward -(f/(t+f+1e-8)) and done (:597-633)

and `conditional_reset` (:422-518) re-injects the initial state of finished envs with
gca_reset_where. observation="rgb" adds the reference's observation (gca_adv_observation:
RGB f32 (E, H, W, 3) of the extension/blur/visibility pipeline, :988-1101, and the reset
observation :401-411); observation="grid" (default) returns the true u8 grid instead.

Device layout per env: grid u8 (ping-pong), fire_age i16 (ping-pong), vegetation /
density / dousing u8, the slopes in the antisymmetric edge layout f32 [4][H][W]
(0.078 * slope toward the 4 preceding neighbours, built once from altitude; the step
derives the other 4 directions and exp in-kernel: gca_alex_step_es), plus per-env
scalars: 25 B of HBM traffic per cell-update. slope_layout="packed" (the default
"auto" when W % 256 == 0 and H % 16 == 0) runs gca_alex_step_packed on the same state with
vegetation|density in one byte, the 0/1 dousing counts as bits and the edge slopes in coalesced
segment order (23.1 B per cell-update; the u8 layers stay the API's context). slope_layout="planes"
keeps the general 8-plane p_slope f32 [8][H][W] = exp(0.078*slope) (41 B per cell-update).
"""
import numpy as np

from ... import _device as dev
from ..._lib import AdvEnvParams, call
from ..operators.ca_alexandridis import alex_constants, make_alex_params
from .bulldozer import ACTION_SETS, bulldozer_timings
from .init_utils import altitude_plan, device_altitude, get_winds, init_density, init_vegetation
from .observation import make_obs_params


class AdvancedForestFireBulldozerEnv:
    def __init__(self, nrows, ncols, key=0, num_envs=8, speed_move=0.12, speed_act=0.03, speed_multiplier=1.0,
                 pos_bull=None, pos_fire=None, t_move=None, t_shoot=None, t_any=0.001, p_tree=0.90, p_empty=0.10,
                 use_hidden=True, middle_fire=False, enable_extensions=False, device=None, env_offset=0,
                 hidden_rng=None, slope_layout="auto", observation="grid", pinecones=False, tile_skip=False):
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
        self._pos_bull = pos_bull
        self._pos_fire = pos_fire
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
        if slope_layout == "packed":  # the packed step updates ages in place: both "buffers" are one (stride 0)
            self.age = torch.zeros((E, H, W), dtype=torch.int16, **kw).unsqueeze(0).expand(2, E, H, W)
        # edge: (E, 4, H, W) edge values for gca_alex_step_es (packed: the same in coalesced order);
        # planes: (E, 8, H, W) p_slope for gca_alex_step
        self.slope_data = torch.zeros((E, 8 if slope_layout == "planes" else 4, H, W), dtype=torch.float32, **kw)
        # packed layout extras: vd = min(veg, 7) | min(den, 7) << 4 and the dousing bits (u16 per 16 columns)
        self.vd = torch.zeros((E, H, W), dtype=torch.uint8, **kw) if slope_layout == "packed" else None
        self.dous_bits = torch.zeros((E, H * W // 16), dtype=torch.int16, **kw) if slope_layout == "packed" else None
        # tile activity map of the packed step (16 x 256 tiles; ping-pong with the grid): tiles whose 3 x 3 tile
        # neighbourhood holds no fire are copied instead of stepped (exact: p_tree = 0 here); all ones = unknown.
        # Opt-in: it makes a sparse state's step ~20% faster and a dense one ~3% slower
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
        self._initial = None
        if observation not in ("grid", "rgb"):
            raise ValueError("observation must be 'grid' or 'rgb'")
        self.observation = observation
        self.enable_extensions = bool(enable_extensions)
        # MDP(should_transform_grid = transform_grid and enable_extensions, ...) (advanced_bulldozer.py:293-302)
        self.obs_params = make_obs_params(self._empty, self._tree, self._fire, self.enable_extensions,
                                          self.enable_extensions, self._day_length)
        self.rgb = torch.zeros((E, H, W, 3), dtype=torch.float32, **kw) if observation == "rgb" else None
        self._build_context_layers(hidden_rng)

    # ------------------------------------------------------------------ init
    def _build_context_layers(self, rng):
        """density / vegetation / altitude -> slope, once per env instance like the reference's
        constructor (advanced_bulldozer.py:182-204). With use_hidden the layers come from the
        init_utils restatement, which consumes `rng` (default: the global np.random state, as the
        reference does) draw for draw; altitude's arithmetic and get_slope run on the device."""
        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        self.altitude = None
        if self.use_hidden:
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
        """Switch the packed step's tile activity map on / off (the map restarts as "every tile active")."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        if on and self.slope_layout != "packed":
            raise ValueError("tile skipping needs the packed layout (W % 256 == 0, H % 16 == 0)")
        self.act = (torch.ones((2, E, (H // 16) * (W // 256)), dtype=torch.uint8, device=self.device) if on
                    else None)

    def _pack_layers(self):
        """vd and dousing bits of the packed layout from the u8 layers (no-op for the other layouts)."""
        if self.vd is None:
            return
        E, H, W = self.num_envs, self.nrows, self.ncols
        call("gca_alex_pack_layers", dev.ptr(self.vegetation), dev.ptr(self.density), dev.ptr(self.dousing),
             dev.ptr(self.vd), dev.ptr(self.dous_bits), E, H, W, dev.stream_ptr(self.device))

    def _slopes_from(self, altitude):
        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        if self.slope_layout == "edge":
            call("gca_alex_edge_slope_from_altitude", dev.ptr(altitude), dev.ptr(self.slope_data), E, H, W, st)
        elif self.slope_layout == "packed":
            import torch

            tmp = torch.empty_like(self.slope_data)
            call("gca_alex_edge_slope_from_altitude", dev.ptr(altitude), dev.ptr(tmp), E, H, W, st)
            call("gca_alex_edge_slope_coalesce", dev.ptr(tmp), dev.ptr(self.slope_data), E, H, W, st)
            del tmp
        else:
            call("gca_alex_slope_from_altitude", dev.ptr(altitude), dev.ptr(self.slope_data), None, E, H, W, st)

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

    def reset(self, seed=None, options=None):
        """Initial state of advanced_bulldozer.py:650-743 for every env."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        st = dev.stream_ptr(self.device)
        rng = np.random.default_rng(self.key if seed is None else seed)
        # grid iid over {EMPTY, TREE} (p_empty, p_tree), two fires with age (N + N//2) * 2 (:650-688)
        cdf = torch.tensor([self._p_empty_init, self._p_empty_init + self._p_tree_init, 1.0], dtype=torch.float32,
                           device=self.device)
        vals = torch.tensor([self._empty, self._tree, self._fire], dtype=torch.uint8, device=self.device)
        self.cur = 0
        call("gca_fill_categorical", dev.ptr(self.grid[0]), H * W, E, self.env_offset,
             (self.key if seed is None else int(seed)) & (2**64 - 1), dev.ptr(cdf), dev.ptr(vals), 3, st)
        self.age[0].zero_()
        if self._pos_fire is not None:
            r, c = self._pos_fire
        elif self.middle_fire:
            r, c = H // 2, W // 2
        else:
            r, c = 3 * H // 4, W // 4
        age0 = (H + H // 2) * 2
        for cc in (c, c - 1):
            self.grid[0][:, r, cc] = self._fire
            self.age[0][:, r, cc] = age0
        br, bc = (int(H * 0.15), int(W * 0.85)) if self._pos_bull is None else self._pos_bull
        self.pos[:, 0], self.pos[:, 1] = br, bc
        wi = rng.integers(0, 8, size=E) if self.use_hidden else np.zeros(E)
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
        self.steps_elapsed.zero_()
        self.reward_accumulated.zero_()
        call("gca_count_cells", dev.ptr(self.grid[0]), E, H, W, self._empty, self._tree, self._fire,
             dev.ptr(self.counts), st)
        self._initial = dict(grid=self.grid[0].clone(), age=self.age[0].clone(), pos=self.pos.clone(),
                             wind_index=self.wind_index.clone(), counts=self.counts.clone())
        if self.rgb is not None:  # the reference's reset observation (advanced_bulldozer.py:405-409)
            call("gca_adv_observation", self.obs_params, 1, E, H, W, dev.ptr(self.grid[0]), dev.ptr(self.dousing),
                 dev.ptr(self.pos), dev.ptr(self.is_night), None, None, 0, dev.ptr(self.rgb), None, st)
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
            put(self.wind_index, wind_index, torch.int32)
        if dousing is not None:
            put(self.dousing, dousing, torch.uint8)
            if self.dous_bits is not None and bool((self.dousing > 1).any()):
                raise ValueError("the packed layout stores dousing counts as bits: values must be 0/1 "
                                 "(use slope_layout='edge' for other counts)")
        if position is not None:
            put(self.pos, position, torch.int32)
        if altitude is not None:
            alt = altitude if dev.is_device_tensor(altitude) else torch.as_tensor(np.asarray(altitude, np.float64),
                                                                                 device=self.device)
            self.altitude = alt.to(self.device, torch.float64).contiguous()
            self._slopes_from(self.altitude)
        if vegetation is not None or density is not None or dousing is not None:
            self._pack_layers()
        if self.act is not None:  # the state may have fire anywhere now
            self.act.fill_(1)
        call("gca_count_cells", dev.ptr(self.grid[self.cur]), E, H, W, self._empty, self._tree, self._fire,
             dev.ptr(self.counts), st)

    # ------------------------------------------------------------------ step
    def _obs(self):
        ctx = {"per_env_context": {"wind_index": self.wind_index, "fire_age": self.age[self.cur],
                                   "dousing_count": self.dousing, "vegetation": self.vegetation,
                                   "density": self.density, "time_step": self.time_step, "is_night": self.is_night,
                                   "true_grid": self.grid[self.cur], "rng_step": self.rng_step},
               "position": self.pos, "time": self.accu}
        return (self.rgb if self.rgb is not None else self.grid[self.cur]), ctx

    def render_observation(self, action=None, channels=None):
        """The step observation (gca_adv_observation mode 0) of the current state into self.rgb; `action`
        (E, >= 3) int32 device tensor carries the extension choice; `channels` (E, H, W, 5) u8 receives the
        channel stack. Uses the post-step is_night / time_step to recover the pre-step day/night."""
        E, H, W = self.num_envs, self.nrows, self.ncols
        a = action if (action is not None and action.shape[-1] >= 3) else None
        call("gca_adv_observation", self.obs_params, 0, E, H, W, dev.ptr(self.grid[self.cur]), dev.ptr(self.dousing),
             dev.ptr(self.pos), dev.ptr(self.is_night), dev.ptr(self.time_step), dev.ptr(a),
             0 if a is None else int(a.shape[-1]), dev.ptr(self.rgb), dev.ptr(channels), dev.stream_ptr(self.device))
        return self.rgb

    def _info(self):
        return {"reward": self.reward, "terminated": self.done.bool(), "steps_elapsed": self.steps_elapsed,
                "reward_accumulated": self.reward_accumulated}

    def ca_step(self):
        """The CA step alone (RepeatCAJax's one step) for every env; swaps the ping-pong buffers."""
        E, H, W = self.num_envs, self.nrows, self.ncols
        a, b = self.cur, 1 - self.cur
        if self.slope_layout == "packed":
            call("gca_alex_step_packed", self.alex_params, E, H, W, dev.ptr(self.grid[a]), dev.ptr(self.grid[b]),
                 dev.ptr(self.age[a]), dev.ptr(self.age[b]), dev.ptr(self.vd), dev.ptr(self.dous_bits),
                 dev.ptr(self.slope_data), dev.ptr(self.wind_index), dev.ptr(self.rng_step), dev.ptr(self.counts),
                 dev.ptr(None if self.act is None else self.act[a]), dev.ptr(None if self.act is None else self.act[b]),
                 dev.stream_ptr(self.device))
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

    def step(self, action):
        """action: (E, 2) or (E, 3) ints (move, shoot[, extension]); device tensor or numpy."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        full = action if dev.is_device_tensor(action) else torch.as_tensor(np.asarray(action), device=self.device)
        full = full.to(torch.int32).reshape(E, -1).contiguous()
        a = full[:, :2].contiguous()
        self.ca_step()
        self.post_step(a)
        if self.rgb is not None:
            self.render_observation(full)
        self.steps_elapsed += 1
        self.reward_accumulated += self.reward
        terminated = self.done.bool()
        return self._obs(), self.reward, terminated, torch.zeros_like(terminated), self._info()

    stateless_step = step

    def post_step(self, action2):
        """gca_advenv_post for (E, 2) int32 device actions: wind change, time, Move/Modify, reward, done."""
        E, H, W = self.num_envs, self.nrows, self.ncols
        call("gca_advenv_post", self.env_params, dev.ptr(action2), dev.ptr(self.pos), dev.ptr(self.accu),
             dev.ptr(self.wind_index), dev.ptr(self.time_step), dev.ptr(self.is_night), dev.ptr(self.dousing),
             dev.ptr(self.dous_bits), H, W, dev.ptr(self.counts), dev.ptr(self.rng_step), dev.ptr(self.reward),
             dev.ptr(self.done), E, dev.stream_ptr(self.device))

    def conditional_reset(self):
        """Re-inject the initial state of terminated envs (:422-518); time_step/is_night are kept."""
        import torch

        E, H, W = self.num_envs, self.nrows, self.ncols
        init = self._initial
        done = self.done.clone()
        mask = done.bool()
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
             dev.ptr(init["pos"]), dev.ptr(self.accu), dev.ptr(self.wind_index), dev.ptr(init["wind_index"]),
             dev.stream_ptr(self.device))
        return self._obs(), self.reward, self.done.bool(), torch.zeros_like(mask), self._info()
