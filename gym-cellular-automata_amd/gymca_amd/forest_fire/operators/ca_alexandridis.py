"""Alexandridis fire spread on the GPU — drop-in for PartiallyObservableForestFireJax
(reference ca_alexandridis_jax.py:47-460).

`PartiallyObservableForestFireJax(grid_size, empty, tree, fire)` builds the same
constants as the reference constructor (:54-160): burn-kernel radius, 5x5 dousing
weights, ring heat weights, fire-age bounds, all rounded to f32 like jnp.array.
`update(grid, action, per_env_context, shared_context)` runs one CA step (+ the
wind change) in libgca_hip.so and returns `(new_grid, per_env_context, shared_context)`.

Random draws: the reference splits a JAX threefry key (:436-451). jax is not available
here, so draws come from Philox4x32-10 keyed by per_env_context["key"] (two uint32
words) with the step counter per_env_context["rng_step"] (added, default 0; the
returned context carries rng_step + 1). `update(..., draws=...)` injects the
reference's own random arrays instead (random_values_burn (N,N,3,3), random_values_grow
(N,N), new_fire_ages (N,N), and the wind-change uniform / randint), which reproduces
_update_grid exactly.
"""
import math

import numpy as np

from ... import _device as dev
from ..._config import TYPE_BOX
from ..._lib import GCA_MAX_RADIUS, AlexParams, call
from ...operator import Operator
from ...spaces import Box

VEG_PROBS = [-999, -0.1, 0.2, 0.5, 0.8, 1.2]  # :170-171
DEN_PROBS = [-999, -0.2, 0.2, 0.5, 0.8, 1.2]  # :173


def layer_weights(R):
    """build_burn_kernel's per-ring weights in Python float64 (:108-130)."""
    total_weight = 0.065
    weights = []
    remaining = total_weight
    for i in range(R):
        cells = (i * 2 + 3) ** 2 - (i * 2 + 1) ** 2
        if i == 0:
            cells += 1
        if i == R - 1:
            weights.append(remaining / cells)
        else:
            weights.append(remaining * 0.60 / cells)
            remaining = remaining * 0.40
    return weights


def alex_constants(grid_size):
    """All constants of the reference constructor, f32-rounded like jnp.array."""
    initial_spread_time = grid_size + (grid_size // 2)
    fire_age_min = initial_spread_time * 1.5
    fire_age_max = initial_spread_time * 1.75
    R = math.ceil(math.log2(grid_size)) - 2
    if R < 1:
        raise ValueError("grid_size must be >= 5: the reference's burn kernel has no layer below that (:131-137)")
    if R > GCA_MAX_RADIUS:
        raise ValueError(f"grid_size must be <= 1024 (burn radius {R} > {GCA_MAX_RADIUS})")
    lw = layer_weights(R)
    ring = np.zeros(R + 2, dtype=np.float32)  # w_k at Chebyshev distance k, w_{R+1} = 0
    ring[0] = np.float32(lw[0])
    for k in range(1, R + 1):
        ring[k] = np.float32(lw[k - 1])
    heat_dw = (ring[:-1] - ring[1:]).astype(np.float32)  # f32 subtraction
    kernel = np.zeros((2 * R + 1, 2 * R + 1), dtype=np.float32)
    for k in range(R, 0, -1):
        kernel[R - k:R + k + 1, R - k:R + k + 1] = ring[k]
    kernel[R, R] = ring[0]
    border = np.float32(0.0007 * fire_age_max * 0.50)
    inner = np.float32(0.006 * fire_age_max * 0.50)
    dousing_weights = np.full((5, 5), border, dtype=np.float32)
    dousing_weights[1:4, 1:4] = inner
    veg1p = (np.float32(1) + np.array(VEG_PROBS, dtype=np.float32)).astype(np.float32)
    den1p = (np.float32(1) + np.array(DEN_PROBS, dtype=np.float32)).astype(np.float32)
    return dict(R=R, ring=ring, heat_dw=heat_dw, burn_kernel=kernel, dous_inner=inner, dous_border=border,
                dousing_weights=dousing_weights, veg1p=veg1p, den1p=den1p, age_lo=int(fire_age_min),
                age_hi=int(fire_age_max), fire_age_min=fire_age_min, fire_age_max=fire_age_max)


def make_alex_params(grid_size, empty, tree, fire, winds, p_tree, seed, env_offset=0):
    c = alex_constants(grid_size)
    p = AlexParams()
    p.R = c["R"]
    for k in range(GCA_MAX_RADIUS + 1):
        p.heat_dw[k] = float(c["heat_dw"][k]) if k <= c["R"] else 0.0
    p.dous_inner, p.dous_border = float(c["dous_inner"]), float(c["dous_border"])
    for i in range(6):
        p.veg1p[i], p.den1p[i] = float(c["veg1p"][i]), float(c["den1p"][i])
    p.p_tree = float(np.float32(p_tree))
    p.age_lo, p.age_hi = c["age_lo"], c["age_hi"]
    p.seed = int(seed) & (2**64 - 1)
    p.env_offset = int(env_offset)
    p.empty, p.tree, p.fire = int(empty), int(tree), int(fire)
    wm = wind_matrices(winds)
    if not 1 <= len(wm) <= 16:
        raise ValueError("1..16 wind matrices supported")
    p.n_winds = len(wm)
    for i, m in enumerate(wm):
        for j in range(9):
            p.winds[i][j] = float(m.reshape(9)[j])
    return p, c


def wind_matrices(winds):
    """shared_context['winds'] is (n, 2, 3, 3) = (wind_matrix, ft) pairs (:428); also accept (n, 3, 3)."""
    if dev.is_device_tensor(winds):
        winds = winds.cpu().numpy()
    w = np.asarray(winds, dtype=np.float32)
    if w.ndim == 4:
        w = w[:, 0]
    return w.reshape(-1, 3, 3)


def key_to_seed(key):
    k = np.asarray(key, dtype=np.uint64).reshape(-1)
    if k.size == 1:
        return int(k[0])
    return int(k[0]) | (int(k[1]) << 32)


class PartiallyObservableForestFireJax(Operator):
    grid_dependant = True
    action_dependant = False
    context_dependant = True

    deterministic = False

    def __init__(self, grid_size, empty, tree, fire, *args, pinecones=False, env_offset=0, key_is_step=False,
                 **kwargs):
        super().__init__(*args, **kwargs)
        self.grid_size = grid_size
        # env_offset: global id of env 0 of a stack (Philox counters carry it, like the batched env's shards);
        # key_is_step: per_env_context["key"] holds the per-env Philox step counter (the Advanced env's context
        # layout, where the operator's own philox_seed is the env's key) instead of a Philox seed
        self.env_offset = int(env_offset)
        self.key_is_step = bool(key_is_step)
        # pinecone spotting (:229-319, :400-420): commented out in the reference; gca_alex_pinecones here
        self.pinecones = bool(pinecones)
        c = alex_constants(grid_size)
        self.initial_spread_time = grid_size + (grid_size // 2)
        self.fire_age_min = c["fire_age_min"]
        self.fire_age_max = c["fire_age_max"]
        self.burn_kernel_radius = c["R"]
        self.dousing_weights = c["dousing_weights"]
        self.burn_kernel = c["burn_kernel"][None, None, ...]
        self.empty, self.tree, self.fire = empty, tree, fire
        dev.check_u8_codes((empty, tree, fire))
        if self.context_space is None:
            self.context_space = Box(0.0, 1.0, shape=(2,), dtype=TYPE_BOX)

    def update(self, grid, action, per_env_context, shared_context, *, draws=None, return_probs=False):
        """One step for one env (grid (H, W)) or a stack (E, H, W) sharing shared_context."""
        import torch

        device = dev.require_device()
        g = np.asarray(grid) if not dev.is_device_tensor(grid) else grid
        shape = tuple(g.shape)
        E = 1 if len(shape) == 2 else shape[0]
        H, W = shape[-2:]
        ctx = per_env_context

        def d(x, dtype, shp):
            if dev.is_device_tensor(x):
                return x.to(device=device, dtype=dtype).reshape(shp).contiguous()
            return dev.to_device(np.asarray(x).reshape(shp), dtype, device)

        def u8(x, shp):
            a = x if dev.is_device_tensor(x) else np.clip(np.rint(np.asarray(x)), 0, 255)
            return d(a, torch.uint8, shp)

        grid_in = u8(g, (E, H, W))
        age = np.asarray(ctx["fire_age"]) if not dev.is_device_tensor(ctx["fire_age"]) else ctx["fire_age"]
        if not dev.is_device_tensor(age) and (np.any(np.abs(age) > 32767) or np.any(np.rint(age) != age)):
            raise ValueError("fire_age must hold integers in the int16 range (the reference's ages are integer-valued)")
        age_in = d(age, torch.int16, (E, H, W))
        veg = u8(ctx["vegetation"], (E, H, W))
        den = u8(ctx["density"], (E, H, W))
        dous = u8(ctx.get("dousing_count", np.zeros((E, H, W))), (E, H, W))
        slope = d(ctx["slope"], torch.float32, (E, H, W, 9))
        p_slope = torch.empty((E, 8, H, W), dtype=torch.float32, device=device)
        wi_src = ctx["wind_index"]
        widx = d(wi_src if dev.is_device_tensor(wi_src) else np.asarray(wi_src).reshape(E), torch.int32, (E,))
        if self.key_is_step:
            k = ctx["key"]
            rng_step = (k.to(device=device, dtype=torch.int32).reshape(E).contiguous() if dev.is_device_tensor(k)
                        else d(np.asarray(k, dtype=np.int64).reshape(-1).astype(np.uint32).view(np.int32)
                               * np.ones(E, dtype=np.int32), torch.int32, (E,)))
            seed = self.philox_seed
        else:
            rng_step = d(np.asarray(ctx.get("rng_step", 0), dtype=np.int64).reshape(-1).astype(np.uint32)
                         .view(np.int32) * np.ones(E, dtype=np.int32), torch.int32, (E,))
            seed = key_to_seed(ctx.get("key", self.philox_seed))
        p, _ = make_alex_params(self.grid_size, self.empty, self.tree, self.fire, shared_context["winds"],
                                shared_context.get("p_tree", 0.0), seed, self.env_offset)
        st = dev.stream_ptr(device)
        call("gca_alex_prepare_slope", dev.ptr(slope), dev.ptr(p_slope), E, H, W, st)
        grid_out = torch.empty_like(grid_in)
        age_out = torch.empty_like(age_in)
        inj = [None, None, None]
        wu = wk = None
        if draws is not None:
            inj = [d(draws["burn"], torch.float32, (E, H, W, 9)), d(draws["grow"], torch.float32, (E, H, W)),
                   d(draws["age"], torch.int32, (E, H, W))]
            if "wind_u" in draws:
                wu = d(np.asarray(draws["wind_u"], dtype=np.float32).reshape(E), torch.float32, (E,))
                wk = d(np.asarray(draws["wind_k"], dtype=np.int32).reshape(E), torch.int32, (E,))
        probs = torch.empty((E, H, W, 8), dtype=torch.float32, device=device) if return_probs else None
        call("gca_alex_step", p, E, H, W, dev.ptr(grid_in), dev.ptr(grid_out), dev.ptr(age_in), dev.ptr(age_out),
             dev.ptr(veg), dev.ptr(den), dev.ptr(dous), dev.ptr(p_slope), dev.ptr(widx), dev.ptr(rng_step),
             dev.ptr(inj[0]), dev.ptr(inj[1]), dev.ptr(inj[2]), dev.ptr(probs), None, st)
        if self.pinecones:  # on the step's output, with the wind of the step (before its change)
            from .pinecones import make_pine_params, s_cdf_tables

            pp = make_pine_params(seed, self.empty, self.tree, self.fire, self.env_offset)
            tabs = torch.as_tensor(s_cdf_tables(shared_context["winds"]).view(np.int32), device=device)
            call("gca_alex_pinecones", pp, E, H, W, dev.ptr(grid_in), dev.ptr(grid_out), dev.ptr(age_out),
                 dev.ptr(veg), dev.ptr(den), dev.ptr(widx), dev.ptr(tabs), dev.ptr(rng_step), None, None, st)
        new_widx = widx.clone()
        call("gca_alex_wind_change", float(np.float32(shared_context.get("p_wind_change", 0.06))), p.n_winds,
             p.seed, self.env_offset, dev.ptr(rng_step), dev.ptr(wu), dev.ptr(wk), dev.ptr(new_widx), E, st)

        out_ctx = dict(ctx)
        if dev.is_device_tensor(grid):
            new_grid = grid_out.reshape(shape)
            out_ctx["fire_age"] = age_out.reshape(shape)
            out_ctx["wind_index"] = new_widx.reshape(tuple(wi_src.shape)) if dev.is_device_tensor(wi_src) else \
                (new_widx if E > 1 else new_widx[0])
        else:
            new_grid = grid_out.cpu().numpy().reshape(shape).astype(np.asarray(grid).dtype)
            out_ctx["fire_age"] = age_out.cpu().numpy().reshape(shape).astype(np.float32)
            wi = new_widx.cpu().numpy()
            out_ctx["wind_index"] = wi.reshape(np.shape(wi_src)) if np.ndim(wi_src) else np.int32(wi[0])
        if self.key_is_step:  # the step counter advances like the env's (gca_advenv_post: rng_step += 1)
            k = ctx["key"]
            out_ctx["key"] = k + 1 if dev.is_device_tensor(k) else np.asarray(k) + 1
        else:
            out_ctx["rng_step"] = int(np.asarray(ctx.get("rng_step", 0)).reshape(-1)[0]) + 1
        if return_probs:
            return new_grid, out_ctx, shared_context, probs.cpu().numpy().reshape(shape + (8,))
        return new_grid, out_ctx, shared_context


# ---------------------------------------------------------------------------- classic variant
# PartiallyObservableForestFire (reference ca_alexandridis.py:18-221, the NumPy per-cell operator):
# p_burn = p_h (1 + p_veg[veg]) (1 + p_den[den]) wind[i,j] exp(0.078 slope[r,c,i,j]) with the constant
# p_h = 0.58 (:92-99), no heat kernel and no dousing; TREE with a FIRE neighbour burns iff any burning
# neighbour's draw is below p_burn (:104-111), new fire age randint[4, 11) (:111); EMPTY -> TREE w.p.
# p_tree (:171-177); FIRE: age -= 1 and EMPTY when it reaches 0 (:179-183); then the wind change
# (:212-220). Pinecone spotting (:184-210) with the reference loop's skip list runs after the step as
# gca_alex_pinecones_classic (pinecones=True, the default: the reference's update always spots; its own
# path cannot run — it draws through `jax.numpy.random`, which does not exist).
CLASSIC_VEG = {1: -0.3, 2: 0.0, 3: 0.3, 4: 0.6, 5: 1.0}  # :92
CLASSIC_DEN = {1: -0.4, 2: 0.0, 3: 0.3, 4: 0.6, 5: 1.0}  # :93
CLASSIC_P_H = 0.58  # :94
CLASSIC_AGE = (4, 11)  # :111, :131


def make_classic_params(empty, tree, fire, winds, p_tree, seed, env_offset=0):
    """gca_alex_params for the classic rule: heat0 = p_h, all heat / dousing weights 0, classic tables,
    ages [4, 11), burn-out when the decremented age reaches 0."""
    p = AlexParams()
    p.R = 1
    p.heat0 = float(np.float32(CLASSIC_P_H))
    p.burnout_eq1 = 1
    veg = [1.0 + CLASSIC_VEG[max(1, min(5, i))] for i in range(6)]
    den = [1.0 + CLASSIC_DEN[max(1, min(5, i))] for i in range(6)]
    for i in range(6):
        p.veg1p[i], p.den1p[i] = float(np.float32(veg[i])), float(np.float32(den[i]))
    p.p_tree = float(np.float32(p_tree))
    p.age_lo, p.age_hi = CLASSIC_AGE
    p.seed = int(seed) & (2**64 - 1)
    p.env_offset = int(env_offset)
    p.empty, p.tree, p.fire = int(empty), int(tree), int(fire)
    wm = wind_matrices(winds)
    if not 1 <= len(wm) <= 16:
        raise ValueError("1..16 wind matrices supported")
    p.n_winds = len(wm)
    for i, m in enumerate(wm):
        for j in range(9):
            p.winds[i][j] = float(m.reshape(9)[j])
    return p


class PartiallyObservableForestFire(Operator):
    """Drop-in for the classic operator (reference ca_alexandridis.py:18-221) on the device.

    `update(grid, action, context)` follows the reference contract: context holds winds (n, 2, 3, 3),
    wind_index, density, vegetation, slope (H, W, 3, 3), altitude, p_tree, p_wind_change, fire_age;
    fire_age and wind_index are updated IN the context dict (the reference mutates it, :146-217) and
    `(new_grid, context)` is returned. Draws: Philox keyed by the operator's seed with a per-call step
    counter, or `draws=` with the reference's own arrays (burn (H,W,3,3) uniforms, grow (H,W), age
    (H,W) ints, optional wind_u / wind_k) for an exact replay of the rule. Pinecones (`pinecones=True`)
    always draw from Philox (seed `philox_seed`, env 0, the call's step counter): see
    oracle/alexandridis_classic.decode_pinecone_draws for the reference arrays they correspond to.
    """

    grid_dependant = True
    action_dependant = False
    context_dependant = True

    deterministic = False

    def __init__(self, empty, tree, fire, *args, pinecones=True, **kwargs):
        super().__init__(*args, **kwargs)
        self.empty, self.tree, self.fire = empty, tree, fire
        self.pinecones = bool(pinecones)
        dev.check_u8_codes((empty, tree, fire))
        if self.context_space is None:
            self.context_space = Box(0.0, 1.0, shape=(2,), dtype=TYPE_BOX)
        self._step = 0

    def update(self, grid, action, context, *, draws=None, return_probs=False):
        import torch

        device = dev.require_device()
        g = np.asarray(grid)
        H, W = g.shape
        veg_h, den_h = np.asarray(context["vegetation"]), np.asarray(context["density"])
        for name, arr, table in (("vegetation", veg_h, CLASSIC_VEG), ("density", den_h, CLASSIC_DEN)):
            bad = ~np.isin(arr, list(table))
            if np.any(bad):  # the reference's dict lookup raises KeyError (:92-93)
                raise KeyError(f"{name} value {arr[bad].reshape(-1)[0]!r} outside 1..5")
        age_h = np.asarray(context["fire_age"])
        if np.any(np.abs(age_h) > 32767) or np.any(np.rint(age_h) != age_h):
            raise ValueError("fire_age must hold integers in the int16 range")

        def d(x, dtype, shp):
            return dev.to_device(np.ascontiguousarray(np.asarray(x).reshape(shp)), dtype, device)

        grid_in = d(g.astype(np.uint8), torch.uint8, (1, H, W))
        age_in = d(age_h.astype(np.int16), torch.int16, (1, H, W))
        veg = d(veg_h.astype(np.uint8), torch.uint8, (1, H, W))
        den = d(den_h.astype(np.uint8), torch.uint8, (1, H, W))
        dous = torch.zeros((1, H, W), dtype=torch.uint8, device=device)
        slope = d(np.asarray(context["slope"], dtype=np.float32), torch.float32, (1, H, W, 9))
        p_slope = torch.empty((1, 8, H, W), dtype=torch.float32, device=device)
        widx = d(np.asarray(context["wind_index"]).reshape(1).astype(np.int32), torch.int32, (1,))
        rng_step = torch.full((1,), self._step, dtype=torch.int32, device=device)
        p = make_classic_params(self.empty, self.tree, self.fire, context["winds"], context.get("p_tree", 0.0),
                                self.philox_seed)
        st = dev.stream_ptr(device)
        call("gca_alex_prepare_slope", dev.ptr(slope), dev.ptr(p_slope), 1, H, W, st)
        grid_out, age_out = torch.empty_like(grid_in), torch.empty_like(age_in)
        inj = [None, None, None]
        wu = wk = None
        if draws is not None:
            inj = [d(np.asarray(draws["burn"], np.float32), torch.float32, (1, H, W, 9)),
                   d(np.asarray(draws["grow"], np.float32), torch.float32, (1, H, W)),
                   d(np.asarray(draws["age"], np.int32), torch.int32, (1, H, W))]
            if "wind_u" in draws:
                wu = d(np.asarray(draws["wind_u"], np.float32).reshape(1), torch.float32, (1,))
                wk = d(np.asarray(draws["wind_k"], np.int32).reshape(1), torch.int32, (1,))
        probs = torch.empty((1, H, W, 8), dtype=torch.float32, device=device) if return_probs else None
        call("gca_alex_step", p, 1, H, W, dev.ptr(grid_in), dev.ptr(grid_out), dev.ptr(age_in), dev.ptr(age_out),
             dev.ptr(veg), dev.ptr(den), dev.ptr(dous), dev.ptr(p_slope), dev.ptr(widx), dev.ptr(rng_step),
             dev.ptr(inj[0]), dev.ptr(inj[1]), dev.ptr(inj[2]), dev.ptr(probs), None, st)
        if self.pinecones:  # :184-210, with the wind of the step (ft read at :137, before the change)
            from ..._lib import GCA_PINEC_LDS_MAX_HW
            from .pinecones import classic_thrust_tables, make_classic_pine_params

            pp = make_classic_pine_params(self.philox_seed, self.empty, self.tree, self.fire)
            tabs = torch.as_tensor(classic_thrust_tables(context["winds"]).view(np.int32), device=device)
            scratch = None if H * W <= GCA_PINEC_LDS_MAX_HW else \
                torch.empty(4 * ((H * W + 31) // 32), dtype=torch.int32, device=device)
            call("gca_alex_pinecones_classic", pp, 1, H, W, dev.ptr(grid_in), dev.ptr(grid_out), dev.ptr(age_out),
                 dev.ptr(veg), dev.ptr(den), dev.ptr(widx), dev.ptr(tabs), dev.ptr(rng_step), None, dev.ptr(scratch),
                 st)
        call("gca_alex_wind_change", float(np.float32(context.get("p_wind_change", 0.0))), p.n_winds, p.seed, 0,
             dev.ptr(rng_step), dev.ptr(wu), dev.ptr(wk), dev.ptr(widx), 1, st)
        self._step += 1
        new_grid = grid_out.cpu().numpy().reshape(H, W).astype(g.dtype)
        new_age = age_out.cpu().numpy().reshape(H, W)
        if isinstance(context["fire_age"], np.ndarray) and context["fire_age"].shape == (H, W):
            np.copyto(context["fire_age"], new_age.astype(context["fire_age"].dtype))  # in place, like :181
        else:
            context["fire_age"] = new_age
        context["wind_index"] = type(context["wind_index"])(int(widx.cpu().item())) \
            if np.isscalar(context["wind_index"]) else np.int64(widx.cpu().item())
        if return_probs:
            return new_grid, context, probs.cpu().numpy().reshape(H, W, 8)
        return new_grid, context
