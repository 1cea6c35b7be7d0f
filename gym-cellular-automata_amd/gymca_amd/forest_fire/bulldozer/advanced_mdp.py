"""The Advanced env's per-env MDP operator — drop-in for ``MDP`` of advanced_bulldozer.py:956-1133.

``MDP.update(grid, action, per_env_context, shared_context, position, time)`` is what the reference's
``stateless_step`` vmaps over the envs (:351-368):

1. ``RepeatCAJax`` (repeat_ca_jax.py:34-71): the time of (move, shoot) plus the time of the state onto ``time``
   (fraction kept), and exactly one ``PartiallyObservableForestFireJax`` step — the device kernel gca_alex_step
   plus the wind change (ca_alexandridis_jax.py:426-460);
2. ``MoveModifyJax`` (move_modify_jax.py:148-157): Move, then ``dousing_count[row, col] = 1`` on a shot;
3. ``true_grid`` = the new grid, ``time_step`` += 1 (:1116-1118);
4. the observation (:1120-1122, build_observation_on_extensions :988-1018 -> grid_to_rgb :1035-1101) of the NEW
   grid and position with the INPUT context's dousing and is_night — gca_adv_observation, mode 0;
5. ``is_night`` toggles when ``time_step % day_length == 0`` (:1123-1127).

Returns ``(rgb, grid, extended_grid), (next_per_env_context, position, next_time)`` like the reference. Every
argument may carry a leading env axis (E, ...), which is the vmapped call; ``action`` is the full action of
``_create_full_actions`` (move, shoot, one binary flag per extension, :308-330), or (move, shoot, extension
choice), or (move, shoot).

``AdvancedForestFireBulldozerEnv.MDP`` builds one wired to the env (its Philox key, env offset and timings, the
context "key" = the per-env step counter), so that ``env.MDP.update`` on the env's state in the reference's
context layout reproduces ``env.step`` bit for bit (tests/test_gpu_operators_jax.py).
"""
import numpy as np

from ... import _device as dev
from ..._lib import call
from ...operator import Operator
from .observation import EXTENSION_LOOKUP, make_obs_params


class _Timings:
    """time_per_action of the Advanced env (advanced_bulldozer.py:745-776): f32 movement[move] + shooting[shoot]."""

    def __init__(self, t_move, t_shoot):
        self.t_move = np.asarray(t_move, dtype=np.float32)
        self.t_shoot = np.asarray(t_shoot, dtype=np.float32)
        self._dev = {}

    def __call__(self, action):
        a0, a1 = action[0], action[1]
        if dev.is_device_tensor(a0):
            import torch

            key = a0.device
            if key not in self._dev:
                self._dev[key] = (torch.as_tensor(self.t_move, device=key), torch.as_tensor(self.t_shoot, device=key))
            tm, ts = self._dev[key]
            return tm[a0.long()] + ts[a1.long()]
        return self.t_move[np.asarray(a0, dtype=np.int64)] + self.t_shoot[np.asarray(a1, dtype=np.int64)]


class MDP(Operator):
    grid_dependant = True
    action_dependant = True
    context_dependant = True

    deterministic = False

    def __init__(self, repeat_ca, move_modify, should_transform_grid, enable_extensions, tree, fire, empty, *args,
                 **kwargs):
        super().__init__(*args, **kwargs)
        self.repeat_ca = repeat_ca
        self.move_modify = move_modify
        self.should_transform_grid = should_transform_grid
        self.enable_extensions = enable_extensions
        self.suboperators = self.repeat_ca, self.move_modify
        self.tree, self.fire, self.empty = tree, fire, empty
        self.obs_params = make_obs_params(empty, tree, fire, enable_extensions, should_transform_grid, 0)

    # ------------------------------------------------------------------ observation
    def _choice_ids(self, action):
        """(E, 3) int32 (move, shoot, extension choice id) from the full action."""
        a = action.cpu().numpy() if dev.is_device_tensor(action) else np.asarray(action)
        a = a.reshape(-1, a.shape[-1]).astype(np.int64)
        n_ext = EXTENSION_LOOKUP.shape[1]
        out = np.zeros((a.shape[0], 3), dtype=np.int32)
        out[:, :2] = a[:, :2]
        if a.shape[1] == 2 + n_ext:  # binary flags (_create_full_actions): back to the lookup row's id
            for e, flags in enumerate(a[:, 2:]):
                hit = np.nonzero((EXTENSION_LOOKUP == flags).all(axis=1))[0]
                if hit.size == 0:
                    raise ValueError(f"extension flags {flags.tolist()} are not a row of the extension lookup")
                out[e, 2] = hit[0]
        elif a.shape[1] == 3:
            out[:, 2] = a[:, 2]
        elif a.shape[1] != 2:
            raise ValueError(f"action must have 2, 3 or {2 + n_ext} columns, got {a.shape[1]}")
        return out

    def build_observation_on_extensions(self, grid, position, actions, per_env_context, shared_context):
        """(rgb (E, H, W, 3) f32, channels (E, H, W, 3 + n_ext) u8) through gca_adv_observation (mode 0) with the
        given context's dousing and is_night (the caller passes the PRE-step context, as :1120-1122 does)."""
        import torch

        device = dev.require_device()
        g = dev.to_device(grid if dev.is_device_tensor(grid) else np.rint(np.asarray(grid)), torch.uint8, device)
        H, W = g.shape[-2:]
        g = g.reshape(-1, H, W).contiguous()
        E = g.shape[0]
        dous = dev.to_device(per_env_context["dousing_count"], torch.uint8, device).reshape(E, H, W).contiguous()
        night = dev.to_device(per_env_context["is_night"], torch.int32, device).reshape(E).contiguous()
        pos = dev.to_device(position, torch.int32, device).reshape(E, 2).contiguous()
        act = torch.as_tensor(self._choice_ids(actions), device=device)
        rgb = torch.empty((E, H, W, 3), dtype=torch.float32, device=device)
        n_ext = self.obs_params.n_ext
        channels = torch.empty((E, H, W, 3 + n_ext), dtype=torch.uint8, device=device)
        call("gca_adv_observation", self.obs_params, 0, E, H, W, dev.ptr(g), dev.ptr(dous), dev.ptr(pos),
             dev.ptr(night), None, dev.ptr(act), 3, dev.ptr(rgb), dev.ptr(channels), None, dev.stream_ptr(device))
        return rgb, channels

    # ------------------------------------------------------------------ step
    def update(self, grid, action, per_env_context, shared_context, position, time):
        single = np.ndim(position) == 1 if not dev.is_device_tensor(position) else position.dim() == 1
        basic_action = (action[..., 0], action[..., 1])
        new_grid, (next_pe, next_time) = self.repeat_ca(grid, basic_action, per_env_context, shared_context, time)
        new_grid, position, next_pe = self.move_modify(new_grid, basic_action, position, next_pe)
        next_pe["true_grid"] = new_grid
        next_pe["time_step"] = next_pe["time_step"] + 1
        rgb, channels = self.build_observation_on_extensions(new_grid, position, action, per_env_context,
                                                             shared_context)
        day = shared_context["day_length"]
        ts, night = next_pe["time_step"], next_pe["is_night"]
        if dev.is_device_tensor(ts):
            import torch

            next_pe["is_night"] = torch.where(ts % day == 0, 1 - night, night)
        else:
            next_pe["is_night"] = np.where(np.asarray(ts) % day == 0, 1 - np.asarray(night), night)
        if not dev.is_device_tensor(new_grid):  # host arrays in, host arrays out (the grid's dtype, like jnp)
            dt = np.asarray(new_grid).dtype
            rgb, channels = rgb.cpu().numpy(), channels.cpu().numpy().astype(dt)
        if single:
            rgb, channels = rgb[0], channels[0]
        return (rgb, new_grid, channels), (next_pe, position, next_time)


def make_env_mdp(env):
    """The MDP operator of an AdvancedForestFireBulldozerEnv (advanced_bulldozer.py:270-303), wired to the env:
    its CA draws from the env's Philox stream (key = env.key, env ids from env.env_offset, per-env step counter in
    the context's "key"), the env's f32 timings and extension settings."""
    from ..operators import MoveJax, MoveModifyJax, ModifyJax, PartiallyObservableForestFireJax, RepeatCAJax
    from .bulldozer import ACTION_SETS

    ca = PartiallyObservableForestFireJax(env.nrows, env._empty, env._tree, env._fire, pinecones=env.pinecones,
                                          env_offset=env.env_offset, key_is_step=True)
    ca.philox_seed = env.key & (2**64 - 1)
    ep = env.env_params
    timings = _Timings([ep.t_move[a] for a in range(9)], [ep.t_shoot[0], ep.t_shoot[1]])
    t_any = np.float32(ep.t_any)
    repeater = RepeatCAJax(ca, timings, lambda state: t_any)
    move_modify = MoveModifyJax(MoveJax(ACTION_SETS), ModifyJax({}))
    return MDP(repeater, move_modify, env.enable_extensions, env.enable_extensions, env._tree, env._fire, env._empty)
