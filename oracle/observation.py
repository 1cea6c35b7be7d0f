"""Observation builders of the Advanced bulldozer env, restated in numpy — test infrastructure only.

Follows the reference literally (array semantics included), so the device kernel (gca_obs.hip) is
checked against the reference's own behaviour, quirks and all:
  apply_blur / apply_visibility / transform_grid / apply_extensions
      reference bulldozer/utils/extension_utils.py:89-196 (f32 blur: grid / 3, edge padding,
      9 products of 1/9 summed in (i, j) order, round half-even of 3x)
  build_observation_on_extensions / grid_to_rgb_with_extensions / grid_to_rgb
      reference advanced_bulldozer.py:988-1101 — `has_extension` is a vmap over axis 0 of the
      channel-last stack (= over ROWS), its argmax then indexes the channel axis (JAX clamps the
      out-of-bounds gather); RGB from the day/night colour table, water tint blended where
      dousing_count == 1, position colour on top
  reset observation: advanced_bulldozer.py:401-411 applies grid_to_rgb_with_extensions to the raw
      (H, W) grid; numpy broadcasting of the same expressions reproduces what JAX computes.
Colours: advanced_bulldozer.py:41-60 (PIL ImageColor of the hex strings).
Pinned (r06) to the reference EXECUTING: tests/golden/observation.npz holds the reference's own builders run as published
under a numpy stand-in for jax (tests/golden/_jax_standin.py); tests/test_observation_golden.py checks this restatement
against it bit for bit.
"""
import numpy as np


def _hex(h):
    h = h.lstrip("#")
    return tuple(int(h[i:i + 2], 16) for i in (0, 2, 4))


DAY = {"empty": _hex("#DDD1D3"), "tree": _hex("#A9C499"), "fire": _hex("#E68181"), "position": _hex("#000000")}
NIGHT = {"empty": _hex("#696969"), "tree": _hex("#2F4F4F"), "fire": _hex("#8B0000"), "position": _hex("#000000")}
TINT_DAY, TINT_NIGHT = (0, 0, 200), (255, 165, 0)
# EXTENSION_REGISTRY: (index, skip_visibility, skip_blur): unblur, see_invisible_fires
EXTENSIONS = ((0, 0, 1), (1, 1, 0))


def apply_visibility(grid, is_night):
    return np.where((grid == 3) & (is_night == 0), 0, grid)


def apply_blur(grid):
    normalized = np.asarray(grid, np.float32) / np.float32(3.0)
    k = np.float32(1.0) / np.float32(9.0)
    H, W = normalized.shape
    padded = np.pad(normalized, ((1, 1), (1, 1)), mode="edge")
    blurred = np.zeros_like(normalized)
    for i in range(3):
        for j in range(3):
            blurred = blurred + k * padded[i:i + H, j:j + W]
    return np.round(blurred * np.float32(3)).astype(np.int32)


def transform_grid(grid, is_night, skip_visibility, skip_blur):
    g = np.asarray(grid, np.float32)
    g = g if skip_blur else apply_blur(g).astype(np.float32)
    g = g if skip_visibility else apply_visibility(g, is_night).astype(np.float32)
    return g


def extension_channels(grid, flags, is_night, enable):
    out = []
    for (idx, skip_vis, skip_blur), flag in zip(EXTENSIONS, flags):
        t = transform_grid(grid, is_night, skip_vis, skip_blur)
        out.append(t if (enable and flag) else np.zeros_like(t))
    return np.stack(out)


def build_channels(grid, flags, is_night, enable, should_transform):
    g = np.asarray(grid, np.float32)
    base = transform_grid(g, is_night, 0, 0) if should_transform else g
    ext = extension_channels(g, flags, is_night, enable)
    return np.stack([base, np.zeros_like(g), np.zeros_like(g), *ext], axis=-1)


def grid_to_rgb(display, is_night, dousing, position, tree=1, fire=2):
    col = NIGHT if is_night else DAY
    rgb = np.broadcast_to(np.array(col["empty"], np.int32), display.shape + (3,))
    rgb = np.where((display == tree)[..., None], np.array(col["tree"], np.int32), rgb)
    rgb = np.where((display == fire)[..., None], np.array(col["fire"], np.int32), rgb)
    strength = np.where(dousing == 1, np.float32(0.75), np.float32(0)).astype(np.float32)
    tint = np.array(TINT_NIGHT if is_night else TINT_DAY, np.int32)
    blend = rgb * (np.float32(1) - strength[..., None]) + tint * strength[..., None]
    rgb = np.where((dousing > 0)[..., None], blend, rgb).astype(np.float32)
    rgb = np.array(np.broadcast_to(rgb, np.broadcast_shapes(rgb.shape, dousing.shape + (1,))), np.float32)
    rgb[position[0], position[1]] = col["position"]
    return rgb


def grid_to_rgb_with_extensions(extended, is_night, dousing, position, tree=1, fire=2):
    base = extended[..., 0]
    exts = extended[..., 3:]
    has = np.array([np.any(x > 0) for x in exts])  # vmap over axis 0
    first = int(np.argmax(has)) if has.size else 0
    first = min(max(first, 0), exts.shape[-1] - 1) if exts.shape[-1] else 0  # clamped gather
    display = exts[..., first] if (has.size and has.any()) else base
    return grid_to_rgb(display, is_night, dousing, position, tree, fire)


def step_observation(grid, position, flags, is_night_pre, dousing_pre, enable, should_transform):
    """(rgb (H, W, 3) f32, channels (H, W, 3 + n_ext)) of one env after a step (MDP.update :1120)."""
    ch = build_channels(grid, flags, is_night_pre, enable, should_transform)
    return grid_to_rgb_with_extensions(ch, is_night_pre, dousing_pre, position), ch


def reset_observation(grid, position, is_night, dousing):
    """The reset observation of one env (grid_to_rgb_with_extensions on the raw grid, :405-409)."""
    return grid_to_rgb_with_extensions(np.asarray(grid, np.float32), is_night, dousing, position)
