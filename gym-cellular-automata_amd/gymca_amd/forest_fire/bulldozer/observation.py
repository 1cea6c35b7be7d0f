"""RGB observations of the Advanced bulldozer env (gca_adv_observation).

Reference: MDP.build_observation_on_extensions / grid_to_rgb_with_extensions / grid_to_rgb
(advanced_bulldozer.py:988-1101), the extension registry and transforms
(bulldozer/utils/extension_utils.py:89-235), the colour constants (advanced_bulldozer.py:41-60) and
the extension action lookup (_create_full_actions :308-330, create_up_to_k_mappings
init_utils.py:119-143).
"""
import itertools

import numpy as np

from ..._lib import GCA_OBS_MAX_EXT, ObsParams

COLORS_DAY = {"empty": "#DDD1D3", "tree": "#A9C499", "fire": "#E68181", "position": "#000000"}
COLORS_NIGHT = {"empty": "#696969", "tree": "#2F4F4F", "fire": "#8B0000", "position": "#000000"}
TINT_DAY, TINT_NIGHT = (0, 0, 200), (255, 165, 0)
# EXTENSION_REGISTRY (extension_utils.py:205-226): (name, skip_visibility, skip_blur), choose = 1
EXTENSIONS = (("unblur", 0, 1), ("see_invisible_fires", 1, 0))
EXTENSION_CHOOSE = 1


def _rgb(h):
    h = h.lstrip("#")
    return [float(int(h[i:i + 2], 16)) for i in (0, 2, 4)]


def up_to_k_mappings(n, k):
    """id -> binary vector over n extensions, combinations of size 0..k in itertools order
    (create_up_to_k_mappings, init_utils.py:119-143)."""
    rows = []
    for i in range(k + 1):
        for combo in itertools.combinations(range(n), i):
            b = [0] * n
            for j in combo:
                b[j] = 1
            rows.append(b)
    return np.asarray(rows, dtype=np.int32)


EXTENSION_LOOKUP = up_to_k_mappings(len(EXTENSIONS), EXTENSION_CHOOSE)  # [[0,0],[1,0],[0,1]]


def make_obs_params(empty, tree, fire, enable_extensions, should_transform, day_length):
    p = ObsParams()
    p.empty, p.tree, p.fire = int(empty), int(tree), int(fire)
    p.n_ext = len(EXTENSIONS)
    assert p.n_ext <= GCA_OBS_MAX_EXT
    for i, (_, sv, sb) in enumerate(EXTENSIONS):
        p.ext_skip_visibility[i], p.ext_skip_blur[i] = sv, sb
    p.enable_extensions = int(bool(enable_extensions))
    p.should_transform = int(bool(should_transform))
    p.day_length = int(day_length)
    for k, name in enumerate(("empty", "tree", "fire", "position")):
        for j in range(3):
            p.color_day[k][j] = _rgb(COLORS_DAY[name])[j]
            p.color_night[k][j] = _rgb(COLORS_NIGHT[name])[j]
    for j in range(3):
        p.tint_day[j], p.tint_night[j] = float(TINT_DAY[j]), float(TINT_NIGHT[j])
    p.n_choices = len(EXTENSION_LOOKUP)
    for c, row in enumerate(EXTENSION_LOOKUP):
        for i, b in enumerate(row):
            p.ext_lookup[c][i] = int(b)
    return p
