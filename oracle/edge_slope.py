"""Edge (antisymmetric) slope layout — test infrastructure only (never imported by the product).

Restates, in numpy float64 like the reference, what gca_alex_edge_slope_from_altitude builds and how
gca_alex_step_es expands it, so the CPU suite can pin the layout against get_slope itself
(reference bulldozer/utils/init_utils.py:166-200, restated in gymca_amd init_utils.get_slope):

    edge[e][k][r][c] = f32(degrees(arctan((alt[r,c] - alt[n]) / (1.414 if diagonal))))
        n = (r,c) + OFF[k], OFF = (-1,-1), (-1,0), (-1,+1), (0,-1); 0 where n is outside the grid
        (no border zeroing: a border cell's slope toward an interior one is still needed by that one)
    (the device stores edge_values(edge) = +-exp_f32(|0.078 s|), see oracle_signed_factors)
    slope9[r,c,(i,j)] = edge[k][r,c]           for (i-1, j-1) = OFF[k]
                      = -edge[k][(r,c)-OFF[k]] for (i-1, j-1) = -OFF[k]
                      = 0 on the grid border and at the centre (get_slope's zero border).
"""
import numpy as np

from . import alex_c

OFF = ((-1, -1), (-1, 0), (-1, 1), (0, -1))


def _shift(a, dr, dc):
    """out[..., r, c] = a[..., r + dr, c + dc], 0 outside."""
    out = np.zeros_like(a)
    H, W = a.shape[-2:]
    rs, re = max(0, -dr), min(H, H - dr)
    cs, ce = max(0, -dc), min(W, W - dc)
    out[..., rs:re, cs:ce] = a[..., rs + dr:re + dr, cs + dc:ce + dc]
    return out


def edge_from_altitude(alt):
    """(E, H, W) float64 altitude -> (E, 4, H, W) float32 edge slopes."""
    alt = np.asarray(alt, dtype=np.float64)
    E, H, W = alt.shape
    out = np.zeros((E, 4, H, W), np.float32)
    for k, (dr, dc) in enumerate(OFF):
        nb = _shift(alt, dr, dc)
        diff = alt - nb
        if dr != 0 and dc != 0:
            diff = diff / 1.414
        s = np.degrees(np.arctan(diff)).astype(np.float32)
        valid = np.zeros((H, W), bool)
        valid[max(0, -dr):H - max(0, dr), max(0, -dc):W - max(0, dc)] = True
        out[:, k] = np.where(valid, s, np.float32(0))
    return out


def slope9_from_edge(edge):
    """(E, 4, H, W) edge slopes -> (E, H, W, 3, 3) float32 slopes as get_slope + f32 cast would give."""
    edge = np.asarray(edge, dtype=np.float32)
    E, _, H, W = edge.shape
    s9 = np.zeros((E, H, W, 3, 3), np.float32)
    for k, (dr, dc) in enumerate(OFF):
        s9[:, :, :, dr + 1, dc + 1] = edge[:, k]
        # the opposite direction of cell X reads the neighbour Y = X - OFF[k], negated
        s9[:, :, :, 1 - dr, 1 - dc] = -_shift(edge[:, k], -dr, -dc)
    s9[:, 0] = 0
    s9[:, -1] = 0
    s9[:, :, 0] = 0
    s9[:, :, -1] = 0
    s9[..., 1, 1] = 0
    return s9


def edge_values(edge_slopes):
    """The device's stored edge values V = +-exp_f32(|0.078 * s|) (sign of s) of (E, 4, H, W) slopes."""
    return alex_c.signed_factors(edge_slopes)
