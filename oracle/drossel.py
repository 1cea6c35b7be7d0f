"""Drossel-Schwabl ForestFire restatement (ca_DrosselSchwabl.py:32-66) with an explicit
uniform stream. Test infrastructure only."""
import numpy as np


def choice_threshold(p):
    q = np.asarray([p, 1 - p], dtype=np.float64)
    q = q / np.sum(q)
    cdf = q.cumsum()
    cdf /= cdf[-1]
    return cdf[0]


def ds_step(grid, p_fire, p_tree, rng, empty=0, tree=1, fire=2):
    """One step consuming rng.random() exactly where the reference's np_random.choice does."""
    g = np.asarray(grid)
    H, W = g.shape
    out = g.copy()
    tf, tt = choice_threshold(p_fire), choice_threshold(p_tree)
    for r in range(H):
        for c in range(W):
            x = g[r, c]
            nb = [g[rr, cc] for rr in range(r - 1, r + 2) for cc in range(c - 1, c + 2)
                  if 0 <= rr < H and 0 <= cc < W and (rr, cc) != (r, c)]
            if x == tree and fire in nb:
                out[r, c] = fire
            elif x == tree:
                out[r, c] = fire if rng.random() < tf else x
            elif x == empty:
                out[r, c] = tree if rng.random() < tt else x
            elif x == fire:
                out[r, c] = empty
    return out
