"""WindyForestFire restatement (reference ca_windy.py:41-139) + the bulldozer MDP
(bulldozer.py:233-400, repeat_ca.py:32-45, move_modify.py:37-134). Test infrastructure only.

`windy_step` is the reference algorithm itself: scipy.signal.convolve2d with the
3x3 kernel (8 on active directions, `empty` on failed ones, 2048 centre), mode="same",
fill=empty, then the three thresholds. It is also the CPU baseline (`kind: port`).
"""
import numpy as np
from scipy.signal import convolve2d

from .philox import philox4x32_10, seed_key, u01_f64

TAG_WINDY_ROLL = 0x574E4459
IDENTITY, PROPAGATION = 2**11, 2**3


def kernel_from_roll(wind, roll, empty):
    """_get_failed_propagations_mask + _get_kernel (ca_windy.py:53-77)."""
    failed = np.asarray(wind) <= np.asarray(roll)
    k = np.full((3, 3), PROPAGATION, dtype=np.int64)
    k[failed] = empty
    k[1, 1] = IDENTITY
    return k


def windy_step(grid, wind, roll, empty=0, tree=3, fire=25):
    """One CA step of one grid with an explicit 3x3 roll."""
    k = kernel_from_roll(wind, roll, empty)
    s = convolve2d(np.asarray(grid, dtype=np.int64), k, mode="same", boundary="fill", fillvalue=empty)
    keep, prop, cons = IDENTITY * tree, IDENTITY * tree + PROPAGATION * fire, IDENTITY * fire
    out = np.full(s.shape, empty, dtype=np.int64)
    out[(s >= keep) & (s < prop)] = tree
    out[(s >= prop) & (s < cons)] = fire
    out[s >= cons] = empty
    return out


def philox_roll(seed, env_id, step):
    """The 3x3 roll the device draws for (env_id, step): 8 doubles, centre unused (0.5)."""
    ctr = np.array([[j, env_id, step, TAG_WINDY_ROLL] for j in range(4)], dtype=np.uint64)
    x = philox4x32_10(ctr, seed_key(seed))
    u = np.empty(8)
    for j in range(4):
        u[2 * j] = u01_f64(x[j, 0], x[j, 1])
        u[2 * j + 1] = u01_f64(x[j, 2], x[j, 3])
    roll = np.full(9, 0.5)
    roll[[0, 1, 2, 3, 5, 6, 7, 8]] = u
    return roll.reshape(3, 3)


def dir_mask(wind, roll):
    m = 0
    for d, idx in enumerate([0, 1, 2, 3, 5, 6, 7, 8]):
        if roll.reshape(9)[idx] < np.asarray(wind).reshape(9)[idx]:
            m |= 1 << d
    return m


# ---------------------------------------------------------------- bulldozer MDP
UP, DOWN, LEFT, RIGHT = {0, 1, 2}, {6, 7, 8}, {0, 3, 6}, {2, 5, 8}


def move(pos, a, H, W):
    r, c = int(pos[0]), int(pos[1])
    if a in UP and r > 0:
        r -= 1
    if a in DOWN and r < H - 1:
        r += 1
    if a in LEFT and c > 0:
        c -= 1
    if a in RIGHT and c < W - 1:
        c += 1
    return r, c


class BulldozerOracle:
    """E independent ForestFireBulldozer envs, numpy; rolls from Philox (or injected)."""

    def __init__(self, grids, positions, wind, t_move, t_shoot, t_any, seed, env_offset=0, empty=0, tree=3, fire=25):
        self.grids = [np.asarray(g, dtype=np.int64).copy() for g in grids]
        self.pos = [tuple(int(v) for v in p) for p in positions]
        self.wind = np.asarray(wind, dtype=np.float64)
        self.t_move, self.t_shoot, self.t_any = t_move, t_shoot, t_any
        self.seed, self.env_offset = seed, env_offset
        self.E, self.T, self.F = empty, tree, fire
        n = len(self.grids)
        self.accu = np.zeros(n)
        self.rng_step = np.zeros(n, dtype=np.int64)
        self.done = np.zeros(n, dtype=bool)
        self.hit = np.zeros(n, dtype=bool)

    def time(self, a):
        move_t = 0.0 if a[0] == 4 else self.t_move
        shoot_t = self.t_shoot if a[1] else 0.0
        return move_t + shoot_t

    def step(self, actions, rolls=None):
        """rolls: optional list (per env) of lists of 3x3 rolls to inject."""
        rewards = np.zeros(len(self.grids))
        for e, g in enumerate(self.grids):
            if self.done[e]:
                continue
            a = (int(actions[e][0]), int(actions[e][1]))
            x = self.accu[e] + (self.time(a) + self.t_any)
            frac, reps = np.modf(x)
            self.accu[e] = frac
            for k in range(int(reps)):
                roll = rolls[e][k] if rolls is not None else philox_roll(self.seed, self.env_offset + e,
                                                                         self.rng_step[e] + k)
                g = windy_step(g, self.wind, roll, self.E, self.T, self.F)
            self.rng_step[e] += int(reps)
            r, c = move(self.pos[e], a[0], *g.shape)
            self.pos[e] = (r, c)
            self.hit[e] = False
            if a[1] and g[r, c] == self.T:
                g[r, c] = self.E
                self.hit[e] = True
            self.grids[e] = g
            t, f = int(np.sum(g == self.T)), int(np.sum(g == self.F))
            rewards[e] = -(f / (t + f)) if t + f else float("nan")
            self.done[e] = f == 0
        return rewards
