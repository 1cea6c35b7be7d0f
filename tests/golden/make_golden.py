"""Capture golden input/output vectors from the reference NumPy operators.

RUNS ONLY IN THE BUILD CONTAINER (it reads /root/reference, which never travels).
The reference source is NOT copied: this script imports the reference's own files
in place, drives them on seeded inputs and stores the resulting *data* as small
.npz fixtures next to this script. The committed fixtures are what the tests use.

gymnasium is not installed here, so a minimal restatement of the gymnasium API in
tests/golden/_stub/ is put on sys.path first. Reference modules are loaded file by
file (the package __init__ chain imports JAX, which is absent: SURVEY.md §0.3).

Fixture inventory:
  windy.npz        WindyForestFire.update            ca_windy.py:41-51
  repeat_ca.npz    RepeatCA.update + Windy           repeat_ca.py:32-45
  move_modify.npz  Move/Modify/MoveModify            move_modify.py:37-134
  bulldozer.npz    ForestFireBulldozerEnv episodes   bulldozer.py:21-400, ca_env.py:27-99
                   (with the {"wind": W} unwrap patch)
  drossel.npz      ForestFire (Drossel-Schwabl)      ca_DrosselSchwabl.py:32-66
  helicopter.npz   ForestFireHelicopterEnv 5x5       helicopter.py:20-236
  moore.npz        moore_n                           neighbors.py:6-147
  alexandridis_classic.npz
                   PartiallyObservableForestFire.update   ca_alexandridis.py:35-221, 8-12 consecutive
                   steps per case with pinecone spotting and skip-list events. The module's
                   `import jax.numpy as np` (:1) gets numpy itself (it only calls exp / array /
                   any / sum / np.random there; jax.numpy lacks np.random, :189, which is why the
                   module cannot run as published). Every draw of op.np_random and of the global
                   np.random.standard_normal is recorded in call order and attributed to the cell
                   being visited, then stored as the array-form draws oracle/alexandridis_classic
                   takes (burn, grow, age, wind; pinecone n / dirs / thrust / u / target age).
  init_utils.npz   init_vegetation / init_density / init_altitude / get_slope after
                   np.random.seed(k) (bulldozer/utils/init_utils.py:10-200). Those functions
                   use numpy and the global legacy np.random state only; the module's own
                   `import jax.numpy` / `from flax import struct` lines get empty stand-in
                   modules here (jax and flax are not installed).
  alexandridis_jax.npz
                   PartiallyObservableForestFireJax.update   ca_alexandridis_jax.py:54-460, the headline rule
                   EXECUTED as published under tests/golden/_jax_standin.py (numpy with jax's x64-disabled
                   dtype rules for jnp; jit = identity; vmap = a loop over in_axes; lax.dynamic_slice; random
                   draws logged in call order): 4 cases, 2-4 chained steps, every random array the rule
                   consumed, its burn probabilities and outputs (grid, fire_age, wind_index).
  pinecones_jax.npz
                   _handle_pinecone_spread (ca_alexandridis_jax.py:208-319) executed the same way: 4 cases,
                   the Poisson / direction / thrust / uniform draws and the landings and burn mask.
  observation.npz  MDP.build_observation_on_extensions / grid_to_rgb_with_extensions / grid_to_rgb
                   (advanced_bulldozer.py:988-1101) with extension_utils.py:89-196, executed the same way:
                   36 cases, the step frame, the channel stack and (square grids) the reset frame.
  advanced_env.npz AdvancedForestFireBulldozerEnv (advanced_bulldozer.py) built, reset and stepped through
                   stateless_step (:332-399) the same way: 2 cases (32^2 x 3 envs x 8 steps; 24^2 x 2 envs x 6
                   steps with extensions), the seeded initial state, each step's actions and every env's draws,
                   and the whole step's outputs (grid, ages, wind, dousing, clock, position, frame, reward,
                   terminated, counters).

Usage:  python tests/golden/make_golden.py [fixture ...]   (default: all)
"""
import importlib.util
import os
import sys
import types
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/gym_cellular_automata"

sys.path.insert(0, os.path.join(HERE, "_stub"))
import gymnasium  # noqa: E402  (the stub)
from gymnasium import spaces as stub_spaces  # noqa: E402


def _pkg(name, path):
    m = types.ModuleType(name)
    m.__path__ = [path]
    sys.modules[name] = m
    return m


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    root = _pkg("gym_cellular_automata", REF)
    _pkg("gym_cellular_automata.forest_fire", f"{REF}/forest_fire")
    ops = _pkg("gym_cellular_automata.forest_fire.operators", f"{REF}/forest_fire/operators")
    _pkg("gym_cellular_automata.forest_fire.utils", f"{REF}/forest_fire/utils")
    _pkg("gym_cellular_automata.forest_fire.bulldozer", f"{REF}/forest_fire/bulldozer")
    _pkg("gym_cellular_automata.forest_fire.helicopter", f"{REF}/forest_fire/helicopter")
    for env in ("bulldozer", "helicopter"):
        _pkg(f"gym_cellular_automata.forest_fire.{env}.utils", f"{REF}/forest_fire/{env}/utils")
        r = types.ModuleType(f"gym_cellular_automata.forest_fire.{env}.utils.render")
        r.render = lambda env: None
        sys.modules[r.__name__] = r

    cfg = _load("gym_cellular_automata._config", f"{REF}/_config.py")
    opm = _load("gym_cellular_automata.operator", f"{REF}/operator.py")
    gs = _load("gym_cellular_automata.grid_space", f"{REF}/grid_space.py")
    ce = _load("gym_cellular_automata.ca_env", f"{REF}/ca_env.py")
    root.Operator = opm.Operator
    root.GridSpace = gs.GridSpace
    root.CAEnv = ce.CAEnv
    nb = _load("gym_cellular_automata.forest_fire.utils.neighbors", f"{REF}/forest_fire/utils/neighbors.py")
    windy = _load("gym_cellular_automata.forest_fire.operators.ca_windy", f"{REF}/forest_fire/operators/ca_windy.py")
    mm = _load("gym_cellular_automata.forest_fire.operators.move_modify", f"{REF}/forest_fire/operators/move_modify.py")
    rep = _load("gym_cellular_automata.forest_fire.operators.repeat_ca", f"{REF}/forest_fire/operators/repeat_ca.py")
    ds = _load("gym_cellular_automata.forest_fire.operators.ca_DrosselSchwabl", f"{REF}/forest_fire/operators/ca_DrosselSchwabl.py")
    ops.WindyForestFire = windy.WindyForestFire
    ops.Move, ops.Modify, ops.MoveModify = mm.Move, mm.Modify, mm.MoveModify
    ops.RepeatCA = rep.RepeatCA
    ops.ForestFire = ds.ForestFire
    bd = _load("gym_cellular_automata.forest_fire.bulldozer.bulldozer", f"{REF}/forest_fire/bulldozer/bulldozer.py")
    he = _load("gym_cellular_automata.forest_fire.helicopter.helicopter", f"{REF}/forest_fire/helicopter/helicopter.py")
    return types.SimpleNamespace(cfg=cfg, Operator=opm.Operator, GridSpace=gs.GridSpace, nb=nb,
                                 windy=windy, mm=mm, rep=rep, ds=ds, bd=bd, he=he)


def crc(grid):
    return zlib.crc32(np.ascontiguousarray(grid, dtype=np.uint8).tobytes()) & 0xFFFFFFFF


# ----------------------------------------------------------------------------- windy
WIND_BULLDOZER = np.array([[0.48, 0.64, 0.98], [0.12, 0.0, 0.64], [0.06, 0.12, 0.48]])


def gen_windy(R, rng):
    cases = {}
    shapes = [(16, 16)] * 12 + [(64, 64)] * 8 + [(1, 1), (1, 7), (7, 1), (3, 5), (17, 23), (32, 48), (2, 2), (5, 5),
                                                (16, 16), (16, 16), (31, 33), (64, 16)]
    values = [(0, 3, 25)] * 26 + [(2, 4, 40), (5, 9, 80), (2, 4, 40), (5, 9, 80), (0, 3, 25), (5, 9, 80)]
    kinds = ["ones", "zeros", "bulldozer", "random"]
    for i, (shape, (E, T, F)) in enumerate(zip(shapes, values)):
        op = R.windy.WindyForestFire(E, T, F)
        p = [[0.1, 0.9, 0.0], [0.1, 0.6, 0.3], [0.3, 0.4, 0.3], [0.0, 0.5, 0.5]][i % 4]
        grid = rng.choice([E, T, F], size=shape, p=p).astype(np.int64)
        if i % 4 == 0 and grid.size > 4:  # single fire seed like the bulldozer env
            grid[grid == F] = T
            grid[shape[0] * 3 // 4, shape[1] // 4] = F
        kind = kinds[i % 4]
        wind = {"ones": np.ones((3, 3)), "zeros": np.zeros((3, 3)), "bulldozer": WIND_BULLDOZER,
                "random": rng.random((3, 3))}[kind]
        stub_spaces.RECORDER.clear()
        out, w_out = op.update(grid.copy(), None, wind)
        roll = stub_spaces.RECORDER[-1]
        assert len(stub_spaces.RECORDER) == 1
        cases[f"c{i}_grid"] = grid.astype(np.uint8)
        cases[f"c{i}_wind"] = wind.astype(np.float64)
        cases[f"c{i}_roll"] = roll.astype(np.float64)
        cases[f"c{i}_out"] = np.asarray(out).astype(np.uint8)
        cases[f"c{i}_values"] = np.array([E, T, F], dtype=np.int64)
    cases["n"] = np.array(len(shapes))
    return cases


def gen_repeat(R, rng):
    cases = {}
    times = [(0.3, 0.0), (1.0, 1.0), (2.0, 0.0), (2.7, 0.0), (0.65, 0.001), (0.031552, 0.001), (0.098656, 0.001), (3.5, 0.25)]
    for i, (ta, tp) in enumerate(times):
        E, T, F = 0, 3, 25
        gspace = R.GridSpace(values=[E, T, F], shape=(12, 10))
        ca = R.windy.WindyForestFire(E, T, F, grid_space=gspace, action_space=stub_spaces.Discrete(1))
        ctx_space = stub_spaces.Tuple((ca.context_space, stub_spaces.Box(np.array(0.0), np.array(1.0), dtype=np.float64)))
        rep = R.rep.RepeatCA(ca, lambda a, ta=ta: ta, lambda s, tp=tp: tp, grid_space=gspace,
                             action_space=stub_spaces.Discrete(1), context_space=ctx_space)
        grid = rng.choice([E, T, F], size=(12, 10), p=[0.1, 0.7, 0.2]).astype(np.int64)
        wind = [np.ones((3, 3)), WIND_BULLDOZER, rng.random((3, 3)), WIND_BULLDOZER][i % 4]
        accu = 0.0
        seq_grids, seq_accu, rolls, nrolls = [], [], [], []
        g = grid.copy()
        for s in range(8):
            stub_spaces.RECORDER.clear()
            g, (w, accu) = rep.update(g, None, (wind, accu))
            accu = float(accu)
            seq_grids.append(np.asarray(g).astype(np.uint8))
            seq_accu.append(accu)
            nrolls.append(len(stub_spaces.RECORDER))
            rolls.extend(stub_spaces.RECORDER)
        cases[f"c{i}_grid"] = grid.astype(np.uint8)
        cases[f"c{i}_wind"] = wind
        cases[f"c{i}_times"] = np.array([ta, tp])
        cases[f"c{i}_grids"] = np.stack(seq_grids)
        cases[f"c{i}_accu"] = np.array(seq_accu)
        cases[f"c{i}_nrolls"] = np.array(nrolls)
        cases[f"c{i}_rolls"] = np.stack(rolls) if rolls else np.zeros((0, 3, 3))
    cases["n"] = np.array(len(times))
    return cases


def gen_move_modify(R, rng):
    sets = {"up": {0, 1, 2}, "down": {6, 7, 8}, "left": {0, 3, 6}, "right": {2, 5, 8}, "not_move": {4}}
    move = R.mm.Move(sets)
    modify = R.mm.Modify({3: 0})
    mm = R.mm.MoveModify(move, modify)
    rows = []
    for (H, W) in [(5, 5), (1, 1), (1, 5), (5, 1), (3, 3), (2, 7)]:
        grid = rng.choice([0, 3, 25], size=(H, W)).astype(np.int64)
        for r in range(H):
            for c in range(W):
                for a in range(9):
                    for shoot in (0, 1):
                        g = grid.copy()
                        g2, pos = mm.update(g, (a, shoot), np.array([r, c]))
                        rows.append((H, W, r, c, a, shoot, int(pos[0]), int(pos[1]), int(grid[pos[0], pos[1]]),
                                     int(g2[pos[0], pos[1]]), int(mm.modify.hit)))
    return {"rows": np.array(rows, dtype=np.int64)}


def gen_bulldozer(R, rng):
    orig = R.windy.WindyForestFire.update

    def patched(self, grid, action, wind):  # unwrap ctx["wind"] (upstream fix)
        if isinstance(wind, dict):
            g, _ = orig(self, grid, action, wind["wind"])
            return g, wind
        return orig(self, grid, action, wind)

    R.windy.WindyForestFire.update = patched
    out = {}
    try:
        for i, (N, steps) in enumerate([(32, 160), (48, 120), (256, 64)]):
            env = R.bd.ForestFireBulldozerEnv(N, N)
            obs, info = env.reset(seed=100 + i)
            grid0 = np.asarray(obs[0]).copy()
            ctx = obs[1]
            actions = np.stack([rng.integers(0, 9, steps), rng.integers(0, 2, steps)], axis=1)
            recs, rolls, nrolls, grids, crcs = [], [], [], [], []
            for s in range(steps):
                stub_spaces.RECORDER.clear()
                obs, rew, term, trunc, info = env.step(actions[s])
                g = np.asarray(obs[0])
                _, pos, t = obs[1]
                counts = env.count_cells(g)
                recs.append((float(rew), float(term), float(info["hit"]), float(pos[0]), float(pos[1]), float(t),
                             counts[0], counts[3], counts[25]))
                nrolls.append(len(stub_spaces.RECORDER))
                rolls.extend(stub_spaces.RECORDER)
                crcs.append(crc(g))
                if N <= 48:
                    grids.append(g.astype(np.uint8))
            out[f"c{i}_N"] = np.array(N)
            out[f"c{i}_grid0"] = grid0.astype(np.uint8)
            out[f"c{i}_pos0"] = np.asarray(ctx[1]).astype(np.int64)
            out[f"c{i}_wind"] = np.asarray(ctx[0]["wind"])
            out[f"c{i}_times"] = np.array([env._t_act_move, env._t_act_shoot, env._t_env_any])
            out[f"c{i}_actions"] = actions
            out[f"c{i}_recs"] = np.array(recs)
            out[f"c{i}_nrolls"] = np.array(nrolls)
            out[f"c{i}_rolls"] = np.stack(rolls) if rolls else np.zeros((0, 3, 3))
            out[f"c{i}_crc"] = np.array(crcs, dtype=np.uint64)
            out[f"c{i}_final"] = np.asarray(obs[0]).astype(np.uint8)
            if grids:
                out[f"c{i}_grids"] = np.stack(grids)
        out["n"] = np.array(3)
        out["meta_patch"] = np.array("ca_windy.update unwraps ctx['wind'] (SURVEY.md 0.4)")
    finally:
        R.windy.WindyForestFire.update = orig
    return out


def gen_drossel(R, rng):
    out = {}
    cases = [(8, 8, 0.033, 0.333), (5, 5, 0.033, 0.333), (8, 8, 0.5, 0.5), (6, 9, 0.0, 1.0), (7, 7, 1.0, 0.0)]
    for i, (H, W, pf, pt) in enumerate(cases):
        op = R.ds.ForestFire(0, 1, 2)
        seed = 1000 + i
        op.seed(seed)
        grid = rng.choice([0, 1, 2], size=(H, W), p=[0.3, 0.5, 0.2]).astype(np.int64)
        new, _ = op.update(grid.copy(), None, np.array([pf, pt]))
        out[f"c{i}_grid"] = grid.astype(np.uint8)
        out[f"c{i}_out"] = np.asarray(new).astype(np.uint8)
        out[f"c{i}_p"] = np.array([pf, pt])
        out[f"c{i}_seed"] = np.array(seed)
    out["n"] = np.array(len(cases))
    return out


def gen_helicopter(R, rng):
    env = R.he.ForestFireHelicopterEnv(5, 5)
    obs, info = env.reset(seed=7)
    env.cellular_automaton.seed(2024)
    grid0 = np.asarray(obs[0]).copy()
    steps = 48
    grids, recs = [], []
    for s in range(steps):
        obs, rew, term, trunc, info = env.step(s % 9)
        _, pos, freeze = obs[1]
        grids.append(np.asarray(obs[0]).astype(np.uint8))
        recs.append((float(rew), float(pos[0]), float(pos[1]), float(freeze), float(info["hit"])))
    return {"grid0": grid0.astype(np.uint8), "grids": np.stack(grids), "recs": np.array(recs),
            "seed": np.array(2024), "max_freeze": np.array(env._max_freeze)}


def gen_moore(R, rng):
    out = {}
    i = 0
    for (H, W) in [(4, 4), (5, 7), (1, 1), (3, 9)]:
        grid = rng.integers(0, 5, size=(H, W))
        for n in (1, 2, 3):
            for r in range(H):
                for c in range(W):
                    out[f"c{i}"] = np.concatenate([[H, W, n, r, c], grid.ravel(), R.nb.moore_n(n, (r, c), grid, 9).ravel()])
                    i += 1
    out["n"] = np.array(i)
    return out


def gen_init_utils(R, rng):
    """Hidden layers of the Advanced env from the reference's own init functions, seeded globally."""
    import contextlib
    import io

    jax = types.ModuleType("jax")
    jax.numpy = np
    flax = types.ModuleType("flax")
    flax.struct = types.SimpleNamespace(dataclass=lambda c: c)
    saved = {k: sys.modules.get(k) for k in ("jax", "jax.numpy", "flax")}
    sys.modules.update({"jax": jax, "jax.numpy": np, "flax": flax})
    try:
        iu = _load("gym_cellular_automata.forest_fire.bulldozer.utils.init_utils",
                   f"{REF}/forest_fire/bulldozer/utils/init_utils.py")
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    out = {}
    for k, (H, W, E) in enumerate([(32, 32, 3), (24, 40, 2), (64, 64, 2)]):
        np.random.seed(1000 + k)
        out[f"veg_{k}"] = iu.init_vegetation(H, W, E)
        out[f"den_{k}"] = iu.init_density(H, W, E)
        out[f"alt_{k}"] = iu.init_altitude(H, W, E)
        with contextlib.redirect_stdout(io.StringIO()):  # get_slope prints a histogram
            out[f"slope_{k}"] = iu.get_slope(out[f"alt_{k}"], H, W, E)
        out[f"shape_{k}"] = np.array([H, W, E])
        out[f"next_{k}"] = np.random.randint(0, 2**31 - 1, size=4)  # stream position after the four calls
    out["n"] = np.array(3)
    return out


def _classic_context(rng, H, W, n_winds=8, fire_frac=0.2):
    """Inputs of one classic case (the reference's context keys, ca_alexandridis.py:137-146)."""
    import math

    grid = rng.choice(np.array([0, 1, 2]), size=(H, W), p=[0.15, 0.85 - fire_frac, fire_frac])
    winds = np.zeros((n_winds, 2, 3, 3))
    for k in range(n_winds):  # calc_pw's (e^0.45 ft, ft) pairs (init_utils.py:225-244), 8 directions
        th = k * 2 * math.pi / n_winds
        for i in range(3):
            for j in range(3):
                if (i, j) != (1, 1):
                    ft = math.exp(1.31 * (math.cos(math.atan2(1 - i, j - 1) - th) - 1))
                    winds[k, :, i, j] = (math.exp(0.45) * ft, ft)
    return {"winds": winds.astype(np.float32), "wind_index": int(rng.integers(0, n_winds)),
            "density": rng.integers(1, 6, (H, W)), "vegetation": rng.integers(1, 6, (H, W)),
            "slope": rng.uniform(-25, 25, (H, W, 3, 3)).astype(np.float32), "altitude": np.zeros((H, W)),
            "p_tree": 0.1, "p_wind_change": 0.3,
            "fire_age": np.where(grid == 2, rng.integers(1, 7, (H, W)), 0).astype(np.int64)}, grid


class _Recorder:
    """op.np_random stand-in: the seeded Generator's own draws, logged in call order with the visited cell."""

    def __init__(self, gen, log, cur):
        self.gen, self.log, self.cur = gen, log, cur

    def _rec(self, kind, v, extra=None):
        self.log.append((kind, self.cur[0], v, extra))
        return v

    def uniform(self, low=0.0, high=1.0, size=None):
        return self._rec("uniform", self.gen.uniform(low, high, size), size)

    def integers(self, low, high=None, size=None):
        return self._rec("integers", self.gen.integers(low, high, size), (low, high))

    def choice(self, a, size=None, replace=True, p=None):
        return self._rec("choice", self.gen.choice(a, size=size, replace=replace, p=p), float(p[0]))

    def poisson(self, lam=1.0, size=None):
        return self._rec("poisson", self.gen.poisson(lam, size), None)


def gen_alexandridis_classic(R, rng):
    """The classic operator run as published with jax.numpy -> numpy, its draws recorded (see module doc)."""
    import contextlib
    import io

    jax = types.ModuleType("jax")
    jax.numpy = np
    saved = {k: sys.modules.get(k) for k in ("jax", "jax.numpy")}
    sys.modules.update({"jax": jax, "jax.numpy": np})
    try:
        cl = _load("gym_cellular_automata.forest_fire.operators.ca_alexandridis",
                   f"{REF}/forest_fire/operators/ca_alexandridis.py")
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    DX, DY = [1, 1, 0, -1, -1, -1, 0, 1], [0, 1, 1, 1, 0, -1, -1, -1]  # :63-64
    LOOKUP = [(0, 0), (0, 1), (0, 2), (1, 0), (1, 2), (2, 0), (2, 1), (2, 2)]  # :50-59
    M = 16
    out = {}
    cases = [(16, 16, 8), (20, 24, 10), (32, 32, 12), (24, 17, 8)]
    for ci, (H, W, steps) in enumerate(cases):
        ctx, grid = _classic_context(rng, H, W)
        out[f"c{ci}_winds"], out[f"c{ci}_density"] = ctx["winds"], ctx["density"]
        out[f"c{ci}_vegetation"], out[f"c{ci}_slope"] = ctx["vegetation"], ctx["slope"]
        out[f"c{ci}_p"] = np.array([ctx["p_tree"], ctx["p_wind_change"]])
        op = cl.PartiallyObservableForestFire(0, 1, 2)
        log, cur = [], [None]
        op.np_random = _Recorder(np.random.default_rng(777 + ci), log, cur)
        np.random.seed(555 + ci)  # the global legacy stream of :189
        orig_nb, orig_sn = cl.neighborhood_at, np.random.standard_normal
        orig_spf = op._set_fire_pinecone

        def nb(grid_, pos, *a, **k):
            cur[0] = tuple(int(v) for v in pos)
            return orig_nb(grid_, pos, *a, **k)

        def sn(n):
            v = orig_sn(n)
            log.append(("normal", cur[0], v, None))
            return v

        def spf(row, col, *a, **k):
            log.append(("pine_target", cur[0], (int(row), int(col)), None))
            return orig_spf(row, col, *a, **k)

        cl.neighborhood_at, np.random.standard_normal, op._set_fire_pinecone = nb, sn, spf
        try:
            for t in range(steps):
                log.clear()
                g_in, a_in, w_in = grid.copy(), ctx["fire_age"].copy(), int(ctx["wind_index"])
                with contextlib.redirect_stdout(io.StringIO()):  # :220 prints the wind change
                    grid, ctx = op.update(grid, None, ctx)
                ft = ctx["winds"][w_in][1]
                burn, grow = np.ones((H, W, 3, 3)), np.ones((H, W))
                age, pine_age = np.full((H, W), 4), np.full((H, W), 4)
                n, dirs = np.zeros((H, W), np.int64), np.zeros((H, W, M), np.int64)
                thrust, u = np.zeros((H, W, M)), np.ones((H, W, M))
                wind_u, wind_k = 1.0, 1
                pine_hits = np.zeros((H, W), np.uint8)
                valid, k_valid, last = {}, {}, None
                for kind, cell, v, extra in log:
                    if kind == "uniform" and extra == (3, 3):  # _set_fire's burn draws (:104)
                        burn[cell] = v
                        last = ("fire", cell)
                    elif kind == "uniform":  # _set_fire_pinecone's draw (:127) for the source's next valid landing
                        i = valid[cell][k_valid[cell]]
                        k_valid[cell] += 1
                        u[cell + (i,)] = v
                        last = ("pine", target)
                    elif kind == "pine_target":
                        target = v
                    elif kind == "integers" and extra == (4, 11):
                        if last[0] == "fire":
                            age[last[1]] = v
                        else:
                            pine_age[last[1]] = v  # the last ignition of a target sets its age
                            pine_hits[last[1]] = 1
                    elif kind == "integers" and extra == (0, 8):  # pinecone directions (:47)
                        nn = len(v)
                        assert nn <= M
                        dirs[cell + (slice(0, nn),)] = v
                    elif kind == "poisson":
                        n[cell] = v
                        valid[cell], k_valid[cell] = [], 0
                    elif kind == "normal":  # thrust of :189-190 and the landings it gives (:191-200)
                        d = dirs[cell][:n[cell]]
                        gi = np.array([LOOKUP[x] for x in d])
                        th = 3 * v
                        th = th * ft[tuple(zip(*gi))]
                        thrust[cell + (slice(0, len(th)),)] = th
                        r, c = cell
                        for i in range(len(th)):
                            nr, nc = round(r + DX[d[i]] * th[i]), round(c + DY[d[i]] * th[i])
                            if 0 <= nr < H and 0 <= nc < W and (nr, nc) != (r, c):
                                valid[cell].append(i)
                    elif kind == "choice" and extra == ctx["p_tree"]:  # growth (:173-175)
                        grow[cell] = 0.0 if v else 1.0
                    elif kind == "choice":  # wind change (:212-214)
                        wind_u = 0.0 if v else 1.0
                    elif kind == "integers" and extra == (1, 8):
                        wind_k = int(v)
                    else:
                        raise AssertionError(f"unexpected draw {kind} {extra}")
                pre = f"c{ci}_s{t}_"
                out.update({pre + "grid": g_in.astype(np.uint8), pre + "age": a_in, pre + "wind": np.array(w_in),
                            pre + "burn": burn, pre + "grow": grow, pre + "draw_age": age,
                            pre + "wind_u": np.array(wind_u), pre + "wind_k": np.array(wind_k),
                            pre + "pine_n": n, pre + "pine_dirs": dirs, pre + "pine_thrust": thrust, pre + "pine_u": u,
                            pre + "pine_age": pine_age, pre + "pine_hits": pine_hits,
                            pre + "out_grid": np.asarray(grid).astype(np.uint8), pre + "out_age": ctx["fire_age"].copy(),
                            pre + "out_wind": np.array(int(ctx["wind_index"]))})
        finally:
            cl.neighborhood_at, np.random.standard_normal = orig_nb, orig_sn
        out[f"c{ci}_steps"] = np.array(steps)
    out["n"] = np.array(len(cases))
    return out


# (grid_size, H, W, steps, fire_frac, hidden slope from altitude, p_tree, p_wind_change, burn-draw scale: the burn
#  uniforms are drawn on [0, scale) so that ignitions are frequent at these small probabilities)
ALEX_JAX_CASES = [(256, 16, 256, 3, 0.10, True, 0.05, 0.5, 0.03),   # configs 3/4: R = 6, ages [576, 672)
                  (512, 16, 512, 2, 0.10, True, 0.05, 0.5, 0.03),   # config 5's grid: R = 7, ages [1152, 1344)
                  (256, 20, 24, 4, 0.25, False, 0.10, 0.9, 0.05),   # ragged small grid, free slopes, hot draws
                  (64, 48, 48, 3, 0.15, True, 0.0, 0.06, 0.1)]      # R = 4, the env's p_tree / p_wind_change


def gen_alexandridis_jax(R, rng):
    """PartiallyObservableForestFireJax (ca_alexandridis_jax.py:54-160 constructor, :164-206 burn probability,
    :321-424 _update_grid, :426-460 update) EXECUTED as published, under tests/golden/_jax_standin.py's numpy
    stand-in for jnp / jit / vmap / lax / random. Several consecutive `update` calls per case, the reference's
    returned per_env_context fed back. Recorded per step: the inputs, every random array in call order (burn
    uniforms (H,W,3,3), grow uniforms (H,W), new fire ages (H,W), wind-change uniform, wind offset), the
    burn probabilities _compute_burn_probability returned, and the outputs (grid, fire_age, wind_index).
    Winds from the reference's get_winds(True) (init_utils.py:233-245); slopes from its get_slope of its
    init_altitude (:76-116, :166-200) where `hidden`, else free normal(0, 20) slopes (not antisymmetric)."""
    import contextlib
    import io

    sys.path.insert(0, HERE)
    import _jax_standin as js

    rlog = js.RandomLog(np.random.default_rng(0))
    with js.installed(rlog):
        iu = _load("gym_cellular_automata.forest_fire.bulldozer.utils.init_utils",
                   f"{REF}/forest_fire/bulldozer/utils/init_utils.py")
        aj = _load("gym_cellular_automata.forest_fire.operators.ca_alexandridis_jax",
                   f"{REF}/forest_fire/operators/ca_alexandridis_jax.py")
    cls = aj.PartiallyObservableForestFireJax
    captured = []
    orig_bp = cls._compute_burn_probability

    def bp(self, *a):
        r = orig_bp(self, *a)
        captured.append(np.asarray(r).copy())
        return r

    cls._compute_burn_probability = bp
    winds = np.asarray(iu.get_winds(True), dtype=np.float64)  # (8, 2, 3, 3), jnp.array -> float32 below
    out = {"winds": winds.astype(np.float32)}
    try:
        for ci, (gs, H, W, steps, ff, hidden, p_tree, p_wc, bscale) in enumerate(ALEX_JAX_CASES):
            crng = np.random.default_rng(4242 + ci)
            grid = crng.choice([0, 1, 2], size=(H, W), p=[0.1, 0.9 - ff, ff])
            fire_age = np.where(crng.random((H, W)) < 0.3, crng.integers(-1, 3, (H, W)),  # burn-outs (age <= 1)
                                crng.integers(1, int(gs * 1.5 * 1.75) + 1, (H, W)))
            age = np.where(grid == 2, fire_age, crng.integers(-2, 3, (H, W))).astype(np.float32)
            veg = crng.integers(0, 7, (H, W))  # 0 and 6 exercise the reference's clip to 1..5 (:176-178)
            den = crng.integers(0, 7, (H, W))
            dous = (crng.random((H, W)) < 0.08).astype(np.int32)
            if hidden:
                np.random.seed(900 + ci)
                alt = iu.init_altitude(H, W, 1)
                with contextlib.redirect_stdout(io.StringIO()):  # get_slope prints a histogram
                    slope = np.asarray(iu.get_slope(alt, H, W, 1))[0]
                out[f"c{ci}_altitude"] = alt[0]
            else:
                slope = crng.normal(0, 20, (H, W, 3, 3)).clip(-89, 89)
                slope[..., 1, 1] = 0
            wrap = js.wrap
            with js.installed(rlog):
                op = cls(gs, 0, 1, 2)
            shared = {"winds": wrap(winds), "p_tree": wrap(np.float32(p_tree)),
                      "p_wind_change": wrap(np.float32(p_wc))}
            ctx = {"wind_index": wrap(np.int32(crng.integers(0, 8))), "density": wrap(den),
                   "vegetation": wrap(veg), "slope": wrap(slope), "fire_age": wrap(age),
                   "dousing_count": wrap(dous), "key": ("key", -1)}
            g = wrap(grid)
            out[f"c{ci}_meta"] = np.array([gs, H, W, steps])
            out[f"c{ci}_p"] = np.array([p_tree, p_wc], dtype=np.float32)
            out[f"c{ci}_veg"], out[f"c{ci}_den"] = veg.astype(np.uint8), den.astype(np.uint8)
            out[f"c{ci}_dous"] = dous.astype(np.uint8)
            out[f"c{ci}_slope"] = np.asarray(ctx["slope"])  # float32 (jax canonicalises float64 inputs)
            rlog.gen = np.random.default_rng(7000 + ci)
            rlog.uniform_scale = lambda shape, bscale=bscale: bscale if len(shape) == 4 else 1.0
            for t in range(steps):
                rlog.log.clear()
                captured.clear()
                pre = f"c{ci}_s{t}_"
                out[pre + "grid"] = np.asarray(g).astype(np.uint8)
                out[pre + "age"] = np.asarray(ctx["fire_age"]).astype(np.float32)
                out[pre + "wind"] = np.array(int(ctx["wind_index"]))
                g, ctx, _ = op.update(g, None, ctx, shared)
                kinds = [(k, len(s)) for k, s, _, _ in rlog.log]
                assert kinds == [("uniform", 4), ("uniform", 2), ("randint", 2), ("uniform", 0), ("randint", 0)], kinds
                assert rlog.log[2][3] == (int(op.fire_age_min), int(op.fire_age_max)) and rlog.log[4][3] == (1, 8)
                assert len(captured) == 1 and captured[0].dtype == np.float32, "jax's f32 arithmetic was not kept"
                out.update({pre + "u_burn": rlog.log[0][2], pre + "u_grow": rlog.log[1][2],
                            pre + "new_ages": rlog.log[2][2], pre + "wind_u": np.float32(rlog.log[3][2]),
                            pre + "wind_k": np.int32(rlog.log[4][2]), pre + "probs": captured[0],
                            pre + "out_grid": np.asarray(g).astype(np.uint8),
                            pre + "out_age": np.asarray(ctx["fire_age"]).astype(np.float32),
                            pre + "out_wind": np.array(int(ctx["wind_index"]))})
                assert np.asarray(ctx["fire_age"]).dtype == np.float32
    finally:
        cls._compute_burn_probability = orig_bp
    out["n"] = np.array(len(ALEX_JAX_CASES))
    return out


def _load_advanced_mdp(js, rlog):
    """advanced_bulldozer.py's MDP class, loaded under the jax stand-in. The module's other imports get what
    they need to import: the operator classes (unused by the observation builders) as placeholders, an empty
    render module; extension_utils.py and init_utils.py are the reference's own files."""
    ops = sys.modules["gym_cellular_automata.forest_fire.operators"]
    for name in ("ModifyJax", "MoveJax", "MoveModifyJax", "RepeatCAJax", "PartiallyObservableForestFireJax"):
        if not hasattr(ops, name):
            setattr(ops, name, type(name, (), {}))
    r = types.ModuleType("gym_cellular_automata.forest_fire.bulldozer.utils.advanced_bulldozer_render")
    r.render, r.plot_grid_attribute = (lambda *a, **k: None), (lambda *a, **k: None)
    sys.modules[r.__name__] = r
    with js.installed(rlog):
        _load("gym_cellular_automata.forest_fire.bulldozer.utils.init_utils",
              f"{REF}/forest_fire/bulldozer/utils/init_utils.py")
        eu = _load("gym_cellular_automata.forest_fire.bulldozer.utils.extension_utils",
                   f"{REF}/forest_fire/bulldozer/utils/extension_utils.py")
        ab = _load("gym_cellular_automata.forest_fire.bulldozer.advanced_bulldozer",
                   f"{REF}/forest_fire/bulldozer/advanced_bulldozer.py")
    return ab, eu


def gen_observation(R, rng):
    """The Advanced env's observation builders EXECUTED as published under the jax stand-in:
    MDP.build_observation_on_extensions (advanced_bulldozer.py:988-1018: transform_grid / apply_extensions of
    extension_utils.py:89-196, then grid_to_rgb_with_extensions :1020-1033 and grid_to_rgb :1035-1101) for the
    step frame, and grid_to_rgb_with_extensions on a plain (H, W) grid for the reset frame (:401-411 applies it
    per env; oracle/observation.reset_observation's convention; square grids only — on a non-square grid those
    expressions do not broadcast, in jax as in numpy). Inputs: grids of codes 0/1/2 (one case also 3,
    the code apply_visibility hides), dousing counts 0..2 (the water tint only at 1, :1081), day / night, the
    position on the border and inside, extension flags of the action (actions[2:]), enable_extensions and
    should_transform_grid on / off."""
    sys.path.insert(0, HERE)
    import _jax_standin as js

    rlog = js.RandomLog(np.random.default_rng(0))
    ab, _ = _load_advanced_mdp(js, rlog)
    wrap = js.wrap
    crng = np.random.default_rng(5150)
    out = {}
    cases = [(5, 5), (8, 8), (17, 23), (64, 64), (1, 6), (32, 16)]
    n = 0
    for H, W in cases:
        for k in range(6):
            codes = [0, 1, 2, 3] if (H, W) == (17, 23) and k < 3 else [0, 1, 2]
            grid = crng.choice(codes, size=(H, W), p=None).astype(np.float32)
            dous = crng.choice([0, 1, 2], size=(H, W), p=[0.7, 0.2, 0.1]).astype(np.int32)
            pos = np.array([crng.integers(0, H), crng.integers(0, W)] if k % 2 else [0, W - 1], np.int32)
            night = np.int32(k % 2 if k < 4 else crng.integers(0, 2))
            flags = [(0, 0), (1, 0), (0, 1), (1, 1)][crng.integers(0, 4)]
            enable, transform = bool(crng.integers(0, 2)), bool(crng.integers(0, 2))
            actions = np.array([crng.integers(0, 9), crng.integers(0, 2), *flags], np.int32)
            mdp = ab.MDP.__new__(ab.MDP)
            mdp.tree, mdp.fire, mdp.empty = 1, 2, 0
            mdp.should_transform_grid, mdp.enable_extensions = transform, enable
            ctx = {"is_night": wrap(night), "dousing_count": wrap(dous)}
            rgb, ch = mdp.build_observation_on_extensions(wrap(grid), wrap(pos), wrap(actions), ctx, {})
            # the reset convention broadcasts (H, 3) against (H, W, 1): defined for square grids only
            reset = mdp.grid_to_rgb_with_extensions(wrap(grid), ctx, wrap(pos)) if H == W else np.zeros(0)
            pre = f"c{n}_"
            out.update({pre + "grid": grid.astype(np.uint8), pre + "dous": dous.astype(np.uint8), pre + "pos": pos,
                        pre + "night": np.array(int(night)), pre + "actions": actions,
                        pre + "flags": np.array([int(enable), int(transform)]),
                        pre + "rgb": np.asarray(rgb), pre + "channels": np.asarray(ch), pre + "reset": np.asarray(reset)})
            assert np.asarray(rgb).dtype == np.float32 and np.asarray(rgb).shape == (H, W, 3)
            n += 1
    out["n"] = np.array(n)
    return out


def gen_pinecones_jax(R, rng):
    """PartiallyObservableForestFireJax._handle_pinecone_spread (ca_alexandridis_jax.py:229-319, with
    _compute_pinecone_burn_probability :208-227) EXECUTED as published under the jax stand-in: the draws it consumed
    (Poisson counts, directions, normal thrusts, burn uniforms, in call order) and its outputs (flat landing rows /
    columns and the burn mask). The reference leaves the spotting disabled in _update_grid (:400-420); the fixture pins
    the function the device's opt-in pinecone pass restates."""
    sys.path.insert(0, HERE)
    import _jax_standin as js

    rlog = js.RandomLog(np.random.default_rng(0))
    with js.installed(rlog):
        aj = _load("gym_cellular_automata.forest_fire.operators.ca_alexandridis_jax",
                   f"{REF}/forest_fire/operators/ca_alexandridis_jax.py")
        iu = _load("gym_cellular_automata.forest_fire.bulldozer.utils.init_utils",
                   f"{REF}/forest_fire/bulldozer/utils/init_utils.py")
        op = aj.PartiallyObservableForestFireJax(256, 0, 1, 2)
    winds = np.asarray(iu.get_winds(True), dtype=np.float32)
    wrap = js.wrap
    out = {}
    cases = [(16, 16, 0.3), (24, 40, 0.15), (64, 64, 0.05), (7, 5, 0.5)]
    for ci, (H, W, ff) in enumerate(cases):
        crng = np.random.default_rng(8800 + ci)
        old = crng.choice([0, 1, 2], size=(H, W), p=[0.2, 0.8 - ff, ff])
        new = np.where(old == 2, crng.choice([0, 2], size=(H, W)), crng.choice([0, 1, 2], size=(H, W), p=[0.1, 0.8, 0.1]))
        veg, den = crng.integers(0, 7, (H, W)), crng.integers(0, 7, (H, W))
        ft = winds[ci % 8, 1]
        ctx = {"current_ft": wrap(ft), "vegetation": wrap(veg), "density": wrap(den)}
        rlog.gen = np.random.default_rng(9900 + ci)
        rlog.log.clear()
        rows, cols, burn = op._handle_pinecone_spread(wrap(new), ("key", ci), ctx, wrap(old == 2))
        kinds = [k for k, *_ in rlog.log]
        assert kinds == ["poisson", "randint", "normal", "uniform"], kinds
        pre = f"c{ci}_"
        out.update({pre + "old": old.astype(np.uint8), pre + "new": new.astype(np.uint8), pre + "veg": veg.astype(np.uint8),
                    pre + "den": den.astype(np.uint8), pre + "ft": ft, pre + "n": rlog.log[0][2],
                    pre + "dirs": rlog.log[1][2], pre + "normal": rlog.log[2][2], pre + "u": rlog.log[3][2],
                    pre + "rows": np.asarray(rows), pre + "cols": np.asarray(cols),
                    pre + "burn": np.asarray(burn).astype(np.uint8)})
    out["n"] = np.array(len(cases))
    return out


def _load_advanced_env(js, rlog):
    """advanced_bulldozer.py with its real operators (ca_alexandridis_jax, move_modify_jax, repeat_ca_jax),
    extension_utils and init_utils, all loaded under the jax stand-in (`rlog` receives every draw)."""
    ops = sys.modules["gym_cellular_automata.forest_fire.operators"]
    r = types.ModuleType("gym_cellular_automata.forest_fire.bulldozer.utils.advanced_bulldozer_render")
    r.render, r.plot_grid_attribute = (lambda *a, **k: None), (lambda *a, **k: None)
    sys.modules[r.__name__] = r
    with js.installed(rlog):
        aj = _load("gym_cellular_automata.forest_fire.operators.ca_alexandridis_jax",
                   f"{REF}/forest_fire/operators/ca_alexandridis_jax.py")
        mmj = _load("gym_cellular_automata.forest_fire.operators.move_modify_jax",
                    f"{REF}/forest_fire/operators/move_modify_jax.py")
        rcj = _load("gym_cellular_automata.forest_fire.operators.repeat_ca_jax",
                    f"{REF}/forest_fire/operators/repeat_ca_jax.py")
        ops.PartiallyObservableForestFireJax = aj.PartiallyObservableForestFireJax
        ops.MoveJax, ops.ModifyJax, ops.MoveModifyJax = mmj.MoveJax, mmj.ModifyJax, mmj.MoveModifyJax
        ops.RepeatCAJax = rcj.RepeatCAJax
        iu = _load("gym_cellular_automata.forest_fire.bulldozer.utils.init_utils",
                   f"{REF}/forest_fire/bulldozer/utils/init_utils.py")
        _load("gym_cellular_automata.forest_fire.bulldozer.utils.extension_utils",
              f"{REF}/forest_fire/bulldozer/utils/extension_utils.py")
        ab = _load("gym_cellular_automata.forest_fire.bulldozer.advanced_bulldozer",
                   f"{REF}/forest_fire/bulldozer/advanced_bulldozer.py")
    return ab, iu


def gen_advanced_env(R, rng):
    """AdvancedForestFireBulldozerEnv (advanced_bulldozer.py) EXECUTED as published under the jax stand-in: the env
    built (use_hidden=True: the reference's own init_vegetation / init_density / init_altitude / get_slope /
    get_winds), reset, a dense mid-episode state written into the reference's own context layout, then consecutive
    `stateless_step` calls (:332-399: RepeatCAJax -> the Alexandridis rule, MoveModifyJax, time_step / is_night, the
    RGB observation, reward, terminated, steps_elapsed / reward_accumulated), every env's draws recorded in call order.
    Pins the batched env step (rows a13-a16, f1) at the env level."""
    import contextlib
    import io

    sys.path.insert(0, HERE)
    import _jax_standin as js

    rlog = js.RandomLog(np.random.default_rng(0))
    ab, iu = _load_advanced_env(js, rlog)
    wrap = js.wrap
    out = {}
    for ci, (N, E, steps, ext) in enumerate([(32, 3, 8, False), (24, 2, 6, True)]):
        np.random.seed(4100 + ci)
        with contextlib.redirect_stdout(io.StringIO()):
            env = ab.AdvancedForestFireBulldozerEnv(N, N, key=wrap(np.array([7, 0], np.uint32)), num_envs=E,
                                                    use_hidden=True, enable_extensions=ext)
            obs, info = env.reset()
        grid, ctx = obs
        pe = ctx["per_env_context"]
        crng = np.random.default_rng(4200 + ci)
        true_grid = crng.choice([0, 1, 2], size=(E, N, N), p=[0.1, 0.75, 0.15]).astype(np.float32)
        fire_age = np.where(true_grid == 2, crng.integers(1, 90, (E, N, N)), 0).astype(np.float32)
        pe["true_grid"] = wrap(true_grid)
        pe["fire_age"] = wrap(fire_age)
        pe["dousing_count"] = wrap((crng.random((E, N, N)) < 0.05).astype(np.int32))
        pe["time_step"] = wrap(np.array([399, 1, 799][:E], np.int32))  # the day / night toggle within the steps
        ctx["shared_context"]["p_wind_change"] = wrap(np.float32(0.5))
        pre = f"c{ci}_"
        out[pre + "meta"] = np.array([N, E, steps, int(ext)])
        for k in ("vegetation", "density", "altitude", "slope", "wind_index", "is_night", "time_step", "dousing_count",
                  "true_grid", "fire_age"):
            out[pre + "init_" + k] = np.asarray(pe[k])
        out[pre + "init_position"] = np.asarray(ctx["position"])
        out[pre + "init_time"] = np.asarray(ctx["time"])
        out[pre + "winds"] = np.asarray(ctx["shared_context"]["winds"])
        out[pre + "times"] = np.array([env._t_act_move, env._t_act_shoot, env._t_env_any])
        rlog.gen = np.random.default_rng(4300 + ci)
        for t in range(steps):
            n_ext = 3 if ext else 1  # extension choices (0 none, 1 unblur, 2 see-invisible-fires)
            action = np.stack([crng.integers(0, 9, E), crng.integers(0, 2, E), crng.integers(0, n_ext, E)], axis=1)
            rlog.log.clear()
            with contextlib.redirect_stdout(io.StringIO()):
                obs, reward, term, trunc, info = env.stateless_step(wrap(action.astype(np.int32)), obs, info)
            rgb, ctx = obs
            pe = ctx["per_env_context"]
            kinds = [(k, len(sh)) for k, sh, _, _ in rlog.log]
            assert kinds == [("uniform", 4), ("uniform", 2), ("randint", 2), ("uniform", 0), ("randint", 0)] * E, kinds
            st = f"{pre}s{t}_"
            out[st + "action"] = action
            for j, name in enumerate(("u_burn", "u_grow", "new_ages", "wind_u", "wind_k")):
                out[st + name] = np.stack([np.asarray(rlog.log[5 * e + j][2]) for e in range(E)])
            for k in ("true_grid", "fire_age", "wind_index", "dousing_count", "time_step", "is_night"):
                out[st + k] = np.asarray(pe[k])
            out[st + "position"] = np.asarray(ctx["position"])
            out[st + "time"] = np.asarray(ctx["time"])
            out[st + "rgb"] = np.asarray(rgb)
            out[st + "reward"] = np.asarray(reward)
            out[st + "terminated"] = np.asarray(term)
            out[st + "steps_elapsed"] = np.asarray(info["steps_elapsed"])
            out[st + "reward_accumulated"] = np.asarray(info["reward_accumulated"])
    out["n"] = np.array(2)
    return out


GENERATORS = {"windy": gen_windy, "repeat_ca": gen_repeat, "move_modify": gen_move_modify, "bulldozer": gen_bulldozer,
              "drossel": gen_drossel, "helicopter": gen_helicopter, "moore": gen_moore, "init_utils": gen_init_utils,
              "alexandridis_classic": gen_alexandridis_classic, "alexandridis_jax": gen_alexandridis_jax,
              "observation": gen_observation, "pinecones_jax": gen_pinecones_jax, "advanced_env": gen_advanced_env}


def main():
    R = load_reference()
    rng = np.random.default_rng(20260101)
    names = sys.argv[1:] or list(GENERATORS)
    order = list(GENERATORS)
    last = max(order.index(n) for n in names)
    for name in order[:last + 1]:
        data = GENERATORS[name](R, rng)  # every earlier generator runs, in order, so the shared rng stream is unchanged
        if name not in names:
            continue
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **data)
        print(f"{name}: {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
