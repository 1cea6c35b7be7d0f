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
  init_utils.npz   init_vegetation / init_density / init_altitude / get_slope after
                   np.random.seed(k) (bulldozer/utils/init_utils.py:10-200). Those functions
                   use numpy and the global legacy np.random state only; the module's own
                   `import jax.numpy` / `from flax import struct` lines get empty stand-in
                   modules here (jax and flax are not installed).

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


GENERATORS = {"windy": gen_windy, "repeat_ca": gen_repeat, "move_modify": gen_move_modify, "bulldozer": gen_bulldozer,
              "drossel": gen_drossel, "helicopter": gen_helicopter, "moore": gen_moore, "init_utils": gen_init_utils}


def main():
    R = load_reference()
    rng = np.random.default_rng(20260101)
    names = sys.argv[1:] or list(GENERATORS)
    for name, fn in GENERATORS.items():
        data = fn(R, rng)  # every generator runs, in order, so the shared rng stream is unchanged
        if name not in names:
            continue
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **data)
        print(f"{name}: {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
