"""CPU cross-check: the reference's own CPU path timed beside the restatement the
bench's CPU legs run (oracle/windy.py), on the same core, same grids, same draws. RUNS IN THE BUILD CONTAINER ONLY (it
imports /root/reference in place through tests/golden/make_golden.py's loader; nothing is copied).

  ref     WindyForestFire.update(grid, None, wind)  (ca_windy.py:41-51, its own np_random roll)
          + CAEnv.count_cells's Counter(grid.flatten().tolist())  (ca_env.py:94-99)
  port    oracle.windy.windy_step(grid, wind, roll) + the same Counter count
  unique  the port with np.unique instead of Counter (the bench's earlier, faster-than-reference count)

Interleaved A/B/A/B passes of `--seconds` each on one core (taskset is not used: the process runs where it runs, all
legs in the same thread), 256x256 grids of {0: .1, 3: .6, 25: .3}. Writes profiles/cpu_crosscheck.json; §8d asks for
port within +-20 % of ref.

    python scripts/cpu_crosscheck.py [--seconds 3]
"""
import argparse
import json
import os
import platform
import sys
import time
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-cellular-automata_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--passes", type=int, default=3)
    args = ap.parse_args()
    import make_golden as mg  # puts the gymnasium stand-in on sys.path, loads the reference file by file

    from oracle import windy as owindy

    R = mg.load_reference()
    wind = mg.WIND_BULLDOZER
    op = R.windy.WindyForestFire(0, 3, 25)
    op.seed(1)
    rng = np.random.default_rng(9)

    def fresh():
        return rng.choice(np.array([0, 3, 25]), size=(256, 256), p=[0.1, 0.6, 0.3]).astype(np.int64)

    def leg(kind, seconds):
        g, steps, t0 = fresh(), 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            if kind == "ref":
                g, _ = op.update(g, None, wind)
                Counter(np.asarray(g).flatten().tolist())
            else:
                g = owindy.windy_step(g, wind, rng.random((3, 3)))
                if kind == "port":
                    Counter(g.flatten().tolist())
                else:
                    np.unique(g, return_counts=True)
            steps += 1
            if steps % 64 == 0:
                g = fresh()  # keep the fire alive (a burnt-out grid is all zeros)
        return 256 * 256 * steps / (time.perf_counter() - t0)

    rates = {"ref": [], "port": [], "unique": []}
    for _ in range(args.passes):
        for kind in rates:
            rates[kind].append(leg(kind, args.seconds))
    med = {k: sorted(v)[len(v) // 2] for k, v in rates.items()}

    # the bulldozer env loop, 256^2, random actions: the reference's ForestFireBulldozerEnv (with the {"wind": W}
    # unwrap make_golden.py applies) against bench.py's restated loop (oracle.windy.BulldozerOracle +
    # the Counter count), env-steps/s
    import bench
    from gymca_amd.forest_fire.bulldozer.bulldozer import DEFAULT_WIND, bulldozer_timings, parse_wind  # noqa: F401

    orig = R.windy.WindyForestFire.update

    def patched(self, grid, action, wind):
        if isinstance(wind, dict):
            g, _ = orig(self, grid, action, wind["wind"])
            return g, wind
        return orig(self, grid, action, wind)

    def ref_env_leg(seconds):
        R.windy.WindyForestFire.update = patched
        try:
            env = R.bd.ForestFireBulldozerEnv(256, 256)
            env.reset(seed=1)
            arng = np.random.default_rng(3)
            steps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < seconds:
                _, _, term, _, _ = env.step(np.array([arng.integers(0, 9), arng.integers(0, 2)]))
                steps += 1
                if term:
                    env.reset()
            return steps / (time.perf_counter() - t0)
        finally:
            R.windy.WindyForestFire.update = orig

    env_rates = {"ref": [], "port": []}
    for _ in range(args.passes):
        env_rates["ref"].append(ref_env_leg(args.seconds))
        env_rates["port"].append(bench.bulldozer_cpu_baseline(args.seconds)["value"])
    env_med = {k: sorted(v)[len(v) // 2] for k, v in env_rates.items()}
    out = {"what": "WindyForestFire 256x256 step + cell count, one core, cell-updates/s (median of interleaved passes)",
           "reference": "ca_windy.py WindyForestFire.update (its own np_random roll) + Counter count (ca_env.py:94-99)",
           "port": "oracle/windy.py windy_step (scipy convolve2d restatement) + the same Counter count",
           "unique": "the port with np.unique counting (faster than the reference's Counter)",
           "median": med, "passes": rates, "port_over_ref": med["port"] / med["ref"],
           "unique_over_ref": med["unique"] / med["ref"],
           "within_20pct": abs(med["port"] / med["ref"] - 1) <= 0.2,
           "bulldozer_env_256": {"what": "ForestFireBulldozerEnv 256x256 env loop, random actions, env-steps/s, one core",
                                 "reference": "bulldozer.py ForestFireBulldozerEnv.step (the {'wind': W} unwrap patch)",
                                 "port": "bench.py bulldozer_cpu_baseline (oracle/windy.py BulldozerOracle + Counter)",
                                 "median": env_med, "passes": env_rates,
                                 "port_over_ref": env_med["port"] / env_med["ref"],
                                 "within_20pct": abs(env_med["port"] / env_med["ref"] - 1) <= 0.2},
           "seconds_per_pass": args.seconds, "cpu": platform.processor() or platform.machine(),
           "numpy": np.__version__}
    path = os.path.join(ROOT, "profiles", "cpu_crosscheck.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
