"""cProfile of the single-env drop-ins (ForestFireBulldozerEnv 256x256 with random actions, ForestFireHelicopterEnv
5x5): where a reference user's per-step time goes. Run on the GPU box; prints the top functions by cumulative time."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def main():
    import numpy as np
    import torch

    from gymca_amd.forest_fire.bulldozer import ForestFireBulldozerEnv

    env = ForestFireBulldozerEnv(256, 256)
    env.reset(seed=0)
    rng = np.random.default_rng(3)
    acts = [(int(rng.integers(0, 9)), int(rng.integers(0, 2))) for _ in range(4000)]
    for a in acts[:50]:
        env.step(a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for a in acts[50:2050]:
        _, _, term, _, _ = env.step(a)
        n += 1
        if term:
            env.reset()
    torch.cuda.synchronize()
    print(f"bulldozer 256: {n / (time.perf_counter() - t0):.0f} env-steps/s", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for a in acts[2050:3050]:
        _, _, term, _, _ = env.step(a)
        if term:
            env.reset()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
