#!/usr/bin/env python3
"""Config4 gap probe (one GPU): the use_hidden=True env's step on its own layers, then on C3's constant
layers copied into the same buffers, then a C3 env built afterwards. Separates the layers' values from
where the env's buffers landed in memory.

    python scripts/ab_c4.py > gpurun_out/ab_c4.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-cellular-automata_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import numpy as np
    import torch

    import bench
    from ab_data import timed
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    dev = torch.device("cuda:0")
    E, N = 4096, 256
    out = {}

    def probe(env, name):
        env.reset()
        bench.synthetic_state(env, 0, dev)
        g0, a0 = env.grid[env.cur].clone(), env.age[env.cur].clone()

        def restore():
            env.grid[env.cur].copy_(g0)
            env.age[env.cur].copy_(a0)

        def step():
            env.ca_step()
            env.cur ^= 1

        out[name] = timed(step, restore)
        print(name, out[name], file=sys.stderr, flush=True)

    env4 = AdvancedForestFireBulldozerEnv(N, N, key=2, num_envs=E, use_hidden=True, device=dev,
                                          hidden_rng=np.random.RandomState(2))
    probe(env4, "c4_layers_ms")
    env4.slope_data.fill_(1.0)
    env4.vd.fill_(3 | (3 << 4))
    probe(env4, "c4_buffers_c3_values_ms")
    del env4
    torch.cuda.empty_cache()
    env3 = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=dev)
    probe(env3, "c3_after_ms")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
