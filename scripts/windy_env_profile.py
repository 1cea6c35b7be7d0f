"""Windy bulldozer env steps for a rocprofv3 kernel trace: E envs, N^2 grids, K eager env steps with device random
actions, fused (gca_bulldozer_step_fused) or the three-kernel sequence. Usage: python scripts/windy_env_profile.py
N E K fused(0/1)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def main(N=256, E=1024, K=100, fused=True):
    import time

    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=0x5EED, materialize_obs=False, fused=fused)
    env.reset()
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)
    st = dev.stream_ptr(device)
    for k in range(K):
        call("gca_random_actions", dev.ptr(action), E, 0, 9, dev.ptr(env.rng_step), st)
        env.step(action)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        call("gca_random_actions", dev.ptr(action), E, 0, 9, dev.ptr(env.rng_step), st)
        env.step(action)
    torch.cuda.synchronize()
    print(f"N={N} E={E} fused={fused}: {(time.perf_counter() - t0) / K * 1e6:.1f} us per eager env step, "
          f"{int((env.steps > 0).sum())} envs stepped the CA in the last step", flush=True)


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    main(*a[:3], bool(a[3]) if len(a) > 3 else True)
