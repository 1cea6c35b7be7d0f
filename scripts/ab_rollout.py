"""Rollout kernel rate vs K (env.rollout_random: K env steps per launch, per-step rewards / done flags recorded) at
BASELINE configs 2 (1024 x 256^2) and 5's shard (1024 x 512^2), from the bench's restored mid-episode state, beside
step_random (one launch per env step). HIP-event / wall timing through bench.timed_loop, median of 3. One JSON line.
Run on the GPU box."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def main():
    import torch

    import bench
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    out = {}
    for N in (256, 512):
        E = 1024
        env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=0x5EED, materialize_obs=False)
        env.reset()
        action = torch.zeros((E, 2), dtype=torch.int32, device=device)
        restore = bench.env_snapshot(env, lambda: env.step(env.sample_actions(action, 9)), 64)
        dt, _ = bench.timed_loop(lambda ev: env.step_random(9, action), 256, 0, None, device, reps=3, prepare=restore)
        out[f"N{N}_step_random"] = E * 256 / dt
        for K in (8, 32, 128, 512):
            out[f"N{N}_rollout_k{K}"] = bench.rollout_rate(env, 9, max(1024 // K, 2) * K, restore, None, device, 1, k=K)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
