"""A/B of the batched Windy bulldozer env step (BASELINE config 2: 1024 x 256^2; config 5's shard: 1024 x 512^2) for
one library build (GCA_LIB_PATH): a hipGraph of 8 env steps (device random actions + env.step), timed from the same
mid-episode state (reset + 64 steps, restored before each repetition), median of `reps`. One JSON line (env-steps/s).
Run on the GPU box."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def main(reps=5):
    import torch

    import bench
    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv
    from gymca_amd.graph import StepGraph

    device = torch.device("cuda", 0)
    out = {}
    for N in (256, 512):
        E = 1024
        env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=0x5EED, materialize_obs=False)
        action = torch.zeros((E, 2), dtype=torch.int32, device=device)

        def one_step():
            call("gca_random_actions", dev.ptr(action), E, 0, 9, dev.ptr(env.rng_step), dev.stream_ptr(device))
            env.step(action)

        restore = bench.env_snapshot(env, one_step, 64)
        graph = StepGraph(one_step, n_steps=8, device=device)
        times = []
        for _ in range(reps):
            restore()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                graph.replay()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / 40)
        times.sort()
        ms = times[len(times) // 2]
        out[f"n{N}_ms_per_env_step"] = round(ms, 5)
        out[f"n{N}_env_steps_per_s"] = E / (ms * 1e-3)
        del env, graph
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
