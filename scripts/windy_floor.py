"""Where the batched Windy env step's time goes (BASELINE config 2: 1024 x 256^2; and 1024 x 512^2): hipGraphs of 8
launches of (a) the bench's env step (device random actions + gca_bulldozer_step_fused) from a restored mid-episode
state, (b) the random-action kernel alone, (c) the fused env step alone (fixed actions), (d) the fused env step with
every env finished (each workgroup leaves after its O(1) work: the launch floor of a 1024-workgroup step), (e) a
one-element torch kernel (the graph's per-launch floor). HIP events around 5 replays, median of 5. One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def timed(graph, restore, reps=5, replays=5, n=8):
    import torch

    ts = []
    for _ in range(reps):
        if restore:
            restore()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(replays):
            graph.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / (replays * n))
    ts.sort()
    return round(ts[len(ts) // 2], 3)


def main():
    import torch

    import bench
    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv
    from gymca_amd.graph import StepGraph

    device = torch.device("cuda", 0)
    out = {"unit": "us per launch (or per env step)"}
    for N in (256, 512):
        E = 1024
        env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=0x5EED, materialize_obs=False)
        action = torch.zeros((E, 2), dtype=torch.int32, device=device)
        def actions():  # the stream is read at call time: under capture it is the graph's capture stream
            call("gca_random_actions", dev.ptr(action), E, 0, 9, dev.ptr(env.rng_step), dev.stream_ptr(device))

        def one_step():
            actions()
            env.step(action)

        restore = bench.env_snapshot(env, one_step, 64)
        g_env = StepGraph(one_step, n_steps=8, device=device)
        out[f"n{N}_env_step"] = timed(g_env, restore)
        g_act = StepGraph(actions, n_steps=8, device=device)
        out[f"n{N}_actions_only"] = timed(g_act, restore)
        restore()
        actions()
        g_step = StepGraph(lambda: env.step(action), n_steps=8, device=device)
        out[f"n{N}_fused_step_only"] = timed(g_step, restore)

        def all_done():
            restore()
            env.done.fill_(1)

        out[f"n{N}_fused_step_all_done"] = timed(g_step, all_done)
        del env, g_env, g_act, g_step
        torch.cuda.empty_cache()
    x = torch.zeros(1, device=device)
    g_tiny = StepGraph(lambda: x.add_(1.0), n_steps=8, device=device)
    out["tiny_kernel"] = timed(g_tiny, None)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
