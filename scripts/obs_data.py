"""r02o: is the RGB observation's write rate data-dependent? Times (HIP events, 20 reps) the observation kernel of the
batched env on its synthetic mid-episode state, on an all-EMPTY grid (one colour everywhere), and write-only fills of the
same buffer with 0.0 / 0.5 and a broadcast copy of one random RGB row (GCA_BENCH_EXT=0: the plain kernel). Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-cellular-automata_amd"))
from gymca_amd.forest_fire.bulldozer.advanced import AdvancedForestFireBulldozerEnv  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


E, N = 4096, 256
dev = torch.device("cuda:0")
env = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=dev, observation="rgb",
                                     enable_extensions=os.environ.get("GCA_BENCH_EXT", "0") != "0")
env.reset()
for _ in range(5):
    env.step(torch.randint(0, 9, (E,), device=dev))
out = {}
out["obs_mid_episode_ms"] = timed(lambda: env.render_observation())
g = env.grid[env.cur]
saved = g.clone()
g.fill_(int(env._empty))
out["obs_all_empty_ms"] = timed(lambda: env.render_observation())
g.copy_(saved)
rgb = env.rgb
out["fill_0_ms"] = timed(lambda: rgb.fill_(0.0))
out["fill_05_ms"] = timed(lambda: rgb.fill_(0.5))
small = torch.rand((1, 1, N, 3), device=dev)
out["expand_copy_random_row_ms"] = timed(lambda: rgb.copy_(small.expand(E, N, N, 3)))
out["gb_written"] = rgb.numel() * 4 / 1e9
print(json.dumps(out))
