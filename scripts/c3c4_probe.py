"""Config 3 vs config 4 (use_hidden) on the SAME grid / fire-age / wind state: the packed Alexandridis launch
with C3's constant layers, with C4's hidden layers, and with C4's buffers refilled by C3's constants.
Every launch starts from the restored state, so the only difference between the groups is the layer VALUES.
Prints one JSON line (mean kernel ms per group, HIP events); under rocprofv3 the dispatches come in the
order: GROUPS x (WARM + K) alex_step launches. Usage: python scripts/c3c4_probe.py [K]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
WARM = 5
E, N = 4096, 256
dev = torch.device("cuda", 0)
env3 = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=dev, observation="grid")
env4 = AdvancedForestFireBulldozerEnv(N, N, key=2, num_envs=E, use_hidden=True, hidden_rng="philox", device=dev,
                                      observation="grid")
for env in (env3, env4):
    env.reset()
bench.synthetic_state(env3, 0, dev)
state = (env3.grid[env3.cur].clone(), env3.age[env3.cur].clone(), env3.wind_index.clone())


def run(env):
    ev = []
    for i in range(WARM + K):
        env.set_state(grid=state[0], fire_age=state[1], wind_index=state[2])
        env.rng_step.fill_(i)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        env.ca_step()
        b.record()
        if i >= WARM:
            ev.append((a, b))
    torch.cuda.synchronize(dev)
    return sum(x.elapsed_time(y) for x, y in ev) / len(ev)


out = {"c3": run(env3), "c4": run(env4)}
# C4's buffers, C3's values: constant layers (veg = den = 3, altitude 0 -> every edge value 1.0)
env4.set_state(vegetation=torch.full((E, N, N), 3, dtype=torch.uint8, device=dev),
               density=torch.full((E, N, N), 3, dtype=torch.uint8, device=dev),
               altitude=torch.zeros((E, N, N), dtype=torch.float64, device=dev))
out["c4_buffers_c3_values"] = run(env4)
out["c3_again"] = run(env3)
out["order"] = ["c3", "c4", "c4_buffers_c3_values", "c3_again"]
out["launches_per_group"] = WARM + K
print(json.dumps(out))
