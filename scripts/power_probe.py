"""Board power and clocks while the headline Alexandridis step runs back to back (is the step power-limited?).
Samples `amd-smi metric --power --clock` (and the static power limit) from a child process while the marching kernel
steps the bench's C3 state for ~`secs` seconds, for the C3 layers (flat altitude) and the hidden (config 4) layers.
Prints one JSON line. Run on the GPU box."""
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def smi(args):
    try:
        return subprocess.run(["amd-smi"] + args, capture_output=True, text=True, timeout=30).stdout
    except Exception as exc:  # noqa: BLE001 - a missing tool is reported, not fatal
        return f"error: {exc}"


def main(E=4096, N=256, secs=6.0):
    lim = smi(["static", "--limit", "-g", "0"])
    out = {"socket_power_limit_w": [float(x) for x in re.findall(r"SOCKET_POWER_LIMIT: ([0-9.]+) W", lim)],
           "note": "amd-smi samples every ~0.5 s while the marching step runs the bench's C3 state (restored every 40 "
                   "steps); gfx_clk_mhz = every GFX_i CLK line of the samples"}
    import torch

    import bench
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    for name, hidden in (("c3_flat", False), ("c4_hidden", True)):
        env = AdvancedForestFireBulldozerEnv(N, N, key=2, num_envs=E, use_hidden=hidden, device=device,
                                             hidden_rng="philox" if hidden else None, observation="grid")
        env.reset()
        bench.synthetic_state(env, 0, device)
        torch.cuda.synchronize()
        sampler = subprocess.Popen(["bash", "-c", "for i in 1 2 3 4 5 6 7 8; do sleep 0.5; amd-smi metric --power --clock -g 0; done"],
                                   stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        t0, n = time.time(), 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ms = []
        while time.time() - t0 < secs:  # the bench's state, restored every 40 steps (untimed)
            bench.synthetic_state(env, 0, device)
            e0.record()
            for _ in range(40):
                env.ca_step()
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1) / 40)
            n += 40
        samples = sampler.communicate(timeout=60)[0]
        out[name] = {"steps": n, "ms_per_step_median": sorted(ms)[len(ms) // 2],
                     "socket_power_w": [float(x) for x in re.findall(r"SOCKET_POWER: ([0-9.]+) W", samples)],
                     "gfx_clk_mhz": [int(x) for x in re.findall(r"GFX_\d+:\s*\n\s*CLK: ([0-9]+) MHz", samples)]}
        del env
        torch.cuda.empty_cache()
        print(f"{name}: {n} steps", flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
