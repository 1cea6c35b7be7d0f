"""A/B of the two Alexandridis step mappings on the headline workload (4096 x 256^2, R = 6, the bench's config-3
state): gca_alex_step_packed (tiled, coalesced slopes) vs gca_alex_step_march (marching, natural slopes), plain and
with the fused frame. Each variant runs K steps from the same restored state, HIP events around the K launches on
the library's stream, median of `reps`. Prints one JSON line (ms per step). Run on the GPU box."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def main(E=4096, N=256, K=10, reps=5, hidden=False, only=None, rgb_modes=(False, True), reset_state=False):
    import torch

    import bench
    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    env = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=hidden, device=device, observation="rgb",
                                         enable_extensions=False, hidden_rng="philox" if hidden else None)
    env.reset()
    st = dev.stream_ptr(device)
    natural = torch.zeros_like(env.slope_data)
    if env.altitude is not None:
        call("gca_alex_edge_slope_from_altitude", dev.ptr(env.altitude), dev.ptr(natural), E, N, N, st)
    else:
        call("gca_alex_edge_slope_from_altitude", None, dev.ptr(natural), E, N, N, st)

    def launch(fn, rgb):
        a, b = env.cur, 1 - env.cur
        slope = env.slope_data if "packed" in fn else natural
        args = [env.alex_params, E, N, N, dev.ptr(env.grid[a]), dev.ptr(env.grid[b]), dev.ptr(env.age[a]),
                dev.ptr(env.age[b]), dev.ptr(env.vd), dev.ptr(env.dous_bits), dev.ptr(slope), dev.ptr(env.wind_index),
                dev.ptr(env.rng_step), dev.ptr(env.counts), None, None]
        if rgb:
            args += [dev.ptr(env.obs_colors), dev.ptr(env.is_night), dev.ptr(env.rgb)]
        call(fn + ("_rgb" if rgb else ""), *args, st)
        env.cur = b

    out = {"E": E, "N": N, "K": K, "reps": reps, "hidden": hidden, "state": "reset" if reset_state else "mid-episode"}
    for rgb in rgb_modes:
        for fn in ("gca_alex_step_packed", "gca_alex_step_march"):
            if only and only not in fn:
                continue
            times = []
            for _ in range(reps):
                if reset_state:  # the episode-start state (2 fires per env): the quiet-tile copies dominate
                    env.reset()
                else:
                    bench.synthetic_state(env, 0, device)
                launch(fn, rgb)  # warm-up
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(K):
                    launch(fn, rgb)
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) / K)
            times.sort()
            out[fn.replace("gca_alex_step_", "") + ("_rgb" if rgb else "") + "_ms"] = round(times[len(times) // 2], 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    # --only march|packed: one mapping; --plain: no fused-frame variants; --reps N; --size N (grid side), --envs E;
    # --reset: time from the reset state instead of the bench's mid-episode state; --rgb-only: the fused-frame variants
    args = sys.argv[1:]
    only = args[args.index("--only") + 1] if "--only" in args else None
    reps = int(args[args.index("--reps") + 1]) if "--reps" in args else 5
    N = int(args[args.index("--size") + 1]) if "--size" in args else 256
    E = int(args[args.index("--envs") + 1]) if "--envs" in args else 4096
    main(E=E, N=N, hidden="--hidden" in args, only=only, reps=reps,
         rgb_modes=(False,) if "--plain" in args else ((True,) if "--rgb-only" in args else (False, True)), reset_state="--reset" in args)
