"""A/B of the flat-terrain march step (edge_slope = NULL: every slope factor 1, no slope planes streamed) against the
general step reading the env's edge planes (all factors 1.0 for use_hidden=False), on the bench's config-3 state
(4096 x 256^2, R = 6): outputs compared bit for bit (grid, ages, counts), then K launches of each from the same
restored state, HIP events on the library's stream, median of `reps`. GCA_LIB_PATH selects a variant library.
Prints one JSON line. Run on the GPU box."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def main(E=4096, N=256, K=10, reps=5, rgb=False):
    import torch

    import bench
    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    env = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=device, observation="rgb")
    env.reset()
    st = dev.stream_ptr(device)
    assert bool((env.slope_data.abs() == 1.0).all())

    assert env.uniform_layers

    def launch(flat):  # flat: 0 general, 1 flat terrain, 2 flat + uniform layers
        a, b = env.cur, 1 - env.cur
        args = [env.alex_params, E, N, N, dev.ptr(env.grid[a]), dev.ptr(env.grid[b]), dev.ptr(env.age[a]),
                dev.ptr(env.age[b]), None if flat == 2 else dev.ptr(env.vd), dev.ptr(env.dous_bits),
                None if flat else dev.ptr(env.slope_data),
                dev.ptr(env.wind_index), dev.ptr(env.rng_step), dev.ptr(env.counts), None, None]
        if rgb:
            args += [dev.ptr(env.obs_colors), dev.ptr(env.is_night), dev.ptr(env.rgb)]
        call("gca_alex_step_march" + ("_rgb" if rgb else ""), *args, st)
        env.cur = b

    out = {"E": E, "N": N, "K": K, "reps": reps, "rgb": rgb, "lib": os.environ.get("GCA_LIB_PATH", "default")}
    res = {}
    for flat in (0, 1, 2):
        bench.synthetic_state(env, 0, device)
        for _ in range(3):
            launch(flat)
        torch.cuda.synchronize()
        res[flat] = (env.grid[env.cur].clone(), env.age[env.cur].clone(), env.counts.clone(),
                     env.rgb.clone() if rgb else None)
    same = all(torch.equal(x, y) for f in (1, 2) for x, y in zip(res[0], res[f]) if x is not None)
    out["bit_exact"] = bool(same)
    del res
    for rep in range(2):
        for flat in (0, 1, 2):
            times = []
            for _ in range(reps):
                bench.synthetic_state(env, 0, device)
                launch(flat)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(K):
                    launch(flat)
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) / K)
            times.sort()
            out[("general", "flat", "flat_uniform")[flat] + f"_p{rep}_ms"] = round(times[len(times) // 2], 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(rgb="--rgb" in sys.argv[1:])
