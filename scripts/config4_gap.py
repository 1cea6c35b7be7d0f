"""Where does config 4 (use_hidden=True: random vegetation / density and hilly altitude) lose time against config 3
(constant layers, flat altitude) on the same kernel? One env of 4096 x 256^2 with the hidden layers; the C3 mid-episode
state; four layer sets timed with HIP events (median of 5 x 10 launches): hidden (config 4), constant veg / den, flat
altitude, both constant (= config 3's layers). Prints one JSON line. Under `rocprofv3 --pmc GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_BUSY_CYCLES` the same run gives the cycles per variant (launch order = the order below)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def main(E=4096, N=256, K=10, reps=5):
    import torch

    import bench
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    env = AdvancedForestFireBulldozerEnv(N, N, key=2, num_envs=E, use_hidden=True, device=device,
                                         hidden_rng="philox", observation="grid")
    env.reset()
    veg0, den0 = env.vegetation.clone(), env.density.clone()
    alt0 = env.altitude.clone()
    const = torch.full_like(veg0, 3)
    flat = torch.zeros_like(alt0)
    variants = [("hidden (config 4)", veg0, den0, alt0), ("constant veg/den", const, const, alt0),
                ("flat altitude", veg0, den0, flat), ("both constant (config 3 layers)", const, const, flat)]
    out = {"E": E, "N": N, "kernel": "alex_march_kernel" if env.march else "alex_step_kernel<PK>"}
    for name, veg, den, alt in variants:
        env.set_state(vegetation=veg, density=den, altitude=alt)
        times = []
        for _ in range(reps):
            bench.synthetic_state(env, 0, device)
            env.ca_step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                env.ca_step()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / K)
        out[name] = round(sorted(times)[reps // 2], 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
