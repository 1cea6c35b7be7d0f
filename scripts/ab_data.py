#!/usr/bin/env python3
"""Data-dependence probe of the packed Alexandridis step (one GPU): the same C3 state and launch with
the slope / vegetation-density layers constant (C3: slope 0 -> every V = 1.0f, veg = den = 3) or random
(C4-like values), plus a same-size device copy of constant vs random bytes. Identical instructions and
byte counts; only the values differ. Also: the write-only rate of a fill of the RGB observation's size
(the ceiling of the store-bound observation kernel).

    python scripts/ab_data.py > gpurun_out/ab_data.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-cellular-automata_amd"))

K, W = 40, 20


def timed(fn, before=None):
    import torch

    ms = []
    for i in range(W + K):
        if before is not None:
            before()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        if i >= W:
            ms.append(s.elapsed_time(e))
    return round(sum(ms) / len(ms), 4)


def main():
    import torch

    import bench
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    dev = torch.device("cuda:0")
    E, N = 4096, 256
    env = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=dev, slope_layout="packed")
    env.reset()
    bench.synthetic_state(env, 0, dev)
    g0, a0 = env.grid[env.cur].clone(), env.age[env.cur].clone()
    const_slope, const_vd = env.slope_data.clone(), env.vd.clone()
    gen = torch.Generator(device=dev).manual_seed(7)
    a = (torch.rand(const_slope.shape, device=dev, generator=gen) * 2 - 1) * 3.0
    rand_slope = torch.sign(a) * torch.exp(a.abs())
    del a
    v = torch.randint(1, 6, const_vd.shape, device=dev, generator=gen, dtype=torch.uint8)
    d = torch.randint(1, 6, const_vd.shape, device=dev, generator=gen, dtype=torch.uint8)
    rand_vd = v | (d << 4)

    def restore():
        env.grid[env.cur].copy_(g0)
        env.age[env.cur].copy_(a0)

    def step():
        env.ca_step()
        env.cur ^= 1  # undo the flip so every launch steps the same state

    out = {}
    for rep in range(2):
        for name, sl, vd in (("const", const_slope, const_vd), ("rand_slope", rand_slope, const_vd),
                             ("rand_vd", const_slope, rand_vd), ("rand_both", rand_slope, rand_vd)):
            env.slope_data.copy_(sl)
            env.vd.copy_(vd)
            env.refresh_terrain()  # "const" runs the flat-terrain / uniform-layers step since r06
            out.setdefault(name + "_ms", []).append(timed(step, restore))
            print(name, out[name + "_ms"][-1], file=sys.stderr, flush=True)
    dst = torch.empty_like(const_slope)
    out["copy_const_slope_ms"] = timed(lambda: dst.copy_(const_slope))
    out["copy_rand_slope_ms"] = timed(lambda: dst.copy_(rand_slope))
    out["slope_bytes"] = const_slope.numel() * 4
    del dst, rand_slope, const_slope
    rgb = torch.empty((E, N, N, 3), dtype=torch.float32, device=dev)
    out["fill_rgb_ms"] = timed(lambda: rgb.fill_(0.5))
    out["rgb_bytes"] = rgb.numel() * 4
    print(json.dumps(out))


if __name__ == "__main__":
    main()
