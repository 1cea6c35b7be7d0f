#!/usr/bin/env python
"""bench.py — BASELINE.json metric: cell-updates/s (+ env-steps/s) of the batched
ForestFireBulldozer CA on 4096 x (256 x 256) grids per MI355X.

Workload (BASELINE config 3): AdvancedForestFireBulldozerEnv,
Alexandridis rule, E = 4096 envs per GPU, N = 256, use_hidden=False (veg = den = 3,
altitude 0 -> p_slope = 1, still read from HBM every step), mid-episode synthetic state
(grid iid {EMPTY .1, TREE .8, FIRE .1}, fire ages iid [1, 672], wind_index iid [0, 8)),
p_tree = 0, p_wind_change = 0.06. One timed step = random actions (device Philox) +
the CA step (gca_alex_step_packed: packed edge-slope layout, 23.1 B/cell moved) + the env step (gca_advenv_post) [+ one RCCL all_gather of the
per-env done mask / reward when --gpus > 1]. Weak scaling: every rank owns E envs.

Also reported: the WindyForestFire bulldozer env (config 2, E = 1024) as `secondary`,
the roofline of the dominant kernel (HIP events over the timed region) and the CPU
baseline (the oracle's C restatement, single core, bounded sample).

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# HBM bytes per Alexandridis cell-update this build moves: grid r+w 2, age r+w 4, veg 1, den 1,
# dousing 1, + slopes: edge layout 4 x f32 = 16 (gca_alex_step_es), 8-plane p_slope 8 x f32 = 32;
# packed env layout (gca_alex_step_packed): veg|den in one byte, dousing 1 bit, edge slopes 16
ALEX_BYTES = {"packed": 23.125, "edge": 25, "planes": 41}
ALEX_BYTES_PER_CELL = 41  # the SURVEY.md §8d figure (8-plane layout), reported alongside
WINDY_BYTES_PER_CELL = 2  # u8 read + u8 write


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    # 20 untimed steps: the first ~15 launches of a fresh process run up to 25% slower (clock / TLB warm-up,
    # profiles/r01l kernel trace), so a short warm-up would fold that ramp into the timed mean
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--gather", choices=["step", "none"], default="step")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--slope-layout", choices=["packed", "edge", "planes"], default="packed")
    ap.add_argument("--tile-skip", action="store_true", help="A/B: headline with the tile activity map on")
    ap.add_argument("--headline-only", action="store_true",
                    help="only the headline loop (no RGB / episode-start loops): every alex_step launch is the "
                         "dense mid-episode one, so rocprofv3 per-kernel averages match kernel_ms")
    return ap.parse_args()


def setup_dist(args):
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    pg = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
        pg = dist
    return world, rank, torch.device("cuda", local), pg


def synthetic_state(env, rank, device):
    """C3 mid-episode state, drawn on the device (Philox for the grid)."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, N = env.num_envs, env.nrows
    cdf = torch.tensor([0.1, 0.9, 1.0], dtype=torch.float32, device=device)
    vals = torch.tensor([0, 1, 2], dtype=torch.uint8, device=device)
    grid = torch.empty((E, N, N), dtype=torch.uint8, device=device)
    call("gca_fill_categorical", dev.ptr(grid), N * N, E, env.env_offset, 1, dev.ptr(cdf), dev.ptr(vals), 3,
         dev.stream_ptr(device))
    gen = torch.Generator(device=device).manual_seed(1000 + rank)
    age = torch.where(grid == 2, torch.randint(1, 673, (E, N, N), device=device, generator=gen, dtype=torch.int16),
                      torch.zeros((), dtype=torch.int16, device=device))
    widx = torch.randint(0, 8, (E,), device=device, generator=gen, dtype=torch.int32)
    env.set_state(grid=grid, fire_age=age, wind_index=widx)


def timed_loop(step_fn, K, W, pg, device):
    import torch

    for _ in range(W):
        step_fn(None)
    torch.cuda.synchronize(device)
    if pg is not None:
        pg.barrier()
    torch.cuda.synchronize(device)
    events = []
    t0 = time.perf_counter()
    for _ in range(K):
        step_fn(events)
    torch.cuda.synchronize(device)
    if pg is not None:
        pg.barrier()
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    kern = [a.elapsed_time(b) * 1e-3 for a, b in events]
    if pg is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        dt = float(t.item())
    return dt, (sum(kern) / len(kern) if kern else None)


def bench_alex(args, world, rank, device, pg):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = args.envs, args.size
    env = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=device,
                                         env_offset=rank * E, slope_layout=args.slope_layout, observation="rgb",
                                         enable_extensions=True, tile_skip=args.tile_skip)
    env.reset()
    synthetic_state(env, rank, device)
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)
    gathered = [torch.empty(E * 5, dtype=torch.uint8, device=device) for _ in range(world)] if world > 1 else None
    st = dev.stream_ptr(device)

    def step(events):
        call("gca_random_actions", dev.ptr(action), E, env.env_offset, 7, dev.ptr(env.rng_step), st)
        if events is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            env.ca_step()
            b.record()
            events.append((a, b))
        else:
            env.ca_step()
        env.post_step(action)
        if gathered is not None and args.gather == "step":
            # RCCL all-gather of the per-env done mask + reward
            payload = torch.cat([env.done, env.reward.view(torch.uint8)])
            pg.all_gather(gathered, payload)

    dt, kern = timed_loop(step, args.steps, args.warmup, pg, device)
    cells = world * E * N * N * args.steps
    res = {
        "value": cells / dt,
        "env_steps_per_s": world * E * args.steps / dt,
        "ms_per_step": dt / args.steps * 1e3,
        "kernel_ms": kern * 1e3,
        "achieved_gbs": ALEX_BYTES[args.slope_layout] * E * N * N / kern / 1e9,
        "survey_equiv_gbs": ALEX_BYTES_PER_CELL * E * N * N / kern / 1e9,
        "fires_left": int((env.counts[:, 2] > 0).sum().item()),
    }
    if args.headline_only:
        return res
    # the full reference env step: + the RGB observation (gca_adv_observation, 12 B/cell of f32 RGB
    # written), extension choice 1 (unblur) in every env
    action3 = torch.zeros((E, 3), dtype=torch.int32, device=device)
    action3[:, 2] = 1

    def step_rgb(events):
        step(None)
        if events is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            env.render_observation(action3)
            b.record()
            events.append((a, b))
        else:
            env.render_observation(action3)

    dt_rgb, kern_rgb = timed_loop(step_rgb, args.steps, args.warmup, pg, device)
    res["with_rgb_observation"] = {"env_steps_per_s": world * E * args.steps / dt_rgb,
                                   "cell_updates_per_s": world * E * N * N * args.steps / dt_rgb,
                                   "obs_kernel_ms": kern_rgb * 1e3,
                                   "obs_gbs": 14 * E * N * N / kern_rgb / 1e9,
                                   "note": "RGB f32 observation per step like the reference's stateless_step"}
    # the same env from its reset state (two burning cells per env, advanced_bulldozer.py:650-688): a
    # real episode's first steps, where the fire-sparsity skip leaves most waves the 7 B/cell of
    # grid/age/dousing traffic. Reported separately; the headline above is the dense mid-episode state.
    env.reset()
    dt_sp, kern_sp = timed_loop(step, args.steps, args.warmup, pg, device)
    res["episode_start"] = {"cell_updates_per_s": world * E * N * N * args.steps / dt_sp,
                            "kernel_ms": kern_sp * 1e3, "state": "reset state (2 fires per env), fire-sparsity skip"}
    # the same episode start with the opt-in tile activity map (tiles without fire nearby copied, not stepped)
    env.set_tile_skip(True)
    env.reset()
    dt_ts, kern_ts = timed_loop(step, args.steps, args.warmup, pg, device)
    res["episode_start"]["tile_skip"] = {"cell_updates_per_s": world * E * N * N * args.steps / dt_ts,
                                         "kernel_ms": kern_ts * 1e3}
    env.set_tile_skip(args.tile_skip)
    return res


def bench_config4(args, world, rank, device, pg):
    """BASELINE config 4: AdvancedBulldozer 256x256 with the hidden foliage / altitude layers
    (use_hidden=True), 4096 envs per GPU. The layers come from the init_utils restatement on a
    seeded legacy stream (same draws as the reference after np.random.seed), altitude arithmetic and
    get_slope on the device; then the same timed step as the headline with a mid-episode state."""
    import numpy as np
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = args.envs, args.size
    t0 = time.perf_counter()
    env = AdvancedForestFireBulldozerEnv(N, N, key=2, num_envs=E, use_hidden=True, device=device,
                                         env_offset=rank * E, hidden_rng=np.random.RandomState(2 + rank),
                                         slope_layout=args.slope_layout)
    torch.cuda.synchronize(device)
    init_s = time.perf_counter() - t0
    env.reset()
    synthetic_state(env, rank, device)
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)
    st = dev.stream_ptr(device)

    def step(events):
        call("gca_random_actions", dev.ptr(action), E, env.env_offset, 13, dev.ptr(env.rng_step), st)
        if events is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            env.ca_step()
            b.record()
            events.append((a, b))
        else:
            env.ca_step()
        env.post_step(action)

    dt, kern = timed_loop(step, args.steps, args.warmup, pg, device)
    out = {"config": "AdvancedBulldozer 256x256, hidden foliage/altitude layers (use_hidden=True), 4096 envs/GPU",
           "cell_updates_per_s": world * E * N * N * args.steps / dt,
           "env_steps_per_s": world * E * args.steps / dt,
           "kernel_ms": kern * 1e3,
           "achieved_gbs": ALEX_BYTES[args.slope_layout] * E * N * N / kern / 1e9,
           "init_s": init_s,
           "init": "patches + altitude draws on the host (legacy np.random order), altitude arithmetic + "
                   "get_slope + exp on the device"}
    del env
    torch.cuda.empty_cache()
    return out


def bench_windy(args, world, rank, device, pg):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    from gymca_amd.graph import StepGraph

    E, N = 1024, 256
    env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=0x5EED, env_offset=rank * E,
                                        materialize_obs=False)
    env.reset()
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)

    def one_step():
        # actions drawn on the device from each env's own counter, then the whole env step
        call("gca_random_actions", dev.ptr(action), E, env.env_offset, 9, dev.ptr(env.rng_step),
             dev.stream_ptr(device))
        env.step(action)

    K = max(args.steps, 40)
    dt_eager, _ = timed_loop(lambda ev: one_step(), K, args.warmup, pg, device)
    # the same steps replayed from one HIP graph per G env steps (no host launch overhead)
    G = 8
    graph = StepGraph(one_step, n_steps=G, device=device)
    Kg = max(K // G, 5)
    dt_env, _ = timed_loop(lambda ev: graph.replay(), Kg, 2, pg, device)
    # CA-only (steps[E] = 1 forced), dense variant {0:.1, 3:.6, 25:.3}
    g = env.grids()
    u = torch.rand(g.shape, device=device)
    g = torch.where(u < 0.1, 0, torch.where(u < 0.7, 3, 25)).to(torch.uint8)
    env.buf[0].copy_(g)
    env.parity.zero_()
    env.dir_mask.copy_(torch.randint(0, 256, (E,), dtype=torch.uint8, device=device))

    def ca_step(events):
        if events is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            env.ca_step_all()
            b.record()
            events.append((a, b))
        else:
            env.ca_step_all()

    dt_ca, kern = timed_loop(ca_step, K, args.warmup, pg, device)
    # the same-size ceiling: a device copy of the CA's bytes (E x H x W in, the same out) on this GPU
    src = torch.empty(E * N * N, dtype=torch.uint8, device=device)
    dst = torch.empty_like(src)

    def copy_step(events):
        if events is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            dst.copy_(src)
            b.record()
            events.append((a, b))
        else:
            dst.copy_(src)

    _, kern_copy = timed_loop(copy_step, K, args.warmup, pg, device)
    del src, dst
    return {
        "config": "ForestFireBulldozer 256x256, 1024 envs/GPU, WindyForestFire",
        "env_steps_per_s": world * E * Kg * G / dt_env,
        "env_steps_per_s_eager": world * E * K / dt_eager,
        "env_step_graph": f"hipGraph of {G} env steps (random actions + RepeatCA/Windy passes + Move/Modify + reward)",
        "ca_only_cell_updates_per_s": world * E * N * N * K / dt_ca,
        "ca_kernel_ms": kern * 1e3,
        "ca_achieved_gbs": WINDY_BYTES_PER_CELL * E * N * N / kern / 1e9,
        "ca_roofline_frac": WINDY_BYTES_PER_CELL * E * N * N / kern / 1e9 / HBM_PEAK_GBS,
        "same_size_copy_ms": kern_copy * 1e3,
        "ca_frac_of_same_size_copy": kern_copy / kern,
    }


def bench_windy512(args, world, rank, device, pg):
    """BASELINE config 5: ForestFireBulldozer 512x512, 1024 envs per GPU (8192 over 8 GPUs), with the
    RCCL all-gather of the per-env done mask + reward (9 B/env) over xGMI — per env step (eager) and
    per 8-step rollout segment (HIP-graph replay of the 8 steps, then one gather)."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv
    from gymca_amd.graph import StepGraph

    E, N = 1024, 512
    env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=0x5EED5, env_offset=rank * E,
                                        materialize_obs=False)
    env.reset()
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)
    gathered = [torch.empty(E * 9, dtype=torch.uint8, device=device) for _ in range(world)] if world > 1 else None

    def one_step():
        call("gca_random_actions", dev.ptr(action), E, env.env_offset, 11, dev.ptr(env.rng_step),
             dev.stream_ptr(device))
        env.step(action)

    def gather():
        if gathered is not None:
            pg.all_gather(gathered, torch.cat([env.done, env.reward.view(torch.uint8)]))

    K = max(args.steps, 40)

    def eager(ev):
        one_step()
        gather()

    dt_eager, _ = timed_loop(eager, K, args.warmup, pg, device)
    G = 8
    graph = StepGraph(one_step, n_steps=G, device=device)

    def seg(ev):
        graph.replay()
        gather()

    Kg = max(K // G, 5)
    dt_g, _ = timed_loop(seg, Kg, 2, pg, device)
    return {"config": "ForestFireBulldozer 512x512, 1024 envs/GPU (BASELINE config 5 at 8 GPUs), WindyForestFire",
            "env_steps_per_s": world * E * Kg * G / dt_g,
            "env_steps_per_s_eager_gather_every_step": world * E * K / dt_eager,
            "gather": "RCCL all_gather of done u8 + reward f64 per env" if world > 1 else "none (1 GPU)"}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_threads():
    """Host cores this process may use, capped at 16 (the GPU box's per-job CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _alex_cpu_rate(args, threads, seconds):
    """cell-updates/s of the oracle's C restatement, `threads` workers x 8 envs each (ctypes releases
    the GIL during the call, so the threads run in parallel; no process is forked)."""
    import threading

    import numpy as np

    from gymca_amd.forest_fire.bulldozer.init_utils import get_winds
    from gymca_amd.forest_fire.operators.ca_alexandridis import make_alex_params
    from oracle import alex_c

    N, Es = args.size, 8
    p, _ = make_alex_params(N, 0, 1, 2, np.asarray(get_winds(False), np.float32), 0.0, 1)
    alex_c.lib()
    done = [0] * threads

    def worker(t):
        rng = np.random.default_rng(1 + t)
        grid = rng.choice(np.array([0, 1, 2], np.uint8), size=(Es, N, N), p=[0.1, 0.8, 0.1])
        age = np.where(grid == 2, rng.integers(1, 673, (Es, N, N)), 0).astype(np.int16)
        three = np.full((Es, N, N), 3, np.uint8)
        dous = np.zeros((Es, N, N), np.uint8)
        ps = np.ones((Es, 8, N, N), np.float32)
        widx = rng.integers(0, 8, Es).astype(np.int32)
        barrier.wait()
        t0, steps = time.perf_counter(), 0
        while time.perf_counter() - t0 < seconds:
            grid, age, _, _ = alex_c.alex_step(p, grid, age, three, three, dous, ps, widx,
                                               rng_step=np.full(Es, steps, np.uint32))
            steps += 1
        done[t] = steps

    barrier = threading.Barrier(threads + 1)
    pool = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for th in pool:
        th.start()
    barrier.wait()
    t0 = time.perf_counter()
    for th in pool:
        th.join()
    dt = time.perf_counter() - t0
    return Es * N * N * sum(done) / dt, sum(done)


def cpu_baseline(args):
    """The oracle's C restatement of the Alexandridis step on the GPU host's cores, bounded sample:
    (i) one core, (ii) every core this job may use (BASELINE.md CPU-baseline plan)."""
    threads = _cpu_threads()
    single, s1 = _alex_cpu_rate(args, 1, args.cpu_seconds / 2)
    multi, sm = _alex_cpu_rate(args, threads, args.cpu_seconds / 2)
    return {"value": multi, "unit": "cell-updates/s", "cores": threads, "kind": "port",
            "sample": f"{threads} threads x 8 envs x {args.size}x{args.size}, {sm} env-batches of Alexandridis steps "
                      f"in {args.cpu_seconds / 2:.0f} s; oracle/gca_oracle.c (gcc -O2), the reference's JAX path "
                      f"cannot run here", "single_core_value": single, "cpu_model": _cpu_model()}


def windy_cpu_baseline(seconds=3.0):
    """The reference algorithm for WindyForestFire (scipy convolve2d + the three threshold masks,
    oracle/windy.py) on one core, 256x256, with the bulldozer env's full-grid cell count per step."""
    import numpy as np

    from gymca_amd.forest_fire.bulldozer.bulldozer import DEFAULT_WIND, parse_wind
    from oracle import windy as owindy

    rng = np.random.default_rng(5)
    grid = rng.choice(np.array([0, 3, 25]), size=(256, 256), p=[0.1, 0.6, 0.3])
    wind = parse_wind(DEFAULT_WIND)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        grid = owindy.windy_step(grid, wind, rng.random((3, 3)))
        np.unique(grid, return_counts=True)
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": 256 * 256 * steps / dt, "unit": "cell-updates/s", "cores": 1, "kind": "port",
            "sample": f"1 env 256x256, {steps} steps of the scipy restatement + cell count"}


def measured_traffic(args):
    """HBM bytes per alex_step launch from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by scripts/pmc_summary.py: 2*FETCH_SIZE + WRITE_SIZE,
    gfx950 correction) — only when this run is the profiled workload."""
    if args.envs != 4096 or args.size != 256:
        return None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        data = json.load(open(tf))
    except (ValueError, OSError):
        return None
    want = {"packed": "alex_step<6, 0, true, true, true>", "edge": "alex_step<6, 0, true, true, false>",
            "planes": "alex_step<6, 0, true, false, false>"}[args.slope_layout]
    for k, v in data.items():  # the Philox-mode FAST kernel at R = 6 (N = 256) of this slope layout
        if k == want:
            return v.get("bytes_per_launch")
    return None


def copy_bandwidth(device, nbytes=2 << 30, reps=10):
    """Live device-to-device copy rate (GB/s, read + write) of torch's copy kernel on this GPU, reported
    beside the 8 TB/s spec (SURVEY.md §8d asks for both). It is a lower bound on the practical ceiling:
    scripts/bw_probe.hip measures the alex_step access pattern itself."""
    import torch

    a = torch.empty(nbytes, dtype=torch.uint8, device=device)
    b = torch.empty_like(a)
    b.copy_(a)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        b.copy_(a)
    e.record()
    e.synchronize()
    gbs = 2.0 * nbytes * reps / (s.elapsed_time(e) * 1e-3) / 1e9
    del a, b
    return gbs


def main():
    args = parse()
    world, rank, device, pg = setup_dist(args)
    import torch

    alex = bench_alex(args, world, rank, device, pg)
    import gc

    gc.collect()
    torch.cuda.empty_cache()
    config4 = None if args.no_secondary else bench_config4(args, world, rank, device, pg)
    secondary = None if args.no_secondary else bench_windy(args, world, rank, device, pg)
    config5 = None if args.no_secondary else bench_windy512(args, world, rank, device, pg)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
        if secondary is not None:
            secondary["cpu_baseline"] = windy_cpu_baseline()
    traffic = measured_traffic(args)
    copy_gbs = copy_bandwidth(device)
    if rank == 0:
        out = {
            "metric": "cell-updates/sec, 4096x(256x256) ForestFireBulldozer (Alexandridis CA), per-GPU batch",
            "value": alex["value"],
            "unit": "cell-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": alex["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8 cells / i16 ages / f32 probabilities",
            "data": "synthetic (device Philox mid-episode state, SURVEY.md §8d C3)",
            "config": {"workload": "AdvancedForestFireBulldozer 256x256, 4096 envs/GPU, Alexandridis rule, "
                                   "use_hidden=False (BASELINE config 3)",
                       "envs_per_gpu": args.envs, "grid": [args.size, args.size],
                       "parallelism": f"env-sharded x{world}" + (", RCCL all_gather done/reward per step"
                                                                  if world > 1 and args.gather == "step" else "")},
            "env_steps_per_s": alex["env_steps_per_s"],
            "episode_start": alex.get("episode_start"),
            "with_rgb_observation": alex.get("with_rgb_observation"),
            # achieved = SURVEY.md §8d's algorithmic figure (41 B per cell-update, "independent of the build's
            # actual layout") x cells / the kernel's mean launch time; the bytes this build actually moves
            # (edge-slope layout: 25 B/cell) and the PMC traffic are reported beside it
            "roofline": {"bound": "hbm", "achieved": alex["survey_equiv_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alex["survey_equiv_gbs"] / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "alex_step_kernel" + {"packed": "<ES, PK>", "edge": "<ES>", "planes": ""}[args.slope_layout],
                         "kernel_ms": alex["kernel_ms"],
                         "algorithmic_bytes_per_cell": ALEX_BYTES_PER_CELL,
                         "slope_layout": args.slope_layout,
                         "moved_bytes_per_cell": ALEX_BYTES[args.slope_layout],
                         "moved_gbs": alex["achieved_gbs"],
                         "moved_frac": alex["achieved_gbs"] / HBM_PEAK_GBS,
                         "traffic_bytes_per_cell": traffic / (args.envs * args.size * args.size) if traffic else None,
                         "device_copy_gbs": copy_gbs,
                         "moved_frac_of_device_copy": alex["achieved_gbs"] / copy_gbs},
            "cpu_baseline": cpu,
            "secondary": secondary,
            "config4": config4,
            "config5": config5,
        }
        print(json.dumps(out))
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
