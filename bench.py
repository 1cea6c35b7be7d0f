#!/usr/bin/env python
"""bench.py — BASELINE.json metric: cell-updates/s (+ env-steps/s) of the batched
ForestFireBulldozer CA on 4096 x (256 x 256) grids per MI355X.

Workload (BASELINE config 3): AdvancedForestFireBulldozerEnv,
Alexandridis rule, E = 4096 envs per GPU, N = 256, use_hidden=False (veg = den = 3,
altitude 0 -> p_slope = 1, still read from HBM every step), mid-episode synthetic state
(grid iid {EMPTY .1, TREE .8, FIRE .1}, fire ages iid [1, 672], wind_index iid [0, 8)),
p_tree = 0, p_wind_change = 0.06. One timed step = random actions (device Philox) +
the CA step (gca_alex_step_march at 256^2: packed edge-slope layout, 23.1 B/cell moved; gca_alex_step_packed
with --step-kernel tiled) + the env step (gca_advenv_post) [+ one RCCL all_gather of the
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
# packed env layout (gca_alex_step_march / _packed): veg|den in one byte, dousing 1 bit, edge slopes 16
ALEX_BYTES = {"packed": 23.125, "edge": 25, "planes": 41}
SLOPE_PLANE_BYTES = 16  # 4 edge planes of f32 per cell, not read by the flat-terrain marching step
VD_BYTES = 1  # the packed vegetation / density byte, not read by the uniform-layers step


def alex_bytes(env, layout):
    """Algorithmic bytes per cell-update of the step env.ca_step() launches: the layout's, minus the slope planes when
    the marching step runs on flat terrain (edge_slope = NULL: 7.125 B) and the vd layer when the layers are uniform
    too (vd = NULL: 6.125 B)."""
    flat = getattr(env, "march", False) and getattr(env, "flat_terrain", False)
    uni = flat and getattr(env, "uniform_layers", False)
    return ALEX_BYTES[layout] - (SLOPE_PLANE_BYTES if flat else 0) - (VD_BYTES if uni else 0)
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
    ap.add_argument("--gather", choices=["async", "step", "none"], default="async",
                    help="N > 1: the per-step RCCL all-gather of the episode stats on a side stream overlapping the "
                         "next step (async), inline (step), or none")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--slope-layout", choices=["packed", "edge", "planes"], default="packed")
    ap.add_argument("--tile-skip", action="store_true", help="A/B: headline with the tile activity map on")
    ap.add_argument("--step-kernel", choices=["auto", "march", "tiled"], default="auto",
                    help="packed layout at W = 256: the marching kernel (auto) or the tiled one")
    ap.add_argument("--headline-only", action="store_true",
                    help="only the headline loop (no RGB / episode-start loops): every alex_step launch is the "
                         "dense mid-episode one, so rocprofv3 per-kernel averages match kernel_ms")
    ap.add_argument("--reps", type=int, default=5, help="timed repetitions of K steps; the median is reported")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the N-rank launch: gloo ranks, env sharding and the episode-stats "
                         "all-gather of gymca_amd.distributed, no GPU touched")
    return ap.parse_args()


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


CPU_JSON_ENV = "GCA_BENCH_CPU_JSON"  # launch_ranks -> rank 0: the CPU legs' results (a temp-file path)


def launch_ranks(args):
    """`bench.py --gpus N` started as a plain process: run the CPU baseline legs here (this process never touches the
    GPU, so the all-core leg may fork), hand them to rank 0 through a temp file (CPU_JSON_ENV), then run N ranks (one
    per GPU) as CHILD processes through torch.distributed.run and return their exit code (no exec)."""
    import subprocess
    import tempfile

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC on this pool
    env.setdefault("OMP_NUM_THREADS", "1")
    tmp = None
    if not args.no_cpu_baseline:
        fd, tmp = tempfile.mkstemp(prefix="gca_bench_cpu_", suffix=".json")
        with os.fdopen(fd, "w") as fh:
            json.dump(run_cpu_legs(args), fh)
        env[CPU_JSON_ENV] = tmp
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    try:
        return subprocess.call(cmd, env=env)
    finally:
        if tmp is not None:
            os.unlink(tmp)


def cpu_legs_for_rank0(args, rank):
    """Rank 0's CPU baseline at any world size (VERDICT r04 missing 3): the legs launch_ranks ran before spawning the
    ranks, or -- launched by an outer torch.distributed.run -- run here, before this process touches the GPU (the
    other ranks wait in the process-group rendezvous meanwhile). None on other ranks or with --no-cpu-baseline."""
    if rank != 0 or args.no_cpu_baseline:
        return None
    path = os.environ.get(CPU_JSON_ENV)
    if path:
        with open(path) as fh:
            legs = json.load(fh)
        legs["alex"]["measured_by"] = "the launching parent process, before the ranks started"
        return legs
    legs = run_cpu_legs(args)
    legs["alex"]["measured_by"] = "rank 0, before it initialised the GPU"
    return legs


def setup_dist(args):
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}: launch N ranks with "
                         f"torch.distributed.run or plain `python bench.py --gpus N`")
    torch.cuda.set_device(local)
    pg = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus
        pg = dist
    return world, rank, torch.device("cuda", local), pg


def dry_run(args):
    """The distributed plumbing of the bench on CPU (gloo): each rank takes its env shard of the global batch
    (gymca_amd.distributed.shard), fills its per-env episode stats from its GLOBAL env ids, all-gathers them
    with the bench's own gather (distributed.all_gather_stats) and checks the gathered rank order."""
    import torch
    import torch.distributed as dist

    from gymca_amd import distributed as gd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--dry-run --gpus {args.gpus} but WORLD_SIZE={world}")
    cpu_legs = cpu_legs_for_rank0(args, rank)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    total = args.envs * world
    off, cnt = gd.shard(total, world, rank)
    gid = torch.arange(off, off + cnt)
    done = (gid % 3 == 0).to(torch.uint8)
    ret = -gid.to(torch.float32) / 8
    length = gid.to(torch.int32) + 1
    stats = gd.StatsGather(cnt, "cpu")  # the bench's own gather (bench_alex), on gloo
    d, r, ln = (x.reshape(-1) for x in stats.gather(done, ret, length))
    allid = torch.arange(total)
    ok = (torch.equal(d, (allid % 3 == 0).to(torch.uint8)) and torch.equal(r, -allid.to(torch.float32) / 8)
          and torch.equal(ln, allid.to(torch.int32) + 1))
    check = gd.verify_gather(stats)  # the same self-check the real N-rank path reports
    oks = [None] * world
    if world > 1:
        dist.all_gather_object(oks, (rank, off, cnt, bool(ok)))
    else:
        oks = [(rank, off, cnt, bool(ok))]
    all_ok = all(o for *_, o in oks) and (check is None or check["gather_ok"])
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "n_gpus": world, "backend": "gloo" if world > 1 else "none",
                          "dry_run": True, "ranks": [{"rank": a, "env_offset": b, "envs": c, "gather_ok": o}
                                                     for a, b, c, o in oks],
                          "gather_ok": all_ok,
                          "gather_check": check,
                          "rccl_world": None if check is None else check["world_seen"],
                          "cpu_baseline": None if cpu_legs is None else cpu_legs["alex"],
                          "cpu_legs": cpu_legs}))
    if world > 1:
        dist.destroy_process_group()
    return 0 if all_ok else 1


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


def env_snapshot(env, step_fn, n_steps):
    """A `prepare` for timed_loop: the env's state after reset + `n_steps` untimed steps of `step_fn` (every env well
    into its episode, the RepeatCA accumulators spread out as in a long run), saved once (a copy of every tensor
    attribute of the env) and restored in place before each loop / repetition, so every figure of a section times the
    same steps from the same mid-episode state."""
    import torch

    env.reset()
    for _ in range(n_steps):
        step_fn()
    saved = {k: v.clone() for k, v in vars(env).items() if isinstance(v, torch.Tensor)}

    def restore():
        for k, v in saved.items():
            getattr(env, k).copy_(v)

    return restore


def timed_loop(step_fn, K, W, pg, device, reps=1, detail=None, prepare=None):
    """W untimed steps, then `reps` repetitions of EXACTLY K steps, each bracketed by barrier + synchronize on
    both sides, max over ranks. Returns (median seconds per K steps, mean kernel seconds from the events
    step_fn records). `prepare` (optional) restores the workload's starting state before the warm-up and
    before every repetition (untimed), so each repetition times the same K steps of the workload rather than
    an ever later stretch of one trajectory. `detail` (dict, optional) receives every repetition's ms per step."""
    import torch

    if prepare is not None:
        prepare()
    for _ in range(W):
        step_fn(None)
    events, dts, per_rank = [], [], []
    for _ in range(max(1, reps)):
        if prepare is not None:
            prepare()
        torch.cuda.synchronize(device)
        if pg is not None:
            pg.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(K):
            step_fn(events)
        torch.cuda.synchronize(device)
        if pg is not None:
            pg.barrier()
        torch.cuda.synchronize(device)
        dt = time.perf_counter() - t0
        if pg is not None:  # every rank's own time (one-hot rows summed), the job's time = the max over ranks
            t = torch.zeros(pg.get_world_size(), dtype=torch.float64, device=device)
            t[pg.get_rank()] = dt
            pg.all_reduce(t)
            per_rank.append(t.tolist())
            dt = float(t.max().item())
        dts.append(dt)
    kern = [a.elapsed_time(b) * 1e-3 for a, b in events]
    med = sorted(dts)[len(dts) // 2]
    if detail is not None:
        detail["reps_ms_per_step"] = [d / K * 1e3 for d in dts]
        detail["median_of"] = len(dts)
        if per_rank:  # the median repetition's per-rank ms per step
            detail["per_rank_ms_per_step"] = [x / K * 1e3 for x in per_rank[dts.index(med)]]
    return med, (sum(kern) / len(kern) if kern else None)


def bench_alex(args, world, rank, device, pg):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = args.envs, args.size
    env = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=device,
                                         env_offset=rank * E, slope_layout=args.slope_layout, observation="rgb",
                                         enable_extensions=False, tile_skip=args.tile_skip,
                                         step_kernel=args.step_kernel if args.slope_layout == "packed" else "auto")
    env.reset()
    synthetic_state(env, rank, device)
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)
    st = dev.stream_ptr(device)
    from gymca_amd import distributed as gd

    stats = gd.StatsGather(E, device, group=None, len_dtype=torch.float32) if world > 1 else None

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
        env.post_step(action, stats=True)  # + info steps_elapsed / reward_accumulated, fused
        if stats is not None and args.gather != "none":
            # RCCL all-gather of the per-env episode stats (return f32 | length f32 | done u8): one
            # pack + one all_gather_into_tensor into a reused buffer, on a side stream under the next step (async)
            stats.gather(env.done, env.reward_accumulated, env.steps_elapsed, async_op=args.gather == "async")

    detail = {}
    prep = lambda: synthetic_state(env, rank, device)  # every repetition times K steps from the C3 state
    dt, kern = timed_loop(step, args.steps, args.warmup, pg, device, reps=args.reps, detail=detail, prepare=prep)
    cells = world * E * N * N * args.steps
    nbytes = alex_bytes(env, args.slope_layout)
    res = {
        "value": cells / dt,
        "env_steps_per_s": world * E * args.steps / dt,
        "ms_per_step": dt / args.steps * 1e3,
        "kernel_ms": kern * 1e3,
        "bytes_per_cell": nbytes,
        "terrain": ("general" if nbytes == ALEX_BYTES[args.slope_layout] else
                    "flat, uniform layers" if getattr(env, "uniform_layers", False) else "flat"),
        "achieved_gbs": nbytes * E * N * N / kern / 1e9,
        "survey_equiv_gbs": ALEX_BYTES_PER_CELL * E * N * N / kern / 1e9,
        "fires_left": int((env.counts[:, 2] > 0).sum().item()),
        "timing": detail,
        "kernel": ("alex_march_kernel" if getattr(env, "march", False) else
                   "alex_step_kernel" + {"packed": "<ES, PK>", "edge": "<ES>", "planes": ""}[args.slope_layout]),
        "kernel_key": headline_kernel_key(env),
        # N > 1: the last timed gather checked against every rank's payload over the group (None at N = 1)
        "gather_check": gd.verify_gather(stats) if args.gather != "none" else None,
    }
    if getattr(env, "march", False) and rank == 0:
        res["tiled_kernel_ms"] = tiled_kernel_ms(env, device)
    res["pattern_floor_ms"] = march_pattern_ms(env, device)
    if res["terrain"] != "general":
        # the same steps with the slope planes streamed (the step every terrain takes; all factors 1 here): the general
        # kernel's figures, the headline of rounds 1-6 before the flat-terrain step
        env.flat_terrain = False
        dt_g, kern_g = timed_loop(step, args.steps, args.warmup, pg, device, reps=3, prepare=prep)
        res["general_terrain"] = {
            "cell_updates_per_s": cells / dt_g, "ms_per_step": dt_g / args.steps * 1e3, "kernel_ms": kern_g * 1e3,
            "kernel_key": headline_kernel_key(env), "bytes_per_cell": ALEX_BYTES[args.slope_layout],
            "achieved_gbs": ALEX_BYTES[args.slope_layout] * E * N * N / kern_g / 1e9,
            "frac": ALEX_BYTES[args.slope_layout] * E * N * N / kern_g / 1e9 / HBM_PEAK_GBS,
            "pattern_floor_ms": march_pattern_ms(env, device),
            "note": "gca_alex_step_march reading the env's edge planes (every value 1.0): the step of any terrain "
                    "(config 4's hidden layers take it)"}
        env.refresh_terrain()
    if args.headline_only:
        return res
    # the full reference env step: + the RGB observation of stateless_step (advanced_bulldozer.py:1120). The reference's
    # default env (enable_extensions=False) gets it from the CA step's own epilogue (gca_alex_step_march_rgb: 12 B/cell
    # of f32 RGB written, no second pass) + the bulldozer's pixel (gca_obs_position)
    fused = env.fused_observation  # the packed layout (the default); --slope-layout edge / planes: its own pass

    def step_rgb(events):
        call("gca_random_actions", dev.ptr(action), E, env.env_offset, 7, dev.ptr(env.rng_step), st)
        if events is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            env.ca_step(render=fused)
            b.record()
            events.append((a, b))
        else:
            env.ca_step(render=fused)
        env.post_step(action, stats=True)
        if fused:
            env.finish_frame()  # the bulldozer's pixel (gca_obs_position)
        else:
            env.render_observation(None)

    dt_rgb, kern_rgb = timed_loop(step_rgb, args.steps, args.warmup, pg, device, reps=3, prepare=prep)

    def step_fill(events):  # the headline loop with a write-only fill_ of the RGB buffer beside it
        step(None)
        if events is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            env.rgb.fill_(0.5)
            b.record()
            events.append((a, b))
        else:
            env.rgb.fill_(0.5)

    _, kern_fill = timed_loop(step_fill, args.steps, args.warmup, pg, device, reps=1, prepare=prep)
    # the extension pipeline (enable_extensions=True, which also sets should_transform_grid, advanced_bulldozer.py:293-302;
    # extension choice 1 = unblur in every env): at W = 256 the frame comes from the CA step's epilogue too
    # (gca_alex_step_march_rgb_ext: the display is the grid while row 0 holds a TREE / FIRE, checked per env; envs whose
    # check fails are re-rendered by gca_adv_observation with env_mask = refit), else its own pass (14 B/cell)
    from gymca_amd.forest_fire.bulldozer.observation import make_obs_params

    plain_params, plain_ext = env.obs_params, env.enable_extensions
    env.obs_params = make_obs_params(0, 1, 2, True, True, env._day_length)
    env.enable_extensions = True
    fused_ext = env.fused_observation
    action3 = torch.zeros((E, 3), dtype=torch.int32, device=device)
    action3[:, 2] = 1

    def make_step_ext(acts, fused_path, mixed):
        def step_ext(events):
            call("gca_random_actions", dev.ptr(action), E, env.env_offset, 7, dev.ptr(env.rng_step), st)
            if mixed:  # a uniform extension choice per env and step (0 none, 1 unblur, 2 see-invisible-fires)
                torch.remainder(action[:, 0], 3, out=acts[:, 2])
            if events is not None:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
            if fused_path:
                env.ca_step(render=True, action=acts)
                env.post_step(action, stats=True)
                env.finish_frame(acts)
            else:
                env.ca_step()
                env.post_step(action, stats=True)
                env.render_observation(acts)
            if events is not None:  # both paths: CA step + env step + the whole frame (refits and pixel included)
                b.record()
                events.append((a, b))
        return step_ext

    dt_ext, kern_ext = timed_loop(make_step_ext(action3, fused_ext, False), args.steps, args.warmup, pg, device, reps=3,
                                  prepare=prep)
    refits = int(env._refit.sum().item()) if fused_ext else None
    # a policy mixing the three extension choices (choice 0 leaves the blurred base grid to the refit pass)
    # through the fused path and through the separate-pass path, the same steps
    action3m = action3.clone()
    mixed = {}
    for name, fp in ((("fused", True),) if fused_ext else ()) + (("separate_pass", False),):
        dtm, km = timed_loop(make_step_ext(action3m, fp, True), args.steps, args.warmup, pg, device, reps=3,
                             prepare=prep)
        mixed[name] = {"env_steps_per_s": world * E * args.steps / dtm, "ms_per_step": dtm / args.steps * 1e3,
                       "step_and_frame_kernels_ms": km * 1e3}
        if fp:
            mixed[name]["refit_envs_last_step"] = int(env._refit.sum().item())
    pattern_frame = march_pattern_ms(env, device, frame=True) if fused else None
    env.obs_params, env.enable_extensions = plain_params, plain_ext
    res["with_rgb_observation"] = {"env_steps_per_s": world * E * args.steps / dt_rgb,
                                   "cell_updates_per_s": world * E * N * N * args.steps / dt_rgb,
                                   "ms_per_step": dt_rgb / args.steps * 1e3,
                                   "fused": fused,
                                   "step_and_frame_kernels_ms": kern_rgb * 1e3,
                                   "observation_cost_ms": (kern_rgb - kern) * 1e3,
                                   "same_buffer_fill_ms": kern_fill * 1e3,
                                   "pattern_floor_ms": pattern_frame,
                                   "kernel_over_pattern_floor": (kern_rgb * 1e3 / pattern_frame
                                                                 if pattern_frame else None),
                                   "note": "the reference's default env step (stateless_step renders RGB f32, "
                                           "enable_extensions=False): the frame from the CA step's epilogue"}
    res["with_rgb_observation_extensions"] = {
        "env_steps_per_s": world * E * args.steps / dt_ext,
        "ms_per_step": dt_ext / args.steps * 1e3,
        "fused": fused_ext,
        ("step_and_frame_kernels_ms" if fused_ext else "step_and_separate_frame_ms"): kern_ext * 1e3,
        "refit_envs_last_step": refits,
        "mixed_choice_policy": mixed,
        "note": ("enable_extensions=True, unblur chosen: the frame from the CA step's epilogue "
                 "(gca_alex_step_march_rgb_ext), refit envs by gca_adv_observation after the env step" if fused_ext else
                 "enable_extensions=True, unblur chosen: its own pass (gca_adv_observation)")}
    # the same env from its reset state (two burning cells per env, advanced_bulldozer.py:650-688): a
    # real episode's first steps, where the fire-sparsity skip leaves most waves the 7 B/cell of
    # grid/age/dousing traffic. Reported separately; the headline above is the dense mid-episode state.
    dt_sp, kern_sp = timed_loop(step, args.steps, args.warmup, pg, device, reps=3, prepare=env.reset)
    res["episode_start"] = {"cell_updates_per_s": world * E * N * N * args.steps / dt_sp,
                            "kernel_ms": kern_sp * 1e3,
                            "state": "reset state (2 fires per env): tiles with no FIRE nearby copied (found from the "
                                     "grid), fire-sparsity skip elsewhere"}
    return res


def bench_config4(args, world, rank, device, pg):
    """BASELINE config 4: AdvancedBulldozer 256x256 with the hidden foliage / altitude layers
    (use_hidden=True), 4096 envs per GPU. The layers follow init_utils.py:10-116's recipe drawn on the device
    (hidden_rng="philox", gca_hidden_init; the np.random-stream restatement is the env's default and takes
    seconds at this size), altitude arithmetic and get_slope on the device; then the same timed step as the
    headline from the same mid-episode state."""
    import numpy as np
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = args.envs, args.size
    t0 = time.perf_counter()
    env = AdvancedForestFireBulldozerEnv(N, N, key=2, num_envs=E, use_hidden=True, device=device,
                                         env_offset=rank * E, hidden_rng="philox", observation="grid",
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

    dt, kern = timed_loop(step, args.steps, args.warmup, pg, device, reps=3,
                          prepare=lambda: synthetic_state(env, rank, device))
    out = {"config": "AdvancedBulldozer 256x256, hidden foliage/altitude layers (use_hidden=True), 4096 envs/GPU",
           "cell_updates_per_s": world * E * N * N * args.steps / dt,
           "env_steps_per_s": world * E * args.steps / dt,
           "kernel_ms": kern * 1e3,
           "achieved_gbs": alex_bytes(env, args.slope_layout) * E * N * N / kern / 1e9,
           "init_s": init_s,
           "init": "hidden_rng='philox': patches, zero fill, noise, hills and slopes drawn on the device "
                   "(gca_hidden_init, keyed by global env id), altitude arithmetic + get_slope + exp on the device"}
    del env
    torch.cuda.empty_cache()
    return out


def bench_windy(args, world, rank, device, pg):
    import torch

    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    from gymca_amd.graph import StepGraph

    E, N = 1024, 256
    env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=0x5EED, env_offset=rank * E,
                                        materialize_obs=False)
    env.reset()
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)

    def one_step():
        # actions drawn on the device from each env's own counter (gca_random_actions), then the whole env step
        env.step(env.sample_actions(action, 9))

    K = max(args.steps, 40)
    # every loop starts from the same mid-episode state (reset + 64 steps, restored in place), so the eager and graph
    # figures time the same stretch of the same trajectories
    G = 8
    Kg = max(K // G, 5)
    restore = env_snapshot(env, one_step, 64)
    dt_eager, _ = timed_loop(lambda ev: one_step(), Kg * G, 0, pg, device, reps=3, prepare=restore)
    # the same steps with the random policy's draw inside the env step (gca_bulldozer_step_fused_random: the same
    # actions bit for bit, one launch per env step instead of two)
    dt_rand, _ = timed_loop(lambda ev: env.step_random(9, action), Kg * G, 0, pg, device, reps=3, prepare=restore)
    # the same steps replayed from HIP graphs (no host launch overhead): G = 8 steps of (sample, step) — two nodes per
    # env step — and step_random (one node per env step) in graphs of 8 and 32 steps
    graphs = {}
    for name, fn, g_steps in (("sample_step_g8", one_step, G), ("step_random_g8", lambda: env.step_random(9, action), 8),
                              ("step_random_g32", lambda: env.step_random(9, action), 32)):
        restore()
        graph = StepGraph(fn, n_steps=g_steps, device=device)
        reps_g = max(Kg * G // g_steps, 2)
        dtg, _ = timed_loop(lambda ev: graph.replay(), reps_g, 0, pg, device, reps=3, prepare=restore)
        graphs[name] = world * E * reps_g * g_steps / dtg
        del graph
    best_graph = max(graphs, key=graphs.get)
    # the same random policy, 32 / 128 env steps per launch (gca_bulldozer_rollout_random: the env's state in registers
    # across the steps), the per-step rewards and done flags recorded
    rollout = {f"k{k}": rollout_rate(env, 9, max(Kg * G // k, 2) * k, restore, pg, device, world, k=k) for k in (32, 128)}
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
        # the fastest capturable path (a HIP graph of env steps), with every other path beside it
        "env_steps_per_s": graphs[best_graph],
        "env_steps_per_s_path": best_graph,
        "env_steps_per_s_eager": world * E * Kg * G / dt_eager,
        "env_steps_per_s_random_policy_fused": world * E * Kg * G / dt_rand,
        "env_steps_per_s_graphs": graphs,
        # the random policy's K-step rollouts, K = 32 / 128 env steps per launch (a PPO-style rollout length)
        "env_steps_per_s_rollout_random": rollout,
        "loops": f"eager, random-policy-fused and the graphs: the same {Kg * G} env steps (graphs: whole graphs, at "
                 f"least 2) from one mid-episode state (reset + 64 steps, restored before each repetition), median of 3",
        "env_step_graph": "hipGraph of env steps: sample_step_g8 = 8 x (gca_random_actions + gca_bulldozer_step_fused), "
                          "step_random_gN = N x gca_bulldozer_step_fused_random (the same actions drawn inside the step)"
                          if env.fused else "hipGraph of RepeatCA/Windy passes + Move/Modify + reward",
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

    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv
    from gymca_amd.graph import StepGraph

    from gymca_amd import distributed as gd

    E, N = 1024, 512
    env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=0x5EED5, env_offset=rank * E,
                                        materialize_obs=False)
    env.reset()
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)

    def one_step():
        env.step(env.sample_actions(action, 11))

    stats = gd.StatsGather(E, device, len_dtype=env.steps_elapsed.dtype) if world > 1 else None

    def gather(async_op=False):
        if stats is not None:  # RCCL all-gather of reward f32 | length | done u8 per env (gymca_amd.distributed)
            stats.gather(env.done, env.reward, env.steps_elapsed, async_op=async_op)

    K = max(args.steps, 40)
    G = 8
    Kg = max(K // G, 5)
    K = Kg * G  # every loop: the same K env steps from the same reset state (env.reset), median of 3

    def eager(ev):
        one_step()
        gather()

    def overlapped(ev):
        one_step()
        gather(async_op=True)

    def random_fused(ev):
        env.step_random(11, action)
        gather()

    restore = env_snapshot(env, one_step, 64)
    dt_eager, _ = timed_loop(eager, K, 0, pg, device, reps=3, prepare=restore)
    dt_async, _ = timed_loop(overlapped, K, 0, pg, device, reps=3, prepare=restore)
    dt_rand, _ = timed_loop(random_fused, K, 0, pg, device, reps=3, prepare=restore)
    # rollout segments from HIP graphs, one gather per segment: G = 8 x (sample, step), and step_random (one node per env
    # step) in segments of 8 and 32
    graphs = {}
    for name, fn, g_steps in (("sample_step_g8", one_step, G), ("step_random_g8", lambda: env.step_random(11, action), 8),
                              ("step_random_g32", lambda: env.step_random(11, action), 32)):
        restore()
        graph = StepGraph(fn, n_steps=g_steps, device=device)

        def seg(ev, graph=graph):
            graph.replay()
            gather()

        reps_g = max(K // g_steps, 2)
        dtg, _ = timed_loop(seg, reps_g, 0, pg, device, reps=3, prepare=restore)
        graphs[name] = world * E * reps_g * g_steps / dtg
        del graph
    best_graph = max(graphs, key=graphs.get)
    rollout = {f"k{k}": rollout_rate(env, 11, max(K // k, 2) * k, restore, pg, device, world, k=k, gather=gather)
               for k in (32, 128)}
    check = gd.verify_gather(stats)
    # CA-only at HBM scale: one forced Windy step of every env, 268 MB per buffer (beyond the 256 MB
    # Infinity Cache, unlike config 2's 64 MiB pair), dense {0:.1, 3:.6, 25:.3}, beside a same-size copy
    ca = windy_ca_only(env, K, args.warmup, pg, device)
    return {"config": "ForestFireBulldozer 512x512, 1024 envs/GPU (BASELINE config 5 at 8 GPUs), WindyForestFire",
            "env_steps_per_s": graphs[best_graph],
            "env_steps_per_s_path": best_graph + " (graph segment + one gather per segment)",
            "env_steps_per_s_graphs": graphs,
            "env_steps_per_s_rollout_random": rollout,  # K = 32 / 128 env steps per launch, one gather per rollout
            "env_step": ("gca_bulldozer_step_fused (one launch per env step)" if env.fused else
                         "pre / Windy passes / post kernels"),
            "env_steps_per_s_eager_gather_every_step": world * E * K / dt_eager,
            "env_steps_per_s_async_gather_every_step": world * E * K / dt_async,
            "env_steps_per_s_random_policy_fused_gather_every_step": world * E * K / dt_rand,
            "loops": f"graph / eager / async: the same {K} env steps from one mid-episode state (reset + 64 steps, "
                     f"restored before each repetition), median of 3",
            "gather": ("RCCL all_gather_into_tensor of reward f32 | length | done u8 per env into a reused buffer "
                       f"(gymca_amd.distributed.StatsGather: 1 pack + 1 collective), world {world}")
                      if world > 1 else "none (1 GPU)",
            "gather_check": check,
            "ca_only_cell_updates_per_s": world * E * N * N / ca["kernel_s"],
            "ca_kernel_ms": ca["kernel_s"] * 1e3,
            "ca_achieved_gbs": WINDY_BYTES_PER_CELL * E * N * N / ca["kernel_s"] / 1e9,
            "ca_roofline_frac": WINDY_BYTES_PER_CELL * E * N * N / ca["kernel_s"] / 1e9 / HBM_PEAK_GBS,
            "same_size_copy_ms": ca["copy_s"] * 1e3,
            "ca_frac_of_same_size_copy": ca["copy_s"] / ca["kernel_s"]}


def bench_windy512_strong(args, world, rank, device, pg, total=8192):
    """BASELINE config 5 as strong scaling: the 8192 envs of 512^2 split over the ranks
    (distributed.shard; at N = 1 all 8192 on one GPU), the random policy through a hipGraph of 8 step_random steps with
    one episode-stats gather per graph, and the 128-step rollout kernel with one gather per rollout. Rates are whole-job
    env-steps/s (the sum of every rank's envs over the max-over-ranks time)."""
    import torch

    from gymca_amd import distributed as gd
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv
    from gymca_amd.graph import StepGraph

    N = 512
    off, E = gd.shard(total, world, rank)
    env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=0x5EED5, env_offset=off, materialize_obs=False)
    env.reset()
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)
    stats = gd.StatsGather(E, device, len_dtype=env.steps_elapsed.dtype) if world > 1 else None

    def gather():
        if stats is not None:
            stats.gather(env.done, env.reward, env.steps_elapsed)

    restore = env_snapshot(env, lambda: env.step(env.sample_actions(action, 11)), 32)
    graph = StepGraph(lambda: env.step_random(11, action), n_steps=8, device=device)

    def seg(ev):
        graph.replay()
        gather()

    dt_g, _ = timed_loop(seg, 8, 0, pg, device, reps=3, prepare=restore)
    del graph
    roll = rollout_rate(env, 11, 256, restore, pg, device, 1, k=128, gather=gather)  # this rank's envs
    # whole job: every rank's rollout rate is E_rank x steps / (its time); the job's is total x steps / max time, which
    # timed_loop's max-over-ranks already gives for the graph; for the rollout use the same total
    out = {"config": f"ForestFireBulldozer 512x512, {total} envs in all over {world} GPU(s) (strong scaling)",
           "envs_this_rank": E,
           "env_steps_per_s_graph_step_random_g8": total * 8 * 8 / dt_g,
           "env_steps_per_s_rollout_random_k128": roll * total / E,
           "gather": "one StatsGather all_gather per graph / per rollout" if world > 1 else "none (1 GPU)"}
    del env
    torch.cuda.empty_cache()
    return out


def rollout_rate(env, seed, steps, restore, pg, device, world, k=32, gather=None):
    """env-steps/s of the random-policy rollout kernel (env.rollout_random: k env steps per launch, every env's
    per-step reward and done flag recorded in (k, E) buffers), `steps` env steps from the restored state, median of 3;
    `gather` (config 5, N > 1): the episode-stats gather once per rollout segment."""
    import torch

    E = env.num_envs
    rew = torch.empty((k, E), dtype=torch.float64, device=device)
    dn = torch.empty((k, E), dtype=torch.uint8, device=device)

    def seg(ev):
        env.rollout_random(k, seed, None, rew, dn)
        if gather is not None:
            gather()

    n = max(steps // k, 2)
    dt, _ = timed_loop(seg, n, 0, pg, device, reps=3, prepare=restore)
    return world * E * n * k / dt


def windy_ca_only(env, K, W, pg, device):
    """Mean duration of one forced Windy CA step over every env of `env` (dense state, random direction masks)
    and of a device copy of the same bytes, both from HIP events."""
    import torch

    E, H, N = env.num_envs, env.nrows, env.ncols
    g = env.grids()
    u = torch.rand(g.shape, device=device)
    g = torch.where(u < 0.1, 0, torch.where(u < 0.7, 3, 25)).to(torch.uint8)
    env.buf[0].copy_(g)
    del g, u
    env.parity.zero_()
    env.dir_mask.copy_(torch.randint(0, 256, (E,), dtype=torch.uint8, device=device))

    def timed(fn):
        def f(events):
            if events is not None:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                fn()
                b.record()
                events.append((a, b))
            else:
                fn()
        return f

    _, kern = timed_loop(timed(env.ca_step_all), K, W, pg, device)
    src = torch.empty(E * H * N, dtype=torch.uint8, device=device)
    dst = torch.empty_like(src)
    _, kern_copy = timed_loop(timed(lambda: dst.copy_(src)), K, W, pg, device)
    del src, dst
    return {"kernel_s": kern, "copy_s": kern_copy}


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


def run_cpu_legs(args):
    """Every CPU baseline leg of the bench line, on this host, bounded (≈ 2 x --cpu-seconds in all): the Alexandridis
    C restatement (1 core, all job cores), the Windy scipy restatement (1 core, all cores), the bulldozer env loop and
    the helicopter 5x5 loop. Must run before the process initialises the GPU (the all-core Windy leg forks)."""
    leg = max(0.25, args.cpu_seconds / 4)
    return {"alex": cpu_baseline(args), "windy_1core": windy_cpu_baseline(leg), "windy_all_cores": windy_cpu_all_cores(leg),
            "bulldozer_env_256": bulldozer_cpu_baseline(leg), "helicopter_5x5": helicopter_cpu_baseline()}


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


def _windy_cpu_loop(seconds, seed, counter=True):
    """One 256x256 env of the Windy restatement (oracle/windy.py: scipy convolve2d + the three threshold masks, the
    reference algorithm ca_windy.py:41-139) with the bulldozer env's cell count every step: the reference's own
    Counter(grid.flatten().tolist()) (ca_env.py:94-99) when `counter`, else np.unique (a faster-than-reference count).
    Returns (steps, seconds)."""
    from collections import Counter

    import numpy as np

    from gymca_amd.forest_fire.bulldozer.bulldozer import DEFAULT_WIND, parse_wind
    from oracle import windy as owindy

    rng = np.random.default_rng(seed)
    grid = rng.choice(np.array([0, 3, 25]), size=(256, 256), p=[0.1, 0.6, 0.3])
    wind = parse_wind(DEFAULT_WIND)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        grid = owindy.windy_step(grid, wind, rng.random((3, 3)))
        if counter:
            Counter(grid.flatten().tolist())
        else:
            np.unique(grid, return_counts=True)
        steps += 1
    return steps, time.perf_counter() - t0


def windy_cpu_baseline(seconds=3.0):
    """The reference algorithm for WindyForestFire on one core, 256x256, with the reference's Counter cell count per
    step; the np.unique count beside it as a faster-than-reference variant."""
    steps, dt = _windy_cpu_loop(seconds / 2, 5, counter=True)
    steps_u, dt_u = _windy_cpu_loop(seconds / 2, 5, counter=False)
    return {"value": 256 * 256 * steps / dt, "unit": "cell-updates/s", "cores": 1, "kind": "port",
            "sample": f"1 env 256x256, {steps} steps of the scipy restatement + Counter cell count (ca_env.py:94-99)",
            "np_unique_count_variant": 256 * 256 * steps_u / dt_u,
            "np_unique_note": "the same loop counting with np.unique: faster than the reference's Counter"}


def _windy_worker(args_tuple):
    """One process of the all-core Windy CPU leg: the scipy restatement + the reference's Counter cell count."""
    seconds, seed = args_tuple
    return _windy_cpu_loop(seconds, seed, counter=True)


def windy_cpu_all_cores(seconds=3.0):
    """BASELINE.md CPU plan (ii): the Windy restatement on every core this job may use, one process per core,
    envs split evenly. Forked BEFORE this process touches the GPU (main() runs the CPU legs first)."""
    import multiprocessing as mp

    n = _cpu_threads()
    with mp.get_context("fork").Pool(n) as pool:
        res = pool.map(_windy_worker, [(seconds, 100 + i) for i in range(n)])
    rate = sum(256 * 256 * st / dt for st, dt in res)
    return {"value": rate, "unit": "cell-updates/s", "cores": n, "kind": "port",
            "sample": f"{n} processes x 1 env 256x256, {sum(st for st, _ in res)} steps of the scipy restatement "
                      f"+ Counter cell count in {seconds:.0f} s"}


def bulldozer_cpu_baseline(seconds=3.0, N=256):
    """The ForestFireBulldozer 256x256 env loop on one core, the reference's CPU path restated (oracle.windy:
    scipy convolve2d CA passes, RepeatCA time, Move/Modify) with the reference's Counter-based cell count per
    step (ca_env.py:94-99) and random actions; reset when the fire is out."""
    from collections import Counter

    import numpy as np

    from gymca_amd.forest_fire.bulldozer.bulldozer import DEFAULT_WIND, bulldozer_timings, parse_wind
    from oracle import windy as owindy

    rng = np.random.default_rng(11)
    t_move, t_shoot = bulldozer_timings(N, N)

    def fresh():
        g = rng.choice(np.array([0, 3]), size=(N, N), p=[0.1, 0.9])
        g[3 * N // 4, N // 4] = 25
        return owindy.BulldozerOracle([g], [(N // 4, 3 * N // 4)], parse_wind(DEFAULT_WIND), t_move, t_shoot, 0.001,
                                      seed=rng.integers(1 << 62))

    env, steps, resets = fresh(), 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        env.step([(int(rng.integers(0, 9)), int(rng.integers(0, 2)))])
        c = Counter(env.grids[0].ravel().tolist())  # the reference's count_cells
        steps += 1
        if not c[25]:
            env, resets = fresh(), resets + 1
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"1 env {N}x{N}, {steps} env steps (random actions, {resets} resets) of the numpy/scipy "
                      f"restatement + Counter cell count"}


def helicopter_cpu_baseline(steps=1000):
    """BASELINE config 1 on one core: ForestFireHelicopter 5x5, seed 0, 1000 steps, actions k % 9 — the
    Drossel-Schwabl per-cell loop restated (oracle.drossel, the reference's draw order), CA every
    max_freeze + 1 steps, Move/Modify {FIRE: EMPTY} (helicopter.py:220-236), reward from cell counts."""
    import numpy as np

    from oracle import drossel
    from oracle import windy as owindy

    rng = np.random.default_rng(0)
    grid = rng.choice(np.array([0, 1, 2]), size=(5, 5))
    pos, freeze, max_freeze = (2, 2), 2, 2
    t0 = time.perf_counter()
    for k in range(steps):
        if freeze == 0:
            grid = drossel.ds_step(grid, 0.033, 0.333, rng)
            freeze = max_freeze
        else:
            freeze -= 1
        pos = owindy.move(pos, k % 9, 5, 5)
        if grid[pos] == 2:
            grid[pos] = 0
        counts = np.bincount(grid.ravel(), minlength=3) / 25.0
        float(np.dot([0.0, 1.0, -1.0], counts))
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"1 env 5x5, {steps} steps, actions k % 9 (Drossel-Schwabl restatement, oracle/drossel.py)"}


def bench_dropins(device):
    """What a reference user swaps in, one env each (no batching): the ForestFireBulldozerEnv drop-in at 256x256
    with random actions (reference: 366 env-steps/s on one core) and BASELINE config 1,
    ForestFireHelicopterEnv(5, 5) for 1000 steps with actions k % 9 (helicopter.py:220-236)."""
    import numpy as np
    import torch

    from gymca_amd.forest_fire.bulldozer import ForestFireBulldozerEnv
    from gymca_amd.forest_fire.helicopter import ForestFireHelicopterEnv

    out = {}
    env = ForestFireBulldozerEnv(256, 256)
    env.reset(seed=0)
    rng = np.random.default_rng(3)
    for _ in range(20):
        env.step((int(rng.integers(0, 9)), int(rng.integers(0, 2))))
    torch.cuda.synchronize(device)
    steps, resets, ca = 0, 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 3.0:
        _, _, term, _, _ = env.step((int(rng.integers(0, 9)), int(rng.integers(0, 2))))
        steps += 1
        if term:
            env.reset()
            resets += 1
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    out["bulldozer_256"] = {"env_steps_per_s": steps / dt, "steps": steps, "resets": resets,
                            "note": "ForestFireBulldozerEnv(256, 256) drop-in, numpy int64 obs per step, grid "
                                    "device-resident; the cell count, position, hit and observation read back in one "
                                    "synchronisation per step"}
    heli = ForestFireHelicopterEnv(5, 5)
    heli.reset(seed=0)
    heli.step(0)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for k in range(1000):
        heli.step(k % 9)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    out["helicopter_5x5"] = {"env_steps_per_s": 1000 / dt, "steps": 1000,
                             "note": "BASELINE config 1: ForestFireHelicopterEnv(5, 5) drop-in, actions k % 9"}
    return out


def bench_alex512(args, world, rank, device, pg):
    """The Alexandridis step at the reference's next grid size, 512^2 (R = 7, ca_alexandridis_jax.py:62), 1024 envs
    (the headline's 268M cells): the env's marching step (two segment waves per strip) against the tiled packed step on
    the same C3-like state, mean launch time from HIP events (median of 3), no host work in the timed region."""
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 1024, 512
    env = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=device, env_offset=rank * E,
                                         observation="grid")
    env.reset()
    synthetic_state(env, rank, device)

    def march_kernel_ms():
        times = []
        for _ in range(3):
            synthetic_state(env, rank, device)
            env.ca_step()
            torch.cuda.synchronize(device)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                env.ca_step()
            b.record()
            torch.cuda.synchronize(device)
            times.append(a.elapsed_time(b) / 10)
        return sorted(times)[1]

    march_ms, key, nbytes = march_kernel_ms(), headline_kernel_key(env), alex_bytes(env, "packed")
    general_ms = None
    if env.flat_terrain:  # the same step reading the slope planes (the step of any terrain)
        env.flat_terrain = False
        general_ms = march_kernel_ms()
        env.refresh_terrain()
    tiled_ms = tiled_kernel_ms(env, device)
    out = {"config": "AdvancedBulldozer 512x512 (R = 7), 1024 envs, use_hidden=False, C3-like mid-episode state",
           "kernel": key, "march_kernel_ms": march_ms, "tiled_kernel_ms": tiled_ms,
           "march_over_tiled": march_ms / tiled_ms,
           "cell_updates_per_s": E * N * N / (march_ms * 1e-3),
           "bytes_per_cell": nbytes,
           "moved_gbs": nbytes * E * N * N / (march_ms * 1e-3) / 1e9,
           "general_terrain_march_kernel_ms": general_ms}
    del env
    torch.cuda.empty_cache()
    return out


def tiled_kernel_ms(env, device, K=10, reps=3):
    """The same C3 state through the tiled packed kernel (gca_alex_step_packed, coalesced slopes) that the marching
    kernel replaced at W = 256: mean launch time (HIP events, median of reps), for the record beside kernel_ms."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, H, W = env.num_envs, env.nrows, env.ncols
    st = dev.stream_ptr(device)
    coal = torch.empty_like(env.slope_data)
    call("gca_alex_edge_slope_coalesce", dev.ptr(env.slope_data), dev.ptr(coal), E, H, W, st)
    times = []
    for _ in range(reps):
        synthetic_state(env, 0, device)
        a0, b0 = env.cur, 1 - env.cur
        for k in range(K + 1):
            if k == 1:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            a, b = (a0, b0) if k % 2 == 0 else (b0, a0)
            call("gca_alex_step_packed", env.alex_params, E, H, W, dev.ptr(env.grid[a]), dev.ptr(env.grid[b]),
                 dev.ptr(env.age[a]), dev.ptr(env.age[b]), dev.ptr(env.vd), dev.ptr(env.dous_bits), dev.ptr(coal),
                 dev.ptr(env.wind_index), dev.ptr(env.rng_step), dev.ptr(env.counts), None, None, st)
        e1.record()
        torch.cuda.synchronize(device)
        times.append(e0.elapsed_time(e1) / K)
    del coal
    synthetic_state(env, 0, device)
    return sorted(times)[len(times) // 2]


# the sources a kernel is compiled from (csrc/), hashed into every profiles/pmc_traffic.json entry by
# scripts/pmc_summary.py: a committed profile describes the timed kernel only while these files are unchanged
KERNEL_SOURCES = {"alex_march": ("gca_alex_march.hip", "gca_alex_rule.h", "gca_common.h"),
                  "alex_step": ("gca_alex.hip", "gca_alex_rule.h", "gca_common.h")}


def kernel_src_sha(short_name):
    """sha256 (16 hex digits) of the csrc/ sources of kernel family `short_name` (+ include/gca.h), or None."""
    import hashlib

    base = short_name.split("<", 1)[0]
    files = KERNEL_SOURCES.get(base)
    if files is None:
        return None
    h = hashlib.sha256()
    for f in (*(os.path.join(ROOT, "gym-cellular-automata_amd", "csrc", x) for x in files),
              os.path.join(ROOT, "include", "gca.h")):
        try:
            with open(f, "rb") as fh:
                h.update(fh.read())
        except OSError:
            return None
    return h.hexdigest()[:16]


def headline_kernel_key(env):
    """The rocprof short name (scripts/pmc_summary.py) of the template instance env.ca_step() launches."""
    R = int(env.alex_params.R)
    grow = "true" if env.alex_params.p_tree > 0 else "false"
    if getattr(env, "march", False):
        flat = getattr(env, "flat_terrain", False)
        fm = 0 if not flat else (2 if getattr(env, "uniform_layers", False) else 1)
        return f"alex_march<{R}, false, {grow}, {int(env.ncols) // 256}, {fm}>"
    es = "true" if env.slope_layout in ("packed", "edge") else "false"
    pk = "true" if env.slope_layout == "packed" else "false"
    return f"alex_step<{R}, 0, true, {es}, {pk}, false>"


def profile_entry(args, key):
    """The committed PMC summary entry (profiles/pmc_traffic.json) of the timed headline kernel `key`, with its
    provenance: the entry counts only when it was profiled on this workload from the SAME kernel sources (source hash
    recorded by scripts/pmc_summary.py); otherwise its figures are not this build's and the bench reports null."""
    info = {"key": key, "tag": None, "src_sha": kernel_src_sha(key), "profile_src_sha": None, "match": False}
    if args.envs != 4096 or args.size != 256:
        info["why"] = "not the profiled workload (4096 x 256^2)"
        return None, info
    try:
        data = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    except (ValueError, OSError):
        info["why"] = "no profiles/pmc_traffic.json"
        return None, info
    e = data.get(key)
    if e is None:
        info["why"] = "the timed kernel has no committed profile"
        return None, info
    info.update(tag=e.get("tag"), profile_src_sha=e.get("src_sha"))
    if e.get("src_sha") is None or e.get("src_sha") != info["src_sha"]:
        info["why"] = "the committed profile predates the kernel's current sources"
        return None, info
    info["match"] = True
    return e, info


def copy_bandwidth(device, nbytes=2 << 30, reps=10):
    """Live device copy rate (GB/s, read + write) of the library's hand-written 16-B copy (gca_bench_copy,
    gca_bench.hip) over 2 GiB (8x the 256 MB Infinity Cache), plain and non-temporal, HIP events over `reps` launches
    after a warm-up: the practical HBM ceiling on this device, reported beside the 8 TB/s spec (the guide's float4
    copy: 6.29 TB/s). Returns (best GB/s, {variant: GB/s})."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    a = torch.empty(nbytes, dtype=torch.uint8, device=device)
    b = torch.empty_like(a)
    a.fill_(1)
    st = dev.stream_ptr(device)
    rates = {}
    for name, nt in (("plain", 0), ("nontemporal", 1)):
        call("gca_bench_copy", dev.ptr(a), dev.ptr(b), nbytes, nt, st)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            call("gca_bench_copy", dev.ptr(a), dev.ptr(b), nbytes, nt, st)
        e.record()
        e.synchronize()
        rates[name] = 2.0 * nbytes * reps / (s.elapsed_time(e) * 1e-3) / 1e9
    del a, b
    return max(rates.values()), rates


def march_pattern_ms(env, device, frame=False, K=10, reps=3):
    """The headline kernel's access-pattern floor in this run (gca_bench_march_pattern: gca_alex_step_march's loads and
    stores at W = 256 with trivial arithmetic, on the env's own packed-layout buffers, without the slope planes when the
    env's step runs on flat terrain; frame=True adds the fused frame's
    RGB stores at the frame kernel's 2 waves / SIMD): mean launch time from HIP events, median of `reps`. Scratch
    outputs (the env's state is untouched; the frame buffer is rewritten by the next rendered step). None off the
    marching step."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    if not getattr(env, "march", False) or env.ncols != 256:
        return None
    E, H, W = env.num_envs, env.nrows, env.ncols
    a = env.cur
    flat = getattr(env, "flat_terrain", False)
    go, ao = torch.empty_like(env.grid[a]), torch.empty_like(env.age[a])
    st = dev.stream_ptr(device)
    args = (int(env.alex_params.R), E, H, W, dev.ptr(env.grid[a]), dev.ptr(go), dev.ptr(env.age[a]), dev.ptr(ao),
            None if flat and getattr(env, "uniform_layers", False) else dev.ptr(env.vd), dev.ptr(env.dous_bits),
            None if flat else dev.ptr(env.slope_data),
            dev.ptr(env.rgb if frame else None), st)
    times = []
    for _ in range(reps):
        for _ in range(3):
            call("gca_bench_march_pattern", *args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            call("gca_bench_march_pattern", *args)
        e1.record()
        e1.synchronize()
        times.append(e0.elapsed_time(e1) / K)
    del go, ao
    return sorted(times)[len(times) // 2]


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args)  # N child ranks; this process never touches the GPU
    if args.dry_run:
        return dry_run(args)
    world_env, rank_env = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    if world_env != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world_env}: launch it as plain "
                         f"`python bench.py --gpus N` (it starts the N ranks) or through torch.distributed.run")
    # CPU legs first, at every world size: the all-core Windy leg forks worker processes, which must happen before this
    # process initialises the GPU
    cpu_legs = cpu_legs_for_rank0(args, rank_env)
    cpu = None if cpu_legs is None else cpu_legs["alex"]
    world, rank, device, pg = setup_dist(args)
    import torch

    alex = bench_alex(args, world, rank, device, pg)
    import gc

    gc.collect()
    torch.cuda.empty_cache()
    config4 = None if args.no_secondary else bench_config4(args, world, rank, device, pg)
    alex512 = None if (args.no_secondary or args.size != 256) else bench_alex512(args, world, rank, device, pg)
    secondary = None if args.no_secondary else bench_windy(args, world, rank, device, pg)
    config5 = None if args.no_secondary else bench_windy512(args, world, rank, device, pg)
    config5_strong = None if args.no_secondary else bench_windy512_strong(args, world, rank, device, pg)
    # the one-env drop-ins on rank 0 only (no collective inside; the other ranks go on to the copy-rate probe)
    dropins = None if (args.no_secondary or rank != 0) else bench_dropins(device)
    if cpu_legs is not None:
        if secondary is not None:
            secondary["cpu_baseline"] = cpu_legs["windy_1core"]
            secondary["cpu_baseline_all_cores"] = cpu_legs["windy_all_cores"]
        if dropins is not None:
            dropins["bulldozer_256"]["cpu_baseline"] = cpu_legs["bulldozer_env_256"]
            dropins["helicopter_5x5"]["cpu_baseline"] = cpu_legs["helicopter_5x5"]
    # HBM bytes per headline launch (2*FETCH_SIZE + WRITE_SIZE, the gfx950 correction, calibrated by
    # scripts/fetch_calib.hip) and VALU busy (SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)) from the
    # committed rocprofv3 summary of the SAME kernel (template and sources), else null
    prof, prof_info = profile_entry(args, alex["kernel_key"])
    traffic = None if prof is None else prof.get("bytes_per_launch")
    valu_busy = None if prof is None else prof.get("valu_busy")
    copy_gbs, copy_rates = copy_bandwidth(device)
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
                       "parallelism": f"env-sharded x{world}" + (
                           f", RCCL all_gather of done/return/length per step ({args.gather})"
                           if world > 1 and args.gather != "none" else "")},
            # N > 1: the world size RCCL reported (an all_reduce of ones over the nccl group), the headline loop's last
            # gather verified against every rank's payload, and every rank's own ms per step; null at N = 1
            "rccl_world": None if alex["gather_check"] is None else alex["gather_check"]["world_seen"],
            "gather_ok": None if alex["gather_check"] is None else alex["gather_check"]["gather_ok"],
            "gather_check": alex["gather_check"],
            "per_rank_ms_per_step": alex["timing"].get("per_rank_ms_per_step"),
            "envs_total": world * args.envs,
            "timing": dict(alex["timing"], note="value / ms_per_step = the median of the repetitions, each "
                                                "exactly `steps` steps between barrier + synchronize"),
            "env_steps_per_s": alex["env_steps_per_s"],
            "episode_start": alex.get("episode_start"),
            "with_rgb_observation": alex.get("with_rgb_observation"),
            "with_rgb_observation_extensions": alex.get("with_rgb_observation_extensions"),
            # achieved = the algorithmic bytes of the step as built (23.125 B per cell-update in the packed layout: every
            # input byte read once, every output byte written once; 7.125 on flat terrain -- use_hidden=False, this
            # config -- where the step reads no slope planes, and 6.125 with its uniform layers, where it reads no vd
            # layer either; that step is VALU-bound, see valu_busy and general_terrain)
            # x cells / the kernel's mean launch time. SURVEY.md
            # §8d's 41 B (the 8-plane layout's bytes) is reported beside it as survey_equiv_*: since the marching
            # kernel it exceeds the 8 TB/s peak (> 1.0), i.e. it no longer measures anything. traffic = PMC bytes.
            "roofline": {"bound": "hbm", "achieved": alex["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alex["achieved_gbs"] / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": alex["kernel"],
                         "kernel_ms": alex["kernel_ms"],
                         "tiled_kernel_ms": alex.get("tiled_kernel_ms"),
                         "algorithmic_bytes_per_cell": alex["bytes_per_cell"],
                         "terrain": alex["terrain"],
                         "survey_bytes_per_cell": ALEX_BYTES_PER_CELL,
                         "survey_equiv_gbs": alex["survey_equiv_gbs"],
                         "survey_equiv_frac": alex["survey_equiv_gbs"] / HBM_PEAK_GBS,
                         "valu_busy": valu_busy,
                         # what binds the timed kernel by its matched profile: VALU issue when the SIMDs are >= 95 % busy
                         # (the flat-terrain step), else the HBM stream (its frac above says how close)
                         "limiter": (None if valu_busy is None else "valu" if valu_busy >= 0.95 else "hbm"),
                         "profile": prof_info,
                         "slope_layout": args.slope_layout,
                         "moved_bytes_per_cell": alex["bytes_per_cell"],
                         "moved_gbs": alex["achieved_gbs"],
                         "moved_frac": alex["achieved_gbs"] / HBM_PEAK_GBS,
                         "traffic_bytes_per_cell": traffic / (args.envs * args.size * args.size) if traffic else None,
                         "traffic_gbs": traffic / (alex["kernel_ms"] * 1e-3) / 1e9 if traffic else None,
                         "traffic_frac": traffic / (alex["kernel_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None,
                         "device_copy_gbs": copy_gbs,
                         "device_copy": dict(copy_rates, kernel="gca_bench_copy: 16-B copy of 2 GiB, one element "
                                                                "per thread, one pass"),
                         "moved_frac_of_device_copy": alex["achieved_gbs"] / copy_gbs,
                         # the same run's floor of the headline kernel's own access pattern (gca_bench_march_pattern)
                         "pattern_floor_ms": alex.get("pattern_floor_ms"),
                         "kernel_over_pattern_floor": (alex["kernel_ms"] / alex["pattern_floor_ms"]
                                                       if alex.get("pattern_floor_ms") else None),
                         # flat terrain: the same step with the slope planes streamed (rounds 1-6's headline kernel)
                         "general_terrain": alex.get("general_terrain")},
            "cpu_baseline": cpu,
            "secondary": secondary,
            "config4": config4,
            "alex_512": alex512,
            "config5": config5,
            "config5_strong": config5_strong,
            "dropins": dropins,
        }
        print(json.dumps(out))
    if pg is not None:
        pg.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
