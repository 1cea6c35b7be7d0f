"""Multi-process path on CPU (gloo, world_size 2) and the sharding convention."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

from gymca_amd.distributed import all_gather_stats, shard
from oracle import windy as owindy


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from gymca_amd.distributed import EpisodeStats, StatsGather

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # built BEFORE the process group exists: they must gather across ranks once it does
    pre, pre_stats = StatsGather(4, "cpu"), EpisodeStats(4, "cpu")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    v = torch.full((4,), float(rank))
    pd, pr, pl = pre.gather(torch.full((4,), rank, dtype=torch.uint8), v, v.to(torch.int32))
    sd, sr, sl = pre_stats.gather(torch.full((4,), rank, dtype=torch.uint8), v, v.to(torch.int32))
    late_ok = (tuple(pd.shape) == (world, 4) and pr[:, 0].tolist() == [float(r) for r in range(world)]
               and tuple(sd.shape) == (world, 4) and sl[:, 0].tolist() == list(range(world)))
    off, n = shard(7, world, rank)
    done = torch.tensor([(off + i) % 2 for i in range(n)], dtype=torch.uint8)
    ret = torch.tensor([-(off + i) / 10 for i in range(n)], dtype=torch.float32)
    ln = torch.tensor([off + i for i in range(n)], dtype=torch.int32)
    # uneven shards are padded to the largest shard before gathering
    E = max(shard(7, world, r)[1] for r in range(world))
    pad = E - n
    done = torch.cat([done, torch.zeros(pad, dtype=torch.uint8)])
    ret, ln = torch.cat([ret, torch.zeros(pad)]), torch.cat([ln, torch.zeros(pad, dtype=torch.int32)])
    d, r, l = all_gather_stats(done, ret, ln)
    assert d.shape == (world, E)  # (world, E) views of the gathered buffer
    # the reused StatsGather: no allocation and two ops (the pack, the collective) per call
    g = StatsGather(E, "cpu", len_dtype=torch.int32)
    g.gather(done, ret, ln)  # warm
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], profile_memory=True) as prof:
        for _ in range(3):
            gd, gr, gl = g.gather(done, ret, ln)
    ops = [e for e in prof.events() if e.name in ("aten::cat", "c10d::_allgather_base_", "c10d::allgather_")
           or "all_gather" in e.name or "allgather" in e.name]

    def in_collective(e):  # gloo's own staging inside the collective (RCCL has none) is not ours
        while e is not None:
            if e.name.startswith("c10d::") or e.name.startswith("gloo:"):
                return True
            e = e.cpu_parent
        return False

    main = {e.thread for e in prof.events() if e.name == "aten::cat"}  # gloo's worker threads are not ours
    allocs = [e for e in prof.events() if getattr(e, "cpu_memory_usage", 0) > 0 and not in_collective(e)
              and e.thread in main]
    q.put((rank, d.reshape(-1).tolist(), r.reshape(-1).tolist(), l.reshape(-1).tolist(),
           sorted({e.name for e in ops}), len([e for e in ops if e.name == "aten::cat"]), len(allocs),
           gd.reshape(-1)[:n].tolist() if rank == 0 else None, late_ok))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_covers_all_envs():
    for n in (1, 7, 8, 4096, 8191):
        for w in (1, 2, 3, 8):
            spans = [shard(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and sum(c for _, c in spans) == n
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(w - 1))


def test_gloo_world2_all_gather_of_episode_stats():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, _, _, _, names, n_cat, n_alloc, _, late_ok in out:
        assert n_cat == 3 and n_alloc == 0, (names, n_cat, n_alloc)  # 3 calls: one pack each, nothing allocated
        assert late_ok  # gathers built before init_process_group follow the group once it exists
        assert any("gather" in nm for nm in names), names
    res = {r: (d, ret, ln) for r, d, ret, ln, *_ in out}
    assert res[0] == res[1]
    d, ret, ln = res[0]
    # rank 0 holds envs 0..3, rank 1 holds 4..6 (+1 pad)
    assert ln[:4] == [0, 1, 2, 3] and ln[4:7] == [4, 5, 6]
    assert d[:4] == [0, 1, 0, 1] and np.allclose(ret[4:7], [-0.4, -0.5, -0.6])


def test_sharded_philox_streams_equal_unsharded():
    """Global env ids in every counter: two shards reproduce the single-shard trajectories."""
    rng = np.random.default_rng(0)
    E, N = 4, 24
    grids = [rng.choice([0, 3, 25], size=(N, N), p=[0.1, 0.7, 0.2]) for _ in range(E)]
    pos = [(6, 18)] * E
    wind = np.full((3, 3), 0.6)
    full = owindy.BulldozerOracle(grids, pos, wind, 0.6, 0.3, 0.001, seed=11)
    a = owindy.BulldozerOracle(grids[:2], pos[:2], wind, 0.6, 0.3, 0.001, seed=11, env_offset=0)
    b = owindy.BulldozerOracle(grids[2:], pos[2:], wind, 0.6, 0.3, 0.001, seed=11, env_offset=2)
    for s in range(30):
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E)], axis=1)
        full.step(act)
        a.step(act[:2])
        b.step(act[2:])
    for e in range(E):
        assert np.array_equal(full.grids[e], (a.grids + b.grids)[e])


def test_all_gather_stats_any_env_count():
    """The packed payload keeps its f32 / i32 views aligned for env counts that are not multiples of 4."""
    for E in (1, 3, 5, 1023):
        done = (torch.arange(E) % 2).to(torch.uint8)
        d, r, ln = all_gather_stats(done, -torch.arange(E, dtype=torch.float32), torch.arange(E, dtype=torch.int32))
        assert d.shape == (1, E)
        d, r, ln = d[0], r[0], ln[0]
        assert torch.equal(d, done) and torch.equal(r, -torch.arange(E, dtype=torch.float32))
        assert torch.equal(ln, torch.arange(E, dtype=torch.int32))


def _bench(*argv, env=None):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *argv], capture_output=True, text=True,
                       timeout=240, env=e, cwd=root)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_gpus2_dry_run_spawns_two_gloo_ranks():
    """`python bench.py --gpus 2 --dry-run` starts two ranks itself (no torchrun in front), each takes its env
    shard and the episode-stats all-gather the bench uses returns every rank's envs in order."""
    rc, out, err = _bench("--gpus", "2", "--dry-run", "--envs", "7", "--no-cpu-baseline")
    assert rc == 0, err[-2000:]
    assert out["n_gpus"] == 2 and out["backend"] == "gloo" and out["gather_ok"]
    assert [(r["rank"], r["env_offset"], r["envs"]) for r in out["ranks"]] == [(0, 0, 7), (1, 7, 7)]
    chk = out["gather_check"]  # the real N-rank path's self-check (StatsGather.verify), here on gloo
    assert chk["gather_ok"] and chk["rank_ok"] == [True, True] and chk["world_seen"] == 2 == out["rccl_world"]
    assert out["cpu_baseline"] is None


def _check_cpu_legs(out, measured_by):
    cpu = out["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["unit"] == "cell-updates/s" and cpu["kind"] == "port"
    assert cpu["cores"] >= 1 and cpu["cpu_model"] and measured_by in cpu["measured_by"]
    legs = out["cpu_legs"]
    for k in ("windy_1core", "windy_all_cores", "bulldozer_env_256", "helicopter_5x5"):
        assert legs[k]["value"] > 0 and legs[k]["cores"] >= 1, k


def test_bench_gpus2_dry_run_carries_the_cpu_baseline_to_rank0():
    """VERDICT r04 missing 3: at N > 1 the bench line carries the CPU baseline. `bench.py --gpus 2` runs the CPU legs
    in the launching parent (before any rank exists, no GPU) and hands them to rank 0, whose line reports them."""
    rc, out, err = _bench("--gpus", "2", "--dry-run", "--envs", "7", "--cpu-seconds", "1")
    assert rc == 0, err[-2000:]
    assert out["n_gpus"] == 2 and out["gather_ok"]
    _check_cpu_legs(out, "parent")


def test_bench_torchrun_launch_measures_the_cpu_baseline_on_rank0():
    """The driver's own N > 1 launch (torch.distributed.run in front of bench.py): rank 0 runs the CPU legs itself
    before it initialises the GPU / joins the process group, and its line carries them."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GCA_BENCH_CPU_JSON")}
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
                        "--gpus", "2", "--dry-run", "--envs", "5", "--cpu-seconds", "1"],
                       capture_output=True, text=True, timeout=240, env=e, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["gather_ok"]
    _check_cpu_legs(out, "rank 0")


def test_bench_torchrun_eight_ranks_rehearsal():
    """The driver's 8-GPU launch shape (torch.distributed.run --nproc-per-node 8 in front of bench.py --gpus 8) on gloo:
    8 ranks of 5 envs each (weak scaling: --envs is per rank), the episode-stats all-gather in rank order."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GCA_BENCH_CPU_JSON")}
    e["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
                        "--gpus", "8", "--dry-run", "--envs", "5", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=240, env=e, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 8 and out["gather_ok"]
    assert [(r["rank"], r["env_offset"], r["envs"]) for r in out["ranks"]] == [(k, 5 * k, 5) for k in range(8)]
    assert out["gather_check"]["rank_ok"] == [True] * 8 and out["rccl_world"] == 8


def test_bench_refuses_a_world_size_mismatch():
    rc, out, err = _bench("--gpus", "2", env={"WORLD_SIZE": "1", "RANK": "0"})
    assert rc != 0 and out is None and "WORLD_SIZE=1" in err


def _group_gather_worker(rank, world, port, q):
    import gc
    import weakref

    import torch
    import torch.distributed as dist

    from gymca_amd import distributed as gd

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        refs = []
        for cycle in range(3):
            g = dist.new_group([0, 1])
            d, r, ln = gd.all_gather_stats(torch.tensor([1, 0], dtype=torch.uint8), torch.tensor([0.5, -1.0]),
                                           torch.tensor([3, 4], dtype=torch.int32), group=g)
            assert d.shape == (2, 2) and float(r[1, 1]) == -1.0
            refs.append(weakref.ref(g))
            dist.destroy_process_group(g)
            del g
        gc.collect()
        alive = sum(ref() is not None for ref in refs)
        q.put((rank, alive, len(gd._GROUP_GATHERS)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None))


def test_all_gather_stats_does_not_keep_destroyed_groups():
    """all_gather_stats caches a StatsGather per explicit group; after destroy_process_group(g) neither the
    group nor its cached gather stays alive (three create / gather / destroy cycles, gloo world 2)."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_group_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == [(0, 0, 0), (1, 0, 0)], res


def _verify_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from gymca_amd import distributed as gd

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        E = 6
        g = gd.StatsGather(E, "cpu")
        base = torch.arange(E, dtype=torch.float32) + 10 * rank
        for step in range(3):
            g.gather((base > 2 + step).to(torch.uint8), base + step, torch.full((E,), step, dtype=torch.int32))
        clean = g.verify()
        # a corrupted delivery on rank 1: one byte of rank 0's row in the buffer the last gather wrote
        if rank == 1:
            g.out[(g.k - 1) % len(g.out)][0, 5] ^= 0x40
        bad = g.verify()
        q.put((rank, clean, bad))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None))


def test_stats_gather_verify_detects_a_corrupted_row():
    """StatsGather.verify (bench.py's gather_check / rccl_world at N > 1) on gloo world 2: a clean
    gather passes on both ranks with world_seen = 2; one flipped byte in the buffer rank 1 received fails rank 1 only,
    and both ranks report it (gather_ok False, rank_ok [True, False])."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_verify_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=120) for _ in ps), key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    for rank, clean, bad in res:
        assert isinstance(clean, dict), clean
        assert clean["gather_ok"] and clean["world_seen"] == 2 and clean["rank_ok"] == [True, True]
        assert not bad["gather_ok"] and bad["rank_ok"] == [True, False]
