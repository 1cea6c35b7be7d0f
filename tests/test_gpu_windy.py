"""GPU parity: WindyForestFire kernels and the ForestFireBulldozer envs vs the reference
(golden vectors) and the CPU oracle (Philox rolls). Bit-exact integer states."""
import numpy as np
import pytest

from _contract import assert_operator
from oracle import windy as owindy

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    return torch


def test_windy_dropin_matches_reference_golden(golden, device):
    from gymca_amd.forest_fire.operators import WindyForestFire

    d = golden("windy")
    for i in range(int(d["n"])):
        E, T, F = (int(v) for v in d[f"c{i}_values"])
        op = WindyForestFire(E, T, F)
        grid = d[f"c{i}_grid"].astype(np.int64)
        out, w = op.update(grid, None, d[f"c{i}_wind"], roll=d[f"c{i}_roll"])
        assert out.dtype == np.int64
        assert np.array_equal(out, d[f"c{i}_out"]), f"case {i} shape {grid.shape} values {(E, T, F)}"


def test_windy_dict_context_is_unwrapped(device):
    from gymca_amd.forest_fire.operators import WindyForestFire

    op = WindyForestFire()
    g = np.full((8, 8), 3)
    g[4, 4] = 25
    ctx = {"wind": np.ones((3, 3))}
    out, ctx_out = op.update(g, None, ctx)
    assert ctx_out is ctx
    assert out[4, 4] == 0 and np.all(out[3:6, 3:6][np.array([[1, 1, 1], [1, 0, 1], [1, 1, 1]], bool)] == 25)


@pytest.mark.parametrize("W", [16, 32, 64, 128, 256, 512, 1024])
def test_fast_kernel_equals_exact_kernel(device, W):
    torch = _torch()
    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, H = 7, 45 if W < 1024 else 19
    rng = np.random.default_rng(W)
    grid = rng.choice(np.array([0, 3, 25], np.uint8), size=(E, H, W), p=[0.2, 0.5, 0.3])
    masks = torch.as_tensor(rng.integers(0, 256, E).astype(np.uint8), device=device)
    src = torch.as_tensor(grid, device=device)
    outs, cnts = [], []
    for exact in (0, 1):
        dst = torch.zeros_like(src)
        counts = torch.zeros((E, 3), dtype=torch.int32, device=device)
        call("gca_windy_step", dev.ptr(src), dev.ptr(dst), None, None, 0, dev.ptr(masks), E, H, W, 0, 3, 25, exact,
             dev.ptr(counts), dev.stream_ptr())
        outs.append(dst.cpu().numpy())
        cnts.append(counts.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    assert np.array_equal(cnts[0], cnts[1])
    # and the oracle (scipy convolve2d restatement) agrees
    for e in (0, E - 1):
        m = int(masks[e].item())
        roll = np.full((3, 3), 0.5)
        wind = np.zeros((3, 3))
        for d, idx in enumerate([0, 1, 2, 3, 5, 6, 7, 8]):
            wind.reshape(9)[idx] = 1.0 if (m >> d) & 1 else 0.0
        ref = owindy.windy_step(grid[e].astype(np.int64), wind, roll)
        assert np.array_equal(outs[0][e], ref)
        assert tuple(cnts[0][e]) == tuple(int(np.sum(ref == v)) for v in (0, 3, 25))


def test_philox_dirmask_matches_oracle(device):
    torch = _torch()
    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, seed = 50, 0x5EED
    rng = np.random.default_rng(3)
    wind = rng.random((E, 9))
    w_d = torch.as_tensor(wind, device=device)
    for step in (0, 1, 77):
        rs = torch.full((E,), step, dtype=torch.int32, device=device)
        m = torch.zeros(E, dtype=torch.uint8, device=device)
        call("gca_windy_dirmask", dev.ptr(w_d), 9, None, seed, dev.ptr(rs), None, 0, 100, dev.ptr(m), E,
             dev.stream_ptr())
        got = m.cpu().numpy()
        for e in range(E):
            assert got[e] == owindy.dir_mask(wind[e], owindy.philox_roll(seed, 100 + e, step))


@pytest.mark.parametrize("N,E,steps", [(32, 6, 120), (64, 4, 80), (256, 3, 60), (40, 5, 60), (512, 3, 160)])
def test_batched_bulldozer_env_matches_oracle(device, N, E, steps):
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=17)
    env.reset(seed=5)
    grids0 = env.grids().cpu().numpy()
    pos0 = env.pos.cpu().numpy()
    o = owindy.BulldozerOracle(grids0, pos0, env.wind[0].cpu().numpy().reshape(3, 3), env.t_act_move,
                               env.t_act_shoot, env.t_any, seed=17)
    rng = np.random.default_rng(1)
    for s in range(steps):
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E)], axis=1)
        _, rew, term, _, info = env.step(act)
        exp = o.step(act)
        got = env.grids().cpu().numpy()
        for e in range(E):
            assert np.array_equal(got[e], o.grids[e]), f"step {s} env {e}"
        r = rew.cpu().numpy()
        assert np.array_equal(np.isnan(r), np.isnan(exp)) and np.allclose(r[~np.isnan(r)], exp[~np.isnan(exp)],
                                                                           rtol=0, atol=0)
        assert np.array_equal(term.cpu().numpy(), o.done)
        assert np.array_equal(env.pos.cpu().numpy(), np.array(o.pos))
        assert np.array_equal(env.accu.cpu().numpy(), o.accu)
        assert np.array_equal(env.hit.cpu().numpy().astype(bool), o.hit)


@pytest.mark.parametrize("case", [0, 1, 2])
def test_dropin_bulldozer_env_replays_reference_episode(golden, device, case):
    import zlib

    from gymca_amd.forest_fire.bulldozer import ForestFireBulldozerEnv

    d = golden("bulldozer")
    N = int(d[f"c{case}_N"])
    env = ForestFireBulldozerEnv(N, N)
    env.reset(seed=0)
    env.grid = d[f"c{case}_grid0"].astype(np.int64)
    env.context = ({"wind": d[f"c{case}_wind"]}, d[f"c{case}_pos0"].astype(np.int64), np.array(0.0))
    env.state = env.grid, env.context
    rolls, nrolls = d[f"c{case}_rolls"], d[f"c{case}_nrolls"]
    k = 0
    for s, (act, rec) in enumerate(zip(d[f"c{case}_actions"], d[f"c{case}_recs"])):
        env.ca.roll_queue = list(rolls[k:k + nrolls[s]])
        k += nrolls[s]
        obs, rew, term, trunc, info = env.step(act)
        grid, (ca_params, pos, t) = obs
        exp_rew, exp_term, exp_hit, pr, pc, tt, cE, cT, cF = rec
        assert rew == exp_rew and bool(term) == bool(exp_term) and bool(info["hit"]) == bool(exp_hit), f"step {s}"
        assert (int(pos[0]), int(pos[1])) == (pr, pc) and float(t) == tt
        assert zlib.crc32(np.asarray(grid).astype(np.uint8).tobytes()) & 0xFFFFFFFF == int(d[f"c{case}_crc"][s])
        assert not env.ca.roll_queue


def test_operator_contracts(device):
    from gymca_amd.forest_fire.bulldozer import ForestFireBulldozerEnv
    from gymca_amd.forest_fire.operators import WindyForestFire

    assert_operator(WindyForestFire(0, 3, 25), strict=False)
    env = ForestFireBulldozerEnv(nrows=32, ncols=32)
    assert_operator(env.MDP, strict=True)


def test_reference_windy_invariants_deterministic_wind(device):
    """test_ca_windy.py:55-102 restated: wind = 1 everywhere -> exact rule checks."""
    from gymca_amd.forest_fire.operators import WindyForestFire
    from gymca_amd.grid_space import GridSpace

    ca = WindyForestFire(0, 3, 25)
    wind = ca.context_space.high
    gs = GridSpace(values=[0, 3, 25], shape=(4, 4))
    for _ in range(16):
        grid = gs.sample()
        for _ in range(4):
            new, _ = ca(grid, None, wind)
            pad = np.pad(grid, 1)
            for r in range(4):
                for c in range(4):
                    nb = pad[r:r + 3, c:c + 3]
                    if grid[r, c] == 3:
                        assert new[r, c] == (25 if (nb == 25).any() else 3)
                    else:
                        assert new[r, c] == 0
            grid = new


def test_reference_repeat_ca_two_steps(device):
    """test_repeat_ca.py:68-90: time 1.0 + 1.0 -> exactly two CA applications, accu back to 0."""
    from gymca_amd.forest_fire.operators import RepeatCA, WindyForestFire
    from gymca_amd.grid_space import GridSpace
    from gymca_amd.spaces import Box, Discrete, Tuple

    gs = GridSpace(values=[0, 3, 25], shape=(8, 8))
    ca = WindyForestFire(0, 3, 25, grid_space=gs, action_space=Discrete(1))
    ctx = Tuple((ca.context_space, Box(np.array(0.0), np.array(1.0), dtype=np.float64)))
    rep = RepeatCA(ca, lambda a: 1.0, lambda s: 1.0, grid_space=gs, action_space=Discrete(1), context_space=ctx)
    assert_operator(rep, strict=True)
    grid = gs.sample()
    params = ca.context_space.high
    observed, (_, accu) = rep(grid.copy(), None, (params, 0.0))
    g2, _ = ca(grid.copy(), None, params)
    g2, _ = ca(g2, None, params)
    assert np.array_equal(observed, g2) and accu == 0.0


@pytest.mark.parametrize("N", [256, 512])  # BASELINE config 2 / config 5's per-GPU shard
def test_full_size_windy_properties(device, N):
    """BASELINE config 2 size (1024 x 256^2) and config 5's per-GPU shard (1024 x 512^2, 268 MB per buffer)
    through the batched env's forced CA step: FIRE -> EMPTY, EMPTY stays, TREE stays or burns, and sampled
    envs equal the oracle."""
    torch = _torch()
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    E = 1024
    env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=3, p_tree=0.6, p_empty=0.1)
    env.reset()
    # dense variant: sprinkle fire
    g = env.grids()
    g[torch.rand(g.shape, device=device) < 0.3] = 25
    env.buf[0].copy_(g)
    env.dir_mask.copy_(torch.randint(0, 256, (E,), dtype=torch.uint8, device=device))
    before = env.grids().clone()
    env.ca_step_all()
    after = env.grids()
    assert torch.all(after[before == 25] == 0) and torch.all(after[before == 0] == 0)
    assert torch.all((after[before == 3] == 3) | (after[before == 3] == 25))
    for e in (0, 511, 1023):
        m = int(env.dir_mask[e].item())
        wind = np.array([1.0 if (m >> d) & 1 else 0.0 for d in range(8)])
        w9 = np.insert(wind, 4, 0.0).reshape(3, 3)
        ref = owindy.windy_step(before[e].cpu().numpy().astype(np.int64), w9, np.full((3, 3), 0.5))
        assert np.array_equal(after[e].cpu().numpy(), ref)


def test_batched_env_graph_replay_equals_eager(device):
    """A HIP-graph replay of G env steps (device action sampling + the whole env step) leaves
    every env in exactly the state G eager steps leave it in (gymca_amd/graph.py)."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv
    from gymca_amd.graph import StepGraph

    E, N, G = 64, 64, 6
    envs = [BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=3, materialize_obs=False) for _ in range(2)]
    acts = [torch.zeros((E, 2), dtype=torch.int32, device=device) for _ in range(2)]
    for env in envs:
        env.reset(seed=11)

    def stepper(k):
        def f():
            call("gca_random_actions", dev.ptr(acts[k]), E, 0, 5, dev.ptr(envs[k].rng_step), dev.stream_ptr(device))
            envs[k].step(acts[k])
        return f

    graph = StepGraph(stepper(0), n_steps=G, device=device, warmup=2)  # warm-up = 2 eager steps
    eager = stepper(1)
    for _ in range(2):
        eager()
    for _ in range(3):
        graph.replay()
        for _ in range(G):
            eager()
    torch.cuda.synchronize(device)
    a, b = envs
    assert torch.equal(a.grids(), b.grids())
    for name in ("pos", "accu", "rng_step", "done", "counts", "reward"):
        ta, tb = getattr(a, name), getattr(b, name)
        assert torch.equal(torch.nan_to_num(ta), torch.nan_to_num(tb)), name


@pytest.mark.parametrize("N,G", [(256, 32), (512, 8)])
def test_step_random_graph_replay_equals_eager(device, N, G):
    """The bench's capturable Windy path: a HIP graph of G env.step_random calls (one launch per
    env step: the random policy's draw inside the fused step) leaves every env exactly as G eager step_random calls
    do, and both equal sample_actions + step."""
    import torch

    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv
    from gymca_amd.graph import StepGraph

    E = 128
    envs = [BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=8, materialize_obs=False) for _ in range(3)]
    outs = [torch.zeros((E, 2), dtype=torch.int32, device=device) for _ in range(3)]
    for env in envs:
        env.reset(seed=3)
        _dense_state(env, device, seed=4, p_fire=0.05)
    graph = StepGraph(lambda: envs[0].step_random(9, outs[0]), n_steps=G, device=device, warmup=1)
    envs[1].step_random(9, outs[1])  # the graph's one eager warm-up step
    envs[2].step(envs[2].sample_actions(outs[2], 9))
    for _ in range(2):
        graph.replay()
        for _ in range(G):
            envs[1].step_random(9, outs[1])
            envs[2].step(envs[2].sample_actions(outs[2], 9))
    torch.cuda.synchronize(device)
    for other in envs[1:]:
        assert torch.equal(envs[0].grids(), other.grids())
        for name in ("pos", "accu", "rng_step", "done", "counts", "reward", "steps_elapsed"):
            assert torch.equal(getattr(envs[0], name), getattr(other, name)), name
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("N,K,chain", [(256, 40, False), (512, 24, False), (256, 1, False), (256, 40, True),
                                       (512, 16, True)])
def test_rollout_random_equals_step_random(device, N, K, chain):
    """gca_bulldozer_rollout_random (env.rollout_random): K env steps in one launch equal K env.step_random calls bit
    for bit -- every state tensor after the rollout, and the per-step actions, rewards and done flags against each
    step's own -- from a state where some envs burn out during the rollout and some are finished before it. chain: a
    Modify effect that can modify a cell twice in a row (TREE -> FIRE -> EMPTY), which takes the kernel's
    barrier-per-step path instead of the SOLO one."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    E = 192
    envs = [BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=31, env_offset=3, materialize_obs=False)
            for _ in range(2)]
    for env in envs:
        if chain:
            env.params.effect[3], env.params.effect[25] = 25, 0
        env.reset(seed=7)
        _dense_state(env, device, seed=5, p_fire=0.05)
        g = env.grids()
        g[:16] = torch.where(g[:16] == 25, torch.tensor(3, dtype=torch.uint8, device=device), g[:16])
        g[:16, N // 2, N // 2] = 25  # one fire: these burn out within a few CA steps
        env.buf[0].copy_(g)
        env.buf[1].copy_(g)
        env.parity.zero_()
        call("gca_count_cells", dev.ptr(env.buf[0]), E, N, N, 0, 3, 25, dev.ptr(env.counts), dev.stream_ptr(device))
        env.done[:4] = 1  # finished before the rollout
        gen = torch.Generator(device=device).manual_seed(11)
        env.accu.copy_(torch.rand(E, dtype=torch.float64, device=device, generator=gen) * 0.9)
    a_step = torch.zeros((E, 2), dtype=torch.int32, device=device)
    acts, rews, dones = [], [], []
    for _ in range(K):
        envs[0].step_random(9, a_step)
        acts.append(a_step.clone())
        rews.append(envs[0].reward.clone())
        dones.append(envs[0].done.clone())
    a_out = torch.full((K, E, 2), -1, dtype=torch.int32, device=device)
    r_out = torch.zeros((K, E), dtype=torch.float64, device=device)
    d_out = torch.full((K, E), 7, dtype=torch.uint8, device=device)
    envs[1].rollout_random(K, 9, a_out, r_out, d_out)
    torch.cuda.synchronize(device)
    assert torch.equal(envs[0].grids(), envs[1].grids())
    for name in ("pos", "accu", "rng_step", "done", "counts", "hit", "steps", "parity", "steps_elapsed"):
        assert torch.equal(getattr(envs[0], name), getattr(envs[1], name)), name
    assert torch.equal(torch.nan_to_num(envs[0].reward), torch.nan_to_num(envs[1].reward))
    assert torch.equal(a_out, torch.stack(acts))
    assert torch.equal(torch.nan_to_num(r_out), torch.nan_to_num(torch.stack(rews)))
    assert torch.equal(d_out, torch.stack(dones))
    assert int(envs[1].steps_elapsed.sum()) >= K * (E - 16)  # envs 4..15 may burn out during the rollout
    if K >= 40 and not chain:  # at 256^2 the single fires burn out within the rollout (~3 CA steps)
        assert int(envs[1].done[4:16].sum()) > 0
    before = [t.clone() for t in (envs[1].accu, envs[1].rng_step)]
    envs[1].rollout_random(0, 9)  # K = 0: nothing changes
    assert torch.equal(before[0], envs[1].accu) and torch.equal(before[1], envs[1].rng_step)


def _windy_pair(device, E, N, seed):
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    full = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=seed)
    shards = [BatchedForestFireBulldozerEnv(E // 2, N, N, device=device, seed=seed, env_offset=k * (E // 2))
              for k in range(2)]
    return full, shards


@pytest.mark.parametrize("N", [64, 512])
def test_sharded_windy_env_equals_unsharded(device, N):
    """two env objects owning envs [0, E/2) and [E/2, E) (env_offset) step bit-identically to one
    env owning all E — reset draws, CA rolls and device actions are keyed by the global env id."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E = 8
    full, shards = _windy_pair(device, E, N, seed=23)
    for env in (full, *shards):
        env.reset(seed=9)
    acts = [torch.zeros((env.num_envs, 2), dtype=torch.int32, device=device) for env in (full, *shards)]
    for s in range(40):
        for env, a in zip((full, *shards), acts):
            call("gca_random_actions", dev.ptr(a), env.num_envs, env.env_offset, 31, dev.ptr(env.rng_step),
                 dev.stream_ptr(device))
            env.step(a)
        assert torch.equal(torch.cat([acts[1], acts[2]]), acts[0])
        assert torch.equal(torch.cat([shards[0].grids(), shards[1].grids()]), full.grids()), f"step {s}"
        for name in ("pos", "accu", "rng_step", "done", "counts", "hit"):
            assert torch.equal(torch.cat([getattr(shards[0], name), getattr(shards[1], name)]), getattr(full, name))
        assert torch.equal(torch.nan_to_num(torch.cat([shards[0].reward, shards[1].reward])),
                           torch.nan_to_num(full.reward))


@pytest.mark.parametrize("parts", [True, False])
@pytest.mark.parametrize("H,W,E,steps", [(256, 256, 48, 120), (512, 512, 16, 120),
                                         # strips that do not split evenly over the parts -- a last
                                         # strip only partly filled (48, 100 at 256; 48, 80 at 512), parts with no
                                         # strip at all (16 and 80 at 512), the bulldozer in the last strip
                                         (48, 256, 32, 120), (100, 256, 32, 120), (16, 512, 16, 120),
                                         (48, 512, 16, 120), (80, 512, 16, 120)])
def test_fused_env_step_equals_three_kernel_step(device, H, W, E, steps, parts):
    """gca_bulldozer_step_fused (one launch per env step; `parts`: with the env's meeting slots, 2 / 4 workgroups per
    env meeting in one atomic, else one workgroup per env) leaves every env exactly as the gca_bulldozer_pre /
    gca_windy_step / gca_bulldozer_post sequence does: grids, parity, accu, steps, counts, pos, hit, reward, done,
    rng_step and steps_elapsed after every step, including envs that finish (no FIRE left) and are stepped again
    (graceful no-op), and under a hipGraph replay; the meeting slots are left zero."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv
    from gymca_amd.graph import StepGraph

    envs = [BatchedForestFireBulldozerEnv(E, H, W, device=device, seed=29, fused=f, materialize_obs=False,
                                          p_tree=0.55, p_empty=0.45) for f in (True, False)]
    assert envs[0].fused and not envs[1].fused
    if not parts:
        envs[0]._meet = None
    acts = [torch.zeros((E, 2), dtype=torch.int32, device=device) for _ in envs]
    # the bulldozer starts in the grid's last strip (the part that owns Modify is the last one with rows)
    start = np.stack([np.full(E, H - 2), (np.arange(E) * 37) % W], axis=1)
    for env in envs:
        env.reset(seed=4, positions=start)
        # a few envs start without FIRE: done after their first step, then stepped as finished envs
        g = env.grids()
        g[: E // 8][g[: E // 8] == 25] = 3
        env.buf[0].copy_(g)
        call("gca_count_cells", dev.ptr(env.buf[0]), E, H, W, 0, 3, 25, dev.ptr(env.counts), dev.stream_ptr(device))

    names = ("parity", "accu", "steps", "counts", "pos", "hit", "reward", "done", "rng_step", "steps_elapsed")

    def check(s):
        a, b = envs
        assert torch.equal(a.grids(), b.grids()), f"grids, step {s}"
        for name in names:
            ta, tb = getattr(a, name), getattr(b, name)
            assert torch.equal(torch.nan_to_num(ta), torch.nan_to_num(tb)), f"{name}, step {s}"

    def stepper(k):
        def f():
            call("gca_random_actions", dev.ptr(acts[k]), E, 0, 13, dev.ptr(envs[k].rng_step), dev.stream_ptr(device))
            envs[k].step(acts[k])
        return f

    ca_steps = 0
    for s in range(steps):
        for k in range(2):
            stepper(k)()
        ca_steps += int((envs[0].steps > 0).sum().item())
        check(s)
    assert ca_steps > steps * E // 60  # the CA really ran (~1 env step in 13 at 256^2, 25 at 512^2, live envs)
    assert int(envs[0].done[: E // 8].sum().item()) == E // 8
    graph = StepGraph(stepper(0), n_steps=8, device=device, warmup=0)
    for _ in range(3):
        graph.replay()
        for _ in range(8):
            stepper(1)()
    torch.cuda.synchronize(device)
    check("graph")
    if parts:
        assert int(envs[0]._meet.abs().sum().item()) == 0


def _dense_state(env, device, seed, p_fire):
    """A mid-episode-like state written into env: fires sprinkled at rate p_fire, accu uniform in [0, 1) (so a
    share of the envs steps the CA on every env step), counts recomputed."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    gen = torch.Generator(device=device).manual_seed(seed)
    g = env.grids()
    g[torch.rand(g.shape, device=device, generator=gen) < p_fire] = 25
    env.buf[0].copy_(g)
    env.parity.zero_()
    env.accu.copy_(torch.rand(env.num_envs, device=device, generator=gen, dtype=torch.float64))
    call("gca_count_cells", dev.ptr(env.buf[0]), env.num_envs, env.nrows, env.ncols, 0, 3, 25, dev.ptr(env.counts),
         dev.stream_ptr(device))


@pytest.mark.parametrize("N", [256, 512])
def test_fused_parts_at_bench_batch(device, N):
    """the bench's own Windy env step -- E = 1024, the parts kernel (2 / 4 workgroups per env
    meeting in one atomic) -- bit-identical to the one-workgroup fused kernel (meet = NULL) and to the three-kernel
    step, every state tensor after every one of 60 env steps with device random actions from a dense mid-episode state;
    the meeting slots are zero afterwards."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    E = 1024
    envs = [BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=41, fused=f, materialize_obs=False)
            for f in (True, True, False)]
    envs[1]._meet = None
    for env in envs:
        env.reset(seed=8)
        _dense_state(env, device, seed=123, p_fire=0.05)
    acts = [torch.zeros((E, 2), dtype=torch.int32, device=device) for _ in envs]
    names = ("parity", "accu", "steps", "counts", "pos", "hit", "reward", "done", "rng_step", "steps_elapsed")
    ca_steps = 0
    for s in range(60):
        for env, a in zip(envs, acts):
            call("gca_random_actions", dev.ptr(a), E, 0, 19, dev.ptr(env.rng_step), dev.stream_ptr(device))
            env.step(a)
        ca_steps += int((envs[0].steps > 0).sum().item())
        ref = envs[2]
        for k in (0, 1):
            assert torch.equal(envs[k].grids(), ref.grids()), f"grids, env object {k}, step {s}"
            for name in names:
                ta, tb = getattr(envs[k], name), getattr(ref, name)
                assert torch.equal(torch.nan_to_num(ta), torch.nan_to_num(tb)), f"{name}, env object {k}, step {s}"
    assert ca_steps > 60 * E // 40  # the CA really ran on many envs per step
    assert int(envs[0]._meet.abs().sum().item()) == 0


@pytest.mark.parametrize("H,W", [(8192, 256), (2048, 512), (2047, 512)])
def test_fused_parts_counts_on_tall_grids(device, H, W):
    """ADVICE / VERDICT r04: the parts kernel packs E / T / F counts into 20-bit fields. At 8192 x 256 and 2048 x 512
    (2^21 / 2^20 cells, an all-TREE grid) a packed field would carry into the next: gca_bulldozer_step_fused must take
    the one-workgroup kernel there (meet untouched); at 2047 x 512 (the largest parts grid) the packed counts sit just
    below 2^20. Counts, reward, done and grids equal the three-kernel step over 12 forced CA steps."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    E = 2
    envs = [BatchedForestFireBulldozerEnv(E, H, W, device=device, seed=7, fused=f, materialize_obs=False,
                                          p_tree=1.0, p_empty=0.0) for f in (True, False)]
    assert envs[0].fused
    acts = [torch.zeros((E, 2), dtype=torch.int32, device=device) for _ in envs]
    for env, a in zip(envs, acts):
        env.reset(seed=3)  # all TREE + the reset's one FIRE per env
        g = env.grids()
        g[:, H // 2, : W // 2] = 25  # a fire line: burns for many steps
        env.buf[0].copy_(g)
        call("gca_count_cells", dev.ptr(env.buf[0]), E, H, W, 0, 3, 25, dev.ptr(env.counts), dev.stream_ptr(device))
        a[:, 0] = 4  # stay
        a[:, 1] = 1  # shoot: Modify TREE -> EMPTY at the bulldozer
    assert int(envs[1].counts[:, 1].max().item()) >= H * W - W  # a TREE count near H*W
    for s in range(12):
        for env, a in zip(envs, acts):
            env.accu.fill_(0.9999)  # every env steps the CA on this env step
            env.step(a)
        fused, three = envs
        assert int(fused.steps.min().item()) == 1
        assert torch.equal(fused.grids(), three.grids()), f"grids, step {s}"
        for name in ("counts", "reward", "done", "hit", "pos", "parity", "rng_step"):
            ta, tb = getattr(fused, name), getattr(three, name)
            assert torch.equal(torch.nan_to_num(ta), torch.nan_to_num(tb)), f"{name}, step {s}"
        # counts are the grid's own
        g = fused.grids()
        exp = torch.stack([(g == v).sum(dim=(1, 2)) for v in (0, 3, 25)], dim=1).to(torch.int32)
        assert torch.equal(fused.counts, exp), f"counts vs grid, step {s}"
    assert int(envs[0]._meet.abs().sum().item()) == 0


def test_eager_step_action_forms_and_sampler(device):
    """The eager host path (pre-bound call): env.sample_actions == gca_random_actions with the same
    tag; the same actions given as the caller's int32 device tensor, an int64 device tensor, a numpy array or a flat
    (2E,) tensor step every env identically; the caller's int32 tensor is used in place (no copy)."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    E, N = 64, 256
    envs = [BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=5, materialize_obs=False) for _ in range(4)]
    for env in envs:
        env.reset(seed=2)
        _dense_state(env, device, seed=9, p_fire=0.05)
    mine = torch.zeros((E, 2), dtype=torch.int32, device=device)
    ref = torch.zeros((E, 2), dtype=torch.int32, device=device)
    for s in range(40):
        call("gca_random_actions", dev.ptr(ref), E, 0, 21, dev.ptr(envs[0].rng_step), dev.stream_ptr(device))
        got = envs[0].sample_actions(mine, 21)
        assert got is mine and torch.equal(mine, ref)
        forms = [mine, mine.to(torch.int64), mine.cpu().numpy(), mine.reshape(-1).clone()]
        for env, a in zip(envs, forms):
            env.step(a)
        assert envs[0]._action(mine) is mine
        for env in envs[1:]:
            assert torch.equal(env.grids(), envs[0].grids()), f"step {s}"
            for name in ("pos", "accu", "counts", "rng_step", "hit", "done"):
                assert torch.equal(getattr(env, name), getattr(envs[0], name)), f"{name} step {s}"


def test_rebind_after_replacing_a_state_tensor(device):
    """The fused step's pre-bound call holds the state tensors by address; an env whose tensor is REPLACED (not updated
    in place) and then rebind()-ed steps exactly like an env that never had it replaced."""
    import torch

    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    E, N = 32, 256
    envs = [BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=13, materialize_obs=False) for _ in range(2)]
    acts = [torch.zeros((E, 2), dtype=torch.int32, device=device) for _ in envs]
    for env in envs:
        env.reset(seed=1)
    for s in range(30):
        if s == 10:  # replace the accumulators and the counts of env 1 by copies, then rebind
            envs[1].accu = envs[1].accu.clone()
            envs[1].counts = envs[1].counts.clone()
            envs[1].rebind()
        for env, a in zip(envs, acts):
            env.step(env.sample_actions(a, 3))
        assert torch.equal(envs[0].grids(), envs[1].grids()), s
        for name in ("accu", "counts", "pos", "rng_step", "done"):
            assert torch.equal(getattr(envs[0], name), getattr(envs[1], name)), (name, s)
    assert envs[1]._ctx["time"] is envs[1].accu


def test_assigning_state_tensors_without_rebind(device):
    """VERDICT r05 next-3 / ADVICE r05: assigning fresh tensors to env.accu, env.pos and env.wind WITHOUT calling
    rebind() (the env's __setattr__ rebinds by itself), retyping the caller's cached action tensor in place (int32 ->
    int64 through .data) and re-pointing step_random's action_out: the env steps bit for bit like a freshly built env
    that had none of it done; a replacement of the wrong dtype / shape is refused."""
    import torch

    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    E, N = 64, 256
    envs = [BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=21, materialize_obs=False) for _ in range(2)]
    for env in envs:
        env.reset(seed=4)
        _dense_state(env, device, seed=12, p_fire=0.05)
    a0 = torch.zeros((E, 2), dtype=torch.int32, device=device)
    a1 = torch.zeros((E, 2), dtype=torch.int32, device=device)
    for s in range(36):
        if s == 8:
            envs[1].accu = envs[1].accu.clone()          # new allocations; the old ones may be freed now
            envs[1].pos = envs[1].pos.clone()
            envs[1].wind = envs[1].wind.clone()
            torch.cuda.empty_cache()
            scratch = [torch.full((E, 2), 7, dtype=torch.int32, device=device) for _ in range(64)]  # reuse freed blocks
            del scratch
        if s == 16:  # the cached action tensor retyped in place: converted, never read as int32 pairs
            a1.data = a1.data.to(torch.int64)
        envs[0].sample_actions(a0, 5)
        envs[1].sample_actions(envs[1]._act_buf, 5)
        a1.copy_(envs[1]._act_buf)  # the same actions, int32 or (from step 16) int64
        envs[0].step(a0)
        envs[1].step(a1)
        assert torch.equal(envs[0].grids(), envs[1].grids()), s
        for name in ("accu", "counts", "pos", "rng_step", "done", "reward", "wind"):
            assert torch.equal(getattr(envs[0], name), getattr(envs[1], name)), (name, s)
    assert envs[1]._ctx["time"] is envs[1].accu and envs[1]._ctx["position"] is envs[1].pos
    # step_random with its action buffer swapped for another tensor
    b0 = torch.zeros((E, 2), dtype=torch.int32, device=device)
    for s in range(8):
        out1 = torch.full((E, 2), -1, dtype=torch.int32, device=device)  # a new tensor every step
        envs[0].step_random(3, b0)
        envs[1].step_random(3, out1)
        assert torch.equal(b0, out1) and torch.equal(envs[0].grids(), envs[1].grids()), s
    with pytest.raises(ValueError):
        envs[1].accu = envs[1].accu.to(torch.float32)
    with pytest.raises(ValueError):
        envs[1].pos = torch.zeros((E, 3), dtype=torch.int32, device=device)
    with pytest.raises(ValueError):
        envs[1].step_random(3, b0.to(torch.int64))


@pytest.mark.parametrize("N,parts", [(256, True), (512, True), (256, False)])
def test_step_random_equals_sample_then_step(device, N, parts):
    """gca_bulldozer_step_fused_random (env.step_random): the random policy's action drawn inside the fused step is
    bit for bit env.sample_actions(a, seed) + env.step(a) -- every state tensor and the drawn actions after each of
    40 env steps from a dense state, with and without the meeting slots."""
    import torch

    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    E = 256
    envs = [BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=77, env_offset=5, materialize_obs=False)
            for _ in range(2)]
    for env in envs:
        if not parts:
            env._meet = None
        env.reset(seed=6)
        _dense_state(env, device, seed=31, p_fire=0.05)
    a_ref = torch.zeros((E, 2), dtype=torch.int32, device=device)
    a_got = torch.full((E, 2), -1, dtype=torch.int32, device=device)
    ca = 0
    for s in range(40):
        envs[0].step(envs[0].sample_actions(a_ref, 17))
        envs[1].step_random(17, a_got)
        ca += int((envs[1].steps > 0).sum().item())
        assert torch.equal(a_got, a_ref), s
        assert torch.equal(envs[0].grids(), envs[1].grids()), s
        for name in ("parity", "accu", "steps", "counts", "pos", "hit", "done", "rng_step", "steps_elapsed"):
            assert torch.equal(getattr(envs[0], name), getattr(envs[1], name)), (name, s)
        assert torch.equal(torch.nan_to_num(envs[0].reward), torch.nan_to_num(envs[1].reward)), s
    assert ca > 40 * E // 40
