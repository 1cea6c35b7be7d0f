"""The batched env's reference API on the GPU: reset / stateless_step(action, obs, info) /
conditional_reset(step_tuple, action), driven the way the reference's PPO rollout drives it
(agents/jax_ppo.py:504-671: obs/info of each call are threaded into the next), checked step by step
against the oracle composition (C oracle CA step + wind change, numpy Move/Modify/time bookkeeping,
oracle/observation.py for the RGB frames, the reference's conditional_reset rules
advanced_bulldozer.py:422-518)."""
import numpy as np
import pytest

from alex_cases import make_case
from oracle import alex_c
from oracle import observation as ob
from oracle.windy import move

pytestmark = pytest.mark.gpu


def _host(x):
    return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)


class OracleEnv:
    """Per-env state of AdvancedForestFireBulldozerEnv restated on the host."""

    def __init__(self, env, grid, age, veg, den, dous, widx, time_step, is_night):
        self.E, self.N = env.num_envs, env.nrows
        self.p, self.ep = env.alex_params, env.env_params
        self.ps = env.p_slope_planes().cpu().numpy()
        init = env._initial
        self.g0, self.a0 = _host(init["grid"]).copy(), _host(init["age"]).copy()
        self.pos0, self.w0 = _host(init["pos"]).copy(), _host(init["wind_index"]).copy()
        self.g, self.a, self.veg, self.den, self.dous = grid.copy(), age.copy(), veg, den, dous.copy()
        self.widx = widx.copy()
        self.pos = self.pos0.copy()
        self.accu = np.zeros(self.E, np.float32)
        self.rs = np.zeros(self.E, np.uint32)
        self.ts, self.night = time_step.copy(), is_night.copy()
        self.steps = np.zeros(self.E, np.float32)
        self.racc = np.zeros(self.E, np.float32)
        self.rgb = None

    @staticmethod
    def award(counts):
        return -(counts[:, 2].astype(np.float32) / (counts[:, 1:].sum(1).astype(np.float32) + np.float32(1e-8)))

    def step(self, act):
        E, N, ep = self.E, self.N, self.ep
        self.g, self.a, counts, _ = alex_c.alex_step(self.p, self.g, self.a, self.veg, self.den, self.dous, self.ps,
                                                     self.widx, rng_step=self.rs)
        self.widx = alex_c.wind_change(np.float32(0.06), 8, ep.seed, 0, self.rs, self.widx)
        night_pre = self.night.copy()
        for e in range(E):
            t = np.float32(np.float32(ep.t_move[act[e, 0]]) + np.float32(ep.t_shoot[act[e, 1]])) + np.float32(ep.t_any)
            na = np.float32(self.accu[e] + t)
            self.accu[e] = np.float32(na - np.float32(np.trunc(na)))
            self.pos[e] = move(self.pos[e], int(act[e, 0]), N, N)
            if act[e, 1] == 1:
                self.dous[e, self.pos[e][0], self.pos[e][1]] = 1
            self.ts[e] += 1
            if self.ts[e] % 400 == 0:
                self.night[e] = 1 - self.night[e]
        self.rs = self.rs + np.uint32(1)
        self.reward = self.award(counts)
        self.term = counts[:, 2] == 0
        self.steps = self.steps + np.float32(1)
        self.racc = (self.racc + self.reward).astype(np.float32)
        self.rgb = np.stack([ob.step_observation(self.g[e].astype(np.int32), tuple(self.pos[e]),
                                                 ob_flags(act[e, 2]), int(night_pre[e]), self.dous[e].astype(np.int32),
                                                 True, True)[0] for e in range(E)])

    def conditional_reset(self, act):
        for e in np.flatnonzero(self.term):
            # observation first: initial grid / position, the step's dousing and is_night (:455-481)
            self.rgb[e] = ob.step_observation(self.g0[e].astype(np.int32), tuple(self.pos0[e]), ob_flags(act[e, 2]),
                                              int(self.night[e]), self.dous[e].astype(np.int32), True, True)[0]
            self.g[e], self.a[e], self.dous[e] = self.g0[e], self.a0[e], 0
            self.widx[e], self.pos[e], self.accu[e], self.rs[e] = self.w0[e], self.pos0[e], 0, 0
            self.steps[e], self.racc[e] = 0, 0
            c = np.array([[np.sum(self.g0[e] == k) for k in range(3)]])
            self.reward[e] = self.award(c)[0]
        self.term = np.zeros(self.E, bool)


def ob_flags(choice):
    from gymca_amd.forest_fire.bulldozer.observation import EXTENSION_LOOKUP

    return EXTENSION_LOOKUP[int(np.clip(choice, 0, len(EXTENSION_LOOKUP) - 1))]


def _check(env_out, orc, s):
    obs, reward, term, trunc, info = env_out
    rgb, ctx = obs
    pe = ctx["per_env_context"]
    assert np.array_equal(_host(pe["true_grid"]), orc.g), f"grid, step {s}"
    assert np.array_equal(_host(pe["fire_age"]), orc.a), f"age, step {s}"
    assert np.array_equal(_host(pe["wind_index"]), orc.widx), f"wind, step {s}"
    assert np.array_equal(_host(pe["dousing_count"]), orc.dous), f"dousing, step {s}"
    assert np.array_equal(_host(pe["time_step"]), orc.ts) and np.array_equal(_host(pe["is_night"]), orc.night)
    assert np.array_equal(_host(pe["key"]).view(np.uint32), orc.rs)
    assert np.array_equal(_host(ctx["position"]), orc.pos) and np.array_equal(_host(ctx["time"]), orc.accu)
    assert np.array_equal(_host(reward), orc.reward) and np.array_equal(_host(info["reward"]), orc.reward)
    assert np.array_equal(_host(term), orc.term) and np.array_equal(_host(info["terminated"]), orc.term)
    assert not _host(trunc).any() and not _host(info["TimeLimit.truncated"]).any()
    assert np.array_equal(_host(info["steps_elapsed"]), orc.steps)
    assert np.array_equal(_host(info["reward_accumulated"]), orc.racc), f"reward_accumulated, step {s}"
    assert rgb.dtype.is_floating_point and tuple(rgb.shape) == orc.rgb.shape
    assert np.array_equal(_host(rgb), orc.rgb), f"rgb, step {s}"


@pytest.mark.parametrize("N", [32, 256])  # 32: edge slope layout; 256: packed (the bench's)
def test_ppo_style_rollout_matches_oracle(device, N):
    """reset -> (stateless_step -> conditional_reset) x 10 with obs/info threaded between the calls, the
    initial mid-episode state handed in through obs (adopted), some envs burning out and re-injected, and a
    day/night toggle inside the run (time_step starts at 398)."""
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E = 6
    env = AdvancedForestFireBulldozerEnv(N, N, key=17, num_envs=E, use_hidden=True, device=device,
                                         enable_extensions=True)
    obs, info = env.reset()
    assert tuple(obs[0].shape) == (E, N, N, 3) and obs[0].dtype == torch.float32  # the reference's RGB obs
    case = make_case(E, N, N, 3, dousing_p=0.0)
    grid, age = case["grid"].copy(), case["age"].copy()
    for e in (0, 3):  # these envs burn out after two steps: one fire of age 2 on an empty grid
        grid[e], age[e] = 0, 0
        grid[e, N // 2, N // 3], age[e, N // 2, N // 3] = 2, 2
    veg, den = np.clip(case["veg"], 1, 5), np.clip(case["den"], 1, 5)
    ts = np.full(E, 398, np.int32)
    night = np.array([0, 1, 0, 1, 0, 0], np.int32)
    # a foreign (host) context: stateless_step must adopt it
    ctx = {"per_env_context": {"true_grid": grid, "fire_age": age, "vegetation": veg, "density": den,
                               "dousing_count": np.zeros_like(grid), "wind_index": case["widx"], "time_step": ts,
                               "is_night": night, "key": np.zeros(E, np.int32)},
           "position": obs[1]["position"].cpu().numpy(), "time": np.zeros(E, np.float32)}
    obs = (obs[0], ctx)
    orc = OracleEnv(env, grid, age, veg, den, np.zeros_like(grid), case["widx"], ts, night)
    rng = np.random.default_rng(4)
    resets = 0
    for s in range(10):
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E), rng.integers(0, 3, E)], axis=1).astype(np.int32)
        act_d = torch.as_tensor(act, device=device)
        out = env.stateless_step(act_d, obs, info)
        orc.step(act)
        _check(out, orc, s)
        resets += int(orc.term.sum())
        out = env.conditional_reset(out, act_d)  # live envs keep their step observation (checked via orc.rgb)
        orc.conditional_reset(act)
        _check(out, orc, s)
        obs, info = out[0], out[4]
    assert resets >= 2  # envs 0 and 3 were re-injected at least once


def test_stateless_step_from_an_older_obs(device):
    """The reference is functional: stepping from a stored obs/info reproduces the step taken from it the
    first time (the RNG key travels in the context), even after the env moved on."""
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 4, 64
    env = AdvancedForestFireBulldozerEnv(N, N, key=5, num_envs=E, use_hidden=True, device=device,
                                         enable_extensions=True)
    obs, info = env.reset()
    rng = np.random.default_rng(1)
    acts = [torch.as_tensor(np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E), rng.integers(0, 3, E)], 1),
                            device=device, dtype=torch.int32) for _ in range(6)]
    snap = None
    for s in range(6):
        if s == 3:  # host snapshot of the obs/info going into step 3
            snap = (obs[0].cpu().numpy(), {"per_env_context": {k: (None if v is None else v.cpu().numpy())
                                                               for k, v in obs[1]["per_env_context"].items()
                                                               if k not in ("slope", "altitude")},
                                           "position": obs[1]["position"].cpu().numpy(),
                                           "time": obs[1]["time"].cpu().numpy()}), \
                {k: v.cpu().numpy() for k, v in info.items()}
        obs, r, term, trunc, info = env.stateless_step(acts[s], obs, info)
        if s == 3:
            want = (obs[0].cpu().numpy(), obs[1]["per_env_context"]["true_grid"].cpu().numpy(),
                    obs[1]["per_env_context"]["fire_age"].cpu().numpy(), r.cpu().numpy(),
                    info["steps_elapsed"].cpu().numpy(), info["reward_accumulated"].cpu().numpy())
    obs2, r2, _, _, info2 = env.stateless_step(acts[3], snap[0], snap[1])
    got = (obs2[0].cpu().numpy(), obs2[1]["per_env_context"]["true_grid"].cpu().numpy(),
           obs2[1]["per_env_context"]["fire_age"].cpu().numpy(), r2.cpu().numpy(),
           info2["steps_elapsed"].cpu().numpy(), info2["reward_accumulated"].cpu().numpy())
    for a, b in zip(got, want):
        assert np.array_equal(a, b)


def test_reference_position_formats(device):
    """pos_bull as a list of per-env (r, c), pos_fire as per-env lists of fire cells
    (advanced_bulldozer.py:664-700); a malformed pos_bull raises instead of unpacking transposed."""
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 3, 32
    fires = [[(10, 10), (10, 9)], [(5, 5)], [(7, 7), (7, 6), (-1, 0)]]
    env = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=device,
                                         pos_bull=[(1, 2), (3, 4), (5, 6)], pos_fire=fires)
    obs, _ = env.reset()
    assert env.pos.cpu().numpy().tolist() == [[1, 2], [3, 4], [5, 6]]
    g, a = env.grid[env.cur].cpu().numpy(), env.age[env.cur].cpu().numpy()
    for e, cells in enumerate(fires):
        want = np.zeros((N, N), bool)
        for r, c in cells:
            want[r % N, c % N] = True
        assert np.array_equal(g[e] == 2, want)
        assert np.all(a[e][want] == (N + N // 2) * 2) and np.all(a[e][~want] == 0)
    env2 = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=2, use_hidden=False, device=device,
                                          pos_bull=[(1, 2), (3, 4)])
    env2.reset()
    assert env2.pos.cpu().numpy().tolist() == [[1, 2], [3, 4]]
    with pytest.raises(ValueError):
        AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=3, use_hidden=False, device=device,
                                       pos_bull=[(1, 2), (3, 4)])
    with pytest.raises(ValueError):
        AdvancedForestFireBulldozerEnv(N, 2 * N, key=1, num_envs=3, use_hidden=False, device=device)  # rgb: square


@pytest.mark.parametrize("N,hidden", [(64, False), (64, True), (256, True)])
def test_sharded_advanced_env_equals_unsharded(device, N, hidden):
    """SURVEY.md §8e for the Alexandridis env: envs [0, E/2) and [E/2, E) in two env objects (env_offset) give
    bit-identical trajectories — grid, ages, wind, dousing, position, reward, RGB observation — to one env
    object with all E (reset draws, hidden layers (hidden_rng="philox") and every Philox counter carry the
    global env id)."""
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E = 6
    kw = dict(key=41, use_hidden=hidden, device=device, enable_extensions=True,
              hidden_rng="philox" if hidden else None)
    full = AdvancedForestFireBulldozerEnv(N, N, num_envs=E, **kw)
    shards = [AdvancedForestFireBulldozerEnv(N, N, num_envs=E // 2, env_offset=k * (E // 2), **kw) for k in range(2)]
    envs = (full, *shards)
    state = [env.reset() for env in envs]  # (obs, info) per env object
    rng = np.random.default_rng(8)
    cat = lambda f: torch.cat([f(o) for o in outs[1:]])
    for s in range(20):
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E), rng.integers(0, 3, E)], 1).astype(np.int32)
        acts = (act, act[:E // 2], act[E // 2:])
        outs = [env.stateless_step(a, *st) for env, a, st in zip(envs, acts, state)]
        outs = [env.conditional_reset(o, torch.as_tensor(a, device=device)) for env, o, a in zip(envs, outs, acts)]
        state = [(o[0], o[4]) for o in outs]
        o0 = outs[0]
        assert torch.equal(cat(lambda o: o[0][0]), o0[0][0]), f"rgb, step {s}"
        for key in ("true_grid", "fire_age", "wind_index", "dousing_count", "vegetation", "density"):
            assert torch.equal(cat(lambda o: o[0][1]["per_env_context"][key]), o0[0][1]["per_env_context"][key]), key
        assert torch.equal(cat(lambda o: o[0][1]["position"]), o0[0][1]["position"])
        assert torch.equal(cat(lambda o: o[1]), o0[1]) and torch.equal(cat(lambda o: o[2]), o0[2])
