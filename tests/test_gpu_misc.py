"""GPU: count_cells, Move/Modify drop-ins vs the reference's golden rows, Drossel-Schwabl and
the helicopter env vs the seeded reference, reset_where."""
import numpy as np
import pytest

from _contract import assert_operator

pytestmark = pytest.mark.gpu


def test_count_cells_matches_numpy(device):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    for E, H, W in [(3, 17, 29), (5, 256, 256), (2, 1, 1), (4, 64, 48)]:
        g = np.random.default_rng(E).choice(np.array([0, 3, 25, 7], np.uint8), size=(E, H, W))
        gd = torch.as_tensor(g, device=device)
        c = torch.zeros((E, 3), dtype=torch.int32, device=device)
        call("gca_count_cells", dev.ptr(gd), E, H, W, 0, 3, 25, dev.ptr(c), dev.stream_ptr())
        exp = np.stack([(g == v).sum(axis=(1, 2)) for v in (0, 3, 25)], axis=1)
        assert np.array_equal(c.cpu().numpy(), exp)


def test_move_modify_dropins_match_reference_rows(golden, device):
    from gymca_amd.forest_fire.operators import Modify, Move, MoveModify

    sets = {"up": {0, 1, 2}, "down": {6, 7, 8}, "left": {0, 3, 6}, "right": {2, 5, 8}, "not_move": {4}}
    mm = MoveModify(Move(sets, backend="hip"), Modify({3: 0}, backend="hip"))  # the kernel, not the host build
    rows = golden("move_modify")["rows"]
    rng = np.random.default_rng(0)
    for H, W, r, c, a, shoot, pr, pc, before, after, hit in rows[rng.choice(len(rows), 300, replace=False)]:
        grid = np.zeros((H, W), dtype=np.int64)
        grid[pr, pc] = before
        g, pos = mm(grid, (int(a), int(shoot)), np.array([r, c]))
        assert tuple(pos) == (pr, pc) and g is grid and grid[pr, pc] == after and mm.modify.hit == bool(hit)


def test_move_modify_device_grid_through_pinned_staging(golden, device):
    """The device-grid call (DeviceIO: one pinned upload, one read-back) on the same golden rows, and a start
    position outside the grid refused on the host before any launch."""
    import torch

    from gymca_amd._lib import GCAError
    from gymca_amd.forest_fire.operators import Modify, Move, MoveModify

    sets = {"up": {0, 1, 2}, "down": {6, 7, 8}, "left": {0, 3, 6}, "right": {2, 5, 8}, "not_move": {4}}
    mm = MoveModify(Move(sets), Modify({3: 0}))
    rows = golden("move_modify")["rows"]
    rng = np.random.default_rng(1)
    for H, W, r, c, a, shoot, pr, pc, before, after, hit in rows[rng.choice(len(rows), 200, replace=False)]:
        grid = torch.zeros((H, W), dtype=torch.uint8, device=device)
        grid[pr, pc] = int(before)
        g, pos = mm(grid, (int(a), int(shoot)), np.array([r, c]))
        assert g is grid and tuple(pos) == (pr, pc) and pos.dtype == np.int64
        assert int(grid[pr, pc]) == after and mm.modify.hit == bool(hit)
    grid = torch.zeros((4, 4), dtype=torch.uint8, device=device)
    with pytest.raises(GCAError):
        mm(grid, (4, 1), np.array([4, 0]))  # not_move from row 4 of a 4-row grid
    grid[3, 0] = 3
    g, pos = mm(grid, (1, 1), np.array([4, 0]))  # up from row 4 lands on row 3, as in the host build
    assert tuple(pos) == (3, 0) and int(grid[3, 0]) == 0 and mm.modify.hit


def test_positions_outside_the_grid_write_nothing(device):
    """Out-of-grid positions: the C-ABI kernels write nothing (the raw call, no host check in between), and the
    env entry points that take a caller's positions refuse them before any launch."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv, BatchedForestFireBulldozerEnv
    from gymca_amd.forest_fire.operators.move_modify import make_params

    E, H, W = 4, 8, 8
    p = make_params({"up": {0, 1, 2}, "down": {6, 7, 8}, "left": {0, 3, 6}, "right": {2, 5, 8}}, {3: 0})
    grid = torch.full((E, H, W), 3, dtype=torch.uint8, device=device)  # an unguarded write would land in env e +- 1
    act = torch.tensor([[4, 1]] * E, dtype=torch.int32, device=device)  # not_move, shoot
    pos = torch.tensor([[H, 0], [-1, 3], [2, W], [3, -1]], dtype=torch.int32, device=device)
    hit = torch.ones(E, dtype=torch.uint8, device=device)
    call("gca_move_modify", p, dev.ptr(act), dev.ptr(pos), dev.ptr(grid), H, W, dev.ptr(hit), E, dev.stream_ptr())
    torch.cuda.synchronize()
    assert bool((grid == 3).all()) and int(hit.sum()) == 0
    env = BatchedForestFireBulldozerEnv(2, 256, 256, device=device, materialize_obs=False)
    with pytest.raises(ValueError):
        env.reset(positions=[[0, 0], [256, 3]])
    adv = AdvancedForestFireBulldozerEnv(16, 16, key=1, num_envs=2, use_hidden=False, device=device, observation="grid")
    obs, info = adv.reset()
    with pytest.raises(ValueError):
        adv.set_state(position=[[0, 0], [3, 16]])
    with pytest.raises(ValueError):
        adv.set_state(wind_index=[0, len(adv._winds)])
    adv.stateless_step(torch.zeros((2, 3), dtype=torch.int32, device=device), obs, info)  # the valid call runs
    bad = dict(obs[1])
    bad["position"] = torch.tensor([[0, 0], [16, 1]], dtype=torch.int32, device=device)
    with pytest.raises(ValueError):
        adv.stateless_step(torch.zeros((2, 3), dtype=torch.int32, device=device), (obs[0], bad), info)
    with pytest.raises(ValueError):
        AdvancedForestFireBulldozerEnv(16, 16, key=1, num_envs=2, use_hidden=False, device=device,
                                       pos_bull=[(0, 0), (0, 16)]).reset()


def test_dropin_bulldozer_one_readback_per_step(device):
    """ForestFireBulldozerEnv on the device reads the count, Move / Modify's position and hit and the observation
    back in one synchronisation: the values equal what the env state holds afterwards, each step returns its own
    position array, and obs_device=True returns the device grid."""
    import torch

    from gymca_amd.forest_fire.bulldozer import ForestFireBulldozerEnv

    for obs_device in (False, True):
        env = ForestFireBulldozerEnv(32, 32, obs_device=obs_device)
        env.reset(seed=3)
        seen = []
        for s in range(40):
            obs, rew, term, trunc, info = env.step(np.array([s % 9, s % 2]))
            grid, (_, pos, _) = obs
            assert torch.is_tensor(grid) == obs_device
            host = grid.cpu().numpy() if obs_device else grid
            assert np.array_equal(host, env.grid.cpu().numpy())
            assert pos.shape == (2,) and np.all((0 <= pos) & (pos < 32)) and all(p is not pos for p in seen)
            assert np.array_equal(pos, env.context[1]) and isinstance(info["hit"], bool)
            counts = env.count_cells(env.grid)
            assert term == (counts[25] == 0)
            if not term:
                assert rew == -(counts[25] / (counts[3] + counts[25]))
            seen.append(pos)
            if term:
                break
        assert env.move_modify._io.pending is None and not env.move_modify._io.in_flight


def test_dropin_bulldozer_hit_resolved_on_the_count_fallback(device):
    """with the one-read-back path off (env.one_readback = False: the separate count_cells path, as for a
    grid the DeviceIO cannot read), Move / Modify's deferred read-back is resolved before CAEnv.step calls _report, so
    info['hit'] is THIS step's hit: at every _report no read is pending, and info['hit'] equals modify.hit after the
    step."""
    from gymca_amd.forest_fire.bulldozer import ForestFireBulldozerEnv

    env = ForestFireBulldozerEnv(32, 32)
    env.one_readback = False
    env.reset(seed=5)
    orig = env._report
    pending_at_report = []

    def report():
        pending_at_report.append(env.move_modify._io.pending is not None)
        return orig()

    env._report = report
    hits = 0
    for s in range(60):
        _, _, term, _, info = env.step(np.array([s % 9, 1]))
        assert info["hit"] == env.modify.hit, s
        hits += int(info["hit"])
        if term:
            break
    assert pending_at_report and not any(pending_at_report)
    assert hits > 0


def test_modify_cyclic_effects_reference_test(device):
    """test_move_modify.py:92-125: cyclic effects on a 3-state grid, in place."""
    from gymca_amd.forest_fire.operators import Modify
    from gymca_amd.grid_space import GridSpace

    effects = {s: range(3)[s - 2] for s in range(3)}
    modify = Modify(effects, backend="hip")
    assert_operator(modify, strict=False)
    gs = GridSpace(n=3, shape=(3, 3))
    rng = np.random.default_rng(2)
    for _ in range(16):
        for action in (True, False):
            grid = gs.sample()
            pos = rng.integers(0, 3, 2)
            target = grid[pos[0], pos[1]]
            g, p = modify(grid, action, pos)
            assert g[pos[0], pos[1]] == (effects[target] if action else target) and np.all(p == pos)


def test_drossel_dropin_matches_seeded_reference(golden, device):
    from gymca_amd.forest_fire.operators import ForestFire

    d = golden("drossel")
    for i in range(int(d["n"])):
        op = ForestFire(0, 1, 2, backend="hip")
        op.seed(int(d[f"c{i}_seed"]))
        out, _ = op.update(d[f"c{i}_grid"].astype(np.int64), None, d[f"c{i}_p"])
        assert np.array_equal(out, d[f"c{i}_out"]), f"case {i}"


def test_helicopter_env_replays_seeded_reference(golden, device):
    from gymca_amd.forest_fire.helicopter import ForestFireHelicopterEnv

    d = golden("helicopter")
    env = ForestFireHelicopterEnv(5, 5, backend="hip")  # the kernels (auto would take the host build at 5x5)
    env.reset(seed=7)
    env.cellular_automaton.seed(int(d["seed"]))
    env.grid = d["grid0"].astype(np.int64)
    ca_params, pos, freeze = env.context
    env.context = (ca_params, pos, freeze)
    for s in range(len(d["grids"])):
        obs, rew, term, trunc, info = env.step(s % 9)
        grid, (cp, pos, fr) = obs
        assert np.array_equal(grid, d["grids"][s]), f"step {s}"
        exp = d["recs"][s]
        assert np.isclose(rew, exp[0], rtol=0, atol=1e-15) and (pos[0], pos[1], int(fr)) == (exp[1], exp[2], exp[3])
        assert bool(info["hit"]) == bool(exp[4])


def test_reset_where(device):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, H, W = 5, 19, 23
    g = torch.randint(0, 3, (E, H, W), dtype=torch.uint8, device=device)
    g0 = torch.randint(0, 3, (E, H, W), dtype=torch.uint8, device=device)
    done = torch.tensor([0, 1, 0, 1, 1], dtype=torch.uint8, device=device)
    ref = torch.where(done.bool()[:, None, None], g0, g)
    pos = torch.zeros((E, 2), dtype=torch.int32, device=device)
    pos0 = torch.ones((E, 2), dtype=torch.int32, device=device)
    call("gca_reset_where", dev.ptr(done), E, H, W, dev.ptr(g), dev.ptr(g0), None, None, None, None, None, dev.ptr(pos),
         dev.ptr(pos0), None, None, None, dev.stream_ptr())
    assert torch.equal(g, ref) and int(done.sum()) == 0
    assert pos[:, 0].tolist() == [0, 1, 0, 1, 1]
