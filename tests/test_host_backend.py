"""CPU: the host build of the C-ABI (libgca_cpu.so, csrc/gca_cpu.cpp) — exports, Philox KAT — and the product
paths that dispatch to it (gymca_amd/_backend.py): Move / Modify / MoveModify on host arrays against the
reference's golden rows, the JAX-contract operators' semantics (move_modify_jax.py:39-157, repeat_ca_jax.py:34-71),
Drossel-Schwabl and the 5x5 helicopter env (BASELINE config 1) against the seeded reference runs. No GPU."""
import numpy as np
import pytest

SETS = {"up": {0, 1, 2}, "down": {6, 7, 8}, "left": {0, 3, 6}, "right": {2, 5, 8}, "not_move": {4}}


def test_host_library_exports_its_symbols():
    from gymca_amd import _lib

    lib = _lib.load_cpu()
    for name in _lib.CPU_SYMBOLS:
        assert hasattr(lib, name), name
        assert name in _lib.EXPORTED_SYMBOLS  # the same C-ABI as libgca_hip.so
    assert lib.gca_version() == 1


def test_host_philox_kat():
    from gymca_amd import _lib
    from test_rng_and_math import KAT

    for ctr, key, exp in KAT:
        c = np.array([ctr], dtype=np.uint32)
        out = np.zeros_like(c)
        _lib.call_cpu("gca_philox", c.ctypes.data, key[0], key[1], out.ctypes.data, 1, None)
        assert tuple(int(v) for v in out[0]) == exp


def test_backend_choice_rule():
    from gymca_amd import GCAError, _backend

    assert _backend.choose("auto", False, 25) == "cpu"
    assert _backend.choose("auto", False, 256 * 256) == "hip"
    assert _backend.choose("auto", False, 256 * 256, o1=True) == "cpu"
    assert _backend.choose("auto", True, 25) == "hip"
    assert _backend.choose("hip", False, 25) == "hip"
    with pytest.raises(GCAError):
        _backend.choose("cpu", True, 25)
    with pytest.raises(ValueError):
        _backend.choose("gpu", False, 25)


@pytest.mark.parametrize("dtype", [np.int64, np.uint8, np.int32])
def test_host_move_modify_matches_reference_rows(golden, dtype):
    from gymca_amd.forest_fire.operators import Modify, Move, MoveModify

    mm = MoveModify(Move(SETS, backend="cpu"), Modify({3: 0}, backend="cpu"))
    rows = golden("move_modify")["rows"]
    for H, W, r, c, a, shoot, pr, pc, before, after, hit in rows:
        grid = np.zeros((H, W), dtype=dtype)
        grid[pr, pc] = before
        g, pos = mm(grid, (int(a), int(shoot)), np.array([r, c]))
        assert tuple(pos) == (pr, pc) and g is grid and grid[pr, pc] == after and mm.modify.hit == bool(hit)
        assert int((grid != 0).sum()) == int(after != 0)  # nothing else touched


def test_host_modify_refuses_positions_outside_the_grid():
    """Every host path refuses a caller's position outside the grid like the C and HIP gca_move_modify (GCA_ERR_ARG):
    numpy indexing would wrap a negative index and modify the wrong cell. The large-grid path (int64,
    above HOST_MAX_CELLS) and the small-grid copy path both."""
    from gymca_amd import GCAError
    from gymca_amd.forest_fire.operators import Modify

    for shape in ((80, 80), (8, 8)):
        for pos in ((-1, 5), (5, -1), (shape[0], 0), (0, shape[1])):
            grid = np.full(shape, 3, dtype=np.int64)
            with pytest.raises(GCAError):
                Modify({3: 0}, backend="cpu")(grid, 1, np.array(pos))
            assert (grid == 3).all()  # nothing written


def test_device_path_position_check_restates_the_host_move():
    """The device Move / Modify path validates a caller's out-of-grid start on the host with _moved before launching;
    _moved must agree with the host build's Move for every action id and start around small grids."""
    from gymca_amd.forest_fire.operators.move_modify import _moved, _run_host, make_params

    sets = {"up": {0, 1, 2}, "down": {6, 7, 8}, "left": {0, 3, 6}, "right": {2, 5, 8}}
    p = make_params(sets, {3: 0})
    for H, W in [(4, 4), (5, 7), (1, 1)]:
        for r in range(-2, H + 2):
            for c in range(-2, W + 2):
                for a in range(-1, 33):
                    exp = _run_host(p, np.zeros((H, W), np.uint8), (a, 0), (r, c), with_grid=False)[0]
                    assert tuple(exp) == _moved(p, a, r, c, H, W), (H, W, r, c, a)


def test_host_modify_large_grid_touches_one_cell():
    """O(1): a 512x512 int64 grid is modified in place at one cell (no whole-grid copy)."""
    from gymca_amd.forest_fire.operators import Modify

    grid = np.full((512, 512), 3, dtype=np.int64)
    g, pos = Modify({3: 0})(grid, True, np.array([100, 200]))
    assert g is grid and grid[100, 200] == 0 and int((grid == 0).sum()) == 1


def test_modify_cyclic_effects_reference_test_host():
    """test_move_modify.py:92-125 on the host backend."""
    from gymca_amd.forest_fire.operators import Modify
    from gymca_amd.grid_space import GridSpace

    effects = {s: range(3)[s - 2] for s in range(3)}
    modify = Modify(effects, backend="cpu")
    gs = GridSpace(n=3, shape=(3, 3))
    rng = np.random.default_rng(2)
    for _ in range(16):
        for action in (True, False):
            grid = gs.sample()
            pos = rng.integers(0, 3, 2)
            target = grid[pos[0], pos[1]]
            g, p = modify(grid, action, pos)
            assert g[pos[0], pos[1]] == (effects[target] if action else target) and np.all(p == pos)


def test_modify_jax_sets_dousing_functionally():
    """ModifyJax.update(grid, action, context, per_env_context) (move_modify_jax.py:102-114): dousing_count[r, c]
    = 1 on action == 1 in a NEW array stored into the given dict; grid, position and the old array untouched."""
    from gymca_amd.forest_fire.operators import ModifyJax

    op = ModifyJax({})
    grid = np.arange(16, dtype=np.float32).reshape(4, 4)
    for dt in (np.int32, np.uint8, np.float32):
        d0 = np.zeros((4, 4), dt)
        d0[0, 0] = 1
        pe = {"dousing_count": d0, "other": 7}
        g, ctx, pe2 = op(grid, 1, np.array([2, 3]), pe)
        assert g is grid and pe2 is pe and np.array_equal(ctx, [2, 3])
        assert pe["dousing_count"] is not d0 and d0.sum() == 1 and pe["dousing_count"].dtype == dt
        assert np.argwhere(pe["dousing_count"]).tolist() == [[0, 0], [2, 3]]
        pe = {"dousing_count": d0}
        op(grid, 0, np.array([2, 3]), pe)
        assert np.array_equal(pe["dousing_count"], d0)


def test_move_modify_jax_contract_and_vmapped_form():
    """MoveModifyJax.update(grid, subactions, position, per_env_context) -> (grid, position, per_env_context)
    (:148-157): Move, then ModifyJax at the NEW position; the leading env axis is the vmapped call."""
    from gymca_amd.forest_fire.operators import MoveJax, MoveModifyJax, ModifyJax
    from oracle.windy import move

    mm = MoveModifyJax(MoveJax(SETS), ModifyJax({}))
    rng = np.random.default_rng(0)
    E, H, W = 16, 7, 9
    pos = np.stack([rng.integers(0, H, E), rng.integers(0, W, E)], axis=1)
    moves, shots = rng.integers(0, 9, E), rng.integers(0, 2, E)
    d = np.zeros((E, H, W), np.int32)
    g, npos, pe = mm(np.zeros((E, H, W)), (moves, shots), pos, {"dousing_count": d})
    want = np.array([move(tuple(p), int(m), H, W) for p, m in zip(pos, moves)])
    assert np.array_equal(npos, want) and d.sum() == 0
    exp = np.zeros_like(d)
    for e in range(E):
        if shots[e]:
            exp[e, want[e][0], want[e][1]] = 1
    assert np.array_equal(pe["dousing_count"], exp)
    for e in range(E):  # the per-env form gives the same
        g1, p1, pe1 = mm(np.zeros((H, W)), (moves[e], shots[e]), pos[e], {"dousing_count": np.zeros((H, W), np.int32)})
        assert np.array_equal(p1, want[e]) and np.array_equal(pe1["dousing_count"], exp[e])


class _CountingCA:
    """A 4-argument CA (PartiallyObservableForestFireJax's contract) that counts its calls."""

    deterministic = False

    def __init__(self):
        self.calls = 0

    def __call__(self, grid, action, per_env, shared):
        self.calls += 1
        pe = dict(per_env)
        pe["n"] = pe.get("n", 0) + 1
        return grid + 1, pe, shared


@pytest.mark.parametrize("accu,t_act,t_state", [(0.0, 0.3, 0.001), (0.5, 0.7, 0.001), (0.9, 2.5, 0.25),
                                                (np.float32(0.75), np.float32(0.031), np.float32(0.001))])
def test_repeat_ca_jax_runs_exactly_one_step(accu, t_act, t_state):
    """repeat_ca_jax.py:34-71: modf of accu + (t_act + t_state) is carried, and the CA runs once whatever the whole
    part (the repeat loop is commented out, :64-69); returns (grid, (per_env, fraction))."""
    from gymca_amd.forest_fire.operators import RepeatCAJax

    ca = _CountingCA()
    seen = []
    op = RepeatCAJax(ca, lambda a: t_act, lambda s: (seen.append(len(s)), t_state)[1])
    grid = np.zeros((3, 3))
    out, (pe, frac) = op(grid, (1, 0), {"n": 0}, {"p_tree": 0.0}, accu)
    assert ca.calls == 1 and pe["n"] == 1 and np.all(out == 1) and seen == [3]
    exp, _ = np.modf(accu + (t_act + t_state))
    assert frac == exp and np.asarray(frac).dtype == np.asarray(exp).dtype


def test_drossel_host_matches_seeded_reference(golden):
    from gymca_amd.forest_fire.operators import ForestFire

    d = golden("drossel")
    for i in range(int(d["n"])):
        grid = d[f"c{i}_grid"]
        op = ForestFire(0, 1, 2, backend="cpu")
        op.seed(int(d[f"c{i}_seed"]))
        out, _ = op.update(grid.astype(np.int64), None, d[f"c{i}_p"])
        assert np.array_equal(out, d[f"c{i}_out"]), f"case {i}"


@pytest.mark.parametrize("backend", ["cpu", "auto"])
def test_helicopter_env_replays_seeded_reference_on_host(golden, backend):
    """BASELINE config 1 with no GPU: ForestFireHelicopterEnv(5, 5) replays the seeded reference episode (grids,
    rewards, positions, freeze, hit) through the host backend."""
    from gymca_amd.forest_fire.helicopter import ForestFireHelicopterEnv

    d = golden("helicopter")
    env = ForestFireHelicopterEnv(5, 5, backend=backend)
    env.reset(seed=7)
    env.cellular_automaton.seed(int(d["seed"]))
    env.grid = d["grid0"].astype(np.int64)
    for s in range(len(d["grids"])):
        obs, rew, term, trunc, info = env.step(s % 9)
        grid, (cp, pos, fr) = obs
        assert np.array_equal(grid, d["grids"][s]), f"step {s}"
        exp = d["recs"][s]
        assert np.isclose(rew, exp[0], rtol=0, atol=1e-15) and (pos[0], pos[1], int(fr)) == (exp[1], exp[2], exp[3])
        assert bool(info["hit"]) == bool(exp[4])
    counts = env.count_cells()
    assert sum(counts.values()) == 25


def test_large_host_grid_refuses_without_gpu():
    """Above HOST_MAX_CELLS a host grid goes to the kernels: with no GPU in this process that fails loudly."""
    import torch

    from gymca_amd import GCAError
    from gymca_amd.forest_fire.operators import ForestFire

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(GCAError):
        ForestFire(0, 1, 2).update(np.zeros((128, 128), np.int64), None, (0.1, 0.1))
