"""GPU parity: the Alexandridis kernel vs the C oracle (bit-exact, both draw modes) and the
numpy restatement of the reference rule; the advanced env step vs its oracle composition."""
import numpy as np
import pytest

from alex_cases import make_case, winds
from oracle import alex_c
from oracle import alexandridis_ref as ref

pytestmark = pytest.mark.gpu


def _dev(x, dtype, device):
    import torch

    return torch.as_tensor(np.ascontiguousarray(x), device=device).to(dtype).contiguous()


def run_kernel(device, p, case, rng_step=None, inj=None, probs=False):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call

    E, H, W = case["grid"].shape
    g = _dev(case["grid"], torch.uint8, device)
    a = _dev(case["age"], torch.int16, device)
    veg, den, dous = (_dev(case[k], torch.uint8, device) for k in ("veg", "den", "dous"))
    slope = _dev(case["slope"].reshape(E, H, W, 9), torch.float32, device)
    ps = torch.empty((E, 8, H, W), dtype=torch.float32, device=device)
    call("gca_alex_prepare_slope", dev.ptr(slope), dev.ptr(ps), E, H, W, dev.stream_ptr())
    wi = _dev(case["widx"], torch.int32, device)
    rs = None if rng_step is None else _dev(np.asarray(rng_step).astype(np.uint32).view(np.int32), torch.int32, device)
    go, ao = torch.empty_like(g), torch.empty_like(a)
    counts = torch.zeros((E, 3), dtype=torch.int32, device=device)
    ij = [None] * 3
    if inj is not None:
        ij = [_dev(inj[0].reshape(E, H, W, 9), torch.float32, device), _dev(inj[1], torch.float32, device),
              _dev(inj[2], torch.int32, device)]
    po = torch.empty((E, H, W, 8), dtype=torch.float32, device=device) if probs else None
    call("gca_alex_step", p, E, H, W, dev.ptr(g), dev.ptr(go), dev.ptr(a), dev.ptr(ao), dev.ptr(veg), dev.ptr(den),
         dev.ptr(dous), dev.ptr(ps), dev.ptr(wi), dev.ptr(rs), dev.ptr(ij[0]), dev.ptr(ij[1]), dev.ptr(ij[2]),
         dev.ptr(po), dev.ptr(counts), dev.stream_ptr())
    return (go.cpu().numpy(), ao.cpu().numpy(), counts.cpu().numpy(), None if po is None else po.cpu().numpy(),
            ps.cpu().numpy())


def params(H, p_tree=0.0, seed=1234):
    from gymca_amd.forest_fire.operators.ca_alexandridis import make_alex_params

    p, _ = make_alex_params(H, 0, 1, 2, winds(), p_tree, seed)
    return p


def test_device_philox_kat(device):
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from test_rng_and_math import KAT

    for ctr, key, exp in KAT:
        c = torch.as_tensor(np.array([ctr], dtype=np.uint32).view(np.int32), device=device)
        out = torch.empty_like(c)
        call("gca_philox", dev.ptr(c), key[0], key[1], dev.ptr(out), 1, dev.stream_ptr())
        assert tuple(int(v) for v in out.cpu().numpy().view(np.uint32)[0]) == exp


def test_prepare_slope_bit_exact(device):
    case = make_case(2, 33, 47, 1)
    *_, ps = run_kernel(device, params(33), case)
    assert np.array_equal(ps.view(np.uint32), alex_c.prepare_slope(case["slope"]).view(np.uint32))


SIZES = [(2, 5, 7, 1), (2, 8, 8, 2), (3, 16, 16, 3), (2, 37, 45, 4), (2, 64, 64, 5), (1, 100, 300, 6),
         (2, 256, 256, 7), (1, 512, 512, 8), (1, 1024, 1024, 9), (1, 130, 33, 10)]


@pytest.mark.parametrize("E,H,W,seed", SIZES)
def test_injected_mode_bit_exact_vs_c_oracle(device, E, H, W, seed):
    case = make_case(E, H, W, seed, p_tree=0.25)
    p = params(H, 0.25)
    inj = case["draws"]
    go, ao, cnt, po, ps = run_kernel(device, p, case, inj=inj, probs=True)
    eg, ea, ec, ep = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"], ps,
                                      case["widx"], inj=(inj[0].reshape(E, H, W, 9), inj[1], inj[2]), want_probs=True)
    assert np.array_equal(po.view(np.uint32), ep.view(np.uint32))
    assert np.array_equal(go, eg) and np.array_equal(ao, ea) and np.array_equal(cnt, ec)


@pytest.mark.parametrize("E,H,W,seed", SIZES)
def test_philox_mode_bit_exact_vs_c_oracle_multi_step(device, E, H, W, seed):
    case = make_case(E, H, W, seed, p_tree=0.01)
    p = params(H, 0.01, seed=seed * 977)
    ps = alex_c.prepare_slope(case["slope"])
    steps = 3 if H * W * E > 200000 else 6
    for s in range(steps):
        rs = np.full(E, 10 * s + 1, np.uint32)
        go, ao, cnt, _, _ = run_kernel(device, p, case, rng_step=rs)
        eg, ea, ec, _ = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"], ps,
                                         case["widx"], rng_step=rs)
        assert np.array_equal(go, eg), f"step {s}: {np.argwhere(go != eg)[:5]}"
        assert np.array_equal(ao, ea) and np.array_equal(cnt, ec)
        case["grid"], case["age"] = go, ao


def test_injected_mode_matches_reference_rule(device):
    """Device (injected draws) vs the numpy restatement of _update_grid as written."""
    E, H, W = 2, 64, 64
    case = make_case(E, H, W, 21, p_tree=0.2)
    p = params(H, 0.2)
    go, ao, _, po, _ = run_kernel(device, p, case, inj=case["draws"], probs=True)
    W8 = winds()[:, 0]
    ub, ug, ua = case["draws"]
    for e in range(E):
        ng, na, rp = ref.update_grid(case["grid"][e], case["age"][e], case["veg"][e].astype(np.int64),
                                     case["den"][e].astype(np.int64), case["slope"][e], case["dous"][e],
                                     W8[case["widx"][e]], 0.2, ub[e], ug[e], ua[e], case["C"])
        rp8 = rp.reshape(H, W, 9)[..., [0, 1, 2, 3, 5, 6, 7, 8]]
        assert np.max(np.abs(po[e] - rp8) / np.maximum(np.abs(rp8), 1.0)) < 1e-6  # TOL 1e-6
        diff = go[e] != ng
        if diff.any():  # only where a uniform sits within rounding of its probability
            close = np.abs(ub[e].reshape(H, W, 9)[..., [0, 1, 2, 3, 5, 6, 7, 8]] - rp8).min(axis=-1) < 1e-6
            assert np.all(close[diff])
        assert np.array_equal(ao[e][~diff], na.astype(np.int16)[~diff])


def _ref_compare(case, e, go, ao, po, slope9, p_tree, C):
    """One env of a device step (injected draws) against the numpy restatement of the reference rule
    (ca_alexandridis_jax.py:321-424) and the independent float64 probability: probabilities within
    1e-6 (TOL), integer states equal except where a uniform lies within 1e-6 of its probability."""
    H, W = case["grid"].shape[1:]
    W8 = winds()[:, 0]
    ub, ug, ua = case["draws"]
    veg, den = case["veg"][e].astype(np.int64), case["den"][e].astype(np.int64)
    ng, na, rp = ref.update_grid(case["grid"][e], case["age"][e], veg, den, slope9[e], case["dous"][e],
                                 W8[case["widx"][e]], p_tree, ub[e], ug[e], ua[e], C)
    sel = [0, 1, 2, 3, 5, 6, 7, 8]
    rp8 = rp.reshape(H, W, 9)[..., sel]
    assert np.max(np.abs(po[e] - rp8) / np.maximum(np.abs(rp8), 1.0)) < 1e-6  # TOL 1e-6 vs the f32 restatement
    p64 = ref.burn_probability_f64(case["grid"][e], veg, den, W8[case["widx"][e]], slope9[e], case["dous"][e],
                                   C).reshape(H, W, 9)[..., sel]
    assert np.max(np.abs(po[e] - p64) / np.maximum(np.abs(p64), 1.0)) < 1e-6  # TOL 1e-6 vs float64
    diff = go[e] != ng
    if diff.any():
        close = np.abs(ub[e].reshape(H, W, 9)[..., sel] - rp8).min(axis=-1) < 1e-6
        assert np.all(close[diff])
    assert diff.sum() <= 8  # near-ties are rare: a systematic rule difference would show thousands
    assert np.array_equal(ao[e][~diff], na.astype(np.int16)[~diff])
    return int((go[e] != case["grid"][e]).sum())


@pytest.mark.parametrize("N,seed", [(256, 71), (512, 72)])
def test_headline_sizes_injected_vs_reference_rule(device, N, seed):
    """BASELINE sizes, deterministically: N = 256 (configs 3/4: heat radius R = 6, 13x13 window) and N = 512
    (config 5's grid: R = 7, 15x15). Hidden-layer slopes from an altitude field (get_slope on the device),
    vegetation / density 0..6 (the clip), dousing, p_tree > 0, E = 2, the reference's own draws injected.
    1. gca_alex_step (8 p_slope planes) and gca_alex_step_es (edge slopes) vs the numpy restatement of
       _update_grid (ca_alexandridis_jax.py:62,108-153,345-349,379-398) and the float64 probability;
    2. the two layouts bit-identical (states, ages, counts, probabilities);
    3. the headline kernels, gca_alex_step_packed (tiled) and gca_alex_step_march (the env's step at W = 256 and
       512; Philox mode, packed layout), bit-identical to gca_alex_step_es in Philox mode on the same state,
       whose probabilities are bit-identical to the injected-mode probabilities checked in 1 — so the timed
       kernel evaluates the reference's p_d."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from test_gpu_edge_slope import altitude, packed_step, slopes, step

    E, p_tree = 2, 0.2
    case = make_case(E, N, N, seed, p_tree=p_tree)
    C = case["C"]
    assert C["R"] == (6 if N == 256 else 7)
    p = params(N, p_tree)
    alt = altitude(E, N, N, seed)
    es, ps = slopes(device, alt)
    a = torch.as_tensor(alt, device=device)
    s9 = torch.empty((E, N, N, 3, 3), dtype=torch.float32, device=device)
    tmp = torch.empty((E, 8, N, N), dtype=torch.float32, device=device)
    call("gca_alex_slope_from_altitude", dev.ptr(a), dev.ptr(tmp), dev.ptr(s9), E, N, N, dev.stream_ptr())
    s9 = s9.cpu().numpy()
    from gymca_amd.forest_fire.bulldozer.init_utils import get_slope

    assert np.allclose(s9, get_slope(alt, N, N, E).astype(np.float32), rtol=3e-6, atol=1e-5)
    case["slope"] = s9
    inj = case["draws"]
    r_planes = step(device, "gca_alex_step", p, case, ps, inj=inj, probs=True)
    r_edge = step(device, "gca_alex_step_es", p, case, es, inj=inj, probs=True)
    for x, y in zip(r_planes, r_edge):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    go, ao, cnt, po = r_edge
    changed = [_ref_compare(case, e, go, ao, po, s9, p_tree, C) for e in range(E)]
    assert min(changed) > 1000  # the step did real work (ignitions, burn-outs, growth)
    assert np.array_equal(cnt, np.stack([(go == v).sum(axis=(1, 2)) for v in (0, 1, 2)], axis=1))
    # the chain to the timed kernel (Philox mode)
    rs = np.full(E, 9, np.uint32)
    case_ph = dict(case, dous=(case["dous"] > 0).astype(np.uint8))  # the packed layout's dousing bits
    g_es, a_es, c_es, po_es = step(device, "gca_alex_step_es", p, case_ph, es, rng_step=rs, probs=True)
    g_pk, a_pk, c_pk, _, _ = packed_step(device, p, case_ph, es, rs)
    assert np.array_equal(g_pk, g_es) and np.array_equal(a_pk, a_es) and np.array_equal(c_pk, c_es)
    if N in (256, 512):  # the env's step at both sizes (W = 512: two segment waves per strip, R = 7)
        from test_gpu_alex_march import _layers, _run

        vd, bits = _layers(device, case_ph)
        g_mr, a_mr, c_mr, _, _ = _run(device, "gca_alex_step_march", p, case_ph, es, rs, vd, bits)
        assert np.array_equal(g_mr, g_es) and np.array_equal(a_mr, a_es) and np.array_equal(c_mr, c_es)
    _, _, _, po_inj = step(device, "gca_alex_step_es", p, case_ph, es, inj=inj, probs=True)
    assert np.array_equal(po_es.view(np.uint32), po_inj.view(np.uint32))


def test_dropin_operator_with_reference_draws(device):
    from gymca_amd.forest_fire.operators import PartiallyObservableForestFireJax

    H = W = 32
    case = make_case(1, H, W, 33)
    op = PartiallyObservableForestFireJax(H, 0, 1, 2)
    assert op.burn_kernel_radius == 3 and op.burn_kernel.shape == (1, 1, 7, 7)
    ctx = {"wind_index": np.int32(case["widx"][0]), "density": case["den"][0].astype(np.int64),
           "vegetation": case["veg"][0].astype(np.int64), "slope": case["slope"][0],
           "fire_age": case["age"][0].astype(np.float32), "dousing_count": case["dous"][0].astype(np.int32),
           "key": np.array([1, 2], np.uint32)}
    shared = {"winds": winds(), "p_tree": np.float32(0.0), "p_wind_change": np.float32(0.06)}
    ub, ug, ua = case["draws"]
    draws = {"burn": ub[0], "grow": ug[0], "age": ua[0], "wind_u": 0.01, "wind_k": 3}
    new_grid, ctx2, _ = op.update(case["grid"][0].astype(np.float32), None, ctx, shared, draws=draws)
    ng, na, _ = ref.update_grid(case["grid"][0], case["age"][0], ctx["vegetation"], ctx["density"], ctx["slope"],
                                ctx["dousing_count"], winds()[case["widx"][0], 0], 0.0, ub[0], ug[0], ua[0],
                                case["C"])
    assert np.array_equal(new_grid, ng)
    assert np.array_equal(ctx2["fire_age"], na)
    assert int(ctx2["wind_index"]) == (int(case["widx"][0]) + 3) % 8
    assert ctx2["rng_step"] == 1


@pytest.mark.parametrize("N", [64, 256])  # 64: edge layout; 256: the packed layout (the env's default there)
def test_advanced_env_matches_oracle_composition(device, N):
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv
    from oracle.windy import move

    E = 4
    env = AdvancedForestFireBulldozerEnv(N, N, key=99, num_envs=E, use_hidden=True, device=device)
    assert env.slope_layout == ("packed" if N == 256 else "edge")
    env.reset()
    case = make_case(E, N, N, 44)
    env.set_state(grid=case["grid"], fire_age=case["age"], vegetation=np.clip(case["veg"], 1, 5),
                  density=np.clip(case["den"], 1, 5), wind_index=case["widx"], dousing=case["dous"])
    g, a = case["grid"].copy(), case["age"].copy()
    veg, den = np.clip(case["veg"], 1, 5), np.clip(case["den"], 1, 5)
    dous = case["dous"].copy()
    ps = env.p_slope_planes().cpu().numpy()
    widx = case["widx"].copy()
    pos = env.pos.cpu().numpy().copy()
    accu = np.zeros(E, np.float32)
    rng = np.random.default_rng(0)
    p = env.alex_params
    ep = env.env_params
    for s in range(12):
        act = np.stack([rng.integers(0, 9, E), rng.integers(0, 2, E)], axis=1)
        _, rew, term, _, _ = env.step(act)
        rs = np.full(E, s, np.uint32)
        g, a, counts, _ = alex_c.alex_step(p, g, a, veg, den, dous, ps, widx, rng_step=rs)
        widx = alex_c.wind_change(np.float32(0.06), 8, ep.seed, 0, rs, widx)
        for e in range(E):
            t = np.float32(np.float32(ep.t_move[act[e, 0]]) + np.float32(ep.t_shoot[act[e, 1]])) + np.float32(ep.t_any)
            na = np.float32(accu[e] + t)
            accu[e] = np.float32(na - np.float32(np.trunc(na)))
            pos[e] = move(pos[e], int(act[e, 0]), N, N)
            if act[e, 1] == 1:
                dous[e, pos[e][0], pos[e][1]] = 1
        exp_rew = -(counts[:, 2].astype(np.float32) / (counts[:, 1:].sum(1).astype(np.float32) + np.float32(1e-8)))
        assert np.array_equal(env.grid[env.cur].cpu().numpy(), g), f"step {s}"
        assert np.array_equal(env.age[env.cur].cpu().numpy(), a)
        assert np.array_equal(env.wind_index.cpu().numpy(), widx)
        assert np.array_equal(env.pos.cpu().numpy(), pos)
        assert np.array_equal(env.accu.cpu().numpy(), accu)
        assert np.array_equal(env.dousing.cpu().numpy(), dous)
        assert np.array_equal(rew.cpu().numpy(), exp_rew.astype(np.float32))
        assert np.array_equal(term.cpu().numpy(), counts[:, 2] == 0)
    assert int(env.time_step[0].item()) == 13


def test_conditional_reset_reinjects_initial_state(device):
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 6, 32
    env = AdvancedForestFireBulldozerEnv(N, N, key=5, num_envs=E, use_hidden=False, device=device)
    env.reset()
    g0, a0 = env.grid[env.cur].clone(), env.age[env.cur].clone()
    for _ in range(3):
        env.step(np.zeros((E, 2), np.int64))
    env.done[torch.tensor([1, 4])] = 1
    env.conditional_reset()
    g, a = env.grid[env.cur], env.age[env.cur]
    assert torch.equal(g[1], g0[1]) and torch.equal(g[4], g0[4])
    assert torch.equal(a[1], a0[1]) and torch.equal(a[4], a0[4]) and not torch.equal(a[0], a0[0])  # fires aged
    assert int(env.done.sum().item()) == 0 and int(env.rng_step[1].item()) == 0 and int(env.rng_step[0].item()) == 3


def test_full_size_config3_step_properties(device):
    """BASELINE config 3 (4096 x 256^2, use_hidden=False) one step: invariants hold for every
    env and sampled envs match the C oracle bit for bit."""
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 4096, 256
    env = AdvancedForestFireBulldozerEnv(N, N, key=1, num_envs=E, use_hidden=False, device=device)
    env.reset()
    gen = torch.Generator(device=device).manual_seed(1)
    u = torch.rand((E, N, N), device=device, generator=gen)
    grid = torch.where(u < 0.1, 0, torch.where(u < 0.9, 1, 2)).to(torch.uint8)
    age = torch.where(grid == 2, torch.randint(1, 673, (E, N, N), device=device, generator=gen), 0).to(torch.int16)
    env.set_state(grid=grid, fire_age=age, wind_index=torch.randint(0, 8, (E,), device=device, generator=gen))
    g0, a0 = grid.clone(), age.clone()
    env.ca_step()
    g1, a1 = env.grid[env.cur], env.age[env.cur]
    assert torch.all(g1[g0 == 0] == 0)
    assert torch.all(g1[(g0 == 2) & (a0 <= 1)] == 0) and torch.all(g1[(g0 == 2) & (a0 > 1)] == 2)
    assert torch.equal(a1[g0 == 2].to(torch.int32), a0[g0 == 2].to(torch.int32) - 1)
    counts = env.counts.cpu().numpy()
    assert np.all(counts.sum(axis=1) == N * N)
    for e in (0, 2047, 4095):
        # env id e: the oracle is called on one env, so shift the Philox env id
        p = alex_c.params_from(env.alex_params)
        p.env_offset = e
        eg, ea, ec, _ = alex_c.alex_step(p, g0[e:e + 1].cpu().numpy(), a0[e:e + 1].cpu().numpy(),
                                         np.full((1, N, N), 3, np.uint8), np.full((1, N, N), 3, np.uint8),
                                         np.zeros((1, N, N), np.uint8), env.p_slope_planes()[e:e + 1].cpu().numpy(),
                                         env.wind_index[e:e + 1].cpu().numpy(), rng_step=np.zeros(1, np.uint32))
        assert np.array_equal(g1[e].cpu().numpy(), eg[0]) and np.array_equal(a1[e].cpu().numpy(), ea[0])
        assert np.array_equal(counts[e], ec[0])


def test_full_size_config4_step_properties(device):
    """BASELINE config 4 (AdvancedBulldozer 256^2 with the hidden foliage / altitude layers, 4096 envs) one step
    through the env, the bench's layers (hidden_rng="philox": init_utils.py:10-116's recipe drawn on the device,
    get_slope on the device): invariants on every env, and three sampled envs vs the C oracle bit for bit with their
    own vegetation / density / slope layers (reference: advanced_bulldozer.py:182-204, ca_alexandridis_jax.py:321-424)."""
    import torch
    import torch.nn.functional as F

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    E, N = 4096, 256
    env = AdvancedForestFireBulldozerEnv(N, N, key=2, num_envs=E, use_hidden=True, device=device, hidden_rng="philox",
                                         observation="grid")
    assert env.slope_layout == "packed" and env.march
    env.reset()
    veg, den = env.vegetation.clone(), env.density.clone()
    assert int(veg.min()) >= 1 and int(veg.max()) <= 5 and int(den.min()) >= 1 and int(den.max()) <= 5
    assert int(veg.float().std(dim=(1, 2)).gt(0).sum()) > E // 2  # hidden layers, not constants
    gen = torch.Generator(device=device).manual_seed(4)
    u = torch.rand((E, N, N), device=device, generator=gen)
    grid = torch.where(u < 0.1, 0, torch.where(u < 0.9, 1, 2)).to(torch.uint8)
    del u
    age = torch.where(grid == 2, torch.randint(1, 673, (E, N, N), device=device, generator=gen), 0).to(torch.int16)
    env.set_state(grid=grid, fire_age=age, wind_index=torch.randint(0, 8, (E,), device=device, generator=gen))
    g0, a0 = grid, age.clone()
    env.ca_step()
    g1, a1 = env.grid[env.cur], env.age[env.cur]
    assert torch.all(g1[g0 == 0] == 0)  # p_tree = 0: nothing grows
    assert torch.all(g1[(g0 == 2) & (a0 <= 1)] == 0) and torch.all(g1[(g0 == 2) & (a0 > 1)] == 2)
    assert torch.equal(a1[g0 == 2].to(torch.int32), a0[g0 == 2].to(torch.int32) - 1)
    # a TREE burns only next to a FIRE (Moore neighbourhood, zero padding); a TREE that stays keeps its age
    fire_nb = F.max_pool2d((g0 == 2).to(torch.float16).unsqueeze(1), 3, stride=1, padding=1).squeeze(1) > 0
    tree = g0 == 1
    assert torch.all(g1[tree & ~fire_nb] == 1)
    assert torch.all((g1[tree] == 1) | (g1[tree] == 2))
    burnt = tree & (g1 == 2)
    assert torch.all(a1[burnt] >= 576) and torch.all(a1[burnt] < 672)  # randint[floor(1.5 S), floor(1.75 S))
    assert torch.equal(a1[tree & (g1 == 1)], a0[tree & (g1 == 1)])
    assert int(burnt.sum()) > 0
    counts = env.counts.cpu().numpy()
    assert np.all(counts.sum(axis=1) == N * N)
    ref_counts = torch.stack([(g1 == k).sum(dim=(1, 2)) for k in range(3)], dim=1).cpu().numpy()
    assert np.array_equal(counts, ref_counts)
    st = dev.stream_ptr(device)
    for e in (0, 1777, 4095):
        planes = torch.empty((1, 8, N, N), dtype=torch.float32, device=device)
        alt = env.altitude[e:e + 1].contiguous()
        call("gca_alex_slope_from_altitude", dev.ptr(alt), dev.ptr(planes), None, 1, N, N, st)
        p = alex_c.params_from(env.alex_params)
        p.env_offset = e  # the oracle steps one env: shift the Philox env id
        eg, ea, ec, _ = alex_c.alex_step(p, g0[e:e + 1].cpu().numpy(), a0[e:e + 1].cpu().numpy(),
                                         veg[e:e + 1].cpu().numpy(), den[e:e + 1].cpu().numpy(),
                                         np.zeros((1, N, N), np.uint8), planes.cpu().numpy(),
                                         env.wind_index[e:e + 1].cpu().numpy(), rng_step=np.zeros(1, np.uint32))
        assert np.array_equal(g1[e].cpu().numpy(), eg[0]) and np.array_equal(a1[e].cpu().numpy(), ea[0])
        assert np.array_equal(counts[e], ec[0])


# ------------------------------------------------------------------ classic variant (row a8)
@pytest.mark.parametrize("H,W,seed", [(16, 16, 0), (21, 37, 1), (64, 64, 2)])
def test_classic_dropin_matches_classic_restatement(device, H, W, seed):
    """PartiallyObservableForestFire (ca_alexandridis.py:18-221) on the device with the reference's
    draws injected vs the float64 per-cell restatement: grid, fire_age (mutated in the context, like
    the reference) and wind_index."""
    from gymca_amd.forest_fire.operators import PartiallyObservableForestFire
    from oracle import alexandridis_classic as cl

    rng = np.random.default_rng(100 + seed)
    ctx = cl.random_context(rng, H, W)
    dr = cl.random_draws(rng, H, W)
    ng, na, nw, rp = cl.update(ctx["grid"], ctx, dr, 0, 1, 2)
    op = PartiallyObservableForestFire(0, 1, 2, pinecones=False)
    age_obj = ctx["fire_age"]
    new_grid, out_ctx, probs = op(ctx["grid"], None, ctx, draws=dr, return_probs=True)
    assert out_ctx is ctx and ctx["fire_age"] is age_obj  # context mutated in place
    rp8 = rp.reshape(H, W, 9)[..., [0, 1, 2, 3, 5, 6, 7, 8]]
    burning_nb = np.any(rp8 != 0, axis=-1)
    assert np.max((np.abs(probs - rp8) / np.maximum(np.abs(rp8), 1.0))[burning_nb]) < 1e-6
    diff = new_grid != ng
    if diff.any():
        close = np.abs(dr["burn"].reshape(H, W, 9)[..., [0, 1, 2, 3, 5, 6, 7, 8]] - rp8).min(axis=-1) < 1e-6
        assert np.all(close[diff])
    assert np.array_equal(ctx["fire_age"][~diff], na[~diff])
    assert int(ctx["wind_index"]) == nw


@pytest.mark.parametrize("H,W", [(64, 64), (256, 256), (45, 77)])
def test_classic_philox_bit_exact_vs_c_oracle(device, H, W):
    """Philox mode with the classic parameters: device == C oracle, several steps."""
    import torch

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.operators.ca_alexandridis import make_classic_params
    from oracle import alexandridis_classic as cl

    E = 3
    rng = np.random.default_rng(H + W)
    ctxs = [cl.random_context(rng, H, W, p_tree=0.05) for _ in range(E)]
    grid = np.stack([c["grid"] for c in ctxs])
    age = np.stack([c["fire_age"] for c in ctxs]).astype(np.int16)
    veg = np.stack([c["vegetation"] for c in ctxs]).astype(np.uint8)
    den = np.stack([c["density"] for c in ctxs]).astype(np.uint8)
    slope = np.stack([c["slope"] for c in ctxs]).reshape(E, H, W, 9).astype(np.float32)
    widx = np.array([c["wind_index"] for c in ctxs], np.int32)
    dous = np.zeros((E, H, W), np.uint8)
    p = make_classic_params(0, 1, 2, ctxs[0]["winds"], 0.05, 77)
    ps = alex_c.prepare_slope(slope)
    T = lambda a, t: torch.as_tensor(np.ascontiguousarray(a)).to(device=device, dtype=t)
    g_d, a_d = T(grid, torch.uint8), T(age, torch.int16)
    v_d, n_d, du_d, ps_d, w_d = T(veg, torch.uint8), T(den, torch.uint8), T(dous, torch.uint8), T(ps, torch.float32), \
        T(widx, torch.int32)
    st = dev.stream_ptr(device)
    for step in range(4):
        rs = np.full(E, step, np.uint32)
        go, ao, co, _ = alex_c.alex_step(p, grid, age, veg, den, dous, ps, widx, rng_step=rs)
        g2, a2 = torch.empty_like(g_d), torch.empty_like(a_d)
        counts = torch.empty((E, 3), dtype=torch.int32, device=device)
        rs_d = T(rs.view(np.int32), torch.int32)
        call("gca_alex_step", p, E, H, W, dev.ptr(g_d), dev.ptr(g2), dev.ptr(a_d), dev.ptr(a2), dev.ptr(v_d),
             dev.ptr(n_d), dev.ptr(du_d), dev.ptr(ps_d), dev.ptr(w_d), dev.ptr(rs_d),
             None, None, None, None, dev.ptr(counts), st)
        assert np.array_equal(g2.cpu().numpy(), go) and np.array_equal(a2.cpu().numpy(), ao), f"step {step}"
        assert np.array_equal(counts.cpu().numpy(), co)
        grid, age, g_d, a_d = go, ao, g2, a2


def test_philox_and_injected_modes_share_probabilities(device):
    """The Philox-mode kernel (MODE 1 = MODE 0 + the debug probability output) and the injected-draw kernel
    (MODE 2) compute bit-identical per-direction burn probabilities on the same state: the draw mode changes
    only how the uniforms are compared, never p_d."""
    E, H, W = 3, 96, 80
    case = make_case(E, H, W, 57, p_tree=0.1)
    p = params(H, 0.1)
    *_, po_philox, _ = run_kernel(device, p, case, rng_step=np.full(E, 3, np.uint32), probs=True)
    *_, po_inj, _ = run_kernel(device, p, case, inj=case["draws"], probs=True)
    assert np.array_equal(po_philox.view(np.uint32), po_inj.view(np.uint32))


def test_packed_fast_kernel_burn_law_chi_square(device):
    """The timed kernel (the env's packed-layout step at 256^2: gca_alex_step_march) against the
    reference's burn law. The reference ignites a TREE iff some burning neighbour d has u_d < p_d with
    independent uniforms (ca_alexandridis_jax.py:379-383), i.e. with probability 1 - prod_d (1 - clamp01(p_d));
    the kernel draws one uniform against that product. 32 envs x 256^2 mid-episode states (hidden layers,
    random dousing) give ~0.6M TREE cells with 1..8 burning neighbours and 0 < law < 1, plus cells with every p_d <= 0
    (dousing) and a few with p_d > 1 (steep slopes); 48 launches
    with distinct Philox steps. Expected p_d: the independent float64 evaluation
    oracle.alexandridis_ref.burn_probability_f64. Cells binned by expected law (40 quantile bins): sum over
    bins of (observed - expected)^2 / variance ~ chi2(40); the test fails above chi2.isf(1e-6, 40) (false-alarm
    rate 1e-6). Cells with every p_d <= 0 must never ignite, cells with some p_d >= 1.001 always."""
    import torch
    from scipy.stats import chi2

    from gymca_amd import _device as dev
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv
    from gymca_amd.forest_fire.bulldozer.init_utils import get_slope

    E, N, T = 32, 256, 48
    env = AdvancedForestFireBulldozerEnv(N, N, key=606, num_envs=E, use_hidden=True, hidden_rng="philox",
                                         device=device, observation="grid", slope_layout="packed")
    env.reset()
    rng = np.random.default_rng(12)
    grid = rng.choice(np.array([0, 1, 2], np.uint8), size=(E, N, N), p=[0.1, 0.6, 0.3])
    age = np.where(grid == 2, 500, 0).astype(np.int16)
    dous = (rng.random((E, N, N)) < 0.03).astype(np.uint8)
    widx = rng.integers(0, 8, E).astype(np.int32)
    env.set_state(grid=grid, fire_age=age, dousing=dous, wind_index=widx)
    g_in = env.grid[env.cur].clone()
    age0 = env.age[env.cur].clone()
    g_out = torch.empty_like(g_in)
    age_buf = torch.empty((E, N, N), dtype=torch.int16, device=device)
    counts = torch.zeros((E, 3), dtype=torch.int32, device=device)
    burned = torch.zeros((E, N, N), dtype=torch.int32, device=device)
    st = dev.stream_ptr(device)
    for t in range(T):
        age_buf.copy_(age0)  # the packed step updates ages in place
        rs = torch.full((E,), 1000 + t, dtype=torch.int32, device=device)
        assert env.march
        call("gca_alex_step_march", env.alex_params, E, N, N, dev.ptr(g_in), dev.ptr(g_out), dev.ptr(age_buf),
             dev.ptr(age_buf), dev.ptr(env.vd), dev.ptr(env.dous_bits), dev.ptr(env.slope_data), dev.ptr(env.wind_index),
             dev.ptr(rs), dev.ptr(counts), None, None, st)
        burned += ((g_out == 2) & (g_in == 1)).to(torch.int32)
    burned = burned.cpu().numpy()
    slope = get_slope(env.altitude.cpu().numpy(), N, N, E).astype(np.float32)
    veg, den = env.vegetation.cpu().numpy(), env.density.cpu().numpy()
    W8 = winds()[:, 0]
    C = ref.constants(N)
    laws, obs, always, never = [], [], [], []
    for e in range(E):
        pd = ref.burn_probability_f64(grid[e], veg[e], den[e], W8[widx[e]], slope[e], dous[e], C).reshape(N, N, 9)
        nbf = (ref._nbhd(grid[e].astype(np.float32), 1) == 2).reshape(N, N, 9)
        nbf[..., 4] = False
        cand = (grid[e] == 1) & nbf.any(-1)
        q = np.where(nbf, 1.0 - np.clip(pd, 0.0, 1.0), 1.0).prod(-1)
        law = 1.0 - q
        hi = (np.where(nbf, pd, -np.inf).max(-1) >= 1.001) & cand
        lo = (np.where(nbf, pd, -np.inf).max(-1) <= 0.0) & cand
        mid = cand & ~hi & ~lo & (law > 0) & (law < 1)
        laws.append(law[mid])
        obs.append(burned[e][mid])
        always.append(burned[e][hi])
        never.append(burned[e][lo])
        assert np.all(burned[e][~cand] == 0)  # no burning neighbour (or not a TREE): never ignites
    laws, obs = np.concatenate(laws), np.concatenate(obs)
    always, never = np.concatenate(always), np.concatenate(never)
    assert laws.size > 500_000 and always.size >= 10 and never.size > 100
    assert np.all(always == T) and np.all(never == 0)
    assert laws.min() < 0.01 and laws.max() > 0.99  # the bins span the whole (0, 1) range
    B = 40
    edges = np.quantile(laws, np.linspace(0, 1, B + 1))
    b = np.clip(np.searchsorted(edges, laws, side="right") - 1, 0, B - 1)
    o = np.bincount(b, weights=obs, minlength=B)
    ex = T * np.bincount(b, weights=laws, minlength=B)
    var = T * np.bincount(b, weights=laws * (1 - laws), minlength=B)
    stat = float(((o - ex) ** 2 / var).sum())
    assert stat < chi2.isf(1e-6, B), (stat, chi2.isf(1e-6, B))


def test_classic_dropin_vs_reference_run(device, golden):
    """The device drop-in PartiallyObservableForestFire (classic params on gca_alex_step, the reference's recorded
    draws injected) against the reference's own update loop (tests/golden/alexandridis_classic.npz, 38 steps):
    every cell no pinecone ignited (the fixture marks them; pinecones draw from Philox on the device and are
    pinned through the oracle: oracle == reference run on this fixture, device == oracle on decoded draws in
    test_gpu_pinecones) equals the reference's grid and fire age; the wind index too. Near-ties of an f64
    uniform against the f32 probability are the only allowed exception."""
    from gymca_amd.forest_fire.operators import PartiallyObservableForestFire
    from oracle import alexandridis_classic as cl
    from test_pinecones_classic_oracle import _classic_fixture_steps

    d = golden("alexandridis_classic")
    n = checked = 0
    for key, ctx, grid, draws, _pine, (eg, ea, ew), pine_hits in _classic_fixture_steps(d):
        op = PartiallyObservableForestFire(0, 1, 2, pinecones=False)
        H, W = grid.shape
        dr = dict(draws, burn=draws["burn"].astype(np.float32), grow=draws["grow"].astype(np.float32))
        new_grid, out_ctx, probs = op(grid.astype(np.int64), None, ctx, draws=dr, return_probs=True)
        keep = pine_hits == 0
        diff = (new_grid != eg) & keep
        if diff.any():  # only where a recorded uniform lies within f32 rounding of the probability
            u = draws["burn"].reshape(H, W, 9)[..., [0, 1, 2, 3, 5, 6, 7, 8]]
            assert np.all(np.abs(u - probs).min(axis=-1)[diff] < 1e-6), key
        assert np.array_equal(np.asarray(out_ctx["fire_age"])[keep & ~diff], ea[keep & ~diff]), key
        assert int(out_ctx["wind_index"]) == ew, key
        n, checked = n + 1, checked + int(keep.sum())
    assert n == 38 and checked > 10000
