"""The Alexandridis per-cell draw convention (r05; include/gca.h GCA_TAG_ALEX_CELL / GCA_TAG_ALEX_AGE): one Philox
block per group of 4 cells of a row (counter r * ceil(W/4) + c/4); cell j tests word j's high 24 bits; the group's
first new fire is aged from the spare word (the four low bytes, which no decision reads), its 2nd..4th from words 0..2
of the group's ALXA block. Checked here on HOT states (45 % FIRE, vegetation = density = 5, steep slopes), where many
groups take two or more new fires, so the rare second-block path runs on every kernel: the marching step (the timed
kernel), the tiled packed step and the general 8-plane step at an odd width (partial groups at the row ends) are bit
for bit the C oracle; and the age law -- randint[lo, hi) of an independent uniform word, the reference's
jax.random.randint (ca_alexandridis_jax.py:366-370, 394-398) -- holds by chi-square for the first new fire of a group
(spare word) and the later ones (ALXA words) separately, with the first two of a group independent of each other."""
import numpy as np
import pytest

from alex_cases import make_case
from oracle import alex_c
from test_gpu_alex_march import _coalesced, _layers, _run
from test_gpu_edge_slope import _t, altitude, params, slopes, step

pytestmark = pytest.mark.gpu


def _hot_case(E, H, W, seed):
    case = make_case(E, H, W, seed, fire_p=0.45, dousing_p=0.0)
    case["veg"][:] = 5
    case["den"][:] = 5
    return case


def _groups_with_multi(g_in, g_out):
    """Number of 4-cell groups (row-aligned, columns 4g .. 4g+3) holding two or more new fires."""
    E, H, W = g_in.shape
    nf = ((g_in == 1) & (g_out == 2))
    pad = (-W) % 4
    nf = np.pad(nf, ((0, 0), (0, 0), (0, pad)))
    return int((nf.reshape(E, H, -1, 4).sum(-1) >= 2).sum())


@pytest.mark.parametrize("W", [256, 512])
def test_march_and_tiled_hot_state_vs_oracle(device, W):
    """Timed kernel (march) and the tiled packed step vs the C oracle on a hot state, three chained steps: grids,
    ages (incl. every 2nd..4th new fire of a group) and counts bit for bit."""
    E, H = 2, 64
    case = _hot_case(E, H, W, 71)
    p = params(H, 0.0, seed=913)
    es, ps = slopes(device, altitude(E, H, W, 71) * 4.0)
    coal = _coalesced(device, es)
    vd, bits = _layers(device, case)
    multi = 0
    for s in range(3):
        rs = np.full(E, 40 + 3 * s, np.uint32)
        g1, a1, c1, _, _ = _run(device, "gca_alex_step_march", p, case, es, rs, vd, bits)
        g0, a0, c0, _, _ = _run(device, "gca_alex_step_packed", p, case, coal, rs, vd, bits)
        go, ao, co, _ = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"],
                                         ps.cpu().numpy(), case["widx"], rng_step=rs)
        assert np.array_equal(g1, go), f"step {s}: {np.argwhere(g1 != go)[:5]}"
        assert np.array_equal(a1, ao), f"step {s}: ages {np.argwhere(a1 != ao)[:5]}"
        assert np.array_equal(c1, co)
        assert np.array_equal(g0, go) and np.array_equal(a0, ao) and np.array_equal(c0, co)
        multi += _groups_with_multi(case["grid"], go)
        case["grid"], case["age"] = go, ao
    assert multi > 200, multi  # the second-block path really ran


@pytest.mark.parametrize("H,W", [(37, 75), (20, 131), (64, 256)])
def test_general_step_partial_groups_vs_oracle(device, H, W):
    """The general 8-plane step (gca_alex_step) at widths that are not multiples of 4: the last group of every row has
    1..3 cells; ages and grids bit for bit the C oracle on a hot state."""
    import torch

    E = 2
    case = _hot_case(E, H, W, 5 + W)
    p = params(H, 0.0, seed=77)
    ps = alex_c.prepare_slope(case["slope"].reshape(E, H, W, 3, 3) * np.float32(1.5))
    ps_d = _t(ps, torch.float32, device)
    rs = np.full(E, 9, np.uint32)
    g1, a1, c1, _ = step(device, "gca_alex_step", p, case, ps_d, rng_step=rs)
    go, ao, co, _ = alex_c.alex_step(p, case["grid"], case["age"], case["veg"], case["den"], case["dous"], ps,
                                     case["widx"], rng_step=rs)
    assert np.array_equal(g1, go), np.argwhere(g1 != go)[:5]
    assert np.array_equal(a1, ao), np.argwhere(a1 != ao)[:5]
    assert np.array_equal(c1, co)
    assert _groups_with_multi(case["grid"], go) > 0


def test_new_fire_age_law_chi_square(device):
    """Ages of new fires ~ randint[576, 672) at 256^2 (ca_alexandridis_jax.py:368, S = N + N // 2), split by the new
    fire's rank in its 4-cell group: rank 0 (the spare word) and ranks 1..3 (ALXA words) each pass a chi-square
    against the uniform law over the 96 ages; the (rank 0, rank 1) ages of groups with two new fires pass an 8 x 8
    independence chi-square. 24 launches with distinct Philox steps on a 16 x 256^2 hot state (~10^6 new fires).
    False-alarm rate of each test 1e-6."""
    import torch
    from scipy.stats import chi2

    E, H, W, T = 16, 256, 256, 24
    case = _hot_case(E, H, W, 404)
    p = params(H, 0.0, seed=4242)
    lo, hi = int(p.age_lo), int(p.age_hi)
    assert (lo, hi) == (576, 672)
    es, _ = slopes(device, altitude(E, H, W, 404) * 4.0)
    vd, bits = _layers(device, case)
    g_in = case["grid"]
    tree = (g_in == 1).reshape(E, H, W // 4, 4)
    rank0, rankn, pairs = [], [], []
    for t in range(T):
        rs = np.full(E, 5000 + t, np.uint32)
        go, ao, _, _, _ = _run(device, "gca_alex_step_march", p, case, es, rs, vd, bits)
        nf = tree & (go == 2).reshape(E, H, W // 4, 4)
        rank = np.cumsum(nf, axis=-1) - 1
        ages = ao.reshape(E, H, W // 4, 4).astype(np.int64)
        assert np.all((ages[nf] >= lo) & (ages[nf] < hi))
        rank0.append(ages[nf & (rank == 0)])
        rankn.append(ages[nf & (rank >= 1)])
        two = nf.sum(-1) >= 2
        first = np.where(nf & (rank == 0), ages, 0).sum(-1)[two]
        second = np.where(nf & (rank == 1), ages, 0).sum(-1)[two]
        pairs.append(np.stack([first, second], -1))
    thr = lambda dof: chi2.isf(1e-6, dof)
    for name, a in (("rank 0", np.concatenate(rank0)), ("rank >= 1", np.concatenate(rankn))):
        assert a.size > 50_000, (name, a.size)
        cnt = np.bincount(a - lo, minlength=hi - lo)
        exp = a.size / (hi - lo)
        stat = float(((cnt - exp) ** 2 / exp).sum())
        assert stat < thr(hi - lo - 1), (name, stat, a.size)
    pr = np.concatenate(pairs)
    assert pr.shape[0] > 50_000
    b = ((pr - lo) * 8) // (hi - lo)  # 8 equal bins of 12 ages each
    tab = np.zeros((8, 8))
    np.add.at(tab, (b[:, 0], b[:, 1]), 1)
    exp = tab.sum(1, keepdims=True) * tab.sum(0, keepdims=True) / tab.sum()
    stat = float(((tab - exp) ** 2 / exp).sum())
    assert stat < thr(49), stat
