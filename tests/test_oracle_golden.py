"""The CPU oracle restatements against golden vectors captured from the reference itself."""
import numpy as np
import pytest

from oracle import drossel, windy

pytestmark = []


def test_windy_oracle_matches_reference(golden):
    d = golden("windy")
    for i in range(int(d["n"])):
        E, T, F = (int(v) for v in d[f"c{i}_values"])
        out = windy.windy_step(d[f"c{i}_grid"].astype(np.int64), d[f"c{i}_wind"], d[f"c{i}_roll"], E, T, F)
        assert np.array_equal(out, d[f"c{i}_out"]), f"case {i}"


def test_windy_closed_form_when_empty_is_zero(golden):
    """With empty == 0 the thresholds reduce to: TREE->FIRE iff an active direction sees FIRE."""
    d = golden("windy")
    checked = 0
    for i in range(int(d["n"])):
        E, T, F = (int(v) for v in d[f"c{i}_values"])
        if E != 0:
            continue
        g = d[f"c{i}_grid"].astype(np.int64)
        active = d[f"c{i}_roll"] < d[f"c{i}_wind"]
        H, W = g.shape
        pad = np.pad(g, 1, constant_values=E)
        out = np.where(g == F, E, g)
        for r in range(H):
            for c in range(W):
                if g[r, c] != T:
                    continue
                for a in range(3):
                    for b in range(3):
                        if (a, b) != (1, 1) and active[a, b] and pad[r + 1 - (a - 1), c + 1 - (b - 1)] == F:
                            out[r, c] = F
        assert np.array_equal(out, d[f"c{i}_out"]), f"case {i}"
        checked += 1
    assert checked >= 20


def test_repeat_ca_oracle_matches_reference(golden):
    d = golden("repeat_ca")
    for i in range(int(d["n"])):
        ta, tp = d[f"c{i}_times"]
        g = d[f"c{i}_grid"].astype(np.int64)
        accu, k = 0.0, 0
        rolls = d[f"c{i}_rolls"]
        for s in range(len(d[f"c{i}_accu"])):
            accu += ta + tp
            accu, reps = np.modf(accu)
            assert int(reps) == int(d[f"c{i}_nrolls"][s])
            for _ in range(int(reps)):
                g = windy.windy_step(g, d[f"c{i}_wind"], rolls[k])
                k += 1
            assert np.array_equal(g, d[f"c{i}_grids"][s]), f"case {i} step {s}"
            assert accu == d[f"c{i}_accu"][s]


def test_move_modify_oracle_matches_reference(golden):
    rows = golden("move_modify")["rows"]
    for H, W, r, c, a, shoot, pr, pc, before, after, hit in rows:
        assert windy.move((r, c), int(a), int(H), int(W)) == (pr, pc)
        exp_after = 0 if (shoot and before == 3) else before
        assert after == exp_after and bool(hit) == bool(shoot and before == 3)


@pytest.mark.parametrize("case", [0, 1, 2])
def test_bulldozer_oracle_matches_reference(golden, case):
    import zlib

    d = golden("bulldozer")
    N = int(d[f"c{case}_N"])
    tm, ts, ta = d[f"c{case}_times"]
    o = windy.BulldozerOracle([d[f"c{case}_grid0"]], [d[f"c{case}_pos0"]], d[f"c{case}_wind"], tm, ts, ta, seed=0)
    rolls, nrolls = d[f"c{case}_rolls"], d[f"c{case}_nrolls"]
    k = 0
    for s, (act, rec) in enumerate(zip(d[f"c{case}_actions"], d[f"c{case}_recs"])):
        rr = [list(rolls[k:k + nrolls[s]])]
        k += nrolls[s]
        was_done = bool(o.done[0])
        rew = o.step([act], rolls=rr)[0]
        g = o.grids[0]
        exp_rew, exp_term, exp_hit, pr, pc, t, cE, cT, cF = rec
        assert rew == exp_rew or (was_done and exp_rew == 0.0), f"step {s}"
        assert bool(o.done[0]) == bool(exp_term)
        if not was_done:
            assert bool(o.hit[0]) == bool(exp_hit)
            assert o.pos[0] == (pr, pc) and o.accu[0] == t
        assert (np.sum(g == 0), np.sum(g == 3), np.sum(g == 25)) == (cE, cT, cF)
        assert zlib.crc32(g.astype(np.uint8).tobytes()) & 0xFFFFFFFF == int(d[f"c{case}_crc"][s])
    assert np.array_equal(o.grids[0], d[f"c{case}_final"])


def test_drossel_oracle_matches_seeded_reference(golden):
    d = golden("drossel")
    for i in range(int(d["n"])):
        pf, pt = d[f"c{i}_p"]
        rng = np.random.default_rng(int(d[f"c{i}_seed"]))
        out = drossel.ds_step(d[f"c{i}_grid"].astype(np.int64), pf, pt, rng)
        assert np.array_equal(out, d[f"c{i}_out"]), f"case {i}"


def test_helicopter_oracle_matches_seeded_reference(golden):
    d = golden("helicopter")
    rng = np.random.default_rng(int(d["seed"]))
    g = d["grid0"].astype(np.int64)
    pos, freeze, mf = (2, 2), int(d["max_freeze"]), int(d["max_freeze"])
    for s in range(len(d["grids"])):
        a = s % 9
        if freeze == 0:
            g = drossel.ds_step(g, 0.033, 0.333, rng)
            freeze = mf
        else:
            freeze -= 1
        pos = windy.move(pos, a, 5, 5)
        hit = g[pos] == 2
        if hit:
            g[pos] = 0
        assert np.array_equal(g, d["grids"][s]), f"step {s}"
        rew = np.dot([0.0, 1.0, -1.0], [np.sum(g == v) / 25 for v in (0, 1, 2)])
        assert np.isclose(rew, d["recs"][s][0], rtol=0, atol=1e-15)
        assert (pos, freeze, hit) == ((d["recs"][s][1], d["recs"][s][2]), d["recs"][s][3], bool(d["recs"][s][4]))


def test_moore_padding_semantics(golden):
    """moore_n (neighbors.py:6-147) = constant padding with the invariant value."""
    d = golden("moore")
    for i in range(int(d["n"])):
        v = d[f"c{i}"]
        H, W, n, r, c = (int(x) for x in v[:5])
        grid = v[5:5 + H * W].reshape(H, W)
        exp = v[5 + H * W:].reshape(2 * n + 1, 2 * n + 1)
        pad = np.pad(grid, n, constant_values=9)
        assert np.array_equal(pad[r:r + 2 * n + 1, c:c + 2 * n + 1], exp)
