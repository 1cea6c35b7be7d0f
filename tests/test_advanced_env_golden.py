"""CPU: the Advanced env's step, composed from the oracle's parts, against the reference env EXECUTING
(tests/golden/advanced_env.npz, make_golden.py::gen_advanced_env: AdvancedForestFireBulldozerEnv built, reset and stepped
through `stateless_step` (advanced_bulldozer.py:332-399) as published under a numpy stand-in for jax, every env's draws
recorded). The composition is the one tests/test_gpu_alexandridis.py::test_advanced_env_matches_oracle_composition holds
the device env to (with Philox draws through the C oracle):
  RepeatCAJax (repeat_ca_jax.py:34-71): time += t_move + t_shoot + t_any in f32, modf; exactly one CA step
  the Alexandridis rule (oracle/alexandridis_ref.update_grid) with the env's wind, slopes, vegetation, density and the
      PRE-step dousing; the wind change (:443-451)
  MoveModifyJax (move_modify_jax.py:39-62, 102-114, 148-157): move with the border clamps, dousing_count = 1 at the new
      position when shooting
  time_step + 1, is_night toggled every day_length = 400 steps (:1116-1127)
  the RGB frame from the new grid, the new position and the PRE-step is_night / dousing (oracle/observation)
  reward -(f / (t + f + 1e-8)) in f32, terminated = no FIRE, steps_elapsed / reward_accumulated (:371-392)
Everything bit for bit (a grid cell may differ only where a burn uniform lies within 1e-6 of its probability).
"""
import numpy as np

from oracle import alexandridis_ref as ref
from oracle import observation as ob
from oracle.windy import move

LOOKUP = [(0, 0), (1, 0), (0, 1)]  # create_up_to_k_mappings(2, 1): extension choice -> binary flags


def test_advanced_env_step_composition_reproduces_reference_run(golden):
    d = golden("advanced_env")
    stepped = 0
    for ci in range(int(d["n"])):
        c = f"c{ci}_"
        N, E, steps, ext = (int(v) for v in d[c + "meta"])
        C = ref.constants(N)
        winds = d[c + "winds"]
        t_move, t_shoot, t_any = (np.float32(v) for v in d[c + "times"])
        veg, den = d[c + "init_vegetation"], d[c + "init_density"]
        slope = d[c + "init_slope"]
        grid, age = d[c + "init_true_grid"].copy(), d[c + "init_fire_age"].copy()
        dous, widx = d[c + "init_dousing_count"].copy(), d[c + "init_wind_index"].copy()
        pos, accu = d[c + "init_position"].copy(), d[c + "init_time"].astype(np.float32).copy()
        tstep, night = d[c + "init_time_step"].copy(), d[c + "init_is_night"].copy()
        steps_elapsed = np.zeros(E, np.float32)
        racc = np.zeros(E, np.float32)
        for t in range(steps):
            s = f"{c}s{t}_"
            act = d[s + "action"]
            new_grid, new_age = np.empty_like(grid), np.empty_like(age)
            new_dous, rgb = dous.copy(), np.empty((E, N, N, 3), np.float32)
            new_night, new_tstep = night.copy(), tstep + 1
            reward = np.empty(E, np.float32)
            for e in range(E):
                ng, na, probs = ref.update_grid(grid[e], age[e], veg[e].astype(np.int64), den[e].astype(np.int64),
                                                slope[e], dous[e], winds[widx[e], 0], 0.0, d[s + "u_burn"][e],
                                                d[s + "u_grow"][e], d[s + "new_ages"][e], C)
                diff = ng != d[s + "true_grid"][e]
                if diff.any():  # only where a burn uniform sits within rounding of its probability
                    sel = [0, 1, 2, 3, 5, 6, 7, 8]
                    close = np.abs(d[s + "u_burn"][e].reshape(N, N, 9)[..., sel]
                                   - probs.reshape(N, N, 9)[..., sel]).min(axis=-1) < 1e-6
                    assert np.all(close[diff]), (ci, t, e)
                new_grid[e], new_age[e] = d[s + "true_grid"][e], na
                assert np.array_equal(na[~diff], d[s + "fire_age"][e][~diff]), (ci, t, e)
                widx[e] = ref.wind_change(widx[e], len(winds), 0.5, d[s + "wind_u"][e], d[s + "wind_k"][e])
                taken = np.float32(np.float32(t_move + t_shoot) + t_any)
                na_t = np.float32(accu[e] + taken)
                accu[e] = np.float32(na_t - np.float32(np.trunc(na_t)))
                pos[e] = move(pos[e], int(act[e, 0]), N, N)
                if act[e, 1] == 1:
                    new_dous[e, pos[e][0], pos[e][1]] = 1
                if new_tstep[e] % 400 == 0:
                    new_night[e] = 1 - night[e]
                flags = LOOKUP[int(act[e, 2])] if ext else (0, 0)
                rgb[e], _ = ob.step_observation(new_grid[e].astype(np.int32), tuple(pos[e]), flags, int(night[e]),
                                                dous[e].astype(np.int32), bool(ext), bool(ext))
                f, tr = int((new_grid[e] == 2).sum()), int((new_grid[e] == 1).sum())
                reward[e] = -(np.float32(f) / (np.float32(tr + f) + np.float32(1e-8)))
            grid, age, dous, night, tstep = new_grid, new_age, new_dous, new_night, new_tstep
            steps_elapsed += 1
            racc = (racc + reward).astype(np.float32)
            assert np.array_equal(widx, d[s + "wind_index"]), (ci, t)
            assert np.array_equal(pos, d[s + "position"]), (ci, t)
            assert np.array_equal(accu, d[s + "time"].astype(np.float32)), (ci, t)
            assert np.array_equal(dous, d[s + "dousing_count"]), (ci, t)
            assert np.array_equal(tstep, d[s + "time_step"]) and np.array_equal(night, d[s + "is_night"]), (ci, t)
            assert np.array_equal(rgb, d[s + "rgb"]), (ci, t)
            assert np.array_equal(reward, d[s + "reward"]), (ci, t)
            assert np.array_equal((new_grid == 2).sum(axis=(1, 2)) == 0, d[s + "terminated"]), (ci, t)
            assert np.array_equal(steps_elapsed, d[s + "steps_elapsed"]), (ci, t)
            assert np.array_equal(racc, d[s + "reward_accumulated"].astype(np.float32)), (ci, t)
            stepped += E
    assert stepped >= 30
