"""GPU: the device Advanced env against the reference env EXECUTING (tests/golden/advanced_env.npz: the reference
AdvancedForestFireBulldozerEnv stepped through stateless_step under the numpy stand-in for jax, see
tests/test_advanced_env_golden.py for the oracle side).

The CA half of each recorded step is the drop-in operator with the reference's own draws injected
(test_gpu_alexandridis_jax_golden.py pins it on the rule fixture; here it runs on the env's state, dousing included).
The rest of the step is the device env's own post-step launch (gca_advenv_post: RepeatCAJax's f32 clock, MoveModify with
the border clamps and the shot, time_step / day-night, reward, terminated, the info counters) and its frame
(gca_adv_observation), started from the reference's pre-step state with the reference's post-CA grid in place. Every
output is compared bit for bit; the wind change draws from the env's Philox stream, so wind_index is checked through the
operator with the recorded draws instead."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ci", [0, 1])
def test_device_env_reproduces_reference_env_run(device, golden, ci):
    import torch

    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv
    from gymca_amd.forest_fire.operators import PartiallyObservableForestFireJax

    d = golden("advanced_env")
    c = f"c{ci}_"
    N, E, steps, ext = (int(v) for v in d[c + "meta"])
    env = AdvancedForestFireBulldozerEnv(N, N, key=7, num_envs=E, use_hidden=False, device=device, observation="rgb",
                                         enable_extensions=bool(ext))
    env.reset()
    op = PartiallyObservableForestFireJax(N, 0, 1, 2)
    shared = {"winds": d[c + "winds"], "p_tree": np.float32(0.0), "p_wind_change": np.float32(0.5)}
    veg, den, slope = d[c + "init_vegetation"], d[c + "init_density"], d[c + "init_slope"]
    pre = {k: d[c + "init_" + k] for k in ("true_grid", "fire_age", "dousing_count", "wind_index", "position", "time",
                                           "time_step", "is_night")}
    se = np.zeros(E, np.float32)
    ra = np.zeros(E, np.float32)

    def put(t, x):
        t.copy_(torch.as_tensor(np.asarray(x), device=device).to(t.dtype).reshape(t.shape))

    for t in range(steps):
        s = f"{c}s{t}_"
        act = d[s + "action"].astype(np.int32)
        # the CA half: the operator on each env's pre-step state with the reference's draws
        for e in range(E):
            ctx = {"density": den[e].astype(np.int64), "vegetation": veg[e].astype(np.int64), "slope": slope[e],
                   "dousing_count": pre["dousing_count"][e].astype(np.int32), "key": np.array([0, 7], np.uint32),
                   "fire_age": pre["fire_age"][e], "wind_index": np.int32(pre["wind_index"][e])}
            draws = {"burn": d[s + "u_burn"][e], "grow": d[s + "u_grow"][e], "age": d[s + "new_ages"][e],
                     "wind_u": d[s + "wind_u"][e], "wind_k": d[s + "wind_k"][e]}
            ng, ctx2, _ = op.update(pre["true_grid"][e].astype(np.float32), None, ctx, shared, draws=draws)
            assert np.array_equal(ng, d[s + "true_grid"][e]), (t, e)
            assert np.array_equal(np.asarray(ctx2["fire_age"]).astype(np.float32), d[s + "fire_age"][e]), (t, e)
            assert int(ctx2["wind_index"]) == int(d[s + "wind_index"][e]), (t, e)
        # the rest of the step: the device env's post-step launch and frame from the reference's pre-step state
        env.set_state(grid=d[s + "true_grid"], dousing=pre["dousing_count"], position=pre["position"])
        put(env.accu, pre["time"])
        put(env.time_step, pre["time_step"])
        put(env.is_night, pre["is_night"])
        put(env.steps_elapsed, se)
        put(env.reward_accumulated, ra)
        full = torch.as_tensor(act, device=device).contiguous()
        env.post_step(full[:, :2].contiguous(), stats=True)
        env.render_observation(full)
        torch.cuda.synchronize(device)
        got = {"position": env.pos, "time": env.accu, "time_step": env.time_step, "is_night": env.is_night,
               "dousing_count": env.dousing, "reward": env.reward, "steps_elapsed": env.steps_elapsed,
               "reward_accumulated": env.reward_accumulated, "rgb": env.rgb}
        for k, v in got.items():
            want = d[s + k]
            assert np.array_equal(v.cpu().numpy().astype(want.dtype).reshape(want.shape), want), (t, k)
        assert np.array_equal(env.done.bool().cpu().numpy(), d[s + "terminated"].astype(bool)), t
        pre = {"true_grid": d[s + "true_grid"], "fire_age": d[s + "fire_age"], "dousing_count": d[s + "dousing_count"],
               "wind_index": d[s + "wind_index"], "position": d[s + "position"], "time": d[s + "time"],
               "time_step": d[s + "time_step"], "is_night": d[s + "is_night"]}
        se, ra = d[s + "steps_elapsed"].astype(np.float32), d[s + "reward_accumulated"].astype(np.float32)
