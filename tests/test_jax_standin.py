"""CPU: the numpy stand-in for jax that tests/golden/make_golden.py runs the reference's JAX modules under
(tests/golden/_jax_standin.py) follows jax's documented semantics where numpy's differ — the fixtures
alexandridis_jax.npz / observation.npz are only as good as these rules."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import _jax_standin as js  # noqa: E402


def _jnp():
    rl = js.RandomLog(np.random.default_rng(0))
    with js.installed(rl) as jax:
        return jax.numpy, jax, rl


def test_x64_disabled_dtypes_and_promotion():
    jnp, _, _ = _jnp()
    assert jnp.array([0.5, 1.0]).dtype == np.float32 and jnp.zeros((2,)).dtype == np.float32
    assert jnp.array(np.arange(3)).dtype == np.int32  # int64 input canonicalised
    i = jnp.array(np.array([1, 2, 3], np.int32))
    f = jnp.array(np.array([0.1, 0.2, 0.3], np.float32))
    assert (i * f).dtype == np.float32  # numpy: float64
    assert (i * 0.5).dtype == np.float32  # an int array meeting a python float: the default float type
    assert (f * 2).dtype == np.float32 and (1 - f).dtype == np.float32
    assert jnp.where(np.array([True, False, True]), i, f).dtype == np.float32
    # int32 * f32 is evaluated in f32 (the int converted first), as XLA does; numpy's float64 product rounds
    # differently: f32(16777217) * 3 = 50331648, while f32(16777217 * 3.0) = 50331652
    big = jnp.array(np.array([16777217], np.int32))
    assert (big * jnp.array(np.array([3.0], np.float32)))[0] == np.float32(50331648.0)
    assert np.float32(np.array([16777217], np.int32) * np.array([3.0], np.float32))[0] == np.float32(50331652.0)


def test_functional_update_clamped_gather_and_immutable_iadd():
    jnp, _, _ = _jnp()
    a = jnp.zeros((3, 3))
    b = a.at[1, 1].set(5.0)
    assert float(a[1, 1]) == 0.0 and float(b[1, 1]) == 5.0
    x = jnp.array(np.arange(4, dtype=np.int32))
    assert int(x[7]) == 3 and int(x[-1]) == 3  # out-of-bounds gathers clamp
    y = x
    y += 1
    assert int(x[0]) == 0 and int(y[0]) == 1  # += rebinds
    assert [int(v) for v in x] == [0, 1, 2, 3]  # iteration stops at the end


def test_vmap_lax_and_logged_random():
    jnp, jax, rl = _jnp()
    out = jax.vmap(lambda r, c, g: g[r, c], in_axes=(0, 0, None))(np.array([0, 1]), np.array([1, 0]),
                                                                     np.array([[1, 2], [3, 4]]))
    assert out.tolist() == [2, 3]
    padded = jnp.pad(np.arange(9).reshape(3, 3), 1, mode="constant", constant_values=0.0)
    assert jax.lax.dynamic_slice(padded, (0, 0), (3, 3)).shape == (3, 3)
    assert jax.lax.switch(5, [lambda: 0, lambda: 1]) == 1  # index clamped
    k1, k2 = jax.random.split(jax.random.PRNGKey(0))
    u = jax.random.uniform(k1, (4,))
    r = jax.random.randint(k2, (3,), 576.0, 672.0)  # float bounds truncated to int, like jax
    assert u.dtype == np.float32 and r.dtype == np.int32 and r.min() >= 576 and r.max() < 672
    assert [e[0] for e in rl.log] == ["uniform", "randint"] and rl.log[1][3] == (576, 672)
