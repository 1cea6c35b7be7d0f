"""CPU: oracle/observation.py against the reference's observation builders EXECUTING (tests/golden/observation.npz,
made by tests/golden/make_golden.py::gen_observation: advanced_bulldozer.py's MDP.build_observation_on_extensions
(:988-1018), grid_to_rgb_with_extensions (:1020-1033) and grid_to_rgb (:1035-1101), with extension_utils.py's
transform_grid / apply_extensions (:89-196), run as published under a numpy stand-in for jax). Bit-exact: the RGB
frame (f32), the channel stack and, on square grids, the reset frame."""
import numpy as np

from oracle import observation as ob


def test_observation_oracle_reproduces_reference_run(golden):
    d = golden("observation")
    seen = set()
    for i in range(int(d["n"])):
        p = f"c{i}_"
        g, dous = d[p + "grid"].astype(np.int32), d[p + "dous"].astype(np.int32)
        enable, transform = (bool(v) for v in d[p + "flags"])
        a, pos, night = d[p + "actions"], tuple(int(v) for v in d[p + "pos"]), int(d[p + "night"])
        rgb, ch = ob.step_observation(g, pos, tuple(int(v) for v in a[2:]), night, dous, enable, transform)
        assert rgb.dtype == d[p + "rgb"].dtype == np.float32
        assert np.array_equal(rgb, d[p + "rgb"]), i
        assert np.array_equal(ch, d[p + "channels"]), i
        if d[p + "reset"].size:
            assert np.array_equal(ob.reset_observation(g, pos, night, dous), d[p + "reset"]), i
        seen.add((enable, transform, night, tuple(a[2:])))
    assert len(seen) >= 10  # flag combinations covered
