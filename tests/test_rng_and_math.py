"""Philox4x32-10 known-answer vectors (Random123 kat_vectors) and the deterministic exp_f32."""
import numpy as np

from oracle import alex_c
from oracle.philox import philox4x32_10

KAT = [  # counter (4), key (2), expected (4)
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_numpy_philox_kat():
    for ctr, key, exp in KAT:
        assert tuple(int(v) for v in philox4x32_10(np.array(ctr), np.array(key))) == exp


def test_c_philox_matches_numpy():
    rng = np.random.default_rng(1)
    ctr = rng.integers(0, 2**32, size=(1000, 4), dtype=np.uint64)
    for k0, k1 in [(0, 0), (123, 456), (0xFFFFFFFF, 7)]:
        a = alex_c.philox(ctr.astype(np.uint32), k0, k1)
        b = philox4x32_10(ctr, np.array([k0, k1]))
        assert np.array_equal(a, b)


def test_exp_f32_accuracy_one_ulp():
    x = np.concatenate([np.linspace(-80, 80, 20001), np.float32(0.078) * np.linspace(-90, 90, 5001)]).astype(np.float32)
    y = alex_c.exp_f32(x)
    ref = np.exp(x.astype(np.float64))
    ulp = np.spacing(ref.astype(np.float32)).astype(np.float64)
    assert np.max(np.abs(y - ref) / ulp) <= 1.0
    assert alex_c.exp_f32(np.float32(0.0)) == 1.0


def test_slope_factor_accuracy_and_reciprocity():
    """p_slope = slope_factor(a): exp_f32(a) for a >= 0, 1/exp_f32(-a) below 0 — within 2 ulp of exp and
    the two directions of an edge are exact reciprocals (what the edge-slope layout relies on)."""
    a = (np.float32(0.078) * np.linspace(-90, 90, 20001).astype(np.float32)).astype(np.float32)
    y = alex_c.slope_factor(a)
    ref = np.exp(a.astype(np.float64))
    ulp = np.spacing(ref.astype(np.float32)).astype(np.float64)
    assert np.max(np.abs(y - ref) / ulp) <= 2.0
    pos = a[a > 0]
    assert np.array_equal(alex_c.slope_factor(-pos), (np.float32(1) / alex_c.slope_factor(pos)).astype(np.float32))
    # the edge layout: V from the slope, then both directions from V alone
    s = np.linspace(-89.9, 89.9, 4001).astype(np.float32)
    own, nbr = alex_c.factor_pairs(alex_c.signed_factors(s))
    a = (np.float32(0.078) * s).astype(np.float32)
    assert np.array_equal(own, alex_c.slope_factor(a))
    assert np.array_equal(nbr, alex_c.slope_factor(-a))
