"""Philox4x32-10 (Salmon et al., SC'11; Random123) in numpy. Test infrastructure only."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """ctr: (..., 4) uint32-like; key: (2,) or (..., 2). Returns (..., 4) uint32."""
    c = np.asarray(ctr, dtype=np.uint64) & MASK
    k = np.asarray(key, dtype=np.uint64) & MASK
    c0, c1, c2, c3 = c[..., 0], c[..., 1], c[..., 2], c[..., 3]
    k0, k1 = np.broadcast_to(k[..., 0], c0.shape).copy(), np.broadcast_to(k[..., 1], c0.shape).copy()
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK, lo1, (hi0 ^ c3 ^ k1) & MASK, lo0
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)


def seed_key(seed):
    seed = int(seed) & (2**64 - 1)
    return np.array([seed & 0xFFFFFFFF, seed >> 32], dtype=np.uint64)


def u01_f32(x):
    return (np.asarray(x, dtype=np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(2.0**-24)


def u01_f64(hi, lo):
    v = ((np.asarray(hi, dtype=np.uint64) << np.uint64(32)) | np.asarray(lo, dtype=np.uint64)) >> np.uint64(11)
    return v.astype(np.float64) * 2.0**-53


def randint_ms(x, lo, hi):
    if hi <= lo:
        return np.full(np.shape(x), lo, dtype=np.int64)
    return lo + ((np.asarray(x, dtype=np.uint64) * np.uint64(hi - lo)) >> np.uint64(32)).astype(np.int64)
