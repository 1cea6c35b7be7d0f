"""Per-env host draws keyed by the GLOBAL env id, so a sharded run (envs [offset, offset + count) per rank)
draws exactly what the unsharded run draws for the same envs. Used for the few O(E) reset
draws made on the host (fire / bulldozer noise, initial wind index); every per-cell draw is Philox on the device.
"""
import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M
    return x ^ (x >> np.uint64(31))


def env_draws(seed, env_ids, tag):
    """uint64 [len(env_ids)]: an independent 64-bit word per (seed, global env id, tag)."""
    with np.errstate(over="ignore"):
        ids = np.asarray(env_ids, dtype=np.uint64)
        h = _splitmix64(np.uint64(int(seed) & 0xFFFFFFFFFFFFFFFF) ^ np.uint64(int(tag) & 0xFFFFFFFF))
        return _splitmix64(h ^ _splitmix64(ids))


def env_integers(seed, env_offset, count, tag, low, high):
    """Integers in [low, high) per env (multiply-shift on the top 32 bits; high - low < 2**32)."""
    ids = np.arange(int(env_offset), int(env_offset) + int(count), dtype=np.uint64)
    span = int(high) - int(low)
    if span <= 0:
        return np.full(int(count), int(low), dtype=np.int64)
    top = env_draws(seed, ids, tag) >> np.uint64(32)
    return int(low) + ((top * np.uint64(span)) >> np.uint64(32)).astype(np.int64)
