"""A numpy stand-in for the five names the reference's JAX modules import (jnp, jit, vmap, random, lax).

Fixture-generation infrastructure for make_golden.py only (it runs in the build container, where the
reference lives and jax is absent). It lets the reference's own JAX code execute as published, so the
fixtures it yields come from the reference running, not from a restatement:

  jnp     numpy, with jax's dtype rules under the default x64-disabled mode: every array is canonical
          (float64 -> float32, int64 -> int32), float literals / jnp.array / jnp.zeros default to float32,
          an integer or bool array meeting a float array is converted to that float type BEFORE the
          operation (jax's promotion lattice: int32 * float32 -> float32, where numpy would give float64),
          python scalars are weakly typed; `.at[idx].set(v)` is the functional update; out-of-bounds integer
          indices are clamped (jax's gather) instead of raising; `x += y` rebinds (jax arrays are immutable)
  jit     identity (also `partial(jit, static_argnums=...)`)
  vmap    an explicit loop over `in_axes` (tuples of arrays map leaf-wise), results stacked on axis 0
  lax     dynamic_slice as a slice (start indices clamped like lax does), switch (index clamped)
  random  keys are opaque tokens; every draw (uniform / randint / normal / poisson) comes from a numpy
          Generator and is logged in call order, so a fixture can inject the very arrays the rule consumed.
          randint truncates non-integer bounds to int first, like jax.random.randint (minval.astype(int)).

What the stand-in cannot reproduce is XLA's own floating-point evaluation order: a sum over a window runs in
numpy's order here (pairwise), and exp is numpy's float32 exp. Both differ from XLA's by at most an ulp or
two, which is why the parity tests hold probabilities to 1e-6 and integer states to equality except where a
uniform draw lies within 1e-6 of its probability.
"""
import dataclasses
import sys
import types
from contextlib import contextmanager

import numpy as np

_CANON = {np.dtype(np.float64): np.dtype(np.float32), np.dtype(np.int64): np.dtype(np.int32),
          np.dtype(np.uint64): np.dtype(np.uint32)}


def _canon_dtype(dt):
    dt = np.dtype(dt)
    return _CANON.get(dt, dt)


class JArray(np.ndarray):
    """ndarray with jax.numpy's (x64-disabled) promotion and the functional .at[] update."""

    def __array_ufunc__(self, ufunc, method, *inputs, out=None, **kw):
        if out is not None:
            raise TypeError("jax arrays are immutable")
        args = _promote(inputs) if method == "__call__" and ufunc.nin == 2 else [_canon(a) for a in inputs]
        args = [np.asarray(a) if isinstance(a, np.ndarray) else a for a in args]
        res = getattr(ufunc, method)(*args, **kw)
        if isinstance(res, tuple):
            return tuple(wrap(r) for r in res)
        return wrap(res)

    def __array_function__(self, func, types_, args, kwargs):
        def strip(x):
            if isinstance(x, JArray):
                return x.view(np.ndarray)
            if isinstance(x, (list, tuple)):
                return type(x)(strip(v) for v in x)
            return x

        res = func(*strip(args), **{k: strip(v) for k, v in kwargs.items()})
        if isinstance(res, np.ndarray):
            return wrap(res)
        if isinstance(res, (list, tuple)):
            return type(res)(wrap(r) if isinstance(r, np.ndarray) else r for r in res)
        return res

    @property
    def at(self):
        return _At(self)

    def __getitem__(self, idx):
        return super().__getitem__(_clamp_index(self.shape, idx))

    def __iter__(self):  # iteration stops at the end (indexing itself clamps and would never raise)
        sup = super().__getitem__
        return (sup(i) for i in range(len(self)))

    # jax arrays are immutable: `x += y` rebinds x to a new array
    def __iadd__(self, o):
        return self + o

    def __isub__(self, o):
        return self - o

    def __imul__(self, o):
        return self * o

    def __itruediv__(self, o):
        return self / o


def _clamp_index(shape, idx):
    """jnp indexing: integer indices (scalars or arrays) are normalised (negative from the end) and then CLAMPED
    to the axis, as jax's gather does out of bounds, instead of raising like numpy."""
    if not isinstance(idx, tuple):
        idx = (idx,)
    n_used = sum(0 if (i is None or i is Ellipsis) else (np.ndim(i) if _is_bool(i) else 1) for i in idx)
    out, ax = [], 0
    for i in idx:
        if i is None:
            out.append(i)
        elif i is Ellipsis:
            out.append(i)
            ax += len(shape) - n_used
        elif isinstance(i, slice) or _is_bool(i):
            out.append(i.view(np.ndarray) if isinstance(i, JArray) else i)
            ax += np.ndim(i) if _is_bool(i) else 1
        elif isinstance(i, (int, np.integer)) or (isinstance(i, np.ndarray) and np.issubdtype(i.dtype, np.integer)):
            d = shape[ax]
            v = np.asarray(i).view(np.ndarray)
            v = np.clip(np.where(v < 0, v + d, v), 0, d - 1)
            out.append(int(v) if v.ndim == 0 else v)
            ax += 1
        else:
            out.append(i)
            ax += 1
    return tuple(out)


def _is_bool(i):
    return isinstance(i, np.ndarray) and i.dtype == np.bool_


class _At:
    def __init__(self, a):
        self.a = a

    def __getitem__(self, idx):
        return _AtIdx(self.a, idx)


class _AtIdx:
    def __init__(self, a, idx):
        self.a, self.idx = a, idx

    def set(self, v):
        r = np.array(self.a.view(np.ndarray), copy=True)
        r[_plain(self.idx)] = np.asarray(v).astype(r.dtype)
        return wrap(r)


def _plain(idx):
    if isinstance(idx, tuple):
        return tuple(_plain(i) for i in idx)
    return idx.view(np.ndarray) if isinstance(idx, JArray) else idx


def _canon(a):
    if isinstance(a, np.ndarray):
        dt = _canon_dtype(a.dtype)
        return a if dt == a.dtype else a.astype(dt)
    if isinstance(a, np.generic):  # numpy scalars are strongly typed in jax, then canonicalised
        return np.asarray(a).astype(_canon_dtype(a.dtype))
    return a


def wrap(x):
    if isinstance(x, np.ndarray) or isinstance(x, np.generic):
        a = np.asarray(x)
        dt = _canon_dtype(a.dtype)
        if dt != a.dtype:
            a = a.astype(dt)
        return a.view(JArray)
    return x


def _promote(inputs):
    """jax's binary promotion: a float operand makes int/bool operands (and python scalars) that float type;
    integers meeting a python float become float32 (the default float type)."""
    xs = [_canon(a) for a in inputs]
    arrs = [a for a in xs if isinstance(a, np.ndarray)]
    fl = [a.dtype for a in arrs if np.issubdtype(a.dtype, np.floating)]
    if fl:
        ft = np.result_type(*fl)
    elif any(isinstance(a, float) for a in xs):
        ft = np.dtype(np.float32)
    else:
        return xs
    out = []
    for a in xs:
        if isinstance(a, np.ndarray):
            out.append(a if np.issubdtype(a.dtype, np.floating) else a.astype(ft))
        elif isinstance(a, (int, float, bool)):
            out.append(ft.type(a))
        else:
            out.append(a)
    return out


# ------------------------------------------------------------------------------------------- jax.numpy
def _make_jnp():
    jnp = types.ModuleType("jax.numpy")

    def array(x, dtype=None):
        if isinstance(x, np.ndarray) and dtype is None:
            return wrap(np.array(x, copy=True))
        a = np.array(x, dtype=dtype)
        if dtype is None and np.issubdtype(a.dtype, np.floating):
            a = a.astype(np.float32)
        return wrap(a)

    def asarray(x, dtype=None):
        return wrap(np.asarray(x, dtype=dtype)) if dtype is not None or isinstance(x, np.ndarray) else array(x)

    def zeros(shape, dtype=None):
        return wrap(np.zeros(shape, dtype=np.float32 if dtype is None else dtype))

    def ones(shape, dtype=None):
        return wrap(np.ones(shape, dtype=np.float32 if dtype is None else dtype))

    def zeros_like(a, dtype=None):
        return wrap(np.zeros(np.shape(a), dtype=np.asarray(a).dtype if dtype is None else dtype))

    def full(shape, fill_value, dtype=None):
        v = np.asarray(fill_value)
        if dtype is None and np.issubdtype(v.dtype, np.floating):
            dtype = np.float32
        return wrap(np.broadcast_to(v.astype(dtype) if dtype is not None else v, shape).copy())

    def where(c, x, y):
        c = np.asarray(c)
        x2, y2 = _promote([x, y])
        return wrap(np.where(c, np.asarray(x2), np.asarray(y2)))

    def pad(a, pad_width, mode="constant", constant_values=0):
        a = np.asarray(a)
        if mode != "constant":
            return wrap(np.pad(a, pad_width, mode=mode))
        return wrap(np.pad(a, pad_width, mode=mode, constant_values=np.asarray(constant_values).astype(a.dtype)))

    def arange(*a, dtype=None):
        r = np.arange(*a)
        return wrap(r.astype(dtype) if dtype is not None else r)

    def meshgrid(*xs, indexing="xy"):
        return [wrap(m) for m in np.meshgrid(*[np.asarray(x) for x in xs], indexing=indexing)]

    def clip(a, lo=None, hi=None):
        return wrap(np.clip(np.asarray(_canon(a)), lo, hi))

    def stack(xs, axis=0):
        return wrap(np.stack([np.asarray(x) for x in xs], axis=axis))

    def passthrough(name):
        f = getattr(np, name)

        def g(*a, **k):
            r = f(*[_canon(x) if isinstance(x, np.ndarray) else x for x in a], **k)
            return tuple(wrap(x) for x in r) if isinstance(r, tuple) else wrap(r)

        g.__name__ = name
        return g

    for name, f in dict(array=array, asarray=asarray, zeros=zeros, ones=ones, zeros_like=zeros_like, full=full,
                        where=where, pad=pad, arange=arange, meshgrid=meshgrid, clip=clip, stack=stack).items():
        setattr(jnp, name, f)
    for name in ("exp", "log", "sqrt", "round", "minimum", "maximum", "max", "min", "sum", "any", "all", "argmax",
                 "abs", "floor", "ceil", "mean", "logical_and", "logical_or", "logical_not", "ones_like",
                 "concatenate", "repeat", "tile", "transpose", "expand_dims", "roll", "sign", "cos", "sin",
                 "arctan2", "arctan", "degrees", "radians", "cumsum", "einsum", "flip", "isclose", "diff", "modf", "take",
                 "invert", "full_like", "trunc", "count_nonzero", "unique"):
        setattr(jnp, name, passthrough(name))
    for name in ("float32", "int32", "uint8", "uint32", "int8", "int16", "bool_", "pi", "newaxis", "ndarray",
                 "issubdtype", "integer", "floating", "inf", "nan"):
        setattr(jnp, name, getattr(np, name))
    jnp.float64, jnp.int64 = np.float32, np.int32  # x64 disabled: the 64-bit names alias the 32-bit types
    return jnp


# ------------------------------------------------------------------------------------------- jit / vmap / lax
def jit(fun=None, **_):
    if fun is None:
        return lambda f: f
    return fun


def _take(a, axis, i):
    """Index i of `a` along `axis`; `axis` may be a pytree prefix of `a` (a dict / tuple of axes, None = unmapped)."""
    if axis is None:
        return a
    if isinstance(axis, dict):
        return {k: _take(v, axis.get(k), i) for k, v in a.items()}
    if isinstance(axis, (tuple, list)):
        return type(a)(_take(x, ax, i) for x, ax in zip(a, axis))
    if isinstance(a, (tuple, list)):
        return type(a)(_take(x, axis, i) for x in a)
    if isinstance(a, dict):
        return {k: _take(v, axis, i) for k, v in a.items()}
    return wrap(np.take(np.asarray(a), i, axis=axis))


def _sizes(a, axis):
    if axis is None:
        return set()
    if isinstance(axis, dict):
        return set().union(*[_sizes(v, axis.get(k)) for k, v in a.items()])
    if isinstance(axis, (tuple, list)):
        return set().union(*[_sizes(x, ax) for x, ax in zip(a, axis)])
    if isinstance(a, (tuple, list)):
        return set().union(*[_sizes(x, axis) for x in a])
    if isinstance(a, dict):
        return set().union(*[_sizes(v, axis) for v in a.values()])
    return {np.shape(a)[axis]}


def _stack_tree(outs):
    o0 = outs[0]
    if isinstance(o0, (tuple, list)):
        return type(o0)(_stack_tree([o[k] for o in outs]) for k in range(len(o0)))
    if isinstance(o0, dict):
        return {k: _stack_tree([o[k] for o in outs]) for k in o0}
    return wrap(np.stack([np.asarray(o) for o in outs]))


def vmap(fun, in_axes=0, out_axes=0):
    assert out_axes == 0

    def mapped(*args):
        axes = tuple(in_axes) if isinstance(in_axes, (tuple, list)) else (in_axes,) * len(args)
        n = set().union(*[_sizes(a, ax) for a, ax in zip(args, axes)])
        assert len(n) == 1, f"vmap: mapped axes differ in size {n}"
        outs = [fun(*[a if ax is None else _take(a, ax, i) for a, ax in zip(args, axes)]) for i in range(n.pop())]
        return _stack_tree(outs)

    return mapped


def _make_lax():
    lax = types.ModuleType("jax.lax")

    def dynamic_slice(a, start, sizes):
        a = np.asarray(a)
        st = [int(min(max(int(s), 0), d - z)) for s, d, z in zip(start, a.shape, sizes)]  # lax clamps starts
        return wrap(a[tuple(slice(s, s + z) for s, z in zip(st, sizes))])

    def switch(index, branches, *operands):
        return branches[int(np.clip(int(index), 0, len(branches) - 1))](*operands)  # lax.switch clamps the index

    lax.dynamic_slice, lax.switch = dynamic_slice, switch
    return lax


# ------------------------------------------------------------------------------------------- jax.random
class RandomLog:
    """jax.random stand-in: draws from `gen`, logged as (kind, shape, value, bounds) in call order.

    `uniform_scale` maps a draw's shape to a factor in (0, 1] applied to that uniform array (a fixture may
    bias one stream towards ignitions; the logged value is what the rule consumed)."""

    def __init__(self, gen, uniform_scale=None):
        self.gen, self.log, self.uniform_scale = gen, [], uniform_scale or (lambda shape: 1.0)
        self._k = 0

    def module(self):
        r = types.ModuleType("jax.random")
        r.split, r.uniform, r.randint, r.normal, r.poisson, r.PRNGKey = (
            self.split, self.uniform, self.randint, self.normal, self.poisson, self.key)
        r.key = self.key
        return r

    def key(self, seed=0):
        self._k += 1
        return wrap(np.array([self._k, 0], dtype=np.uint32))

    def split(self, key, num=2):
        """An array of `num` fresh key tokens, shape (num, 2) like jax's keys (rows unpack and vmap like them)."""
        rows = []
        for _ in range(num):
            self._k += 1
            rows.append((self._k, 0))
        return wrap(np.array(rows, dtype=np.uint32))

    def uniform(self, key, shape=(), dtype=None, minval=0.0, maxval=1.0):
        shape = tuple(shape)
        v = self.gen.random(shape, dtype=np.float32) * np.float32(self.uniform_scale(shape))
        v = (np.float32(minval) + v * np.float32(maxval - minval)).astype(np.float32)
        self.log.append(("uniform", shape, v, (minval, maxval)))
        return wrap(v)

    def randint(self, key, shape, minval, maxval, dtype=None):
        lo, hi = int(minval), int(maxval)  # jax.random.randint: non-integer bounds -> astype(int)
        v = self.gen.integers(lo, hi, size=tuple(shape)).astype(np.int32)
        self.log.append(("randint", tuple(shape), v, (lo, hi)))
        return wrap(v)

    def normal(self, key, shape=(), dtype=None):
        v = self.gen.standard_normal(tuple(shape), dtype=np.float32)
        self.log.append(("normal", tuple(shape), v, None))
        return wrap(v)

    def poisson(self, key, lam, shape=()):
        v = self.gen.poisson(lam, size=tuple(shape)).astype(np.int32)
        self.log.append(("poisson", tuple(shape), v, lam))
        return wrap(v)


@contextmanager
def installed(rlog):
    """Put jax / jax.numpy / jax.random / jax.lax (and an empty flax) into sys.modules for the duration."""
    jax = types.ModuleType("jax")
    jnp, lax, rnd = _make_jnp(), _make_lax(), rlog.module()
    jax.numpy, jax.lax, jax.random, jax.jit, jax.vmap = jnp, lax, rnd, jit, vmap
    jax.debug = types.SimpleNamespace(callback=lambda *a, **k: None, print=lambda *a, **k: None)
    flax = types.ModuleType("flax")
    flax.struct = types.SimpleNamespace(dataclass=lambda c=None, **k: dataclasses.dataclass(frozen=True)(c)
                                        if c is not None else dataclasses.dataclass(frozen=True))
    names = ("jax", "jax.numpy", "jax.lax", "jax.random", "flax", "flax.struct")
    saved = {k: sys.modules.get(k) for k in names}
    sys.modules.update({"jax": jax, "jax.numpy": jnp, "jax.lax": lax, "jax.random": rnd, "flax": flax,
                        "flax.struct": flax.struct})
    try:
        yield jax
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
