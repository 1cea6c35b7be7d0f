"""The C-ABI library loads and exports every symbol include/gca.h declares; ctypes
struct layouts equal the C compiler's. No compute calls (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gca.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gca_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from gymca_amd import _lib

    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_lib.EXPORTED_SYMBOLS), set(names) ^ set(_lib.EXPORTED_SYMBOLS)


def declared_arities():
    """{function: number of parameters} from the prototypes in include/gca.h."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(gca_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_ctypes_signatures_match_the_header_arity():
    """Every ctypes signature passes as many arguments as the header's prototype takes (a stale table shifts every
    argument after the difference)."""
    from gymca_amd import _lib

    ar = declared_arities()
    assert len(ar) >= 20
    bad = {n: (len(_lib._SIGNATURES[n][0]), k) for n, k in ar.items() if len(_lib._SIGNATURES[n][0]) != k}
    assert not bad, bad


def test_version_and_error_calls_need_no_gpu():
    from gymca_amd import _lib

    lib = _lib.load()
    assert lib.gca_version() == 1
    assert isinstance(lib.gca_last_error(), bytes)


def test_argument_errors_are_reported_without_touching_the_gpu():
    from gymca_amd import _lib

    with pytest.raises(_lib.GCAError, match="E, H, W must be positive"):
        _lib.call("gca_windy_step", 1, 1, None, None, 0, 1, 0, 4, 4, 0, 3, 25, 0, None, None)
    with pytest.raises(_lib.GCAError, match="burn radius"):
        p = _lib.AlexParams()
        p.R = 0
        _lib.call("gca_alex_step", p, 1, 4, 4, *([1] * 9), None, None, None, None, None, None, None)


C_LAYOUT = r"""
#include <stdio.h>
#include <stddef.h>
#include "gca.h"
#define P(T, f) printf("%s.%s %zu\n", #T, #f, offsetof(T, f));
int main(void) {
  printf("gca_bulldozer_params %zu\n", sizeof(gca_bulldozer_params));
  P(gca_bulldozer_params, t_shoot) P(gca_bulldozer_params, seed) P(gca_bulldozer_params, right_mask)
  P(gca_bulldozer_params, effect)
  printf("gca_alex_params %zu\n", sizeof(gca_alex_params));
  P(gca_alex_params, heat_dw) P(gca_alex_params, p_tree) P(gca_alex_params, seed) P(gca_alex_params, n_winds)
  P(gca_alex_params, winds)
  printf("gca_advenv_params %zu\n", sizeof(gca_advenv_params));
  P(gca_advenv_params, day_length) P(gca_advenv_params, seed) P(gca_advenv_params, right_mask)
  printf("gca_obs_params %zu\n", sizeof(gca_obs_params));
  P(gca_obs_params, ext_skip_blur) P(gca_obs_params, day_length) P(gca_obs_params, color_night)
  P(gca_obs_params, tint_night) P(gca_obs_params, ext_lookup)
  printf("gca_pine_params %zu\n", sizeof(gca_pine_params));
  P(gca_pine_params, max_pinecones) P(gca_pine_params, dy) P(gca_pine_params, scale) P(gca_pine_params, den1p)
  P(gca_pine_params, seed) P(gca_pine_params, fire)
  printf("gca_pine_classic_params %zu\n", sizeof(gca_pine_classic_params));
  P(gca_pine_classic_params, dx) P(gca_pine_classic_params, burn_thr) P(gca_pine_classic_params, age_hi)
  P(gca_pine_classic_params, seed) P(gca_pine_classic_params, fire)
  return 0;
}
"""


def test_struct_layouts_match_the_header(tmp_path):
    from gymca_amd import _lib

    src = tmp_path / "layout.c"
    src.write_text(C_LAYOUT)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = dict(line.rsplit(" ", 1) for line in out if line)
    py = {"gca_bulldozer_params": _lib.BulldozerParams, "gca_alex_params": _lib.AlexParams,
          "gca_advenv_params": _lib.AdvEnvParams, "gca_obs_params": _lib.ObsParams,
          "gca_pine_params": _lib.PineParams, "gca_pine_classic_params": _lib.PineClassicParams}
    for key, val in got.items():
        if "." in key:
            t, f = key.split(".")
            assert getattr(py[t], f).offset == int(val), key
        else:
            assert ctypes.sizeof(py[key]) == int(val), key


def test_bound_call_converts_once_and_checks_arity():
    """_lib.BoundCall (the batched envs' pre-bound step call): every argument converted to its declared ctypes type
    at bind time, structs by reference, SLOT positions rebound per call; wrong arities refused before any call."""
    from gymca_amd import _lib

    p = _lib.BulldozerParams()
    args = [p, _lib.SLOT] + [0x1000 + 16 * i for i in range(4)] + [9] + [0x2000 + 16 * i for i in range(4)] + \
        [256, 256] + [0x3000 + 16 * i for i in range(6)] + [1024, _lib.SLOT]
    bc = _lib.BoundCall("gca_bulldozer_step_fused", *args)
    assert len(bc._slots) == 2 and len(bc._args) == len(args)
    assert isinstance(bc._args[6], ctypes.c_int64) and bc._args[6].value == 9
    assert isinstance(bc._args[2], ctypes.c_void_p) and bc._args[2].value == 0x1000
    p.t_any = 0.25  # bound by reference: the call sees later edits of the struct
    assert ctypes.cast(bc._args[0], ctypes.POINTER(_lib.BulldozerParams)).contents.t_any == 0.25
    with pytest.raises(TypeError):
        _lib.BoundCall("gca_bulldozer_step_fused", *args[:-1])
    with pytest.raises(TypeError):
        _lib.BoundCall("gca_bulldozer_step_fused", _lib.SLOT, *args[1:])
    with pytest.raises(TypeError):
        bc(0x4000)  # two per-call values expected
