"""Timeline of one batched Windy env step (gca_bulldozer_step_fused) from a diagnostic build of the library with
s_memrealtime stamps (100 MHz) at the phase boundaries of every workgroup (thread 0): entry, inputs loaded, direction
mask + barrier, the CA strips (wave 0), the count barrier, the final stores. Run with GCA_LIB_PATH pointing at that
build (scripts/build_variant.sh from a stamped source tree; not shipped). One JSON line of per-phase statistics."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def main(N=256, steps=8):
    import torch

    import bench
    from gymca_amd import _device as dev
    from gymca_amd import _lib
    from gymca_amd._lib import call
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    E = 1024
    env = BatchedForestFireBulldozerEnv(E, N, N, device=device, seed=0x5EED, materialize_obs=False)
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)

    def one_step():
        call("gca_random_actions", dev.ptr(action), E, 0, 9, dev.ptr(env.rng_step), dev.stream_ptr(device))
        env.step(action)

    restore = bench.env_snapshot(env, one_step, 64)
    restore()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    buf = np.zeros((4096, 8), np.uint64)
    rows = []
    for _ in range(steps):
        call("gca_random_actions", dev.ptr(action), E, 0, 9, dev.ptr(env.rng_step), dev.stream_ptr(device))
        torch.cuda.synchronize()
        env.step(action)
        torch.cuda.synchronize()
        assert lib.gca_debug_windy_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
        st = buf[:E].astype(np.int64)
        n = (st[:, 7] & 0xFF).astype(np.int64) - 16
        t0 = st[:, 0].min()
        rel = (st[:, :6] - t0) * 10 / 1000.0  # us
        stepping = n > 0
        done_before = n < 0
        row = {"n_stepping": int(stepping.sum()), "start_skew_us": float(rel[:, 0].max()),
               "span_us": float(rel[~done_before, 5].max())}
        for k, name in ((1, "inputs"), (2, "mask_barrier"), (3, "strips"), (4, "count_barrier"), (5, "post")):
            prev = 0 if k != 5 else 4
            prev = k - 1 if k != 5 else 4
            d = rel[stepping, k] - rel[stepping, prev]
            row[f"stepping_{name}_us"] = float(d.mean()) if d.size else None
        ns = (~stepping) & (~done_before)
        row["nonstepping_total_us"] = float((rel[ns, 5] - rel[ns, 0]).mean()) if ns.any() else None
        row["stepping_end_us_max"] = float(rel[stepping, 5].max()) if stepping.any() else None
        row["stepping_start_us_mean"] = float(rel[stepping, 0].mean()) if stepping.any() else None
        rows.append(row)
    keys = rows[0].keys()
    out = {"N": N, "E": E, "steps": steps}
    for k in keys:
        vals = [r[k] for r in rows if r[k] is not None]
        out[k] = round(float(np.mean(vals)), 3) if vals else None
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(N=int(sys.argv[1]) if len(sys.argv) > 1 else 256)
