"""Phase profile of the headline Alexandridis step (diagnostics build, scripts/build_variant.sh stamps
-DGCA_ALEX_STAMPS): s_memtime at the phase boundaries of every 64th workgroup of one 4096 x 256^2 launch
from the bench's config-3 state. Prints one JSON line: mean cycles per wave in each phase and the span of
workgroup lifetimes. Run: GCA_LIB_PATH=.../variants/stamps.so python scripts/alex_stamps.py"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]

PHASES = ["staging+LDS writes (to the 1st barrier)", "column prefix (to the 2nd barrier)", "heat",
          "direction pass (slope loads)", "draws + rule", "stores (+ frame)"]


def main():
    import torch

    import bench
    from gymca_amd import _lib
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    env = AdvancedForestFireBulldozerEnv(256, 256, key=1, num_envs=4096, use_hidden=False, device=device,
                                         observation="grid")
    env.reset()
    for _ in range(6):
        bench.synthetic_state(env, 0, device)
        env.ca_step()
    torch.cuda.synchronize()
    bench.synthetic_state(env, 0, device)
    torch.cuda.synchronize()
    env.ca_step()
    torch.cuda.synchronize()
    lib = _lib.load()
    buf = (ctypes.c_ulonglong * (4096 * 4 * 7))()
    assert lib.gca_debug_alex_stamps(buf) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4, 7).astype(np.int64)
    st = st[(st[:, :, 0] > 0).all(axis=1)]
    d = np.diff(st, axis=2)  # (samples, 4 waves, 6 phases)
    mean = d.mean(axis=(0, 1))
    life = st[:, :, 6].max(axis=1) - st[:, :, 0].min(axis=1)
    t0 = st[:, :, 0].min()
    out = {"samples": int(st.shape[0]), "mean_cycles_per_phase": {p: round(float(m), 1) for p, m in zip(PHASES, mean)},
           "phase_frac": {p: round(float(m / mean.sum()), 3) for p, m in zip(PHASES, mean)},
           "wave_life_cycles_mean": round(float(d.sum(axis=2).mean()), 1),
           "wg_life_cycles_mean": round(float(life.mean()), 1),
           "launch_span_cycles": int(st[:, :, 6].max() - t0),
           "wg_start_spread_cycles": int(st[:, :, 0].min(axis=1).max() - t0)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
