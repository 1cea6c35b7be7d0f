"""A/B of the forced Windy CA step alone (bench.py windy_ca_only: every env steps once, dense state) for one library
build (GCA_LIB_PATH), 1024 x 256^2 and 1024 x 512^2, beside a device copy of the same bytes. One JSON line (us per
launch). Run on the GPU box."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def main():
    import torch

    import bench
    from gymca_amd.forest_fire.bulldozer import BatchedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    out = {}
    for N in (256, 512):
        env = BatchedForestFireBulldozerEnv(1024, N, N, device=device, seed=0x5EED, materialize_obs=False)
        r = bench.windy_ca_only(env, 40, 5, None, device)
        out[f"n{N}_ca_us"] = round(r["kernel_s"] * 1e6, 2)
        out[f"n{N}_copy_us"] = round(r["copy_s"] * 1e6, 2)
        del env
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
