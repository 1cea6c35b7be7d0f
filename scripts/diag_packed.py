"""Diagnostic: run the packed Alexandridis step on fixed random cases with the library selected by GCA_LIB_PATH and
save the outputs (python scripts/diag_packed.py out.npz); compare two libraries with --compare a.npz b.npz."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gym-cellular-automata_amd"))

SHAPES = [(2, 256, 256, 31), (1, 48, 512, 32), (1, 32, 1024, 33), (1, 32, 256, 35), (1, 16, 1024, 36),
          (1, 64, 768, 37)]


def run(out):
    import torch
    from test_gpu_edge_slope import altitude, make_case, packed_step, params, slopes
    dev = torch.device("cuda:0")
    res = {}
    for E, H, W, seed in SHAPES:
        case = make_case(E, H, W, seed, p_tree=0.01, dousing_p=0.2)
        p = params(H, 0.01, seed=seed * 7)
        es, _ = slopes(dev, altitude(E, H, W, seed))
        g1, a1, c1, _, _ = packed_step(dev, p, case, es, np.full(E, 1, np.uint32))
        res[f"g_{H}_{W}"] = g1
        res[f"a_{H}_{W}"] = a1
    np.savez(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    for k in A.files:
        d = A[k] != B[k]
        if d.any():
            idx = np.argwhere(d)
            rows = np.unique(idx[:, 1])
            cols = np.unique(idx[:, 2])
            print(k, "mismatch", int(d.sum()), "of", d.size, "rows", rows[:40].tolist(), "cols%256", np.unique(cols % 256)[:40].tolist(),
                  "tiles_c", np.unique(cols // 256).tolist())
        else:
            print(k, "equal")


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
