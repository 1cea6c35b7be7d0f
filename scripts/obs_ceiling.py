"""Write-dominated ceilings for the RGB observation (4096 x 256^2 x 3 f32 = 3.2 GB written per frame), timed with
HIP events on one GPU: a write-only fill_, and torch's fused broadcast cast that reads the u8 grid (1 B/cell) and writes
its f32 RGB (12 B/cell) — the observation kernel's own read/write mix minus the dousing byte.
Prints one JSON line."""
import json

import torch


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


E, H, W = 4096, 256, 256
dev = torch.device("cuda:0")
rgb = torch.empty((E, H, W, 3), dtype=torch.float32, device=dev)
grid = torch.randint(0, 3, (E, H, W), dtype=torch.uint8, device=dev)
fill_ms = timed(lambda: rgb.fill_(1.0))
cast_ms = timed(lambda: rgb.copy_(grid.unsqueeze(-1).expand(E, H, W, 3)))
n = E * H * W
print(json.dumps({"fill_ms": fill_ms, "fill_gbs": 12 * n / fill_ms / 1e6, "cast_u8_to_rgb_ms": cast_ms,
                  "cast_gbs": 13 * n / cast_ms / 1e6}))
