"""Replay a batched env step as one HIP graph (the env step on the device
without host round-trips).

A Windy bulldozer env step is ~5 short launches (pre, P CA passes, interpass, post) over E
envs; at E = 1024 most of its wall time is host-side launch overhead, not GPU work. Every
entry point of libgca_hip is capturable (no allocation, no synchronisation, explicit stream),
so the whole step — including device-side action sampling, which reads its counter from
device memory — is captured once and replayed with a single launch per `n_steps` steps.
Per-env state (RNG counters, accu, parity, positions) lives in device tensors that the graph
updates in place, so replays continue the trajectory exactly as eager calls would.
"""
import torch


class StepGraph:
    """Capture `fn()` (which must only launch work on the current stream) `n_steps` times.

        g = StepGraph(lambda: env.step(action), n_steps=8, device=dev)
        g.replay()          # = 8 eager calls of fn
    """

    def __init__(self, fn, n_steps=1, device=None, warmup=2):
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.n_steps = int(n_steps)
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):  # warm-up off the default stream (allocator pools, lazy init)
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream(self.device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for _ in range(self.n_steps):
                fn()

    def replay(self):
        self.graph.replay()
