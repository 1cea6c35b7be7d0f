"""Run by tests/test_gpu_rccl.py in a child process on the GPU box: a one-rank RCCL ("nccl") process group on cuda:0
— the communicator bootstrap, all_gather_into_tensor and all_reduce through RCCL — and StatsGather's side-stream
branch with the real RCCL collective inside its seam (rank 0's row gathered by RCCL, the second row a device copy),
rotating under env.post_step as bench.py does at N > 1 (reference analogue: agents/jax_ppo.py:1325-1348).
Prints one JSON line; exit code 0 when every check holds."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cellular-automata_amd")]


def main():
    import torch
    import torch.distributed as dist

    from gymca_amd.distributed import StatsGather
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=device)
    res = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    checks = {}
    x = torch.arange(1000, dtype=torch.int32, device=device)
    out = torch.full((1000,), -1, dtype=torch.int32, device=device)
    dist.all_gather_into_tensor(out, x)
    y = torch.arange(37, dtype=torch.float32, device=device)
    dist.all_reduce(y)
    torch.cuda.synchronize(device)
    checks["all_gather_into_tensor"] = bool(torch.equal(out, x))
    checks["all_reduce"] = bool(torch.equal(y, torch.arange(37, dtype=torch.float32, device=device)))

    E, world, calls = 64, 2, 6
    env = AdvancedForestFireBulldozerEnv(256, 256, key=11, num_envs=E, use_hidden=False, device=device,
                                         observation="grid")
    env.reset()
    delivered = []

    def rccl_pair(out_flat, payload, group=None):  # row 0 through RCCL, row 1 a reversed device copy
        rows = out_flat.view(world, -1)
        dist.all_gather_into_tensor(rows[0], payload, group=group)
        rows[1].copy_(payload.flip(0))
        delivered.append(rows.clone())

    g = StatsGather(E, device, world=world, collective=rccl_pair, buffers=2, len_dtype=env.steps_elapsed.dtype)
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)
    expected = []
    for i in range(calls):
        action[:, 0] = i % 9
        action[:, 1] = i % 2
        env.ca_step()
        env.post_step(action, stats=True)
        expected.append(torch.cat([env.reward_accumulated.view(torch.uint8), env.steps_elapsed.view(torch.uint8),
                                   env.done.view(torch.uint8), torch.zeros(g.pad, dtype=torch.uint8, device=device)]))
        g.gather(env.done, env.reward_accumulated, env.steps_elapsed, async_op=True)
    torch.cuda.synchronize(device)
    checks["side_stream_rotation"] = len(delivered) == calls and all(
        torch.equal(d[0], e) and torch.equal(d[1], e.flip(0)) for d, e in zip(delivered, expected))
    # the real one-rank gather (no seam): the pack writes the result row itself, no collective
    g1 = StatsGather(E, device)
    d1, r1, l1 = g1.gather(env.done, env.reward_accumulated, env.steps_elapsed)
    checks["one_rank_gather"] = (g1.world == 1 and torch.equal(d1[0], env.done) and torch.equal(r1[0],
                                 env.reward_accumulated) and torch.equal(l1[0], env.steps_elapsed))
    dist.destroy_process_group()
    res["checks"] = checks
    res["ok"] = all(checks.values())
    print(json.dumps(res), flush=True)
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
