"""GPU: the episode-statistics gather's side-stream branch (gymca_amd/distributed.py StatsGather, async_op=True) on
real HIP streams, single process. The collective is replaced through StatsGather's test seam (`world=2`,
`collective=`) by a slow device copy on the side stream, so the stream / event rotation that bench.py runs at N > 1
(reference analogue: the episode-statistics all_gather, agents/jax_ppo.py:1325-1348) executes here with the env's
post_step writing the next payload while the previous gather is still in flight."""
import pytest
import torch

from gymca_amd.distributed import StatsGather

pytestmark = pytest.mark.gpu


def _spin(ms):
    """Keep the current stream busy for about `ms` milliseconds."""
    try:
        torch.cuda._sleep(int(ms * 2.0e6))  # clock cycles (~2 GHz)
    except (AttributeError, RuntimeError):
        a = torch.randn(1024, 1024, device="cuda")
        for _ in range(int(ms * 4)):
            a = a @ a * 1e-3


@pytest.mark.parametrize("buffers", [2, 3])
def test_stats_gather_async_rotation_on_hip_streams(buffers):
    from gymca_amd.forest_fire.bulldozer import AdvancedForestFireBulldozerEnv

    device = torch.device("cuda", 0)
    E, world, calls = 64, 2, 7
    env = AdvancedForestFireBulldozerEnv(256, 256, key=9, num_envs=E, use_hidden=False, device=device,
                                         observation="grid")
    env.reset()
    delivered = {}  # call index -> what the gather delivered (snapshot taken on the side stream, after the copy)
    n = [0]

    def slow_collective(out_flat, payload, group=None):
        assert torch.cuda.current_stream(device) == g.stream  # the collective is issued on the side stream
        _spin(3.0)  # the gather is still in flight while the next env steps and packs are issued
        out = out_flat.view(world, -1)
        for r in range(world):  # rank r's row: this rank's payload, byte-reversed for r = 1 (rows are told apart)
            out[r].copy_(payload if r == 0 else payload.flip(0))
        delivered[n[0]] = out.clone()
        n[0] += 1

    g = StatsGather(E, device, world=world, collective=slow_collective, buffers=buffers,
                    len_dtype=env.steps_elapsed.dtype)
    assert g.stream is not None and g.world == world
    action = torch.zeros((E, 2), dtype=torch.int32, device=device)
    expected, events = [], []
    for i in range(calls):
        action[:, 0] = i % 9
        action[:, 1] = i % 2
        env.ca_step()
        env.post_step(action, stats=True)  # writes done / reward_accumulated / steps_elapsed: the next payload
        expected.append((env.done.clone(), env.reward_accumulated.clone(), env.steps_elapsed.clone()))
        d, r, ln, ev = g.gather(env.done, env.reward_accumulated, env.steps_elapsed, async_op=True)
        assert ev is not None and d.shape == (world, E)
        events.append(ev)
    torch.cuda.synchronize(device)
    assert n[0] == calls and all(ev.query() for ev in events)
    for i, (d, r, ln) in enumerate(expected):
        out = delivered[i]
        row = torch.cat([r.view(torch.uint8), ln.view(torch.uint8), d.view(torch.uint8),
                         torch.zeros(g.pad, dtype=torch.uint8, device=device)])
        # no payload was overwritten by a later pack before its gather read it
        assert torch.equal(out[0], row), f"call {i}: rank-0 row differs from the payload packed at that call"
        assert torch.equal(out[1], row.flip(0))
    # the views of the last call alias its buffer and hold its values once its event has completed
    d, r, ln = g._views[(calls - 1) % buffers]
    assert torch.equal(d[0], expected[-1][0]) and torch.equal(r[0], expected[-1][1])
    assert torch.equal(ln[0], expected[-1][2])


def test_stats_gather_eager_branch_matches_async():
    """The inline (eager) branch of the same seam gives the same rows as the side-stream branch."""
    device = torch.device("cuda", 0)
    E = 37  # not a multiple of 4: the padded row
    rows = {}

    def copy_collective(out_flat, payload, group=None):
        out_flat.view(2, -1).copy_(payload.expand(2, -1))

    for mode in (False, True):
        g = StatsGather(E, device, world=2, collective=copy_collective)
        done = (torch.arange(E, device=device) % 3 == 0).to(torch.uint8)
        ret = -torch.arange(E, device=device, dtype=torch.float32) / 7
        ln = torch.arange(E, device=device, dtype=torch.int32)
        res = g.gather(done, ret, ln, async_op=mode)
        if mode:
            torch.cuda.current_stream(device).wait_event(res[3])
        rows[mode] = tuple(x.clone() for x in res[:3])
        assert torch.equal(rows[mode][0][1], done) and torch.equal(rows[mode][1][1], ret)
        assert torch.equal(rows[mode][2][1], ln)
    for a, b in zip(rows[False], rows[True]):
        assert torch.equal(a, b)
