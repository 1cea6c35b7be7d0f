"""Multi-GPU: one process per GPU, envs sharded in contiguous blocks, RCCL all-gather of
the per-env done mask and episode statistics.

Envs are independent (no cross-env data in any operator), so a rank owns envs
[offset, offset + count) and runs the CA with no collective at all. Every Philox
counter carries the GLOBAL env id (env_offset + e), so a sharded run reproduces the
single-GPU trajectories env for env. The only exchange is what an RL learner needs
from every rank: done flags and episode returns / lengths (reference analogue: the
disabled jax.lax.all_gather of EpisodeStatistics, agents/jax_ppo.py:1325-1348).
Messages are ~9 KB per rank per env step: latency-bound, one all_gather per call.
"""
import torch
import torch.distributed as dist


def shard(num_envs, world_size, rank):
    """(offset, count) of this rank's contiguous env block; the remainder goes to the low ranks."""
    base, rem = divmod(int(num_envs), int(world_size))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def init_from_env(backend=None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun); returns (rank, world)."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend or ("nccl" if torch.cuda.is_available() else "gloo"), rank=rank,
                                world_size=world)
    return rank, world


class EpisodeStats:
    """Per-env running return / length on the device, all-gathered across ranks."""

    def __init__(self, num_envs, device, group=None):
        self.ret = torch.zeros(num_envs, dtype=torch.float32, device=device)
        self.len = torch.zeros(num_envs, dtype=torch.int32, device=device)
        self.group = group

    def update(self, reward, done):
        self.ret += reward.to(torch.float32)
        self.len += 1
        d = done.bool()
        finished_ret = torch.where(d, self.ret, torch.zeros_like(self.ret))
        finished_len = torch.where(d, self.len, torch.zeros_like(self.len))
        self.ret.masked_fill_(d, 0.0)
        self.len.masked_fill_(d, 0)
        return finished_ret, finished_len

    def gather(self, done, finished_ret, finished_len):
        """All ranks' (done u8[E], return f32[E], length i32[E]) concatenated in rank order."""
        return all_gather_stats(done, finished_ret, finished_len, self.group)


def all_gather_stats(done, ret, length, group=None):
    """One all_gather of a packed [ret f32 | len i32 | done u8] byte buffer (9 bytes per env; the 4-byte
    fields first so their views stay aligned for any env count)."""
    E = done.numel()
    payload = torch.cat([ret.reshape(-1).to(torch.float32).view(torch.uint8),
                         length.reshape(-1).to(torch.int32).view(torch.uint8), done.reshape(-1).to(torch.uint8)])
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        parts = [payload]
    else:
        parts = [torch.empty_like(payload) for _ in range(dist.get_world_size(group))]
        dist.all_gather(parts, payload, group=group)
    dones, rets, lens = [], [], []
    for part in parts:
        rets.append(part[:4 * E].view(torch.float32))
        lens.append(part[4 * E:8 * E].view(torch.int32))
        dones.append(part[8 * E:9 * E])
    return torch.cat(dones), torch.cat(rets), torch.cat(lens)
