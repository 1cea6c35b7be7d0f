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
import weakref
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
        self._gather = None  # built on the first gather: the process group may not exist yet

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
        """All ranks' (done u8, return f32, length i32), each (world, E) in rank order (views of a reused
        buffer, valid until the next gather on the same buffer)."""
        if self._gather is None:
            self._gather = StatsGather(self.ret.numel(), self.ret.device, group=self.group)
        return self._gather.gather(done, finished_ret, finished_len)


def _dist_world(group):
    """(world size, rank) of `group` as of now: (1, 0) without an initialised process group."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


class StatsGather:
    """The per-env episode-statistics all-gather, preallocated and reused: per call ONE pack (a single torch.cat
    of the three fields' bytes into a payload row) and ONE all_gather_into_tensor into a [world, row] byte buffer;
    no allocation, no host sync, so a step loop can run it eagerly, on a side stream (`async_op=True`,
    overlapping the next step) or capture it.

    Row layout (bytes): [ret f32 x E | length (4-byte dtype) x E | done u8 x E | pad to a multiple of 4]; the
    results are strided (world, E) views of the gathered buffer (the 4-byte fields stay aligned for any E).
    `buffers` payload / result pairs rotate so that an asynchronous gather never has its payload overwritten by
    the next pack (the pack waits for the gather that last used its buffer). With one rank the pack writes the
    result row directly: one launch, no collective.

    The world size is read from torch.distributed on every call (a gather built before init_process_group, or
    across a destroy / re-init, rebuilds its buffers instead of silently skipping the collective). `world` and
    `collective` override both for tests: `collective(out_flat, payload, group=...)` stands in for
    dist.all_gather_into_tensor (e.g. a device copy on one GPU, so the side-stream rotation runs on HIP streams
    without a second rank).
    """

    def __init__(self, num_envs, device, group=None, buffers=2, len_dtype=torch.int32, world=None, collective=None):
        self.E = int(num_envs)
        self.device = torch.device(device)
        # an explicit group is held weakly (torch keeps it alive until destroy_process_group): a cached gather must
        # not keep a destroyed group and its buffers alive (all_gather_stats)
        self._group = None if group is None else weakref.ref(group)
        self.buffers = int(buffers)
        self.len_dtype = len_dtype
        self._world_override = None if world is None else int(world)
        self._collective = collective if collective is not None else dist.all_gather_into_tensor
        self.pad = (-self.E) % 4
        self.row = 9 * self.E + self.pad
        self._zero_pad = torch.zeros(self.pad, dtype=torch.uint8, device=self.device)
        self.world = None
        self.stream = None
        self._build(*self._world_now())

    @property
    def group(self):
        if self._group is None:
            return None
        g = self._group()
        if g is None:
            raise RuntimeError("StatsGather: its process group has been destroyed")
        return g

    def _world_now(self):
        if self._world_override is not None:
            return self._world_override, 0
        return _dist_world(self.group)

    def _build(self, world, rank):
        if self.world is not None and self.device.type == "cuda":
            for ev in self._events:  # a rebuild must not free buffers a side-stream gather still reads
                if ev is not None:
                    torch.cuda.current_stream(self.device).wait_event(ev)
        self.world, self.rank = world, rank
        self.out = [torch.zeros((world, self.row), dtype=torch.uint8, device=self.device)
                    for _ in range(self.buffers)]
        # one rank: the pack writes the result row itself; several: a payload the collective reads
        self.payload = [o[0] if world == 1 else torch.zeros(self.row, dtype=torch.uint8, device=self.device)
                        for o in self.out]
        self._views = [self._make_views(o) for o in self.out]
        self._events = [None] * self.buffers
        self.k = 0
        if self.device.type == "cuda" and world > 1 and self.stream is None:
            self.stream = torch.cuda.Stream(self.device)

    def _make_views(self, o):
        E = self.E
        return (o[:, 8 * E:9 * E], o[:, :4 * E].view(torch.float32), o[:, 4 * E:8 * E].view(self.len_dtype))

    def gather(self, done, ret, length, async_op=False):
        """(done u8, ret f32, length) (world, E) views of this call's gathered buffer. async_op=True (CUDA, world >
        1): the collective runs on a side stream and the returned event must be waited on (event.wait() on the
        consuming stream) before the views are read: returns (done, ret, length, event)."""
        E = self.E
        if ret.dtype != torch.float32 or length.element_size() != 4 or done.element_size() != 1:
            raise ValueError("gather takes ret f32, a 4-byte length and a 1-byte done flag")
        if ret.numel() != E or length.numel() != E or done.numel() != E:
            raise ValueError(f"gather sized for {E} envs per rank")
        world, rank = self._world_now()
        if world != self.world or rank != self.rank:
            self._build(world, rank)
        if length.dtype != self.len_dtype:
            self.len_dtype = length.dtype
            self._views = [self._make_views(o) for o in self.out]
        k = self.k
        self.k = (k + 1) % len(self.out)
        on_cuda = self.device.type == "cuda"
        if on_cuda and self._events[k] is not None:  # the side stream's last gather of this buffer is done
            torch.cuda.current_stream(self.device).wait_event(self._events[k])
            self._events[k] = None
        parts = [ret.reshape(-1).view(torch.uint8), length.reshape(-1).view(torch.uint8),
                 done.reshape(-1).view(torch.uint8)]
        if self.pad:
            parts.append(self._zero_pad)
        torch.cat(parts, out=self.payload[k])  # the one pack
        event = None
        if self.world > 1:
            flat = self.out[k].view(-1)
            if async_op and self.stream is not None:
                self.stream.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(self.stream):
                    self._collective(flat, self.payload[k], group=self.group)
                    event = torch.cuda.Event()
                    event.record(self.stream)
                self._events[k] = event
            else:
                self._collective(flat, self.payload[k], group=self.group)
        d, r, ln = self._views[k]
        return (d, r, ln, event) if async_op else (d, r, ln)

    def verify(self):
        """Check the LAST gather against what every rank sent (VERDICT r05 missing 3): each rank hashes every row of
        its gathered buffer and its own payload (two int64 hashes: the byte sum and a position-weighted byte sum),
        the payload hashes are summed into a [world, 2] table over the group (each rank fills its own row), and each
        rank compares that table with the rows it received. Returns {"gather_ok", "rank_ok" [world],
        "world_seen", "rows_checked", "bytes_per_row"}: world_seen is an all_reduce of ones over the group (what the
        backend delivered, not the configured size). With one rank: None (nothing was exchanged)."""
        if self.world is None or self.world == 1 or not dist.is_initialized():
            return None
        k = (self.k - 1) % len(self.out)
        if self.device.type == "cuda" and self._events[k] is not None:
            torch.cuda.current_stream(self.device).wait_event(self._events[k])
        i64 = torch.int64
        wts = torch.arange(self.row, device=self.device, dtype=i64) % 65521 + 1
        got = self.out[k].to(i64)
        rows = torch.stack([got.sum(1), (got * wts).sum(1)], dim=1)        # (world, 2) as received here
        mine = self.payload[k].to(i64)
        sent = torch.zeros((self.world, 2), dtype=i64, device=self.device)
        sent[self.rank, 0], sent[self.rank, 1] = mine.sum(), (mine * wts).sum()
        dist.all_reduce(sent, group=self.group)                            # every rank's payload hashes
        ok_here = bool(torch.equal(rows, sent))
        flags = torch.zeros(self.world, dtype=i64, device=self.device)
        flags[self.rank] = int(ok_here)
        dist.all_reduce(flags, group=self.group)
        ones = torch.ones(1, dtype=i64, device=self.device)
        dist.all_reduce(ones, group=self.group)
        rank_ok = [bool(v) for v in flags.tolist()]
        return {"gather_ok": all(rank_ok), "rank_ok": rank_ok, "world_seen": int(ones.item()),
                "rows_checked": self.world, "bytes_per_row": self.row}


def verify_gather(stats):
    """StatsGather.verify() of `stats` (None for a missing gather or one rank): shared by bench.py's real N-rank path
    and its --dry-run rehearsal."""
    return None if stats is None else stats.verify()


# cached StatsGathers: the default group's by (E, device); an explicit group's in a dict held WEAKLY by the group
# object (keying a plain dict by the group kept every destroyed group and its [world, row] device buffers
# alive across init / destroy cycles)
_GATHERS = {}
_GROUP_GATHERS = weakref.WeakKeyDictionary()


def all_gather_stats(done, ret, length, group=None):
    """One all-gather of the per-env (done u8, return f32, length) of every rank: (world, E) tensors in rank order
    (9 bytes per env on the wire), through a StatsGather kept per (E, device, group) — the collective allocates
    nothing; the results are fresh clones (the hot path that wants the reused views calls StatsGather directly).
    The StatsGather re-reads the world size on every call, so a cached one follows a re-initialised group."""
    cache = _GATHERS if group is None else _GROUP_GATHERS.setdefault(group, {})
    key = (done.numel(), str(done.device))
    g = cache.get(key)
    if g is None:
        g = cache[key] = StatsGather(done.numel(), done.device, group=group, len_dtype=length.dtype)
    return tuple(x.clone() for x in g.gather(done, ret, length))
