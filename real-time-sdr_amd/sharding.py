"""Channel sharding across GPUs (one process per GPU) and the per-block-step gather.

SURVEY 8(e): channels are independent, so the path partitions by channel with no exchange during
the DSP. Each rank owns a contiguous channel range (weak scaling: a fixed number of channels per
GPU); the only collective is the gather of each block-step's stereo int16 audio and RDS bits to
rank 0 (RCCL over xGMI on the GPU, gloo in the CPU tests), where rank r's rows are the r-th part of
the gathered list, i.e. global channels [r*nch, (r+1)*nch).
"""
from __future__ import annotations


def channel_range(channels_per_rank: int, rank: int) -> tuple[int, int]:
    """[first, first+count) global channel ids owned by `rank` (contiguous blocks)."""
    if channels_per_rank <= 0 or rank < 0:
        raise ValueError("channels_per_rank must be > 0 and rank >= 0")
    return rank * channels_per_rank, channels_per_rank


class BlockGather:
    """Gather each rank's [nch][...] outputs of one block-step to rank `dst`.

    Rows travel as raw bytes (uint8 views): RCCL has no int16 type and gloo lacks several, so one
    byte-typed collective per output serves every dtype on both backends. A gather, not an
    all-gather: only the receiving rank pays the (world-1) x nch rows of receive traffic."""

    def __init__(self, torch, dist, world: int, shapes: dict, device, dst: int = 0):
        self.torch, self.dist, self.world, self.dst = torch, dist, world, dst
        self.rank = dist.get_rank()
        self.shapes = {k: (tuple(s), dt) for k, (s, dt) in shapes.items()}
        # gloo moves host tensors only: device rows are staged through host memory (a blocking copy
        # on the current stream; the GPU rank path uses RCCL, where rows stay on the device)
        self.host_staged = dist.get_backend() == "gloo" and torch.device(device).type != "cpu"
        buf_dev = "cpu" if self.host_staged else device
        self.out = {}
        self.row_bytes = {}
        for k, (s, dt) in self.shapes.items():
            rb = torch.empty((1,) + s[1:], dtype=dt).element_size()
            for d in s[1:]:
                rb *= d
            self.row_bytes[k] = rb
            if self.rank == dst:
                self.out[k] = [torch.empty((s[0], rb), dtype=torch.uint8, device=buf_dev) for _ in range(world)]
        self.steps = 0

    def gather(self, **tensors) -> dict | None:
        """Returns {name: [world tensors of the original shape and dtype]} on dst, None elsewhere."""
        res = {}
        for k, t in tensors.items():
            shape, dt = self.shapes[k]
            if tuple(t.shape) != shape or t.dtype != dt:
                raise ValueError(f"{k}: expected {shape} {dt}, got {tuple(t.shape)} {t.dtype}")
            src = t.contiguous().view(shape[0], -1).view(self.torch.uint8)
            if self.host_staged:
                src = src.cpu()
            parts = self.out.get(k) if self.rank == self.dst else None
            self.dist.gather(src, parts, dst=self.dst)
            if parts is not None:
                res[k] = [p.view(dt).view(shape) for p in parts]
        self.steps += 1
        return res if self.rank == self.dst else None

    def check_last(self, world: int) -> dict:
        """Summary of the gather on the receiving rank (bytes per block-step, ranks, steps)."""
        per_step = sum(self.shapes[k][0][0] * self.row_bytes[k] for k in self.shapes) * world
        return {"dst_rank": self.dst, "ranks": world, "bytes_per_step": per_step, "steps": self.steps,
                "outputs": sorted(self.shapes)}


def max_over_ranks(torch, dist, seconds: float, device) -> float:
    """The job's time is the slowest rank's (bench contract: max over ranks)."""
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
