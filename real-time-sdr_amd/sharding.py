"""Channel sharding across GPUs (one process per GPU) and the per-block-step gather.

SURVEY 8(e): channels are independent, so the path partitions by channel with no exchange during
the DSP. Each rank owns a contiguous channel range (weak scaling: a fixed number of channels per
GPU); the only collective is the gather of each block-step's stereo int16 audio and RDS bits to
every rank (RCCL over xGMI on the GPU, gloo in the CPU tests), after which rank r's rows sit at
[r*nch, (r+1)*nch) of the gathered tensors.
"""
from __future__ import annotations


def channel_range(channels_per_rank: int, rank: int) -> tuple[int, int]:
    """[first, first+count) global channel ids owned by `rank` (contiguous blocks)."""
    if channels_per_rank <= 0 or rank < 0:
        raise ValueError("channels_per_rank must be > 0 and rank >= 0")
    return rank * channels_per_rank, channels_per_rank


class BlockGather:
    """Gather [nch][...] per-rank outputs of one block-step into [world*nch][...] on every rank.

    Rows travel as raw bytes (uint8 views): RCCL has no int16 type and gloo lacks several, so one
    byte-typed collective per output serves every dtype on both backends."""

    def __init__(self, torch, dist, world: int, shapes: dict, device):
        self.torch, self.dist, self.world = torch, dist, world
        self.shapes = {k: (tuple(s), dt) for k, (s, dt) in shapes.items()}
        self.out = {}
        for k, (s, dt) in self.shapes.items():
            row_bytes = torch.empty((1,) + s[1:], dtype=dt).element_size()
            for d in s[1:]:
                row_bytes *= d
            self.out[k] = torch.empty((world * s[0], row_bytes), dtype=torch.uint8, device=device)
        self._flat = dist.get_backend() != "gloo"

    def gather(self, **tensors) -> dict:
        res = {}
        for k, t in tensors.items():
            shape, dt = self.shapes[k]
            if tuple(t.shape) != shape or t.dtype != dt:
                raise ValueError(f"{k}: expected {shape} {dt}, got {tuple(t.shape)} {t.dtype}")
            src = t.contiguous().view(shape[0], -1).view(self.torch.uint8)
            dst = self.out[k]
            if self._flat:
                self.dist.all_gather_into_tensor(dst, src)
            else:
                parts = [self.torch.empty_like(src) for _ in range(self.world)]
                self.dist.all_gather(parts, src)
                self.torch.cat(parts, 0, out=dst)
            res[k] = dst.view(dt).view((self.world * shape[0],) + shape[1:])
        return res


def max_over_ranks(torch, dist, seconds: float, device) -> float:
    """The job's time is the slowest rank's (bench contract: max over ranks)."""
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
