"""Multi-GPU tile sharding of one frame: column blocks dealt round-robin to ranks, gathered to rank 0.

The reference parallelises only over image columns: worker i of N renders px = i, i + N, ...
(src/renderers.js:21,88; src/worker.js:30) and the main thread overlays the workers' frames
(src/raytrace_launcher.js:92-97).  Here rank r of N renders the columns of blocks b with
b % N == r (blocks of `col_block` columns; col_block = 1 is exactly the reference's interleave), into
a device buffer laid out as [owned column][row] u32 RGBA8 (include/jsrt.h jsrt_render_device).
Pixels never split across ranks, so every pixel's samples are accumulated in the reference's order
on one GPU and the composite is bit-identical to a single-GPU render (keyed RNG: partition
invariant).  The only exchange is one gather of the per-rank tiles to rank 0 (RCCL over xGMI with
the nccl backend; gloo in the CPU tests), then a permute into image order.
"""
import numpy as np


def owned_px(width, rank, world, col_block=1):
    """Image columns owned by `rank`, in owned-column order (jsrt.h owned_to_px)."""
    px = np.arange(width)
    if col_block <= 1:
        return px[(px >= rank) & ((px - rank) % world == 0)]
    return px[(px // col_block) % world == rank]


def max_owned(width, world, col_block=1):
    return max(len(owned_px(width, r, world, col_block)) for r in range(world))


def column_permutation(width, world, col_block=1):
    """For the gathered [rank][max_owned] column slots: the slot holding each image column."""
    m = max_owned(width, world, col_block)
    slot = np.empty(width, np.int64)
    for r in range(world):
        cols = owned_px(width, r, world, col_block)
        slot[cols] = r * m + np.arange(len(cols))
    return slot


class FrameGather:
    """Gathers per-rank [max_owned * H] u32 tiles to rank 0 and permutes them into an [H, W] image.

    One collective per frame (torch.distributed.gather: RCCL gather over xGMI under the nccl
    backend).  Works on any device the tensors live on, so the same code runs under gloo on CPU."""

    def __init__(self, width, height, rank, world, col_block=1, device="cpu"):
        import torch
        self.W, self.H, self.rank, self.world, self.cb = width, height, rank, world, col_block
        self.ncols = len(owned_px(width, rank, world, col_block))
        self.maxcols = max_owned(width, world, col_block)
        self.local = torch.zeros(self.maxcols * height, dtype=torch.int32, device=device)
        self.parts = [torch.empty_like(self.local) for _ in range(world)] if rank == 0 else None
        self.slot = torch.as_tensor(column_permutation(width, world, col_block), device=device) if rank == 0 else None
        self.image = torch.empty((height, width), dtype=torch.int32, device=device) if rank == 0 else None

    def gather(self):
        """Collective: every rank calls it after its tile is rendered into self.local.  Returns the
        [H, W] int32 (packed RGBA8) image on rank 0, None elsewhere."""
        import torch
        import torch.distributed as dist
        if self.world > 1:
            dist.gather(self.local, self.parts if self.rank == 0 else None, dst=0)
        else:
            self.parts = [self.local]
        if self.rank != 0:
            return None
        allc = torch.stack(self.parts).view(self.world * self.maxcols, self.H)  # [slot][row]
        self.image.copy_(allc.index_select(0, self.slot).t())
        return self.image

    @staticmethod
    def to_rgba8(image):
        """[H, W] int32 packed RGBA8 (little-endian R first) -> [H, W, 4] uint8 numpy."""
        return image.cpu().numpy().view(np.uint8).reshape(image.shape[0], image.shape[1], 4)
