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


def render_progressive(scene, fg, dev_tile, on_preview, timelimit_ms=0.0, host_tiles=False, **kw):
    """Progressive multi-rank render of one frame: the reference's workers post their partial image at every
    `timelimit` tick (src/worker.js:30-32, src/renderers.js:103-112) and the main thread overlays them
    (src/raytrace_launcher.js:92-97).  Every rank renders its tile with jsrt_render_device_progress, one
    sample per pixel per pass, so its device tile holds the running mean of passes 0..p at each callback.
    Rank 0's clock decides whether a preview is due (one broadcast per pass keeps the ranks' collectives in
    step); when it is, the ranks' tiles are gathered (FrameGather, RCCL over xGMI or gloo) and rank 0 gets
    on_preview(pass, image [H, W] int32 RGBA8).  The frame's final tile is left in dev_tile.

    kw: jsrt_render_device parameters (width, height, spp, max_depth, kind, seed, x_offset, x_delt)."""
    import time

    import torch
    import torch.distributed as dist
    last = [time.perf_counter()]
    flag = torch.zeros(1, dtype=torch.int32, device="cpu" if host_tiles or fg.world == 1 else dev_tile.device)

    def cb(p, _completion):
        if fg.rank == 0:
            now = time.perf_counter()
            due = (now - last[0]) * 1e3 >= timelimit_ms
            if due:
                last[0] = now
            flag.fill_(1 if due else 0)
        if fg.world > 1:
            dist.broadcast(flag, src=0)
        if not int(flag.item()):
            return
        fg.local.copy_(dev_tile.view(-1)[:fg.local.numel()].to(fg.local.device))
        img = fg.gather()
        if fg.rank == 0:
            on_preview(p, img)

    # every pass calls back on every rank (a 1e-9 ms library cadence); the preview cadence is rank 0's
    scene.render_device(dev_tile.data_ptr(), progress=cb, timelimit_ms=1e-9, samples_per_launch=1, stats=False,
                        col_block=fg.cb, **kw)
