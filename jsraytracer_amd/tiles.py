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


def _group_matches(world):
    """True when this gatherer runs a collective: a process group is initialised.  Its size must be the
    gatherer's world (a one-rank group still runs the collective, as the RCCL one-rank test does); a gatherer
    built for another world size would gather over the whole default group with the wrong number of slots
    and hang or fail, so that is refused here instead (advisor, round 5)."""
    import torch.distributed as dist
    if not dist.is_initialized():
        if world > 1:
            raise RuntimeError(f"gather over {world} ranks needs an initialised process group")
        return False
    if dist.get_world_size() != world:
        raise RuntimeError(f"gatherer built for {world} ranks in a process group of {dist.get_world_size()}")
    return True


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

    def _collective(self):
        return _group_matches(self.world)

    def gather(self):
        """Collective: every rank calls it after its tile is rendered into self.local.  Returns the
        [H, W] int32 (packed RGBA8) image on rank 0, None elsewhere."""
        import torch
        import torch.distributed as dist
        if self._collective():
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


class AccumGather:
    """The accumulator exchange: gathers per-rank f32 accumulator tiles ([max_owned * H] pixels x 4 f32, as
    jsrt_render_device_accum writes them) to rank 0 and permutes them into image order ([H * W] pixels x 4), so
    rank 0 holds the frame's accumulators -- the f32 state the reference's workers sum their samples into
    (src/renderers.js:93-97) -- and finishes them with one k_final (jsrt_finish_accum: setColor's RGBA8).
    Pixels never split across ranks, so the composite accumulators, and the RGBA8 finished from them, are the
    single-GPU frame's bit for bit.  Four times the RGBA8 exchange's bytes (16 B per pixel), for a caller that
    combines or re-normalises passes on rank 0.  One collective per frame, like FrameGather."""

    def __init__(self, width, height, rank, world, col_block=1, device="cpu"):
        import torch
        self.W, self.H, self.rank, self.world, self.cb = width, height, rank, world, col_block
        self.ncols = len(owned_px(width, rank, world, col_block))
        self.maxcols = max_owned(width, world, col_block)
        self.local = torch.zeros(self.maxcols * height * 4, dtype=torch.float32, device=device)
        self.parts = [torch.empty_like(self.local) for _ in range(world)] if rank == 0 else None
        self.slot = torch.as_tensor(column_permutation(width, world, col_block), device=device) if rank == 0 else None
        self.image = torch.empty((height, width, 4), dtype=torch.float32, device=device) if rank == 0 else None

    def _collective(self):
        return _group_matches(self.world)

    def gather(self):
        """Collective: every rank calls it after its accumulator tile is in self.local.  Returns the [H, W, 4] f32
        accumulators on rank 0 (image order), None elsewhere."""
        import torch
        import torch.distributed as dist
        if self._collective():
            dist.gather(self.local, self.parts if self.rank == 0 else None, dst=0)
        else:
            self.parts = [self.local]
        if self.rank != 0:
            return None
        allc = torch.stack(self.parts).view(self.world * self.maxcols, self.H, 4)  # [slot][row][4]
        self.image.copy_(allc.index_select(0, self.slot).permute(1, 0, 2))
        return self.image

    @staticmethod
    def finish(image, kind, passes):
        """rank 0: the RGBA8 frame [H, W] int32 (packed) of gathered accumulators [H, W, 4] on a GPU
        (jsrt_finish_accum, on torch's current stream of that device)."""
        import torch

        from .renderer import finish_accum
        acc = image.contiguous()
        out = torch.empty(acc.shape[0] * acc.shape[1], dtype=torch.int32, device=acc.device)
        finish_accum(acc.data_ptr(), out.numel(), kind, passes, out.data_ptr(), None,
                     torch.cuda.current_stream(acc.device).cuda_stream)
        return out.view(acc.shape[0], acc.shape[1])


def render_progressive(scene, fg, dev_tile, on_preview, timelimit_ms=0.0, host_tiles=False, **kw):
    """Progressive multi-rank render of one frame: the reference's workers post their partial image at every
    `timelimit` tick (src/worker.js:30-32, src/renderers.js:103-112) and the main thread overlays them
    (src/raytrace_launcher.js:92-97).  Every rank renders its tile with jsrt_render_device_progress, one
    sample per pixel per pass, so its device tile holds the running mean of passes 0..p at each callback.
    Rank 0's clock decides whether a preview is due (one all-reduce per pass keeps the ranks' collectives in
    step); when it is, the ranks' tiles are gathered (FrameGather, RCCL over xGMI or gloo) and rank 0 gets
    on_preview(pass, image [H, W] int32 RGBA8).  The frame's final tile is left in dev_tile.

    kw: jsrt_render_device parameters (width, height, spp, max_depth, kind, seed, x_offset, x_delt).

    Every rank calls back for the same passes (jsrt_render_device_progress_ex reports each pass, clean or not,
    and a rank that owns no column reports them too), and each callback runs ONE all-reduce of the ranks'
    status {a batch poisoned (that tile is not the pass's running mean), a failure, a preview due by rank 0's
    clock, a rank done}: a preview is gathered only when every tile is clean, and a failure on any rank stops
    every rank's frame together (the failing rank re-raises, the others raise JsrtError).  A rank leaves with
    one closing all-reduce (done = 1) unless a progress all-reduce already met a done peer's closing one: every
    all-reduce of one rank is matched by exactly one of every other rank, so none is left waiting."""
    import time

    import torch
    import torch.distributed as dist
    if kw.get("kind", 1) != 1:
        # the running-mean previews are the Incremental renderer's (renderers.js:70-117); Simple / Random report
        # per batch, and a rank that owns no column has no batches to report, so the ranks' per-callback
        # collectives could not stay in step (advisor, round 5)
        raise ValueError("render_progressive renders the Incremental kind (kind=1) only")
    last = [time.perf_counter()]
    dev = "cpu" if host_tiles or fg.world == 1 else dev_tile.device
    status = torch.zeros(4, dtype=torch.int32, device=dev)  # unclean, failed, due, done: max over ranks
    failed, closed, peer_failed = [], [False], [False]

    def exchange(unclean, due, done):
        status.copy_(torch.tensor([unclean, 1 if failed else 0, due, done], dtype=torch.int32))
        if fg.world > 1:
            dist.all_reduce(status, op=dist.ReduceOp.MAX)
        return [int(x) for x in status.tolist()]

    def cb(p, _completion, clean):
        due = 0
        if fg.rank == 0:
            due = 1 if (time.perf_counter() - last[0]) * 1e3 >= timelimit_ms else 0
        unclean, fail, due_all, done = exchange(0 if clean else 1, due, 0)
        if done:  # a peer has left its render (it failed): this all-reduce was its closing one
            closed[0] = True
            peer_failed[0] = True
            return True
        if fail:
            peer_failed[0] = True
            return True  # abort this rank's frame (every rank sees the same status)
        if unclean or not due_all:
            return False
        if fg.rank == 0:
            last[0] = time.perf_counter()
        try:
            fg.local.copy_(dev_tile.view(-1)[:fg.local.numel()].to(fg.local.device))
            img = fg.gather()
            if fg.rank == 0:
                on_preview(p, img)
        except Exception as e:  # noqa: BLE001 -- reported to the peers at the next exchange, re-raised below
            failed.append(e)
        return False

    # every pass calls back on every rank (a 1e-9 ms library cadence); the preview cadence is rank 0's
    try:
        scene.render_device(dev_tile.data_ptr(), progress_ex=cb, timelimit_ms=1e-9, samples_per_launch=1, stats=False,
                            col_block=fg.cb, **kw)
    except Exception as e:  # noqa: BLE001 -- this rank's render failed: its peers learn it below
        failed.append(e)
    if not closed[0] and exchange(0, 0, 1)[1]:  # the closing exchange: a failure in the last pass reaches all
        peer_failed[0] = True
    if failed:
        raise failed[0]
    if peer_failed[0]:
        from ._native import JsrtError
        raise JsrtError("render_progressive: another rank's render or progress callback failed; frame aborted")
