"""The multi-GPU tile path with real HIP tiles: 2 rank processes on device 0 (RCCL refuses two ranks on
one GPU, so the gather runs over gloo here; bench.py uses the nccl backend = RCCL over xGMI across GPUs).

Each rank renders its 16-column blocks with jsrt_render_device (the bench's step), hands the tile to
FrameGather, and rank 0 composites.  The result must be bit-equal to a 1-rank render of the same
frame -- the reference's column split across workers (src/raytrace_launcher.js:65-101,
src/renderers.js:88) composited by the main thread (raytrace_launcher.js:92-97)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SPP, DEPTH = 256, 192, 8, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, cb, outdir):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import jsraytracer_amd as jr
    from jsraytracer_amd.tiles import FrameGather
    from oracle import pyoracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0)
    fg = FrameGather(W, H, rank, world, cb)  # host tiles: gloo gathers CPU tensors
    dev = torch.zeros(fg.maxcols * H, dtype=torch.int32, device="cuda:0")
    sc.render_device(dev.data_ptr(), col_block=cb, width=W, height=H, spp=SPP, max_depth=DEPTH, kind=1, seed=1,
                     x_offset=rank, x_delt=world, stats=False)
    torch.cuda.synchronize()
    fg.local.copy_(dev.cpu())
    img = fg.gather()
    if rank == 0:
        np.save(os.path.join(outdir, "composite.npy"), FrameGather.to_rgba8(img))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cb", [(2, 16), (3, 8)])
def test_gpu_rank_tiles_gather_to_single_rank_frame(tmp_path, world, cb):
    import jsraytracer_amd as jr
    from oracle import pyoracle
    mp.start_processes(_rank, args=(world, _free_port(), cb, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    comp = np.load(os.path.join(tmp_path, "composite.npy"))
    full, _, _ = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0).render(W, H, SPP, DEPTH, 1, 1,
                                                                                     want_colors=False)
    assert np.array_equal(comp, full)
    # and the composite's columns of every rank against the oracle (not only HIP against HIP)
    _, ref, _ = pyoracle.render(pyoracle.golden_scene("cornell_box_path"), W, H, SPP, DEPTH, 1, 1, 5, 41)
    cols = list(range(5, W, 41))
    assert len({(c // cb) % world for c in cols}) == world
    assert np.array_equal(comp.reshape(H, W, 4)[:, cols], ref[:, cols])


PSPP = 4  # progressive frame: passes 0..PSPP-2 call back, the last pass is the final frame


def _rank_progressive(rank, world, port, cb, outdir, W=W, H=H):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import jsraytracer_amd as jr
    from jsraytracer_amd.tiles import FrameGather, render_progressive
    from oracle import pyoracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0)
    fg = FrameGather(W, H, rank, world, cb)  # host tiles: gloo gathers CPU tensors
    dev = torch.zeros(fg.maxcols * H, dtype=torch.int32, device="cuda:0")

    def keep(p, img):
        np.save(os.path.join(outdir, f"pass{p}.npy"), FrameGather.to_rgba8(img))

    render_progressive(sc, fg, dev, keep, timelimit_ms=0.0, host_tiles=True, width=W, height=H, spp=PSPP,
                       max_depth=DEPTH, kind=1, seed=1, x_offset=rank, x_delt=world)
    fg.local.copy_(dev.cpu())
    img = fg.gather()
    if rank == 0:
        np.save(os.path.join(outdir, "final.npy"), FrameGather.to_rgba8(img))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cb,w", [(2, 16, W), (3, 8, W), (3, 16, 32)])
def test_gpu_progressive_previews_gather_to_running_mean(tmp_path, world, cb, w):
    """The multi-GPU tile path with progress (jsrt_render_device_progress + tiles.render_progressive): at
    every pass p the ranks' tiles hold the running mean of samples 0..p (renderers.js:93-112), rank 0
    gathers them, and the composite equals the single-rank frame of spp = p + 1 bit for bit (keyed RNG:
    sample k of a pixel does not depend on spp); the final gather equals the full frame.  (3, 16, 32): rank 2
    owns no column (jsrt_render_device_progress_ex still reports its passes, so its collectives keep step)."""
    import jsraytracer_amd as jr
    from oracle import pyoracle
    mp.start_processes(_rank_progressive, args=(world, _free_port(), cb, str(tmp_path), w, H), nprocs=world, join=True,
                       start_method="spawn")
    sc = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0)
    for p in range(PSPP - 1):
        got = np.load(os.path.join(tmp_path, f"pass{p}.npy"))
        ref, _, _ = sc.render(w, H, p + 1, DEPTH, 1, 1, want_colors=False)
        assert np.array_equal(got, ref), f"pass {p}: {int((got != ref).any(-1).sum())} pixels differ"
    full, _, _ = sc.render(w, H, PSPP, DEPTH, 1, 1, want_colors=False)
    assert np.array_equal(np.load(os.path.join(tmp_path, "final.npy")), full)


def _rank_accum(rank, world, port, cb, outdir):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import jsraytracer_amd as jr
    from jsraytracer_amd.tiles import AccumGather
    from oracle import pyoracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0)
    ag = AccumGather(W, H, rank, world, cb)  # host tiles: gloo gathers CPU tensors
    dev = torch.zeros(ag.maxcols * H * 4, dtype=torch.float32, device="cuda:0")
    sc.render_device_accum(dev.data_ptr(), col_block=cb, width=W, height=H, spp=SPP, max_depth=DEPTH, kind=1, seed=1,
                           x_offset=rank, x_delt=world, stats=False)
    torch.cuda.synchronize()
    ag.local.copy_(dev.cpu())
    acc = ag.gather()
    if rank == 0:
        np.save(os.path.join(outdir, "accum.npy"), acc.numpy())
        img = AccumGather.finish(acc.to("cuda:0"), 1, SPP)  # one k_final on rank 0
        torch.cuda.synchronize()
        np.save(os.path.join(outdir, "composite.npy"), img.cpu().numpy().view(np.uint8).reshape(H, W, 4))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cb", [(2, 16), (3, 8)])
def test_gpu_accum_tiles_gather_to_single_rank_frame(tmp_path, world, cb):
    """The accumulator exchange with real HIP tiles (jsrt_render_device_accum per rank, tiles.AccumGather, one
    jsrt_finish_accum on rank 0): the finished composite equals the 1-rank frame's RGBA8 bit for bit, and its
    accumulators equal the oracle's on an oracle-sized crop of the frame (src/renderers.js:93-98: the
    accumulator, then times(1 / passes) and setColor)."""
    import jsraytracer_amd as jr
    from oracle import pyoracle
    mp.start_processes(_rank_accum, args=(world, _free_port(), cb, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    full, _, _ = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0).render(W, H, SPP, DEPTH, 1, 1,
                                                                                     want_colors=False)
    assert np.array_equal(np.load(os.path.join(tmp_path, "composite.npy")), full)
    acc = np.load(os.path.join(tmp_path, "accum.npy"))
    _, _, _, ref = pyoracle.render(pyoracle.golden_scene("cornell_box_path"), W, H, SPP, DEPTH, 1, 1, 37, 64,
                                   accum=True)
    cols = list(range(37, W, 64))
    assert np.array_equal(acc[:, cols].view(np.uint32), ref[:, cols].view(np.uint32))


def _rank_nccl_one(_i, port, cb, outdir):
    """One rank of a one-rank nccl (RCCL) group: its tile is the whole frame, and both gathers run RCCL's gather
    on the device (the collective bench.py's N-GPU path runs over xGMI; one GPU is all this box has)."""
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import jsraytracer_amd as jr
    from jsraytracer_amd.tiles import AccumGather, FrameGather
    from oracle import pyoracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    sc = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0)
    fg = FrameGather(W, H, 0, 1, cb, device="cuda:0")
    sc.render_device(fg.local.data_ptr(), col_block=cb, width=W, height=H, spp=SPP, max_depth=DEPTH, kind=1, seed=1,
                     x_offset=0, x_delt=1, stats=False)
    torch.cuda.synchronize()
    img = fg.gather()
    ag = AccumGather(W, H, 0, 1, cb, device="cuda:0")
    sc.render_device_accum(ag.local.data_ptr(), col_block=cb, width=W, height=H, spp=SPP, max_depth=DEPTH, kind=1,
                           seed=1, x_offset=0, x_delt=1)
    torch.cuda.synchronize()
    fin = AccumGather.finish(ag.gather(), 1, SPP)
    torch.cuda.synchronize()
    np.save(os.path.join(outdir, "composite.npy"), FrameGather.to_rgba8(img))
    np.save(os.path.join(outdir, "composite_accum.npy"), FrameGather.to_rgba8(fin))
    dist.barrier()
    dist.destroy_process_group()


def test_gpu_nccl_one_rank_gather(tmp_path):
    """FrameGather / AccumGather through a real RCCL gather (nccl backend, one rank on device 0): the composite
    equals the one-rank render bit for bit."""
    import jsraytracer_amd as jr
    from oracle import pyoracle
    mp.start_processes(_rank_nccl_one, args=(_free_port(), 16, str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    full, _, _ = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0).render(W, H, SPP, DEPTH, 1, 1,
                                                                                     want_colors=False)
    assert np.array_equal(np.load(os.path.join(tmp_path, "composite.npy")), full)
    assert np.array_equal(np.load(os.path.join(tmp_path, "composite_accum.npy")), full)
