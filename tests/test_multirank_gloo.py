"""N>1 path on CPU: world_size 2 and 3 gloo process groups running the bench's tile sharding
(jsraytracer_amd/tiles.py) — column blocks per rank, one gather to rank 0, permute to image order.

Each rank's tile is the oracle's render of exactly its owned columns (the oracle is the checker; on
the GPU the tile comes from jsrt_render_device, whose block layout test_gpu_parity.py checks), so the
composite must equal the single-process frame bit for bit, which in turn equals the reference's own
x_delt=3 worker images (tests/golden, src/renderers.js:88)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, cb, tag, outdir):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from jsraytracer_amd.tiles import FrameGather, owned_px
    from oracle import pyoracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = pyoracle.golden_index()[tag]
    blob = pyoracle.golden_scene(r["scene"])
    # this rank's columns, rendered column by column in the reference's x_offset/x_delt form
    # (a block of `cb` columns = cb interleave workers of stride W, one per column)
    cols = owned_px(W, rank, world, cb)
    fg = FrameGather(W, H, rank, world, cb)
    tile = np.zeros((fg.maxcols, H), np.uint32)
    for c, px in enumerate(cols):
        _, rgba, _ = pyoracle.render(blob, W, H, r["spp"], r["depth"], r["kind"], r["seed"], int(px), W, threads=1)
        tile[c] = rgba[:, px].view(np.uint32).reshape(H)
    fg.local.copy_(torch.from_numpy(tile.view(np.int32).reshape(-1)))
    img = fg.gather()
    if rank == 0:
        np.save(os.path.join(outdir, "composite.npy"), FrameGather.to_rgba8(img))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cb", [(2, 8), (3, 4), (3, 1)])
def test_gloo_tile_gather_matches_reference(tmp_path, world, cb):
    from oracle import pyoracle
    tag = "cornell_box_path_incremental_32x32_s2_d8_seed5"
    W = H = 32
    mp.start_processes(_worker, args=(world, _free_port(), W, H, cb, tag, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    got = np.load(tmp_path / "composite.npy")
    _, grgba = pyoracle.golden_image(tag, W, H)
    assert np.array_equal(got, grgba)


def test_owned_columns_cover_the_frame_once():
    from jsraytracer_amd import owned_columns
    from jsraytracer_amd.tiles import column_permutation, max_owned, owned_px
    for W in (1, 7, 32, 1000, 1024):
        for world in (1, 2, 3, 8):
            for cb in (1, 4, 16):
                allc = np.concatenate([owned_px(W, r, world, cb) for r in range(world)])
                assert sorted(allc.tolist()) == list(range(W))
                for r in range(world):
                    assert len(owned_px(W, r, world, cb)) == owned_columns(W, r, world, cb)
                slot = column_permutation(W, world, cb)
                assert len(set(slot.tolist())) == W and slot.max() < world * max_owned(W, world, cb)


class _OracleTileScene:
    """Stands in for jr.Scene on the CPU: render_device fills `tile` pass by pass with the oracle's running
    mean of the rank's owned columns (the oracle's spp = p + 1 render, which the keyed RNG makes the
    Incremental renderer's image after pass p) and calls progress after every pass but the last, as
    jsrt_render_device_progress does."""

    def __init__(self, blob, tile, W, H, cols, fail_at=None, unclean_at=None):
        self.blob, self.tile, self.W, self.H, self.cols = blob, tile, W, H, cols
        self.fail_at, self.unclean_at = fail_at, unclean_at  # (test hooks: a failing / poisoned pass)

    def render_device(self, ptr, progress_ex=None, timelimit_ms=0.0, samples_per_launch=0, stats=False, col_block=1,
                      width=0, height=0, spp=1, max_depth=4, kind=1, seed=1, x_offset=0, x_delt=1):
        import torch

        from oracle import pyoracle
        assert samples_per_launch == 1 and timelimit_ms > 0 and progress_ex is not None
        for p in range(spp):
            t = np.zeros((len(self.cols), self.H), np.uint32)
            for c, px in enumerate(self.cols):
                _, rgba, _ = pyoracle.render(self.blob, self.W, self.H, p + 1, max_depth, kind, seed, int(px), self.W,
                                             threads=1)
                t[c] = rgba[:, px].view(np.uint32).reshape(self.H)
            self.tile.zero_()
            self.tile[:t.size].copy_(torch.from_numpy(t.view(np.int32).reshape(-1)))
            if p == self.fail_at:
                raise RuntimeError(f"injected failure at pass {p}")
            if p < spp - 1 and progress_ex(p, (p + 1) / spp, p != self.unclean_at):
                return None  # aborted (jsrt_render_device_progress_ex returns -4)


def _progressive_worker(rank, world, port, W, H, cb, spp, outdir, fail=None, unclean=None, preview_fail=None):
    """fail / unclean: (rank, pass) whose render raises / whose pass is reported unclean; preview_fail: a pass
    at which rank 0's on_preview raises.  Each rank writes its outcome to outdir/rank<r>.txt."""
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from jsraytracer_amd.tiles import FrameGather, owned_px, render_progressive
    from oracle import pyoracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fg = FrameGather(W, H, rank, world, cb)
    tile = torch.zeros(fg.maxcols * H, dtype=torch.int32)
    sc = _OracleTileScene(pyoracle.golden_scene("cornell_box_path"), tile, W, H, owned_px(W, rank, world, cb),
                          fail_at=fail[1] if fail and fail[0] == rank else None,
                          unclean_at=unclean[1] if unclean and unclean[0] == rank else None)

    def keep(p, img):
        if p == preview_fail:
            raise ValueError(f"injected preview failure at pass {p}")
        np.save(os.path.join(outdir, f"pass{p}.npy"), FrameGather.to_rgba8(img))

    try:
        render_progressive(sc, fg, tile, keep, timelimit_ms=0.0, host_tiles=True, width=W, height=H, spp=spp,
                           max_depth=8, kind=1, seed=5, x_offset=rank, x_delt=world)
        out = "ok"
    except Exception as e:  # noqa: BLE001
        out = type(e).__name__
    with open(os.path.join(outdir, f"rank{rank}.txt"), "w") as f:
        f.write(out)
    dist.barrier()
    dist.destroy_process_group()


def _run_progressive(tmp_path, world, cb, W, spp, **kw):
    mp.start_processes(_progressive_worker, args=(world, _free_port(), W, W, cb, spp, str(tmp_path), kw.get("fail"),
                                                  kw.get("unclean"), kw.get("preview_fail")),
                       nprocs=world, join=True, start_method="spawn")
    return [open(os.path.join(tmp_path, f"rank{r}.txt")).read() for r in range(world)]


@pytest.mark.parametrize("world,cb,W", [(2, 8, 16), (3, 4, 16), (3, 8, 16)])
def test_gloo_progressive_previews(tmp_path, world, cb, W):
    """tiles.render_progressive on CPU ranks: one all-reduce per pass keeps the ranks' gathers in step, and
    each pass's gathered preview is the single-process spp = p + 1 frame (oracle tiles; on the GPU the tiles
    come from jsrt_render_device_progress_ex, tests/test_gpu_multirank.py).  (3, 8, 16): rank 2 owns no
    column and still takes part in every pass."""
    from oracle import pyoracle
    spp = 3
    assert _run_progressive(tmp_path, world, cb, W, spp) == ["ok"] * world
    blob = pyoracle.golden_scene("cornell_box_path")
    for p in range(spp - 1):
        _, ref, _ = pyoracle.render(blob, W, W, p + 1, 8, 1, 5, 0, 1, threads=1)
        assert np.array_equal(np.load(os.path.join(tmp_path, f"pass{p}.npy")), ref), f"pass {p}"


def test_gloo_progressive_unclean_pass_is_not_previewed(tmp_path):
    """A pass that one rank reports unclean (a poisoned batch: its tile is not the running mean) is previewed
    by no rank; the other passes are."""
    assert _run_progressive(tmp_path, 2, 8, 16, 4, unclean=(1, 1)) == ["ok", "ok"]
    assert [os.path.exists(os.path.join(tmp_path, f"pass{p}.npy")) for p in range(3)] == [True, False, True]


@pytest.mark.parametrize("kw,expect", [
    ({"fail": (1, 0)}, ["JsrtError", "RuntimeError"]),          # rank 1's render fails in pass 0
    ({"fail": (0, 2)}, ["RuntimeError", "JsrtError"]),          # rank 0's fails after the last reported pass
    ({"preview_fail": 0}, ["ValueError", "JsrtError"]),         # rank 0's on_preview raises
    ({"preview_fail": 1}, ["ValueError", "JsrtError"]),         # ... in the last reported pass
])
def test_gloo_progressive_failure_reaches_every_rank(tmp_path, kw, expect):
    """A failure on one rank (its render, or rank 0's preview callback) ends every rank's render_progressive with
    an exception instead of leaving its peers blocked in a collective (the test would time out)."""
    assert _run_progressive(tmp_path, 2, 8, 16, 3, **kw) == expect


def _accum_worker(rank, world, port, W, H, cb, spp, outdir):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from jsraytracer_amd.tiles import AccumGather, owned_px
    from oracle import pyoracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blob = pyoracle.golden_scene("cornell_box_path")
    ag = AccumGather(W, H, rank, world, cb)
    tile = np.zeros((ag.maxcols, H, 4), np.float32)  # [owned column][row][4], as jsrt_render_device_accum
    for c, px in enumerate(owned_px(W, rank, world, cb)):
        _, _, _, acc = pyoracle.render(blob, W, H, spp, 8, 1, 5, int(px), W, threads=1, accum=True)
        tile[c] = acc[:, px]
    ag.local.copy_(torch.from_numpy(tile.reshape(-1)))
    img = ag.gather()
    if rank == 0:
        np.save(os.path.join(outdir, "accum.npy"), img.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cb", [(2, 8), (3, 4)])
def test_gloo_accum_gather_is_the_single_process_accumulator(tmp_path, world, cb):
    """tiles.AccumGather (the f32 accumulator exchange, jsrt_render_device_accum's tiles): each rank's tile is the
    oracle's accumulators of its owned columns; the gathered composite must equal the single-process frame's
    accumulators bit for bit (pixels never split across ranks: each pixel's samples are summed in order on one
    rank, src/renderers.js:93-97)."""
    from oracle import pyoracle
    W = H = 16
    spp = 3
    mp.start_processes(_accum_worker, args=(world, _free_port(), W, H, cb, spp, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(os.path.join(tmp_path, "accum.npy"))
    _, _, _, ref = pyoracle.render(pyoracle.golden_scene("cornell_box_path"), W, H, spp, 8, 1, 5, threads=1, accum=True)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def _mismatch_worker(rank, world, port, outdir):
    import torch.distributed as dist
    from jsraytracer_amd.tiles import AccumGather, FrameGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    errs = []
    for cls in (FrameGather, AccumGather):
        g = cls(8, 4, 0, 1)  # a one-rank gatherer inside a two-rank group
        try:
            g.gather()
        except RuntimeError as e:
            errs.append(str(e))
    with open(os.path.join(outdir, f"err{rank}.txt"), "w") as f:
        f.write("\n".join(errs))
    dist.barrier()
    dist.destroy_process_group()


def test_gatherer_refuses_a_group_of_another_size(tmp_path):
    """A one-rank FrameGather / AccumGather in a process whose default group has two ranks must refuse to gather
    (a gather over the whole group with one slot would hang or fail; advisor, round 5), on every rank."""
    mp.start_processes(_mismatch_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        errs = open(os.path.join(tmp_path, f"err{r}.txt")).read().splitlines()
        assert len(errs) == 2 and all("built for 1 ranks in a process group of 2" in e for e in errs)


def test_progressive_refuses_non_incremental_kinds():
    """render_progressive is the Incremental renderer's running-mean preview (renderers.js:70-117); the Simple
    and Random kinds report per batch, which a rank owning no column cannot match (advisor, round 5)."""
    from jsraytracer_amd.tiles import render_progressive
    for kind in (0, 2):
        with pytest.raises(ValueError, match="Incremental"):
            render_progressive(None, None, None, None, kind=kind)
