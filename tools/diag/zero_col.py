"""Diagnostic: 3 gloo ranks on device 0, W=32, col_block 16 (rank 2 owns no column), render_progressive with every
callback and exchange printed."""
import os
import socket
import sys

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_main(rank, world, port):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import jsraytracer_amd as jr
    from jsraytracer_amd import tiles
    from oracle import pyoracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0)
    fg = tiles.FrameGather(32, 192, rank, world, 16)
    dev = torch.zeros(fg.maxcols * 192, dtype=torch.int32, device="cuda:0")
    orig = sc.render_device

    def traced(ptr, progress_ex=None, **kw):
        def cb(p, c, clean):
            r = progress_ex(p, c, clean)
            print(f"rank {rank}: pass {p} completion {c:.3f} clean {clean} -> abort {r}", flush=True)
            return r
        out = orig(ptr, progress_ex=cb, **kw)
        print(f"rank {rank}: render_device returned {out}", flush=True)
        return out
    sc.render_device = traced
    tiles.render_progressive(sc, fg, dev, lambda p, img: print(f"preview {p}", flush=True), timelimit_ms=0.0,
                             host_tiles=True, width=32, height=192, spp=4, max_depth=8, kind=1, seed=1, x_offset=rank,
                             x_delt=world)
    print(f"rank {rank}: done", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(rank_main, args=(3, port), nprocs=3, join=True, start_method="spawn")
