"""Projected multi-GPU strong scaling from ONE GPU: every rank's share of the frame timed on device 0.

    python tools/project_scaling.py [--config cornell_box_path] [--ranks 1,2,4,8] [--steps 3] [--out FILE]

bench.py --gpus N splits a frame into 16-column blocks dealt round-robin (jsraytracer_amd/tiles.py; the
reference's column split, src/raytrace_launcher.js:65-101, src/renderers.js:88) and ends each step with one
gather.  A one-GPU box cannot run N ranks side by side, but each rank's share is an independent render on its
own GPU: its time on one MI355X is its time in the N-GPU job.  For each N this renders every rank's share
(jsrt_render_device, col_block 16, x_offset = r, x_delt = N) for `steps` timed frames after one warmup frame
of that shape, and reports per-share ms, the slowest share (the job's render time: the step waits for the
last rank), and the implied efficiency T1 / (N * max share) -- before the gather, whose bytes (4 B per pixel,
RGBA8, over xGMI) are listed beside it.  This is a projection, not a measured multi-GPU curve."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cornell_box_path")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--stages", action="store_true", help="per share, one more render on one stream with HIP events "
                    "around every launch: its per-stage ms (where a share's time goes) and batch count")
    ap.add_argument("--col-block", type=int, default=16, help="columns per block dealt round-robin to ranks (bench.py "
                    "--col-block; W / N: one contiguous strip per rank)")
    ap.add_argument("--only-rank0", action="store_true", help="time rank 0's share only at N > 1 (a quicker stage split)")
    args = ap.parse_args()
    import torch

    import bench
    import jsraytracer_amd as jr
    from jsraytracer_amd.tiles import owned_px
    from oracle import pyoracle  # fixture loader only (the scene blob / mesh skeleton)
    scene_name, W, H, spp, kind, depth, _ = bench.CONFIGS[args.config]
    blob = pyoracle.mesh_scene(scene_name, jr)[0] if scene_name in bench.MESH_SCENES else pyoracle.golden_scene(scene_name)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    rows = []
    t1 = None
    for n in [int(x) for x in args.ranks.split(",")]:
        cb = (args.col_block if args.col_block > 0 else W // n) if n > 1 else 1
        shares = []
        for r in range(1 if (args.only_rank0 and n > 1) else n):
            sc = jr.Scene(blob, device=0)  # each rank's own scene (its own learned pools and bounds)
            ncols = len(owned_px(W, r, n, cb))
            tile = torch.zeros(max(ncols, 1) * H, dtype=torch.int32, device="cuda:0")
            kw = dict(stream_ptr=stream.cuda_stream, col_block=cb, width=W, height=H, spp=spp, max_depth=depth,
                      kind=kind, seed=1, x_offset=r if n > 1 else 0, x_delt=n, stats=False)
            sc.render_device(tile.data_ptr(), **kw)  # warmup: learns this share's pools and launch bounds
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                sc.render_device(tile.data_ptr(), **kw)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            share = {"rank": r, "columns": ncols, "paths": ncols * H * spp, "ms": ms}
            if args.stages:
                st = sc.render_device(tile.data_ptr(), **dict(kw, stats=True, stage_events=jr._native.EVENTS_ONE_STREAM))
                share["stages_ms"] = {k: round(v, 3) for k, v in st["stage_ms"].items() if v}
                share["batches"], share["attempts"] = st["batches"], st["attempts"]
                print(f"   stages {share['stages_ms']} batches {st['batches']} attempts {st['attempts']}", file=sys.stderr,
                      flush=True)
            shares.append(share)
            sc.close()
            print(f"N={n} rank {r}: {ncols} columns, {ms:.2f} ms", file=sys.stderr, flush=True)
        worst = max(s["ms"] for s in shares)
        if len(shares) < n:  # --only-rank0: rank 0's share stands for every share
            shares += [dict(shares[0], rank=r, projected_from_rank0=True) for r in range(1, n)]
        if n == 1:
            t1 = worst
        row = {"n": n, "max_share_ms": worst, "mean_share_ms": sum(s["ms"] for s in shares) / n,
               "projected_samples_per_s": W * H * spp / (worst * 1e-3),
               "efficiency_vs_1": (t1 / (n * worst)) if t1 else None,
               "gather_bytes": W * H * 4 if n > 1 else 0, "shares": shares}
        row["col_block"] = cb
        rows.append(row)
        print(json.dumps({k: v for k, v in row.items() if k != "shares"}), flush=True)
    out = {"config": args.config, "workload": f"{scene_name} {W}x{H} {spp}spp depth {depth}", "steps": args.steps,
           "build_id": jr._native.build_id(), "knobs": bench.knobs(), "rows": rows,
           "note": "each rank's share rendered alone on one MI355X (its time in the N-GPU job); the gather of 4 B "
                   "per pixel to rank 0 is not included; a projection, not a measured multi-GPU curve"}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
