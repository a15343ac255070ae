"""Benchmark: pixel-samples/s of the HIP renderer on BASELINE.json's headline workload.

Workload (BASELINE.json configs[1]): tests/cornell_box_path, 1024x1024, 64 spp, maxRecursionDepth 8,
IncrementalMultisamplingRenderer semantics, keyed RNG seed 1 — the reference's own scene graph
(committed as tests/golden/scenes/cornell_box_path.jsrt.gz, exported from the live reference).
A "step" renders one full frame (all 64 spp of every pixel) into HBM; with N GPUs the frame's columns
are dealt to ranks in 16-column blocks (rank r owns blocks b with b % N == r) and gathered to rank 0
over RCCL (torch.distributed nccl backend) — strong scaling of one fixed frame.

    python bench.py [--gpus N --steps K --warmup W] [--config cornell_box_path|dragon|bunny|SDF_Menger]

Prints ONE JSON line on rank 0 (contract in the task statement), including:
  roofline      — algorithmic bytes per launch (SURVEY.md §8(d) formula with counts measured by the
                  oracle on the CPU-baseline sample) / measured launch time (HIP events on the render
                  stream) vs 8 TB/s; traffic from committed rocprofv3 PMC passes when present.
  cpu_baseline  — the C oracle (port of the reference path) on a bounded column subsample, host cores.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (scene, W, H, spp, kind, max_depth or None = scene's)
    "cornell_box_path": ("cornell_box_path", 1024, 1024, 64, 1, 8),
    "bunny": ("bunny", 1920, 1080, 16, 1, 4),
    "SDF_Menger": ("SDF_Menger", 1024, 1024, 32, 1, 4),
    "ASimpleScene": ("ASimpleScene", 256, 256, 1, 1, 4),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (HBM3E 8 TB/s spec)


def env_int(name, default):
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


def algorithmic_bytes_per_sample(counts, spp):
    """node visits x 32 B + triangle tests x 64 B + top-level object tests x 128 B,
    plus the per-pixel RGBA8 output (4 B) amortised over spp."""
    return counts["node_visits"] * 32 + counts["tri_tests"] * 64 + counts["object_tests"] * 128 + 4.0 / spp


def cpu_baseline(blob, W, H, spp, kind, depth, target_s=12.0):
    """The oracle (C port of the reference path) timed on a bounded column subsample of the same frame."""
    from oracle import pyoracle
    threads = min(16, os.cpu_count() or 1)
    # probe: a thin slice to estimate speed, then size the sample to ~target_s
    stride = max(1, W // max(threads, 1))
    t = time.time()
    _, _, st = pyoracle.render(blob, W, H, spp, depth, kind, 1, 0, stride, threads=threads)
    dt = max(time.time() - t, 1e-3)
    rate = st["samples"] / dt
    want = rate * target_s
    per_col = H * spp
    ncols = int(max(threads, min(W, want / per_col)))
    stride = max(1, W // ncols)
    t = time.time()
    _, _, st = pyoracle.render(blob, W, H, spp, depth, kind, 1, 0, stride, threads=threads)
    dt = time.time() - t
    counts = {k: st[k] / st["samples"] for k in st}
    sample = f"columns px%{stride}==0 of the {W}x{H}x{spp} frame ({st['samples']} pixel-samples, {dt:.1f} s)"
    return {"value": st["samples"] / dt, "unit": "pixel-samples/s", "cores": threads, "kind": "port",
            "sample": sample}, counts


def load_pmc(config):
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    return d.get(config)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="cornell_box_path", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--col-block", type=int, default=16)
    args = ap.parse_args()

    rank, world, local = env_int("RANK", 0), env_int("WORLD_SIZE", 1), env_int("LOCAL_RANK", 0)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import jsraytracer_amd as jr
    from oracle import pyoracle  # fixture loader only; the oracle runs only in the cpu_baseline leg

    scene_name, W, H, spp, kind, depth = CONFIGS[args.config]
    blob = pyoracle.golden_scene(scene_name)
    scene = jr.Scene(blob, device=local)

    cb = args.col_block if world > 1 else 1
    ncols = jr.owned_columns(W, rank, world, cb) if world > 1 else W
    maxcols = max(jr.owned_columns(W, r, world, cb) for r in range(world)) if world > 1 else W
    out = torch.zeros(maxcols * H, dtype=torch.int32, device=f"cuda:{local}")
    gather = [torch.empty_like(out) for _ in range(world)] if (world > 1 and rank == 0) else None
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        st = scene.render_device(out.data_ptr(), stream_ptr=stream, col_block=cb, width=W, height=H, spp=spp,
                                 max_depth=depth, kind=kind, seed=1, x_offset=rank if world > 1 else 0,
                                 x_delt=world)
        if world > 1:
            dist.gather(out, gather, dst=0)
        return st

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = [step() for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tt = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())

    kernel_ms = sum(s["kernel_ms"] for s in stats) / len(stats)
    stage_ms = {k: sum(s["stage_ms"][k] for s in stats) / len(stats) for k in stats[0]["stage_ms"]}
    stage_launches = stats[0]["stage_launches"]
    kt = torch.tensor([kernel_ms], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(kt, op=dist.ReduceOp.MAX)
    kernel_ms = float(kt.item())

    if rank == 0:
        total = W * H * spp
        value = total * args.steps / elapsed
        cpu, counts = (None, None)
        if not args.no_cpu_baseline and world == 1:
            cpu, counts = cpu_baseline(blob, W, H, spp, kind, depth)
        roof = None
        if counts is not None:
            bps = algorithmic_bytes_per_sample(counts, spp)
            per_launch = bps * ncols * H * spp
            achieved = per_launch / (kernel_ms * 1e-3) / 1e9
            pmc = load_pmc(args.config)
            roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
                    "bytes_per_sample": bps, "kernel_ms": kernel_ms,
                    "counts_per_sample": {k: round(v, 4) for k, v in counts.items() if k != "samples"}}
        line = {
            "metric": "pixel-samples/sec + %HBM-roofline, cornell_box_path 1024² @1/2/4/8 GPU",
            "value": value, "unit": "pixel-samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64", "data": "reference scene graph (synthetic-free), keyed RNG seed 1",
            "config": {"workload": f"{scene_name} {W}x{H} {spp}spp depth {depth} (Incremental)", "width": W,
                       "height": H, "spp": spp, "max_depth": depth, "parallelism": f"tiles{world}",
                       "col_block": cb},
            "roofline": roof, "cpu_baseline": cpu,
            "stages_ms_per_step": {k: round(v, 3) for k, v in stage_ms.items()},
            "stage_launches_per_step": stage_launches,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
