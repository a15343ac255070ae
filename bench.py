"""Benchmark: pixel-samples/s of the HIP renderer on BASELINE.json's headline workload.

Workload (BASELINE.json configs[1]): tests/cornell_box_path, 1024x1024, 64 spp, maxRecursionDepth 8,
IncrementalMultisamplingRenderer semantics, keyed RNG seed 1 — the reference's own scene graph
(committed as tests/golden/scenes/cornell_box_path.jsrt.gz, exported from the live reference).
A "step" renders one full frame (all 64 spp of every pixel) into HBM.  With N GPUs the frame's
columns are dealt to ranks in 16-column blocks (jsraytracer_amd/tiles.py), each rank renders its
tile, and the step ends with one gather of the tiles to rank 0 (RCCL over xGMI, nccl backend) plus the
permute into image order — strong scaling of one fixed frame.

    python bench.py [--gpus N --steps K --warmup W] [--config cornell_box_path|bunny|SDF_Menger|dragon|ASimpleScene]

Prints ONE JSON line on rank 0 (contract in the task statement), including:
  roofline      — for the DOMINANT kernel (largest share of render-kernel time): SURVEY.md §8(d)
                  algorithmic bytes per unit x units per launch / its average launch duration (HIP
                  events on the render stream, measured live) vs 8 TB/s.  traffic = HBM bytes per launch
                  from the committed rocprofv3 PMC passes (profiles/pmc_summary.json; FETCH_SIZE
                  doubled per the gfx950 correction of MI355X_MICROARCH.md, + WRITE_SIZE).  The "valu"
                  member carries the compute side, which binds for the analytic/SDF scenes.
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
    # name: (scene, W, H, spp, kind, max_depth)
    "cornell_box_path": ("cornell_box_path", 1024, 1024, 64, 1, 8),
    "bunny": ("bunny", 1920, 1080, 16, 1, 4),
    "SDF_Menger": ("SDF_Menger", 1024, 1024, 32, 1, 4),
    "ASimpleScene": ("ASimpleScene", 256, 256, 1, 1, 4),
    # BASELINE.json configs[4]: the dragon mesh is built natively from its OBJ (include/jsrt_mesh.h) on
    # the box, since the reference-built blob is ~47 MB; its tree is bit-identical (tests/test_mesh_build.py)
    "dragon": ("dragon", 4096, 4096, 256, 1, 4),
}
MESH_SCENES = ("dragon",)  # loaded as skeleton + OBJ from tests/golden/meshes
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md chip table (HBM3E 8 TB/s spec)
F64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector (half the 157.3 TF FP32 vector rate)
CLOCK_HZ = 2.4e9            # max clock, MI355X_MICROARCH.md chip table
SIMDS = 256 * 4
# issue cycles per wave64 VALU instruction on a SIMD-32 (MI355X_MICROARCH.md: f32 2 cyc; f64 at half
# the f32 rate; transcendentals 4x)
ISSUE_CYC = {"f64": 4.0, "trans_f64": 16.0, "trans_f32": 8.0, "other": 2.0}


def env_int(name, default):
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


def kernel_units(counts, kname):
    """(units per pixel-sample, algorithmic bytes per unit, unit name) of one kernel, SURVEY.md §8(d):
    node visits x 32 B + triangle tests x 64 B + top-level object tests x 128 B per cast."""
    if kname.startswith("k_shadow"):
        n = counts["shadow_casts"]
        b = counts["shadow_node_visits"] * 32 + counts["shadow_tri_tests"] * 64 + counts["shadow_object_tests"] * 128
        return n, (b / n if n else 0.0), "shadow cast"
    if kname.startswith("k_extend"):
        n = counts["casts"] - counts["shadow_casts"]
        b = ((counts["node_visits"] - counts["shadow_node_visits"]) * 32 +
             (counts["tri_tests"] - counts["shadow_tri_tests"]) * 64 +
             (counts["object_tests"] - counts["shadow_object_tests"]) * 128)
        return n, (b / n if n else 0.0), "closest-hit cast"
    return None, None, None


def cpu_baseline(blob, W, H, spp, kind, depth, target_s=12.0):
    """The oracle (C port of the reference path) timed on a bounded column subsample of the same frame."""
    from oracle import pyoracle
    threads = min(16, os.cpu_count() or 1)
    stride = max(1, W // max(threads, 1))  # probe: a thin slice to estimate speed, then size the sample
    t = time.time()
    _, _, st = pyoracle.render(blob, W, H, spp, depth, kind, 1, 0, stride, threads=threads)
    dt = max(time.time() - t, 1e-3)
    want = st["samples"] / dt * target_s
    ncols = int(max(threads, min(W, want / (H * spp))))
    stride = max(1, W // ncols)
    t = time.time()
    _, _, st = pyoracle.render(blob, W, H, spp, depth, kind, 1, 0, stride, threads=threads)
    dt = time.time() - t
    counts = {k: st[k] / st["samples"] for k in st}
    sample = f"columns px%{stride}==0 of the {W}x{H}x{spp} frame ({st['samples']} pixel-samples, {dt:.1f} s)"
    return {"value": st["samples"] / dt, "unit": "pixel-samples/s", "cores": threads, "kind": "port",
            "sample": sample}, counts


def load_pmc(config, kname):
    """Counters of kernel `kname` (any template instance: one kernel profile runs per scene)."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None, None, kname
    d = json.load(open(p)).get(config)
    if not d:
        return None, None, kname
    hits = [k for k in d["kernels"] if k == kname or k.startswith(kname + "<")]
    if len(hits) != 1:
        return None, None, kname
    return d["kernels"][hits[0]], d.get("source"), hits[0]


def roofline(config, dom, avg_ms, launches, counts, samples_per_frame):
    """dom: the dominant kernel; avg_ms: its average launch duration from the HIP events that
    bracketed its launches in the timed region (on the render stream)."""
    kname = dom
    per_sample, bpu, unit = kernel_units(counts, dom) if counts else (None, None, None)
    r = {"bound": "hbm", "kernel": kname, "unit": "GB/s", "peak": HBM_PEAK_GBS, "avg_launch_ms": avg_ms,
         "launches_per_step": launches, "achieved": None, "frac": None, "traffic": None}
    if per_sample:
        units_per_launch = per_sample * samples_per_frame / launches
        per_launch = bpu * units_per_launch
        r.update(achieved=per_launch / (avg_ms * 1e-3) / 1e9, algorithmic_bytes_per_launch=per_launch,
                 bytes_per_unit=bpu, work_unit=unit, units_per_launch=units_per_launch)
        r["frac"] = r["achieved"] / HBM_PEAK_GBS
    pmc, src, r["kernel"] = load_pmc(config, kname)
    if pmc:
        n = pmc["dispatches"]
        traffic = (2 * pmc.get("FETCH_SIZE", 0) + pmc.get("WRITE_SIZE", 0)) * 1024 / n  # KB -> B, gfx950 x2
        r["traffic"] = traffic
        r["traffic_GBs"] = traffic / (avg_ms * 1e-3) / 1e9
        r["traffic_frac"] = r["traffic_GBs"] / HBM_PEAK_GBS
        f64 = pmc.get("SQ_INSTS_VALU_ADD_F64", 0) + pmc.get("SQ_INSTS_VALU_MUL_F64", 0) + pmc.get("SQ_INSTS_VALU_FMA_F64", 0)
        tr64, tr32 = pmc.get("SQ_INSTS_VALU_TRANS_F64", 0), pmc.get("SQ_INSTS_VALU_TRANS_F32", 0)
        other = pmc.get("SQ_INSTS_VALU", 0) - f64 - tr64 - tr32
        lane = pmc["SQ_THREAD_CYCLES_VALU"] / (64 * pmc["SQ_ACTIVE_INST_VALU"]) if pmc.get("SQ_ACTIVE_INST_VALU") else None
        issue = (f64 * ISSUE_CYC["f64"] + tr64 * ISSUE_CYC["trans_f64"] + tr32 * ISSUE_CYC["trans_f32"] +
                 other * ISSUE_CYC["other"]) / n
        flops = (pmc.get("SQ_INSTS_VALU_ADD_F64", 0) + pmc.get("SQ_INSTS_VALU_MUL_F64", 0) +
                 2 * pmc.get("SQ_INSTS_VALU_FMA_F64", 0)) * 64 * (lane or 1) / n
        r["valu"] = {"issue_frac": issue / (SIMDS * CLOCK_HZ * avg_ms * 1e-3), "lane_utilisation": lane,
                     "f64_tflops": flops / (avg_ms * 1e-3) / 1e12, "f64_peak_tflops": F64_PEAK_TFLOPS,
                     "valu_insts_per_launch": pmc.get("SQ_INSTS_VALU", 0) / n}
        r["pmc_source"] = src
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="cornell_box_path", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--col-block", type=int, default=16)
    ap.add_argument("--no-events", action="store_true", help="A/B: time steps without per-launch HIP events")
    ap.add_argument("--spp", type=int, default=0, help="profiling only: override the config's spp (same launch "
                    "shapes, fewer batches); a bench line with it is not the config's number")
    args = ap.parse_args()

    rank, world, local = env_int("RANK", 0), env_int("WORLD_SIZE", 1), env_int("LOCAL_RANK", 0)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import jsraytracer_amd as jr
    from jsraytracer_amd.tiles import FrameGather
    from oracle import pyoracle  # fixture loader only; the oracle runs only in the cpu_baseline leg

    scene_name, W, H, spp, kind, depth = CONFIGS[args.config]
    if args.spp > 0:
        spp = args.spp
    t_load = time.perf_counter()
    if scene_name in MESH_SCENES:
        meshes = os.path.join(ROOT, "tests", "golden", "meshes")
        with open(os.path.join(meshes, "topology.json")) as f:
            topo = json.load(f)[scene_name]
        import gzip
        with gzip.open(os.path.join(meshes, topo["skeleton"]), "rb") as f:
            skel = f.read()
        blob, _ = jr.load_obj_scene(skel, os.path.join(meshes, topo["obj_fixture"]))
    else:
        blob = pyoracle.golden_scene(scene_name)
    t_build = time.perf_counter() - t_load
    scene = jr.Scene(blob, device=local)
    t_upload = time.perf_counter() - t_load - t_build

    cb = args.col_block if world > 1 else 1
    fg = FrameGather(W, H, rank, world, cb, device=f"cuda:{local}")
    stream = torch.cuda.current_stream().cuda_stream

    STAGES = jr._native.STAGES

    def step(events=None):
        """events: None = no HIP events; 0 = every stage; else a bitmask of stages (jsrt.h stage_events)."""
        st = scene.render_device(fg.local.data_ptr(), stream_ptr=stream, col_block=cb, width=W, height=H, spp=spp,
                                 max_depth=depth, kind=kind, seed=1, x_offset=rank if world > 1 else 0,
                                 x_delt=world, stats=events is not None, stage_events=events or 0)
        fg.gather()
        return st

    # warmup; the last warmup step is fully instrumented and names the dominant kernel
    st_full = None
    for w in range(max(args.warmup, 1)):
        st_full = step(0 if w == max(args.warmup, 1) - 1 else None)
    dom = max(st_full["stage_ms"], key=lambda k: st_full["stage_ms"][k])
    # timed region: HIP events bracket only the dominant kernel's launches (its average launch
    # duration for the roofline); events on every launch would add launch gaps to the step
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = [step(None if args.no_events else (1 << STAGES.index(dom))) for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tt = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())
    if args.no_events:
        stats = [step(1 << STAGES.index(dom))]
    dom_ms = sum(s["stage_ms"][dom] for s in stats) / len(stats)
    dom_launches = stats[0]["stage_launches"][dom]
    # per-stage split: one more step after the timed region with every launch bracketed
    st_after = step(0)
    stage_ms, stage_launches, kernel_ms = st_after["stage_ms"], st_after["stage_launches"], st_after["kernel_ms"]

    if rank == 0:
        total = W * H * spp
        value = total * args.steps / elapsed
        cpu, counts = (None, None)
        if not args.no_cpu_baseline and world == 1:
            cpu, counts = cpu_baseline(blob, W, H, spp, kind, depth)
        roof = roofline(args.config, dom, dom_ms / max(dom_launches, 1), dom_launches, counts, fg.ncols * H * spp)
        line = {
            "metric": "pixel-samples/sec + %HBM-roofline, cornell_box_path 1024² @1/2/4/8 GPU",
            "value": value, "unit": "pixel-samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64",
            "data": "reference scene graph (exported from the live reference, not synthetic), keyed RNG seed 1",
            "config": {"workload": f"{scene_name} {W}x{H} {spp}spp depth {depth} (Incremental)", "width": W,
                       "height": H, "spp": spp, "max_depth": depth, "parallelism": f"tiles{world}",
                       "col_block": cb},
            "roofline": roof, "cpu_baseline": cpu,
            "kernel_ms_per_step": kernel_ms,
            "scene_build_s": round(t_build, 3), "scene_upload_s": round(t_upload, 3),
            "events_lost": {"timed": sum(x["events_lost"] for x in stats), "stage_split": st_after["events_lost"]},
            "frame_attempts": [x["attempts"] for x in stats],
            "stages_note": "stage split from one fully-instrumented step after the timed region",
            "stages_ms_per_step": {k: round(v, 3) for k, v in stage_ms.items()},
            "stage_launches_per_step": stage_launches,
            "counts_per_sample": {k: round(v, 4) for k, v in counts.items() if k != "samples"} if counts else None,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
