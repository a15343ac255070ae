"""Benchmark: pixel-samples/s of the HIP renderer on BASELINE.json's workloads.

Headline (BASELINE.json configs[1]): tests/cornell_box_path, 1024x1024, 64 spp, maxRecursionDepth 8,
IncrementalMultisamplingRenderer semantics, keyed RNG seed 1 -- the reference's own scene graph
(committed as tests/golden/scenes/cornell_box_path.jsrt.gz, exported from the live reference).
A "step" renders one full frame (all spp of every pixel) into HBM.  With N GPUs the frame's columns
are dealt to ranks in 16-column blocks (jsraytracer_amd/tiles.py), each rank renders its tile, and
the step ends with one gather of the tiles to rank 0 (RCCL over xGMI, nccl backend) plus the permute
into image order -- strong scaling of one fixed frame (the reference's column split across workers,
src/raytrace_launcher.js:65-101, src/renderers.js:88).

    python bench.py [--gpus N --steps K --warmup W] [--config cornell_box_path|bunny|SDF_Menger|dragon|ASimpleScene]

--gpus N > 1 without a torch.distributed environment spawns N rank processes of this script (one per
GPU, RANK/LOCAL_RANK/WORLD_SIZE set, rendezvous on 127.0.0.1) before anything touches a GPU; under
torchrun the environment is used as given.

Prints ONE JSON line on rank 0 (contract in the task statement), including:
  roofline      -- for the DOMINANT kernel (largest share of render-kernel time), against the resource
                   that binds it: "valu" (scene cache-resident: cornell, bunny, Menger,
                   ASimpleScene) reports the kernel's f64 TFLOP/s (PMC-counted f64 flops per launch, from
                   the committed rocprofv3 passes in profiles/pmc_summary.json, over its average launch
                   duration measured live with HIP events on the render stream) against 78.6 TF, with
                   the VALU issue fraction and HBM traffic beside it; "hbm" (dragon: 13 MB of BVH and
                   triangles) reports SURVEY.md §8(d) algorithmic bytes per launch over the same live
                   duration against 8 TB/s.
  cpu_baseline  -- the C oracle (port of the reference path) on a bounded column subsample, host cores,
                   with the reference JS web-worker figure recorded in BASELINE.md beside it.
  parity        -- the last timed frame's columns checked against the oracle's render of the same columns:
                   RGBA8 bit-exact, f32 colour |d| <= 1e-5 (north_star), at the benchmark's full size.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (scene, W, H, spp, kind, max_depth, binding resource)
    "cornell_box_path": ("cornell_box_path", 1024, 1024, 64, 1, 8, "valu"),
    "bunny": ("bunny", 1920, 1080, 16, 1, 4, "valu"),
    "SDF_Menger": ("SDF_Menger", 1024, 1024, 32, 1, 4, "valu"),
    "ASimpleScene": ("ASimpleScene", 256, 256, 1, 1, 4, "valu"),
    # BASELINE.json configs[4]: the dragon mesh is built natively from its OBJ (include/jsrt_mesh.h) on
    # the box, since the reference-built blob is ~47 MB; its tree is bit-identical (tests/test_mesh_build.py)
    "dragon": ("dragon", 4096, 4096, 256, 1, 4, "hbm"),
}
HEADLINE = "cornell_box_path"
METRIC = "pixel-samples/sec + %HBM-roofline, {scene} {size} @1/2/4/8 GPU"  # BASELINE.json metric, per config
MESH_SCENES = ("dragon",)  # loaded as skeleton + OBJ from tests/golden/meshes
# the reference JS web-worker path, measured in the survey container:
# node 12 worker_threads, 8 workers, column interleave; it cannot run on the GPU box (no reference there)
REFERENCE_JS = {"cornell_box_path": (10751, "64^2x4spp / 128^2x2spp"), "bunny": (18388, "128^2x1spp"),
                "dragon": (21816, "128^2x1spp (Incremental forced to 1 spp)"), "SDF_Menger": (3306, "64^2x1spp"),
                "ASimpleScene": (29627, "128^2x1spp")}
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md chip table (HBM3E 8 TB/s spec)
F64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector (half the 157.3 TF FP32 vector rate)
CLOCK_HZ = 2.4e9            # max clock, MI355X_MICROARCH.md chip table
SIMDS = 256 * 4
# issue cycles per wave64 VALU instruction (MI355X_MICROARCH.md: f32 / int on a SIMD-32 2 cyc; f64 at
# half the f32 rate 4; transcendentals 4x their type's rate)
ISSUE_CYC = {"f64": 4.0, "trans_f64": 16.0, "trans_f32": 8.0, "other": 2.0}
TOL = 1e-5                  # north_star: RGB L-inf on the f32 colour handed to setColor
# Whether FETCH_SIZE counts 4-B-per-lane coalesced loads at their full bytes on gfx950.  Measured (tools/fetch_calib.hip,
# profiles/fetch_calib_r05.json, 1 GiB streams): FETCH_SIZE reads 0.500 of the bytes of 4-B and of 16-B coalesced
# loads alike, WRITE_SIZE 1.000 of coalesced 4-B and 16-B stores, and a lone 4-B store to a line costs 32 B (one
# 32-B sector) -- so the x2 on FETCH_SIZE holds for this path's SoA planes too.
FETCH_4B_EXACT = False


def env_int(name, default):
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """One process per GPU (rank r on device r), started before this process touches a GPU.  Rank 0
    prints the bench line.  If any rank fails the others are stopped (they would wait in a collective)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.2)
    return rc


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


def oracle_columns(blob, W, H, spp, kind, depth, x_offset, x_delt, threads):
    from oracle import pyoracle
    t = time.time()
    col, rgba, st = pyoracle.render(blob, W, H, spp, depth, kind, 1, x_offset, x_delt, threads=threads)
    return col, rgba, st, time.time() - t


def cpu_baseline(blob, W, H, spp, kind, depth, target_s=12.0):
    """The oracle (C port of the reference path) timed on a bounded column subsample of the same frame.
    Returns the baseline record, per-sample counts, and the oracle's columns (kept for the parity check)."""
    threads = min(16, os.cpu_count() or 1)
    stride = max(1, W // max(threads, 1))  # probe: a thin slice to estimate speed, then size the sample
    _, _, st, dt = oracle_columns(blob, W, H, spp, kind, depth, 0, stride, threads)
    want = st["samples"] / max(dt, 1e-3) * target_s
    ncols = int(max(threads, min(W, want / (H * spp))))
    stride = max(1, W // ncols)
    col, rgba, st, dt = oracle_columns(blob, W, H, spp, kind, depth, 0, stride, threads)
    counts = {k: st[k] / st["samples"] for k in st}
    sample = f"columns px%{stride}==0 of the {W}x{H}x{spp} frame ({st['samples']} pixel-samples, {dt:.1f} s)"
    base = {"value": st["samples"] / dt, "unit": "pixel-samples/s", "cores": threads, "kind": "port",
            "sample": sample}
    return base, counts, (col, rgba, 0, stride)


def parity(image, colors, ref):
    """image: [H, W, 4] u8 of the timed frame (rank 0, after the gather); colors: [H, W, 4] f32 or None;
    ref: (oracle colours, oracle rgba, x_offset, x_delt) of the same frame's columns."""
    import numpy as np
    ocol, orgba, x0, dx = ref
    cols = list(range(x0, image.shape[1], dx))
    bad = (image[:, cols] != orgba[:, cols]).any(-1)
    out = {"columns": len(cols), "column_stride": dx, "pixels": int(bad.size), "rgba8_pixels_differing": int(bad.sum()),
           "rgba8_max_abs": int(np.abs(image[:, cols].astype(int) - orgba[:, cols].astype(int)).max())}
    if colors is not None:
        g, o = colors[:, cols, :3], ocol[:, cols, :3]
        fin = np.isfinite(o)
        out["f32_max_abs"] = float(np.abs(g[fin] - o[fin]).max()) if fin.any() else 0.0
        out["f32_nonfinite_pattern_equal"] = bool(np.array_equal(np.isfinite(g), fin))
        out["f32_bit_exact"] = bool(np.array_equal(g.view(np.uint32), o.view(np.uint32)))
        out["tolerance"] = TOL
        out["pass"] = out["rgba8_pixels_differing"] == 0 and out["f32_max_abs"] <= TOL and out["f32_nonfinite_pattern_equal"]
    else:
        out["pass"] = out["rgba8_pixels_differing"] == 0
    return out


# environment knobs that change the library's schedule (A/B experiments, tools/ab_env.sh) or swap the library
# itself (JSRT_LIB: a variant build); JSRT_BENCH_BACKEND only picks the multi-rank gather backend
# (JSRT_OFFLOAD_ARCH is a build variable: it never changes a built library's behaviour at run time)
NOT_KNOBS = ("JSRT_BENCH_BACKEND", "JSRT_OFFLOAD_ARCH")


def knobs():
    """Every JSRT_* environment variable set for this run that can change what is timed."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("JSRT_") and k not in NOT_KNOBS}


def exit_status(par):
    """Process exit status after the bench line: non-zero when the timed frame failed its parity check."""
    if par is not None and not par["pass"]:
        print(f"bench: PARITY FAILURE against the oracle: {par}", file=sys.stderr)
        return 3
    return 0


def _stage_kernel(kernels, kname, weight):
    """The stage's kernel among `kernels` (any template instance, or its persistent-cast form k_extend_q)."""
    hits = [k for k in kernels if k.split("<")[0] in (kname, kname + "_q")]
    return max(hits, key=lambda h: weight(kernels[h])) if hits else None


def load_pmc(config, kname):
    """Counters of kernel `kname` (any template instance: one kernel profile runs per scene), the summary's
    source and the library build its passes ran (tools/pmc_summary.py)."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None, None, kname, None
    d = json.load(open(p)).get(config)
    if not d:
        return None, None, kname, None
    k = _stage_kernel(d["kernels"], kname, lambda c: c.get("SQ_WAVE_CYCLES", c.get("dispatches", 0)))
    if k is None:
        return None, None, kname, None
    return d["kernels"][k], d.get("source"), k, d.get("build_id")


def load_rocprof(config, kname, build_id):
    """The committed rocprofv3 kernel summary of this build and config (profiles/*_kernel_stats.meta.json,
    tools/stamp_stats.py): (file, kernel, average launch ms) of the stage's kernel, or None."""
    import glob
    for meta in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_kernel_stats.meta.json"))):
        try:
            m = json.load(open(meta))
        except ValueError:
            continue
        if m.get("build_id") != build_id or m.get("config") != config:
            continue
        k = _stage_kernel(m["kernels"], kname, lambda c: c["calls"] * c["avg_ms"])
        if k:  # the instrumented step's launches (tools/stamp_stats.py) are the ones the live figure times
            c = m["kernels"][k]
            return os.path.relpath(meta, ROOT), k, c.get("instrumented_step", c)["avg_ms"], c["avg_ms"]
    return None


def roofline(config, bound, dom, avg_ms, launches, counts, samples_per_frame, build_id=None):
    """dom: the dominant kernel; avg_ms: its average launch duration from the HIP events that bracketed
    its launches in the timed region (on the render stream); build_id: the timed library's."""
    per_sample, bpu, unit = kernel_units(counts, dom) if counts else (None, None, None)
    r = {"bound": bound, "kernel": dom, "avg_launch_ms": avg_ms, "launches_per_step": launches,
         "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
         "timing_note": "avg_launch_ms: HIP events around the kernel's launches in one instrumented step after the "
                        "timed region; a render with per-launch events runs on one stream (its launches do not "
                        "overlap other batches', DESIGN.md §4.2), so this is the kernel's own launch time -- the "
                        "timed steps run the two-stream schedule without events"}
    sec = avg_ms * 1e-3
    if per_sample:
        units_per_launch = per_sample * samples_per_frame / launches
        per_launch = bpu * units_per_launch
        r["algorithmic"] = {"bytes_per_launch": per_launch, "bytes_per_unit": bpu, "work_unit": unit,
                            "units_per_launch": units_per_launch, "GBs": per_launch / sec / 1e9,
                            "frac_of_hbm": per_launch / sec / 1e9 / HBM_PEAK_GBS,
                            "note": "SURVEY.md §8(d) scene-record bytes; > 1 of HBM means cache-served"}
    pmc, src, r["kernel"], pmc_bid = load_pmc(config, dom)
    rp = load_rocprof(config, dom, build_id)
    if rp:  # the committed rocprofv3 summary of the same build: its average launch time beside the live one
        r["rocprof"] = {"file": rp[0], "kernel": rp[1], "avg_launch_ms": rp[2], "live_over_rocprof": avg_ms / rp[2],
                        "avg_launch_ms_all_frames": rp[3]}
    if pmc:
        n = pmc["dispatches"]
        # FETCH_SIZE (KB): MI355X_MICROARCH.md reads 1/2 of the bytes of wide (16 B/lane) coalesced streaming
        # loads on gfx950; the calibration of this path's 4-B SoA planes (FETCH_4B_EXACT above) decides which
        # reading is `traffic`; both are reported.
        raw = (pmc.get("FETCH_SIZE", 0) + pmc.get("WRITE_SIZE", 0)) * 1024 / n
        x2 = (2 * pmc.get("FETCH_SIZE", 0) + pmc.get("WRITE_SIZE", 0)) * 1024 / n
        traffic = raw if FETCH_4B_EXACT else x2
        r["traffic"] = traffic
        r["traffic_readings"] = {"fetch_x1": raw, "fetch_x2": x2, "used": "fetch_x1" if FETCH_4B_EXACT else "fetch_x2"}
        r["traffic_GBs"] = traffic / sec / 1e9
        r["traffic_frac"] = r["traffic_GBs"] / HBM_PEAK_GBS
        f64 = pmc.get("SQ_INSTS_VALU_ADD_F64", 0) + pmc.get("SQ_INSTS_VALU_MUL_F64", 0) + pmc.get("SQ_INSTS_VALU_FMA_F64", 0)
        tr64, tr32 = pmc.get("SQ_INSTS_VALU_TRANS_F64", 0), pmc.get("SQ_INSTS_VALU_TRANS_F32", 0)
        other = pmc.get("SQ_INSTS_VALU", 0) - f64 - tr64 - tr32
        lane = pmc["SQ_THREAD_CYCLES_VALU"] / (64 * pmc["SQ_ACTIVE_INST_VALU"]) if pmc.get("SQ_ACTIVE_INST_VALU") else None
        issue = (f64 * ISSUE_CYC["f64"] + tr64 * ISSUE_CYC["trans_f64"] + tr32 * ISSUE_CYC["trans_f32"] +
                 other * ISSUE_CYC["other"]) / n
        flops = (pmc.get("SQ_INSTS_VALU_ADD_F64", 0) + pmc.get("SQ_INSTS_VALU_MUL_F64", 0) +
                 2 * pmc.get("SQ_INSTS_VALU_FMA_F64", 0)) * 64 * (lane or 1) / n
        r["valu"] = {"f64_flops_per_launch": flops, "f64_tflops": flops / sec / 1e12, "f64_peak_tflops": F64_PEAK_TFLOPS,
                     "issue_frac": issue / (SIMDS * CLOCK_HZ * sec), "lane_utilisation": lane,
                     "valu_insts_per_launch": pmc.get("SQ_INSTS_VALU", 0) / n,
                     "note": "issue_frac: wave64 VALU issue cycles (f64 4, f32/int 2, transcendental 8/16) over "
                             "1024 SIMDs x 2.4 GHz x launch time -- the resource that binds a cache-resident scene"}
        r["pmc_source"] = {"summary": src, "build_id": pmc_bid, "timed_build_id": build_id,
                           "same_build": pmc_bid is not None and pmc_bid == build_id}
        if not r["pmc_source"]["same_build"]:  # counters of another build than the one timed: flagged, not hidden
            r["pmc_build_mismatch"] = True
    if bound == "hbm" and "algorithmic" in r:
        r.update(unit="GB/s", peak=HBM_PEAK_GBS, achieved=r["algorithmic"]["GBs"], frac=r["algorithmic"]["frac_of_hbm"])
        # the BVH and triangles (16 MB for the dragon) are served from L2 / MALL: `frac` counts algorithmic
        # bytes, not HBM transfers; the physical traffic and the latency figures that bind sit beside it
        a = r["algorithmic"]
        r["frac_kind"] = "cache-served algorithmic bytes (SURVEY.md §8(d)), not physical HBM traffic"
        if per_sample and counts:
            visits = (counts.get("node_visits", 0) - counts.get("shadow_node_visits", 0)) if dom.startswith("k_extend") \
                else counts.get("shadow_node_visits", 0)
            a["node_visits_per_launch"] = visits * samples_per_frame / launches
            a["node_visits_per_us"] = a["node_visits_per_launch"] / (avg_ms * 1e3)
        binding = {"resource": "dependent-load latency (BVH node -> child -> triangle chains)"}
        if "traffic_frac" in r:
            binding["physical_hbm_frac"] = r["traffic_frac"]
        if "valu" in r:
            binding["valu_issue_frac"] = r["valu"]["issue_frac"]
            binding["lane_utilisation"] = r["valu"]["lane_utilisation"]
        r["binding"] = binding
    elif bound == "valu" and "valu" in r:
        r.update(unit="TFLOP/s", peak=F64_PEAK_TFLOPS, achieved=r["valu"]["f64_tflops"],
                 frac=r["valu"]["f64_tflops"] / F64_PEAK_TFLOPS)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=HEADLINE, choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle check of the frame's columns")
    ap.add_argument("--col-block", type=int, default=16)
    ap.add_argument("--events", action="store_true",
                    help="bracket the dominant kernel's launches in the timed steps with HIP events (serialises the "
                         "render onto one stream); by default the timed steps run the two-stream schedule without "
                         "events and one instrumented one-stream step follows them")
    ap.add_argument("--spp", type=int, default=0, help="profiling only: override the config's spp (same launch "
                    "shapes, fewer batches); a bench line with it is not the config's number")
    ap.add_argument("--gather", choices=["rgba8", "accum"], default="rgba8",
                    help="the multi-GPU exchange: packed RGBA8 tiles (4 B per pixel, the reference workers' ImageData), "
                         "or the f32 accumulators (16 B per pixel) finished by one k_final on rank 0 "
                         "(jsrt_render_device_accum, tiles.AccumGather); the image is the same bit for bit")
    ap.add_argument("--ab", action="store_true", help="allow JSRT_* environment knobs / JSRT_LIB variants (A/B runs; "
                    "the line records them under `knobs`)")
    args = ap.parse_args()
    if knobs() and not args.ab:
        print(f"bench: refusing to time with library knobs set {knobs()} (A/B only: pass --ab)", file=sys.stderr)
        sys.exit(2)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    rank, world, local = env_int("RANK", 0), env_int("WORLD_SIZE", 1), env_int("LOCAL_RANK", 0)
    if world != args.gpus:
        print(f"bench: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)
    import numpy as np
    import torch
    import torch.distributed as dist

    # JSRT_BENCH_BACKEND=gloo rehearses the N > 1 path on fewer GPUs than ranks (ranks share devices
    # round-robin, tiles are gathered through host memory); the bench proper uses nccl = RCCL over xGMI
    backend = os.environ.get("JSRT_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    import jsraytracer_amd as jr
    from jsraytracer_amd.tiles import AccumGather, FrameGather
    from oracle import pyoracle  # fixture loader only; the oracle runs only in the cpu_baseline / parity legs

    scene_name, W, H, spp, kind, depth, bound = CONFIGS[args.config]
    if args.spp > 0:
        spp = args.spp
    t_load = time.perf_counter()
    if scene_name in MESH_SCENES:
        blob, _ = pyoracle.mesh_scene(scene_name, jr)  # skeleton + OBJ through the native ingest
    else:
        blob = pyoracle.golden_scene(scene_name)
    t_build = time.perf_counter() - t_load
    scene = jr.Scene(blob, device=local)
    t_upload = time.perf_counter() - t_load - t_build

    cb = args.col_block if world > 1 else 1
    host_tiles = world > 1 and backend != "nccl"
    fg = FrameGather(W, H, rank, world, cb, device="cpu" if host_tiles else f"cuda:{local}")
    tile = torch.zeros_like(fg.local, device=f"cuda:{local}") if host_tiles else fg.local
    stream = torch.cuda.current_stream().cuda_stream
    STAGES = jr._native.STAGES
    ONE = jr._native.EVENTS_ONE_STREAM  # instrumented steps: every stage's own launch times (one stream)

    accum = args.gather == "accum"
    if accum:  # the accumulator exchange: f32 tiles gathered to rank 0, finished there by one k_final
        ag = AccumGather(W, H, rank, world, cb, device="cpu" if host_tiles else f"cuda:{local}")
        atile = torch.zeros_like(ag.local, device=f"cuda:{local}") if host_tiles else ag.local

    def step(events=None, colors=None):
        """events: None = no HIP events; 0 = every stage; else a bitmask of stages (jsrt.h stage_events)."""
        kw = dict(stream_ptr=stream, col_block=cb, width=W, height=H, spp=spp, max_depth=depth, kind=kind, seed=1,
                  x_offset=rank if world > 1 else 0, x_delt=world, stats=events is not None, stage_events=events or 0)
        if accum:
            st = scene.render_device_accum(atile.data_ptr(), **kw)
            if host_tiles:
                ag.local.copy_(atile.cpu())
            acc = ag.gather()
            if rank == 0:
                fg.image.copy_(AccumGather.finish(acc.to(f"cuda:{local}"), kind, spp).to(fg.image.device))
            return st
        st = scene.render_device(tile.data_ptr(), colors.data_ptr() if colors is not None else None, **kw)
        if host_tiles:
            fg.local.copy_(tile.cpu())
        fg.gather()
        return st

    # warmup; the last warmup step is fully instrumented and names the dominant kernel
    st_full = None
    for w in range(max(args.warmup, 1)):
        st_full = step(ONE if w == max(args.warmup, 1) - 1 else None)
    dom = max(st_full["stage_ms"], key=lambda k: st_full["stage_ms"][k])
    # timed region: HIP events bracket only the dominant kernel's launches (its average launch
    # duration for the roofline); events on every launch would add launch gaps to the step.  The last
    # timed step also writes the f32 colours handed to setColor (k_final, 16 B per pixel): the parity
    # block checks that frame itself.
    colors = torch.empty(fg.maxcols * H * 4, dtype=torch.float32, device=f"cuda:{local}") \
        if world == 1 and not accum else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = [step(((1 << STAGES.index(dom)) | ONE) if args.events else None, colors if k == args.steps - 1 else None)
             for k in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timed_image = FrameGather.to_rgba8(fg.image).copy() if rank == 0 else None  # the last timed frame
    timed_cols = colors.view(fg.maxcols, H, 4)[:W].permute(1, 0, 2).cpu().numpy() if colors is not None else None
    tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if host_tiles else f"cuda:{local}")
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())
    if not args.events:  # the dominant kernel's launches, timed on the one-stream schedule
        stats = [step((1 << STAGES.index(dom)) | ONE)]
    dom_ms = sum(s["stage_ms"][dom] for s in stats) / len(stats)
    dom_launches = stats[0]["stage_launches"][dom]
    # per-stage split: one more step after the timed region with every launch bracketed
    st_after = step(ONE)
    stage_ms, stage_launches, kernel_ms = st_after["stage_ms"], st_after["stage_launches"], st_after["kernel_ms"]
    torch.cuda.synchronize()

    par = None
    if rank == 0:
        total = W * H * spp
        value = total * args.steps / elapsed
        cpu, counts, ref = None, None, None
        if not args.no_cpu_baseline and world == 1:
            cpu, counts, ref = cpu_baseline(blob, W, H, spp, kind, depth)
            js, js_sample = REFERENCE_JS.get(scene_name, (None, None))
            if js:
                cpu["reference_js"] = {"value": js, "unit": "pixel-samples/s", "cores": 8, "kind": "reference",
                                       "sample": f"reference src/ under node 12, 8 worker_threads, {js_sample}; "
                                                 "measured in the build container (BASELINE.md §2) -- the "
                                                 "reference is absent on the GPU box"}
        par = None
        if not args.no_parity:
            if ref is None:  # a few columns spread over the ranks' tiles (multi-GPU: checks the gather too)
                threads = min(16, os.cpu_count() or 1)
                dx = W // 4 + 17
                ocol, orgba, _, _ = oracle_columns(blob, W, H, spp, kind, depth, 5, dx, threads)
                ref = (ocol, orgba, 5, dx)
            # the last timed frame (world 1, col_block 1: owned column c is image column c)
            par = parity(timed_image, timed_cols, ref)
            par["frame"] = "last timed step"
        roof = roofline(args.config, bound, dom, dom_ms / max(dom_launches, 1), dom_launches, counts, fg.ncols * H * spp,
                        jr._native.build_id())
        size = f"{W}²" if W == H else f"{W}x{H}"
        line = {
            "metric": METRIC.format(scene=scene_name, size=size),
            "value": value, "unit": "pixel-samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64",
            "data": "reference scene graph (exported from the live reference, not synthetic), keyed RNG seed 1",
            "config": {"workload": f"{scene_name} {W}x{H} {spp}spp depth {depth} (Incremental)", "width": W,
                       "height": H, "spp": spp, "max_depth": depth, "parallelism": f"tiles{world}",
                       "col_block": cb, "headline": args.config == HEADLINE and args.spp == 0,
                       "gather_backend": backend if world > 1 else None, "gather": args.gather},
            "roofline": roof, "cpu_baseline": cpu, "parity": par,
            "build_id": jr._native.build_id(), "knobs": knobs(),
            "kernel_ms_per_step": kernel_ms,
            "scene_build_s": round(t_build, 3), "scene_upload_s": round(t_upload, 3),
            "events_lost": {"timed": sum(x["events_lost"] for x in stats), "stage_split": st_after["events_lost"]},
            "frame_attempts": [x["attempts"] for x in stats],
            "stages_note": "stage split from one fully-instrumented step after the timed region, run on one "
                           "stream so each launch's time is its own (the timed steps overlap two batch streams)",
            "stages_ms_per_step": {k: round(v, 3) for k, v in stage_ms.items() if v},
            "stage_launches_per_step": {k: v for k, v in stage_launches.items() if v},
            "counts_per_sample": {k: round(v, 4) for k, v in counts.items() if k != "samples"} if counts else None,
        }
        print(json.dumps(line))
        sys.stdout.flush()
    if world > 1:
        dist.destroy_process_group()
    return exit_status(par)


if __name__ == "__main__":
    sys.exit(main())
