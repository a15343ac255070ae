"""bench.py's N > 1 path end to end on the GPU box: `bench.py --gpus 2` spawns its two rank processes
before anything touches a GPU (one process per GPU, as src/raytrace_launcher.js:65-101 spawns one worker
per slot), each renders its 16-column blocks of the frame with the HIP kernels, the tiles are gathered
to rank 0 and permuted into image order, and rank 0 checks the gathered frame's columns against the
oracle.  JSRT_BENCH_BACKEND=gloo lets both ranks share the box's one GPU (tiles gathered through host
memory); the nccl (RCCL over xGMI) branch runs on the driver's 8-GPU node."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_two_ranks_gloo_gather_parity():
    env = dict(os.environ, JSRT_BENCH_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=380, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints the one bench line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "tiles2" and d["config"]["gather_backend"] == "gloo"
    assert d["config"]["headline"] and d["value"] > 0 and d["steps"] == 1
    par = d["parity"]
    # the checked columns land on both ranks' tiles (16-column blocks dealt round-robin)
    cols = range(5, 1024, par["column_stride"])
    assert {(c // 16) % 2 for c in cols} == {0, 1}
    assert par["pass"] and par["rgba8_pixels_differing"] == 0, par
