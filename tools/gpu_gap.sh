#!/bin/bash
# GPU-box probe: wall time vs kernel time of a config (events / no events) + kernel trace for gap analysis.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${1:-dragon}; SPP=${2:-16}; TAG=${3:-gap}
timeout -k 10 300 python bench.py --config $CFG --spp $SPP --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_ev.json 2>&1 || exit $?
timeout -k 10 300 python bench.py --config $CFG --spp $SPP --steps 2 --warmup 1 --no-cpu-baseline --no-events > gpurun_out/${TAG}_noev.json 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trace -o run -- python bench.py --config $CFG --spp $SPP --steps 1 --warmup 0 --no-cpu-baseline --no-events > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
python - <<'PY'
import json
for t in ("ev", "noev"):
    d = json.loads(open(f"gpurun_out/${TAG}_{t}.json").read().strip().splitlines()[-1])
    print(t, "ms/step", round(d["ms_per_step"], 1), "kernel ms", round(d["kernel_ms_per_step"], 1))
PY
