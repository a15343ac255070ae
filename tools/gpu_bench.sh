#!/bin/bash
# GPU-box helper: bench line + rocprofv3 kernel-trace summary of the same command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFG=${1:-cornell_box_path}
STEPS=${2:-3}
timeout -k 10 900 python bench.py --config "$CFG" --steps "$STEPS" --warmup 1 > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err || exit $?
cat gpurun_out/bench_$CFG.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$CFG -o run -- \
    python bench.py --config "$CFG" --steps "$STEPS" --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$CFG.json 2> gpurun_out/prof_$CFG.err || exit $?
find gpurun_out/prof_$CFG -name "*stats*" | head
