#!/bin/bash
# GPU-box helper: bench line (with CPU baseline) + rocprofv3 kernel-trace summary per config.
#   bash tools/gpu_configs.sh TAG CFG [CFG ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for CFG in "$@"; do
  timeout -k 10 600 python bench.py --config "$CFG" --steps 3 --warmup 1 > gpurun_out/bench_${TAG}_$CFG.json 2> gpurun_out/bench_${TAG}_$CFG.err || exit $?
  cat gpurun_out/bench_${TAG}_$CFG.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$CFG -o run -- \
      python bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --events > gpurun_out/bench_prof_${TAG}_$CFG.json 2> gpurun_out/prof_${TAG}_$CFG.err || exit $?
  python tools/stamp_stats.py gpurun_out/bench_prof_${TAG}_$CFG.json gpurun_out/prof_${TAG}_$CFG/run_kernel_stats.csv $CFG || exit 1
  head -4 gpurun_out/prof_${TAG}_$CFG/run_kernel_stats.csv
done
