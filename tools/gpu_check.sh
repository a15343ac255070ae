#!/bin/bash
# GPU-box round check: parity tests, headline bench (with CPU baseline), rocprofv3 kernel-trace summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-cur}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline --events > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err || exit $?
python tools/stamp_stats.py gpurun_out/bench_prof_$TAG.json gpurun_out/prof_$TAG/run_kernel_stats.csv cornell_box_path || exit 1
cat gpurun_out/prof_$TAG/run_kernel_stats.csv
