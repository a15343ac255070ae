#!/bin/bash
# GPU-box: parity tests, then the dragon config (BASELINE.json configs[4]) bench + rocprofv3 summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-cur}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --config dragon --steps 2 --warmup 1 > gpurun_out/bench_${TAG}_dragon.json 2> gpurun_out/bench_${TAG}_dragon.err || exit $?
cat gpurun_out/bench_${TAG}_dragon.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_dragon -o run -- \
    python bench.py --config dragon --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_${TAG}_dragon.json 2> gpurun_out/prof_${TAG}_dragon.err || exit $?
rm -f gpurun_out/prof_${TAG}_dragon/run_kernel_trace.csv
head -6 gpurun_out/prof_${TAG}_dragon/run_kernel_stats.csv
