#!/bin/bash
# GPU-box: parity tests, then bench lines (no CPU baseline) for the configs given.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for CFG in "$@"; do
  timeout -k 10 600 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/q_${TAG}_$CFG.json 2> gpurun_out/q_${TAG}_$CFG.err || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/q_${TAG}_$CFG.json').read().strip().splitlines()[-1]); print('$CFG', round(d['value']/1e6,1), 'Ms/s', round(d['ms_per_step'],1), 'ms', d['stages_ms_per_step'])"
done
