#!/bin/bash
# GPU-box: parity tests of one file set + A/B of library variants on one config.
#   bash tools/gpu_quick.sh CFG "pytest selection" VARIANT...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=$1; SEL=$2; shift 2
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
  tail -3 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 bash tools/ab_bench.sh $CFG "$@" || exit $?
