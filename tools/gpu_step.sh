#!/bin/bash
# GPU-box helper: the -m gpu suite, then (unless it faulted, aborted or timed out) A/B runs.
#   bash tools/gpu_step.sh TAG "CFG spec..." ["CFG spec..." ...]   (specs as tools/ab_env.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
  tail -4 gpurun_out/gpu_tests_$TAG.log
  case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
fi
for ab in "$@"; do
  bash tools/ab_env.sh $ab || exit $?
done
