#!/bin/bash
# round 6 s13: GPU suite with the SDF sponge form's early exit, then its A/B on SDF_Menger (x0 = JSRT_SDF_EXIT=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s13.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s13.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh SDF_Menger 8 2 x0=JSRT_SDF_EXIT=0 x1= 2>&1 | tail -2 | tee gpurun_out/ab_r06_s13_menger.txt || exit 1
