#!/bin/bash
# round 6 s26: GPU suite with the SDF k_shade at 3 waves per SIMD, then 3 (default) against 2 on SDF_Menger
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s26.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s26.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh SDF_Menger 8 2 def= so2=@so2 2>&1 | tail -2 | tee gpurun_out/ab_r06_s26_menger.txt || exit 1
