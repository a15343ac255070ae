#!/bin/bash
# round 6 s14: GPU suite with the one-division toPrecision(8) parse, then its A/B on SDF_Menger (old = round 5's parse)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s14.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s14.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh SDF_Menger 8 3 old=@tp8old new= 2>&1 | tail -2 | tee gpurun_out/ab_r06_s14_menger.txt || exit 1
