#!/bin/bash
# round 6 s15: the toPrecision(8) power from a constant table (tab) against the formed power (default), SDF_Menger
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_casts.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "Menger or SDF or menger" > gpurun_out/gpu_tests_r06_s15.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s15.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh SDF_Menger 8 3 def= tab=@tp8tab 2>&1 | tail -2 | tee gpurun_out/ab_r06_s15_menger.txt || exit 1
