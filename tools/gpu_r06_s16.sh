#!/bin/bash
# round 6 s16: GPU suite with the Menger cross union (sdf_cross) and the table powers of toPrecision(8); then, on
# SDF_Menger, the default against the reciprocal parse (rcp) and against the generic union (nox = JSRT_SDF_CROSS=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s16.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s16.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh SDF_Menger 8 3 def= rcp=@tp8rcp nox=JSRT_SDF_CROSS=0 2>&1 | tail -3 | tee gpurun_out/ab_r06_s16_menger.txt || exit 1
