#!/bin/bash
# round 6 s3: GPU suite with the world-ray filters, then their interleaved A/B on cornell (JSRT_WORLD_FILTERS=0: off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s3.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s3.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh cornell_box_path 8 3 nowf=JSRT_WORLD_FILTERS=0 wf= 2>&1 | tee gpurun_out/ab_r06_s3.txt || exit 1
