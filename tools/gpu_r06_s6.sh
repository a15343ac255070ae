#!/bin/bash
# round 6 s6: GPU suite (both path orders), then the pixel-major path order A/B: cornell and bunny interleaved,
# the dragon's full frame, and its N = 8 shares (col_block 16) projected
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s6.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s6.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh cornell_box_path 8 3 pm0=JSRT_PIXEL_MAJOR=0 pm1=JSRT_PIXEL_MAJOR=1 2>&1 | tail -2 | tee gpurun_out/ab_r06_s6_cornell.txt || exit 1
bash tools/ab_interleave.sh bunny 8 3 pm0=JSRT_PIXEL_MAJOR=0 pm1=JSRT_PIXEL_MAJOR=1 2>&1 | tail -2 | tee gpurun_out/ab_r06_s6_bunny.txt || exit 1
bash tools/ab_interleave.sh dragon 1 2 pm0=JSRT_PIXEL_MAJOR=0 pm1=JSRT_PIXEL_MAJOR=1 2>&1 | tail -2 | tee gpurun_out/ab_r06_s6_dragon.txt || exit 1
JSRT_PIXEL_MAJOR=1 timeout -k 10 300 python tools/project_scaling.py --config dragon --ranks 8 --steps 1 --col-block 16 --out gpurun_out/proj_r06_s6_dragon_pm1.json > gpurun_out/proj_r06_s6_dragon_pm1.txt 2>&1 || exit 1
tail -1 gpurun_out/proj_r06_s6_dragon_pm1.txt
