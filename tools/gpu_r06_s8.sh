#!/bin/bash
# round 6 s8: GPU suite (fused exact dot3), cornell stage times, the dragon at 64 / 128 / 256 samples per batch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s8.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s8.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh cornell_box_path 8 2 dot3= 2>&1 | tail -1 | tee gpurun_out/ab_r06_s8_cornell.txt || exit 1
bash tools/ab_interleave.sh dragon 1 2 spb64=JSRT_BATCH_SPP=64 spb128=JSRT_BATCH_SPP=128 spb256=JSRT_BATCH_SPP=256 2>&1 | tail -3 | tee gpurun_out/ab_r06_s8_dragon.txt || exit 1
bash tools/ab_interleave.sh bunny 8 1 dot3= 2>&1 | tail -1 | tee gpurun_out/ab_r06_s8_bunny.txt || exit 1
bash tools/ab_interleave.sh SDF_Menger 4 1 dot3= 2>&1 | tail -1 | tee gpurun_out/ab_r06_s8_menger.txt || exit 1
