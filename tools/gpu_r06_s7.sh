#!/bin/bash
# round 6 s7: GPU suite; the dragon's samples per pixel-major batch (8 / 16 / 32 / 64); SDF_Menger in either order
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s7.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s7.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh dragon 1 2 spb8=JSRT_BATCH_SPP=8 spb16= spb32=JSRT_BATCH_SPP=32 spb64=JSRT_BATCH_SPP=64 2>&1 | tail -4 | tee gpurun_out/ab_r06_s7_dragon.txt || exit 1
bash tools/ab_interleave.sh SDF_Menger 4 3 pm0=JSRT_PIXEL_MAJOR=0 pm1= 2>&1 | tail -2 | tee gpurun_out/ab_r06_s7_menger.txt || exit 1
bash tools/ab_interleave.sh bunny 8 2 spb16= spb8=JSRT_BATCH_SPP=8 2>&1 | tail -2 | tee gpurun_out/ab_r06_s7_bunny.txt || exit 1
# mesh occupancy under the pixel-major order: k_extend at 6 / 4 waves, k_shadow at 5 (libjsrt_ext6 / ext4 / msh5)
bash tools/ab_interleave.sh bunny 8 2 base= ext6=@ext6 ext4=@ext4 msh5=@msh5 2>&1 | tail -4 | tee gpurun_out/ab_r06_s7_bunny_occ.txt || exit 1
bash tools/ab_interleave.sh dragon 1 1 base= ext6=@ext6 ext4=@ext4 msh5=@msh5 2>&1 | tail -4 | tee gpurun_out/ab_r06_s7_dragon_occ.txt || exit 1
