#!/bin/bash
# round 6 s12: GPU suite (tile-ordered pixel-major batches), then the tile size A/B (0 = patch raster) on bunny, the
# dragon and SDF_Menger
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s12.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s12.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh bunny 8 2 t0=JSRT_TILE_PATCHES=0 t8= t16=JSRT_TILE_PATCHES=16 t32=JSRT_TILE_PATCHES=32 2>&1 | tail -4 | tee gpurun_out/ab_r06_s12_bunny.txt || exit 1
bash tools/ab_interleave.sh dragon 1 1 t0=JSRT_TILE_PATCHES=0 t4=JSRT_TILE_PATCHES=4 t8= t16=JSRT_TILE_PATCHES=16 2>&1 | tail -4 | tee gpurun_out/ab_r06_s12_dragon.txt || exit 1
bash tools/ab_interleave.sh SDF_Menger 4 2 t0=JSRT_TILE_PATCHES=0 t8= 2>&1 | tail -2 | tee gpurun_out/ab_r06_s12_menger.txt || exit 1
