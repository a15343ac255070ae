#!/bin/bash
# round 6 s9: bunny's split of a one-batch frame -- two pixel halves (every sample) vs two sample halves; the dragon's
# projected N = 1 / 2 / 4 / 8 shares with 256-sample pixel-major batches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_interleave.sh bunny 8 3 samples= pixels=JSRT_SPLIT_PIXELS=1 2>&1 | tail -2 | tee gpurun_out/ab_r06_s9_bunny.txt || exit 1
bash tools/ab_interleave.sh SDF_Menger 4 2 base= pixels=JSRT_SPLIT_PIXELS=1 2>&1 | tail -2 | tee gpurun_out/ab_r06_s9_menger.txt || exit 1
timeout -k 10 600 python tools/project_scaling.py --config dragon --ranks 1,2,4,8 --steps 1 --out gpurun_out/proj_r06_s9_dragon.json > gpurun_out/proj_r06_s9_dragon.txt 2>&1 || { tail -5 gpurun_out/proj_r06_s9_dragon.txt; exit 1; }
grep '^{' gpurun_out/proj_r06_s9_dragon.txt
timeout -k 10 300 python tools/project_scaling.py --config cornell_box_path --ranks 1,2,4,8 --steps 3 --out gpurun_out/proj_r06_s9_cornell.json > gpurun_out/proj_r06_s9_cornell.txt 2>&1 || { tail -5 gpurun_out/proj_r06_s9_cornell.txt; exit 1; }
grep '^{' gpurun_out/proj_r06_s9_cornell.txt
