#!/bin/bash
# round 6 s25: the SDF k_shade's occupancy after the four-distance normal (4 waves default; 5, 3), SDF_Menger
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_interleave.sh SDF_Menger 8 2 def= so5=@so5 so3=@so3 2>&1 | tail -3 | tee gpurun_out/ab_r06_s25_menger.txt || exit 1
