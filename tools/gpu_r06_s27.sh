#!/bin/bash
# round 6 s27: the mesh k_shade's occupancy (4 waves default; 3, 5) on bunny and the dragon
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_interleave.sh bunny 8 2 def= m3=@m3 m5=@m5 2>&1 | tail -3 | tee gpurun_out/ab_r06_s27_bunny.txt || exit 1
bash tools/ab_interleave.sh dragon 1 2 def= m3=@m3 m5=@m5 2>&1 | tail -3 | tee gpurun_out/ab_r06_s27_dragon.txt || exit 1
