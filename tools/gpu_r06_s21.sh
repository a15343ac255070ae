#!/bin/bash
# round 6 s21: cornell occupancy of the flat k_extend (6 waves default; 5, 8) and k_shade (5 default; 4, 6)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_interleave.sh cornell_box_path 8 2 def= ex5=@ex5 ex8=@ex8 sh4=@sh4 sh6=@sh6 2>&1 | tail -5 | tee gpurun_out/ab_r06_s21_cornell.txt || exit 1
