#!/bin/bash
# round 6 s29: batch size (JSRT_MAX_PATHS) on cornell (16 M: four batches of 16 samples) and the dragon (64 M paths)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_interleave.sh cornell_box_path 8 3 def= m16=JSRT_MAX_PATHS=16777216 2>&1 | tail -2 | tee gpurun_out/ab_r06_s29_cornell.txt || exit 1
bash tools/ab_interleave.sh dragon 1 2 def= m64=JSRT_MAX_PATHS=67108864 2>&1 | tail -2 | tee gpurun_out/ab_r06_s29_dragon.txt || exit 1
