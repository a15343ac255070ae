#!/bin/bash
# round 6 s19: the persistent SDF march's refill knobs on SDF_Menger after the cheaper evaluation:
# default (8 steps while >= 56 lanes march, 1 wave/SIMD bound) against keep 48 / 60, 16 steps, 2 waves/SIMD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_interleave.sh SDF_Menger 8 2 def= k48=@k48 k60=@k60 s16=@s16 oc2=@oc2 2>&1 | tail -5 | tee gpurun_out/ab_r06_s19_menger.txt || exit 1
