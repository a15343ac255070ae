#!/bin/bash
# round 6 s20: lower keep thresholds of the persistent SDF march (SDF_Menger)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_interleave.sh SDF_Menger 8 2 k48=@k48 k40=@k40 k32=@k32 k24=@k24 k40s16=@k40s16 2>&1 | tail -5 | tee gpurun_out/ab_r06_s20_menger.txt || exit 1
