#!/bin/bash
# round 6 s22: projected N = 1 / 2 / 4 / 8 shares of every config on the shipped build (each rank's share rendered
# alone on one MI355X; the gather is not included)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in dragon:1 cornell_box_path:3 bunny:3 SDF_Menger:2; do
  cfg=${c%%:*}; st=${c##*:}
  timeout -k 10 600 python tools/project_scaling.py --config $cfg --ranks 1,2,4,8 --steps $st --out gpurun_out/proj_r06_s22_$cfg.json > gpurun_out/proj_r06_s22_$cfg.txt 2>&1 || { tail -5 gpurun_out/proj_r06_s22_$cfg.txt; exit 1; }
  grep '^{' gpurun_out/proj_r06_s22_$cfg.txt | cut -c1-400
done
