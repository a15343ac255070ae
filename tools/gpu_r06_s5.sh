#!/bin/bash
# round 6 s5: (1) cornell batch shape: one 64 M-path batch on one stream vs the default two halves on two streams,
# and k_shadow at 8 waves (libjsrt_so8), interleaved; (2) the dragon's N = 8 shares at column blocks 16 / 128 / 512
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_interleave.sh cornell_box_path 8 3 base= one=JSRT_MAX_PATHS=67108864,JSRT_SPLIT_FRAME=0 so8=@so8 2>&1 | tee gpurun_out/ab_r06_s5.txt || exit 1
for cb in 16 128 512; do
  timeout -k 10 300 python tools/project_scaling.py --config dragon --ranks 8 --steps 1 --col-block $cb --out gpurun_out/proj_r06_s5_dragon_cb$cb.json > gpurun_out/proj_r06_s5_dragon_cb$cb.txt 2>&1 || { echo "proj cb $cb failed"; tail -5 gpurun_out/proj_r06_s5_dragon_cb$cb.txt; exit 1; }
  tail -1 gpurun_out/proj_r06_s5_dragon_cb$cb.txt
done
