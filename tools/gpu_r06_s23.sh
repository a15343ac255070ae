#!/bin/bash
# round 6 s23: small shares (rank 0 of N = 8) in more, smaller batches (JSRT_MAX_PATHS) so the two batch streams
# overlap their level launches: cornell, SDF_Menger, bunny
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # tag cfg steps [env]
  local tag=$1 cfg=$2 st=$3; shift 3
  env "$@" timeout -k 10 300 python tools/project_scaling.py --config $cfg --ranks 1,8 --only-rank0 --steps $st --out gpurun_out/proj_r06_s23_${cfg}_$tag.json > gpurun_out/proj_r06_s23_${cfg}_$tag.txt 2>&1 || { tail -5 gpurun_out/proj_r06_s23_${cfg}_$tag.txt; exit 1; }
  echo "$cfg $tag $(grep '^{' gpurun_out/proj_r06_s23_${cfg}_$tag.txt | cut -c1-120 | tr '\n' ' ')"
}
run def cornell_box_path 3 X=1
run m2 cornell_box_path 3 JSRT_MAX_PATHS=2097152
run m1 cornell_box_path 3 JSRT_MAX_PATHS=1048576
run def SDF_Menger 2 X=1
run m2 SDF_Menger 2 JSRT_MAX_PATHS=2097152
run m1 SDF_Menger 2 JSRT_MAX_PATHS=1048576
run def bunny 3 X=1
run m5 bunny 3 JSRT_MAX_PATHS=524288
