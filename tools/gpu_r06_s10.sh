#!/bin/bash
# round 6 s10: GPU suite (near-child-first shadow BVH walks, pixel-halves split), then the near-first A/B on bunny
# and the dragon (JSRT_BVH_NEAR=0: the reference's greater-first order for the shadow casts too)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s10.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s10.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh bunny 8 3 gf=JSRT_BVH_NEAR=0 near= 2>&1 | tail -2 | tee gpurun_out/ab_r06_s10_bunny.txt || exit 1
bash tools/ab_interleave.sh dragon 1 2 gf=JSRT_BVH_NEAR=0 near= 2>&1 | tail -2 | tee gpurun_out/ab_r06_s10_dragon.txt || exit 1
