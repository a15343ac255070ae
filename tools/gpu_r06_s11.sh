#!/bin/bash
# round 6 s11: GPU suite (leader-only bucket atomics in k_extend; the near-first BVH order reverted), stage times of
# cornell, bunny and the dragon on this build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s11.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s11.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh cornell_box_path 8 3 lead= 2>&1 | tail -1 | tee gpurun_out/ab_r06_s11_cornell.txt || exit 1
bash tools/ab_interleave.sh bunny 8 2 lead= 2>&1 | tail -1 | tee gpurun_out/ab_r06_s11_bunny.txt || exit 1
bash tools/ab_interleave.sh dragon 1 1 lead= 2>&1 | tail -1 | tee gpurun_out/ab_r06_s11_dragon.txt || exit 1
