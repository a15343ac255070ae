#!/bin/bash
# round 6 s18: GPU suite with the Menger form's four materialData distances evaluated together (sdf_form_normal4)
# and getMaterialData's choice from them; then SDF_Menger default against JSRT_SDF_N4=0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s18.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s18.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh SDF_Menger 8 3 n4= old=JSRT_SDF_N4=0 2>&1 | tail -2 | tee gpurun_out/ab_r06_s18_menger.txt || exit 1
