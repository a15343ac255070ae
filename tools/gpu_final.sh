#!/bin/bash
# GPU-box: the measurement set of one build, in two calls (each fits gpurun's 20-minute limit).
#   bash tools/gpu_final.sh TAG pmc      -m gpu suite, then the six PMC passes of every config (gpu_pmc_all.sh),
#                                        merged into profiles/pmc_summary.json stamped with the build id
#   bash tools/gpu_final.sh TAG configs  bench line + stamped rocprofv3 kernel summary per config
#                                        (gpu_configs.sh), reading the PMC summary of the same build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; MODE=$2; shift 2
CFGS=${*:-cornell_box_path bunny SDF_Menger dragon}
case $MODE in
  pmc)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
    tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_pmc_all.sh $TAG $CFGS || exit $?
    ;;
  configs)
    bash tools/gpu_configs.sh $TAG $CFGS || exit $?
    ;;
  *) echo "mode: pmc | configs"; exit 2 ;;
esac
