#!/bin/bash
# GPU-box: the -m gpu suite, the headline bench line + its rocprofv3 kernel summary (tools/gpu_check.sh), then the
# FETCH_SIZE / WRITE_SIZE calibration (tools/gpu_calib.sh).   bash tools/gpu_round.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-cur}
bash tools/gpu_check.sh $TAG || exit $?
bash tools/gpu_calib.sh $TAG || exit $?
