#!/bin/bash
# GPU-box: FETCH_SIZE / WRITE_SIZE calibration of the renderer's access shapes (tools/fetch_calib.hip, built in
# the container), one rocprofv3 --pmc pass per counter; ratios by tools/fetch_calib.py.
#   bash tools/gpu_calib.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-calib}
D=gpurun_out/fetch_calib_$TAG
mkdir -p $D
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/fetch -o run -- tools/fetch_calib > $D/known.json 2> $D/fetch.err || { echo "fetch pass failed"; tail -5 $D/fetch.err; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/write -o run -- tools/fetch_calib > $D/known2.json 2> $D/write.err || { echo "write pass failed"; tail -5 $D/write.err; exit 1; }
python tools/fetch_calib.py $D/fetch $D/write $D/known.json | tee $D/ratios.json
