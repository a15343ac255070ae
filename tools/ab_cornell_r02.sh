#!/bin/bash
# A/B on the headline config: stage ablations (where k_shadow / k_shade time goes) + per-object cull counts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 bash tools/ab_bench.sh cornell_box_path "$@" || exit $?
JSRT_LIB=$PWD/jsraytracer_amd/_build/libjsrt_dbg.so timeout -k 10 120 python tools/dbg_counts.py cornell_box_path 512 512 16 8
