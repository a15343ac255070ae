set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_BENCH_ARGS="--steps 8" timeout -k 10 700 bash tools/ab_bench.sh cornell_box_path base so8 sh6 base so8 sh6 > gpurun_out/ab6_cornell.txt 2>&1; rc=$?; cat gpurun_out/ab6_cornell.txt; exit $rc
