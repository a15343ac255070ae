set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_BENCH_ARGS="--steps 4" timeout -k 10 500 bash tools/ab_bench.sh bunny wtbase ncf wtbase ncf wtbase ncf > gpurun_out/ab5_bunny.txt 2>&1; rc=$?; cat gpurun_out/ab5_bunny.txt; [ $rc -eq 0 ] || exit $rc
AB_BENCH_ARGS="--steps 1" timeout -k 10 500 bash tools/ab_bench.sh dragon wtbase ncf > gpurun_out/ab5_dragon.txt 2>&1; rc=$?; cat gpurun_out/ab5_dragon.txt; exit $rc
