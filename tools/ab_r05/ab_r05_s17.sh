set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1_tests.log 2>&1; rc=$?
tail -2 gpurun_out/ab1_tests.log; [ $rc -eq 0 ] || exit $rc
AB_BENCH_ARGS="--steps 8" timeout -k 10 600 bash tools/ab_bench.sh cornell_box_path old base sn old base sn > gpurun_out/ab1_cornell.txt 2>&1; rc=$?; cat gpurun_out/ab1_cornell.txt; [ $rc -eq 0 ] || exit $rc
AB_BENCH_ARGS="--steps 4" timeout -k 10 400 bash tools/ab_bench.sh bunny old base bf base bf > gpurun_out/ab1_bunny.txt 2>&1; rc=$?; cat gpurun_out/ab1_bunny.txt; [ $rc -eq 0 ] || exit $rc
AB_BENCH_ARGS="--steps 1" timeout -k 10 400 bash tools/ab_bench.sh dragon base bf > gpurun_out/ab1_dragon.txt 2>&1; rc=$?; cat gpurun_out/ab1_dragon.txt; exit $rc
