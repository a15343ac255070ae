set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
JSRT_LIB=$PWD/jsraytracer_amd/_build/libjsrt_menger.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_material.py tests/test_gpu_fullsize.py tests/test_gpu_casts.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2_tests.log 2>&1; rc=$?
tail -2 gpurun_out/ab2_tests.log; [ $rc -eq 0 ] || exit $rc
AB_BENCH_ARGS="--steps 4" timeout -k 10 600 bash tools/ab_bench.sh SDF_Menger base menger base menger > gpurun_out/ab2_menger.txt 2>&1; rc=$?; cat gpurun_out/ab2_menger.txt; [ $rc -eq 0 ] || exit $rc
AB_BENCH_ARGS="--steps 8" timeout -k 10 400 bash tools/ab_bench.sh cornell_box_path base menger > gpurun_out/ab2_cornell.txt 2>&1; rc=$?; cat gpurun_out/ab2_cornell.txt; exit $rc
