set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r05_s24.log 2>&1; rc=$?
tail -12 gpurun_out/gpu_tests_r05_s24.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r05_s24.log 2>&1; rc=$?; tail -3 gpurun_out/smoke_r05_s24.log; exit $rc
