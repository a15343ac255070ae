set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_final.sh r05_s21 configs || exit $?
bash tools/ab_r05/ab_r05_s20.sh
