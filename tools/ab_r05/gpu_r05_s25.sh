set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/project_scaling.py --config cornell_box_path --steps 3 --out gpurun_out/proj_r05_s25_cornell.json > gpurun_out/proj_r05_s25_cornell.txt 2>&1 || exit $?
cat gpurun_out/proj_r05_s25_cornell.txt
timeout -k 10 500 python tools/project_scaling.py --config dragon --steps 1 --out gpurun_out/proj_r05_s25_dragon.json > gpurun_out/proj_r05_s25_dragon.txt 2>&1 || exit $?
cat gpurun_out/proj_r05_s25_dragon.txt
