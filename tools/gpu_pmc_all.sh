#!/bin/bash
# GPU-box: PMC passes (tools/pmc.sh) for cornell (full frame) and dragon (spp 16: same launch shapes,
# fewer batches), raw csv removed so only the summaries travel back.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-cur}
bash tools/pmc.sh cornell_box_path "" ${TAG}_cornell > gpurun_out/pmc_${TAG}_cornell.log 2>&1 || { tail -20 gpurun_out/pmc_${TAG}_cornell.log; exit 1; }
rm -rf gpurun_out/pmc_${TAG}_cornell/p?
PMC_BENCH_ARGS="--spp 16" bash tools/pmc.sh dragon "" ${TAG}_dragon > gpurun_out/pmc_${TAG}_dragon.log 2>&1 || { tail -20 gpurun_out/pmc_${TAG}_dragon.log; exit 1; }
rm -rf gpurun_out/pmc_${TAG}_dragon/p?
grep -c "==" gpurun_out/pmc_${TAG}_cornell/summary.txt gpurun_out/pmc_${TAG}_dragon/summary.txt
