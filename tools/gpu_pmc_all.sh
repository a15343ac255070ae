#!/bin/bash
# GPU-box: PMC passes (tools/pmc.sh) for every BASELINE config at its full size, raw csv removed so only
# the summaries travel back; each config is merged into gpurun_out/pmc_summary.json.
#   bash tools/gpu_pmc_all.sh TAG [CFG ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-cur}; shift
CFGS=${@:-cornell_box_path bunny SDF_Menger dragon}
cp profiles/pmc_summary.json gpurun_out/pmc_summary.json 2>/dev/null
for CFG in $CFGS; do
  timeout -k 10 900 bash tools/pmc.sh $CFG "" ${TAG}_$CFG > gpurun_out/pmc_${TAG}_$CFG.log 2>&1 || { tail -20 gpurun_out/pmc_${TAG}_$CFG.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc_${TAG}_$CFG --config $CFG --merge gpurun_out/pmc_summary.json > /dev/null
  rm -rf gpurun_out/pmc_${TAG}_$CFG/p?
  echo "$CFG: $(grep -c '==' gpurun_out/pmc_${TAG}_$CFG/summary.txt) kernels"
done
