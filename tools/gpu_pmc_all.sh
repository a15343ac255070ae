#!/bin/bash
# GPU-box: the six PMC passes (tools/pmc.sh) for every BASELINE config with the current library, merged
# into profiles/pmc_summary.json on the box (which bench.py reads for its roofline block) and copied to
# gpurun_out/ so the same summary can be committed.   bash tools/gpu_pmc_all.sh TAG [CFG ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
CFGS=${*:-cornell_box_path bunny SDF_Menger dragon}
for CFG in $CFGS; do
  timeout -k 10 900 bash tools/pmc.sh $CFG '' ${TAG}_$CFG > gpurun_out/pmc_${TAG}_$CFG.log 2>&1 || { echo "pmc $CFG failed"; tail -5 gpurun_out/pmc_${TAG}_$CFG.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc_${TAG}_$CFG --config $CFG --merge profiles/pmc_summary.json > /dev/null || exit 1
  rm -rf gpurun_out/pmc_${TAG}_$CFG/p[0-9]*  # the raw per-dispatch csvs (tens of MB): the summaries stay
  echo "pmc $CFG done"
done
cp profiles/pmc_summary.json gpurun_out/pmc_summary_${TAG}.json
