#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config dragon --spp 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/probe2_dragon.json 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/probe2_dragon.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'], d['events_lost'], d['roofline']['avg_launch_ms'])"
PMC_BENCH_ARGS="--spp 16" bash tools/pmc.sh dragon "" dragon_s16 > gpurun_out/pmc_dragon.log 2>&1 || { tail -20 gpurun_out/pmc_dragon.log; exit 1; }
rm -rf gpurun_out/pmc_dragon_s16/p?
grep -A 45 "k_extend" gpurun_out/pmc_dragon_s16/summary.txt | head -46
