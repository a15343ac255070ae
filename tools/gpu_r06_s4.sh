#!/bin/bash
# round 6 s4: (1) cornell memory-latency counters per kernel, (2) the dragon's per-share stage split (N = 1, 8),
# (3) bunny: the round-4 build (worktree ab_wt_r4, commit 6671744) against this tree, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r06_s4
timeout -s KILL 180 rocprofv3 --pmc SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES \
  --kernel-trace --output-format csv -d gpurun_out/pmc_r06_s4/lat -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity --ab > gpurun_out/pmc_r06_s4/lat.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_r06_s4/lat.log; exit 1; }
echo pmc ok
timeout -k 10 300 python tools/project_scaling.py --config dragon --ranks 1,8 --steps 1 --stages --only-rank0 --out gpurun_out/proj_r06_s4_dragon.json 2>&1 | tee gpurun_out/proj_r06_s4_dragon.txt || exit 1
for rep in 1 2 3; do
  for v in r4 head; do
    if [ $v = r4 ]; then d=ab_wt_r4; else d=.; fi
    ( cd $d && timeout -k 10 300 python bench.py --config bunny --steps 8 --warmup 1 --no-cpu-baseline --ab > $GRAFT_REPO_ROOT/gpurun_out/bunny_${v}_$rep.json 2> $GRAFT_REPO_ROOT/gpurun_out/bunny_${v}_$rep.err ) || { echo "bunny $v failed"; tail -3 gpurun_out/bunny_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/bunny_${v}_$rep.json')); print('$v', $rep, round(d['value']/1e6,1), d.get('parity',{}).get('pass'), {k: v for k, v in d.get('stages_ms_per_step', {}).items() if v > 0.05})"
  done
done
