#!/bin/bash
# A/B: bench one config under several environment settings (NAME=VAR=VALUE[,VAR=VALUE]), no CPU baseline.
#   bash tools/ab_env.sh CFG base= nofuse=JSRT_FUSED=0 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CFG=$1; shift
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  read -r -a extra <<< "${AB_BENCH_ARGS:-}"  # split on blanks before IFS changes below
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 600 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --ab "${extra[@]}" > gpurun_out/ab_${CFG}_$name.json 2> gpurun_out/ab_${CFG}_$name.err )
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc  # 3: the line was printed, parity failed (shown below)
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_${CFG}_$name.json')); p=d.get('parity') or {}; print('$name', '%.1f Ms/s'%(d['value']/1e6), '%.1f ms/step'%d['ms_per_step'], 'parity=%s'%p.get('pass'), {k:v for k,v in d['stages_ms_per_step'].items() if v})"
done
