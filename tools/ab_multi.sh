#!/bin/bash
# A/B: bench each library variant on each config (no CPU baseline); dragon at spp 16 (same launch shapes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARS=$1; shift
for CFG in "$@"; do
  EXTRA=""; [ "$CFG" = dragon ] && EXTRA="--spp 16"
  for v in $VARS; do
    JSRT_LIB=$PWD/jsraytracer_amd/_build/libjsrt_$v.so timeout -k 10 300 python bench.py --config $CFG $EXTRA --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_${CFG}_$v.json 2> gpurun_out/ab_${CFG}_$v.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/ab_${CFG}_$v.json').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']; print('$CFG $v', '%.1f Ms/s'%(d['value']/1e6), 'ext %.1f shd %.1f shade %.1f'%(s['k_extend'], s['k_shadow'], s['k_shade']))"
  done
done
