#!/bin/bash
# A/B: wavefront batch size (JSRT_MAX_PATHS) per config, default library, no CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for CFG in "$@"; do
  EXTRA=""; [ "$CFG" = dragon ] && EXTRA="--spp 16"
  for mp in ${MPS:-2097152 4194304 8388608}; do
    JSRT_MAX_PATHS=$mp timeout -k 10 300 python bench.py --config $CFG $EXTRA --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/mp_${CFG}_$mp.json 2> gpurun_out/mp_${CFG}_$mp.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/mp_${CFG}_$mp.json').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']; print('$CFG $mp', '%.1f Ms/s'%(d['value']/1e6), d['frame_attempts'], 'ext %.1f shd %.1f shade %.1f red %.1f'%(s['k_extend'], s['k_shadow'], s['k_shade'], s['k_reduce']))"
  done
done
