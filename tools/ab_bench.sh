#!/bin/bash
# A/B: bench each named library variant (JSRT_LIB) on one config, no CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
CFG=$1; shift
for v in "$@"; do
  lib=$PWD/jsraytracer_amd/_build/libjsrt_$v.so; [ "$v" = base ] && lib=$PWD/jsraytracer_amd/_build/libjsrt.so
  read -r -a extra <<< "${AB_BENCH_ARGS:-}"  # e.g. --no-parity for timing-only variants, --steps 8
  JSRT_LIB=$lib timeout -k 10 600 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --ab "${extra[@]}" > gpurun_out/ab_${CFG}_$v.json 2> gpurun_out/ab_${CFG}_$v.err
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc  # 3: the line was printed, parity failed
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_${CFG}_$v.json')); p=d.get('parity') or {}; print('$v', '%.1f Ms/s'%(d['value']/1e6), '%.1f ms/step'%d['ms_per_step'], 'parity=%s'%p.get('pass'), d['stages_ms_per_step'])"
done
