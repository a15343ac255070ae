#!/bin/bash
# (diagnostic) one rocprofv3 --pmc pass (instruction counts) of a one-step cornell bench per library variant.
#   bash tools/diag/pmc_ab.sh TAG VAR...   (VAR: base or a libjsrt_VAR.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
for v in "$@"; do
  lib=$PWD/jsraytracer_amd/_build/libjsrt_$v.so; [ "$v" = base ] && lib=$PWD/jsraytracer_amd/_build/libjsrt.so
  D=gpurun_out/pmcab_${TAG}_$v; mkdir -p $D
  JSRT_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace --output-format csv -d $D -o run -- \
      python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity --ab > $D/bench.log 2>&1 || { echo "pmc $v failed"; tail -3 $D/bench.log; exit 1; }
  python tools/pmc_summary.py $D | grep -E "^== k_(shadow|shade|extend)|/ wave" | grep -v "x4 cyc" | sed "s/^/$v /"
done
