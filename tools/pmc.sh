#!/bin/bash
# GPU-box helper: PMC passes (one rocprofv3 --pmc pass per counter group, kernel-trace only) on a
# one-step bench of CFG using library variant LIBV (JSRT_LIB), output under gpurun_out/pmc_<tag>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFG=${1:-cornell_box_path}; LIBV=${2:-}; TAG=${3:-$CFG}
[ -n "$LIBV" ] && export JSRT_LIB=$PWD/jsraytracer_amd/_build/libjsrt_$LIBV.so
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"
P3="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
P6="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_SMEM SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5" "$P6"; do
  i=$((i+1))
  mkdir -p gpurun_out/pmc_$TAG; timeout -k 10 600 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_$TAG/p$i -o run -- \
     python bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline --no-parity --ab ${PMC_BENCH_ARGS:-} > gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_$TAG --config "$CFG" --merge gpurun_out/pmc_$TAG/pmc_merge.json > gpurun_out/pmc_$TAG/summary.txt && cat gpurun_out/pmc_$TAG/summary.txt
