#!/bin/bash
# round 6 s2: GPU suite, k_shadow decomposition (timing-only variants), instruction / scalar cache counters of cornell
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s2.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s2.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh cornell_box_path 8 2 base= nocast=@nocast cullonly=@cullonly 2>&1 | tee gpurun_out/ab_r06_s2.txt || exit 1
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/avail_r06.txt 2>&1
grep -i "icache\|dcache\|IFETCH" gpurun_out/avail_r06.txt | head -40
mkdir -p gpurun_out/pmc_r06_s2
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES --kernel-trace --output-format csv \
  -d gpurun_out/pmc_r06_s2/ic -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity --ab > gpurun_out/pmc_r06_s2/ic.log 2>&1
echo "pmc rc=$?"
