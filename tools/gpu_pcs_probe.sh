#!/bin/bash
# GPU-box probe: which PC-sampling configurations rocprofv3 offers on this device.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_list.txt 2>&1
grep -i -B2 -A12 "pc.sampl\|pc_sampl" gpurun_out/rocprof_list.txt | head -60
exit 0
