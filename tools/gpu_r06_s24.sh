#!/bin/bash
# round 6 s24: round-end rehearsal on the shipped build: smoke(), then bench.py with no flags (the driver's N = 1 line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r06_s24.log 2>&1 || { tail -5 gpurun_out/smoke_r06_s24.log; exit 1; }
tail -1 gpurun_out/smoke_r06_s24.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r06_s24.json 2> gpurun_out/bench_r06_s24.err || { tail -5 gpurun_out/bench_r06_s24.err; exit 1; }
cat gpurun_out/bench_r06_s24.json
