set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_BENCH_ARGS="--steps 3" timeout -k 10 600 bash tools/ab_bench.sh SDF_Menger base menger so4 sh5 > gpurun_out/ab3_menger.txt 2>&1; rc=$?; cat gpurun_out/ab3_menger.txt; [ $rc -eq 0 ] || exit $rc
JSRT_LIB=$PWD/jsraytracer_amd/_build/libjsrt_menger.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab3 -o run -- \
    python bench.py --config SDF_Menger --steps 1 --warmup 1 --no-cpu-baseline --no-parity --events --ab > gpurun_out/ab3_prof.json 2> gpurun_out/ab3_prof.err || exit $?
head -12 gpurun_out/prof_ab3/run_kernel_stats.csv
