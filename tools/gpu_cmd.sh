timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
cp jsraytracer_amd/_build/libjsrt.so jsraytracer_amd/_build/libjsrt_cur.so && bash tools/ab_bench.sh cornell_box_path cur s4 || exit 1
for v in cur s4; do python -c "import json; d=json.load(open('gpurun_out/ab_cornell_box_path_$v.json')); print('$v', d['stages_ms_per_step'])"; done
