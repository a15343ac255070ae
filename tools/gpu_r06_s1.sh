cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r06_s1.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r06_s1.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_interleave.sh cornell_box_path 8 3 base=JSRT_SHADOW_FLAT=0 flat= 2>&1 | tee gpurun_out/ab_r06_s1.txt
