set -o pipefail
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py tests/test_gpu_pipe.py --timeout 120 --timeout-method thread > gpurun_out/t6_tests.log 2>&1; rc=$?; tail -3 gpurun_out/t6_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/predict_gap.py > gpurun_out/gap_headline.txt 2>gpurun_out/gap.err && cat gpurun_out/gap_headline.txt &&
timeout -k 10 300 python -u tools/predict_gap.py --self-exchange > gpurun_out/gap_selfx.txt 2>>gpurun_out/gap.err && cat gpurun_out/gap_selfx.txt &&
timeout -k 10 300 python -u tools/predict_gap.py --size 4096 --width 32768 --self-exchange > gpurun_out/gap_strip.txt 2>>gpurun_out/gap.err && cat gpurun_out/gap_strip.txt &&
tools/bench_reps.sh 3 "$S" &&
tools/trace_run.sh strip_split6 $S
