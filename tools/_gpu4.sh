set -o pipefail
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py tests/test_gpu_pipe.py tests/test_gpu_engine.py --timeout 120 --timeout-method thread > gpurun_out/t4_tests.log 2>&1; rc=$?; tail -5 gpurun_out/t4_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
tools/bench_reps.sh 2 "$S" "GOL_SCHEDULE=split $S" "GOL_SCHEDULE=split GOL_SPLIT_ORDER=interior $S" "--self-exchange" "GOL_SUBTILE_OVERLAP=2 --self-exchange" "" "GOL_SUBTILES=0 --no-graph" "GOL_SUBTILES=0" &&
GOL_SCHEDULE=split tools/trace_run.sh strip_split4 $S &&
GOL_SUBTILE_OVERLAP=2 tools/trace_run.sh selfx_xf --self-exchange &&
GOL_SUBTILES=0 tools/trace_run.sh onetile_eager --no-graph &&
mv gpurun_out/bench_reps.txt gpurun_out/bench_reps_a.txt &&
tools/bench_reps.sh 2 "--size 8192 --width 32768 --self-exchange" "--size 16384 --width 32768 --self-exchange" "--size 32768 --width 16384 --decomp 2d --self-exchange" && mv gpurun_out/bench_reps.txt gpurun_out/bench_reps_b.txt &&
GOL_SUBTILE_XGRAPH=1 tools/bench_reps.sh 2 "--self-exchange" "GOL_SUBTILE_OVERLAP=2 --self-exchange" && mv gpurun_out/bench_reps.txt gpurun_out/bench_reps_c.txt && GOL_SUBTILE_XGRAPH=1 tools/trace_run.sh selfx_xgraph --self-exchange
