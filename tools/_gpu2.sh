set -o pipefail
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
P="GOL_KERNEL=pipe GOL_PIPE=11,2,1"
timeout -k 10 300 python -u -m pytest -v tests/test_gpu_rccl.py -x -q --timeout 120 --timeout-method thread -k "split_pipe" > gpurun_out/t2_tests.log 2>&1 && tail -3 gpurun_out/t2_tests.log &&
tools/bench_reps.sh 2 "$S" "$P $S" "$P GOL_SCHEDULE=split GOL_GRAPH_RCCL=0 $S" "$P GOL_SCHEDULE=split GOL_GRAPH_RCCL=1 $S" "$P GOL_SCHEDULE=split GOL_GRAPH_RCCL=1 GOL_SPLIT_BANDS_COMM=1 $S" "$P GOL_SCHEDULE=split GOL_GRAPH_RCCL=0 GOL_SPLIT_BANDS_COMM=1 $S" &&
GOL_KERNEL=pipe GOL_PIPE=11,2,1 GOL_SCHEDULE=split GOL_GRAPH_RCCL=1 GOL_SPLIT_BANDS_COMM=1 tools/trace_run.sh split_graph_bandscomm $S &&
GOL_KERNEL=pipe GOL_PIPE=11,2,1 GOL_SCHEDULE=split GOL_GRAPH_RCCL=0 GOL_SPLIT_BANDS_COMM=1 tools/trace_run.sh split_eager_bandscomm $S &&
GOL_KERNEL=pipe GOL_PIPE=11,2,1 tools/trace_run.sh pipe20_auto $S &&
GOL_KERNEL=pipe GOL_PIPE=11,2,1 GOL_SCHEDULE=split GOL_GRAPH_RCCL=0 tools/trace_run.sh split_eager $S
