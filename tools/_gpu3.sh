set -o pipefail
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
timeout -k 10 900 python -u -m pytest -x -q tests -m gpu --timeout 120 --timeout-method thread > gpurun_out/t3_tests.log 2>&1; rc=$?; tail -15 gpurun_out/t3_tests.log; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
tools/bench_reps.sh 2 "$S" "GOL_SCHEDULE=split $S" "GOL_SCHEDULE=full GOL_GRAPH_RCCL=1 $S" "" "--self-exchange" &&
tools/trace_run.sh strip_auto $S &&
GOL_SCHEDULE=split tools/trace_run.sh strip_split $S
