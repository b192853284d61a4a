set -o pipefail
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py --timeout 120 --timeout-method thread > gpurun_out/t8_tests.log 2>&1; rc=$?; tail -2 gpurun_out/t8_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
tools/bench_reps.sh 3 "GOL_SCHEDULE=split $S" "GOL_SCHEDULE=split GOL_BAND_PRIO=1 $S" "GOL_SCHEDULE=split GOL_SPLIT_ORDER=interior $S" "GOL_SCHEDULE=split GOL_BAND_PRIO=1 GOL_SPLIT_ORDER=interior $S" &&
GOL_SCHEDULE=split GOL_BAND_PRIO=1 GOL_SPLIT_ORDER=interior tools/trace_run.sh strip_prio_int $S &&
GOL_SCHEDULE=split GOL_BAND_PRIO=1 tools/trace_run.sh strip_prio $S
