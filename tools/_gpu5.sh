set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q tests -m gpu --timeout 120 --timeout-method thread > gpurun_out/t5_tests.log 2>&1; rc=$?; tail -5 gpurun_out/t5_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t5_smoke.log 2>&1 && tail -1 gpurun_out/t5_smoke.log &&
tools/bench_reps.sh 3 "" "--self-exchange" "--size 4096 --width 32768 --self-exchange" "--size 4096 --width 32768"
