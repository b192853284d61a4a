set -o pipefail
cd $GRAFT_REPO_ROOT
tools/trace_run.sh strip_selfx --size 4096 --width 32768 --self-exchange &&
tools/trace_run.sh strip_selfx_b --size 4096 --width 32768 --self-exchange &&
tools/trace_run.sh t32768_selfx --self-exchange &&
tools/trace_run.sh t32768 &&
tools/bench_reps.sh 3 "--size 4096 --width 32768 --self-exchange" "--self-exchange" ""
