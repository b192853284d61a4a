set -o pipefail
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/bench_reps.*; tools/bench_reps.sh 3 "" "GOL_PREDICT_FIRST=1" "--self-exchange" "GOL_PREDICT_FIRST=1 --self-exchange" "--size 4096 --width 32768 --self-exchange" "GOL_PREDICT_FIRST=1 --size 4096 --width 32768 --self-exchange"
