set -o pipefail
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
timeout -k 10 300 python -u tools/predict_gap.py > gpurun_out/gap7_headline.txt 2>gpurun_out/gap7.err && cat gpurun_out/gap7_headline.txt &&
timeout -k 10 300 python -u tools/predict_gap.py --self-exchange > gpurun_out/gap7_selfx.txt 2>>gpurun_out/gap7.err && grep -v "RCCL\|version\|Hostname\|Librccl" gpurun_out/gap7_selfx.txt &&
tools/bench_reps.sh 3 "$S" "" &&
bash tools/rehearse_torchrun.sh
