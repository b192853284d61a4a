#!/bin/bash
# Round-5 evidence on one MI355X: GPU suite, smoke, the driver's bench command x5, the per-rank tiles of
# the scaling configs through the RCCL self-exchange at the driver's cut, the BASELINE configs that fit
# one GPU, and a rocprofv3 kernel-trace/stats profile of the driver command.  Every GPU step has its own
# time limit; a fatal status ends the script.  Output: gpurun_out/final5/ (summary.txt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final5; mkdir -p $O
export TMPDIR=/tmp
S=$O/summary.txt; : > $S
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "== pytest -m gpu rc=$rc: $(tail -1 $O/pytest_gpu.log)" >> $S; fatal $rc && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "== smoke rc=$rc: $(tail -1 $O/smoke.log)" >> $S; fatal $rc && exit $rc
rm -f gpurun_out/bench_reps.*
tools/bench_reps.sh 5 "" > /dev/null || exit 1
{ echo "== driver command: bench.py --gpus 1 --steps 20 --warmup 5 (x5)"; cat gpurun_out/bench_reps.txt; } >> $S; mv gpurun_out/bench_reps.jsonl $O/driver.jsonl; rm -f gpurun_out/bench_reps.txt
tools/bench_reps.sh 3 "--self-exchange" "--size 4096 --width 32768 --self-exchange" > /dev/null || exit 1
tools/bench_reps.sh 2 "--size 8192 --width 32768 --self-exchange" "--size 16384 --width 32768 --self-exchange" "--size 32768 --width 16384 --decomp 2d --self-exchange" "--size 4096 --width 32768" > /dev/null || exit 1
{ echo "== per-rank tiles through the RCCL self-exchange (and the N = 8 strip without neighbours), driver's cut"; cat gpurun_out/bench_reps.txt; } >> $S; mv gpurun_out/bench_reps.jsonl $O/tiles.jsonl
bash tools/baseline_configs.sh cfg1 cfg2 cfg2b cfg3 cfg4 > $O/configs.log 2>&1; rc=$?
{ echo "== BASELINE configs (tools/baseline_configs.sh) rc=$rc"; for f in gpurun_out/configs/cfg1_cpu_256.log gpurun_out/configs/cfg2_cli_8192.log; do echo "$(basename $f .log): $(grep -h TOTAL $f)"; done; for f in gpurun_out/configs/cfg2_bench_8192.log gpurun_out/configs/cfg3_bench_32768.log gpurun_out/configs/cfg4_bench_65536_2d.log; do grep -h '^{' $f | python3 tools/bench_line.py "$(basename $f .log)"; done; } >> $S; fatal $rc && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1; rc=$?
echo "== rocprofv3 --kernel-trace --stats of the driver command rc=$rc" >> $S; fatal $rc && exit $rc
cat $S
