#!/bin/bash
# Round-5 GPU batches, one function each (on the GPU box: bash tools/round5_batches.sh <name>).
# Each was run once as its own script during round 5; the summaries kept are in profiles/ (named in
# docs/PERFORMANCE.md §16 and docs/REVIEW_RESPONSE.md).  The final evidence batch is tools/final_round5.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp

# gpu1: formerly tools/_gpu1.sh
cmd_gpu1() {
cd $GRAFT_REPO_ROOT
tools/trace_run.sh strip_selfx --size 4096 --width 32768 --self-exchange &&
tools/trace_run.sh strip_selfx_b --size 4096 --width 32768 --self-exchange &&
tools/trace_run.sh t32768_selfx --self-exchange &&
tools/trace_run.sh t32768 &&
tools/bench_reps.sh 3 "--size 4096 --width 32768 --self-exchange" "--self-exchange" ""
}

# gpu2: formerly tools/_gpu2.sh
cmd_gpu2() {
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
P="GOL_KERNEL=pipe GOL_PIPE=11,2,1"
timeout -k 10 300 python -u -m pytest -v tests/test_gpu_rccl.py -x -q --timeout 120 --timeout-method thread -k "split_pipe" > gpurun_out/t2_tests.log 2>&1 && tail -3 gpurun_out/t2_tests.log &&
tools/bench_reps.sh 2 "$S" "$P $S" "$P GOL_SCHEDULE=split GOL_GRAPH_RCCL=0 $S" "$P GOL_SCHEDULE=split GOL_GRAPH_RCCL=1 $S" "$P GOL_SCHEDULE=split GOL_GRAPH_RCCL=1 GOL_SPLIT_BANDS_COMM=1 $S" "$P GOL_SCHEDULE=split GOL_GRAPH_RCCL=0 GOL_SPLIT_BANDS_COMM=1 $S" &&
GOL_KERNEL=pipe GOL_PIPE=11,2,1 GOL_SCHEDULE=split GOL_GRAPH_RCCL=1 GOL_SPLIT_BANDS_COMM=1 tools/trace_run.sh split_graph_bandscomm $S &&
GOL_KERNEL=pipe GOL_PIPE=11,2,1 GOL_SCHEDULE=split GOL_GRAPH_RCCL=0 GOL_SPLIT_BANDS_COMM=1 tools/trace_run.sh split_eager_bandscomm $S &&
GOL_KERNEL=pipe GOL_PIPE=11,2,1 tools/trace_run.sh pipe20_auto $S &&
GOL_KERNEL=pipe GOL_PIPE=11,2,1 GOL_SCHEDULE=split GOL_GRAPH_RCCL=0 tools/trace_run.sh split_eager $S
}

# gpu3: formerly tools/_gpu3.sh
cmd_gpu3() {
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
timeout -k 10 900 python -u -m pytest -x -q tests -m gpu --timeout 120 --timeout-method thread > gpurun_out/t3_tests.log 2>&1; rc=$?; tail -15 gpurun_out/t3_tests.log; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
tools/bench_reps.sh 2 "$S" "GOL_SCHEDULE=split $S" "GOL_SCHEDULE=full GOL_GRAPH_RCCL=1 $S" "" "--self-exchange" &&
tools/trace_run.sh strip_auto $S &&
GOL_SCHEDULE=split tools/trace_run.sh strip_split $S
}

# gpu4: formerly tools/_gpu4.sh
cmd_gpu4() {
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
}

# gpu5: formerly tools/_gpu5.sh
cmd_gpu5() {
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q tests -m gpu --timeout 120 --timeout-method thread > gpurun_out/t5_tests.log 2>&1; rc=$?; tail -5 gpurun_out/t5_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t5_smoke.log 2>&1 && tail -1 gpurun_out/t5_smoke.log &&
tools/bench_reps.sh 3 "" "--self-exchange" "--size 4096 --width 32768 --self-exchange" "--size 4096 --width 32768"
}

# gpu6: formerly tools/_gpu6.sh
cmd_gpu6() {
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py tests/test_gpu_pipe.py --timeout 120 --timeout-method thread > gpurun_out/t6_tests.log 2>&1; rc=$?; tail -3 gpurun_out/t6_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/predict_gap.py > gpurun_out/gap_headline.txt 2>gpurun_out/gap.err && cat gpurun_out/gap_headline.txt &&
timeout -k 10 300 python -u tools/predict_gap.py --self-exchange > gpurun_out/gap_selfx.txt 2>>gpurun_out/gap.err && cat gpurun_out/gap_selfx.txt &&
timeout -k 10 300 python -u tools/predict_gap.py --size 4096 --width 32768 --self-exchange > gpurun_out/gap_strip.txt 2>>gpurun_out/gap.err && cat gpurun_out/gap_strip.txt &&
tools/bench_reps.sh 3 "$S" &&
tools/trace_run.sh strip_split6 $S
}

# gpu7: formerly tools/_gpu7.sh
cmd_gpu7() {
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
timeout -k 10 300 python -u tools/predict_gap.py > gpurun_out/gap7_headline.txt 2>gpurun_out/gap7.err && cat gpurun_out/gap7_headline.txt &&
timeout -k 10 300 python -u tools/predict_gap.py --self-exchange > gpurun_out/gap7_selfx.txt 2>>gpurun_out/gap7.err && grep -v "RCCL\|version\|Hostname\|Librccl" gpurun_out/gap7_selfx.txt &&
tools/bench_reps.sh 3 "$S" "" &&
bash tools/rehearse_torchrun.sh
}

# gpu8: formerly tools/_gpu8.sh
cmd_gpu8() {
cd $GRAFT_REPO_ROOT
S="--size 4096 --width 32768 --self-exchange"
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py --timeout 120 --timeout-method thread > gpurun_out/t8_tests.log 2>&1; rc=$?; tail -2 gpurun_out/t8_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
tools/bench_reps.sh 3 "GOL_SCHEDULE=split $S" "GOL_SCHEDULE=split GOL_BAND_PRIO=1 $S" "GOL_SCHEDULE=split GOL_SPLIT_ORDER=interior $S" "GOL_SCHEDULE=split GOL_BAND_PRIO=1 GOL_SPLIT_ORDER=interior $S" &&
GOL_SCHEDULE=split GOL_BAND_PRIO=1 GOL_SPLIT_ORDER=interior tools/trace_run.sh strip_prio_int $S &&
GOL_SCHEDULE=split GOL_BAND_PRIO=1 tools/trace_run.sh strip_prio $S
}

# gpu10: formerly tools/_gpu10.sh
cmd_gpu10() {
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_headline.py tests/test_gpu_rccl.py --timeout 300 --timeout-method thread > gpurun_out/t10_tests.log 2>&1; rc=$?; tail -2 gpurun_out/t10_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/configs; bash tools/baseline_configs.sh cfg2b cfg4 > gpurun_out/t10_configs.log 2>&1 || exit 1
for f in gpurun_out/configs/cfg2_bench_8192.log gpurun_out/configs/cfg4_bench_65536_2d.log; do grep -h '^{' $f | python3 tools/bench_line.py "$(basename $f .log)"; done
}

# gpu11: formerly tools/_gpu11.sh
cmd_gpu11() {
cd $GRAFT_REPO_ROOT
GOL_INIT_LOG=1 timeout -k 10 300 python bench.py --size 65536 --scaling strong --decomp 2d --steps 400 --warmup 40 > gpurun_out/cfg4_dbg.log 2>&1; echo "rc=$?"; grep -v "RCCL\|version\|Hostname\|Librccl" gpurun_out/cfg4_dbg.log | tail -25 | cut -c1-250
}

# gpu12: formerly tools/_gpu12.sh
cmd_gpu12() {
cd $GRAFT_REPO_ROOT
GOL_INIT_LOG=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/k10.log 2>&1; echo "rc=$?"; grep "pass costs\|prediction" gpurun_out/k10.log | tail -16; grep '^{' gpurun_out/k10.log | python3 tools/bench_line.py k10
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/k10.log') if l.startswith('{')][0]);print(' '.join(t for t in d['config']['autotune'].split() if t.startswith(('pass','cut'))))"
timeout -k 10 300 python -u -m pytest -x -q tests/test_gpu_headline.py tests/test_gpu_engine.py --timeout 300 --timeout-method thread > gpurun_out/t12_tests.log 2>&1; rc=$?; tail -2 gpurun_out/t12_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/bench_reps.*; tools/bench_reps.sh 5 ""
}

# gpu13: formerly tools/_gpu13.sh
cmd_gpu13() {
cd $GRAFT_REPO_ROOT
GOL_INIT_LOG=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/k10p.log 2>&1; echo "rc=$?"; grep '^{' gpurun_out/k10p.log | python3 tools/bench_line.py k10p
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/k10p.log') if l.startswith('{')][0]);print(' '.join(t for t in d['config']['autotune'].split() if t.startswith(('pass','cut'))))"
}

# gpu14: formerly tools/_gpu14.sh
cmd_gpu14() {
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/bench_reps.*; tools/bench_reps.sh 3 "" "GOL_PREDICT_FIRST=1" "--self-exchange" "GOL_PREDICT_FIRST=1 --self-exchange" "--size 4096 --width 32768 --self-exchange" "GOL_PREDICT_FIRST=1 --size 4096 --width 32768 --self-exchange"
}

name=$1; shift || true
declare -F "cmd_$name" > /dev/null || { echo "usage: $0 {gpu1..gpu14}"; exit 2; }
"cmd_$name" "$@"
