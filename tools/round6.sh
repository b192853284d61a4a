#!/bin/bash
# Round-6 GPU batches on one MI355X.  Every GPU step has its own time limit; a fatal status (fault,
# abort, segfault, time limit) ends the script.  Output: gpurun_out/r6/<batch>/ (summary.txt).
#   tools/round6.sh <batch>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=$1
O=gpurun_out/r6/$B; mkdir -p $O
S=$O/summary.txt; : > $S
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
pyt() {  # pyt <log> <pytest args...>
  local log=$1; shift
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > $O/$log 2>&1; local rc=$?
  echo "== pytest $* rc=$rc: $(tail -1 $O/$log)" >> $S; return $rc
}
reps() {  # reps <n> <variants...>: tools/bench_reps.sh, lines appended to the summary
  rm -f gpurun_out/bench_reps.txt
  tools/bench_reps.sh "$@" > /dev/null; local rc=$?
  cat gpurun_out/bench_reps.txt >> $S; cat gpurun_out/bench_reps.jsonl >> $O/bench.jsonl 2>/dev/null
  rm -f gpurun_out/bench_reps.txt gpurun_out/bench_reps.jsonl; return $rc
}
case $B in
b1)
  # the round-6 tests first (ADVICE fixes, the capture guard, the prediction without a snapshot)
  pyt new_tests.log tests/test_gpu_rccl.py tests/test_gpu_engine.py -k "unaligned_width or capture_refused or without_snapshot or split_pipe" || exit 1
  reps 3 "" "--self-exchange" || exit 1
  # the forked-stream RCCL capture: the origin-stream and eager forms first, the crashing form last
  for m in eager origin+reg fork fork+reg; do
    timeout -k 10 120 build/rccl_capture_probe $m > $O/capture_$m.log 2>&1; rc=$?
    echo "== rccl_capture_probe $m rc=$rc: $(tail -1 $O/capture_$m.log)" >> $S
    fatal $rc && break
  done
  ;;
b2)
  # the pair-shared rule (stencil_device.hpp): the whole GPU suite, a kbench A/B of the old rule (r0) against
  # the pair rule (r1) interleaved, the driver's bench and the per-rank tiles, then two more capture probes
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "== pytest -m gpu rc=$rc: $(tail -1 $O/pytest_gpu.log)" >> $S; [ $rc -ne 0 ] && exit $rc
  kb() {  # kb <label> <env...> -- <args...>
    local lab=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    for v in r0 r1; do
      r=$(env "${envs[@]}" timeout -k 5 90 build/kbench_$v "$@" 2>&1 | tail -1); rc=$?
      echo "[kb $lab $v] $(echo "$r" | grep -o '"us_per_gen": [0-9.]*')" >> $S
      fatal $rc && exit $rc
    done
  }
  for round in 1 2 3; do
    kb T8 -- 32768 8 1920
    kb H8 KB_SPLIT2=1 KB_BPC=2 -- 32768 8 1920
    kb H12 KB_SPLIT2=1 KB_BPC=1 -- 32768 12 1920
    kb F32 KB_FOLD=1 -- 8192 32 1920 0 0 8 0 4
    kb P20 KB_W=32768 KB_PIPE=2 -- 4096 20 1920 0 0 11
    kb P24 KB_PIPE=3 KB_PIPE_WG=2 -- 32768 24 1920 0 0 9
  done
  reps 3 "" || exit 1
  reps 1 "--self-exchange" "--size 4096 --width 32768 --self-exchange" "--size 8192 --steps 1000" || exit 1
  for m in query unjoined; do
    timeout -k 10 120 build/rccl_capture_probe $m > $O/capture_$m.log 2>&1; rc=$?
    echo "== rccl_capture_probe $m rc=$rc: $(tail -1 $O/capture_$m.log)" >> $S
    fatal $rc && break
  done
  ;;
b9)
  # step_temporal with the pair rule and the two-triple loop at K = 8 (tp, GOL_TEMPORAL_PAIR=1) against the
  # default build (r1: rule32 in step_temporal), interleaved
  for round in 1 2 3; do
    for cfg in "T8 -- 32768 8 1920" "H8 KB_SPLIT2=1 KB_BPC=2 -- 32768 8 1920" "H12 KB_SPLIT2=1 KB_BPC=1 -- 32768 12 1920" \
               "T6 -- 32768 6 1920" "T5 -- 32768 5 1920"; do
      set -- $cfg; lab=$1; shift; envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
      for v in r1 tp; do
        r=$(env "${envs[@]}" timeout -k 5 90 build/kbench_$v "$@" 2>&1 | tail -1); rc=$?
        echo "[kb $lab $v] $(echo "$r" | grep -o '"us_per_gen": [0-9.]*')" >> $S
        fatal $rc && exit $rc
      done
    done
  done
  ;;
b10)
  # (GOL_COMM_CUS and its layout / plan-size knobs were removed after b10-b13: profiles/comm_cus_round6.txt)
  # VERDICT round 5 item 1's CU-reserved comm stream (GOL_COMM_CUS): the compute cost of the mask on the local
  # tile (both layouts), then the weak-scaling rank's cut through the self-exchange, split and auto, 8 and 16 CUs,
  # the 2-D tile and the strip; one kernel trace of the masked split
  pyt cu_tests.log tests/test_gpu_rccl.py -k "comm_cus or split" || exit 1
  reps 2 "" "GOL_COMM_CUS=8" "GOL_COMM_CUS=8 GOL_COMM_CU_LAYOUT=1" || exit 1
  reps 2 "--self-exchange" "GOL_COMM_CUS=8 --self-exchange" "GOL_COMM_CUS=8 GOL_SCHEDULE=split --self-exchange" \
    "GOL_COMM_CUS=16 GOL_SCHEDULE=split --self-exchange" "GOL_COMM_CUS=8 GOL_COMM_CU_LAYOUT=1 GOL_SCHEDULE=split --self-exchange" || exit 1
  reps 2 "--size 32768 --width 16384 --decomp 2d --self-exchange" "GOL_COMM_CUS=8 --size 32768 --width 16384 --decomp 2d --self-exchange" \
    "--size 4096 --width 32768 --self-exchange" "GOL_COMM_CUS=8 --size 4096 --width 32768 --self-exchange" || exit 1
  GOL_COMM_CUS=8 GOL_SCHEDULE=split bash tools/trace_run.sh cu8_split --self-exchange > /dev/null || exit 1
  cat gpurun_out/trace_cu8_split.txt >> $S
  ;;
b11)
  # GOL_COMM_CUS sweep: 2 and 4 reserved CUs (8 and 16 in b10), local and the self-exchange cut
  reps 2 "GOL_COMM_CUS=2" "GOL_COMM_CUS=4" "GOL_COMM_CUS=2 --self-exchange" "GOL_COMM_CUS=4 --self-exchange" \
    "GOL_COMM_CUS=4 GOL_SCHEDULE=split --self-exchange" "GOL_SUBTILES=0" || exit 1
  ;;
b12)
  # is it the masked queue? the compute stream's mask with every CU (layout 2), local
  reps 2 "GOL_COMM_CUS=8 GOL_COMM_CU_LAYOUT=2" "GOL_SUBTILES=0" "GOL_COMM_CUS=8 GOL_COMM_CU_LAYOUT=2 GOL_KERNEL=temporal" "GOL_SUBTILES=0 GOL_KERNEL=temporal" || exit 1
  ;;
b13)
  # 8 CUs masked off the compute stream (layout 0), plans sized for 256 / 248 / 240 / 224 / 192 CUs, step_temporal
  reps 1 "GOL_SUBTILES=0 GOL_KERNEL=temporal" || exit 1
  for pc in 256 248 240 224 192; do reps 1 "GOL_COMM_CUS=8 GOL_PLAN_CUS=$pc GOL_KERNEL=temporal" || exit 1; done
  for pc in 256 224; do reps 1 "GOL_COMM_CUS=8 GOL_COMM_CU_LAYOUT=1 GOL_PLAN_CUS=$pc GOL_KERNEL=temporal" || exit 1; done
  ;;
b14)
  # HIP runtime knobs against the driver command's fixed cost (launch to first kernel, last kernel to sync)
  reps 3 "" "ROC_ACTIVE_WAIT_TIMEOUT=1000" "ROC_ACTIVE_WAIT_TIMEOUT=0" "ROC_CPU_WAIT_FOR_SIGNAL=0" "HIP_FORCE_DEV_KERNARG=0" \
    "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "ROC_SKIP_KERNEL_ARG_COPY=1" || exit 1
  ;;
b15)
  # confirm_schedule: close calls of the schedule timing settled on the real run() path; the RCCL, engine and
  # P = 8 thread-rank tests, then the per-rank tiles whose candidates time within a few % of each other
  pyt confirm_tests.log tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py tests/test_gpu_engine.py || exit 1
  reps 3 "--size 32768 --width 16384 --decomp 2d --self-exchange" "--self-exchange" "" "--size 4096 --width 32768 --self-exchange" || exit 1
  ;;
b16)
  # step_pipe as two halves on two streams (KB_SPLIT2 with KB_PIPE) against the headline's two step_temporal halves
  # and the one-tile step_pipe, 32768^2, 2 rounds
  for round in 1 2; do
    for cfg in "H8t KB_SPLIT2=1 KB_BPC=2 -- 32768 8 1920" "P24 KB_PIPE=3 KB_PIPE_WG=2 -- 32768 24 1920 0 0 9" \
               "HP24w1 KB_SPLIT2=1 KB_PIPE=3 KB_PIPE_WG=1 -- 32768 24 1920 0 0 9" "HP24w2 KB_SPLIT2=1 KB_PIPE=3 KB_PIPE_WG=2 -- 32768 24 1920 0 0 9" \
               "P36 KB_PIPE=3 -- 32768 36 1920 0 0 13" "HP36 KB_SPLIT2=1 KB_PIPE=3 -- 32768 36 1920 0 0 13" \
               "HP16 KB_SPLIT2=1 KB_PIPE=2 -- 32768 16 1920 0 0 9" "HP20 KB_SPLIT2=1 KB_PIPE=2 -- 32768 20 1920 0 0 11"; do
      set -- $cfg; lab=$1; shift; envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
      r=$(env "${envs[@]}" timeout -k 5 90 build/kbench_r1 "$@" 2>&1 | tail -1); rc=$?
      echo "[kb $lab] $(echo "$r" | grep -o '"us_per_gen": [0-9.]*')" >> $S
      fatal $rc && exit $rc
    done
  done
  ;;
b18)
  # the round-6 final tree (1/2): the whole GPU suite, smoke, the driver's command x5
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "== pytest -m gpu rc=$rc: $(tail -1 $O/pytest_gpu.log)" >> $S; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
  echo "== smoke rc=$rc: $(tail -1 $O/smoke.log)" >> $S; fatal $rc && exit $rc
  reps 5 "" || exit 1
  ;;
b19)
  # the round-6 final tree (2/2): the per-rank tiles through RCCL, BASELINE configs 1/3/4, the 8-process torchrun
  # rehearsal of the driver's multi-GPU launch (host-staged halos: 8 ranks share the one GPU)
  reps 2 "--self-exchange" "--size 32768 --width 16384 --decomp 2d --self-exchange" "--size 4096 --width 32768 --self-exchange" || exit 1
  bash tools/baseline_configs.sh cfg1 cfg3 cfg4 > $O/configs.log 2>&1; rc=$?
  { echo "== BASELINE configs rc=$rc"; echo "cfg1: $(grep -h TOTAL gpurun_out/configs/cfg1_cpu_256.log)"; for f in gpurun_out/configs/cfg3_bench_32768.log gpurun_out/configs/cfg4_bench_65536_2d.log; do grep -h '^{' $f | python3 tools/bench_line.py "$(basename $f .log)"; done; } >> $S; fatal $rc && exit $rc
  rm -f gpurun_out/rehearse/summary.txt
  bash tools/rehearse_torchrun.sh > $O/rehearse.log 2>&1; rc=$?
  echo "== tools/rehearse_torchrun.sh rc=$rc" >> $S; cat gpurun_out/rehearse/summary.txt >> $S
  ;;
b20)
  # the split superstep's interior issued before the exchange for every interior kernel (GOL_SPLIT_INT_FIRST=1; by
  # default only a step_pipe interior of a one-pass superstep goes first): config 4's 2-D tile, the weak rank, the strip
  reps 3 "GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" "GOL_SPLIT_INT_FIRST=1 GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" \
    "GOL_SCHEDULE=split --self-exchange" "GOL_SPLIT_INT_FIRST=1 GOL_SCHEDULE=split --self-exchange" || exit 1
  GOL_SPLIT_INT_FIRST=1 GOL_SCHEDULE=split bash tools/trace_run.sh t2d_intfirst --size 32768 --width 16384 --decomp 2d --self-exchange > /dev/null || exit 1
  GOL_SCHEDULE=split bash tools/trace_run.sh t2d_split --size 32768 --width 16384 --decomp 2d --self-exchange > /dev/null || exit 1
  cat gpurun_out/trace_t2d_intfirst.txt gpurun_out/trace_t2d_split.txt >> $S
  ;;
b21)
  # interior-first as the split default: the split / RCCL / thread-rank / pipe tests, then the per-rank tiles through
  # the auto schedule timing, new order against the old (GOL_SPLIT_INT_FIRST=0), interleaved
  pyt split_tests.log tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py tests/test_gpu_pipe.py tests/test_gpu_engine.py -k "split or rccl or p8 or pipe" || exit 1
  reps 3 "--size 32768 --width 16384 --decomp 2d --self-exchange" "GOL_SPLIT_INT_FIRST=0 --size 32768 --width 16384 --decomp 2d --self-exchange" \
    "--self-exchange" "GOL_SPLIT_INT_FIRST=0 --self-exchange" "--size 4096 --width 32768 --self-exchange" "GOL_SPLIT_INT_FIRST=0 --size 4096 --width 32768 --self-exchange" || exit 1
  ;;
b22)
  # config 4's 2-D tile: forced split against the auto schedule timing (which picks split), same box, interleaved
  reps 3 "GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" "--size 32768 --width 16384 --decomp 2d --self-exchange" || exit 1
  ;;
b23)
  # no ready-event record between a superstep's first and second pass (GOL_FIRST_PASS_MARK=1: the old record): tests,
  # then config 4's 2-D tile, the forced-split weak rank, the strip, interleaved; a trace of the 2-D tile
  pyt mark_tests.log tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py tests/test_gpu_engine.py tests/test_gpu_pipe.py || exit 1
  reps 3 "--size 32768 --width 16384 --decomp 2d --self-exchange" "GOL_FIRST_PASS_MARK=1 --size 32768 --width 16384 --decomp 2d --self-exchange" \
    "GOL_SCHEDULE=split --self-exchange" "GOL_FIRST_PASS_MARK=1 GOL_SCHEDULE=split --self-exchange" "--size 4096 --width 32768 --self-exchange" || exit 1
  bash tools/trace_run.sh t2d_nomark --size 32768 --width 16384 --decomp 2d --self-exchange > /dev/null || exit 1
  cat gpurun_out/trace_t2d_nomark.txt >> $S
  ;;
b24)
  # (GOL_EXP_NO_END_RECORD was an experiment-only knob, removed after this batch: profiles/end_record_round6.txt)
  # the headline's end-of-superstep event records: default (watchdog markers), --watchdog 0 (plain records), --watchdog 0
  # with no end records (experiment knob, valid only because bench.py synchronises before the timed run), interleaved
  reps 4 "" "--watchdog 0" "GOL_EXP_NO_END_RECORD=1 --watchdog 0" || exit 1
  ;;
b26)
  # (GOL_SPLIT_SWAP was removed after this batch: profiles/split_order_round6.txt, b26)
  # GOL_SPLIT_SWAP=1: a split superstep's interior on the comm stream, exchange + bands + later passes on the compute
  # stream; the split tests with it, then config 4's 2-D tile and the forced-split weak rank, interleaved; a trace
  GOL_SPLIT_SWAP=1 pyt swap_tests.log tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py -k "split or 2d or p8 or confirm" || exit 1
  reps 3 "--size 32768 --width 16384 --decomp 2d --self-exchange" "GOL_SPLIT_SWAP=1 --size 32768 --width 16384 --decomp 2d --self-exchange" \
    "GOL_SCHEDULE=split --self-exchange" "GOL_SPLIT_SWAP=1 GOL_SCHEDULE=split --self-exchange" || exit 1
  GOL_SPLIT_SWAP=1 bash tools/trace_run.sh t2d_swap --size 32768 --width 16384 --decomp 2d --self-exchange > /dev/null || exit 1
  cat gpurun_out/trace_t2d_swap.txt >> $S
  ;;
b27)
  # n row bands of 32768^2 on n streams, step_temporal (kbench KB_SPLIT2=n), plans sized for KB_BPC waves per SIMD
  for round in 1 2; do
    for cfg in "n2b2 KB_SPLIT2=2 KB_BPC=2 -- 32768 8 1920" "n3b1 KB_SPLIT2=3 KB_BPC=1 -- 32768 8 1920" "n3b2 KB_SPLIT2=3 KB_BPC=2 -- 32768 8 1920" \
               "n4b1 KB_SPLIT2=4 KB_BPC=1 -- 32768 8 1920" "n4b2 KB_SPLIT2=4 KB_BPC=2 -- 32768 8 1920" "n2k12 KB_SPLIT2=2 KB_BPC=1 -- 32768 12 1920" \
               "n3k12 KB_SPLIT2=3 KB_BPC=1 -- 32768 12 1920" "n4k12 KB_SPLIT2=4 KB_BPC=1 -- 32768 12 1920"; do
      set -- $cfg; lab=$1; shift; envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
      r=$(env "${envs[@]}" timeout -k 5 90 build/kbench_r1 "$@" 2>&1 | tail -1); rc=$?
      echo "[kb $lab] $(echo "$r" | grep -o '"us_per_gen": [0-9.]*')" >> $S
      fatal $rc && exit $rc
    done
  done
  ;;
b28)
  # confirm_schedule over up to two runners-up: the RCCL / thread-rank / engine tests, then the weak rank and the 2-D
  # tile through the auto timing
  pyt confirm3_tests.log tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py tests/test_gpu_engine.py || exit 1
  reps 3 "--self-exchange" "--size 32768 --width 16384 --decomp 2d --self-exchange" || exit 1
  ;;
b29)
  # kernel traces of the weak rank's split superstep (the confirmed schedule) and of the local headline
  GOL_SCHEDULE=split bash tools/trace_run.sh selfx_split --self-exchange > /dev/null || exit 1
  bash tools/trace_run.sh local_head > /dev/null || exit 1
  cat gpurun_out/trace_selfx_split.txt gpurun_out/trace_local_head.txt >> $S
  ;;
b30)
  # GOL_SPLIT_BANDS_COMM=1: a multi-pass split superstep's bands on the comm stream right after the exchange, beside the
  # interior; the split tests with it, then the forced-split weak rank and config 4's 2-D tile, interleaved; traces
  GOL_SPLIT_BANDS_COMM=1 pyt bandscomm_tests.log tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py -k "split or 2d or p8 or confirm" || exit 1
  reps 3 "GOL_SCHEDULE=split --self-exchange" "GOL_SPLIT_BANDS_COMM=1 GOL_SCHEDULE=split --self-exchange" \
    "GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" "GOL_SPLIT_BANDS_COMM=1 GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" || exit 1
  GOL_SPLIT_BANDS_COMM=1 GOL_SCHEDULE=split bash tools/trace_run.sh selfx_bandscomm --self-exchange > /dev/null || exit 1
  GOL_SPLIT_BANDS_COMM=1 GOL_SCHEDULE=split bash tools/trace_run.sh t2d_bandscomm --size 32768 --width 16384 --decomp 2d --self-exchange > /dev/null || exit 1
  cat gpurun_out/trace_selfx_bandscomm.txt gpurun_out/trace_t2d_bandscomm.txt >> $S
  ;;
b31)
  # the split bands beside the interior as the default: the whole GPU suite, then the per-rank tiles through the auto
  # schedule timing (weak rank, config 4's 2-D tile, config 3's strip) and the driver's command
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "== pytest -m gpu rc=$rc: $(tail -1 $O/pytest_gpu.log)" >> $S; [ $rc -ne 0 ] && exit $rc
  reps 3 "--self-exchange" "--size 32768 --width 16384 --decomp 2d --self-exchange" "--size 4096 --width 32768 --self-exchange" "" || exit 1
  ;;
b32)
  # (GOL_SPLIT_RESERVE was removed after this batch: profiles/split_order_round6.txt, b32)
  # GOL_SPLIT_RESERVE=n: the split interior's one-round plan leaves n workgroup slots free for the exchange's kernels;
  # forced split, weak rank and config 4's 2-D tile, n = 0 / 8 / 16 / 32 interleaved; a trace of the 2-D tile at n = 16
  reps 2 "GOL_SCHEDULE=split --self-exchange" "GOL_SPLIT_RESERVE=8 GOL_SCHEDULE=split --self-exchange" "GOL_SPLIT_RESERVE=16 GOL_SCHEDULE=split --self-exchange" "GOL_SPLIT_RESERVE=32 GOL_SCHEDULE=split --self-exchange" || exit 1
  reps 2 "GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" "GOL_SPLIT_RESERVE=8 GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" \
    "GOL_SPLIT_RESERVE=16 GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" "GOL_SPLIT_RESERVE=32 GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" || exit 1
  GOL_SPLIT_RESERVE=16 GOL_SCHEDULE=split bash tools/trace_run.sh t2d_res16 --size 32768 --width 16384 --decomp 2d --self-exchange > /dev/null || exit 1
  GOL_SPLIT_RESERVE=16 GOL_SCHEDULE=split bash tools/trace_run.sh selfx_res16 --self-exchange > /dev/null || exit 1
  cat gpurun_out/trace_t2d_res16.txt gpurun_out/trace_selfx_res16.txt >> $S
  ;;
b33)
  # GOL_SPLIT_VALUE_WAIT=1: the compute stream waits for the split bands with hipStreamWaitValue32 on a value the comm stream
  # writes after them, instead of an event; tests, then forced split on the weak rank and config 4's 2-D tile; traces
  GOL_SPLIT_VALUE_WAIT=1 pyt valuewait_tests.log tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py -k "split or 2d or p8 or confirm" || exit 1
  reps 3 "GOL_SCHEDULE=split --self-exchange" "GOL_SPLIT_VALUE_WAIT=1 GOL_SCHEDULE=split --self-exchange" \
    "GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" "GOL_SPLIT_VALUE_WAIT=1 GOL_SCHEDULE=split --size 32768 --width 16384 --decomp 2d --self-exchange" || exit 1
  GOL_SPLIT_VALUE_WAIT=1 GOL_SCHEDULE=split bash tools/trace_run.sh selfx_vw --self-exchange > /dev/null || exit 1
  GOL_SPLIT_VALUE_WAIT=1 GOL_SCHEDULE=split bash tools/trace_run.sh t2d_vw --size 32768 --width 16384 --decomp 2d --self-exchange > /dev/null || exit 1
  cat gpurun_out/trace_selfx_vw.txt gpurun_out/trace_t2d_vw.txt >> $S
  ;;
b34)
  # the value wait as the default: the whole GPU suite, then the per-rank tiles through the auto schedule timing and the
  # driver's command
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "== pytest -m gpu rc=$rc: $(tail -1 $O/pytest_gpu.log)" >> $S; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
  echo "== smoke rc=$rc: $(tail -1 $O/smoke.log)" >> $S; fatal $rc && exit $rc
  reps 3 "--self-exchange" "--size 32768 --width 16384 --decomp 2d --self-exchange" "--size 4096 --width 32768 --self-exchange" "" || exit 1
  ;;
b35)
  # (GOL_SPLIT_KERNEL_SIGNAL and the tile kernels' signal_done epilogue were removed after this batch: profiles/split_order_round6.txt, b35)
  # the split bands' tile kernel publishes the stream value itself (last workgroup, GOL_SPLIT_KERNEL_SIGNAL=1): one small
  # test under a short limit first, then the split tests, then the A/B against the runtime's write and traces
  timeout -k 10 150 python -u -m pytest -x -v --timeout 60 --timeout-method thread 'tests/test_gpu_rccl.py::test_rccl_split_order_knobs[1d-0-0-1-1]' > $O/first.log 2>&1; rc=$?
  echo "== first test rc=$rc: $(tail -1 $O/first.log)" >> $S; [ $rc -ne 0 ] && exit $rc
  pyt ksig_tests.log tests/test_gpu_rccl.py tests/test_gpu_multirank_p8.py -k "split or 2d or p8 or confirm" || exit 1
  reps 3 "--self-exchange" "GOL_SPLIT_KERNEL_SIGNAL=0 --self-exchange" \
    "--size 32768 --width 16384 --decomp 2d --self-exchange" "GOL_SPLIT_KERNEL_SIGNAL=0 --size 32768 --width 16384 --decomp 2d --self-exchange" || exit 1
  GOL_SCHEDULE=split bash tools/trace_run.sh selfx_ksig --self-exchange > /dev/null || exit 1
  GOL_SCHEDULE=split bash tools/trace_run.sh t2d_ksig --size 32768 --width 16384 --decomp 2d --self-exchange > /dev/null || exit 1
  cat gpurun_out/trace_selfx_ksig.txt gpurun_out/trace_t2d_ksig.txt >> $S
  ;;
b36)
  # config 3's strip: the auto cut (one step_pipe pass of 20) against forced pass depths, now that a multi-pass split
  # superstep runs its bands beside the interior; 2 interleaved rounds
  reps 2 "--size 4096 --width 32768 --self-exchange" "--kernel-depth 12 --size 4096 --width 32768 --self-exchange" \
    "--kernel-depth 10 --size 4096 --width 32768 --self-exchange" "--kernel-depth 8 --size 4096 --width 32768 --self-exchange" || exit 1
  ;;
b3)
  # full+gate (exchange flag gating the first pass's ghost-row segments), the pair rule in tile/pipe only, the
  # widened step_pipe pass-cost candidates: tests, then the driver's cut on the weak-scaling rank and the strip
  pyt gate_tests.log tests/test_gpu_rccl.py tests/test_gpu_gate_p8.py tests/test_gpu_multirank_p8.py tests/test_gpu_pipe.py || exit 1
  reps 3 "" "--self-exchange" "GOL_SCHEDULE=gate --self-exchange" "GOL_SCHEDULE=gate GOL_GATE_ORDER=1 --self-exchange" "--size 4096 --width 32768 --self-exchange" || exit 1
  reps 1 "--size 8192 --steps 1000" "--size 32768 --width 16384 --decomp 2d --self-exchange" || exit 1
  ;;
b4)
  # full+gate with upward-streaming top segments and a mid-stream gate (ROWS_GATE); BASELINE config 5 on the
  # round-6 tree (the 2^20-row tile: its init runs predict_run's no-snapshot branch)
  pyt gate_tests.log tests/test_gpu_rccl.py tests/test_gpu_gate_p8.py tests/test_gpu_multirank_p8.py -k "gate or p8" || exit 1
  reps 3 "--self-exchange" "GOL_SCHEDULE=gate --self-exchange" "" || exit 1
  reps 2 "--size 4096 --width 32768 --self-exchange" "GOL_SCHEDULE=gate --size 4096 --width 32768 --self-exchange" || exit 1
  GOL_INIT_LOG=1 timeout -k 10 900 python3 bench.py --size 1048576 --steps 16 --warmup 8 > $O/cfg5.json 2> $O/cfg5.err; rc=$?
  { echo "== config 5 (bench.py --size 1048576 --steps 16 --warmup 8) rc=$rc: init $(grep -c 'init' $O/cfg5.err) timed init steps, last: $(grep 'init' $O/cfg5.err | tail -1)"; grep -h '^{' $O/cfg5.json | python3 tools/bench_line.py cfg5; } >> $S
  fatal $rc && exit $rc
  ;;
b5)
  # kernel traces of the weak-scaling rank's driver cut through the RCCL self-exchange: full+gate vs full+graph
  for v in 1 2; do
    GOL_SCHEDULE=gate GOL_SUBTILES=0 bash tools/trace_run.sh gate$v --self-exchange > /dev/null || exit 1
    GOL_GATE=0 GOL_SUBTILES=0 bash tools/trace_run.sh graph$v --self-exchange > /dev/null || exit 1
  done
  cat gpurun_out/trace_gate1.txt gpurun_out/trace_graph1.txt gpurun_out/trace_gate2.txt gpurun_out/trace_graph2.txt >> $S
  ;;
b6)
  # full+gate, passes replayed from captured graphs (flag values 1/2 alternating), exchange eager on the comm stream
  pyt gate_tests.log tests/test_gpu_rccl.py tests/test_gpu_gate_p8.py tests/test_gpu_multirank_p8.py -k "gate or p8" || exit 1
  reps 3 "--self-exchange" "GOL_SCHEDULE=gate --self-exchange" "" || exit 1
  reps 2 "--size 4096 --width 32768 --self-exchange" "GOL_SCHEDULE=gate --size 4096 --width 32768 --self-exchange" || exit 1
  GOL_SCHEDULE=gate bash tools/trace_run.sh gate_graph --self-exchange > /dev/null || exit 1
  cat gpurun_out/trace_gate_graph.txt >> $S
  # step_pipe wait attribution (diagnostic build -DGOL_PIPE_STAMPS): 32768^2 8 x 3 at 2/CU, the strip's 10 x 2
  { echo "== kbench_stamps 32768^2 step_pipe<9,3> 2/CU"; KB_PIPE=3 KB_PIPE_WG=2 KB_PIPE_STAMPS=1 timeout -k 5 90 build/kbench_stamps 32768 24 960 0 0 9; } >> $S 2>&1 || exit 1
  { echo "== kbench_stamps 4096 x 32768 step_pipe<11,2> 1/CU"; KB_W=32768 KB_PIPE=2 KB_PIPE_STAMPS=1 timeout -k 5 90 build/kbench_stamps 4096 20 960 0 0 11; } >> $S 2>&1 || exit 1
  ;;
b7)
  # the round-6 tree without full+gate: the whole GPU suite; config 3's strip six times in sequence, traced
  # (the outlier hunt), one with the init log (the widened step_pipe pass-cost sweep); the driver's command;
  # config 2 through the CLI; the other per-rank tiles
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "== pytest -m gpu rc=$rc: $(tail -1 $O/pytest_gpu.log)" >> $S; [ $rc -ne 0 ] && exit $rc
  for v in 1 2 3 4 5 6; do
    bash tools/trace_run.sh strip$v --size 4096 --width 32768 --self-exchange > /dev/null || exit 1
    cat gpurun_out/trace_strip$v.txt >> $S
  done
  GOL_INIT_LOG=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --size 4096 --width 32768 --self-exchange > $O/strip_initlog.json 2> $O/strip_initlog.err || exit 1
  grep -h '^{' $O/strip_initlog.json | python3 tools/bench_line.py strip_initlog >> $S
  reps 3 "" || exit 1
  for v in 1 2; do timeout -k 10 120 build/gol 5 8192 1000 256 0 > $O/cfg2_cli_$v.log 2>&1 || exit 1; echo "[cfg2 CLI gol 5 8192 1000 256 0] $(grep TOTAL $O/cfg2_cli_$v.log)" >> $S; done
  reps 1 "--size 8192 --steps 1000" "--size 8192 --width 32768 --self-exchange" "--size 16384 --width 32768 --self-exchange" "--size 32768 --width 16384 --decomp 2d --self-exchange" "--size 32768 --steps 2000 --warmup 200" || exit 1
  ;;
b8)
  # evidence: smoke, the driver's command x5, BASELINE configs 1/3/4 (tools/baseline_configs.sh), a rocprofv3
  # kernel-trace/stats profile of the driver's command, and a PMC A/B of the pair rule (kbench r0 vs r1)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
  echo "== smoke rc=$rc: $(tail -1 $O/smoke.log)" >> $S; fatal $rc && exit $rc
  reps 5 "" || exit 1
  bash tools/baseline_configs.sh cfg1 cfg3 cfg4 > $O/configs.log 2>&1; rc=$?
  { echo "== BASELINE configs rc=$rc"; echo "cfg1: $(grep -h TOTAL gpurun_out/configs/cfg1_cpu_256.log)"; for f in gpurun_out/configs/cfg3_bench_32768.log gpurun_out/configs/cfg4_bench_65536_2d.log; do grep -h '^{' $f | python3 tools/bench_line.py "$(basename $f .log)"; done; } >> $S; fatal $rc && exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1; rc=$?
  echo "== rocprofv3 --kernel-trace --stats of the driver command rc=$rc: $(grep -h '^{' $O/prof.log | python3 tools/bench_line.py prof)" >> $S; fatal $rc && exit $rc
  ctr="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_WAVE_CYCLES"
  for v in r0 r1; do
    KB_FOLD=1 timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_f32_$v -o p --output-format csv -- build/kbench_$v 8192 32 960 0 0 8 0 4 > $O/pmc_f32_$v.log 2>&1 || exit 1
    KB_W=32768 KB_PIPE=2 timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_p20_$v -o p --output-format csv -- build/kbench_$v 4096 20 960 0 0 11 > $O/pmc_p20_$v.log 2>&1 || exit 1
  done
  for f in $(find $O -name "*counter_collection.csv" | sort); do echo "== $f"; python3 tools/pmc_summary.py "$f" | grep -A12 "step_tile_fold\|step_pipe"; done >> $O/pmc_summary.txt 2>&1
  # 8192^2 folded tiles with the pair rule: 8 vs 16 waves per workgroup (the 16-wave LV = 4 kernel now 101 VGPRs)
  for round in 1 2; do for nw in 8 16; do for k in 24 32; do
    echo "[kb fold nw=$nw K=$k] $(KB_FOLD=1 timeout -k 5 90 build/kbench_r1 8192 $k 1920 0 0 $nw 0 4 2>&1 | tail -1 | grep -o '"us_per_gen": [0-9.]*')" >> $S
  done; done; done
  ;;
*) echo "unknown batch $B"; exit 2 ;;
esac
cat $S
