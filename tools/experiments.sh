#!/bin/bash
# Experiment scripts (rounds 1-2), one function each: bash tools/experiments.sh <name> [args].
# Each was a standalone tools/<name>.sh; the profiles/ files they produced cite them by name.
# GPU steps run through gpurun on the box; every one has its own timeout.

cmd_cfg2_check() {
# BASELINE config 2 on one GPU: bench.py at 8192^2 and the reference CLI (8192^2 x 1000).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg2
timeout -k 10 120 python bench.py --size 8192 --steps 2000 --warmup 200 > gpurun_out/cfg2/bench8192.log 2>&1 || exit 3
for i in 1 2 3; do timeout -k 10 120 ./build/gol 5 8192 1000 256 0 >> gpurun_out/cfg2/cli8192.log 2>&1 || exit 3; done
grep '^{' gpurun_out/cfg2/bench8192.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('bench8192', round(d['ms_per_step']*1e3,3), 'us/gen', c['kernel'], c['kernel_depth'], c['halo_depth'], c['graph_launches'])"
grep TOTAL gpurun_out/cfg2/cli8192.log
}

cmd_cfg2_steps_ab() {
# Config 2 board: bench.py at 1000 vs 2000 timed steps and the CLI, alternating (fixed per-run cost of the bench path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg2steps
for rep in 1 2; do
  for st in 1000 2000; do
    timeout -k 10 120 python bench.py --size 8192 --steps $st --warmup 100 > gpurun_out/cfg2steps/b.log 2>&1 || exit 3
    grep '^{' gpurun_out/cfg2steps/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('bench steps=$st', round(d['ms_per_step']*1e3,4), 'us/gen', 'graph_launches', c['graph_launches'])"
  done
  timeout -k 10 120 ./build/gol 5 8192 1000 256 0 | grep TOTAL || exit 3
done | tee gpurun_out/cfg2steps/ab.txt
}

cmd_cfg2_sweep() {
# Config-2 sweep of bench.py at 8192^2: kernel:halo-depth:kernel-depth specs (auto vs fixed tile depths).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg2
for spec in "auto:16:0" "tile:16:16" "tile:32:32" "tile:32:16" "tile:24:24"; do
  IFS=: read kern R K <<< "$spec"
  timeout -k 10 120 python bench.py --size 8192 --steps 2000 --warmup 200 --kernel $kern --halo-depth $R --kernel-depth $K > gpurun_out/cfg2/$kern-$R-$K.log 2>&1 || { echo "$spec failed"; tail -3 gpurun_out/cfg2/$kern-$R-$K.log; continue; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/cfg2/$kern-$R-$K.log') if l.startswith('{')][-1]); c=d['config']; print('$spec %.4e %.3f us/gen kernel=%s K=%s waves=%s %s' % (d['value'], d['ms_per_step']*1e3, c['kernel'], c['kernel_depth'], c['tile_waves'], c['autotune'][:100]))"
done
}

cmd_cfg2_trace() {
# Kernel trace of the BASELINE config-2 CLI run (gol 5 8192 1000 256 0): GPU idle between step
# kernels (graph replays vs eager launches).  Output: gpurun_out/cfg2_trace/*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cfg2_trace
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/cfg2_trace -o cli -- $R/build/gol 5 8192 1000 256 0 > $R/gpurun_out/cfg2_trace/cli.log 2>&1 || exit 3
f=$(find $R/gpurun_out/cfg2_trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_gaps.py $f 60 > $R/gpurun_out/cfg2_trace/gaps.txt
cat $R/gpurun_out/cfg2_trace/cli.log $R/gpurun_out/cfg2_trace/gaps.txt
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
st = [r for r in rows if "step_" in r["Kernel_Name"]][-60:]
prev = None
for r in st:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - prev) / 1e3 if prev else 0
    print(f"{(e - s) / 1e3:8.1f} us  gap {g:7.1f} us  {r['Kernel_Name'][:60]}")
    prev = e
PY
}

cmd_cfg2_warmup_ab() {
# bench.py at 8192^2, 1000 timed steps, warmup 0 / 96 / 100 / 200 (graph parity and eager remainders before the timed run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg2steps
for rep in 1 2; do
  for w in 0 96 100 200; do
    timeout -k 10 120 python bench.py --size 8192 --steps 1000 --warmup $w > gpurun_out/cfg2steps/w.log 2>&1 || exit 3
    grep '^{' gpurun_out/cfg2steps/w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('warmup=$w', round(d['ms_per_step']*1e3,4), 'us/gen', 'graph_launches', c['graph_launches'])"
  done
done | tee gpurun_out/cfg2steps/warmup_ab.txt
}

cmd_driver_trace() {
# Driver-style bench (bench.py --gpus 1 --steps 20 --warmup 5) three times, then a kernel trace of
# the same command (per-dispatch timeline of the timed region).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dtrace
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dtrace/bench_$i.json 2> gpurun_out/dtrace/bench_$i.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/dtrace/bench_$i.json')); print('run $i', d['ms_per_step']*1e3, 'us/gen', d['config']['schedule'])"
done
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dtrace/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dtrace/prof.log 2>&1
}

cmd_events_ab() {
# Full multi-rank schedule on one GPU (thread ranks, RCCL-semantics transport): ready-event record
# per superstep (GOL_READY_EVENTS=always) vs none (default), alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/events
out=gpurun_out/events/ab.txt; : > $out
for r in 1 2; do
  for ev in always default; do
    echo "== $ev" >> $out
    GOL_SCHEDULE=full GOL_READY_EVENTS=$ev timeout -k 10 200 python -u tools/rehearse_multirank.py --configs 1d:2:32768,1d:4:32768 --gens 2560 >> $out 2>&1 || exit 3
  done
done
cat $out
}

cmd_fold_ab() {
# Folded tile kernel (STEP_TILE_FOLD) vs the tile kernel: correctness (KB_CHECK=1: K generations vs K
# single-generation temporal passes, every word) and alternating timing at 8192^2 and the 4096 x 32768
# strip of config 3 strong-scaled over 8 GPUs.  kbench args: N K gens pf skew nw rows lv.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fold
export TMPDIR=/tmp
K() { timeout -k 5 60 build/kbench_main "$@"; }
set -o pipefail
{
echo "## correctness"
for cfg in "8192 24 960 0 0 8 0 4" "8192 16 960 0 0 8 0 2" "8192 7 960 0 0 4 0 1" "4096 24 960 0 0 8 0 4" "1024 9 960 0 0 8 0 4" "3072 13 960 0 0 8 0 2"; do
  echo "fold $cfg"; KB_CHECK=1 KB_FOLD=1 K $cfg || exit $?
done
echo "base 8192 24 960 0 0 8 0 4"; KB_CHECK=1 K 8192 24 960 0 0 8 0 4 || exit $?
echo "## timing 8192^2 (us/gen)"
for rep in 1 2; do
  for k in 16 24 32; do
    for nw in 8 16; do
      echo "base K=$k nw=$nw"; K 8192 $k 960 0 0 $nw 0 4 || exit $?
      echo "fold K=$k nw=$nw"; KB_FOLD=1 K 8192 $k 960 0 0 $nw 0 4 || exit $?
    done
  done
done
echo "## timing 4096 x 32768 (KB_W=32768)"
for k in 16 24 32; do
  echo "base K=$k"; KB_W=32768 K 4096 $k 960 0 0 8 0 4 || exit $?
  echo "base-inplace K=$k"; KB_INPLACE=1 KB_W=32768 K 4096 $k 960 0 0 8 0 4 || exit $?
  echo "fold K=$k"; KB_FOLD=1 KB_W=32768 K 4096 $k 960 0 0 8 0 4 || exit $?
done
} 2>&1 | tee gpurun_out/fold/fold_ab.txt
}

cmd_fold_check() {
# Folded tiles in the engine: GPU suite, config 2 (bench + CLI) with GOL_TILE_FOLD auto (=on) vs 0,
# alternating, and the driver command (unchanged path) for regressions.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/foldeng
export TMPDIR=/tmp
o=gpurun_out/foldeng
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for f in -1 0; do
    GOL_TILE_FOLD=$f timeout -k 10 120 python bench.py --size 8192 --steps 2000 --warmup 200 > $o/b8192_$f.log 2>&1 || exit 3
    grep '^{' $o/b8192_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('fold=$f bench8192', round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['kernel'], c['kernel_depth'], c['halo_depth'], c['autotune'])"
    for i in 1 2; do GOL_TILE_FOLD=$f timeout -k 10 120 ./build/gol 5 8192 1000 256 0 > $o/cli_$f.log 2>&1 || exit 3; echo "fold=$f cli $(grep TOTAL $o/cli_$f.log)"; done
  done
done
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/drv$i.log 2>&1 || exit 3
  grep '^{' $o/drv$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver', round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], d['config']['schedule'])"; done
}

cmd_fold_depth() {
# Folded tiles at 8192^2: pass depth 32 vs 40 / 48 / 64 (kbench, alternating, 8 waves, 4 levels per LDS pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fold
for rep in 1 2 3; do for k in 32 40 48 64; do
  echo "fold K=$k $(KB_FOLD=1 timeout -k 5 60 build/kbench_main 8192 $k 1920 0 0 8 0 4 | grep -o '"rows": [0-9]*\|"us_per_gen": [0-9.]*' | tr '\n' ' ')" || exit 1
done; done | tee gpurun_out/fold/fold_depth.txt
}

cmd_fold_strip() {
# The 4096 x 32768 per-rank strip (config 3 strong-scaled over 8 GPUs): folded in-place tiles (one
# round) vs the in-place tile kernel, alternating (kbench, KB_W=32768), with word-by-word checks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fold
K() { timeout -k 5 60 build/kbench_main "$@"; }
{
for cfg in "4096 24 960 0 0 8 0 2" "4096 13 960 0 0 8 0 4" "2048 7 960 0 0 16 0 2"; do
  echo "check fold-inplace $cfg"; KB_CHECK=1 KB_INPLACE=1 KB_FOLD=1 KB_W=32768 K $cfg || exit $?
done
for rep in 1 2; do
  for k in 16 24 32; do
    for lv in 2 4; do
      echo "fold-inplace K=$k lv=$lv"; KB_INPLACE=1 KB_FOLD=1 KB_W=32768 K 4096 $k 960 0 0 8 0 $lv || exit $?
    done
    echo "base-inplace K=$k lv=2"; KB_INPLACE=1 KB_W=32768 K 4096 $k 960 0 0 8 0 2 || exit $?
  done
done
} 2>&1 | tee gpurun_out/fold/fold_strip.txt
}

cmd_kb_ab() {
# Generic A/B of two kbench builds, alternating on one box: tools/experiments.sh kb_ab <a> <b> [rounds]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_ab_$1_$2.txt; : > $out
for r in $(seq ${3:-3}); do
  for v in $1 $2; do
    echo "== $v" >> $out
    timeout -k 5 60 build/kbench_$v 32768 8 1920 >> $out 2>&1 || exit 3
    timeout -k 5 60 build/kbench_$v 16384 8 1920 >> $out 2>&1 || exit 3
    timeout -k 5 60 build/kbench_$v 65536 8 480 >> $out 2>&1 || exit 3
  done
done
cat $out
}

cmd_kb_bperm() {
# A/B: DPP lane exchange (kbench_dpp) vs ds_bpermute (kbench_bperm), alternating on one box.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_bperm.txt; : > $out
for v in dpp bperm dpp bperm; do
  echo "== $v" >> $out
  timeout -k 5 60 build/kbench_$v 32768 8 960 >> $out 2>&1 || exit 3
  timeout -k 5 60 build/kbench_$v 32768 8 960 0 1 >> $out 2>&1 || exit 3
  timeout -k 5 60 build/kbench_$v 65536 8 480 >> $out 2>&1 || exit 3
  timeout -k 5 60 build/kbench_$v 8192 24 1920 0 0 8 0 2 >> $out 2>&1 || exit 3
done
cat $out
}

cmd_kb_depth_sweep() {
# Per-pass-depth throughput of step_temporal at 32768^2: one tile vs two half-tiles on two streams,
# plan occupancy (waves/SIMD) 2, 3, 4 and the kernel's own maximum.  Each line: us per generation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for K in 1 2 3 4 5 6 7 8; do
  for bpc in 2 3 4 8; do
    for s2 in 0 1; do
      r=$(KB_BPC=$bpc KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_main 32768 $K $((K*40)) 2>&1 | tail -1)
      echo "K=$K bpc=$bpc split2=$s2 $r"
    done
  done
done
}

cmd_kb_occ_sweep() {
# Temporal kernel: pass depth K x plan occupancy (waves per SIMD the one-round plan is sized for).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_occ_sweep.txt; : > $out
for N in 16384 32768 65536; do
  g=1920; [ $N = 65536 ] && g=480
  for K in 4 6 8; do
    for b in 1 2 3 4; do
      echo "== N=$N K=$K bpc=$b" >> $out
      KB_BPC=$b timeout -k 5 60 build/kbench_cur $N $K $((g / K * K)) >> $out 2>&1 || exit 3
    done
  done
done
cat $out
}

cmd_kb_rounds() {
# Temporal kernel: one-round plan vs 2-3 rounds of shorter segments (tail overlap vs more halo).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_rounds.txt; : > $out
for r in 1 2; do
  for rows in 0 45 30 60; do
    echo "== 32768 rows=$rows" >> $out
    timeout -k 5 60 build/kbench_cur 32768 8 1920 0 0 0 $rows >> $out 2>&1 || exit 3
    KB_BPC=2 timeout -k 5 60 build/kbench_cur 32768 8 1920 0 0 0 $rows >> $out 2>&1 || exit 3
  done
done
cat $out
}

cmd_kb_split2() {
# One kernel per pass over the whole board vs two concurrent half-board kernels (two streams, each a
# one-round plan for the whole GPU, no cross-stream ordering: the timing of two sub-tiles per GPU).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_split2.txt; : > $out
for r in 1 2 3; do
  for sp in 0 1; do
    for b in 3 2; do
      echo "== split2=$sp bpc=$b" >> $out
      KB_SPLIT2=$sp KB_BPC=$b timeout -k 5 60 build/kbench_cur 32768 8 3840 >> $out 2>&1 || exit 3
    done
  done
done
cat $out
}

cmd_kb_tile_sweep() {
# Tile-kernel sweep at 8192^2 (BASELINE config 2): depth K x waves per workgroup x tile rows, LV=2.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_tile_sweep.txt; : > $out
for K in 16 24 32; do
  for nw in 4 8 16; do
    for rows in 0 34 23; do
      timeout -k 5 60 build/kbench_base 8192 $K 1920 0 0 $nw $rows 2 >> $out 2>&1 || exit 3
    done
  done
done
cat $out
}

cmd_occ_check() {
# bench.py at 8192^2 / 16384^2 / 32768^2 (autotune strings show the 3- vs 2-waves/SIMD temporal plans) and the
# one-GPU multi-rank rehearsal at strong-scaling tile sizes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/occ
for n in 8192 16384 32768; do
  timeout -k 10 120 python bench.py --size $n --steps 2000 --warmup 200 > gpurun_out/occ/b$n.log 2>&1 || exit 3
done
timeout -k 10 300 python -u tools/rehearse_multirank.py --configs 1d:8:32768,1d:4:32768 > gpurun_out/occ/rm.txt 2>&1 || exit 3
for f in gpurun_out/occ/b*.log; do grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$f', round(d['ms_per_step']*1e3,3), c['kernel'], c['kernel_depth'], c['autotune'])"; done
cat gpurun_out/occ/rm.txt
}

cmd_pmc_fold() {
# Folded tile kernel at 8192^2: levels-per-LDS-pass x waves sweep (kbench), then PMC of the folded
# (K=32, 8 waves, 4 levels) and plain (K=24, the previous auto choice) tile kernels.  One counter set
# per run, --kernel-trace only.  Output: gpurun_out/pmc_fold/*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/pmc_fold
mkdir -p $o
for k in 24 32; do for nw in 4 8; do for lv in 2 4; do
  echo "fold K=$k nw=$nw lv=$lv $(KB_FOLD=1 timeout -k 5 60 $R/build/kbench_main 8192 $k 960 0 0 $nw 0 $lv | grep -o '"us_per_gen": [0-9.]*')" || exit 1
done; done; done > $o/sweep.txt
cat $o/sweep.txt
pmc() {  # pmc <name> <counters> <env> -- <kbench args>
  local name=$1 ctr=$2 fold=$3; shift 3
  KB_FOLD=$fold timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $ctr -d $o/$name -o $name --output-format csv -- $R/build/kbench_main "$@" > $o/$name.log 2>&1 || { echo "$name failed"; return 1; }
  echo "$name ok"
}
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
B="SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES"
pmc fold_a "$A" 1 8192 32 480 0 0 8 0 4 && pmc fold_b "$B" 1 8192 32 480 0 0 8 0 4 &&
pmc plain_a "$A" 0 8192 24 480 0 0 8 0 4 && pmc plain_b "$B" 0 8192 24 480 0 0 8 0 4 &&
for n in fold_a fold_b plain_a plain_b; do
  f=$(find $o/$n -name '*counter_collection.csv' | head -1)
  echo "== $n"; python3 $R/tools/pmc_summary.py "$f"
done > $o/summary.txt
cat $o/summary.txt
}

cmd_pmc_k7() {
# Why is a K=7 step_temporal pass nearly as slow as K=8?  PMC of K=6, 7, 8 at 32768^2 (one tile, 3 waves/SIMD plans).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/pmc_k7
mkdir -p $o
for K in 6 7 8; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $o/k$K -o k$K --output-format csv -- $R/build/kbench_main 32768 $K $((K*24)) > $o/k$K.log 2>&1 || { echo "K=$K failed"; exit 1; }
  f=$(find $o/k$K -name '*counter_collection.csv' | head -1)
  echo "== K=$K $(grep us_per_gen $o/k$K.log | sed 's/.*"rows"/rows/' | cut -c1-120)"
  python3 $R/tools/pmc_summary.py "$f" | grep -A12 step_temporal
done
}

cmd_pmc_k7_after() {
# Why is a K=7 step_temporal pass nearly as slow as K=8?  PMC of K=6, 7, 8 at 32768^2 (one tile, 3 waves/SIMD plans).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/pmc_k7_after
mkdir -p $o
for K in 7 8 12; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $o/k$K -o k$K --output-format csv -- $R/build/kbench_main 32768 $K $((K*24)) > $o/k$K.log 2>&1 || { echo "K=$K failed"; exit 1; }
  f=$(find $o/k$K -name '*counter_collection.csv' | head -1)
  echo "== K=$K $(grep us_per_gen $o/k$K.log | sed 's/.*"rows"/rows/' | cut -c1-120)"
  python3 $R/tools/pmc_summary.py "$f" | grep -A12 step_temporal
done
}

cmd_pmc_temporal() {
# PMC counters of the hot kernels (kbench, 32768^2: temporal K=8; 8192^2: tile K=16).  Counter runs
# use --kernel-trace only (no sys/runtime traces).  Output: gpurun_out/pmc_temporal/*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/pmc_temporal
mkdir -p $o
pmc() {  # pmc <name> <counters> -- <kbench args>
  local name=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $o/$name -o $name --output-format csv -- $R/build/kbench_tile "$@" > $o/$name.log 2>&1
  echo "$name rc=$?"
}
pmc t_a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" 32768 8 240 0 0 0
pmc t_b "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" 32768 8 240 0 0 0
pmc t_c "FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE" 32768 8 240 0 0 0
pmc tile_a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" 8192 16 480 0 0 8 0 2
pmc tile_c "FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE" 8192 16 480 0 0 8 0 2
}

cmd_pmc_tile() {
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_tile
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_tile/a -o a --output-format csv -- $R/build/kbench_tile 32768 8 480 0 0 16 > $R/gpurun_out/pmc_tile/a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/pmc_tile/b -o b --output-format csv -- $R/build/kbench_tile 32768 8 480 0 0 16 > $R/gpurun_out/pmc_tile/b.log 2>&1 || exit $?
}

cmd_pmc_tile_round2() {
# PMC of the round-2 tile kernel at its auto configuration for 8192^2 (K=24, 8 waves, 4 generations
# per LDS pass, double-buffered), for comparison with the round-1 PMC (K=16, 2 per LDS pass).
# One counter set per run, --kernel-trace only.  Output: gpurun_out/pmc_tile_r2/*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/pmc_tile_r2
mkdir -p $o
pmc() {  # pmc <name> <counters> -- <kbench args>
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $ctr -d $o/$name -o $name --output-format csv -- $R/build/kbench_main "$@" > $o/$name.log 2>&1 || { echo "$name failed"; return 1; }
  echo "$name ok"
}
pmc tile_a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" 8192 24 480 0 0 8 0 4 &&
pmc tile_b "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" 8192 24 480 0 0 8 0 4 &&
pmc tile_old_a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" 8192 16 480 0 0 8 0 2 &&
pmc tile_old_b "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" 8192 16 480 0 0 8 0 2 &&
for n in tile_a tile_b tile_old_a tile_old_b; do
  f=$(find $o/$n -name '*counter_collection.csv' | head -1)
  echo "== $n"; python3 $R/tools/pmc_summary.py "$f"
done > $o/summary.txt
}

cmd_power_probe() {
# Clock/power while the flagship kernel runs flat out: a long bench in the background, rocm-smi
# samples every ~0.5 s (read-only queries).  Output: gpurun_out/power/*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/power
mkdir -p $o
rocm-smi --showpower --showclocks --showmaxpower > $o/idle.txt 2>&1
timeout -k 10 120 python bench.py --steps 300000 --warmup 400 > $o/bench_long.log 2>&1 &
pid=$!
for i in $(seq 1 40); do
  sleep 0.5
  kill -0 $pid 2>/dev/null || break
  { date +%T.%N; rocm-smi --showpower --showclocks 2>&1 | grep -E "Power|sclk|fclk|mclk"; } >> $o/samples.txt
done
wait $pid
echo "bench rc=$?"
tail -c 600 $o/bench_long.log
}

cmd_prof_ab() {
# Kernel-trace A/B: the standalone kbench timing loop vs the engine (bench.py) on the same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kb -o kb --output-format csv -- build/kbench_tile 32768 8 960 > gpurun_out/prof_kb.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python3 bench.py --steps 2000 --warmup 200 > gpurun_out/prof_bench.log 2>&1 || exit 3
grep -h step_temporal gpurun_out/prof_kb/kb_kernel_stats.csv gpurun_out/prof_bench/bench_kernel_stats.csv
}

cmd_split_bench() {
# Host-timed bench of the split (multi-GPU) schedule on one GPU, no profiler.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/split_bench; mkdir -p $o
for v in "nosplit:GOL_FORCE_SPLIT=0" "split_R8:GOL_FORCE_SPLIT=1 GOL_HALO_DEPTH=8" \
         "split_R32K8:GOL_FORCE_SPLIT=1 GOL_HALO_DEPTH=32 GOL_KERNEL_DEPTH=8" \
         "split_R64K8:GOL_FORCE_SPLIT=1 GOL_HALO_DEPTH=64 GOL_KERNEL_DEPTH=8" \
         "nosplit_R32K8:GOL_FORCE_SPLIT=0 GOL_HALO_DEPTH=32 GOL_KERNEL_DEPTH=8" \
         "split_R32K8_8192:GOL_FORCE_SPLIT=1 GOL_HALO_DEPTH=32 GOL_KERNEL_DEPTH=8 --size 8192" \
         "nosplit_8192:GOL_FORCE_SPLIT=0 --size 8192"; do
  name=${v%%:*}; rest=${v#*:}
  envs=$(echo $rest | tr ' ' '\n' | grep '=' | tr '\n' ' '); args=$(echo $rest | tr ' ' '\n' | grep -v '=' | tr '\n' ' ')
  timeout -k 10 300 env $envs python bench.py --steps 2048 --warmup 256 $args > $o/$name.log 2>&1 || exit $?
  echo "$name $(grep -o '"value": [0-9.e+]*\|"kernel": "[^"]*"' $o/$name.log | tr '\n' ' ')"
done
}

cmd_split_cost() {
# Cost of the multi-GPU superstep structure on one GPU (GOL_FORCE_SPLIT=1: interior/boundary split,
# comm stream and cross-stream events with an empty exchange), eager vs graph-replayed, 32768^2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/split_cost
mkdir -p $o
run() {  # run <name> <env...> -- <bench args>
  local name=$1; shift
  timeout -k 10 180 env "$@" > $o/$name.log 2>&1
  local rc=$?
  python3 -c "import json,sys; d=json.loads([l for l in open('$o/$name.log') if l.startswith('{')][-1]); c=d['config']; print('%-22s %.4e  %.3f us/gen  sched=%s kernel=%s graphs=%s' % ('$name', d['value'], d['ms_per_step']*1e3, c['schedule'], c['kernel'], c['graph_launches']))" || { echo "$name rc=$rc"; tail -5 $o/$name.log; }
  [ $rc -ge 124 ] && exit $rc
  return 0
}
B="python bench.py --steps 4000 --warmup 400 --halo-depth 32"
run unsplit_graph   GOL_FORCE_SPLIT=0 $B
run unsplit_eager   GOL_FORCE_SPLIT=0 $B --no-graph
run split_graph     GOL_FORCE_SPLIT=1 $B
run split_eager     GOL_FORCE_SPLIT=1 $B --no-graph
run split_eager_devscope GOL_FORCE_SPLIT=1 GOL_EVENT_SCOPE=device $B --no-graph
}

cmd_split_cost_r() {
# Split-schedule cost vs halo depth R (GOL_FORCE_SPLIT=1, eager supersteps as on multi-GPU runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/split_cost
mkdir -p $o
for R in 32 48 64; do
  timeout -k 10 180 env GOL_FORCE_SPLIT=1 python bench.py --steps 4000 --warmup 400 --halo-depth $R --no-graph > $o/split_r$R.log 2>&1 || exit 3
  python3 -c "import json; d=json.loads([l for l in open('$o/split_r$R.log') if l.startswith('{')][-1]); c=d['config']; print('R=$R %.4e %.3f us/gen kernel=%s' % (d['value'], d['ms_per_step']*1e3, c['kernel']))"
done
}

cmd_split_trace() {
# Kernel timelines of the interior/boundary edge schedule on one GPU (GOL_FORCE_SPLIT=1).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/split
mkdir -p $o
run() {  # run <name> <env...>
  local name=$1; shift
  timeout -k 10 300 env "$@" rocprofv3 --kernel-trace -d $o/$name -o $name --output-format csv -- python3 $R/bench.py --steps 400 --warmup 40 > $o/$name.log 2>&1 || exit $?
}
run nosplit GOL_FORCE_SPLIT=0
run split_graph GOL_FORCE_SPLIT=1
run split_nograph GOL_FORCE_SPLIT=1 GOL_GRAPH=0
run split_nograph_nomask GOL_FORCE_SPLIT=1 GOL_GRAPH=0 GOL_EDGE_CUS=0
}

cmd_subtiles_check() {
# GOL_SUBTILES=2 (two half-tiles per rank on two streams) vs one tile: bench.py at 32768^2 / 16384^2,
# halo depth 32 and 64, alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sub
out=gpurun_out/sub/bench.txt; : > $out
for r in 1 2; do
  for n in 32768 16384; do
    for cfg in 0:0 2:0 2:64; do
      sub=${cfg%%:*}; hd=${cfg#*:}
      GOL_SUBTILES=$sub GOL_HALO_DEPTH=$hd timeout -k 10 150 python bench.py --size $n --steps 2048 --warmup 128 > gpurun_out/sub/b.log 2>&1 || { tail -5 gpurun_out/sub/b.log; exit 3; }
      grep '^{' gpurun_out/sub/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('sub=$sub R=$hd', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['kernel'], c['schedule'])" >> $out
    done
  done
done
cat $out
}

cmd_subtiles_check2() {
# GOL_SUBTILES=2 at 65536^2 and 32768^2 (R=64) vs one tile, and thread ranks (1-D P=2) with sub-tiles.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sub
out=gpurun_out/sub/bench2.txt; : > $out
for r in 1 2; do
  for cfg in 65536:0:0 65536:2:64 32768:0:0 32768:2:64; do
    IFS=: read n sub hd <<< "$cfg"
    st=1024; [ $n = 65536 ] && st=256
    GOL_SUBTILES=$sub GOL_HALO_DEPTH=$hd timeout -k 10 150 python bench.py --size $n --steps $st --warmup 64 > gpurun_out/sub/b.log 2>&1 || { tail -5 gpurun_out/sub/b.log; exit 3; }
    grep '^{' gpurun_out/sub/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('sub=$sub R=$hd', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['schedule'])" >> $out
  done
done
for sub in 0 2; do
  GOL_SUBTILES=$sub GOL_SCHEDULE=full timeout -k 10 200 python -u tools/rehearse_multirank.py --configs 1d:2:32768 --gens 2560 | sed "s/^/sub=$sub /" >> $out || exit 3
done
cat $out
}

cmd_subtiles_occ() {
# Two sub-tiles: halves planned for 2 waves/SIMD (default) vs the single-tile tuned occupancy, alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sub
out=gpurun_out/sub/occ.txt; : > $out
for r in 1 2 3; do
  for so in 2 3; do
    GOL_SUB_OCC=$so timeout -k 10 150 python bench.py --size 32768 --steps 2048 --warmup 128 > gpurun_out/sub/b.log 2>&1 || { tail -5 gpurun_out/sub/b.log; exit 3; }
    grep '^{' gpurun_out/sub/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('sub_occ=$so', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['schedule'])" >> $out
  done
done
for so in 2 3; do
  GOL_SUB_OCC=$so timeout -k 10 150 python bench.py --size 65536 --steps 256 --warmup 32 > gpurun_out/sub/b.log 2>&1 || exit 3
  grep '^{' gpurun_out/sub/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('sub_occ=$so', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['schedule'])" >> $out
done
cat $out
}

cmd_subtiles_r128() {
# Two sub-tiles: 64- vs 128-generation supersteps (the streams meet once per superstep), alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sub
out=gpurun_out/sub/r128.txt; : > $out
for r in 1 2 3; do
  for hd in 64 128; do
    GOL_HALO_DEPTH=$hd timeout -k 10 150 python bench.py --size 32768 --steps 2048 --warmup 128 > gpurun_out/sub/b.log 2>&1 || { tail -5 gpurun_out/sub/b.log; exit 3; }
    grep '^{' gpurun_out/sub/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('R=$hd', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['schedule'])" >> $out
  done
done
cat $out
}

cmd_sync_spin_ab() {
# Driver command with GOL_SYNC_SPIN=0 (hipStreamSynchronize) vs 1 (busy-poll hipStreamQuery first), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/spin
for i in 1 2 3 4; do for v in 0 1; do
  GOL_SYNC_SPIN=$v timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/spin/b_$v_$i.log 2>&1 || exit 3
  grep '^{' gpurun_out/spin/b_$v_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('spin=$v', round(d['ms_per_step']*1e3,3), 'us/gen')"
done; done | tee gpurun_out/spin/ab.txt
}

cmd_tune_check() {
# bench.py three times at 32768^2 and once at 16384^2 / 8192^2: autotune picks and their stability.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
for n in 32768 32768 32768 16384 8192; do
  timeout -k 10 120 python bench.py --size $n --steps 2000 --warmup 200 >> gpurun_out/tune/b.log 2>&1 || exit 3
done
grep '^{' gpurun_out/tune/b.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); c=d['config']; print(c['board'][0], round(d['ms_per_step']*1e3,3), c['kernel'], c['kernel_depth'], c['autotune'][:150])"
}

cmd_oneshot() {
# Round 3: one-shot full-board passes at 32768^2 (one launch per timed rep, best of 3): the pass kernels a
# 20-generation run could use, temporal K=8/12 and step_pipe geometries (NW x L at 1-2 workgroups per CU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/oneshot
out=gpurun_out/oneshot/oneshot.txt; : > $out
kb=build/kbench_${1:-default}
for rep in 1 2; do
  for spec in "t:8" "t:12" "t:16" "p:9:3:2" "p:9:3:1" "p:11:2:1" "p:11:2:2" "p:5:4:2" "p:9:2:2" "p:13:2:1" "p:9:32:2" "p:9:32:1"; do
    IFS=: read kind a b c <<< "$spec"
    if [ $kind = t ]; then
      r=$(timeout -k 5 60 $kb 32768 $a $a) || exit 3
    else
      if [ $b -ge 10 ]; then k=$(( (a - 1) / 2 * (b / 10) + (a - 1 - (a - 1) / 2) * (b % 10) )); else k=$(( (a - 1) * b )); fi
      r=$(KB_PIPE=$b KB_PIPE_WG=$c timeout -k 5 60 $kb 32768 $k $k 0 0 $a) || exit 3
    fi
    echo "$spec $r" | python3 -c "
import sys,json
l=sys.stdin.read(); sp,js=l.split(' ',1); d=json.loads(js)
print(sp, 'K', d['K'], 'pass_us', round(d['us_per_gen']*d['K'],1), 'us_per_gen', d['us_per_gen'], 'bpc', d['blocks_per_cu'])" | tee -a $out
  done
done
}

cmd_bigboard_rounds() {
# Round 3: one-tile K=8 passes on big boards, kbench: one-round plan (default rows) vs multi-round plans (fewer rows per
# wave) vs two concurrent half-board kernels on two streams (KB_SPLIT2=1, no cross-stream ordering: an upper bound).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bigb
out=gpurun_out/bigb/bigboard_rounds.txt; : > $out
kb=build/kbench_${1:-default}
for rep in 1 2; do
  for n in 65536 131072; do
    for rows in 0 720 360 180; do
      r=$(timeout -k 5 120 $kb $n 8 64 0 0 0 $rows) || exit 3
      echo "N=$n rows=$rows $r" | tee -a $out
    done
    r=$(KB_SPLIT2=1 timeout -k 5 120 $kb $n 8 64) || exit 3
    echo "N=$n split2 $r" | tee -a $out
  done
done
}

cmd_rounds_engine() {
# Round 3: the engine with multi-round plans for big tiles (default, GOL_ROUND_ROWS_PER_LEVEL=45) vs one round (=0):
# bench.py at 131072^2 with one tile (GOL_SUBTILES=0) and BASELINE config 5 (2^20 x 2^20, 256 GB of boards); the driver
# command as a check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rounds
out=gpurun_out/rounds/rounds_engine.txt; : > $out
summ() { grep '^{' "$1" | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); c=d['config']
print('$2', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.4e'%d['value'], c['schedule'], 'plan_waves', c['plan_waves'], 'init_s', d['timing']['init_s'], c['autotune'][:160])" | tee -a $out; }
for rep in 1 2; do
  for v in 45 0; do
    GOL_SUBTILES=0 GOL_ROUND_ROWS_PER_LEVEL=$v timeout -k 10 240 python bench.py --size 131072 --steps 256 --warmup 32 > gpurun_out/rounds/b131k_$v.log 2>&1 || exit 3
    summ gpurun_out/rounds/b131k_$v.log "onetile rr=$v"
  done
done
for v in 45 0; do
  GOL_INIT_LOG=1 GOL_ROUND_ROWS_PER_LEVEL=$v timeout -k 10 400 python bench.py --size 1048576 --steps 16 --warmup 8 > gpurun_out/rounds/b1m_$v.log 2>&1 || exit 3
  summ gpurun_out/rounds/b1m_$v.log "cfg5 rr=$v"
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rounds/drv.log 2>&1 || exit 3
  summ gpurun_out/rounds/drv.log driver
done
}

cmd_launch_trace() {
# Round 3: where the driver command's ~15 us from run() to the first kernel go: roctx marks around the first launch of the
# sub-tile superstep (host side) vs the first kernel's start (kernel trace), three traced runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ltrace
: > gpurun_out/ltrace/summary.txt
export TMPDIR=/tmp GOL_ROCTX=1
for kv in "${@:-X=0}"; do
for i in 1 2 3; do
  rm -rf gpurun_out/ltrace/p$i
  echo "== $kv run $i" | tee -a gpurun_out/ltrace/summary.txt
  export "$kv"
  timeout -k 10 180 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/ltrace/p$i -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-phases > gpurun_out/ltrace/b$i.log 2>&1 || exit 3
  python3 tools/timed_trace.py gpurun_out/ltrace/p$i | tail -5 | tee -a gpurun_out/ltrace/summary.txt
done
done
unset GOL_ROCTX
for rep in 1 2 3; do
  for kv in "${@:-X=0}"; do
    env "$kv" timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ltrace/d.log 2>&1 || exit 3
    grep '^{' gpurun_out/ltrace/d.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('driver $kv', round(d['ms_per_step']*1e3,3), 'us/gen')" | tee -a gpurun_out/ltrace/summary.txt
  done
done
}

cmd_end_sync_ab() {
# Round 3: the driver command with the engine's stream syncs + torch's device sync after the timed run (both) vs torch's
# device sync alone (torch), alternating; then a check that torch's sync alone waits for the engine's streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/esync
out=gpurun_out/esync/end_sync.txt; : > $out
for rep in $(seq ${1:-4}); do
  for v in both torch; do
    BENCH_END_SYNC=$v timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/esync/d.log 2>&1 || exit 3
    grep '^{' gpurun_out/esync/d.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step']*1e3,3), 'us/gen')" | tee -a $out
  done
done
timeout -k 10 120 python tools/sync_check.py | tee -a $out
}

cmd_driver_ab() {
# Round 3: the driver command with extra bench.py flags (or one VAR=value environment setting) A vs B, alternating pairs:
# tools/experiments.sh driver_ab "<A>" "<B>" [pairs]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dab
out=gpurun_out/dab/driver_ab.txt; : > $out; : > gpurun_out/dab/detail.txt
for rep in $(seq ${3:-8}); do
  for v in "$1" "$2"; do
    case "$v" in *=*) ev="$v"; fl="";; *) ev="X_AB=1"; fl="$v";; esac
    env "$ev" timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 $fl > gpurun_out/dab/d.log 2>&1 || exit 3
    grep '^{' gpurun_out/dab/d.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('[$v]', round(d['ms_per_step']*1e3,3))" | tee -a $out
    grep '^{' gpurun_out/dab/d.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); c=d['config']; print(round(d['ms_per_step']*1e3,3), c['schedule'], c['kernel'], c['kernel_depth'], c['plan_waves'], ' '.join(x for x in c['autotune'].split() if x.startswith(('sched:','pass8','pass12','0:temporal'))), 'init', d['timing']['init_s'])" >> gpurun_out/dab/detail.txt
  done
done
python3 - $out <<'PY'
import sys
from statistics import mean, median
d = {}
for l in open(sys.argv[1]):
    k, v = l.rsplit(' ', 1)
    d.setdefault(k, []).append(float(v))
for k, v in d.items():
    print(k, len(v), 'mean %.3f median %.3f min %.3f max %.3f' % (mean(v), median(v), min(v), max(v)))
PY
}

name=${1:-}; shift || true
if ! declare -F "cmd_$name" >/dev/null; then
  echo "usage: $0 <name> [args]; names: driver_ab end_sync_ab launch_trace rounds_engine oneshot bigboard_rounds cfg2_check cfg2_steps_ab cfg2_sweep cfg2_trace cfg2_warmup_ab driver_trace events_ab fold_ab fold_check fold_depth fold_strip kb_ab kb_bperm kb_depth_sweep kb_occ_sweep kb_rounds kb_split2 kb_tile_sweep occ_check pmc_fold pmc_k7 pmc_k7_after pmc_temporal pmc_tile pmc_tile_round2 power_probe prof_ab split_bench split_cost split_cost_r split_trace subtiles_check subtiles_check2 subtiles_occ subtiles_r128 sync_spin_ab tune_check" >&2; exit 2
fi
"cmd_$name" "$@"
