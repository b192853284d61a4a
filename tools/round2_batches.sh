#!/bin/bash
# Round-2 measurement batches, one function each: bash tools/round2_batches.sh <id> (was
# tools/round2/gpu_round2<id>.sh).  Each writes gpurun_out/r2<id>/; the results are summarised in
# profiles/ and docs/PERFORMANCE.md §6-§10, whose headers cite the batch id.

batch_a() {
# Round-2 GPU session A: RCCL self-probe (teardown variants), RCCL self-exchange tests, engine
# suite, driver-style bench + kernel trace.  Every GPU step has its own limit; a crash/timeout ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2a/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 6 "gpurun_out/r2a/$name.log"
  return $rc
}
#run probe_eager_only 40 ./build/rccl_self_probe 1
#run probe_graph 40 ./build/rccl_self_probe 0
run pytest_rccl 300 python -u -m pytest tests/test_gpu_rccl.py -x -v -m gpu --timeout 120 --timeout-method thread || exit $?
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
for i in 1 2 3; do
  run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
done
run bench_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 || exit $?
run bench_self_rccl 200 python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange || exit $?
run prof 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2a/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5
}

batch_aa() {
# row-major plan order: full GPU suite, driver bench x3, long bench, BASELINE configs on one GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2aa
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2aa/pytest.log 2>&1 || { tail -30 gpurun_out/r2aa/pytest.log; exit 1; }
tail -1 gpurun_out/r2aa/pytest.log
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > gpurun_out/r2aa/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r2aa/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/r2aa/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"])')"
}
for i in 1 2 3 4 5; do b bench20_$i --steps 20 --warmup 5; done
b bench2000 --steps 2000 --warmup 200
b c2 --steps 2000 --warmup 200 --size 8192
b b16k --steps 1000 --warmup 100 --size 16384
b s3_self --steps 1280 --warmup 128 --size 4096 --width 32768 --self-exchange
b c4_2d_self --steps 1120 --warmup 112 --size 32768 --width 16384 --decomp 2d --self-exchange
b w_self --steps 1280 --warmup 128 --self-exchange
b b65k --steps 256 --warmup 32 --size 65536
for i in 1 2 3; do timeout -k 10 60 ./build/gol 5 8192 1000 256 0 > gpurun_out/r2aa/cfg2_$i.txt || exit 1; head -1 gpurun_out/r2aa/cfg2_$i.txt; done
}

batch_ab() {
# with the row-major plan order: XCD permutation on/off (kbench), sub-tile plan occupancy 2 vs 3 (bench, alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2ab
for a in "32768 8 320" "32768 4 160" "32768 1 40" "16384 8 320"; do for s2 in 0 1; do for x in 8 1; do
  r=$(KB_XCDS=$x KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_po $a 2>&1 | tail -1) || exit 1
  echo "xcds=$x split2=$s2 $a $r" | tee -a gpurun_out/r2ab/xcds.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-110
done; done; done
for x in 8 1; do r=$(KB_XCDS=$x timeout -k 5 60 ./build/kbench_po 8192 24 960 0 0 8 0 4 2>&1 | tail -1) || exit 1; echo "xcds=$x tile8192 $r" | tee -a gpurun_out/r2ab/xcds.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-110; done
for i in 1 2; do for occ in 2 3; do
  GOL_SUB_OCC=$occ timeout -k 10 150 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/r2ab/occ$occ_$i.log 2>&1 || exit 1
  echo "sub_occ=$occ 2000 steps: $(tail -1 gpurun_out/r2ab/occ$occ_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f us/gen" % (d["ms_per_step"]*1e3))')"
  GOL_SUB_OCC=$occ timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2ab/occ20_$occ_$i.log 2>&1 || exit 1
  echo "sub_occ=$occ 20 steps: $(tail -1 gpurun_out/r2ab/occ20_$occ_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f us/gen" % (d["ms_per_step"]*1e3))')"
done; done
}

batch_ac() {
# row pitch 514 words (even) vs 528 (128-byte aligned rows), row-major plans (kbench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2ac
for a in "32768 8 320" "32768 4 160" "32768 1 40" "16384 8 320" "8192 24 960 0 0 8 0 4"; do for s2 in 0 1; do for v in p2 p16; do
  r=$(KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$v $a 2>&1 | tail -1) || exit 1
  echo "$v split2=$s2 $a $r" | tee -a gpurun_out/r2ac/pitch.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-110
done; done; done
}

batch_ad() {
# n row bands on n streams (n = 1, 2, 3, 4), plan occupancy 2 or 3 waves/SIMD, 32768^2 / 65536^2 K=8 (kbench, row-major plans)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2ad
for N in 32768 65536; do for n in 0 2 3 4; do for bpc in 2 3; do
  r=$(KB_BPC=$bpc KB_SPLIT2=$n timeout -k 5 100 ./build/kbench_sn $N 8 $([ $N = 32768 ] && echo 320 || echo 160) 2>&1 | tail -1) || exit 1
  echo "N=$N parts=$n bpc=$bpc $r" | tee -a gpurun_out/r2ad/splitn.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-110
done; done; done
}

batch_ae() {
# driver command traced with host markers (GOL_ROCTX=1: gol.run ranges) + kernels: where the timed region's time goes
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2ae
GOL_ROCTX=1 timeout -k 10 200 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $R/gpurun_out/r2ae/t -o t -- python $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/r2ae/t.log 2>&1 || { tail -5 $R/gpurun_out/r2ae/t.log; exit 1; }
ls $R/gpurun_out/r2ae/t/
tail -1 $R/gpurun_out/r2ae/t.log | cut -c150-260
}

batch_af() {
# sub-tile waits skipped on completed events: sub-tile tests, driver bench x5, traced once
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2af
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py tests/test_gpu_headline.py -x -q -m gpu -k "subtiles or hint or headline or seam or graphs" --timeout 200 --timeout-method thread > gpurun_out/r2af/pytest.log 2>&1 || { tail -30 gpurun_out/r2af/pytest.log; exit 1; }
tail -1 gpurun_out/r2af/pytest.log
for i in 1 2 3 4 5; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2af/b20_$i.log 2>&1 || exit 1; tail -1 gpurun_out/r2af/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("20 steps: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'; done
timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/r2af/b2000.log 2>&1 || exit 1; tail -1 gpurun_out/r2af/b2000.log | python -c 'import json,sys; d=json.load(sys.stdin); print("2000 steps: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'
cd /tmp
R=$GRAFT_REPO_ROOT
GOL_ROCTX=1 timeout -k 10 200 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $R/gpurun_out/r2af/t -o t -- python $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/r2af/t.log 2>&1 || exit 1
}

batch_ag() {
# round-2 validation: full GPU suite, smoke, driver bench x3, long bench, capacity config (2^20 x 2^20 tile)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2ag
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2ag/pytest.log 2>&1 || { tail -30 gpurun_out/r2ag/pytest.log; exit 1; }
tail -1 gpurun_out/r2ag/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2ag/b20_$i.log 2>&1 || exit 1; tail -1 gpurun_out/r2ag/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("20 steps: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'; done
timeout -k 10 120 python bench.py --gpus 1 > gpurun_out/r2ag/bdefault.log 2>&1 || exit 1; tail -1 gpurun_out/r2ag/bdefault.log | python -c 'import json,sys; d=json.load(sys.stdin); print("defaults (%d steps): %.3f us/gen %.3e" % (d["steps"], d["ms_per_step"]*1e3, d["value"]))'
timeout -k 10 300 python bench.py --gpus 1 --steps 40 --warmup 8 --size 1048576 > gpurun_out/r2ag/bcap.log 2>&1 || { tail -5 gpurun_out/r2ag/bcap.log; exit 1; }
tail -1 gpurun_out/r2ag/bcap.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("2^20 x 2^20: %.3f ms/gen %.3e" % (d["ms_per_step"], d["value"]), c["schedule"], c["kernel"])'
}

batch_ah() {
# final rocprof evidence: kernel stats of the driver command and of a 2000-generation run; PMC of the hot kernel
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2ah
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2ah/d20 -o d20 -- python $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/r2ah/d20.log 2>&1 || { tail -5 $R/gpurun_out/r2ah/d20.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2ah/d2000 -o d2000 -- python $R/bench.py --gpus 1 --steps 2000 --warmup 200 > $R/gpurun_out/r2ah/d2000.log 2>&1 || { tail -5 $R/gpurun_out/r2ah/d2000.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r2ah/pmc -o pmc -- $R/build/kbench_po 32768 8 320 > $R/gpurun_out/r2ah/pmc.log 2>&1 || { tail -5 $R/gpurun_out/r2ah/pmc.log; exit 1; }
ls $R/gpurun_out/r2ah/d20 $R/gpurun_out/r2ah/d2000 $R/gpurun_out/r2ah/pmc
}

batch_ai() {
# row-major plans: shallow-pass occupancy sweep (waves/SIMD the plan is sized for), one kernel and two halves
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2ai
for K in 1 2 4 5 6 7 8; do for s2 in 0 1; do for bpc in 2 3 4 8; do
  r=$(KB_BPC=$bpc KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_rm 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
  echo "K=$K split2=$s2 bpc=$bpc $r" | tee -a gpurun_out/r2ai/occ.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-130
done; done; done
}

batch_aj() {
# temporal-kernel workgroup size (waves per block 1/2/4/8) at 2 and 3 waves/SIMD plans, 32768^2 (kbench, row-major plans)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2aj
run() { # variant bpc K split2
  r=$(KB_BPC=$2 KB_SPLIT2=$4 timeout -k 5 60 ./build/kbench_$1 32768 $3 $(( $3 * 40 )) 2>&1 | tail -1) || exit 1
  echo "$1 bpc=$2 K=$3 split2=$4 $r" | tee -a gpurun_out/r2aj/wpb.txt | sed 's/"skew.*"waves"/waves/' | cut -c1-140
}
for K in 8 4; do for s2 in 0 1; do
  run w4 2 $K $s2; run w4 3 $K $s2
  run w1 8 $K $s2; run w1 12 $K $s2
  run w2 4 $K $s2; run w2 6 $K $s2
  run w8 1 $K $s2
done; done
}

batch_ak() {
# two sub-tiles forced on smaller tiles (below the auto threshold of 24576 rows): 16384^2, 4096 x 32768, 8192^2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2ak
b() {  # name, env, bench args...
  local n=$1 e=$2; shift 2
  env $e timeout -k 10 150 python bench.py --gpus 1 "$@" > gpurun_out/r2ak/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r2ak/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/r2ak/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["schedule"], c["kernel"], "R=%s" % c["halo_depth"], [x for x in c["autotune"].split() if x.startswith("sched")])')"
}
for i in 1 2; do
b b16k_auto_$i GOL_SUBTILES=auto --steps 1024 --warmup 128 --size 16384
b b16k_sub_$i GOL_SUBTILES=2 --steps 1024 --warmup 128 --size 16384
b s3_auto_$i GOL_SUBTILES=auto --steps 1024 --warmup 128 --size 4096 --width 32768
b s3_sub_$i GOL_SUBTILES=2 --steps 1024 --warmup 128 --size 4096 --width 32768
b s3self_sub_$i GOL_SUBTILES=2 --steps 1024 --warmup 128 --size 4096 --width 32768 --self-exchange
b c2_sub_$i GOL_SUBTILES=2 --steps 1024 --warmup 128 --size 8192
done
}

batch_al() {
# Deep passes (K = 12, 16) vs K = 6..8 at 32768^2, two half-board plans on two streams, plan occupancy 1-3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/deep_k.txt
: > $out
for K in 8 12 16 6; do
  for bpc in 1 2 3; do
    r=$(KB_BPC=$bpc KB_SPLIT2=1 timeout -k 5 60 ./build/kbench_main 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
    echo "K=$K bpc=$bpc split2=1 $r" | tee -a $out
  done
done
for K in 8 12 16; do
  r=$(KB_BPC=3 KB_SPLIT2=0 timeout -k 5 60 ./build/kbench_main 16384 $K $((K*80)) 2>&1 | tail -1) || exit 1
  echo "16384 K=$K bpc=3 $r" | tee -a $out
done
}

batch_am() {
# round-2 validation after splitting the engine source: full GPU suite, smoke, driver bench x3, long bench, capacity config (2^20 x 2^20 tile)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2am
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2am/pytest.log 2>&1 || { tail -30 gpurun_out/r2am/pytest.log; exit 1; }
tail -1 gpurun_out/r2am/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2am/b20_$i.log 2>&1 || exit 1; tail -1 gpurun_out/r2am/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("20 steps: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'; done
timeout -k 10 120 python bench.py --gpus 1 > gpurun_out/r2am/bdefault.log 2>&1 || exit 1; tail -1 gpurun_out/r2am/bdefault.log | python -c 'import json,sys; d=json.load(sys.stdin); print("defaults (%d steps): %.3f us/gen %.3e" % (d["steps"], d["ms_per_step"]*1e3, d["value"]))'
timeout -k 10 300 python bench.py --gpus 1 --steps 40 --warmup 8 --size 1048576 > gpurun_out/r2am/bcap.log 2>&1 || { tail -5 gpurun_out/r2am/bcap.log; exit 1; }
tail -1 gpurun_out/r2am/bcap.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("2^20 x 2^20: %.3f ms/gen %.3e" % (d["ms_per_step"], d["value"]), c["schedule"], c["kernel"])'
}

batch_an() {
# K = 9, 10 passes (natural registers: 2 waves/SIMD; capped at 3 waves/SIMD with spills) vs K = 8, 32768^2 two halves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/k9k10.txt
: > $out
for bin in k10 k10o3; do
  for K in 8 9 10; do
    for bpc in 1 2 3; do
      r=$(KB_BPC=$bpc KB_SPLIT2=1 timeout -k 5 60 ./build/kbench_$bin 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
      echo "$bin K=$K bpc=$bpc split2=1 $r" | tee -a $out
    done
  done
done
}

batch_ao() {
# Non-temporal row loads (GOL_NT_LOADS) vs plain loads in step_temporal, 32768^2, alternating A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ntld.txt
: > $out
for rep in 1 2; do
  for K in 1 4 8; do
    for s2 in 0 1; do
      for bin in base ntld; do
        r=$(KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$bin 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
        echo "$bin K=$K split2=$s2 $r" | tee -a $out
      done
    done
  done
done
}

batch_ap() {
# Kernel trace of the bench with halos through a real 1-rank RCCL communicator (--self-exchange):
# the ncclDevKernel* kernels next to the stencil kernels.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2ap
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2ap/prof -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 128 --warmup 16 --self-exchange > $R/gpurun_out/r2ap/bench.log 2>&1 || { tail -20 $R/gpurun_out/r2ap/bench.log; exit 1; }
tail -1 $R/gpurun_out/r2ap/bench.log | cut -c1-400
f=$(find $R/gpurun_out/r2ap/prof -name '*kernel_stats.csv' | head -1)
cp "$f" $R/gpurun_out/r2ap/kernel_stats.csv
cut -c1-160 $R/gpurun_out/r2ap/kernel_stats.csv | head -20
}

batch_aq() {
# RCCL p2p channel knobs vs the halo-exchange kernel time (1-rank self-exchange, 32768^2 bench).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r2aq
mkdir -p $o
run() {  # run <name> <env...>
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 $R/bench.py --gpus 1 --steps 256 --warmup 32 --self-exchange > $o/$name.log 2>&1 || { tail -5 $o/$name.log; return 1; }
  grep '^{"metric"' $o/$name.log | python3 -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("'$name'", "%.3e %.3f us/gen" % (d["value"], d["ms_per_step"]*1e3), c["schedule"], [t for t in c["autotune"].split() if t.startswith("sched")])'
}
prof() {
  local name=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/p_$name -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 128 --warmup 16 --self-exchange > $o/p_$name.log 2>&1 || { tail -5 $o/p_$name.log; return 1; }
  f=$(find $o/p_$name -name '*kernel_stats.csv' | head -1)
  echo "$name $(grep rcclGeneric $f | cut -d, -f3- | cut -c1-80)"
}
run base &&
run minp2p8 NCCL_MIN_P2P_NCHANNELS=8 &&
run perpeer8 NCCL_NCHANNELS_PER_PEER=8 &&
run minp2p8b NCCL_MIN_P2P_NCHANNELS=8 &&
run base2 &&
prof base &&
NCCL_MIN_P2P_NCHANNELS=8 prof minp2p8 &&
NCCL_NCHANNELS_PER_PEER=8 prof perpeer8
}

batch_ar() {
# Sub-tile exchange overlap (GOL_SUBTILE_OVERLAP): GPU tests of the sub-tile and RCCL paths, then the
# self-exchange bench with the init-time timing of both variants, and each variant forced.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2ar
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_engine.py -k "subtile or rccl or run_hint" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
b() {  # b <name> <env...>
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 bench.py --gpus 1 --steps $STEPS --warmup 16 --self-exchange > $o/$name.log 2>&1 || { tail -5 $o/$name.log; return 1; }
  grep '^{"metric"' $o/$name.log | python3 -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("'$name'", "%.3e %.3f us/gen" % (d["value"], d["ms_per_step"]*1e3), c["schedule"], [t for t in c["autotune"].split() if t.startswith("sched")])'
}
STEPS=256 b auto256 GOL_SUBTILE_OVERLAP=auto &&
STEPS=256 b ov0_256 GOL_SUBTILE_OVERLAP=0 &&
STEPS=256 b ov1_256 GOL_SUBTILE_OVERLAP=1 &&
STEPS=20 b ov0_20 GOL_SUBTILE_OVERLAP=0 &&
STEPS=20 b ov1_20 GOL_SUBTILE_OVERLAP=1 &&
STEPS=256 b ov0_256b GOL_SUBTILE_OVERLAP=0 &&
STEPS=256 b ov1_256b GOL_SUBTILE_OVERLAP=1 &&
STEPS=20 b ov0_20b GOL_SUBTILE_OVERLAP=0 &&
STEPS=20 b ov1_20b GOL_SUBTILE_OVERLAP=1
}

batch_as() {
# After making the sub-tile overlap opt-in: the sub-tile / RCCL / headline GPU tests and the driver bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2as
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_engine.py tests/test_gpu_headline.py -k "subtile or rccl or run_hint or headline" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for i in 1 2; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1; grep '^{"metric"' $o/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("20 steps: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), d["config"]["schedule"])'; done
}

batch_at() {
# Does the GPU clock ramp matter for the driver's 20-step timed region?  --warmup 5 (driver) vs a
# 2000-generation warmup that keeps the GPU busy until just before the timed steps.  Alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2at
mkdir -p $o
for rep in 1 2 3; do
  for w in 5 2000; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup $w > $o/w${w}_$rep.log 2>&1 || exit 1
    grep '^{"metric"' $o/w${w}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("warmup '$w': %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'
  done
done
}

batch_au() {
# Pass order of a short superstep (GOL_PASS_ORDER=asc: 4 + 8 + 8 instead of 8 + 8 + 4), driver command, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2au
mkdir -p $o
for rep in 1 2 3; do
  for ord in desc asc; do
    timeout -k 10 120 env GOL_PASS_ORDER=$ord python bench.py --gpus 1 --steps 20 --warmup 5 > $o/${ord}_$rep.log 2>&1 || exit 1
    grep '^{"metric"' $o/${ord}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$ord': %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'
  done
done
}

batch_av() {
# Kernel trace of a 512-generation bench run (8 supersteps of 64): per-queue gaps at superstep boundaries.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r2av
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/prof -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 512 --warmup 64 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
grep '^{"metric"' $o/bench.log | cut -c1-200
f=$(find $o/prof -name '*kernel_trace.csv' | head -1)
cp $f $o/kernel_trace.csv
python3 $R/tools/trace_queues.py $o/kernel_trace.csv --last-us 5400 > $o/queues.txt
cat $o/queues.txt | tail -60
}

batch_aw() {
# Asynchronous sub-tile superstep starts (GOL_SUBTILE_ASYNC): sub-tile GPU tests, headline oracle, then
# alternating benches (20, 256, 2000 steps) with and without.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2aw
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_headline.py tests/test_gpu_rccl.py -k "subtile or headline or run_hint or rccl" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for rep in 1 2; do
  for steps in 20 256 2000; do
    for as in 0 1; do
      timeout -k 10 120 env GOL_SUBTILE_ASYNC=$as python bench.py --gpus 1 --steps $steps --warmup 5 > $o/a${as}_${steps}_$rep.log 2>&1 || exit 1
      grep '^{"metric"' $o/a${as}_${steps}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("async '$as' steps '$steps': %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), d["config"]["schedule"])'
    done
  done
done
}

batch_ax() {
# Unequal sub-tile halves (GOL_SUB_SPLIT per mille for half 0, which runs ahead): 20 and 2000 steps, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2ax
mkdir -p $o
for rep in 1 2; do
  for steps in 20 2000; do
    for f in 500 520 540; do
      timeout -k 10 120 env GOL_SUB_SPLIT=$f python bench.py --gpus 1 --steps $steps --warmup 5 > $o/f${f}_${steps}_$rep.log 2>&1 || exit 1
      grep '^{"metric"' $o/f${f}_${steps}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("split '$f' steps '$steps': %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'
    done
  done
done
}

batch_ay() {
# Two-triple (ping-pong) steady loop vs the one-triple loop, step_temporal K = 5..8 and 12, 32768^2, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2ay
mkdir -p $o
: > $o/ab.txt
for rep in 1 2; do
  for K in 5 6 7 8 12; do
    for s2 in 1 0; do
      for bin in base pp; do
        r=$(KB_SPLIT2=$s2 KB_BPC=$((s2 ? 2 : 3)) timeout -k 5 60 ./build/kbench_$bin 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
        echo "$bin K=$K split2=$s2 $r" | sed 's/"skew.*"us_per_gen"/us_per_gen/' | tee -a $o/ab.txt
      done
    done
  done
done
}

batch_az() {
# Ping-pong loop for K = 6, 7, 12 and deeper pass costs in the pass-cut DP: full GPU suite, smoke,
# driver bench x3, long bench, 16384^2 and 65536^2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2az
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
j() { python -c 'import json,sys
for l in sys.stdin:
    if l.startswith("{\"metric\""):
        d=json.loads(l); c=d["config"]; print("'$1'", "%d steps: %.3f us/gen %.3e" % (d["steps"], d["ms_per_step"]*1e3, d["value"]), c["schedule"], [t for t in c["autotune"].split() if t.startswith("pass")])'; }
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1; j b20 < $o/b20_$i.log; done
timeout -k 10 120 python bench.py --gpus 1 > $o/bdef.log 2>&1 || exit 1; j default < $o/bdef.log
timeout -k 10 120 python bench.py --gpus 1 --size 16384 --steps 2000 --warmup 100 > $o/b16k.log 2>&1 || exit 1; j 16384 < $o/b16k.log
timeout -k 10 200 python bench.py --gpus 1 --size 65536 --steps 640 --warmup 64 > $o/b64k.log 2>&1 || exit 1; j 65536 < $o/b64k.log
}

batch_b() {
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2b
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2b/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 8 "gpurun_out/r2b/$name.log"
  return $rc
}
run short 300 python tools/short_run_probe.py --variants sub2,sub0,sub2-nograph,sub0-nograph,sub0-r32 || exit $?
run short_torch 200 python tools/short_run_probe.py --variants sub2,sub0 --torch-sync || exit $?
GOL_SUBTILES=2 run prof_self_sub 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2b/prof_self_sub -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 5 --self-exchange
}

batch_ba() {
# Driver command x8 (spread of the 20-step figure with the 12 + 8 cut).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2ba
mkdir -p $o
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1
  grep '^{"metric"' $o/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), [t for t in c["autotune"].split() if t.startswith(("pass8","pass12","pass4"))])'
done
}

batch_bb() {
# Kernel traces of 8 driver-command runs (12 + 8 cut): the timed region's kernels per queue, to see what the slow runs do.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r2bb
mkdir -p $o
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $o/p$i -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $o/b$i.log 2>&1 || { tail -5 $o/b$i.log; exit 1; }
  f=$(find $o/p$i -name '*kernel_trace.csv' | head -1)
  v=$(grep '^{"metric"' $o/b$i.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print("%.3f" % (d["ms_per_step"]*1e3))')
  echo "== run $i: $v us/gen"
  python3 $R/tools/trace_queues.py $f --last-us 600 --show 8 | grep -v "^  busy" | head -24
done > $o/summary.txt
grep "== run" $o/summary.txt
}

batch_bc() {
# Spread of the driver command with the 12 + 8 cut: pass order 12, 8 (desc) vs 8, 12 (asc), 12 runs each, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bc
mkdir -p $o
: > $o/all.txt
for i in $(seq 1 12); do
  for ord in desc asc; do
    timeout -k 10 120 env GOL_PASS_ORDER=$ord python bench.py --gpus 1 --steps 20 --warmup 5 > $o/${ord}_$i.log 2>&1 || exit 1
    grep '^{"metric"' $o/${ord}_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$ord' %.3f" % (d["ms_per_step"]*1e3))' >> $o/all.txt
  done
done
for ord in desc asc; do echo "$ord: $(grep "^$ord" $o/all.txt | cut -d' ' -f2 | sort -n | tr '\n' ' ')"; done
}

batch_bd() {
# Ping-pong loop for K = 6, 7, 12 and deeper pass costs in the pass-cut DP: full GPU suite, smoke,
# driver bench x3, long bench, 16384^2 and 65536^2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bd
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
j() { python -c 'import json,sys
for l in sys.stdin:
    if l.startswith("{\"metric\""):
        d=json.loads(l); c=d["config"]; print("'$1'", "%d steps: %.3f us/gen %.3e" % (d["steps"], d["ms_per_step"]*1e3, d["value"]), c["schedule"], [t for t in c["autotune"].split() if t.startswith("pass")])'; }
for i in 1 2 3 4; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1; j b20 < $o/b20_$i.log; done
timeout -k 10 120 python bench.py --gpus 1 > $o/bdef.log 2>&1 || exit 1; j default < $o/bdef.log
timeout -k 10 120 python bench.py --gpus 1 --size 16384 --steps 2000 --warmup 100 > $o/b16k.log 2>&1 || exit 1; j 16384 < $o/b16k.log
timeout -k 10 200 python bench.py --gpus 1 --size 65536 --steps 640 --warmup 64 > $o/b64k.log 2>&1 || exit 1; j 65536 < $o/b64k.log
}

batch_be() {
# Tile kernel band loop: two register triples (GOL_TILE_PINGPONG=1) vs one, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2be
mkdir -p $o
: > $o/ab.txt
run() {  # run <label> <env...> -- <kbench args>
  local label=$1; shift
  for bin in tbase tpp; do
    r=$(env "$@" timeout -k 5 60 ./build/kbench_$bin $KBARGS 2>&1 | tail -1) || return 1
    echo "$bin $label $r" | sed 's/"skew.*"tile_nw"/tile_nw/' | tee -a $o/ab.txt
  done
}
for rep in 1 2; do
  KBARGS="8192 24 960 0 0 8 0 4" run "8192 K24 lv4 db" KB_INPLACE=0 || exit 1
  KBARGS="8192 16 960 0 0 8 0 2" run "8192 K16 lv2 db" KB_INPLACE=0 || exit 1
  KBARGS="4096 16 640 0 0 8 0 2" run "4096x32768 K16 lv2 ip" KB_W=32768 KB_INPLACE=1 || exit 1
  KBARGS="16384 16 640 0 0 8 0 2" run "16384 K16 lv2 ip" KB_INPLACE=1 || exit 1
done
}

batch_bf() {
# Tile kernel with the two-triple band loop at 4 levels: tile GPU tests, config 2 CLI x3, bench 8192^2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bf
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_cli.py -k "tile or known_physics or perf or auto or cfg or 8192" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for i in 1 2 3; do (cd $o && timeout -k 10 120 ../../build/gol 5 8192 1000 256 0 | tail -1); done
timeout -k 10 120 python bench.py --gpus 1 --size 8192 --steps 1000 --warmup 24 > $o/b8k.log 2>&1 || exit 1
grep '^{"metric"' $o/b8k.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("8192^2 bench: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), c["kernel"], c["kernel_depth"])'
}

batch_bg() {
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r2bg
for i in 1 2 3 4; do (cd gpurun_out/r2bg && timeout -k 10 120 ../../build/gol 5 8192 1000 256 0 | grep TOTAL); done
}

batch_bh() {
# Per-rank tiles of the multi-GPU configs through RCCL self-exchange, after the two-triple loop and the deeper pass costs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bh
mkdir -p $o
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > $o/$n.log 2>&1 || { echo "$n failed"; tail -5 $o/$n.log; exit 1; }
  echo "$n $(grep '^{"metric"' $o/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"], [x for x in c["autotune"].split() if x.startswith("sched")])')"
}
b s3_self --steps 1280 --warmup 128 --size 4096 --width 32768 --self-exchange
b c4_2d_self --steps 1120 --warmup 112 --size 32768 --width 16384 --decomp 2d --self-exchange
b c4_1d_self --steps 1280 --warmup 128 --size 8192 --width 65536 --self-exchange
b w_self --steps 1280 --warmup 128 --self-exchange
b w_self20 --steps 20 --warmup 5 --self-exchange
b w_self20b --steps 20 --warmup 5 --self-exchange
}

batch_bi() {
# 20-step runs with halos through RCCL self-exchange: sub-tile exchange overlap off / on, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bi
mkdir -p $o
for i in 1 2 3; do
  for ov in 0 1; do
    timeout -k 10 150 env GOL_SUBTILE_OVERLAP=$ov python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange > $o/ov${ov}_$i.log 2>&1 || exit 1
    grep '^{"metric"' $o/ov${ov}_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("ov'$ov' %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), c["schedule"])'
  done
done
}

batch_bj() {
# Ping-pong loop for K = 6, 7, 12 and deeper pass costs in the pass-cut DP: full GPU suite, smoke,
# driver bench x3, long bench, 16384^2 and 65536^2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bj
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
j() { python -c 'import json,sys
for l in sys.stdin:
    if l.startswith("{\"metric\""):
        d=json.loads(l); c=d["config"]; print("'$1'", "%d steps: %.3f us/gen %.3e" % (d["steps"], d["ms_per_step"]*1e3, d["value"]), c["schedule"], [t for t in c["autotune"].split() if t.startswith("pass")])'; }
for i in 1 2 3 4; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1; j b20 < $o/b20_$i.log; done
timeout -k 10 120 python bench.py --gpus 1 > $o/bdef.log 2>&1 || exit 1; j default < $o/bdef.log
timeout -k 10 120 python bench.py --gpus 1 --size 16384 --steps 2000 --warmup 100 > $o/b16k.log 2>&1 || exit 1; j 16384 < $o/b16k.log
timeout -k 10 200 python bench.py --gpus 1 --size 65536 --steps 640 --warmup 64 > $o/b64k.log 2>&1 || exit 1; j 65536 < $o/b64k.log
}

batch_bk() {
# Driver command x16 (frequency of slow runs with the final build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bk
mkdir -p $o
: > $o/all.txt
for i in $(seq 1 16); do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1
  grep '^{"metric"' $o/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f" % (d["ms_per_step"]*1e3))' >> $o/all.txt
done
sort -n $o/all.txt | tr '\n' ' '; echo
}

batch_bl() {
# Sub-tile superstep length: halo depth 64 (auto) vs 128 vs 96, 2000 steps, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bl
mkdir -p $o
for rep in 1 2; do
  for R in 64 128 96; do
    timeout -k 10 150 python bench.py --gpus 1 --steps 2048 --warmup 128 --halo-depth $R > $o/r${R}_$rep.log 2>&1 || exit 1
    grep '^{"metric"' $o/r${R}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("R='$R' %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), c["schedule"], c["halo_depth"])'
  done
done
}

batch_bm() {
# Auto halo depth 128 for sub-tile ranks: full GPU suite, smoke, driver command x4, long runs, 65536^2, self-exchange.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bm
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 | cut -c1-60 || exit 1
j() { python -c 'import json,sys
for l in sys.stdin:
    if l.startswith("{\"metric\""):
        d=json.loads(l); c=d["config"]; print("'$1'", "%d steps: %.3f us/gen %.3e" % (d["steps"], d["ms_per_step"]*1e3, d["value"]), c["schedule"], "R=%s" % c["halo_depth"], [t for t in c["autotune"].split() if t.startswith("sched")])'; }
for i in 1 2 3 4; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1; j b20 < $o/b20_$i.log; done
timeout -k 10 120 python bench.py --gpus 1 > $o/bdef.log 2>&1 || exit 1; j default < $o/bdef.log
timeout -k 10 150 python bench.py --gpus 1 --steps 2048 --warmup 128 > $o/b2k.log 2>&1 || exit 1; j long < $o/b2k.log
timeout -k 10 200 python bench.py --gpus 1 --size 65536 --steps 640 --warmup 128 > $o/b64k.log 2>&1 || exit 1; j 65536 < $o/b64k.log
timeout -k 10 150 python bench.py --gpus 1 --steps 1280 --warmup 128 --self-exchange > $o/bself.log 2>&1 || exit 1; j self1280 < $o/bself.log
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange > $o/bself20.log 2>&1 || exit 1; j self20 < $o/bself20.log
}

batch_bn() {
# One-tile strips with neighbours (RCCL self-exchange): halo depth 64 (auto) vs 128, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bn
mkdir -p $o
for rep in 1 2; do
  for R in 64 128; do
    for cfg in "s3 --size 4096 --width 32768" "c4_1d --size 8192 --width 65536" "s2 --size 16384 --width 32768"; do
      set -- $cfg; n=$1; shift
      timeout -k 10 150 python bench.py --gpus 1 --steps 1280 --warmup 128 --self-exchange --halo-depth $R "$@" > $o/${n}_$R_$rep.log 2>&1 || exit 1
      grep '^{"metric"' $o/${n}_$R_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("'$n' R='$R' %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), c["schedule"], c["halo_depth"])'
    done
  done
done
}

batch_bo() {
# Auto halo depth 128 for 1-D strips with neighbours: GPU engine + RCCL tests, per-rank tiles through self-exchange.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bo
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py tests/test_gpu_cli.py -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > $o/$n.log 2>&1 || { echo "$n failed"; tail -5 $o/$n.log; exit 1; }
  echo "$n $(grep '^{"metric"' $o/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"], [x for x in c["autotune"].split() if x.startswith("sched")])')"
}
b s3_self --steps 1280 --warmup 128 --size 4096 --width 32768 --self-exchange
b s2_self --steps 1280 --warmup 128 --size 16384 --width 32768 --self-exchange
b c4_2d_self --steps 1120 --warmup 112 --size 32768 --width 16384 --decomp 2d --self-exchange
b c4_1d_self --steps 1280 --warmup 128 --size 8192 --width 65536 --self-exchange
}

batch_bp() {
# Auto halo depth 128 for sub-tile ranks: full GPU suite, smoke, driver command x4, long runs, 65536^2, self-exchange.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bp
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 | cut -c1-60 || exit 1
j() { python -c 'import json,sys
for l in sys.stdin:
    if l.startswith("{\"metric\""):
        d=json.loads(l); c=d["config"]; print("'$1'", "%d steps: %.3f us/gen %.3e" % (d["steps"], d["ms_per_step"]*1e3, d["value"]), c["schedule"], "R=%s" % c["halo_depth"], [t for t in c["autotune"].split() if t.startswith("sched")])'; }
for i in 1 2 3 4; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1; j b20 < $o/b20_$i.log; done
timeout -k 10 120 python bench.py --gpus 1 > $o/bdef.log 2>&1 || exit 1; j default < $o/bdef.log
timeout -k 10 150 python bench.py --gpus 1 --steps 2048 --warmup 128 > $o/b2k.log 2>&1 || exit 1; j long < $o/b2k.log
timeout -k 10 200 python bench.py --gpus 1 --size 65536 --steps 640 --warmup 128 > $o/b64k.log 2>&1 || exit 1; j 65536 < $o/b64k.log
timeout -k 10 150 python bench.py --gpus 1 --steps 1280 --warmup 128 --self-exchange > $o/bself.log 2>&1 || exit 1; j self1280 < $o/bself.log
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange > $o/bself20.log 2>&1 || exit 1; j self20 < $o/bself20.log
}

batch_bq() {
# The driver's multi-GPU launch line rehearsed on one GPU (ranks share the card: host-staged halos), default board.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bq
mkdir -p $o
for P in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $P --master-addr 127.0.0.1 --master-port 2961$P bench.py --gpus $P --steps 20 --warmup 5 --allow-host-staging > $o/torchrun_p$P.log 2>&1 || { tail -20 $o/torchrun_p$P.log; exit 1; }
  grep '^{' $o/torchrun_p$P.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("P=%d: %.3e cell-updates/s, %.3f us/gen, n_gpus %d, board %s, %s, R=%s, %s" % ('$P', d["value"], d["ms_per_step"]*1e3, d["n_gpus"], c["board"], c["schedule"], c["halo_depth"], c["transport"]))'
done
}

batch_br() {
# Kernel trace of the driver command with halos through RCCL self-exchange: where the ~30 us of the exchange go.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r2br
mkdir -p $o
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/p -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange > $o/b.log 2>&1 || { tail -5 $o/b.log; exit 1; }
f=$(find $o/p -name '*kernel_trace.csv' | head -1)
cp $f $o/kernel_trace.csv
python3 - $o/kernel_trace.csv <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
end = max(e for _, e, _, _ in rows)
t0 = end - 700e3
for s, e, q, k in rows:
    if s >= t0:
        n = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("gol::hipk::", "")
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {n[:60]}")
PY
grep '^{"metric"' $o/b.log | cut -c1-150
}

batch_bs() {
# Sub-tile events with a device-scope release (GOL_SUB_EVENT_SCOPE=device) vs system scope, alternating:
# 20 steps with RCCL self-exchange (one exchange + cross-queue wait per run), 20 steps local, 2048 steps local.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bs
mkdir -p $o
for rep in 1 2 3; do
  for sc in system device; do
    for cfg in "self20 --steps 20 --warmup 5 --self-exchange" "loc20 --steps 20 --warmup 5" "loc2k --steps 2048 --warmup 128"; do
      set -- $cfg; n=$1; shift
      timeout -k 10 150 env GOL_SUB_EVENT_SCOPE=$sc python bench.py --gpus 1 "$@" > $o/${n}_${sc}_$rep.log 2>&1 || exit 1
      grep '^{"metric"' $o/${n}_${sc}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$n' '$sc' %.3f us/gen" % (d["ms_per_step"]*1e3))'
    done
  done
done
}

batch_bt() {
# RCCL launch knobs vs the exchange cost of a 20-step run through RCCL self-exchange, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bt
mkdir -p $o
for rep in 1 2 3; do
  for v in default mix0 lo1; do
    case $v in default) e="GOL_X=1";; mix0) e="NCCL_GRAPH_MIXING_SUPPORT=0";; lo1) e="NCCL_LAUNCH_ORDER_IMPLICIT=1";; esac
    timeout -k 10 150 env $e python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange > $o/${v}_$rep.log 2>&1 || { tail -3 $o/${v}_$rep.log; exit 1; }
    grep '^{"metric"' $o/${v}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$v' %.3f us/gen" % (d["ms_per_step"]*1e3))'
  done
done
}

batch_bu() {
# Sub-tile cross-stream signals in signal memory (GOL_SUB_SYNC=value, default) vs events: tests, then alternating benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bu
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py tests/test_gpu_headline.py -k "subtile or rccl or headline or run_hint or checkpoint" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for rep in 1 2 3; do
  for sy in event value; do
    for cfg in "self20 --steps 20 --warmup 5 --self-exchange" "loc20 --steps 20 --warmup 5" "loc2k --steps 2048 --warmup 128"; do
      set -- $cfg; n=$1; shift
      timeout -k 10 150 env GOL_SUB_SYNC=$sy python bench.py --gpus 1 "$@" > $o/${n}_${sy}_$rep.log 2>&1 || { tail -3 $o/${n}_${sy}_$rep.log; exit 1; }
      grep '^{"metric"' $o/${n}_${sy}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$n' '$sy' %.3f us/gen" % (d["ms_per_step"]*1e3))'
    done
  done
done
}

batch_bv() {
# Sub-tile cross-stream signals in signal memory (GOL_SUB_SYNC=value, default) vs events: tests, then alternating benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r2bv
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py tests/test_gpu_headline.py -k "subtile or rccl or headline or run_hint or checkpoint" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for rep in 1 2 3; do
  for sy in event value; do
    for cfg in "self20 --steps 20 --warmup 5 --self-exchange" "loc20 --steps 20 --warmup 5" "loc2k --steps 2048 --warmup 128"; do
      set -- $cfg; n=$1; shift
      timeout -k 10 150 env GOL_SUB_SYNC=$sy python bench.py --gpus 1 "$@" > $o/${n}_${sy}_$rep.log 2>&1 || { tail -3 $o/${n}_${sy}_$rep.log; exit 1; }
      grep '^{"metric"' $o/${n}_${sy}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$n' '$sy' %.3f us/gen" % (d["ms_per_step"]*1e3))'
    done
  done
done
}

batch_c() {
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2c
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2c/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/r2c/$name.log" | cut -c1-1500
  return $rc
}
run self_rccl 200 python bench.py --gpus 1 --steps 640 --warmup 64 --self-exchange || exit $?
GOL_SUBTILES=2 run prof_self_sub 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2c/prof_self_sub -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 5 --self-exchange || exit $?
run short 300 python tools/short_run_probe.py --variants sub2,sub0 || exit $?
run kbsweep 400 bash tools/experiments.sh kb_depth_sweep
}

batch_d() {
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2d
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2d/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/r2d/$name.log" | cut -c1-2500
  return $rc
}
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
for i in 1 2 3; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run short 300 python tools/short_run_probe.py --variants sub2,sub0 || exit $?
run bench_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 || exit $?
run prof 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2d/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5
}

batch_e() {
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2e
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2e/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/r2e/$name.log" | cut -c1-600
  return $rc
}
run prof_graph 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2e/prof_graph -o run -- python3 bench.py --gpus 1 --steps 256 --warmup 5 || exit $?
GOL_GRAPH=0 run prof_eager 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2e/prof_eager -o run -- python3 bench.py --gpus 1 --steps 256 --warmup 5 || exit $?
run short 300 python tools/short_run_probe.py --variants sub2,sub0,sub2-nograph,sub0-nograph || exit $?
run short256 300 python tools/short_run_probe.py --steps 256 --reps 5 --variants sub2,sub0,sub2-nograph,sub0-nograph || exit $?
}

batch_f() {
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2f
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2f/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/r2f/$name.log" | cut -c1-700
  return $rc
}
run headline 300 python -u -m pytest tests/test_gpu_headline.py -x -v -m gpu --timeout 280 --timeout-method thread || exit $?
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
for i in 1 2 3; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run bench_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 || exit $?
run bench_self 200 python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange || exit $?
run bench_self_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 --self-exchange || exit $?
}

batch_g() {
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2g
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2g/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 1 "gpurun_out/r2g/$name.log" | cut -c1-400
  return $rc
}
for i in 1 2 3 4; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run prof 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2g/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5
}

batch_h() {
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2h
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2h/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/r2h/$name.log" | cut -c1-300
  return $rc
}
run pytest_sub 300 python -u -m pytest tests/test_gpu_engine.py -k "subtiles or hint" -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py tests/test_gpu_headline.py -x -q -m gpu --timeout 200 --timeout-method thread || exit $?
for i in 1 2 3; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run bench_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 || exit $?
run bench_self 200 python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange || exit $?
run short 300 python tools/short_run_probe.py --variants sub2,sub0 || exit $?
}

batch_i() {
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2i
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2i/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 1 "gpurun_out/r2i/$name.log" | cut -c150-260
  return $rc
}
for i in 1 2 3 4 5; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run pytest_sub 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py -k "subtiles or hint" -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
}

batch_j() {
# round 2 re-entry: full GPU suite + driver bench + kernel trace of the driver bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2j
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2j/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/r2j/$name.log" | cut -c1-400
  return $rc
}
run pytest_all 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread || exit $?
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
for i in 1 2; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run prof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2j/prof -o bench -- python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
}

batch_k() {
# shallow-pass prefetch depth A/B (kbench, 32768^2) + engine bench + tile-kernel PMC at 8192^2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2k
export TMPDIR=/tmp
for K in 1 2 3 4; do
  for bpc in 3 8; do
    for s2 in 0 1; do
      for v in pf0 pf1; do
        r=$(KB_BPC=$bpc KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$v 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
        echo "$v K=$K bpc=$bpc split2=$s2 $r" | tee -a gpurun_out/r2k/pf_sweep.txt
      done
    done
  done
done
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2k/bench_$i.log 2>&1 || exit 1; tail -1 gpurun_out/r2k/bench_$i.log | cut -c1-330; done
timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/r2k/bench_long.log 2>&1 || exit 1; tail -1 gpurun_out/r2k/bench_long.log | cut -c1-330
cd /tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/r2k/pmc_a -o a --output-format csv -- $R/build/kbench_pf1 8192 24 960 0 0 8 0 2 > $R/gpurun_out/r2k/pmc_a.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/r2k/pmc_b -o b --output-format csv -- $R/build/kbench_pf1 8192 24 960 0 0 8 0 2 > $R/gpurun_out/r2k/pmc_b.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_WAVE32_INSTS GRBM_GUI_ACTIVE SQ_IFETCH SQ_INSTS_BRANCH -d $R/gpurun_out/r2k/pmc_c -o c --output-format csv -- $R/build/kbench_pf1 8192 24 960 0 0 8 0 2 > $R/gpurun_out/r2k/pmc_c.log 2>&1 || echo "pmc_c failed (optional)"
echo done
}

batch_l() {
# tile kernel: software-pipelined LDS band reads (tnew) vs the previous kernel (told), + tile tests + config 2 CLI
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2l
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_cli.py -x -q -m gpu -k "tile or auto or cfg or perf" --timeout 120 --timeout-method thread > gpurun_out/r2l/pytest.log 2>&1 || { tail -20 gpurun_out/r2l/pytest.log; exit 1; }
tail -2 gpurun_out/r2l/pytest.log
for N in 8192 16384; do
  for K in 16 24 32; do
    for nw in 8 16; do
      for lv in 1 2; do
        for v in told tnew; do
          r=$(timeout -k 5 60 ./build/kbench_$v $N $K $((K*40)) 0 0 $nw 0 $lv 2>&1 | tail -1) || exit 1
          echo "$v N=$N K=$K nw=$nw lv=$lv $r" | tee -a gpurun_out/r2l/tile_ab.txt | cut -c1-60,150-
        done
      done
    done
  done
done
for i in 1 2 3; do timeout -k 10 60 ./build/gol 5 8192 1000 256 0 | head -1; done
}

batch_m() {
# per-rank tiles of the scaling configs on one GPU (rectangular boards, RCCL self-exchange) + 2-D vs 1-D rehearsal traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2m
export TMPDIR=/tmp
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > gpurun_out/r2m/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r2m/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/r2m/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["parallelism"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"], c["autotune"][:200])')"
}
# config 3 strong-scaled over 8 GPUs: the per-rank strip 4096 x 32768
b s3_local --steps 1000 --warmup 100 --size 4096 --width 32768
b s3_self --steps 1000 --warmup 100 --size 4096 --width 32768 --self-exchange
# config 2 board
b c2 --steps 1000 --warmup 100 --size 8192
# config 4 (65536^2 over 8 GPUs): 2-D 4x2 per-rank tile 32768 x 16384 vs the 1-D strip 8192 x 65536, both through RCCL
b c4_2d_self --steps 640 --warmup 64 --size 32768 --width 16384 --decomp 2d --self-exchange
b c4_1d_self --steps 640 --warmup 64 --size 8192 --width 65536 --self-exchange
b c4_2d_local --steps 640 --warmup 64 --size 32768 --width 16384
# 2x2 vs 1-D P=4 rehearsal (thread ranks sharing the GPU), kernel traces
cd /tmp
R=$GRAFT_REPO_ROOT
for cfg in 2d:2x2:32768 1d:4:32768; do
  tag=$(echo $cfg | tr ':' '_')
  GOL_SCHEDULE=full timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r2m/tr_$tag -o tr -- python $R/tools/rehearse_multirank.py --configs $cfg --gens 640 --warm 64 > $R/gpurun_out/r2m/tr_$tag.log 2>&1 || { echo "trace $cfg failed"; tail -5 $R/gpurun_out/r2m/tr_$tag.log; exit 1; }
  grep '^{' $R/gpurun_out/r2m/tr_$tag.log | cut -c1-200
  python $R/tools/kernel_summary.py $(ls $R/gpurun_out/r2m/tr_$tag/*kernel_trace.csv | head -1) --last-us 20000 | head -14
done
}

batch_n() {
# kernel traces of one rank holding the per-rank tiles of configs 3 (strong, 8 GPUs) and 4 (2-D 4x2) with
# halos through a 1-rank RCCL communicator; + the interleaved sub-tile launch order on the driver bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2n
export TMPDIR=/tmp
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2n/bench_$i.log 2>&1 || exit 1; tail -1 gpurun_out/r2n/bench_$i.log | cut -c170-260; done
cd /tmp
R=$GRAFT_REPO_ROOT
tr() {  # tag, env..., -- bench args
  local tag=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r2n/$tag -o tr -- python $R/bench.py --gpus 1 "$@" > $R/gpurun_out/r2n/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $R/gpurun_out/r2n/$tag.log; exit 1; }
  echo "== $tag: $(tail -1 $R/gpurun_out/r2n/$tag.log | cut -c1-120)"
  python $R/tools/kernel_summary.py $R/gpurun_out/r2n/$tag/tr_kernel_trace.csv --last-us 3000 > $R/gpurun_out/r2n/$tag.summary.txt
  head -12 $R/gpurun_out/r2n/$tag.summary.txt
}
tr bench20 --steps 20 --warmup 5
export GOL_SCHEDULE=split
tr c4_2d_split --steps 320 --warmup 64 --size 32768 --width 16384 --decomp 2d --self-exchange
export GOL_SCHEDULE=full
tr c4_2d_full --steps 320 --warmup 64 --size 32768 --width 16384 --decomp 2d --self-exchange
tr s3_full --steps 640 --warmup 64 --size 4096 --width 32768 --self-exchange
export GOL_SCHEDULE=split
tr s3_split --steps 640 --warmup 64 --size 4096 --width 32768 --self-exchange
}

batch_o() {
# tile kernel 4-level LDS passes A/B; deeper auto halos + fixed schedule timing on the per-rank tiles; GPU engine tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r2o/pytest.log 2>&1 || { tail -30 gpurun_out/r2o/pytest.log; exit 1; }
tail -1 gpurun_out/r2o/pytest.log
for N in 8192 16384; do for K in 16 24 32; do for nw in 8 16; do for lv in 2 4; do
  r=$(timeout -k 5 60 ./build/kbench_tl $N $K $((K*40)) 0 0 $nw 0 $lv 2>&1 | tail -1) || exit 1
  echo "N=$N K=$K nw=$nw lv=$lv $r" | tee -a gpurun_out/r2o/tile_lv.txt | cut -c1-40,170-
done; done; done; done
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > gpurun_out/r2o/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r2o/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/r2o/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"], [x for x in c["autotune"].split() if x.startswith("sched")])')"
}
b s3_self --steps 1280 --warmup 128 --size 4096 --width 32768 --self-exchange
b c4_2d_self --steps 1120 --warmup 112 --size 32768 --width 16384 --decomp 2d --self-exchange
b c4_1d_self --steps 1280 --warmup 128 --size 8192 --width 65536 --self-exchange
b w_self --steps 1280 --warmup 128 --self-exchange
b bench20 --steps 20 --warmup 5
}

batch_p() {
# tile kernel time breakdown: s_memtime stamps per LDS pass (diagnostic build kbench_stamp)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2p
for args in "8192 24 960 0 0 8 0 2" "8192 24 960 0 0 8 0 1" "8192 24 960 0 0 8 0 4" "8192 24 960 0 0 4 0 2" "8192 24 960 0 0 16 0 2" "8192 8 960 0 0 8 0 2" "16384 24 960 0 0 8 0 2" "32768 24 960 0 0 8 0 2"; do
  echo "== $args" | tee -a gpurun_out/r2p/stamps.txt
  timeout -k 5 60 ./build/kbench_stamp $args 2>&1 | tail -2 | tee -a gpurun_out/r2p/stamps.txt | cut -c1-400 || exit 1
done
}

batch_q() {
# in-place LDS tile (one buffer, private halo copies) vs double-buffered: correctness (tile tests) + kbench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2q
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_cli.py -x -q -m gpu -k "tile or auto or cfg or perf" --timeout 120 --timeout-method thread > gpurun_out/r2q/pytest.log 2>&1 || { tail -30 gpurun_out/r2q/pytest.log; exit 1; }
tail -1 gpurun_out/r2q/pytest.log
for shape in "8192 8192" "16384 16384" "4096 32768" "32768 32768"; do set -- $shape; N=$1; W=$2
  for K in 16 24 32; do for lv in 2 4; do for ip in 0 1; do
    r=$(KB_W=$W KB_INPLACE=$ip timeout -k 5 60 ./build/kbench_tl $N $K $((K*40)) 0 0 8 0 $lv 2>&1 | tail -1) || exit 1
    echo "N=$N W=$W K=$K lv=$lv inplace=$ip $r" | tee -a gpurun_out/r2q/inplace_ab.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-150
  done; done; done
done
for i in 1 2; do timeout -k 10 60 ./build/gol 5 8192 1000 256 0 | head -1; done
timeout -k 10 150 python bench.py --gpus 1 --steps 1000 --warmup 100 --size 4096 --width 32768 > gpurun_out/r2q/s3_local.log 2>&1 || exit 1; tail -1 gpurun_out/r2q/s3_local.log | cut -c170-600
timeout -k 10 150 python bench.py --gpus 1 --steps 1000 --warmup 100 --size 16384 > gpurun_out/r2q/b16k.log 2>&1 || exit 1; tail -1 gpurun_out/r2q/b16k.log | cut -c170-600
}

batch_r() {
# tile variant per plan (double-buffered when one round fits, else in place): tests + configs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2r
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_cli.py -x -q -m gpu -k "tile or auto or cfg or perf" --timeout 120 --timeout-method thread > gpurun_out/r2r/pytest.log 2>&1 || { tail -30 gpurun_out/r2r/pytest.log; exit 1; }
tail -1 gpurun_out/r2r/pytest.log
for i in 1 2 3; do timeout -k 10 60 ./build/gol 5 8192 1000 256 0 > gpurun_out/r2r/cfg2_$i.txt || exit 1; head -1 gpurun_out/r2r/cfg2_$i.txt; done
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > gpurun_out/r2r/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r2r/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/r2r/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"], c["autotune"][:300])')"
}
b c2 --steps 2000 --warmup 200 --size 8192
b s3_local --steps 1280 --warmup 128 --size 4096 --width 32768
b s3_self --steps 1280 --warmup 128 --size 4096 --width 32768 --self-exchange
b b16k --steps 1000 --warmup 100 --size 16384
}

batch_s() {
# full GPU suite; torchrun 2- and 4-process bench sharing the one GPU (host-staged halos: the
# bootstrap/control-plane/collective-autotune path of the driver's multi-GPU run); CLI tile levels A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2s
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2s/pytest.log 2>&1 || { tail -40 gpurun_out/r2s/pytest.log; exit 1; }
tail -1 gpurun_out/r2s/pytest.log
for P in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $P --master-addr 127.0.0.1 --master-port 2951$P bench.py --gpus $P --steps 64 --warmup 8 --size 8192 --allow-host-staging > gpurun_out/r2s/torchrun_p$P.log 2>&1 || { tail -20 gpurun_out/r2s/torchrun_p$P.log; exit 1; }
  grep '^{' gpurun_out/r2s/torchrun_p$P.log | cut -c1-200; grep -h "RCCL\|host" gpurun_out/r2s/torchrun_p$P.log | head -3
done
for lv in 2 4; do for i in 1 2; do GOL_TILE_LEVELS=$lv timeout -k 10 60 ./build/gol 5 8192 1000 256 0 > gpurun_out/r2s/cfg2_lv$lv_$i.txt || exit 1; echo "lv=$lv $(head -1 gpurun_out/r2s/cfg2_lv$lv_$i.txt)"; done; done
}

batch_t() {
# small tiles, two workgroups per CU (staging of one overlaps the other's compute): kbench sweep at 8192^2 and 4096x32768
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2t
for shape in "8192 8192" "4096 32768"; do set -- $shape; N=$1; W=$2
for cfg in "24 8 0 4 0" "8 4 34 2 1" "8 4 34 4 1" "12 4 34 2 1" "16 4 34 2 1" "8 8 34 2 1" "8 4 34 2 0" "8 4 34 4 0" "12 4 34 4 0" "16 4 34 4 0" "8 4 23 4 0" "12 4 23 4 0" "16 8 34 4 0" "16 4 45 4 0" "24 4 45 4 1"; do
  set -- $cfg; K=$1; nw=$2; rows=$3; lv=$4; ip=$5
  r=$(KB_W=$W KB_INPLACE=$ip timeout -k 5 60 ./build/kbench_tl $N $K $((K*40)) 0 0 $nw $rows $lv 2>&1 | tail -1) || exit 1
  echo "N=$N W=$W K=$K nw=$nw rows=$rows lv=$lv ip=$ip $r" | tee -a gpurun_out/r2t/sweep.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-175
done; done
}

batch_u() {
# shallow passes: rotating 6-row prefetch (pf2) vs queue-shift prefetch (pf1, previous build), 32768^2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2u
for K in 1 2 3 4 8; do for s2 in 0 1; do for v in pf1 pf2; do
  r=$(KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$v 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
  echo "$v K=$K split2=$s2 $r" | tee -a gpurun_out/r2u/ab.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-140
done; done; done
}

batch_v() {
# private trash words for non-storing lanes (tr) vs the shared trash row (base = HEAD), 32768^2 and 8192^2 tile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2v
for K in 1 2 4 8; do for s2 in 0 1; do for v in base tr; do
  r=$(KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$v 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
  echo "$v K=$K split2=$s2 $r" | tee -a gpurun_out/r2v/ab.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-140
done; done; done
for v in base tr; do for args in "8192 24 960 0 0 8 0 4" "4096 32 960 0 0 8 0 2"; do
  r=$(KB_W=$([ "${args%% *}" = 4096 ] && echo 32768 || echo 8192) KB_INPLACE=$([ "${args%% *}" = 4096 ] && echo 1 || echo 0) timeout -k 5 60 ./build/kbench_$v $args 2>&1 | tail -1) || exit 1
  echo "$v tile $args $r" | tee -a gpurun_out/r2v/ab.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-150
done; done
}

batch_w() {
# why a K=1 pass streams at ~55% of the HBM rate: PMC of step_temporal<1> (kbench) vs the column-walk copy (bw_probe)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2w
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $R/gpurun_out/r2w/a -o a --output-format csv -- $R/build/kbench_tr 32768 1 40 > $R/gpurun_out/r2w/a.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/r2w/b -o b --output-format csv -- $R/build/kbench_tr 32768 1 40 > $R/gpurun_out/r2w/b.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $R/gpurun_out/r2w/c -o c --output-format csv -- $R/build/bw_probe > $R/gpurun_out/r2w/c.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/r2w/d -o d --output-format csv -- $R/build/bw_probe > $R/gpurun_out/r2w/d.log 2>&1 || exit 1
for x in a b c d; do python3 $R/tools/pmc_summary.py $R/gpurun_out/r2w/$x/${x}_counter_collection.csv | grep -A12 "step_temporal<1\|colwalk" | head -30; done
}

batch_x() {
# shallow-pass diagnosis: stores removed (nost), halo lanes not storing (mst), default (tr); kbench 32768^2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2x
for K in 1 4 8; do for s2 in 0 1; do for v in tr mst nost; do
  r=$(KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$v 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
  echo "$v K=$K split2=$s2 $r" | tee -a gpurun_out/r2x/ab.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-140
done; done; done
}

batch_y() {
# per-half sub-tile graphs: sub-tile tests, then bench (20 and 2000 steps) with graphs vs --no-graph, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2y
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py tests/test_gpu_headline.py -x -q -m gpu -k "subtiles or hint or headline or seam" --timeout 200 --timeout-method thread > gpurun_out/r2y/pytest.log 2>&1 || { tail -30 gpurun_out/r2y/pytest.log; exit 1; }
tail -1 gpurun_out/r2y/pytest.log
for i in 1 2 3; do for g in "" "--no-graph"; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 $g > gpurun_out/r2y/b20_$i$g.log 2>&1 || exit 1
  echo "20 steps ${g:-graph}: $(tail -1 gpurun_out/r2y/b20_$i$g.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f us/gen" % (d["ms_per_step"]*1e3), "graph_launches", d["config"]["graph_launches"])')"
done; done
for g in "" "--no-graph"; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 $g > gpurun_out/r2y/b2000$g.log 2>&1 || exit 1
  echo "2000 steps ${g:-graph}: $(tail -1 gpurun_out/r2y/b2000$g.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f us/gen" % (d["ms_per_step"]*1e3), "graph_launches", d["config"]["graph_launches"])')"
done
timeout -k 10 120 python bench.py --gpus 1 --steps 1280 --warmup 128 --self-exchange > gpurun_out/r2y/bself.log 2>&1 || exit 1
echo "self-exchange 1280: $(tail -1 gpurun_out/r2y/bself.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f us/gen" % (d["ms_per_step"]*1e3), "graph_launches", d["config"]["graph_launches"], d["config"]["schedule"])')"
}

batch_z() {
# plan order A/B: column-major (default) vs row-major segments, 32768^2, all depths (kbench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2z
for K in 1 2 4 8; do for s2 in 0 1; do for o in col row; do
  r=$(GOL_PLAN_ORDER=$o KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_po 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
  echo "$o K=$K split2=$s2 $r" | tee -a gpurun_out/r2z/ab.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-100
done; done; done
for o in col row; do for a in "8192 24 960 0 0 8 0 4" "16384 8 320"; do
  r=$(GOL_PLAN_ORDER=$o timeout -k 5 60 ./build/kbench_po $a 2>&1 | tail -1) || exit 1
  echo "$o $a $r" | tee -a gpurun_out/r2z/ab.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-100
done; done
}

id=${1:-}; shift || true
if ! declare -F "batch_$id" >/dev/null; then
  echo "usage: $0 <id> [args]; ids: a aa ab ac ad ae af ag ah ai aj ak al am an ao ap aq ar as at au av aw ax ay az b ba bb bc bd be bf bg bh bi bj bk bl bm bn bo bp bq br bs bt bu bv c d e f g h i j k l m n o p q r s t u v w x y z" >&2; exit 2
fi
"batch_$id" "$@"
