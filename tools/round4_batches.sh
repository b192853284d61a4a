#!/bin/bash
# Round-4 GPU batches, one function each (on the GPU box: bash tools/round4_batches.sh <name> [args]).
# Every GPU step has its own time limit; a batch stops at the first failure.  Results land in gpurun_out/;
# the summaries kept are in profiles/ (named in docs/PERFORMANCE.md §15 and docs/REVIEW_RESPONSE.md).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp

# flow_a: GPU batch (round 4): flow kernel checks, GPU tests, the 32768^2 cut sweep, the driver's bench A/B
# (auto vs forced flow) and a kernel trace of the flow bench.  Every step has its own time limit; the
# batch stops at the first failure.
cmd_flow_a() {
step() { echo "[batch] $(date +%T) $*"; }
step flowbench-small
timeout -k 10 60 build/flowbench 4096 2,2 5 1.0 > gpurun_out/fb_small.txt 2>&1 || { echo "flowbench small rc=$?"; cat gpurun_out/fb_small.txt; exit 1; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_rccl.py tests/test_gpu_resident.py -x -v \
    --timeout 180 --timeout-method thread -k "flow or registered or timeout" > gpurun_out/test_flow.txt 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/test_flow.txt; exit 1; }
step sweep
bash tools/flow_sweep.sh gpurun_out/flow_sweep.txt || exit 1
step bench-ab
cmd_flow_bench_ab gpurun_out/flow_bench_ab.jsonl 5 > gpurun_out/flow_bench_ab.txt 2>&1 || { cat gpurun_out/flow_bench_ab.txt; exit 1; }
step trace
GOL_SCHEDULE=flow GOL_ROCTX=1 timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/prof_flow -o flow -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-phases > gpurun_out/prof_flow_bench.txt 2>&1 || { echo "trace rc=$?"; tail -20 gpurun_out/prof_flow_bench.txt; exit 1; }
python3 tools/timed_trace.py gpurun_out/prof_flow > gpurun_out/prof_flow_timed.txt 2>&1 || true
step done
}

# batch_b: GPU batch B (round 4): BASELINE configs on the final tree, the 8-process torchrun rehearsal (per-rank
# arrays), self-exchange runs (RCCL registered / unregistered, flow+ov), and PMC counters of the flow
# kernel vs the pass kernel.  Each step has its own time limit; a fatal status ends the batch.
cmd_batch_b() {
step() { echo "[batch-b] $(date +%T) $*"; }
step configs
bash tools/baseline_configs.sh cfg2 cfg2f cfg2nf cfg2 cfg2f cfg2nf cfg2b cfg3 cfg4 > gpurun_out/configs_summary.txt 2>&1 || { cat gpurun_out/configs_summary.txt; exit 1; }
step self-exchange
for v in "GOL_RCCL_REGISTER=1" "GOL_RCCL_REGISTER=0" "GOL_SCHEDULE=flow+ov" "GOL_SCHEDULE=flow"; do
  env $v timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange > gpurun_out/selfx_$(echo $v | tr '=+' '__').json 2> gpurun_out/selfx_err.txt || { echo "self-exchange $v failed"; tail gpurun_out/selfx_err.txt; exit 1; }
done
step rehearsal
timeout -k 10 900 bash tools/rehearse_torchrun.sh > gpurun_out/rehearse_summary.txt 2>&1 || { tail -30 gpurun_out/rehearse_summary.txt; exit 1; }
step pmc
for kn in flow temporal; do
  if [ $kn = flow ]; then envs="GOL_SCHEDULE=flow"; else envs="GOL_SUBTILES=0"; fi
  env $envs timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/pmc_$kn -o pmc -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-phases > gpurun_out/pmc_$kn.txt 2>&1 || { echo "pmc $kn rc=$?"; tail gpurun_out/pmc_$kn.txt; exit 1; }
done
step done
}

# batch_c: GPU batch C (round 4): launch-latency probe, the flow GPU tests (tile fallback, flow+ov on the
# CU-restricted stream, forced flow on small boards), then batch B (configs with flow A/B,
# self-exchange, rehearsal, PMC).  Each step has its own time limit; the batch stops at a failure.
cmd_batch_c() {
echo "[batch-c] $(date +%T) launch probe"
timeout -k 10 120 build/launch_probe 64 > gpurun_out/launch_probe.txt 2>&1 || { echo "launch_probe rc=$?"; exit 1; }
echo "[batch-c] $(date +%T) flow tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_rccl.py -x -v --timeout 180 --timeout-method thread \
    -k "flow or registered" > gpurun_out/test_flow.txt 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/test_flow.txt; exit 1; }
tail -3 gpurun_out/test_flow.txt
cmd_batch_b
}

# batch_d: GPU batch D (round 4): the full GPU test suite and smoke on the current tree, the driver's bench
# command x5 (headline), the 8-process rehearsal (strong / 2-D after the per-rank kernel fix), and
# PMC of config 2 (tile passes vs tile flow).  Each step has its own time limit; stops at a failure.
cmd_batch_d() {
s() { echo "[batch-d] $(date +%T) $*"; }
s tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
s smoke
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail gpurun_out/smoke.log; exit 1; }
s driver-bench
: > gpurun_out/driver_bench.jsonl
for i in 1 2 3 4 5; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/driver_bench.jsonl 2>gpurun_out/driver_bench.err || { echo "bench rc=$?"; tail gpurun_out/driver_bench.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/driver_bench.jsonl'):
    d=json.loads(l); print('%.3f us/gen' % (d['ms_per_step']*1e3), d['config']['schedule'], d['config']['kernel'])
"
s rehearsal
timeout -k 10 900 bash tools/rehearse_torchrun.sh > gpurun_out/rehearse_summary.txt 2>&1 || { tail -30 gpurun_out/rehearse_summary.txt; exit 1; }
grep -E "^==|rc=|value" gpurun_out/rehearse_summary.txt
s pmc
for kn in flow tile; do
  if [ $kn = flow ]; then envs="GOL_SCHEDULE=flow"; else envs="GOL_SCHEDULE=auto"; fi
  env $envs timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/pmc_cfg2_$kn -o pmc -- ./build/gol 5 8192 1000 256 0 > gpurun_out/pmc_cfg2_$kn.txt 2>&1 || { echo "pmc $kn rc=$?"; tail gpurun_out/pmc_cfg2_$kn.txt; exit 1; }
done
s done
}

# batch_e: GPU batch E (round 4): the 8192^2 warmup anomaly against the XCD-aware plan order (GOL_PLAN_XCDS=8 / 1,
# warmups 96 / 100), config 2 with the flow candidates timed (GOL_FLOW=1: equal-span timing), and the
# driver's cut through the RCCL self-exchange x3.  Each step has its own time limit.
cmd_batch_e() {
o=gpurun_out/warmup_xcds.txt
: > $o
for round in 1 2; do
  for x in 8 1; do
    for w in 96 100; do
      r=$(GOL_PLAN_XCDS=$x timeout -k 10 120 python3 bench.py --size 8192 --steps 1000 --warmup $w --no-phases 2>/dev/null) || { echo "bench rc=$? (xcds $x warmup $w)"; exit 1; }
      echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('xcds $x warmup $w: %.4f us/gen' % (d['ms_per_step']*1e3), d['config']['schedule'], d['config']['kernel'])" | tee -a $o
    done
  done
done
for i in 1 2; do
  echo "== cfg2 CLI GOL_FLOW=1" | tee -a $o
  GOL_BACKEND=hip GOL_FLOW=1 GOL_METRICS_JSON=gpurun_out/cfg2_flowtimed.json timeout -k 10 120 ./build/gol 5 8192 1000 256 0 > gpurun_out/cfg2_flowtimed.log 2>&1 || { echo "cli rc=$?"; tail gpurun_out/cfg2_flowtimed.log; exit 1; }
  grep -E "TOTAL" gpurun_out/cfg2_flowtimed.log | tee -a $o
  python3 -c "import json; d=json.load(open('gpurun_out/cfg2_flowtimed.json')); s=json.dumps(d); import re; print(re.findall(r'\"schedule\": \"[^\"]*\"', s)[:1], re.findall(r'sched:[a-z+]*=[0-9.]*', s))" | tee -a $o
done
for i in 1 2 3; do
  r=$(timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange 2>/dev/null) || { echo "selfx rc=$?"; exit 1; }
  echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; p=d['phases']; print('self-exchange: %.3f us/gen' % (d['ms_per_step']*1e3), c['schedule'], c['kernel'], 'registered', c['rccl_registered'], 'exchange_us', p.get('exchange_us_max'), 'superstep_us', p.get('superstep_us_max'))" | tee -a $o
done
}

# batch_f: GPU batch F (round 4): the driver command against the round-3 tree after the K=12 fix, and the
# driver's cut through the RCCL self-exchange x3.
cmd_batch_f() {
bash tools/gpu_ab_tree.sh build/r3src 5 || exit 1
o=gpurun_out/selfx_round4.txt
: > $o
for i in 1 2 3; do
  r=$(timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange 2>/dev/null) || { echo "selfx rc=$?"; exit 1; }
  echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; p=d['phases']; print('self-exchange: %.3f us/gen' % (d['ms_per_step']*1e3), c['schedule'], c['kernel'], 'registered', c['rccl_registered'], 'exchange_us', p.get('exchange_us_max'), 'superstep_us', p.get('superstep_us_max'))" | tee -a $o || exit 1
done
}

# traces: GPU batch G (round 4): kernel traces of the driver's timed run, the default schedule and the flow
# schedule (one dispatch per superstep), summarised by tools/timed_trace.py.
cmd_traces() {
export TMPDIR=/tmp GOL_ROCTX=1
for s in auto flow; do
  rm -rf gpurun_out/trace_$s; mkdir -p gpurun_out/trace_$s
  for i in 1 2; do
    GOL_SCHEDULE=$s timeout -k 10 180 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/trace_$s/r$i -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-phases > gpurun_out/trace_$s/b$i.log 2>&1 || { echo "trace $s rc=$?"; tail -5 gpurun_out/trace_$s/b$i.log; exit 1; }
    echo "== schedule $s run $i" >> gpurun_out/trace_summary.txt
    python3 tools/timed_trace.py gpurun_out/trace_$s/r$i >> gpurun_out/trace_summary.txt 2>&1
  done
done
cat gpurun_out/trace_summary.txt
}

# age: GPU: age-weighted plan heights (build_plan age_weights): one stamped pass per weight set
# (tools/stamp_probe.hip), then the driver's bench command with GOL_AGE_WEIGHTS A/B (3 runs each).
cmd_age() {
f=gpurun_out/stamp_weights.txt
: > $f
for spec in ${WEIGHTS:-3:1 3:1.3,1.0,0.7 3:1.6,1.15,0.75 3:2.0,1.4,1.0 3:1.8,1.2,0.6 2:1 2:1.3,0.7 2:1.5,0.67 2:1.8,0.8}; do
  bpc=${spec%%:*}; w=${spec#*:}
  timeout -k 10 60 build/stamp_probe 32768 $w 1 $bpc >> $f 2>&1 || { echo "stamp_probe rc=$? at $spec"; exit 1; }
done
grep -E "^weights" $f
# (the bench A/B of the removed GOL_AGE_WEIGHTS knob: profiles/stamp_age_weights.txt)
}

# selfx_ab: GPU: the sub-tile overlap tests, then the driver's cut through the RCCL self-exchange x4 and one trace.
cmd_selfx_ab() {
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py -x -q --timeout 180 --timeout-method thread -k "subtile or overlap or self" > gpurun_out/test_subtiles.txt 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/test_subtiles.txt; exit 1; }
tail -2 gpurun_out/test_subtiles.txt
o=gpurun_out/selfx_round4b.txt
: > $o
for i in 1 2 3 4; do
  r=$(timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange 2>/dev/null) || { echo "selfx rc=$?"; exit 1; }
  echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; p=d['phases']; print('self-exchange: %.3f us/gen' % (d['ms_per_step']*1e3), c['schedule'], c['kernel'], 'exchange_us', p.get('exchange_us_max'), 'superstep_us', p.get('superstep_us_max'), [x for x in c['autotune'].split() if x.startswith('sched:')])" | tee -a $o || exit 1
done
cmd_trace_selfx
}

# trace_selfx: GPU: kernel traces of the driver's cut through the RCCL self-exchange (a rank with neighbours on one
# GPU), summarised by tools/timed_trace.py (RCCL's kernels included).
cmd_trace_selfx() {
mkdir -p gpurun_out/trace_selfx
export TMPDIR=/tmp GOL_ROCTX=1
: > gpurun_out/trace_selfx/summary.txt
for i in 1 2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/trace_selfx/r$i -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange --no-phases > gpurun_out/trace_selfx/b$i.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/trace_selfx/b$i.log; exit 1; }
  echo "== run $i" >> gpurun_out/trace_selfx/summary.txt
  python3 tools/timed_trace.py gpurun_out/trace_selfx/r$i >> gpurun_out/trace_selfx/summary.txt 2>&1
done
cat gpurun_out/trace_selfx/summary.txt
}

# flow_check: GPU: step_flow checks — flowbench on a small board, the flow GPU tests, then the 32768^2 cut sweep.
cmd_flow_check() {
timeout -k 10 60 build/flowbench 4096 2,2 5 1.0 > gpurun_out/fb_small.txt 2>&1 || { echo "flowbench small rc=$?" >> gpurun_out/fb_small.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_rccl.py tests/test_gpu_resident.py -x -v \
    --timeout 180 --timeout-method thread -k "flow or registered or timeout" > gpurun_out/test_flow.txt 2>&1 || { echo "pytest rc=$?" >> gpurun_out/test_flow.txt; exit 1; }
bash tools/flow_sweep.sh gpurun_out/flow_sweep2.txt
}

# flow_bench_ab: GPU: the driver's bench command, alternating the default schedule choice (auto) with forced flow
# supersteps, N pairs; one JSON line per run in $out, a summary line per run on stdout.
# Usage: tools/round4_batches.sh flow_bench_ab [out=gpurun_out/flow_bench_ab.jsonl] [pairs=5] [extra bench args...]
cmd_flow_bench_ab() {
out=${1:-gpurun_out/flow_bench_ab.jsonl}
pairs=${2:-5}
shift 2
mkdir -p "$(dirname "$out")"
for i in $(seq 1 "$pairs"); do
  for mode in auto flow; do
    if [ "$mode" = auto ]; then env_sched=""; else env_sched="GOL_SCHEDULE=flow"; fi
    line=$(env $env_sched timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 "$@" 2>gpurun_out/bench_ab_err.txt | grep '^{') || { echo "bench failed ($mode)"; cat gpurun_out/bench_ab_err.txt; exit 1; }
    echo "{\"mode\": \"$mode\", \"run\": $line}" >> "$out"
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('$mode', round(d['ms_per_step']*1e3,3), 'us/gen', d['config']['schedule'], d['config']['kernel'])" "$line"
  done
done
}

# final: GPU (round 4, final tree): the full GPU suite and smoke, the driver's bench command x3 and its cut
# through the RCCL self-exchange x3.  Each step has its own time limit; stops at the first failure.
cmd_final() {
s() { echo "[final] $(date +%T) $*"; }
s tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_final.log
s smoke
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { echo "smoke rc=$?"; tail gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
s bench
o=gpurun_out/final_bench.txt
: > $o
for v in "" "--self-exchange"; do
  for i in 1 2 3; do
    r=$(timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 $v 2>/dev/null) || { echo "bench rc=$? ($v)"; exit 1; }
    echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('[$v] %.3f us/gen' % (d['ms_per_step']*1e3), '%.4g' % d['value'], c['schedule'], c['kernel'])" | tee -a $o || exit 1
  done
done
s done
}

name=$1; shift || true
if ! declare -F "cmd_$name" > /dev/null; then
  echo "usage: $0 <name> [args]; names: flow_a batch_b batch_c batch_d batch_e batch_f traces age selfx_ab trace_selfx flow_check flow_bench_ab final" >&2; exit 2
fi
"cmd_$name" "$@"
