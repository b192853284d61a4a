#!/bin/bash
# GPU: age-weighted plan heights (build_plan age_weights): one stamped pass per weight set
# (tools/stamp_probe.hip), then the driver's bench command with GOL_AGE_WEIGHTS A/B (3 runs each).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
f=gpurun_out/stamp_weights.txt
: > $f
for spec in ${WEIGHTS:-3:1 3:1.3,1.0,0.7 3:1.6,1.15,0.75 3:2.0,1.4,1.0 3:1.8,1.2,0.6 2:1 2:1.3,0.7 2:1.5,0.67 2:1.8,0.8}; do
  bpc=${spec%%:*}; w=${spec#*:}
  timeout -k 10 60 build/stamp_probe 32768 $w 1 $bpc >> $f 2>&1 || { echo "stamp_probe rc=$? at $spec"; exit 1; }
done
grep -E "^weights" $f
b=gpurun_out/age_bench.jsonl
: > $b
for rep in 1 2 3; do
  for w in ${BENCH_WEIGHTS:-1 1.5,0.67 1.6,1.15,0.75}; do
    echo "== GOL_AGE_WEIGHTS=$w rep $rep" >> $b
    GOL_SUBTILES=${SUBTILES:-0} GOL_AGE_WEIGHTS=$w timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $b 2>gpurun_out/age_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/age_bench.err; exit 1; }
  done
done
python3 - "$b" <<'PY'
import json, sys
w = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        w = line.split()[1]
        continue
    try:
        d = json.loads(line)
    except Exception:
        continue
    print(w, "%.3f us/gen" % (d["ms_per_step"] * 1e3), d.get("config", {}).get("schedule", ""), d.get("config", {}).get("kernel", ""))
PY
