#!/bin/bash
# GPU: the driver's bench command, alternating this tree and another built tree (a git worktree of an
# earlier commit under build/, built in place), N pairs on one box.
#   tools/gpu_ab_tree.sh <other tree> [pairs=6] [bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
other=$1; pairs=${2:-6}; shift 2
args=${*:---gpus 1 --steps 20 --warmup 5}
o=gpurun_out/ab_tree.txt
: > $o
for i in $(seq 1 $pairs); do
  for t in . "$other"; do
    r=$(cd "$t" && timeout -k 10 240 python3 bench.py $args 2>/dev/null) || { echo "bench rc=$? in $t"; exit 1; }
    echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t: %.3f us/gen' % (d['ms_per_step']*1e3), d['config']['schedule'], d['config']['kernel'])" | tee -a $o
  done
done
