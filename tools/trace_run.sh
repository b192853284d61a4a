#!/bin/bash
# GPU: kernel + roctx-marker trace of bench.py's timed run, summarised per queue by tools/timed_trace.py.
#   tools/trace_run.sh <name> [bench args ...]     (defaults: --gpus 1 --steps 20 --warmup 5 --no-phases)
# Output: gpurun_out/trace_<name>/ (rocprofv3 csv), gpurun_out/trace_<name>.txt (the timeline).
# rocprofv3 runs python3 itself (no env/launcher hop); GOL_ROCTX is exported beforehand.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp GOL_ROCTX=1
name=$1; shift
d=gpurun_out/trace_$name
mkdir -p "$d"
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d "$d" -o t --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-phases "$@" > "$d.log" 2>&1 || { echo "trace $name rc=$?"; tail -5 "$d.log"; exit 1; }
{ echo "# bench.py $* (rocprofv3 --kernel-trace --marker-trace, GOL_ROCTX=1)"; grep -h '^{' "$d.log" | python3 tools/bench_line.py "$name"; python3 tools/timed_trace.py "$d"; } > "$d.txt"
cat "$d.txt"
