#!/bin/bash
# round-2 validation after splitting the engine source: full GPU suite, smoke, driver bench x3, long bench, capacity config (2^20 x 2^20 tile)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2am
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2am/pytest.log 2>&1 || { tail -30 gpurun_out/r2am/pytest.log; exit 1; }
tail -1 gpurun_out/r2am/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2am/b20_$i.log 2>&1 || exit 1; tail -1 gpurun_out/r2am/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("20 steps: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'; done
timeout -k 10 120 python bench.py --gpus 1 > gpurun_out/r2am/bdefault.log 2>&1 || exit 1; tail -1 gpurun_out/r2am/bdefault.log | python -c 'import json,sys; d=json.load(sys.stdin); print("defaults (%d steps): %.3f us/gen %.3e" % (d["steps"], d["ms_per_step"]*1e3, d["value"]))'
timeout -k 10 300 python bench.py --gpus 1 --steps 40 --warmup 8 --size 1048576 > gpurun_out/r2am/bcap.log 2>&1 || { tail -5 gpurun_out/r2am/bcap.log; exit 1; }
tail -1 gpurun_out/r2am/bcap.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("2^20 x 2^20: %.3f ms/gen %.3e" % (d["ms_per_step"], d["value"]), c["schedule"], c["kernel"])'
