#!/bin/bash
# Ping-pong loop for K = 6, 7, 12 and deeper pass costs in the pass-cut DP: full GPU suite, smoke,
# driver bench x3, long bench, 16384^2 and 65536^2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
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
