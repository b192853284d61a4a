#!/bin/bash
# Auto halo depth 128 for sub-tile ranks: full GPU suite, smoke, driver command x4, long runs, 65536^2, self-exchange.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
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
