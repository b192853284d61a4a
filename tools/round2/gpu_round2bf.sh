#!/bin/bash
# Tile kernel with the two-triple band loop at 4 levels: tile GPU tests, config 2 CLI x3, bench 8192^2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bf
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_cli.py -k "tile or known_physics or perf or auto or cfg or 8192" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for i in 1 2 3; do (cd $o && timeout -k 10 120 ../../build/gol 5 8192 1000 256 0 | tail -1); done
timeout -k 10 120 python bench.py --gpus 1 --size 8192 --steps 1000 --warmup 24 > $o/b8k.log 2>&1 || exit 1
grep '^{"metric"' $o/b8k.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("8192^2 bench: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), c["kernel"], c["kernel_depth"])'
