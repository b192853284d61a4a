#!/bin/bash
# After making the sub-tile overlap opt-in: the sub-tile / RCCL / headline GPU tests and the driver bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2as
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_engine.py tests/test_gpu_headline.py -k "subtile or rccl or run_hint or headline" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for i in 1 2; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1; grep '^{"metric"' $o/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("20 steps: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), d["config"]["schedule"])'; done
