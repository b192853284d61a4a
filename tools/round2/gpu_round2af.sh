#!/bin/bash
# sub-tile waits skipped on completed events: sub-tile tests, driver bench x5, traced once
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2af
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py tests/test_gpu_headline.py -x -q -m gpu -k "subtiles or hint or headline or seam or graphs" --timeout 200 --timeout-method thread > gpurun_out/r2af/pytest.log 2>&1 || { tail -30 gpurun_out/r2af/pytest.log; exit 1; }
tail -1 gpurun_out/r2af/pytest.log
for i in 1 2 3 4 5; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2af/b20_$i.log 2>&1 || exit 1; tail -1 gpurun_out/r2af/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("20 steps: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'; done
timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/r2af/b2000.log 2>&1 || exit 1; tail -1 gpurun_out/r2af/b2000.log | python -c 'import json,sys; d=json.load(sys.stdin); print("2000 steps: %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'
cd /tmp
R=$GRAFT_REPO_ROOT
GOL_ROCTX=1 timeout -k 10 200 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $R/gpurun_out/r2af/t -o t -- python $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/r2af/t.log 2>&1 || exit 1
