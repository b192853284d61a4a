#!/bin/bash
# per-half sub-tile graphs: sub-tile tests, then bench (20 and 2000 steps) with graphs vs --no-graph, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2y
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py tests/test_gpu_headline.py -x -q -m gpu -k "subtiles or hint or headline or seam" --timeout 200 --timeout-method thread > gpurun_out/r2y/pytest.log 2>&1 || { tail -30 gpurun_out/r2y/pytest.log; exit 1; }
tail -1 gpurun_out/r2y/pytest.log
for i in 1 2 3; do for g in "" "--no-graph"; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 $g > gpurun_out/r2y/b20_$i$g.log 2>&1 || exit 1
  echo "20 steps ${g:-graph}: $(tail -1 gpurun_out/r2y/b20_$i$g.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f us/gen" % (d["ms_per_step"]*1e3), "graph_launches", d["config"]["graph_launches"])')"
done; done
for g in "" "--no-graph"; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 $g > gpurun_out/r2y/b2000$g.log 2>&1 || exit 1
  echo "2000 steps ${g:-graph}: $(tail -1 gpurun_out/r2y/b2000$g.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f us/gen" % (d["ms_per_step"]*1e3), "graph_launches", d["config"]["graph_launches"])')"
done
timeout -k 10 120 python bench.py --gpus 1 --steps 1280 --warmup 128 --self-exchange > gpurun_out/r2y/bself.log 2>&1 || exit 1
echo "self-exchange 1280: $(tail -1 gpurun_out/r2y/bself.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f us/gen" % (d["ms_per_step"]*1e3), "graph_launches", d["config"]["graph_launches"], d["config"]["schedule"])')"
