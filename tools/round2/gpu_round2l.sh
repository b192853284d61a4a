#!/bin/bash
# tile kernel: software-pipelined LDS band reads (tnew) vs the previous kernel (told), + tile tests + config 2 CLI
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2l
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_cli.py -x -q -m gpu -k "tile or auto or cfg or perf" --timeout 120 --timeout-method thread > gpurun_out/r2l/pytest.log 2>&1 || { tail -20 gpurun_out/r2l/pytest.log; exit 1; }
tail -2 gpurun_out/r2l/pytest.log
for N in 8192 16384; do
  for K in 16 24 32; do
    for nw in 8 16; do
      for lv in 1 2; do
        for v in told tnew; do
          r=$(timeout -k 5 60 ./build/kbench_$v $N $K $((K*40)) 0 0 $nw 0 $lv 2>&1 | tail -1) || exit 1
          echo "$v N=$N K=$K nw=$nw lv=$lv $r" | tee -a gpurun_out/r2l/tile_ab.txt | cut -c1-60,150-
        done
      done
    done
  done
done
for i in 1 2 3; do timeout -k 10 60 ./build/gol 5 8192 1000 256 0 | head -1; done
