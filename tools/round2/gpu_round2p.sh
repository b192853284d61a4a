#!/bin/bash
# tile kernel time breakdown: s_memtime stamps per LDS pass (diagnostic build kbench_stamp)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2p
for args in "8192 24 960 0 0 8 0 2" "8192 24 960 0 0 8 0 1" "8192 24 960 0 0 8 0 4" "8192 24 960 0 0 4 0 2" "8192 24 960 0 0 16 0 2" "8192 8 960 0 0 8 0 2" "16384 24 960 0 0 8 0 2" "32768 24 960 0 0 8 0 2"; do
  echo "== $args" | tee -a gpurun_out/r2p/stamps.txt
  timeout -k 5 60 ./build/kbench_stamp $args 2>&1 | tail -2 | tee -a gpurun_out/r2p/stamps.txt | cut -c1-400 || exit 1
done
