#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r2bg
for i in 1 2 3 4; do (cd gpurun_out/r2bg && timeout -k 10 120 ../../build/gol 5 8192 1000 256 0 | grep TOTAL); done
