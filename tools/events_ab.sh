#!/bin/bash
# Full multi-rank schedule on one GPU (thread ranks, RCCL-semantics transport): ready-event record
# per superstep (GOL_READY_EVENTS=always) vs none (default), alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/events
out=gpurun_out/events/ab.txt; : > $out
for r in 1 2; do
  for ev in always default; do
    echo "== $ev" >> $out
    GOL_SCHEDULE=full GOL_READY_EVENTS=$ev timeout -k 10 200 python -u tools/rehearse_multirank.py --configs 1d:2:32768,1d:4:32768 --gens 2560 >> $out 2>&1 || exit 3
  done
done
cat $out
