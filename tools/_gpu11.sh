set -o pipefail
cd $GRAFT_REPO_ROOT
GOL_INIT_LOG=1 timeout -k 10 300 python bench.py --size 65536 --scaling strong --decomp 2d --steps 400 --warmup 40 > gpurun_out/cfg4_dbg.log 2>&1; echo "rc=$?"; grep -v "RCCL\|version\|Hostname\|Librccl" gpurun_out/cfg4_dbg.log | tail -25 | cut -c1-250
