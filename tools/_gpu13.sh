set -o pipefail
cd $GRAFT_REPO_ROOT
GOL_INIT_LOG=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/k10p.log 2>&1; echo "rc=$?"; grep '^{' gpurun_out/k10p.log | python3 tools/bench_line.py k10p
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/k10p.log') if l.startswith('{')][0]);print(' '.join(t for t in d['config']['autotune'].split() if t.startswith(('pass','cut'))))"
