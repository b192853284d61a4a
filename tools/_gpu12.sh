set -o pipefail
cd $GRAFT_REPO_ROOT
GOL_INIT_LOG=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/k10.log 2>&1; echo "rc=$?"; grep "pass costs\|prediction" gpurun_out/k10.log | tail -16; grep '^{' gpurun_out/k10.log | python3 tools/bench_line.py k10
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/k10.log') if l.startswith('{')][0]);print(' '.join(t for t in d['config']['autotune'].split() if t.startswith(('pass','cut'))))"
timeout -k 10 300 python -u -m pytest -x -q tests/test_gpu_headline.py tests/test_gpu_engine.py --timeout 300 --timeout-method thread > gpurun_out/t12_tests.log 2>&1; rc=$?; tail -2 gpurun_out/t12_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/bench_reps.*; tools/bench_reps.sh 5 ""
