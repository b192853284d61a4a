set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_headline.py tests/test_gpu_rccl.py --timeout 300 --timeout-method thread > gpurun_out/t10_tests.log 2>&1; rc=$?; tail -2 gpurun_out/t10_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/configs; bash tools/baseline_configs.sh cfg2b cfg4 > gpurun_out/t10_configs.log 2>&1 || exit 1
for f in gpurun_out/configs/cfg2_bench_8192.log gpurun_out/configs/cfg4_bench_65536_2d.log; do grep -h '^{' $f | python3 tools/bench_line.py "$(basename $f .log)"; done
