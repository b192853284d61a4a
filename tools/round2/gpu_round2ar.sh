#!/bin/bash
# Sub-tile exchange overlap (GOL_SUBTILE_OVERLAP): GPU tests of the sub-tile and RCCL paths, then the
# self-exchange bench with the init-time timing of both variants, and each variant forced.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2ar
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_engine.py -k "subtile or rccl or run_hint" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
b() {  # b <name> <env...>
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 bench.py --gpus 1 --steps $STEPS --warmup 16 --self-exchange > $o/$name.log 2>&1 || { tail -5 $o/$name.log; return 1; }
  grep '^{"metric"' $o/$name.log | python3 -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("'$name'", "%.3e %.3f us/gen" % (d["value"], d["ms_per_step"]*1e3), c["schedule"], [t for t in c["autotune"].split() if t.startswith("sched")])'
}
STEPS=256 b auto256 GOL_SUBTILE_OVERLAP=auto &&
STEPS=256 b ov0_256 GOL_SUBTILE_OVERLAP=0 &&
STEPS=256 b ov1_256 GOL_SUBTILE_OVERLAP=1 &&
STEPS=20 b ov0_20 GOL_SUBTILE_OVERLAP=0 &&
STEPS=20 b ov1_20 GOL_SUBTILE_OVERLAP=1 &&
STEPS=256 b ov0_256b GOL_SUBTILE_OVERLAP=0 &&
STEPS=256 b ov1_256b GOL_SUBTILE_OVERLAP=1 &&
STEPS=20 b ov0_20b GOL_SUBTILE_OVERLAP=0 &&
STEPS=20 b ov1_20b GOL_SUBTILE_OVERLAP=1
