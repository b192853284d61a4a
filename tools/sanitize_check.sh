#!/bin/bash
# Host sanitizer runs of the native core (CPU paths: engines, thread/TCP transports, planner, I/O,
# watchdog).  GPU sanitizers are not used on this pool; the HIP sources are compiled without them.
#   bash tools/sanitize_check.sh [address|thread ...]
set -e
cd "$(dirname "$0")/.."
for san in "${@:-address thread}"; do
  for s in $san; do
    b=${GOL_SAN_BUILD_DIR:-/tmp}/gol-san-$s
    cmake -S . -B $b -DGOL_SANITIZE=$s -DGOL_WITH_PYTHON=OFF -DGOL_WITH_MPI=OFF -DCMAKE_BUILD_TYPE=RelWithDebInfo > $b.log 2>&1
    cmake --build $b -j8 --target gol_unit gol >> $b.log 2>&1
    echo "== $s"
    if [ $s = thread ]; then export OMP_NUM_THREADS=1 TSAN_OPTIONS="halt_on_error=1"; else export ASAN_OPTIONS="detect_leaks=1"; fi
    GOL_BACKEND=cpu $b/gol_unit | tail -1
    # the CLI's multi-rank I/O: 2-D dumps routed point to point, a checkpoint written by a 2x2 grid
    # and resumed by 3 strips (thread ranks)
    w=$(mktemp -d)
    (cd $w && GOL_BACKEND=cpu GOL_NRANKS=4 GOL_GLOBAL=1 GOL_DECOMP=2d GOL_GRID=2x2 GOL_CHECKPOINT_EVERY=8 \
        GOL_CHECKPOINT_PATH=$w/ck $b/gol 5 256 16 256 1 > /dev/null &&
     GOL_BACKEND=cpu GOL_NRANKS=3 GOL_GLOBAL=1 GOL_RESTART=$w/ck $b/gol 5 256 24 256 1 > /dev/null &&
     echo "CLI dump/checkpoint run clean")
    rm -rf $w
  done
done
