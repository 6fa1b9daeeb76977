#!/bin/bash
# Driver sequence on a fresh lease: the driver's bench command FIRST (nothing
# warmed), then the GPU tests and smoke, then the cleanup A/B (reference mode
# "off" vs recycle "on", alternated, 300 timed jobs each).
set -o pipefail
OUT=${OUT:-gpurun_out/r04_fresh}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1 &&
for arm in off on off on off on; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cleanup $arm >> $OUT/ab_$arm.log 2>&1 || exit $?
done
rc=$?
tail -2 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
for f in $OUT/bench_driver.log $OUT/ab_*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"
done
exit $rc
