#!/bin/bash
# Round-end rehearsal: GPU tests, smoke(), headline bench.
set -o pipefail
OUT=gpurun_out/r02_check
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 300 --warmup 10 > $OUT/bench.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -3 $OUT/smoke.log; grep '^{' $OUT/bench.log | cut -c1-400
exit $rc
