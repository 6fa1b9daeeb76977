#!/bin/bash
# Round-5 tree check on one MI355X box: GPU tests, build()+smoke(), the driver's default bench.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_check}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 200 python bench.py > $OUT/bench_default.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_a.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
for f in $OUT/bench_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"; done
exit $rc
