#!/bin/bash
# Closing check at the final tree: GPU tests, smoke, the
# driver's default bench and two 300-step headline runs at the restored tree.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_close}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_default.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_a.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_b.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
for f in $OUT/bench_*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ') $(grep -o '"cpu_ms_per_job[^}]*' $f)"
done
exit $rc
