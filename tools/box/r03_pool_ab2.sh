#!/bin/bash
# GPU tests + smoke at the tree, then the 8-worker pool with one L3 domain per
# worker spread over both sockets (worker i on domain 2i) vs consecutive
# CPU-id slices, alternated x2.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_pool_ab2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
for rep in 1 2; do
  [ $rc = 0 ] || break
  for v in l3 slice; do
    timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 --placement $v > $OUT/pool_${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
tail -1 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
for f in $OUT/pool_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done
exit $rc
