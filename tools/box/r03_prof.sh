#!/bin/bash
# Round-3 CPU attribution on the box: headline with the sampling profiler,
# headline without it (overhead check), the 8-worker pool, and GPU tests.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_a.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/headline.prof > $OUT/bench_prof.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_b.log 2>&1 &&
timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 > $OUT/pool8_10m.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log
for f in $OUT/bench_*.log $OUT/pool8_10m.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f)"; done
head -12 $OUT/headline.prof.txt
exit $rc
