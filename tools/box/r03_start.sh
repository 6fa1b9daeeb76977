#!/bin/bash
# Round-3 opening check at the round-2 HEAD: GPU tests, smoke, headline x2,
# 8-worker pool (the numbers this round's CPU work is measured against).
set -o pipefail
OUT=${OUT:-gpurun_out/r03_start}
mkdir -p $OUT
export TMPDIR=/tmp
nproc > $OUT/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $OUT/nproc.txt 2>/dev/null
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $OUT/bench_a.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_b.log 2>&1 &&
timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 > $OUT/pool8_10m.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
for f in $OUT/bench_*.log $OUT/pool8_10m.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f)"; done
exit $rc
